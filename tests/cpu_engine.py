"""CPU stand-in for ``pcm_amd.engine.Engine`` backed by the oracle (TEST ONLY).

It mirrors the device engine's contract -- int64 statistics tensor that the
driver all-reduces, device-side gating (halt/done), the held snapshot of a
halted iteration, 32-byte relocation records -- so that the multi-rank driver
in ``pcm_amd.lloyd`` (sharding, global fixed-point exponents, relocation
all-gather, halt/resume, chunked enqueue) can be exercised with the ``gloo``
backend on CPU.  The product never imports this.
"""
import numpy as np
import torch

from oracle import lloyd_ref as R

REC = np.dtype([("key", "<u8"), ("label", "<i4"), ("valid", "<i4"), ("xq", "<i4", (4,))])
assert REC.itemsize == 32


class OracleEngine:
    def __init__(self, d, k, max_iter=300):
        self.d, self.k, self.max_iter_cap = d, k, max_iter
        self.stats_device = torch.device("cpu")
        self.stats = None

    # ---------------- layout
    def bbox(self, X):
        self.rows = None
        self.X = np.ascontiguousarray(X.cpu().numpy(), dtype=np.float32)
        self.n = self.X.shape[0]
        if self.n == 0:
            z = np.zeros(self.d)
            return z, z, z
        lo, hi = self.X.min(0).astype(np.float64), self.X.max(0).astype(np.float64)
        return lo, hi, np.maximum(np.abs(lo), np.abs(hi))

    def build(self, X, q, gidx0=0):
        self.q = np.asarray(q, dtype=np.int32)
        if getattr(self, "rows", None) is None:
            self.gidx0 = int(gidx0)
        self.stats = torch.zeros(self.k * (self.d + 1) + 1, dtype=torch.int64)

    # ---------------- spatial slab sharding (numpy restatement of csrc/pcm_shard.hip)
    def set_shard(self, rows, n_global):
        self.rows = rows.numpy().astype(np.uint32).astype(np.int64)
        self.gidx0 = self.rows              # far_candidates takes the per-row global index

    @staticmethod
    def _bins(X, axis, lo, inv, nbins):
        x = np.ascontiguousarray(X.cpu().numpy())[:, axis].astype(np.float32).astype(np.float64)
        return np.clip(np.floor((x - lo) * inv), 0, nbins - 1).astype(np.int64)

    def shard_hist(self, X, axis, lo, inv, nbins):
        return torch.from_numpy(np.bincount(self._bins(X, axis, lo, inv, nbins), minlength=nbins).astype(np.int64))

    def shard_partition(self, X, axis, lo, inv, nbins, owner, world, gidx0):
        dest = np.asarray(owner, np.int64)[self._bins(X, axis, lo, inv, nbins)]
        order = np.argsort(dest, kind="stable")
        counts = np.bincount(dest, minlength=world).astype(np.int64)
        rows = (order + int(gidx0)).astype(np.int64).astype(np.int32)
        return X[torch.from_numpy(order)].contiguous(), torch.from_numpy(rows), counts

    def shard_scatter_labels(self, labels, rows, gidx0, n):
        out = np.empty(n, np.int32)
        out[rows.numpy().astype(np.uint32).astype(np.int64) - int(gidx0)] = labels.numpy()
        return torch.from_numpy(out)

    # ---------------- iterations
    def begin(self, C0, tol, max_iter):
        self.C = np.ascontiguousarray(C0.cpu().numpy(), dtype=np.float32)
        self.lab = np.full(self.n, -1, np.int32)
        self.halt = self.done = self.it = self.n_empty = 0
        self.resume = False
        self.tol, self.max_iter = float(tol), int(max_iter)
        self.hist_changed, self.hist_shift = [], []
        self.inertia = 0.0
        self.limbs = [0, 0, 0]
        self.prev = np.zeros(self.k * (self.d + 1), np.int64)   # raw statistics of the previous iteration
        self.neq_saved = 0

    def _decode(self, st):
        k, d = self.k, self.d
        body = st[: k * (d + 1)].reshape(k, d + 1)
        return body[:, :d].copy(), body[:, d].copy(), int(st[-1])

    def iter_local(self):
        if self.halt or self.done:
            return
        lab, sums, cnt, nch = R.local_stats(self.X, self.C, self.lab, self.q)
        self.lab = lab
        st = np.zeros(self.k * (self.d + 1) + 1, np.int64)
        body = st[: self.k * (self.d + 1)].reshape(self.k, self.d + 1)
        body[:, : self.d] = sums
        body[:, self.d] = cnt
        st[-1] = nch
        self.stats.copy_(torch.from_numpy(st))

    def iter_global(self):
        if self.halt or self.done:
            return
        st = self.stats.numpy().copy()
        sums, cnt, _ = self._decode(st)
        # convergence as the device does it: raw statistics equal the previous ones
        if not self.resume:
            body = st[: self.k * (self.d + 1)]
            nch = int(np.count_nonzero(body != self.prev))
            self.prev = body.copy()
        else:
            nch = self.neq_saved
        if (cnt == 0).any() and not self.resume:
            self.held = st
            self.halt, self.n_empty = 1, int((cnt == 0).sum())
            self.neq_saved = nch
            return
        Cn = R.average(sums, cnt, self.q, self.C)
        shift = R.shift_total(Cn, self.C)
        self.hist_changed.append(nch)
        self.hist_shift.append(shift)
        self.C, self.resume = Cn, False
        done = 1 if nch == 0 else (2 if shift <= self.tol else 0)
        self.it += 1
        if not done and self.it >= self.max_iter:
            done = 3
        self.done = done

    def iterate(self, n):
        for _ in range(n):
            self.iter_local()
            self.iter_global()

    def status(self):
        return dict(halt=self.halt, done=self.done, iter=self.it, n_empty=self.n_empty, inertia=self.inertia,
                    inertia_limbs=list(self.limbs), inertia_scale=R.inertia_scale(self.q), inertia_overflow=0, list_rebuilds=0,
                    last_changed=self.hist_changed[-1] if self.hist_changed else 0,
                    last_shift=self.hist_shift[-1] if self.hist_shift else 0.0)

    # ---------------- relocation (same 32-byte records as the device)
    def reloc_candidates(self, m):
        rec = np.zeros(m, REC)
        if self.n:
            dist, gidx, lab, xr, _ = R.far_candidates(self.X, self.C, self.lab, self.gidx0, m)
            t = len(dist)
            rec["key"][:t] = (dist.astype(np.float32).view(np.uint32).astype(np.uint64) << np.uint64(32)) | \
                (np.uint64(0xFFFFFFFF) - gidx.astype(np.uint64))
            rec["label"][:t] = lab
            rec["valid"][:t] = 1
            rec["xq"][:t, : self.d] = R.to_fixed(xr, self.q)
        return torch.from_numpy(rec.view(np.uint8).copy())

    def reloc_apply(self, records):
        rec = records.numpy().view(REC)
        rec = rec[rec["valid"] == 1]
        rec = rec[np.argsort(rec["key"])[::-1]]          # keys are unique: exact descending order
        st = self.held.copy()
        k, d = self.k, self.d
        body = st[: k * (d + 1)].reshape(k, d + 1)
        if len(rec) and (rec["key"][0] >> np.uint64(32)) != 0:
            i = 0
            for j in np.flatnonzero(body[:, d] == 0):    # fixed before any move
                if i >= len(rec):
                    break
                old = int(rec["label"][i])
                xq = rec["xq"][i, :d].astype(np.int64)
                body[old, :d] -= xq
                body[old, d] -= 1
                body[j, :d] = xq
                body[j, d] = 1
                i += 1
        self.stats.copy_(torch.from_numpy(st))
        self.halt, self.resume = 0, True
        self.iter_global()

    # ---------------- outputs
    def final(self):
        self.lab = R.assign(self.X, self.C)
        s = R.inertia_scale(self.q)
        w = np.ldexp(R.sqdist_rows(self.X, self.C[self.lab]).astype(np.float64), s).astype(np.uint64)
        lo = int(np.sum(w & np.uint64(0xFFFFFFFF), dtype=np.uint64))
        hi = int(np.sum(w >> np.uint64(32), dtype=np.uint64))
        self.limbs = [lo & 0xFFFFFFFF, (lo >> 32) + hi, 0]     # same integer as the device's limbs
        self.inertia = R.inertia_exact(R.sqdist_rows(self.X, self.C[self.lab]), s) if self.n else 0.0

    def labels(self):
        return torch.from_numpy(self.lab.copy())

    def centers(self):
        return torch.from_numpy(self.C.copy())

    def history(self, n):
        return np.asarray(self.hist_changed[:n], np.int64), np.asarray(self.hist_shift[:n])

    def layout_info(self):
        return dict(ncells=0, ntiles=0, grid=[])
