"""Golden vectors from the reference's OWN stereo code (build container only).

The reference package ``members.rafael.disparity`` cannot be imported here
(ImportError on rasterio/cv2/osgeo, and ``constants.py:36-49`` creates
directories at import time -- SURVEY.md §0 forbids importing it again).  The
functions this build accelerates are plain NumPy, so this script reads their
source TEXT from /root/reference at generation time, extracts them with
``ast`` (no package import, no module-level code, no file I/O) and runs them on
synthetic inputs.  Only the resulting arrays are committed; neither this
script nor the tests embed any reference source.

  stereo/consistency.npz   members/rafael/disparity/processing.py:94-115
                           photoconsistency_map and disparity.py:229-250
                           left_right_consistency on 3 synthetic pairs (NaN,
                           out-of-range, below-min_disp and x.5 rounding cases)
  stereo/cloud.npz         members/rafael/disparity/plugin.py:147-192 (the
                           per-pair cloud assembly block, run as extracted
                           statements with utils.py:9-14 normalise_for_display)

Re-run with:  python tests/golden/make_stereo_golden.py
"""
import ast
import os
import types

import numpy as np

REF = "/root/reference/members/rafael/disparity"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "stereo")


def _functions(path, names):
    tree = ast.parse(open(path).read(), filename=path)
    mod = ast.Module(body=[n for n in tree.body if isinstance(n, ast.FunctionDef) and n.name in names],
                     type_ignores=[])
    ns = {"np": np}
    exec(compile(mod, path, "exec"), ns)
    return {k: ns[k] for k in names}


def _cloud_block():
    """The statements of plugin.py from `height_map = ...` to `points_coords = ...`."""
    path = os.path.join(REF, "plugin.py")
    tree = ast.parse(open(path).read(), filename=path)
    for node in ast.walk(tree):
        body = getattr(node, "body", None)
        if not isinstance(body, list):
            continue
        starts = [i for i, st in enumerate(body) if isinstance(st, ast.Assign) and
                  any(isinstance(t, ast.Name) and t.id == "height_map" for t in st.targets)]
        ends = [i for i, st in enumerate(body) if isinstance(st, ast.Assign) and
                any(isinstance(t, ast.Name) and t.id == "points_coords" for t in st.targets)]
        if starts and ends:
            mod = ast.Module(body=body[starts[0]:ends[0] + 1], type_ignores=[])
            return compile(mod, path, "exec"), body[starts[0]].lineno, body[ends[0]].lineno
    raise RuntimeError("cloud block not found")


def consistency_cases():
    rng = np.random.default_rng(20)
    cases = []
    for H, W in [(37, 53), (64, 200), (9, 300)]:
        left = rng.uniform(0, 255, (H, W)).astype(np.float32)
        right = rng.uniform(0, 255, (H, W)).astype(np.float32)
        ld = rng.uniform(-150, 60, (H, W))
        rd = -ld + rng.normal(0, 2, (H, W))
        ld[rng.random((H, W)) < 0.05] = np.nan                       # undefined
        ld.flat[rng.integers(0, H * W, 20)] = np.round(rng.uniform(-20, 20, 20)) + 0.5   # x.5 ties
        ld[:, :3] = -200.0                                           # below min_disp
        ld[-1, -4:] = 10 * W                                         # far out of range
        cases.append((left, right, ld, rd))
    return cases


def main():
    os.makedirs(OUT, exist_ok=True)
    f = _functions(os.path.join(REF, "processing.py"), ["photoconsistency_map"])
    g = _functions(os.path.join(REF, "disparity.py"), ["left_right_consistency"])
    out = {}
    for i, (left, right, ld, rd) in enumerate(consistency_cases()):
        out[f"left{i}"], out[f"right{i}"], out[f"ld{i}"], out[f"rd{i}"] = left, right, ld, rd
        out[f"photo{i}"] = f["photoconsistency_map"](left, right, ld, -(288 // 2))
        out[f"lr{i}"] = g["left_right_consistency"](ld, rd, -(288 // 2))
    np.savez_compressed(os.path.join(OUT, "consistency.npz"), **out)
    print("consistency.npz", len(out), "arrays")

    code, l0, l1 = _cloud_block()
    norm = _functions(os.path.join(REF, "utils.py"), ["normalise_for_display"])["normalise_for_display"]
    rng = np.random.default_rng(21)
    out = {"lines": np.array([l0, l1])}
    for i, (H, W) in enumerate([(90, 120), (200, 160)]):
        yy, xx = np.mgrid[0:H, 0:W]
        disp = -16.0 * (8 * np.sin(xx / 23.0) + 5 * np.cos(yy / 17.0) + 0.01 * xx + rng.normal(0, 0.3, (H, W)))
        disp[rng.random((H, W)) < 0.03] = 16.0 * 1000                # sentinel (beyond MAX_DISP / 2)
        disp[rng.random((H, W)) < 0.02] = np.nan
        valid = rng.random((H, W)) > 0.1
        ns = {"np": np, "disparity": disp, "validity_mask": valid, "C": types.SimpleNamespace(MAX_DISP=288),
              "normalise_for_display": norm, "layers": [], "PREFIX": "[Multi-day 3D Point Cloud]"}
        exec(code, ns)
        out[f"disp{i}"], out[f"valid{i}"] = disp, valid
        out[f"points{i}"] = ns["points_coords"]
        out[f"hnorm{i}"] = ns["property_table"]["height"]
        out[f"normal{i}"] = ns["normal"]
    np.savez_compressed(os.path.join(OUT, "cloud.npz"), **out)
    print("cloud.npz", {k: v.shape for k, v in out.items()})


if __name__ == "__main__":
    main()
