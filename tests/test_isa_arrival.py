"""CPU: ISA check of k_updlists' early-issued arrival.

``arrive_issue`` (csrc/pcm_kernels.hpp) is an inline-asm ``global_atomic_add
... sc0`` whose returned value stays in flight through the block's list work
until ``arrive_read``'s explicit ``s_waitcnt vmcnt(0)`` + ``v_readfirstlane``.
hipcc's waitcnt pass does not see the asm, so nothing but the generated code
guarantees that the destination VGPR is not read, overwritten, copied or
spilled in between.  This test disassembles every k_updlists instantiation of
the built libpcmkm.so (the gfx950 code object extracted with llvm-objdump
--offloading) and checks, in program order from the atomic to the
``v_readfirstlane`` of its destination: no instruction names that VGPR (alone
or inside a register range), no scratch access (spill) occurs, and an
``s_waitcnt vmcnt(0)`` precedes the read.
"""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"


def _regs(operands: str):
    out = set()
    for a, b in re.findall(r"\bv\[(\d+):(\d+)\]", operands):
        out.update(range(int(a), int(b) + 1))
    for a in re.findall(r"\bv(\d+)\b", operands):
        out.add(int(a))
    return out


@pytest.fixture(scope="module")
def disasm(tmp_path_factory):
    from pcm_amd import _lib
    if not os.path.exists(_lib.SO_PATH):
        _lib.build()
    if not os.path.exists(OBJDUMP):
        pytest.skip("llvm-objdump not available")
    tmp = tmp_path_factory.mktemp("isa")
    so = tmp / "libpcmkm.so"
    shutil.copy(_lib.SO_PATH, so)
    subprocess.run([OBJDUMP, "--offloading", str(so)], cwd=tmp, check=True, capture_output=True)
    text = []
    for f in sorted(os.listdir(tmp)):
        if f.endswith("gfx950"):
            r = subprocess.run([OBJDUMP, "-d", "--mcpu=gfx950", str(tmp / f)], capture_output=True, text=True,
                               check=True)
            if "k_updlists" in r.stdout:
                text.append(r.stdout)
    assert text, "no code object with k_updlists"
    return "\n".join(text)


def _functions(text, name):
    heads = [(m.start(), m.group(1)) for m in re.finditer(r"^[0-9a-f]+ <([^>]+)>:", text, flags=re.M)]
    for k, (pos, sym) in enumerate(heads):
        if name in sym:
            end = heads[k + 1][0] if k + 1 < len(heads) else len(text)
            yield sym, [ln.split("//")[0].strip() for ln in text[pos:end].splitlines()[1:]]


def test_updlists_arrival_register_untouched_until_its_wait(disasm):
    seen = 0
    for sym, lines in _functions(disasm, "k_updlists"):
        if "Lb1EE" in sym:   # PUB = true: a dedicated publisher waits for plain arrivals (no returned place)
            continue
        lines = [ln for ln in lines if ln]
        at = [i for i, ln in enumerate(lines) if re.match(r"global_atomic_add v\d+, v\[\d+:\d+\], v\d+, off sc0$", ln)]
        assert len(at) == 1, (sym, [lines[i] for i in at])
        i0 = at[0]
        dst = int(re.match(r"global_atomic_add v(\d+),", lines[i0]).group(1))
        rd = next((i for i in range(i0 + 1, len(lines))
                   if re.match(rf"v_readfirstlane_b32 s\d+, v{dst}$", lines[i])), None)
        assert rd is not None, f"{sym}: no v_readfirstlane of v{dst} after the arrival"
        waited = False
        for ln in lines[i0 + 1:rd]:
            op, _, operands = ln.partition(" ")
            assert not op.startswith("scratch_"), f"{sym}: spill inside the arrival window: {ln}"
            assert dst not in _regs(operands), f"{sym}: v{dst} used before its wait: {ln}"
            if re.match(r"s_waitcnt .*vmcnt\(0\)", ln):
                waited = True
        assert waited, f"{sym}: no s_waitcnt vmcnt(0) between the arrival and its read"
        seen += 1
    assert seen >= 2   # the D = 1..3 x R = 1, 2 last-arriver instantiations
