"""Kernel resources from the gfx950 code objects (tools/kernel_meta.py), no
GPU needed: no kernel of the product path uses scratch (a private segment
means a spilled or dynamically indexed register array), and the lap grid's
residency is capped by the per-SIMD register bound where the occupancy API
reads one workgroup per CU high (MI355X_MICROARCH.md:463)."""
import ctypes
import glob
import os
import re
import subprocess
import sys

import pytest

from conftest import PKG_DIR

sys.path.insert(0, os.path.join(PKG_DIR, "tools"))


@pytest.fixture(scope="module")
def meta(tsa):
    import kernel_meta
    objs = sorted(glob.glob(os.path.join(PKG_DIR, "build", "*.o")))
    objs = [o for o in objs if not o.endswith("kernel_meta.o")]
    if not objs:
        pytest.skip("no build objects (prebuilt library only)")
    return kernel_meta.object_meta_all(objs)


def test_every_kernel_is_listed(meta):
    names = " ".join(meta)
    for k in ("pencil_kernel", "lap_kernel", "literal_kernel", "plane_step_kernel", "tb_walk", "lap_certify"):
        assert k in names, k


def test_no_scratch_outside_the_widest_helix(meta):
    """Only the M = 8 helix (LC 513..1024, 4 f16/int16 pairs x 8 registers x 7
    states) runs out of the 256 VGPRs a 512-thread workgroup allows; every
    other kernel, the literal helix and the lap kernel included, keeps its
    registers in registers."""
    scratch = {k: v["scratch"] for k, v in meta.items() if v.get("scratch", 0)}
    for k in scratch:
        assert k.startswith("_ZN3tsa13pencil_kernelILi8E"), (k, scratch[k])
    assert all(s <= 512 for s in scratch.values())
    assert not [k for k in scratch if "literal_kernel" in k or "pencil_kernelILi2E" in k]


def test_generated_table_matches_objects(meta):
    cpp = os.path.join(PKG_DIR, "build", "kernel_meta.cpp")
    rows = dict((m.group(1), int(m.group(2))) for m in re.finditer(r'\{"([^"]+)", (\d+),', open(cpp).read()))
    assert rows == {k: v["sgpr"] for k, v in meta.items()}


def vgpr_waves(vgpr):
    return min(8, 512 // ((vgpr + 7) // 8 * 8))


def sgpr_waves(sgpr):
    return 800 // (((sgpr + 15) // 16) * 16 + 16)


@pytest.mark.parametrize("M", [1, 2, 4])
@pytest.mark.parametrize("NW", [4, 8])
def test_lap_residency_sgpr_cap(tsa, meta, M, NW):
    """lap_simd_blocks_per_cu(M, NW, f16, sop, lit) = the SGPR / VGPR waves per
    SIMD over the waves a workgroup may put on one SIMD, taken over EVERY
    instantiation of that shape and form -- single-device, checked (CHK) and
    split (SYS) -- so the plan holds whichever of them launches; the literal
    form (LIT, int16, M <= 2) has its own."""
    fn = getattr(tsa.lib(), "_ZN3tsa22lap_simd_blocks_per_cuEiibbb")
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_bool, ctypes.c_bool, ctypes.c_bool]
    forms = [(f16, sop, False) for f16 in (False, True) for sop in (False, True)]
    if M <= 2:
        forms += [(False, sop, True) for sop in (False, True)]
    for f16, sop, lit in forms:
        pres = [f"_ZN3tsa10lap_kernelILi{M}ELi{NW}ELb{int(f16)}ELb{int(sop)}ELb{chk}ELb{sys}ELb{int(lit)}E"
                for chk in (0, 1) for sys in (0, 1)]
        rows = [v for k, v in meta.items() if any(k.startswith(p) for p in pres)]
        sg = max(v["sgpr"] for v in rows)
        vg = max(v["vgpr"] + v.get("agpr", 0) for v in rows)
        want = min(sgpr_waves(sg), vgpr_waves(vg)) // ((NW + 1 + 3) // 4)
        assert fn(M, NW, f16, sop, lit) == want, (f16, sop, lit)
        assert want >= 1
        # no instantiation of the form (checked / split included) admits fewer
        # workgroups per CU than the bound the plan uses
        for v in rows:
            own = min(sgpr_waves(v["sgpr"]), vgpr_waves(v["vgpr"] + v.get("agpr", 0))) // ((NW + 1 + 3) // 4)
            assert own >= want
    if M <= 2:  # the literal form keeps its registers in registers
        lit = [k for k in meta if re.match(rf"_ZN3tsa10lap_kernelILi{M}ELi{NW}ELb0ELb[01]ELb0ELb0ELb1E(Lb0E)?E", k)]
        assert len(lit) == 2 and all(meta[k].get("scratch", 0) == 0 for k in lit)
    # measured (tools/lap_trace.py start stamps): M = 1 NW = 8 runs two
    # 9-wave workgroups per CU (the f16 forms, <= 80 VGPRs; the int16 form's
    # checked instantiation takes 85, so that form plans one); M = 2 (96
    # VGPRs, 5 waves per SIMD) one -- the occupancy API said 2 -- so its
    # 1024^3 grid runs two dispatch rounds
    if NW == 8 and M == 1:
        assert fn(M, NW, True, False, False) == 2 and fn(M, NW, True, True, False) == 2
    if NW == 8 and M == 2:
        assert fn(M, NW, False, False, False) == 1
    # the edge the guide names: 97-112 SGPRs leave 6 waves per SIMD, 7 below it
    assert sgpr_waves(106) == 6 and sgpr_waves(80) == 8
    assert vgpr_waves(96) == 5 and vgpr_waves(80) == 6


def test_isa_loops_counts_the_lap_step():
    """tools/isa_loops.py (the per-step ISA census DESIGN.md 4.4 quotes) finds
    the four-step group loop of the single-cube bench kernel
    (lap_kernel<1,4,f16>, RTL s3) in the built object: a loop whose no-spin
    pass issues 4 steps' worth of VALU (the cell's 17 v_pk_maximum3 per step
    alone is 68 per pass) and at most 80 VALU per step."""
    obj = os.path.join(PKG_DIR, "build", "lap_kernel.o")
    if not os.path.exists(obj):
        pytest.skip("no built lap_kernel.o (make)")
    sys.path.insert(0, os.path.join(PKG_DIR, "tools"))
    import isa_loops
    ins = isa_loops.kernel_insts(isa_loops.disassemble(obj), "lap_kernelILi1ELi4ELb1ELb0ELb0ELb0ELb0ELb0E")
    assert ins, "kernel not found"
    loops = [(t, a) for a, mn, ops in ins if isa_loops.BR.match(mn)
             for t in [isa_loops.target(ops, a)] if t is not None and t < a]
    passes = []
    for head, tail in loops:
        inner = [(h, t) for h, t in loops if head < h and t < tail]
        c = isa_loops.fast_path(ins, head, tail, inner)
        if c["valu"] and c["ds"] >= 20:  # a step loop: 6+ LDS ops per step
            passes.append(c)
    group = [c for c in passes if 4 * 60 <= c["valu"] <= 4 * 80]
    assert group, passes
