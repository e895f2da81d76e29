"""The pencil kernel's schedule (helix positions, systolic shifts, LDS record
hand-off, global ring with face rows) replayed on CPU by tools/pencil_emu.py
must reproduce the oracle. Guards the algorithm independently of the GPU."""
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))


@pytest.mark.parametrize("skew", [1, 2])
@pytest.mark.parametrize("la,lb,lc,sop", [(64, 64, 64, 0), (47, 17, 128, 1), (60, 1, 65, 0),
                                          (130, 20, 200, 0), (5, 40, 3, 1), (300, 3, 40, 0)])
def test_emulated_schedule_matches_oracle(orc, la, lb, lc, sop, skew):
    # skew 2 is the kernel's M <= 2 schedule (waves two steps apart, four
    # record slots per wave), skew 1 its M >= 4 one
    import pencil_emu
    rng = np.random.default_rng(la * 1000 + lb * 10 + lc)
    a, b, c = (rng.integers(0, 5, n) for n in (la, lb, lc))
    got = pencil_emu.emulate(a, b, c, sop=bool(sop), skew=skew)
    assert got == orc.score(a, b, c, orc.default_params(s3_mode=sop))
