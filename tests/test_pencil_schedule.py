"""The pencil kernel's schedule (helix positions, systolic shifts, LDS record
hand-off, global ring with face rows) replayed on CPU by tools/pencil_emu.py
must reproduce the oracle. Guards the algorithm independently of the GPU."""
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))


@pytest.mark.parametrize("la,lb,lc,sop", [(64, 64, 64, 0), (47, 17, 128, 1), (60, 1, 65, 0),
                                          (130, 20, 200, 0), (5, 40, 3, 1), (300, 3, 40, 0)])
def test_emulated_schedule_matches_oracle(orc, la, lb, lc, sop):
    import pencil_emu
    rng = np.random.default_rng(la * 1000 + lb * 10 + lc)
    a, b, c = (rng.integers(0, 5, n) for n in (la, lb, lc))
    assert pencil_emu.emulate(a, b, c, sop=bool(sop)) == orc.score(a, b, c, orc.default_params(s3_mode=sop))
