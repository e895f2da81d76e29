"""The single-cube lap kernel's schedule (csrc/lap_kernel.hip) replayed on the
CPU by tools/lap_emu.py -- two DP rows per wave in the 16-bit halves, laps of
2*NW rows chained through tagged y records, z-tiles of 64*M positions chained
through z records -- must reproduce the oracle exactly, including the tile and
lap seams the adversarial inputs stress (all-mismatch and all-match cubes)."""
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
from lap_emu import emulate  # noqa: E402

CASES = [((20, 11, 70), 2, 1), ((5, 3, 1), 2, 1), ((1, 1, 1), 2, 1), ((30, 9, 130), 2, 2),
         ((7, 17, 64), 4, 1), ((40, 4, 65), 2, 1), ((50, 8, 129), 4, 2), ((12, 13, 300), 2, 4),
         # the seam cell (1, y, 64M+1) of a deep cube: its step-0 inputs come from the
         # left tile's records ZT-2 / ZT-1 (all-mismatch exposes a face value there)
         ((10, 20, 66), 2, 1), ((20, 40, 70), 2, 1), ((16, 24, 130), 4, 2)]


@pytest.mark.parametrize("sk", [1, 2])
@pytest.mark.parametrize("shape,nw,m", CASES)
@pytest.mark.parametrize("kind", ["random", "mismatch", "match"])
def test_lap_schedule_vs_oracle(orc, shape, nw, m, kind, sk):
    la, lb, lc = shape
    rng = np.random.default_rng(la * 7 + lb * 3 + lc)
    if kind == "random":
        a, b, c = (rng.integers(0, 4, n).astype(np.uint8) for n in shape)
    elif kind == "mismatch":
        a, b, c = (np.full(n, v, np.uint8) for n, v in zip(shape, (0, 1, 2)))
    else:
        a, b, c = (np.zeros(n, np.uint8) for n in shape)
    sop = bool(rng.integers(0, 2))
    op = orc.default_params(score_bits=16, s3_mode=int(sop))
    assert emulate(a, b, c, sop=sop, NW=nw, M=m, SK=sk) == orc.score(a, b, c, op)
