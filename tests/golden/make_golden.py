"""Generate tests/golden/golden.json -- TEST INFRASTRUCTURE.

Fixtures are data only: inputs + expected outputs. Expected values come from
the CPU restatement (oracle/tsa_oracle.c, literal RTL arithmetic) and, for
inputs inside the RTL envelope, from the cycle-level RTL model
(oracle/rtl_model.c); the script asserts the two agree before writing. Every
default-parameter case with lengths that are multiples of 8 (LA <= 512) also
records the 2-cycle RTL model's result (oracle/rtl_model_2cyc.c) and whether
it agrees -- by that model the 2-cycle variant's y-face SRAM banking breaks
some shapes, non-power-of-two cubes among them. Those
`rtl2_model` records are MODEL-DERIVED: one transliteration of the RTL, not
confirmed by a Verilog simulation (none exists in the image).
Inputs: the reference's own dat triple (dat/{A,B,C}_seq.dat, copied as
numbers), the testbench's all-A input (src/TriAlign_tb.sv:423-1960), prefixes,
homopolymers, seeded random triples (uniform + related), RTL and SOP scoring,
12/16-bit and unbounded arithmetic, and a low-bit (8) run that forces wraps.

Run:  python tests/golden/make_golden.py [/root/reference]
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle  # noqa: E402

REF = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
RTL2_SOURCE = "model-derived: oracle/rtl_model_2cyc.c transliteration, unverified by simulation"


def read_dat(path):
    with open(path) as f:
        return [int(t) for t in f.read().split()]


def in_env(la, lb, lc):
    return la % 8 == 0 and lb % 8 == 0 and lc % 8 == 0 and la <= 512 and lb <= la


def case(name, a, b, c, **pk):
    p = oracle.default_params(**pk)
    s, fin = oracle.score(a, b, c, p, final_states=True)
    s2 = oracle.score(a, b, c, p, method="diag")
    assert s == s2, (name, s, s2)
    rec = {"name": name, "a": list(map(int, a)), "b": list(map(int, b)), "c": list(map(int, c)),
           "params": {k: getattr(p, k) for k, _ in p._fields_}, "score": s, "final7": list(fin)}
    default = (p.match, p.mismatch, p.gap_open, p.gap_extend, p.s3_mode, p.score_bits) == (1, -1, 2, 1, 0, 12)
    if default and in_env(len(a), len(b), len(c)):
        r, isx, cyc = oracle.rtl_run(a, b, c)
        assert not isx and r == s, (name, r, isx, s)
        rec["rtl_model"] = {"score": r, "cycles": cyc}
    if default and all(n % 8 == 0 for n in (len(a), len(b), len(c))) and len(a) <= 512:
        r2, isx2, cyc2 = oracle.rtl2_run(a, b, c)
        rec["rtl2_model"] = {"score": r2, "x": isx2, "cycles": cyc2, "agrees": (not isx2) and r2 == s,
                             "source": RTL2_SOURCE}
    return rec


def main():
    A = read_dat(os.path.join(REF, "dat", "A_seq.dat"))
    B = read_dat(os.path.join(REF, "dat", "B_seq.dat"))
    C = read_dat(os.path.join(REF, "dat", "C_seq.dat"))
    cases = [case("dat", A, B, C), case("dat_sop", A, B, C, s3_mode=1),
             case("dat_wide", A, B, C, score_bits=0), case("dat_prefix8", A[:8], B[:8], C[:8]),
             case("dat_prefix16", A[:16], B[:16], C[:16]),
             case("tb_allA_64", [0] * 64, [0] * 64, [0] * 64),
             case("homopolymers_16", [0] * 16, [1] * 16, [2] * 16)]
    for n in (8, 16, 24, 40):
        cases.append(case(f"allA_{n}", [0] * n, [0] * n, [0] * n))
    # N aliases A through the 2-bit PE symbol registers (src/PE_1cyc.v:63-66)
    cases.append(case("N_alias", [4, 0, 4, 1] * 4, [0, 4, 0, 1] * 4, [4, 4, 0, 1] * 4))
    rng = np.random.default_rng(20241015)
    for k in range(24):
        la, lb, lc = (int(v) for v in rng.integers(1, 41, 3))
        a, b, c = (rng.integers(0, 5, n).astype(np.uint8) for n in (la, lb, lc))
        cases.append(case(f"rand_{k}", a, b, c, s3_mode=int(k % 2)))
    for k in range(8):  # in-envelope random: RTL model agreement recorded
        la = 8 * int(rng.integers(1, 7)); lb = 8 * int(rng.integers(1, la // 8 + 1)); lc = 8 * int(rng.integers(1, 7))
        a, b, c = (rng.integers(0, 4, n).astype(np.uint8) for n in (la, lb, lc))
        cases.append(case(f"env_{k}", a, b, c))
    for k in range(4):  # related: high scores
        r2 = np.random.default_rng(100 + k)
        a = r2.integers(0, 4, 48).astype(np.uint8)
        b = a.copy(); c = a.copy()
        b[r2.random(48) < 0.1] = r2.integers(0, 4, int((r2.random(48) < 0.1).sum() or 1))[0]
        c[r2.random(48) < 0.1] = 3
        cases.append(case(f"related_{k}", a, b, c))
    # low-bit arithmetic forces the RTL's wordsize wrap (src/PE_1cyc.v:127-133)
    cases.append(case("wrap8_allA_48", [0] * 48, [0] * 48, [0] * 48, score_bits=8))
    cases.append(case("wrap6_rand", rng.integers(0, 4, 30), rng.integers(0, 4, 30), rng.integers(0, 4, 30), score_bits=6))
    cases.append(case("bits16_params", rng.integers(0, 4, 20), rng.integers(0, 4, 25), rng.integers(0, 4, 18),
                      match=5, mismatch=-4, gap_open=10, gap_extend=1, score_bits=16))
    # cubes and near-cubes for the 2-cycle variant: power-of-two and other
    # sizes, LB != LA, a single z pencil (no y face ever read)
    r3 = np.random.default_rng(2026)
    for la, lb, lc in ((8, 8, 8), (16, 16, 16), (24, 24, 24), (32, 32, 32), (40, 40, 40),
                       (48, 48, 48), (56, 56, 56), (64, 64, 64), (72, 72, 72), (80, 80, 80),
                       (96, 96, 96), (64, 64, 32), (64, 32, 64), (32, 64, 8), (48, 48, 96)):
        a, b, c = (r3.integers(0, 4, n).astype(np.uint8) for n in (la, lb, lc))
        cases.append(case(f"cube2_{la}x{lb}x{lc}", a, b, c))
    out = {"generator": "tests/golden/make_golden.py", "oracle": "oracle/tsa_oracle.c (+ rtl_model.c, rtl_model_2cyc.c)",
           "rtl2_model_source": RTL2_SOURCE, "cases": cases}
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden.json")
    with open(path, "w") as f:
        json.dump(out, f, separators=(",", ":"))
    print(f"wrote {len(cases)} cases to {path}")


if __name__ == "__main__":
    main()
