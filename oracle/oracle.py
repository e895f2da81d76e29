"""TEST INFRASTRUCTURE -- ctypes binding of the CPU oracle (oracle/_build/libtsa_oracle.so).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use
this module, and only as the checker / CPU baseline. The product library
(hw-accelerator-three-sequence-alignment_amd/lib/libtrialign.so) never loads it.

Functions mirror oracle/tsa_oracle.h; every one cites the RTL lines it restates
there (src/PE_1cyc.v:1-32,55-66,159-218; src/TriAlign_1cyc.v:141-142,155-190).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SO_PATH = os.path.join(ROOT, "oracle", "_build", "libtsa_oracle.so")


class OracleParams(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int32) for n in
                ("match", "mismatch", "gap_open", "gap_extend", "s3_mode", "score_bits")]


def default_params(**kw) -> OracleParams:
    p = OracleParams(1, -1, 2, 1, 0, 12)
    for k, v in kw.items():
        setattr(p, k, v)
    return p


def _build():
    subprocess.run(["make", "-s", "oracle"], cwd=ROOT, check=True)


_lib = None


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(SO_PATH):
            _build()
        L = ctypes.CDLL(SO_PATH)
        u8p, i32p, i64p = (ctypes.POINTER(ctypes.c_uint8), ctypes.POINTER(ctypes.c_int32),
                           ctypes.POINTER(ctypes.c_int64))
        pp = ctypes.POINTER(OracleParams)
        three = [u8p, ctypes.c_int32, u8p, ctypes.c_int32, u8p, ctypes.c_int32]
        for name in ("tsao_score_xplane", "tsao_score_diag"):
            getattr(L, name).argtypes = three + [pp, i32p, i32p]
            getattr(L, name).restype = ctypes.c_int
        L.tsao_score_msg.argtypes = three + [pp, i32p]
        L.tsao_score_msg.restype = ctypes.c_int
        L.tsao_state_range.argtypes = three + [pp, i32p, i32p]
        L.tsao_state_range.restype = ctypes.c_int
        L.tsao_score_batch.argtypes = [u8p, i64p, ctypes.c_int32, pp, i32p, ctypes.c_int32]
        L.tsao_score_batch.restype = ctypes.c_int
        L.tsao_rtl_run.argtypes = three + [ctypes.c_int32, i32p, i32p,
                                           ctypes.POINTER(ctypes.c_int64)]
        L.tsao_rtl_run.restype = ctypes.c_int
        L.tsao_rtl2_run.argtypes = three + [i32p, i32p, ctypes.POINTER(ctypes.c_int64)]
        L.tsao_rtl2_run.restype = ctypes.c_int
        L.tsao_align.argtypes = three + [pp, i32p, u8p, ctypes.c_int32, i32p, i32p]
        L.tsao_align.restype = ctypes.c_int
        L.tsao_gen_uniform.argtypes = [ctypes.c_uint64, u8p, ctypes.c_int32]
        L.tsao_gen_uniform.restype = None
        L.tsao_now.argtypes = []
        L.tsao_now.restype = ctypes.c_double
        _lib = L
    return _lib


def _u8(s) -> np.ndarray:
    return np.ascontiguousarray(np.asarray(s, dtype=np.uint8))


def _p(a, t):
    return a.ctypes.data_as(ctypes.POINTER(t))


def score(a, b, c, params: OracleParams | None = None, method: str = "xplane",
          final_states: bool = False):
    """Literal restatement score (method xplane|diag) or factored form (msg)."""
    p = params or default_params()
    A, B, C = _u8(a), _u8(b), _u8(c)
    out = ctypes.c_int32(0)
    fin = (ctypes.c_int32 * 7)()
    args = [_p(A, ctypes.c_uint8), len(A), _p(B, ctypes.c_uint8), len(B),
            _p(C, ctypes.c_uint8), len(C), ctypes.byref(p), ctypes.byref(out)]
    if method == "msg":
        rc = lib().tsao_score_msg(*args)
    else:
        fn = lib().tsao_score_xplane if method == "xplane" else lib().tsao_score_diag
        rc = fn(*args, fin)
    if rc:
        raise ValueError(f"oracle rc={rc}")
    if final_states:
        return int(out.value), tuple(int(v) for v in fin)
    return int(out.value)


def align(a, b, c, params: OracleParams | None = None):
    """Traceback of the literal form: (score, (x0, y0, z0), moves) with moves
    the state index of each alignment column in forward order."""
    p = params or default_params()
    A, B, C = _u8(a), _u8(b), _u8(c)
    cap = len(A) + len(B) + len(C)
    mv = np.zeros(cap, dtype=np.uint8)
    sc, n = ctypes.c_int32(0), ctypes.c_int32(0)
    st = (ctypes.c_int32 * 3)()
    rc = lib().tsao_align(_p(A, ctypes.c_uint8), len(A), _p(B, ctypes.c_uint8), len(B),
                          _p(C, ctypes.c_uint8), len(C), ctypes.byref(p), ctypes.byref(sc),
                          _p(mv, ctypes.c_uint8), cap, ctypes.byref(n), st)
    if rc:
        raise ValueError(f"oracle rc={rc}")
    return int(sc.value), tuple(int(v) for v in st), mv[: n.value].copy()


def state_range(a, b, c, params: OracleParams | None = None) -> tuple[int, int]:
    p = params or default_params()
    A, B, C = _u8(a), _u8(b), _u8(c)
    lo, hi = ctypes.c_int32(0), ctypes.c_int32(0)
    rc = lib().tsao_state_range(_p(A, ctypes.c_uint8), len(A), _p(B, ctypes.c_uint8), len(B),
                                _p(C, ctypes.c_uint8), len(C), ctypes.byref(p),
                                ctypes.byref(lo), ctypes.byref(hi))
    if rc:
        raise ValueError(f"oracle rc={rc}")
    return int(lo.value), int(hi.value)


def rtl_run(a, b, c, a_total_len: int = 512) -> tuple[int, bool, int]:
    """Cycle-level RTL model (oracle/rtl_model.c): (score, score_is_x, cycles)."""
    A, B, C = _u8(a), _u8(b), _u8(c)
    s, isx, cyc = ctypes.c_int32(0), ctypes.c_int32(0), ctypes.c_int64(0)
    rc = lib().tsao_rtl_run(_p(A, ctypes.c_uint8), len(A), _p(B, ctypes.c_uint8), len(B),
                            _p(C, ctypes.c_uint8), len(C), a_total_len, ctypes.byref(s),
                            ctypes.byref(isx), ctypes.byref(cyc))
    if rc:
        raise ValueError(f"rtl model rc={rc}")
    return int(s.value), bool(isx.value), int(cyc.value)


def rtl2_run(a, b, c) -> tuple[int, bool, int]:
    """Cycle-level model of the 2-cycle RTL variant (oracle/rtl_model_2cyc.c):
    (score, score_is_x, cycles)."""
    A, B, C = _u8(a), _u8(b), _u8(c)
    s, isx, cyc = ctypes.c_int32(0), ctypes.c_int32(0), ctypes.c_int64(0)
    rc = lib().tsao_rtl2_run(_p(A, ctypes.c_uint8), len(A), _p(B, ctypes.c_uint8), len(B),
                             _p(C, ctypes.c_uint8), len(C), ctypes.byref(s), ctypes.byref(isx),
                             ctypes.byref(cyc))
    if rc:
        raise ValueError(f"rtl2 model rc={rc}")
    return int(s.value), bool(isx.value), int(cyc.value)


def score_batch(seqs: np.ndarray, offsets: np.ndarray, params: OracleParams | None = None,
                nthreads: int = 1) -> np.ndarray:
    p = params or default_params()
    seqs = _u8(seqs)
    offsets = np.ascontiguousarray(offsets, dtype=np.int64)
    n = (len(offsets) - 1) // 3
    out = np.zeros(max(n, 1), dtype=np.int32)
    rc = lib().tsao_score_batch(_p(seqs, ctypes.c_uint8), _p(offsets, ctypes.c_int64), n,
                                ctypes.byref(p), _p(out, ctypes.c_int32), nthreads)
    if rc:
        raise ValueError(f"oracle rc={rc}")
    return out[:n]


def gen_uniform(seed: int, length: int) -> np.ndarray:
    out = np.zeros(max(length, 1), dtype=np.uint8)
    lib().tsao_gen_uniform(ctypes.c_uint64(seed), _p(out, ctypes.c_uint8), length)
    return out[:length]


def now() -> float:
    return float(lib().tsao_now())
