"""trialign-mi355x host API: Python mirror of the reference's TRIALIGN boundary.

The reference exposes one operator: the ``TRIALIGN`` module
(``src/TriAlign_1cyc.v:1-22``) -- parameters ``A/B/C_TOTAL_LEN, PE_LEN,
SCORE_BITS, SRAM_ADDR_BITS``; a ``start_align`` pulse; sequence lengths on
``A_idx/B_idx/C_idx``; symbols pulled through ``A/B/C_addr``/``*_symbol``; and
``Score``/``finish`` out. Its only caller is the testbench FSM
(``src/TriAlign_tb.sv:279-353``), which prints ``TriAlign Score: <n>``.

This module keeps that shape (:class:`TriAlign` with the same parameter names
and a ``run`` that plays start->finish) over the C-ABI in ``include/trialign.h``
(``lib/libtrialign.so``, HIP/gfx950). There is no CPU fallback: if the shared
library is missing, importing this module raises; on a host without a GPU every
scoring call raises :class:`TsaError` with ``TSA_ENODEV``.

Load it with :func:`load` from the repo root helpers, or::

    spec = importlib.util.spec_from_file_location(
        "tsa_amd", "<repo>/hw-accelerator-three-sequence-alignment_amd/__init__.py")
"""
from __future__ import annotations

import ctypes
import os
from typing import Iterable, Optional, Sequence

import numpy as np

# One HIP runtime per process: torch ships its own libamdhip64 (soname
# libamdhip64.so.7, NEEDED as "libamdhip64.so"). Importing torch first makes
# libtrialign.so bind to that same runtime, so torch device pointers and
# streams passed through the C-ABI are valid; loading ours first would pull a
# second runtime from /opt/rocm and break torch's device init.
import torch  # noqa: F401  (device memory / streams plumbing)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "lib", "libtrialign.so")

TSA_OK = 0
TSA_EINVAL = -1
TSA_ERANGE = -2
TSA_ENODEV = -3
TSA_EDEVICE = -4
TSA_ENOMEM = -5
TSA_EINTERNAL = -6

S3_RTL = 0
S3_SOP = 1

KERNEL_AUTO = 0
KERNEL_PLANE = 1
KERNEL_PENCIL = 2
KERNEL_CHECKED = 3
KERNELS = {"auto": KERNEL_AUTO, "plane": KERNEL_PLANE, "pencil": KERNEL_PENCIL,
           "checked": KERNEL_CHECKED}

# testbench symbol encoding, src/TriAlign_tb.sv:42-46
SYMBOLS = {"A": 0, "T": 1, "C": 2, "G": 3, "N": 4}

# The C-ABI entry points include/trialign.h declares (checked by the tests).
EXPORTS = (
    "tsa_default_params", "tsa_validate", "tsa_score_gpu", "tsa_score_gpu_ex",
    "tsa_score_batch", "tsa_batch_workspace_size", "tsa_score_batch_async",
    "tsa_device_count", "tsa_strerror", "tsa_version", "tsa_describe_plan", "tsa_align_gpu",
    "tsa_fallback_count", "tsa_check_fallback_count", "tsa_score_batch_async_p2", "tsa_pack2",
    "tsa_score_gpu_multi", "tsa_score_batch_devices",
)

# Score of a triple the device could not score (include/trialign.h).
SCORE_INVALID = -(2 ** 31)
# Score of a triple the checked kernel could not certify (rescore with PLANE).
SCORE_UNCERTIFIED = -(2 ** 31) + 1

# Alignment columns (tsa_align_gpu): the state of each column and which of
# (A, B, C) it consumes -- the predecessor offsets of src/PE_1cyc.v:164-218.
MOVES = ("M", "Ix", "Iy", "Iz", "Ixy", "Iyz", "Ixz")
MOVE_CONSUMES = ((1, 1, 1), (1, 0, 0), (0, 1, 0), (0, 0, 1), (1, 1, 0), (0, 1, 1), (1, 0, 1))


class TsaParams(ctypes.Structure):
    """``tsa_params`` (include/trialign.h); defaults = PE localparams
    MATCH=1, MISMATCH=-1, GO=2, GE=1 (src/PE_1cyc.v:55-58), RTL s3,
    SCORE_BITS=12 (src/TriAlign_tb.sv:56)."""

    _fields_ = [
        ("match", ctypes.c_int32),
        ("mismatch", ctypes.c_int32),
        ("gap_open", ctypes.c_int32),
        ("gap_extend", ctypes.c_int32),
        ("s3_mode", ctypes.c_int32),
        ("score_bits", ctypes.c_int32),
    ]

    @classmethod
    def default(cls, **kw) -> "TsaParams":
        p = cls(1, -1, 2, 1, S3_RTL, 12)
        for k, v in kw.items():
            setattr(p, k, v)
        return p

    def as_tuple(self):
        return tuple(getattr(self, f) for f, _ in self._fields_)


class TsaError(RuntimeError):
    def __init__(self, rc: int, what: str = ""):
        self.rc = rc
        msg = _lib.tsa_strerror(rc).decode() if _lib is not None else str(rc)
        super().__init__(f"{what}: {msg} ({rc})" if what else f"{msg} ({rc})")


def _load_lib() -> ctypes.CDLL:
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"libtrialign.so not built ({LIB_PATH}); run `make` or __graft_entry__.build()")
    lib = ctypes.CDLL(LIB_PATH)
    u8p = ctypes.POINTER(ctypes.c_uint8)
    i32p = ctypes.POINTER(ctypes.c_int32)
    i64p = ctypes.POINTER(ctypes.c_int64)
    pp = ctypes.POINTER(TsaParams)
    lib.tsa_default_params.argtypes = [pp]
    lib.tsa_default_params.restype = None
    lib.tsa_validate.argtypes = [u8p, ctypes.c_int32, u8p, ctypes.c_int32, u8p, ctypes.c_int32, pp]
    lib.tsa_score_gpu.argtypes = [u8p, ctypes.c_int32, u8p, ctypes.c_int32, u8p, ctypes.c_int32,
                                  pp, i32p, ctypes.c_int32]
    lib.tsa_score_gpu_ex.argtypes = [u8p, ctypes.c_int32, u8p, ctypes.c_int32, u8p,
                                     ctypes.c_int32, pp, ctypes.c_int32, i32p, i32p,
                                     ctypes.c_int32]
    lib.tsa_score_batch.argtypes = [u8p, i64p, ctypes.c_int32, pp, i32p, ctypes.c_int32]
    lib.tsa_score_batch_devices.argtypes = [u8p, i64p, ctypes.c_int32, pp, i32p, i32p,
                                            ctypes.c_int32]
    lib.tsa_batch_workspace_size.argtypes = [ctypes.c_int32] * 4 + [pp, ctypes.c_int32,
                                                                   ctypes.POINTER(ctypes.c_size_t)]
    lib.tsa_score_batch_async.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int32,
                                          ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, pp,
                                          ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p,
                                          ctypes.c_size_t, ctypes.c_void_p]
    lib.tsa_describe_plan.argtypes = [ctypes.c_int32] * 4 + [pp, ctypes.c_int32, ctypes.c_int32,
                                                            ctypes.c_char_p, ctypes.c_size_t]
    lib.tsa_align_gpu.argtypes = [u8p, ctypes.c_int32, u8p, ctypes.c_int32, u8p, ctypes.c_int32,
                                  pp, i32p, u8p, ctypes.c_int32, i32p, i32p, ctypes.c_int32]
    lib.tsa_score_gpu_multi.argtypes = [u8p, ctypes.c_int32, u8p, ctypes.c_int32, u8p,
                                        ctypes.c_int32, pp, i32p, ctypes.c_int32, i32p,
                                        ctypes.POINTER(ctypes.c_double)]
    lib.tsa_fallback_count.argtypes = []
    lib.tsa_fallback_count.restype = ctypes.c_int64
    lib.tsa_score_batch_async_p2.argtypes = lib.tsa_score_batch_async.argtypes
    lib.tsa_pack2.argtypes = [u8p, ctypes.c_int64, u8p]
    lib.tsa_check_fallback_count.argtypes = []
    lib.tsa_check_fallback_count.restype = ctypes.c_int64
    lib.tsa_device_count.argtypes = []
    lib.tsa_strerror.argtypes = [ctypes.c_int]
    lib.tsa_strerror.restype = ctypes.c_char_p
    lib.tsa_version.argtypes = []
    lib.tsa_version.restype = ctypes.c_char_p
    for name in ("tsa_validate", "tsa_score_gpu", "tsa_score_gpu_ex", "tsa_score_batch",
                 "tsa_batch_workspace_size", "tsa_score_batch_async", "tsa_device_count",
                 "tsa_describe_plan", "tsa_align_gpu", "tsa_score_batch_async_p2", "tsa_pack2",
                 "tsa_score_gpu_multi", "tsa_score_batch_devices"):
        getattr(lib, name).restype = ctypes.c_int
    return lib


_lib: Optional[ctypes.CDLL] = None
_lib = _load_lib()


def lib() -> ctypes.CDLL:
    return _lib


def version() -> str:
    """tsa_version(): "trialign-mi355x gfx950 src=<hash>" -- the hash of the
    sources the loaded binary was built from (srchash.py)."""
    return _lib.tsa_version().decode()


def source_hash() -> str:
    """Hash of the library sources in this tree (srchash.py)."""
    from . import srchash
    return srchash.source_hash()


def build_info() -> dict:
    """Which binary is loaded and whether it was built from this tree."""
    v = version()
    tree = source_hash()
    return {"version": v, "lib": LIB_PATH, "tree_src": tree, "current": v.endswith("src=" + tree)}


def device_count() -> int:
    return int(_lib.tsa_device_count())


def fallback_count() -> int:
    """Lap hand-offs that timed out on the synchronous paths so far (each was
    rescored without the lap schedule); 0 in a healthy run."""
    return int(_lib.tsa_fallback_count())


def check_fallback_count() -> int:
    """Triples the checked kernel could not certify on the synchronous paths
    so far (each was rescored in the literal arithmetic, kernel="plane")."""
    return int(_lib.tsa_check_fallback_count())


def _as_u8(seq) -> np.ndarray:
    if isinstance(seq, str):
        try:
            seq = [SYMBOLS[ch] for ch in seq.upper()]
        except KeyError as e:
            raise TsaError(TSA_EINVAL, f"symbol {e}") from None
    src = np.asarray(seq)
    if src.dtype != np.uint8:
        # no silent wrap into a valid symbol (256 -> 0 = 'A', -1 -> 255)
        if src.size and (src.dtype.kind not in "iub" or int(src.min()) < 0 or int(src.max()) > 255):
            raise TsaError(TSA_EINVAL, "symbols must be integers 0..4")
    arr = np.ascontiguousarray(src, dtype=np.uint8)
    if arr.ndim != 1:
        raise TsaError(TSA_EINVAL, "sequence must be 1-D")
    return arr


def _ptr(arr: np.ndarray, ctype):
    return arr.ctypes.data_as(ctypes.POINTER(ctype))


def _check(rc: int, what: str):
    if rc != TSA_OK:
        raise TsaError(rc, what)


def validate(a, b, c, params: Optional[TsaParams] = None) -> int:
    """tsa_validate: returns the rc (0 = ok) without raising."""
    p = params or TsaParams.default()
    A, B, C = _as_u8(a), _as_u8(b), _as_u8(c)
    return int(_lib.tsa_validate(_ptr(A, ctypes.c_uint8), len(A), _ptr(B, ctypes.c_uint8), len(B),
                                 _ptr(C, ctypes.c_uint8), len(C), ctypes.byref(p)))


def score(a, b, c, params: Optional[TsaParams] = None, kernel: str | int = "auto",
          device: int = 0, final_states: bool = False):
    """Optimal 3-D DP score of one triple on GPU ``device``.

    ``final_states=True`` also returns the 7 states {M,Ix,Iy,Iz,Ixy,Iyz,Ixz}
    of cell (LA,LB,LC) (runs the literal kernels: kernel="plane")."""
    p = params or TsaParams.default()
    A, B, C = _as_u8(a), _as_u8(b), _as_u8(c)
    k = KERNELS[kernel] if isinstance(kernel, str) else int(kernel)
    out = ctypes.c_int32(0)
    fin = (ctypes.c_int32 * 7)()
    rc = _lib.tsa_score_gpu_ex(_ptr(A, ctypes.c_uint8), len(A), _ptr(B, ctypes.c_uint8), len(B),
                               _ptr(C, ctypes.c_uint8), len(C), ctypes.byref(p), k,
                               ctypes.byref(out), fin if final_states else None, device)
    _check(rc, "tsa_score_gpu_ex")
    if final_states:
        return int(out.value), tuple(int(v) for v in fin)
    return int(out.value)


def score_multi(a, b, c, devices: Sequence[int], params: Optional[TsaParams] = None):
    """One triple's cube split over several GPUs by laps (tsa_score_gpu_multi):
    ``(score, wall_us)``. The reference's pencil slicing with face SRAMs
    between pencils (src/TriAlign_1cyc.v:78-98,127-140) spread over devices;
    a device listed twice runs its parts one after another on one GPU."""
    p = params or TsaParams.default()
    A, B, C = _as_u8(a), _as_u8(b), _as_u8(c)
    devs = np.ascontiguousarray(np.asarray(list(devices), dtype=np.int32))
    out = ctypes.c_int32(0)
    wall = ctypes.c_double(0.0)
    rc = _lib.tsa_score_gpu_multi(_ptr(A, ctypes.c_uint8), len(A), _ptr(B, ctypes.c_uint8), len(B),
                                  _ptr(C, ctypes.c_uint8), len(C), ctypes.byref(p),
                                  _ptr(devs, ctypes.c_int32), len(devs), ctypes.byref(out),
                                  ctypes.byref(wall))
    _check(rc, "tsa_score_gpu_multi")
    return int(out.value), float(wall.value)


def align(a, b, c, params: Optional[TsaParams] = None, device: int = 0):
    """Optimal alignment of one triple (tsa_align_gpu): ``(score, start, moves)``.

    ``moves`` holds one state index per alignment column in forward order
    (``MOVES`` names them, ``MOVE_CONSUMES`` says which sequences each
    consumes); ``start`` = (x0, y0, z0), the symbols of A, B, C before the path
    (free start at the zero faces). An extension: the reference's
    alignment-output ports are commented out (src/TriAlign_tb.sv:239-260)."""
    p = params or TsaParams.default()
    A, B, C = _as_u8(a), _as_u8(b), _as_u8(c)
    cap = len(A) + len(B) + len(C)
    mv = np.zeros(max(cap, 1), dtype=np.uint8)
    sc, n = ctypes.c_int32(0), ctypes.c_int32(0)
    st = (ctypes.c_int32 * 3)()
    rc = _lib.tsa_align_gpu(_ptr(A, ctypes.c_uint8), len(A), _ptr(B, ctypes.c_uint8), len(B),
                            _ptr(C, ctypes.c_uint8), len(C), ctypes.byref(p), ctypes.byref(sc),
                            _ptr(mv, ctypes.c_uint8), cap, ctypes.byref(n), st, device)
    _check(rc, "tsa_align_gpu")
    return int(sc.value), tuple(int(v) for v in st), mv[: n.value].copy()


def penalty_table(params: Optional[TsaParams] = None):
    """P[target][source] of src/PE_1cyc.v:164-218 (target/source order MOVES)."""
    p = params or TsaParams.default()
    GO, GE = p.gap_open, p.gap_extend
    GO2, GE2, GOGE = 2 * GO, 2 * GE, GO + GE
    return ((0, 0, 0, 0, 0, 0, 0),
            (GO2, GE2, GOGE, GOGE, GOGE, GO2, GOGE),
            (GO2, GOGE, GE2, GOGE, GOGE, GOGE, GO2),
            (GO2, GOGE, GOGE, GE2, GO2, GOGE, GOGE),
            (GO, GE, GE, GO, GE, GO, GO),
            (GO, GO, GE, GE, GO, GE, GO),
            (GO, GE, GO, GE, GO, GO, GE))


def path_score(a, b, c, start, moves, params: Optional[TsaParams] = None) -> int:
    """Score of an alignment path re-added transition by transition (no
    SCORE_BITS wrap): the first column leaves the zero face, every later one
    pays P[state][previous state] and adds its pair/triple score
    (src/PE_1cyc.v:159-218). Equals the DP score whenever nothing wraps."""
    p = params or TsaParams.default()
    A, B, C = _as_u8(a), _as_u8(b), _as_u8(c)
    P = penalty_table(p)

    def s2(u, v):
        return p.match if (u & 3) == (v & 3) else p.mismatch

    def s3(u, v, w):
        if p.s3_mode == S3_SOP:
            return s2(u, v) + s2(v, w) + s2(u, w)
        u, v, w = u & 3, v & 3, w & 3
        if u == v:
            return 3 * p.match if v == w else 2 * (p.match + p.mismatch)
        return 3 * p.mismatch

    x, y, z = start
    total, prev = 0, None
    for t in moves:
        dx, dy, dz = MOVE_CONSUMES[t]
        x, y, z = x + dx, y + dy, z + dz
        ax, by, cz = int(A[x - 1]), int(B[y - 1]), int(C[z - 1])
        add = (s3(ax, by, cz) if t == 0 else s2(ax, by) if t == 4 else s2(by, cz) if t == 5
               else s2(ax, cz) if t == 6 else 0)
        total += add - (min(P[t]) if prev is None else P[t][prev])
        prev = t
    return total


def render_alignment(a, b, c, start, moves) -> tuple[str, str, str]:
    """The three rows of an alignment (symbols A,T,C,G,N; '-' = gap), from
    the first aligned column on."""
    A, B, C = _as_u8(a), _as_u8(b), _as_u8(c)
    letters = "ATCGN"
    pos = list(start)
    rows = ([], [], [])
    for t in moves:
        for k, (seq, d) in enumerate(zip((A, B, C), MOVE_CONSUMES[t])):
            if d:
                rows[k].append(letters[int(seq[pos[k]])])
                pos[k] += 1
            else:
                rows[k].append("-")
    return tuple("".join(r) for r in rows)


def pack_batch(triples: Iterable[Sequence]) -> tuple[np.ndarray, np.ndarray]:
    """Lay triples out back to back as tsa_score_batch expects."""
    parts, offs, pos = [], [0], 0
    for (a, b, c) in triples:
        for s in (a, b, c):
            arr = _as_u8(s)
            parts.append(arr)
            pos += len(arr)
            offs.append(pos)
    seqs = np.concatenate(parts) if parts else np.zeros(1, np.uint8)
    return np.ascontiguousarray(seqs), np.asarray(offs, dtype=np.int64)


def score_batch(triples=None, params: Optional[TsaParams] = None, n_devices: int = 0,
                seqs: Optional[np.ndarray] = None, offsets: Optional[np.ndarray] = None) -> np.ndarray:
    """Scores of many triples, sharded over the node's GPUs (tsa_score_batch)."""
    p = params or TsaParams.default()
    if seqs is None:
        seqs, offsets = pack_batch(triples)
    seqs = np.ascontiguousarray(seqs, dtype=np.uint8)
    offsets = np.ascontiguousarray(offsets, dtype=np.int64)
    n = (len(offsets) - 1) // 3
    out = np.zeros(max(n, 1), dtype=np.int32)
    rc = _lib.tsa_score_batch(_ptr(seqs, ctypes.c_uint8), _ptr(offsets, ctypes.c_int64), n,
                              ctypes.byref(p), _ptr(out, ctypes.c_int32), n_devices)
    _check(rc, "tsa_score_batch")
    return out[:n]


def score_batch_devices(triples=None, devices: Sequence[int] = (0,),
                        params: Optional[TsaParams] = None, seqs: Optional[np.ndarray] = None,
                        offsets: Optional[np.ndarray] = None) -> np.ndarray:
    """tsa_score_batch_devices: contiguous shards of the batch, shard s on
    ``devices[s]``; a device may repeat ((0, 0, 0) shards three ways on one
    GPU, its shards run one after another)."""
    p = params or TsaParams.default()
    if seqs is None:
        seqs, offsets = pack_batch(triples)
    seqs = np.ascontiguousarray(seqs, dtype=np.uint8)
    offsets = np.ascontiguousarray(offsets, dtype=np.int64)
    devs = np.ascontiguousarray(np.asarray(list(devices), dtype=np.int32))
    n = (len(offsets) - 1) // 3
    out = np.zeros(max(n, 1), dtype=np.int32)
    rc = _lib.tsa_score_batch_devices(_ptr(seqs, ctypes.c_uint8), _ptr(offsets, ctypes.c_int64), n,
                                      ctypes.byref(p), _ptr(out, ctypes.c_int32),
                                      _ptr(devs, ctypes.c_int32), len(devs))
    _check(rc, "tsa_score_batch_devices")
    return out[:n]


def workspace_size(n: int, max_la: int, max_lb: int, max_lc: int,
                   params: Optional[TsaParams] = None, kernel: str | int = "auto") -> int:
    p = params or TsaParams.default()
    k = KERNELS[kernel] if isinstance(kernel, str) else int(kernel)
    sz = ctypes.c_size_t(0)
    _check(_lib.tsa_batch_workspace_size(n, max_la, max_lb, max_lc, ctypes.byref(p), k,
                                         ctypes.byref(sz)), "tsa_batch_workspace_size")
    return int(sz.value)


def describe_plan(n: int, max_la: int, max_lb: int, max_lc: int,
                  params: Optional[TsaParams] = None, kernel: str | int = "auto",
                  sync: bool = True) -> str:
    """The kernel, arithmetic and schedule a batch of these sizes runs
    (tsa_describe_plan; host-only). ``sync``: the tsa_score_batch path."""
    p = params or TsaParams.default()
    k = KERNELS[kernel] if isinstance(kernel, str) else int(kernel)
    buf = ctypes.create_string_buffer(128)
    _check(_lib.tsa_describe_plan(n, max_la, max_lb, max_lc, ctypes.byref(p), k, int(sync), buf,
                                  len(buf)), "tsa_describe_plan")
    return buf.value.decode()


def score_batch_async(d_seqs_ptr: int, d_offsets_ptr: int, n: int, max_la: int, max_lb: int,
                      max_lc: int, d_scores_ptr: int, d_ws_ptr: int, ws_bytes: int,
                      stream_ptr: int = 0, params: Optional[TsaParams] = None,
                      kernel: str | int = "auto") -> None:
    """Device-resident batch (tsa_score_batch_async). Pointers are raw device
    addresses (e.g. ``tensor.data_ptr()``), stream a hipStream_t handle."""
    p = params or TsaParams.default()
    k = KERNELS[kernel] if isinstance(kernel, str) else int(kernel)
    rc = _lib.tsa_score_batch_async(ctypes.c_void_p(d_seqs_ptr), ctypes.c_void_p(d_offsets_ptr),
                                    n, max_la, max_lb, max_lc, ctypes.byref(p), k,
                                    ctypes.c_void_p(d_scores_ptr), ctypes.c_void_p(d_ws_ptr),
                                    ctypes.c_size_t(ws_bytes), ctypes.c_void_p(stream_ptr))
    _check(rc, "tsa_score_batch_async")


def pack2(seqs) -> np.ndarray:
    """Symbols (0..4) -> 2-bit packed bytes, four per byte, symbol i at bits
    2(i%4) of byte i/4 (tsa_pack2; N = 4 packs as A, as the RTL's 2-bit
    registers hold it)."""
    s = _as_u8(seqs)
    out = np.zeros(max((len(s) + 3) // 4, 1), dtype=np.uint8)
    _check(_lib.tsa_pack2(_ptr(s, ctypes.c_uint8), len(s), _ptr(out, ctypes.c_uint8)), "tsa_pack2")
    return out[: (len(s) + 3) // 4]


def score_batch_async_p2(d_packed_ptr: int, d_offsets_ptr: int, n: int, max_la: int, max_lb: int,
                         max_lc: int, d_scores_ptr: int, d_ws_ptr: int, ws_bytes: int,
                         stream_ptr: int = 0, params: Optional[TsaParams] = None,
                         kernel: str | int = "auto") -> None:
    """score_batch_async on 2-bit packed sequences (tsa_score_batch_async_p2):
    d_packed holds pack2(seqs), offsets still count symbols."""
    p = params or TsaParams.default()
    k = KERNELS[kernel] if isinstance(kernel, str) else int(kernel)
    rc = _lib.tsa_score_batch_async_p2(ctypes.c_void_p(d_packed_ptr), ctypes.c_void_p(d_offsets_ptr),
                                       n, max_la, max_lb, max_lc, ctypes.byref(p), k,
                                       ctypes.c_void_p(d_scores_ptr), ctypes.c_void_p(d_ws_ptr),
                                       ctypes.c_size_t(ws_bytes), ctypes.c_void_p(stream_ptr))
    _check(rc, "tsa_score_batch_async_p2")


# ---- the testbench's sequence RAM image (src/TriAlign_tb.sv:94-96,149-169) ----
# ``reg [127:0] seqX_ram [...]``: 32 four-bit symbols per 128-bit word, symbol
# i in word i >> 5 at bits [4*(i & 31) + 3 : 4*(i & 31)] (the read mux of
# src/TriAlign_tb.sv:149-169). As little-endian bytes that is two symbols per
# byte, the even one in the low nibble.
RAM_WORD_SYMBOLS = 32


def pack_ram128(seq) -> np.ndarray:
    """Symbols -> the testbench RAM image, as an (n_words, 16) uint8 array of
    little-endian 128-bit words (unused nibbles zero)."""
    s = _as_u8(seq)
    if s.size and int(s.max()) > 15:
        raise TsaError(TSA_EINVAL, "symbol does not fit a 4-bit RAM nibble")
    nw = max(1, -(-len(s) // RAM_WORD_SYMBOLS))
    nib = np.zeros(nw * RAM_WORD_SYMBOLS, np.uint8)
    nib[: len(s)] = s
    return (nib[0::2] | (nib[1::2] << 4)).reshape(nw, 16)


def unpack_ram128(words, length: int) -> np.ndarray:
    """The first ``length`` symbols of a testbench RAM image ((n, 16) uint8
    little-endian words, or raw bytes)."""
    b = np.ascontiguousarray(np.asarray(words, dtype=np.uint8)).reshape(-1)
    if length < 0 or length > 2 * b.size:
        raise TsaError(TSA_EINVAL, "RAM image shorter than the sequence")
    nib = np.empty(2 * b.size, np.uint8)
    nib[0::2] = b & 15
    nib[1::2] = b >> 4
    return nib[:length].copy()


def ram128_hex_lines(seq) -> list[str]:
    """The RAM image as ``$readmemh`` lines: one 128-bit word per line, 32 hex
    digits, most significant nibble (symbol 31 of the word) first."""
    return ["".join(f"{v:x}" for v in unpack_ram128(w, 32)[::-1]) for w in pack_ram128(seq)]


def _parse_ram_hex(text: str, length: Optional[int]) -> np.ndarray:
    words = []
    for ln in text.splitlines():
        ln = ln.split("//")[0].strip().replace("_", "")
        if not ln or ln.startswith("@"):
            continue
        if len(ln) > 32 or any(ch not in "0123456789abcdefABCDEF" for ch in ln):
            raise TsaError(TSA_EINVAL, f"RAM word {ln!r}")
        nibs = [int(ch, 16) for ch in ln.rjust(32, "0")][::-1]  # symbol 0 = lowest nibble
        words.extend(nibs)
    seq = np.asarray(words, dtype=np.uint8)
    return seq if length is None else seq[:length]


_TB_INIT = None


def _parse_tb_initial(text: str, name: str) -> np.ndarray:
    """Symbols a testbench ``initial`` block writes into ``name``: lines
    ``seqA_ram[w][hi:lo] <= A;`` (src/TriAlign_tb.sv:423-1960), symbol index
    32*w + lo/4, names A/T/C/G/N or numbers (src/TriAlign_tb.sv:42-46)."""
    import re
    global _TB_INIT
    if _TB_INIT is None:
        _TB_INIT = re.compile(r"(\w+)\[(\d+)\]\[(\d+):(\d+)\]\s*<?=\s*(?:4'[dhb])?(\w+)\s*;")
    got = {}
    for m in _TB_INIT.finditer(text):
        if m.group(1) != name:
            continue
        w, hi, lo, v = int(m.group(2)), int(m.group(3)), int(m.group(4)), m.group(5)
        if hi - lo != 3 or lo % 4 or hi >= 128:
            raise TsaError(TSA_EINVAL, f"RAM nibble [{hi}:{lo}]")
        sym = SYMBOLS[v] if v in SYMBOLS else int(v, 0)
        if sym > 4:
            raise TsaError(TSA_EINVAL, f"symbol {v}")
        got[32 * w + lo // 4] = sym
    if not got:
        raise TsaError(TSA_EINVAL, f"no {name} writes found")
    n = max(got) + 1
    if sorted(got) != list(range(n)):
        raise TsaError(TSA_EINVAL, f"{name}: symbols missing")
    return np.asarray([got[i] for i in range(n)], dtype=np.uint8)


def read_sequence(path: str, fmt: str = "auto", length: Optional[int] = None,
                  ram: str = "seqA_ram") -> np.ndarray:
    """Read one sequence. Formats (``fmt``):

    * ``dat`` -- one decimal symbol per line, CRLF tolerant (dat/A_seq.dat);
    * ``fasta`` -- A=0 T=1 C=2 G=3 N=4 (src/TriAlign_tb.sv:42-46);
    * ``ramhex`` -- the testbench's 128-bit sequence RAM as ``$readmemh`` text,
      32 symbols per word (src/TriAlign_tb.sv:94-96,149-169); ``length``
      trims the padding of the last word;
    * ``ramraw`` -- the same RAM image as raw little-endian 16-byte words
      (``length`` required);
    * ``tb`` -- the ``seqX_ram[w][hi:lo] <= SYM;`` writes of a testbench
      ``initial`` block (src/TriAlign_tb.sv:423-1960), RAM named by ``ram``.

    ``auto`` tells FASTA (``>``), testbench initial blocks (``<=``) and dat
    apart; RAM images need an explicit ``fmt``."""
    if fmt == "ramraw":
        if length is None:
            raise TsaError(TSA_EINVAL, "ramraw needs the sequence length")
        return unpack_ram128(np.fromfile(path, dtype=np.uint8), length)
    with open(path, "r") as f:
        text = f.read()
    if fmt == "ramhex":
        return _parse_ram_hex(text, length)
    body = text.lstrip()
    if fmt == "tb" or (fmt == "auto" and "<=" in body and "_ram[" in body):
        seq = _parse_tb_initial(body, ram)
        return seq if length is None else seq[:length]
    if fmt not in ("auto", "dat", "fasta"):
        raise TsaError(TSA_EINVAL, f"format {fmt!r}")
    if body.startswith(">"):
        lines = body.splitlines()[1:]
        seq = []
        for ln in lines:
            if ln.startswith(">"):
                break
            for ch in ln.strip().upper():
                if ch == "U":
                    ch = "T"
                if ch not in SYMBOLS:
                    raise TsaError(TSA_EINVAL, f"FASTA symbol {ch!r}")
                seq.append(SYMBOLS[ch])
        return np.asarray(seq, dtype=np.uint8)
    vals = [int(t) for t in body.split()]
    if any(v < 0 or v > 4 for v in vals):
        raise TsaError(TSA_EINVAL, "dat symbol outside 0..4")
    return np.asarray(vals, dtype=np.uint8)


def rtl_envelope(la: int, lb: int, lc: int, a_total_len: int = 512, pe_len: int = 8,
                 variant: str = "1cyc") -> bool:
    """True when (la,lb,lc) lies inside the RTL's operating envelope, where
    the reference hardware would compute the same score.

    1cyc (TRIALIGN_1cyc): lengths multiples of PE_LEN (src/TriAlign_1cyc.v:
    50-51), LA <= A_TOTAL_LEN (SRAM depth, :7,492) and LB <= LA (y-face ring,
    :44,330-332).

    2cyc (TRIALIGN_2cyc, the ASIC variant): multiples of PE_LEN, LA <= 512
    (z SRAM depth, src/TriAlign_2cyc.v:135), and a y-face store whose pencil
    slots never share an SRAM bank they must not share (`_rtl2_ring_ok`).
    The 2cyc rule is MODEL-DERIVED: it reproduces where the one cycle-level
    transliteration (oracle/rtl_model_2cyc.c) agrees, and no Verilog
    simulation has confirmed the shapes it rejects."""
    base = (la % pe_len == 0 and lb % pe_len == 0 and lc % pe_len == 0 and 0 < la <= a_total_len
            and lb > 0 and lc > 0)
    if variant == "1cyc":
        return base and lb <= la
    if variant == "2cyc":
        return base and la <= 512 and _rtl2_ring_ok(la, lb, lc, pe_len)
    raise TsaError(TSA_EINVAL, f"unknown RTL variant {variant!r}")


def _rtl2_slot_bank(q: int, lb: int, pe_len: int) -> tuple:
    """(group, pair, page) of y-face slot q (index 8q) in TRIALIGN_2cyc: group
    2 when one of the index's bits 6..9 is also set in B_idx, else bit 4;
    pair = bit 3; page = bits 9..5 of the index within a 13-bit address, none
    in group 2's 9-bit SRAMs (src/TriAlign_2cyc.v:85-92,141-157,176-180)."""
    idx = pe_len * q
    if idx & lb & 0x3C0:
        return (2, (idx >> 3) & 1, 0)
    return ((idx >> 4) & 1, (idx >> 3) & 1, (idx >> 5) & 0xF)


def _rtl2_ring_ok(la: int, lb: int, lc: int, pe_len: int = 8) -> bool:
    """Whether TRIALIGN_2cyc's y-face ring carries every pencil's face to its
    reader (checked against the cycle-level model, tests/test_oracle.py).
    Pencil s = (slice_z, slice_y) writes slot s mod R and reads slot
    (s + 2) mod R, R = LA/8 + 2 (write index from 0, read index from 16, both
    +8 per pencil, wrapping at A_idx + 8: src/TriAlign_2cyc.v:448-450,650-651);
    the corner reads slot (s + 1) mod R's last SRAM (:177,213-219). The
    reader of a face is the pencil LB/8 later, so LB must equal LA unless no
    face is ever read (LC = 8); and a pencil fails when its write bank is its
    read or corner bank (an SRAM reads or writes, not both: :305-331), when
    its read and corner banks coincide (the read group's address shift
    overrides the corner's, :563-596), or when a slot's storage is
    overwritten before its reader comes."""
    ny, nz = lb // pe_len, lc // pe_len
    if nz == 1:
        return True
    R = la // pe_len + 2
    if ny != R - 2:
        return False
    for s in range(ny * nz):
        sz, sy = divmod(s, ny)
        w = _rtl2_slot_bank(s % R, lb, pe_len)
        r = _rtl2_slot_bank((s + 2) % R, lb, pe_len)
        c = _rtl2_slot_bank((s + 1) % R, lb, pe_len)
        later = sz < nz - 1  # this pencil's face is read
        if sz >= 1 and r[:2] == w[:2]:
            return False
        if sz >= 1 and sy >= 1 and (c[:2] == r[:2] or (later and c[:2] == w[:2])):
            return False
        if later and any(_rtl2_slot_bank(t % R, lb, pe_len) == w for t in range(s + 1, s + ny)):
            return False
    return True


class TriAlign:
    """Mirror of the ``TRIALIGN`` module (src/TriAlign_1cyc.v:1-22).

    Parameters keep the RTL names; ``PE_LEN`` and ``SRAM_ADDR_BITS`` only
    describe the envelope (the GPU has no 8x8 array or SRAM depth). ``run``
    plays the testbench's one-shot start_align -> finish handshake
    (src/TriAlign_tb.sv:279-333) and returns ``Score``."""

    def __init__(self, A_TOTAL_LEN: int = 512, B_TOTAL_LEN: int = 512, C_TOTAL_LEN: int = 512,
                 PE_LEN: int = 8, SCORE_BITS: int = 12, SRAM_ADDR_BITS: int = 9,
                 params: Optional[TsaParams] = None, device: int = 0, kernel: str = "auto"):
        self.A_TOTAL_LEN, self.B_TOTAL_LEN, self.C_TOTAL_LEN = A_TOTAL_LEN, B_TOTAL_LEN, C_TOTAL_LEN
        self.PE_LEN, self.SCORE_BITS, self.SRAM_ADDR_BITS = PE_LEN, SCORE_BITS, SRAM_ADDR_BITS
        self.params = params or TsaParams.default(score_bits=SCORE_BITS)
        self.device, self.kernel = device, kernel
        self.Score: Optional[int] = None
        self.finish = False

    def in_envelope(self, la: int, lb: int, lc: int) -> bool:
        return (rtl_envelope(la, lb, lc, min(self.A_TOTAL_LEN, 1 << self.SRAM_ADDR_BITS),
                             self.PE_LEN) and lb <= self.B_TOTAL_LEN and lc <= self.C_TOTAL_LEN)

    def run(self, A, B, C) -> int:
        """start_align -> ... -> finish; returns Score."""
        self.finish = False
        self.Score = score(A, B, C, self.params, kernel=self.kernel, device=self.device)
        self.finish = True
        return self.Score

    def display(self) -> str:
        """The testbench's print line (src/TriAlign_tb.sv:341)."""
        return f"TriAlign Score:        \t{self.Score}"
