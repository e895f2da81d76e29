"""Synthetic inputs for the bench and the GPU parity tests.

Uniform DNA: splitmix64(seed) words, 32 two-bit symbols per word, low bits
first; the seed of triple i, sequence s in {A,B,C} is SEED_BASE + 3*i + s.
Bit-identical to oracle/tsa_oracle.c:tsao_gen_uniform (checked by the tests).
"Related" triples (B, C = A with substitutions and indels) exercise high scores.
"""
from __future__ import annotations

import numpy as np

SEED_BASE = 0x7A1A11670000
_GOLDEN = np.uint64(0x9E3779B97F4A7C15)
_C1 = np.uint64(0xBF58476D1CE4E5B9)
_C2 = np.uint64(0x94D049BB133111EB)


def splitmix64_words(seed: int, nwords: int) -> np.ndarray:
    with np.errstate(over="ignore"):
        k = np.arange(1, nwords + 1, dtype=np.uint64)
        z = np.uint64(seed) + k * _GOLDEN
        z = (z ^ (z >> np.uint64(30))) * _C1
        z = (z ^ (z >> np.uint64(27))) * _C2
        return z ^ (z >> np.uint64(31))


def gen_uniform(seed: int, length: int) -> np.ndarray:
    nw = (length + 31) // 32
    w = splitmix64_words(seed, nw)
    shifts = (2 * np.arange(32, dtype=np.uint64))
    sym = ((w[:, None] >> shifts[None, :]) & np.uint64(3)).astype(np.uint8).reshape(-1)
    return sym[:length]


def triple(i: int, la: int, lb: int | None = None, lc: int | None = None):
    lb = la if lb is None else lb
    lc = la if lc is None else lc
    return (gen_uniform(SEED_BASE + 3 * i, la), gen_uniform(SEED_BASE + 3 * i + 1, lb),
            gen_uniform(SEED_BASE + 3 * i + 2, lc))


def batch(i0: int, n: int, la: int, lb: int | None = None, lc: int | None = None):
    """Triples i0 .. i0+n-1 packed back to back: (seqs uint8, offsets int64[3n+1])."""
    lb = la if lb is None else lb
    lc = la if lc is None else lc
    per = la + lb + lc
    seqs = np.empty(n * per, dtype=np.uint8)
    offs = np.empty(3 * n + 1, dtype=np.int64)
    for j in range(n):
        a, b, c = triple(i0 + j, la, lb, lc)
        base = j * per
        seqs[base:base + la] = a
        seqs[base + la:base + la + lb] = b
        seqs[base + la + lb:base + per] = c
        offs[3 * j] = base
        offs[3 * j + 1] = base + la
        offs[3 * j + 2] = base + la + lb
    offs[3 * n] = n * per
    return seqs, offs


def mutate(src: np.ndarray, rng: np.random.Generator, sub: float = 0.10, indel: float = 0.02,
           length: int | None = None) -> np.ndarray:
    out = []
    for s in src:
        r = rng.random()
        if r < indel / 2:
            continue  # deletion
        if r < indel:
            out.append(int(rng.integers(0, 4)))  # insertion before s
        out.append(int(rng.integers(0, 4)) if rng.random() < sub else int(s))
    arr = np.asarray(out, dtype=np.uint8)
    if length is not None:
        if len(arr) < length:
            arr = np.concatenate([arr, rng.integers(0, 4, length - len(arr)).astype(np.uint8)])
        arr = arr[:length]
    return arr


def related_triple(seed: int, length: int, sub: float = 0.10, indel: float = 0.02):
    rng = np.random.default_rng(seed)
    a = rng.integers(0, 4, length).astype(np.uint8)
    return a, mutate(a, rng, sub, indel, length), mutate(a, rng, sub, indel, length)
