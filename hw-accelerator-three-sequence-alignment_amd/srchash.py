"""Hash of the product library's sources (csrc/*.hip, csrc/*.h, include/trialign.h).

The Makefile bakes it into libtrialign.so (``tsa_version()`` ends in
``src=<hash>``), so a bench line, a smoke run or a test session can show
which sources the loaded binary was built from, and the test/bench helpers
can rebuild a library whose hash is not the tree's.

    python3 srchash.py          # prints the hash (the Makefile calls this)

No third-party imports: it runs before anything is built.
"""
from __future__ import annotations

import glob
import hashlib
import os

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG_DIR)
LIB_PATH = os.path.join(PKG_DIR, "lib", "libtrialign.so")
MARKER = b"src="


def source_files() -> list[str]:
    """Repo-relative paths, sorted (the order the hash covers them in)."""
    files = glob.glob(os.path.join(PKG_DIR, "csrc", "*.hip")) + \
        glob.glob(os.path.join(PKG_DIR, "csrc", "*.h")) + [os.path.join(ROOT, "include", "trialign.h")]
    return sorted(os.path.relpath(f, ROOT) for f in files)


def source_hash() -> str:
    h = hashlib.sha256()
    for rel in source_files():
        with open(os.path.join(ROOT, rel), "rb") as f:
            h.update(rel.encode() + b"\0" + f.read() + b"\0")
    return h.hexdigest()[:16]


def built_hash(lib_path: str = LIB_PATH) -> str | None:
    """The hash a built library carries (read from the file, not loaded)."""
    try:
        with open(lib_path, "rb") as f:
            data = f.read()
    except OSError:
        return None
    key = b"trialign-mi355x gfx950 " + MARKER
    i = data.find(key)
    if i < 0:
        return None
    j = i + len(key)
    return data[j:j + 16].decode("ascii", "replace")


def is_current(lib_path: str = LIB_PATH) -> bool:
    return built_hash(lib_path) == source_hash()


if __name__ == "__main__":
    print(source_hash())
