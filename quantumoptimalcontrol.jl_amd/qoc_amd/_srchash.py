"""Source hash of libqoc_mi355x.so: sha256 over the HIP sources and the ABI header.

``__graft_entry__.build_lib`` compiles the hash into the library (``qoc_source_hash()``) and rebuilds
whenever it differs from the tree; ``_lib.load`` refuses a library whose hash does not match the sources
next to it, so a stale or foreign binary can never be the one that runs.
"""
from __future__ import annotations

import hashlib
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
PKG_ROOT = os.path.dirname(_HERE)
CSRC = os.path.join(PKG_ROOT, "csrc")
HEADER = os.path.join(os.path.dirname(PKG_ROOT), "include", "qoc.h")


def source_files() -> list[str]:
    if not os.path.isdir(CSRC):
        return []
    fs = sorted(os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith((".hip", ".hpp", ".h")))
    if os.path.exists(HEADER):
        fs.append(HEADER)
    return fs


def source_hash() -> str | None:
    """sha256 hex digest of (name, bytes) of every source; None when the sources are not in the tree."""
    fs = source_files()
    if not fs:
        return None
    h = hashlib.sha256()
    for f in fs:
        h.update(os.path.basename(f).encode() + b"\0")
        with open(f, "rb") as fh:
            h.update(fh.read())
        h.update(b"\0")
    return h.hexdigest()
