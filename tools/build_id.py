#!/usr/bin/env python3
"""Source hash of libmocohip.so (mh_build_id): SHA-256 over the bytes of
every file the library is compiled from, in sorted path order.  The Makefile
bakes it into the library; tests/conftest.py and __graft_entry__.smoke()
compare it with the tree so that a stale prebuilt library is rebuilt (here)
or refused (on a GPU box) instead of silently tested."""
import glob
import hashlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "opensim-moco_amd", "csrc")


def source_files():
    pats = ["*.hip", "*.hpp", "generated/*.hip", "generated/models_table.inc", "Makefile"]
    files = [f for p in pats for f in glob.glob(os.path.join(CSRC, p))]
    files += glob.glob(os.path.join(ROOT, "include", "*.h"))
    return sorted(set(files), key=lambda f: os.path.relpath(f, ROOT))


def build_id() -> str:
    h = hashlib.sha256()
    for f in source_files():
        h.update(os.path.relpath(f, ROOT).encode() + b"\0")
        with open(f, "rb") as fh:
            h.update(fh.read())
        h.update(b"\0")
    return h.hexdigest()[:16]


if __name__ == "__main__":
    sys.stdout.write(build_id())
