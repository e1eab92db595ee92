#!/usr/bin/env python3
"""Hash of the library's sources (csrc/*.hip, *.h, *.cpp and include/rtx.h,
sorted by path, contents concatenated): sha256, first 16 hex digits. The
Makefile compiles it into librtx.so (rtx_build_info); bench.py recomputes it
from the tree to show the loaded library was built from these sources."""
import glob
import hashlib
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def src_sha16(root: str = ROOT) -> str:
    src = os.path.join(root, "raytrace-we-gpu_amd", "csrc")
    files = sorted(glob.glob(os.path.join(src, "*.hip")) + glob.glob(os.path.join(src, "*.h")) +
                   glob.glob(os.path.join(src, "*.cpp")))
    files = sorted(os.path.relpath(f, root) for f in files) + ["include/rtx.h"]
    h = hashlib.sha256()
    for rel in files:
        h.update(rel.encode() + b"\0")
        with open(os.path.join(root, rel), "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16]


if __name__ == "__main__":
    print(src_sha16())
