#!/usr/bin/env python3
"""Source hash of libchunky_ec.so: SHA-256 over the library's sources (every csrc/*.cpp, *.hip,
*.hpp, the Makefile and include/chunky_ec.h), each as its path relative to the repo root, a NUL,
its bytes and a NUL, in sorted path order; printed as 16 hex digits.

The Makefile compiles this value into the library (`cec_build_id()`), and chunky_ec refuses on
import a library whose id differs from the hash of the sources shipped beside it, so a GPU run can
only use a library built from the tree it was given (build provenance)."""
import hashlib
import os
import sys

CSRC = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(CSRC))


def source_files(root: str = ROOT):
    csrc = os.path.join(root, "chunky-bits_amd", "csrc")
    files = [os.path.join(csrc, n) for n in os.listdir(csrc)
             if n.endswith((".cpp", ".hip", ".hpp")) or n == "Makefile"]
    files.append(os.path.join(root, "include", "chunky_ec.h"))
    return sorted(os.path.relpath(f, root) for f in files)


def source_hash(root: str = ROOT) -> str:
    h = hashlib.sha256()
    for rel in source_files(root):
        h.update(rel.encode() + b"\0")
        with open(os.path.join(root, rel), "rb") as f:
            h.update(f.read())
        h.update(b"\0")
    return h.hexdigest()[:16]


if __name__ == "__main__":
    sys.stdout.write(source_hash() + "\n")
