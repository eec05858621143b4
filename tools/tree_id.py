#!/usr/bin/env python3
"""Identity of the kernel sources a profile or bench line was made from:
sha1 over the HIP sources and public headers (pipelinedp_amd/csrc/*.hip,
*.h and include/*.h, in name order).  bench.py joins a PMC summary only when
the summary's "tree" equals this value for the tree it runs on.
Usage: python tools/tree_id.py  (prints the id)"""
import glob
import hashlib
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def source_tree_id(root=ROOT):
    h = hashlib.sha1()
    files = sorted(glob.glob(os.path.join(root, "pipelinedp_amd", "csrc", "*.hip")) +
                   glob.glob(os.path.join(root, "pipelinedp_amd", "csrc", "*.h")) +
                   glob.glob(os.path.join(root, "include", "*.h")))
    for f in files:
        h.update(os.path.relpath(f, root).encode())
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


if __name__ == "__main__":
    print(source_tree_id())
