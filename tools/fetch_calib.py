#!/usr/bin/env python3
"""Summarises tools/fetch_calib's rocprofv3 --pmc passes: counter bytes per
kernel against the bytes of distinct 128-byte lines each kernel touches.
Usage: python tools/fetch_calib.py <pmc dir> <out.json>"""
import collections
import csv
import glob
import json
import os
import re
import sys

G = 8 << 20                      # distinct lines per gather kernel (fetch_calib.hip kGathers)
LINE = 128
TOUCHED = {                      # bytes of the distinct lines each kernel touches
    "k_stream16": 2 << 30, "k_gather8": G * LINE, "k_gather4": G * LINE, "k_gather8x2": G * LINE,
    "k_gather8h": G * LINE, "k_scatter8": G * LINE, "k_stream16w": 2 << 30,
}
ACCESSED = {                     # bytes the loads / stores themselves request
    "k_stream16": 2 << 30, "k_gather8": G * 8, "k_gather4": G * 4, "k_gather8x2": G * 16,
    "k_gather8h": 2 * G * 8, "k_scatter8": G * 8, "k_stream16w": 2 << 30,
}


def main():
    src, out = sys.argv[1], sys.argv[2]
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(os.path.join(src, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            m = re.search(r"(k_[a-z0-9]+)", r["Kernel_Name"])
            if m:
                vals[m.group(1)][r["Counter_Name"]].append(float(r["Counter_Value"]))
    res = {}
    for k, d in vals.items():
        e = {c: sum(v) / len(v) for c, v in d.items()}
        if k in TOUCHED:
            for c in ("FETCH_SIZE", "WRITE_SIZE"):
                if c in e:
                    b = e[c] * 1024.0
                    e[c + "_bytes"] = b
                    e[c + "_per_touched_line_byte"] = b / TOUCHED[k]
                    e[c + "_per_requested_byte"] = b / ACCESSED[k]
        res[k] = e
    json.dump({"lines": G, "line_bytes": LINE, "kernels": res}, open(out, "w"), indent=1, sort_keys=True)
    for k in sorted(res):
        e = res[k]
        print(k, {c: round(v, 4) for c, v in e.items() if c.endswith("per_touched_line_byte")})


if __name__ == "__main__":
    main()
