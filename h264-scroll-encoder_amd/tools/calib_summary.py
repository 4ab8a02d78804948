#!/usr/bin/env python3
"""FETCH_SIZE / WRITE_SIZE calibration per access width (tools/fetch_calib.cpp).

    calib_summary.py FETCH_DIR WRITE_DIR OUT.json

FETCH_DIR / WRITE_DIR: run_counter_collection.csv of `rocprofv3 --pmc
FETCH_SIZE` / `--pmc WRITE_SIZE` over ./fetch_calib.  Each kernel moves
exactly 1 GiB; the counter (KB per dispatch) over that byte count is the
factor a kernel's counter must be divided by at that width.
"""
import collections
import csv
import json
import os
import sys

BYTES = 1 << 30


def per_kernel(path, counter):
    vals = collections.defaultdict(float)
    names = {}
    with open(os.path.join(path, "run_counter_collection.csv")) as f:
        for r in csv.DictReader(f):
            if r["Counter_Name"] != counter:
                continue
            vals[int(r["Dispatch_Id"])] += float(r["Counter_Value"])
            names[int(r["Dispatch_Id"])] = r["Kernel_Name"]
    return [(names[k], vals[k]) for k in sorted(vals)]


def width_of(name):
    for key, w in (("unsigned char", 1), ("HIP_vector_type<unsigned int, 4u>", 16),
                   ("HIP_vector_type<unsigned int, 2u>", 8), ("unsigned int", 4)):
        if key in name:
            return w
    return None


def main():
    fdir, wdir, out = sys.argv[1:4]
    res = {"bytes_per_kernel": BYTES, "read": {}, "write": {},
           "how": "tools/fetch_calib.cpp: 1 GiB per kernel, whole waves over contiguous bytes, "
                  "grid stride; FETCH_SIZE / WRITE_SIZE in KB per dispatch (rocprofv3, separate passes)"}
    for name, kb in per_kernel(fdir, "FETCH_SIZE"):
        if "k_read" in name:
            w = width_of(name)
            res["read"][f"{w}B_per_lane"] = {"counter_bytes": kb * 1024, "factor": round(kb * 1024 / BYTES, 4)}
    for name, kb in per_kernel(wdir, "WRITE_SIZE"):
        if "k_write" in name:
            w = width_of(name)
            res["write"][f"{w}B_per_lane"] = {"counter_bytes": kb * 1024, "factor": round(kb * 1024 / BYTES, 4)}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
