#!/usr/bin/env python3
"""HBM traffic of k_emit per launch from two rocprofv3 --pmc passes.

    traffic.py FETCH_DIR WRITE_DIR OUT.json [--alg-bytes N] [--kernel K1,K2,..] [--label L]

With several kernels (a call made of several launches, e.g. ingest) the
figure is the sum of their per-dispatch means, and --label names the whole.

FETCH_DIR / WRITE_DIR hold run_counter_collection.csv of a `--pmc FETCH_SIZE`
and a `--pmc WRITE_SIZE` pass over the same command (separate passes: the two
TCC counters do not fit one pass).  Values are KB per dispatch.  gfx950
correction (MI355X_MICROARCH.md, HBM section): FETCH_SIZE reports half the
bytes of wide coalesced reads -> doubled; WRITE_SIZE is exact for 16-B-per-lane
stores.  Averages over every k_emit dispatch of the run.
"""
import argparse
import collections
import csv
import json
import os


def per_dispatch(path, counter, kernel):
    vals = collections.defaultdict(float)
    with open(os.path.join(path, "run_counter_collection.csv")) as f:
        for r in csv.DictReader(f):
            if kernel + "(" in r["Kernel_Name"] and r["Counter_Name"] == counter:
                vals[r["Dispatch_Id"]] += float(r["Counter_Value"])
    return list(vals.values())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_dir")
    ap.add_argument("write_dir")
    ap.add_argument("out")
    ap.add_argument("--kernel", default="k_emit")
    ap.add_argument("--alg-bytes", type=float, default=0.0)
    ap.add_argument("--label", default="")
    ap.add_argument("--fetch-scale", type=float, default=2.0,
                    help="gfx950 FETCH_SIZE correction: 2, calibrated for 1-, 4-, 8- and 16-byte "
                         "lanes over whole lines (tools/fetch_calib.cpp, profiles/r06_fetch_calib.json)")
    ap.add_argument("--revision", default="", help="the source revision measured")
    a = ap.parse_args()
    raw = write = 0.0
    nd = []
    for k in a.kernel.split(","):
        fk = per_dispatch(a.fetch_dir, "FETCH_SIZE", k)
        wk = per_dispatch(a.write_dir, "WRITE_SIZE", k)
        if not fk or not wk:                        # a kernel this build does not launch
            continue
        raw += 1024 * sum(fk) / len(fk)             # KB -> bytes
        write += 1024 * sum(wk) / len(wk)
        nd.append([k, len(fk), len(wk)])
    fetch = a.fetch_scale * raw
    out = {"kernel": a.label or a.kernel, "dispatches": nd if len(nd) > 1 else nd[0][1:],
           "fetch_size_raw_bytes_per_launch": round(raw),
           "fetch_bytes_per_launch": round(fetch), "write_bytes_per_launch": round(write),
           "hbm_bytes_per_launch": round(fetch + write),
           "method": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes); "
                     f"FETCH_SIZE x {a.fetch_scale} (gfx950 correction, calibrated per access width: "
                     "profiles/r06_fetch_calib.json)"}
    if a.revision:
        out["revision"] = a.revision
    if a.alg_bytes:
        out["alg_bytes_per_launch"] = a.alg_bytes
        out["traffic_over_alg"] = round((fetch + write) / a.alg_bytes, 4)
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
