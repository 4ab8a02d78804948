#!/usr/bin/env python3
"""Per-kernel SQ counter summary from one rocprofv3 --pmc pass.

    sq_summary.py PMC_DIR OUT.json KERNEL [KERNEL ...]

PMC_DIR holds run_counter_collection.csv of a pass with SQ_WAVE_CYCLES
SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU
SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS GRBM_GUI_ACTIVE.  Per kernel:
counters per launch (mean over its dispatches), GPU cycles per launch
(GRBM_GUI_ACTIVE summed over the 8 XCDs / 8), VALU issue utilisation =
VALU instructions / (cycles x 256 CUs x 2 wave64 VALU issues per CU-cycle:
4 SIMD-32 units, 2 cycles per wave64 instruction), and the split of wave
time into parked (s_waitcnt / barrier), issue-stalled and active (the SQ
wait/active counters count quad-cycles like SQ_WAVE_CYCLES).
"""
import collections
import csv
import json
import os
import sys


def main():
    d, out, kernels = sys.argv[1], sys.argv[2], sys.argv[3:]
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    names = {}
    with open(os.path.join(d, "run_counter_collection.csv")) as f:
        for r in csv.DictReader(f):
            for k in kernels:
                if k + "(" in r["Kernel_Name"]:
                    per[(k, r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
                    names[k] = True
    res = {}
    for k in kernels:
        disp = [v for (kk, _), v in per.items() if kk == k]
        if not disp:
            continue
        keys = sorted(disp[0])
        mean = {c: sum(x[c] for x in disp) / len(disp) for c in keys}
        cyc = mean.get("GRBM_GUI_ACTIVE", 0) / 8
        wc = mean.get("SQ_WAVE_CYCLES", 1) or 1
        res[k] = {
            "dispatches": len(disp),
            "counters_per_launch": {c: round(v) for c, v in mean.items()},
            "gpu_cycles_per_launch": round(cyc),
            "valu_issue_utilisation": round(mean.get("SQ_INSTS_VALU", 0) / max(cyc * 256 * 2, 1), 4),
            "wave_time_parked_frac": round(mean.get("SQ_WAIT_ANY", 0) / wc, 4),
            "wave_time_issue_stall_frac": round(mean.get("SQ_WAIT_INST_ANY", 0) / wc, 4),
            "wave_time_active_frac": round(mean.get("SQ_ACTIVE_INST_ANY", 0) / wc, 4),
        }
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
