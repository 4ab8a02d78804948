#!/bin/bash
# abl_sq.sh OUTDIR VARIANT... -- per profiling variant (build_variant.sh) a
# p720dyn bench line and one SQ counter pass (rocprofv3 --pmc, its own run)
# over the dynamic-rect kernels: VALU / SALU / LDS instruction counts and
# wave-cycle split per launch.  Every GPU step has its own time limit; the
# first failing step ends the script.
set -e -o pipefail
O=$1; shift
mkdir -p "$O"
export TMPDIR=/tmp
for v in "$@"; do
    L=variants/$v/libh264scroll.so
    H264SCROLL_LIB=$L timeout -k 10 120 python3 bench.py --steps 10 --warmup 2 --no-cpu --no-verify > "$O/$v.json" 2> "$O/$v.err"
    python3 -c "import json; d=json.load(open('$O/$v.json')); print('$v', d['ms_per_step'], d['roofline']['kernel_ms_avg'])" >> "$O/variants.txt"
    H264SCROLL_LIB=$L timeout -k 10 120 rocprofv3 --output-format csv --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS GRBM_GUI_ACTIVE -d "$O/pmc_$v" -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu --no-verify > "$O/pmc_$v.log" 2>&1
    python3 h264-scroll-encoder_amd/tools/sq_summary.py "$O/pmc_$v" "$O/sq_$v.json" "k_dyn_row<false>" > /dev/null
    python3 -c "import json; d=json.load(open('$O/sq_$v.json')); [print('$v', k, v['counters_per_launch']['SQ_INSTS_VALU'], v['counters_per_launch']['SQ_INSTS_SALU'], v['gpu_cycles_per_launch'], v['valu_issue_utilisation']) for k, v in d.items()]" >> "$O/variants.txt"
done
echo done > "$O/DONE"
