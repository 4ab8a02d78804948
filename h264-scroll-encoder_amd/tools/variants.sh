#!/bin/bash
# variants.sh OUTDIR NAME... -- bench line (p720dyn, no CPU leg, no check) of
# each profiling variant built by build_variant.sh; one line per variant in
# OUTDIR/variants.txt.  Each run has its own time limit; a failing run ends
# the script.
set -e -o pipefail
O=$1; shift
mkdir -p "$O"
for v in "$@"; do
    H264SCROLL_LIB=variants/$v/libh264scroll.so timeout -k 10 120 python3 bench.py --steps 10 --warmup 2 --no-cpu --no-verify $EXTRA > "$O/$v.json" 2> "$O/$v.err"
    python3 -c "import json,sys; d=json.load(open('$O/$v.json')); k=d['roofline']['kernel_ms_avg']; print('$v', d['ms_per_step'], k)" >> "$O/variants.txt"
done
