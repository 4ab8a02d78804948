#!/bin/bash
# ipcm_sweep.sh OUT -- I_PCM file writer variants (round 6): the tree's two
# passes ("cur"), the one pass at 4 KB chunks (ip1) and at 8 KB (ip8), and
# ip8's two passes (SCROLL_IPCM_TWOPASS=1), alternating twice; then the
# I_PCM / ingest GPU tests on ip8.  Each run has its own time limit.
set -e -o pipefail
O=$1; mkdir -p "$O"; export TMPDIR=/tmp
run() { # name lib env...
    local nm=$1 lib=$2; shift 2
    env "$@" H264SCROLL_LIB=$lib timeout -k 10 200 python3 bench.py --steps 20 --warmup 3 --no-cpu --no-host --workload ipcm720 > "$O/$nm.json" 2> "$O/$nm.err"
}
for rep in 1 2; do
    run cur_$rep ""
    run ip1_$rep variants/ip1/libh264scroll.so
    run ip8_$rep variants/ip8/libh264scroll.so
    run ip8two_$rep variants/ip8/libh264scroll.so SCROLL_IPCM_TWOPASS=1
done
H264SCROLL_LIB=variants/ip8/libh264scroll.so timeout -k 10 300 python -u -m pytest tests/test_gpu_ipcm.py tests/test_gpu_ingest.py -x -q -m gpu --timeout 120 --timeout-method thread > "$O/tests_ip8.log" 2>&1
echo done > "$O/DONE"
