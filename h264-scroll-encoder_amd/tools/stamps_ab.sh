#!/bin/bash
# stamps_ab.sh OUT VARIANT... -- the per-workgroup phase stamps
# (dyn_stamps.py) of each library variant and the tree's build ("cur"),
# then ab_bench.sh over the same set.  Every step has its own time limit;
# the first failure ends it.
set -e -o pipefail
O=$1; shift
mkdir -p "$O"
export TMPDIR=/tmp
W=${AB_WORKLOAD:-p720dyn}
for v in "$@" cur; do
    if [ "$v" = cur ]; then L=""; else L=variants/$v/libh264scroll.so; fi
    H264SCROLL_LIB=$L timeout -k 10 200 python3 h264-scroll-encoder_amd/tools/dyn_stamps.py --workload $W > "$O/stamps_$v.txt" 2>&1
done
bash h264-scroll-encoder_amd/tools/ab_bench.sh "$O/ab" "$@"
echo done > "$O/DONE"
