#!/bin/bash
# traffic_ab.sh OUT WORKLOAD VARIANT... -- the FETCH_SIZE / WRITE_SIZE passes
# (separate runs) of one bench workload for library variants
# (variants/NAME/libh264scroll.so) and the tree's build ("cur"); then
# tools/traffic.py per variant on the build host.  Every run has its own time
# limit; the first failure ends it.
set -e -o pipefail
O=$1; W=$2; shift 2
mkdir -p "$O"
export TMPDIR=/tmp
for v in "$@" cur; do
    if [ "$v" = cur ]; then L=""; else L=variants/$v/libh264scroll.so; fi
    for c in FETCH_SIZE WRITE_SIZE; do
        H264SCROLL_LIB=$L timeout -s KILL 150 rocprofv3 --output-format csv --pmc $c -d "$O/pmc_${v}_$c" -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu --no-host --no-verify --workload $W > "$O/pmc_${v}_$c.log" 2>&1
    done
done
echo done > "$O/DONE"
