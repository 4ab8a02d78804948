#!/bin/bash
# ab_bench.sh OUT VARIANT... -- config-3 bench lines of library variants
# (variants/NAME/libh264scroll.so, built from other revisions or with other
# defines) next to the tree's own build ("cur"), alternating twice so box
# drift shows.  Every step has its own time limit; the first failure ends it.
set -e -o pipefail
O=$1; shift
mkdir -p "$O"
export TMPDIR=/tmp
W=${AB_WORKLOAD:-p720dyn}
A=${AB_ARGS:-}          # extra bench.py arguments, e.g. "--frames 1 --steps 50"
for rep in 1 2; do
    for v in "$@" cur; do
        if [ "$v" = cur ]; then L=""; else L=variants/$v/libh264scroll.so; fi
        H264SCROLL_LIB=$L timeout -k 10 200 python3 bench.py --steps 20 --warmup 3 --no-cpu --no-host --workload $W $A > "$O/bench_${v}_$rep.json" 2> "$O/bench_${v}_$rep.err"
    done
done
echo done > "$O/DONE"
