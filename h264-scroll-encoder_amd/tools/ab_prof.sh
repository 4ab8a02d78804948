#!/bin/bash
# ab_prof.sh OUT VARIANT... -- rocprofv3 kernel stats of the bench under each
# library variant (variants/NAME/libh264scroll.so) and the tree's own build
# ("cur"), alternating twice.  Every step has its own time limit; the first
# failure ends it.
set -e -o pipefail
O=$1; shift
mkdir -p "$O"
export TMPDIR=/tmp
W=${AB_WORKLOAD:-p720dyn}
V=--no-verify
[ "${AB_VERIFY:-0}" = 1 ] && V=""                  # the bench's post-timing check of every stream
for rep in 1 2; do
    for v in "$@" cur; do
        if [ "$v" = cur ]; then L=""; else L=variants/$v/libh264scroll.so; fi
        H264SCROLL_LIB=$L timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/${v}_$rep" -o run -- python3 bench.py --steps 20 --warmup 3 --no-cpu --no-host $V --workload $W > "$O/bench_${v}_$rep.json" 2> "$O/bench_${v}_$rep.err"
    done
done
echo done > "$O/DONE"
