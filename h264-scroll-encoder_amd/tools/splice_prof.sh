#!/bin/bash
# splice_prof.sh OUT -- the splice GPU tests, the p720splicerows bench line
# and its rocprofv3 kernel stats.  Every GPU step has its own time limit;
# the first failing step ends the script.
set -e -o pipefail
O=$1
mkdir -p "$O"
export TMPDIR=/tmp
T="timeout -k 10"
$T 400 python3 -u -m pytest tests/test_gpu_splice.py tests/test_gpu_hintdyn.py -x -v --timeout 120 --timeout-method thread > "$O/tests.log" 2>&1
$T 240 python3 bench.py --steps 10 --warmup 2 --workload p720splicerows > "$O/bench.json" 2> "$O/bench.err"
$T 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/stats" -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu --no-host --no-verify --workload p720splicerows > "$O/stats.log" 2>&1
echo done > "$O/DONE"
