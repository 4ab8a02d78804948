#!/bin/bash
# gpu_ab.sh OUT VARIANT... -- A/B of profiling variants (build_variant.sh):
# bench line + one SQ pass each (abl_sq.sh); with GPU_AB_TESTS="test files"
# those tests of the default build first, and GPU_AB_BENCH=1 a full bench
# line of the default build (all legs).  Every step has its own time
# limit; the first failing step ends the script.
set -e -o pipefail
O=$1; shift
mkdir -p "$O"
git_rev=$(cat .revision 2>/dev/null || true)
echo "revision: $git_rev" > "$O/revision"
if [ -n "${GPU_AB_TESTS:-}" ]; then
    timeout -k 10 400 python3 -u -m pytest $GPU_AB_TESTS -x -v --timeout 240 --timeout-method thread > "$O/tests.log" 2>&1
fi
if [ "${GPU_AB_BENCH:-0}" = 1 ]; then
    timeout -k 10 300 python3 bench.py > "$O/bench.json" 2> "$O/bench.err"
fi
bash h264-scroll-encoder_amd/tools/abl_sq.sh "$O" "$@"
