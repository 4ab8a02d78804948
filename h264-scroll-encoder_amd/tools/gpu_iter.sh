#!/bin/bash
# gpu_iter.sh TAG [pytest files...] -- one build -> measure iteration on the GPU
# box (through gpurun, from the repo root): the dynamic-rect parity tests (or
# the files named), the config-3 bench line, and rocprofv3 kernel stats of it.
# Every GPU step has its own time limit; the first failing step ends the script.
set -e -o pipefail
TAG=${1:-iter}
shift || true
FILES=${*:-tests/test_gpu_dyn.py tests/test_gpu_scale.py}
O=gpurun_out/$TAG
mkdir -p "$O"
export TMPDIR=/tmp
REV=$(cat .revision 2>/dev/null | tr '\n' ' ')
echo "revision: $REV" > "$O/tests.log"
timeout -k 10 600 python3 -u -m pytest $FILES -m gpu -x -v --timeout 300 --timeout-method thread >> "$O/tests.log" 2>&1
timeout -k 10 200 python3 bench.py --steps 20 --warmup 3 > "$O/bench.json" 2> "$O/bench.err"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/stats" -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu --no-host > "$O/stats.log" 2>&1
echo "revision: $REV" > "$O/DONE"
