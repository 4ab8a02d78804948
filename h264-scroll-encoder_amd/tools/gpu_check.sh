#!/bin/bash
# gpu_check.sh TAG -- the parity + bench run of a revision on the GPU box
# (through gpurun, from the repo root).  .revision (written on the build host
# before the call: `git rev-parse HEAD`, plus "dirty" for uncommitted changes)
# heads every log, so each result names the source it ran.  Every GPU step has
# its own time limit; the first failing step ends the script.
set -e -o pipefail
TAG=${1:-check}
O=gpurun_out/$TAG
mkdir -p "$O"
export TMPDIR=/tmp
REV=$(cat .revision 2>/dev/null | tr '\n' ' ')
for f in gpu_tests.log smoke.log; do echo "revision: $REV" > "$O/$f"; done
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread >> "$O/gpu_tests.log" 2>&1
timeout -k 10 180 python3 -c "import __graft_entry__ as g; g.smoke()" >> "$O/smoke.log" 2>&1
timeout -k 10 300 python3 bench.py > "$O/bench.json" 2> "$O/bench.err"
echo "revision: $REV" > "$O/DONE"
