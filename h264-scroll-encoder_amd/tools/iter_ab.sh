#!/bin/bash
# iter_ab.sh TAG [VARIANT...] -- one build -> measure call on the GPU box
# (through gpurun, from the repo root): the dynamic-rect parity tests (or
# $ITER_TESTS), A/B bench lines of the named library variants against the
# tree's build (ab_bench.sh), and one SQ counter pass of the tree's build
# (sq_pass.sh; ITER_SQ=0 skips it).  Every GPU step has its own time limit;
# the first failing step ends the script.
set -e -o pipefail
O=gpurun_out/$1
shift
mkdir -p "$O"
export TMPDIR=/tmp
echo "revision: $(cat .revision 2>/dev/null | tr '\n' ' ')" > "$O/revision"
T=${ITER_TESTS:-tests/test_gpu_dyn.py tests/test_gpu_scale.py}
if [ "$T" != none ]; then
    timeout -k 10 600 python3 -u -m pytest $T -m gpu -x -q --timeout 300 --timeout-method thread > "$O/tests.log" 2>&1
fi
bash h264-scroll-encoder_amd/tools/ab_bench.sh "$O/ab" "$@"
if [ "${ITER_SQ:-1}" != 0 ]; then
    bash h264-scroll-encoder_amd/tools/sq_pass.sh "$O/sq"
fi
echo done > "$O/DONE"
