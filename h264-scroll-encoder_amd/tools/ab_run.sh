#!/bin/bash
# ab_run.sh TAG [VARIANT...] -- one build -> measure call on the GPU box
# (through gpurun, from the repo root): every GPU test of the tree's build,
# the per-workgroup stamps of k_dyn_row / k_dyn_epfix / k_dyn_gather
# (dyn_stamps.py), then ab_prof.sh over the named library variants
# (build_variant.sh) and the tree's build.  AB_TESTS=0 skips the tests,
# AB_SQ=1 adds one SQ counter pass (sq_pass.sh) of the tree's build.
# Every GPU step has its own time limit; the first failing step ends it.
set -e -o pipefail
O=gpurun_out/$1
shift
mkdir -p "$O"
export TMPDIR=/tmp
if [ "${AB_TESTS:-1}" != 0 ]; then
    timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$O/tests.log" 2>&1
fi
timeout -k 10 200 python3 h264-scroll-encoder_amd/tools/dyn_stamps.py > "$O/stamps.txt" 2>&1
bash h264-scroll-encoder_amd/tools/ab_prof.sh "$O/ab" "$@"
if [ "${AB_SQ:-0}" = 1 ]; then
    bash h264-scroll-encoder_amd/tools/sq_pass.sh "$O/sq"
fi
echo done > "$O/DONE"
