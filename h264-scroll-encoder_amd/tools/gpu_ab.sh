#!/bin/bash
# gpu_ab.sh OUT VARIANT... -- A/B of profiling variants (build_variant.sh):
# bench line + one SQ pass each (abl_sq.sh); with GPU_AB_TESTS=1 the dynamic
# rect parity tests of the default build first.  Every step has its own time
# limit; the first failing step ends the script.
set -e -o pipefail
O=$1; shift
mkdir -p "$O"
git_rev=$(cat .revision 2>/dev/null || true)
echo "revision: $git_rev" > "$O/revision"
if [ "${GPU_AB_TESTS:-0}" = 1 ]; then
    timeout -k 10 300 python3 -u -m pytest tests/test_gpu_dyn.py tests/test_gpu_scale.py -x -q --timeout 240 --timeout-method thread > "$O/tests.log" 2>&1
fi
bash h264-scroll-encoder_amd/tools/abl_sq.sh "$O" "$@"
