#!/bin/bash
# round6_final.sh OUT -- the round's closing check on one box: the whole GPU
# suite, smoke(), the default bench line and the rocprofv3 kernel stats of the
# same command (so the bench's HIP-event time and rocprof's average come from
# one box), then the SQ / LDS / stamp passes.  Each step has its own time
# limit; the first failure ends it.
set -e -o pipefail
O=$1; mkdir -p "$O"; export TMPDIR=/tmp
REV=$(cat .revision 2>/dev/null | tr '\n' ' ')
echo "revision: $REV" > "$O/REVISION"
timeout -k 10 700 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > "$O/gpu_tests.log" 2>&1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$O/smoke.log" 2>&1
timeout -k 10 300 python3 bench.py > "$O/bench_p720dyn.json" 2> "$O/bench_p720dyn.err"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/stats_default" -o run -- python3 bench.py > "$O/stats_default.log" 2>&1
bash h264-scroll-encoder_amd/tools/sq_pass.sh "$O/sq_p720dyn"
SQ_WORKLOAD=p4kdyn bash h264-scroll-encoder_amd/tools/sq_pass.sh "$O/sq_p4kdyn"
bash h264-scroll-encoder_amd/tools/lds_abl.sh "$O/lds"
timeout -k 10 150 python3 h264-scroll-encoder_amd/tools/dyn_stamps.py > "$O/dyn_stamps_p720dyn.txt" 2>&1
echo done > "$O/DONE"
