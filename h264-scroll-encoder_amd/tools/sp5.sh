set -e -o pipefail
O=gpurun_out/sp5
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_splice.py tests/test_gpu_hintdyn.py -m gpu -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1
timeout -k 10 300 python3 bench.py --workload p720splicerows --steps 10 --warmup 2 --no-cpu > $O/bench_rows.json 2> $O/bench_rows.err
timeout -k 10 300 python3 bench.py --workload p720splice --steps 10 --warmup 2 --no-cpu > $O/bench_splice.json 2> $O/bench_splice.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats_rows -o run -- python3 bench.py --workload p720splicerows --steps 5 --warmup 2 --no-cpu --no-verify > $O/stats.log 2>&1
SQ_WORKLOAD=p720splicerows bash h264-scroll-encoder_amd/tools/sq_pass.sh $O/sq k_splice_lanes k_splice_stage k_splice_parse k_splice_unesc k_splice_units
echo done > $O/DONE
