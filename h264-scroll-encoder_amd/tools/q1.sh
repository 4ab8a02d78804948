set -e -o pipefail
O=gpurun_out/q1
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_dyn.py tests/test_gpu_scale.py tests/test_gpu_hintdyn.py tests/test_gpu_splice.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1
timeout -k 10 200 python3 bench.py --steps 20 --warmup 3 > $O/bench.json 2> $O/bench.err
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu --no-host > $O/stats.log 2>&1
echo done > $O/DONE
