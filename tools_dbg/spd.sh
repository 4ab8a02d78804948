set -e -o pipefail
mkdir -p gpurun_out/spdbg
export TMPDIR=/tmp
timeout -k 10 300 python3 -u tools_dbg/spdump.py > gpurun_out/spdbg/log.txt 2>&1
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_dyn.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/spdbg/dyn.log 2>&1
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_splice.py -m gpu -v --timeout 200 --timeout-method thread -k "intra or pcm or multislice" > gpurun_out/spdbg/tests.log 2>&1 || true
