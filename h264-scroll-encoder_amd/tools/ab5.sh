set -e -o pipefail
O=gpurun_out/ab5
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
timeout -k 10 200 python3 h264-scroll-encoder_amd/tools/dyn_stamps.py > $O/stamps.txt 2>&1
bash h264-scroll-encoder_amd/tools/ab_prof.sh $O/ab
echo done > $O/DONE
