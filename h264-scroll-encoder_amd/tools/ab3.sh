set -e -o pipefail
O=gpurun_out/ab3
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 python3 h264-scroll-encoder_amd/tools/dyn_stamps.py > $O/stamps.txt 2>&1
bash h264-scroll-encoder_amd/tools/ab_prof.sh $O/ab epf256l epf128l epf64l
echo done > $O/DONE
