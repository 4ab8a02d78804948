set -e -o pipefail
O=gpurun_out/ab7
mkdir -p $O
export TMPDIR=/tmp
bash h264-scroll-encoder_amd/tools/ab_prof.sh $O/ab nowin cb2 t256
echo done > $O/DONE
