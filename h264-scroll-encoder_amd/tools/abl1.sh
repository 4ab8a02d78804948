set -e -o pipefail
O=gpurun_out/abl1
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_dyn.py tests/test_gpu_scale.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
bash h264-scroll-encoder_amd/tools/ab_prof.sh $O/ovl noovl
bash h264-scroll-encoder_amd/tools/abl_sq.sh $O/abl stop0 stop1 stop2 stop3 stop4 full
for v in nosort full; do
    H264SCROLL_LIB=variants/$v/libh264scroll.so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/p_$v" -o run -- python3 bench.py --steps 20 --warmup 3 --no-cpu --no-host --no-verify > "$O/b_$v.json" 2> "$O/b_$v.err"
done
echo done > $O/DONE
