set -e -o pipefail
O=gpurun_out/abl1
mkdir -p $O
export TMPDIR=/tmp
bash h264-scroll-encoder_amd/tools/abl_sq.sh $O/abl stop0 stop1 stop2 stop3 stop4 full
for v in nosort full; do
    H264SCROLL_LIB=variants/$v/libh264scroll.so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/p_$v" -o run -- python3 bench.py --steps 20 --warmup 3 --no-cpu --no-host --no-verify > "$O/b_$v.json" 2> "$O/b_$v.err"
done
echo done > $O/DONE
