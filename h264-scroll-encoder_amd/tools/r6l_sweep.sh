set -e -o pipefail
O=gpurun_out/r6l; mkdir -p $O; export TMPDIR=/tmp
for rep in 1 2; do
  for v in sr8 sr16; do
    H264SCROLL_LIB=variants/$v/libh264scroll.so timeout -k 10 200 python3 bench.py --steps 20 --warmup 3 --no-cpu --no-host --workload p4kdyn > $O/${v}_$rep.json 2> $O/${v}_$rep.err
  done
  for z in 2 4 6; do
    SCROLL_GATHER_Z=$z H264SCROLL_LIB=variants/sr16/libh264scroll.so timeout -k 10 200 python3 bench.py --steps 20 --warmup 3 --no-cpu --no-host --workload p4kdyn > $O/sr16z${z}_$rep.json 2> $O/sr16z${z}_$rep.err
  done
done
H264SCROLL_LIB=variants/sr8/libh264scroll.so timeout -k 10 300 python -u -m pytest tests/test_gpu_dyn.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/tests_sr8.log 2>&1
echo done > $O/DONE
