#!/bin/bash
# ingest_prof.sh OUT -- the ingest720 workload's GPU tests, bench line,
# rocprofv3 kernel stats and FETCH_SIZE / WRITE_SIZE passes (separate runs)
# for tools/traffic.py.  Every GPU step has its own time limit; the first
# failing step ends the script.
set -e -o pipefail
O=$1
mkdir -p "$O"
export TMPDIR=/tmp
T="timeout -k 10"
$T 300 python3 -u -m pytest tests/test_gpu_ingest.py tests/test_gpu_ipcm.py tests/test_gpu_refupdate.py -x -v --timeout 120 --timeout-method thread > "$O/tests.log" 2>&1
$T 240 python3 bench.py --steps 10 --warmup 2 --workload ingest720 > "$O/bench.json" 2> "$O/bench.err"
$T 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/stats" -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu --no-host --workload ingest720 > "$O/stats.log" 2>&1
for c in FETCH_SIZE WRITE_SIZE; do
    $T 120 rocprofv3 --output-format csv --pmc $c -d "$O/pmc_$c" -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu --no-verify --workload ingest720 > "$O/pmc_$c.log" 2>&1
done
echo done > "$O/DONE"
