#!/bin/bash
# round_profile.sh TAG [bench|prof|all] -- the measurement set committed under
# profiles/ each round (run on the GPU box from the repo root, e.g. through
# gpurun; "bench" and "prof" fit one gpurun call each):
#   bench: bench lines of every workload (+ config 3 at 1024 streams);
#   prof:  rocprofv3 kernel stats of p720dyn / p4kdyn / p720splicerows /
#          ingest720 / ipcm720, FETCH_SIZE and WRITE_SIZE passes (separate
#          runs) over k_dyn_row (and the splice / ingest launches), one SQ counter pass over the dynamic-rect
#          kernels, and the per-workgroup stamps (dyn_stamps.py).
# Every GPU step has its own time limit; the first failing step ends the script.
set -e -o pipefail
TAG=${1:-r04}
PART=${2:-all}
O=gpurun_out/prof_$TAG
mkdir -p "$O"
export TMPDIR=/tmp
T="timeout -k 10"
if [ "$PART" = bench ] || [ "$PART" = all ]; then
    $T 300 python3 bench.py --steps 20 --warmup 3 > "$O/bench_p720dyn.json" 2> "$O/bench_p720dyn.err"
    for w in p720 p4kdyn p720hint p720splice p720splicerows ingest720 ipcm720; do
        $T 240 python3 bench.py --steps 10 --warmup 2 --workload $w > "$O/bench_$w.json" 2> "$O/bench_$w.err"
    done
    $T 200 python3 bench.py --steps 10 --warmup 2 --streams 1024 --no-cpu > "$O/bench_p720dyn_1024streams.json" 2> /dev/null
fi
if [ "$PART" = prof ] || [ "$PART" = all ]; then
    for w in p720dyn p4kdyn p720splicerows ingest720 ipcm720; do
        $T 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/stats_$w" -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu --no-host --workload $w > "$O/stats_$w.log" 2>&1
    done
    $T 120 rocprofv3 --output-format csv --pmc FETCH_SIZE -d "$O/pmc_fetch" -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu --no-host > "$O/pmc_fetch.log" 2>&1
    $T 120 rocprofv3 --output-format csv --pmc WRITE_SIZE -d "$O/pmc_write" -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu --no-host > "$O/pmc_write.log" 2>&1
    for c in FETCH_SIZE WRITE_SIZE; do          # the splice and ingest launches' traffic (tools/traffic.py)
        $T 120 rocprofv3 --output-format csv --pmc $c -d "$O/pmc_splice_$c" -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu --no-verify --workload p720splicerows > "$O/pmc_splice_$c.log" 2>&1
        $T 120 rocprofv3 --output-format csv --pmc $c -d "$O/pmc_ingest_$c" -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu --no-verify --workload ingest720 > "$O/pmc_ingest_$c.log" 2>&1
    done
    bash h264-scroll-encoder_amd/tools/sq_pass.sh "$O/sq"
    $T 120 python3 h264-scroll-encoder_amd/tools/dyn_stamps.py > "$O/dyn_stamps.txt" 2>&1
fi
echo done > "$O/DONE_$PART"
