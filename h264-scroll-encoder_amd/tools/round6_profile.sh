#!/bin/bash
# round6_profile.sh TAG PART -- the round-6 measurement set (run on the GPU
# box from the repo root through gpurun; each PART fits one call):
#   bench: bench lines of every workload, config 3 at 1024 streams and at
#          --frames 1 (one real-time tick per stream: 256 frames per compose,
#          src/composer.c:255-264 is one call per frame);
#   prof:  rocprofv3 kernel stats of every compose workload and the raw
#          FETCH_SIZE / WRITE_SIZE passes (separate runs) of each dominant
#          kernel; tools/traffic.py turns them into profiles/traffic_*.json
#          on the build host with the bench lines' algorithmic bytes;
#   sq:    SQ counter passes (config 3 and config 5), the LDS / texture
#          counters of k_dyn_row, the per-workgroup stamps.
# Every GPU step has its own time limit; the first failing step ends it.
set -e -o pipefail
TAG=${1:-r06}
PART=${2:-bench}
O=gpurun_out/prof_$TAG
mkdir -p "$O"
export TMPDIR=/tmp
T="timeout -k 10"
REV=$(cat .revision 2>/dev/null | tr '\n' ' ')
echo "revision: $REV" > "$O/REVISION_$PART"
if [ "$PART" = bench ]; then
    $T 300 python3 bench.py --steps 20 --warmup 3 > "$O/bench_p720dyn.json" 2> "$O/bench_p720dyn.err"
    for w in p720 p4kdyn p720full p720hint p720splice p720splicerows ingest720 ipcm720; do
        $T 240 python3 bench.py --steps 10 --warmup 2 --workload $w > "$O/bench_$w.json" 2> "$O/bench_$w.err"
    done
    $T 200 python3 bench.py --steps 10 --warmup 2 --streams 1024 --no-cpu > "$O/bench_p720dyn_1024streams.json" 2> "$O/bench_p720dyn_1024streams.err"
    $T 200 python3 bench.py --steps 50 --warmup 5 --frames 1 --no-cpu > "$O/bench_p720dyn_frames1.json" 2> "$O/bench_p720dyn_frames1.err"
fi
if [ "$PART" = prof ]; then
    for w in p720dyn p4kdyn p720 p720full p720splicerows ingest720 ipcm720; do
        $T 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/stats_$w" -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu --no-host --no-verify --workload $w > "$O/stats_$w.log" 2>&1
    done
    for w in p720dyn p4kdyn p720 p720full p720splicerows ingest720 ipcm720; do
        for c in FETCH_SIZE WRITE_SIZE; do
            $T 150 rocprofv3 --output-format csv --pmc $c -d "$O/pmc_${w}_$c" -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu --no-host --no-verify --workload $w > "$O/pmc_${w}_$c.log" 2>&1
        done
    done
fi
if [ "$PART" = sq ]; then
    bash h264-scroll-encoder_amd/tools/sq_pass.sh "$O/sq_p720dyn"
    SQ_WORKLOAD=p4kdyn bash h264-scroll-encoder_amd/tools/sq_pass.sh "$O/sq_p4kdyn"
    bash h264-scroll-encoder_amd/tools/lds_abl.sh "$O/lds"
    $T 150 python3 h264-scroll-encoder_amd/tools/dyn_stamps.py > "$O/dyn_stamps_p720dyn.txt" 2>&1
    $T 200 python3 h264-scroll-encoder_amd/tools/dyn_stamps.py --workload p4kdyn > "$O/dyn_stamps_p4kdyn.txt" 2>&1
fi
echo done > "$O/DONE_$PART"
