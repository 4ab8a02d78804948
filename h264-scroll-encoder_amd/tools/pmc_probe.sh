#!/bin/bash
# pmc_probe.sh OUT -- the counter list of the box (rocprofv3 -L) and three
# extra counter passes over a config-3 bench step (each its own run and time
# limit): LDS / memory-instruction SQ counters, then texture-path busy
# counters, then L2 (TCC) hit / miss and L1 (TCP) requests.  The first
# failing step ends the script.
set -e -o pipefail
O=$1
mkdir -p "$O"
export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > "$O/counters.txt" 2>&1
timeout -s KILL 120 rocprofv3 --output-format csv --pmc SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAIT_ANY -d "$O/pmc1" -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu --no-verify --no-host > "$O/pmc1.log" 2>&1
echo ok1 > "$O/DONE1"
timeout -s KILL 120 rocprofv3 --output-format csv --pmc TA_TA_BUSY_sum TD_TD_BUSY_sum GRBM_GUI_ACTIVE -d "$O/pmc2" -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu --no-verify --no-host > "$O/pmc2.log" 2>&1
echo ok2 > "$O/DONE2"
timeout -s KILL 120 rocprofv3 --output-format csv --pmc TCC_HIT_sum TCC_MISS_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum -d "$O/pmc3" -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu --no-verify --no-host > "$O/pmc3.log" 2>&1
echo ok3 > "$O/DONE3"
