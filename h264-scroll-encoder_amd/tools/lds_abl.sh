#!/bin/bash
# lds_abl.sh OUTDIR VARIANT... -- per library variant (build_variant.sh, e.g.
# the -DSCROLL_ABL_STOP=n phase cuts) and the tree's build ("cur"): one
# counter pass over a p720dyn bench step -- LDS instructions, bank-conflict
# and LDS-active cycles, LDS waits, vector-memory loads, texture address /
# data busy.  Each run has its own time limit; the first failure ends it.
set -e -o pipefail
O=$1; shift
mkdir -p "$O"
export TMPDIR=/tmp
for v in "$@" cur; do
    if [ "$v" = cur ]; then L=""; else L=variants/$v/libh264scroll.so; fi
    H264SCROLL_LIB=$L timeout -s KILL 120 rocprofv3 --output-format csv --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE TA_TA_BUSY_sum TD_TD_BUSY_sum -d "$O/pmc_$v" -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu --no-verify --no-host > "$O/pmc_$v.log" 2>&1
done
echo done > "$O/DONE"
