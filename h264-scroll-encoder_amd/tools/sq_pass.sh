#!/bin/bash
# sq_pass.sh OUT -- one SQ counter pass (rocprofv3 --pmc, its own run) over the
# config-3 step of the tree's build, summarised per dynamic-rect kernel
# (tools/sq_summary.py).  Its own time limit.
set -e -o pipefail
O=$1
mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --output-format csv --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS GRBM_GUI_ACTIVE -d "$O/pmc" -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu --no-verify --no-host > "$O/pmc.log" 2>&1
python3 h264-scroll-encoder_amd/tools/sq_summary.py "$O/pmc" "$O/sq.json" "k_dyn_row<false>" "k_dyn_emit_gather<1, true>" k_dyn_epfix k_dyn_static k_dyn_epscan k_dyn_rows k_plan k_emit > /dev/null
