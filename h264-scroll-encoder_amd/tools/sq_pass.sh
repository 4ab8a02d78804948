#!/bin/bash
# sq_pass.sh OUT [KERNEL...] -- one SQ counter pass (rocprofv3 --pmc, its own
# run) over a bench step of the tree's build (workload $SQ_WORKLOAD, default
# the config-3 p720dyn), summarised per kernel (tools/sq_summary.py; default
# the dynamic-rect kernels).  Its own time limit.
set -e -o pipefail
O=$1
shift
mkdir -p "$O"
export TMPDIR=/tmp
W=${SQ_WORKLOAD:-p720dyn}
K=("$@")
if [ ${#K[@]} -eq 0 ]; then
    K=("k_dyn_row<false>" "k_dyn_gather" k_dyn_epfix k_dyn_static k_dyn_epscan k_dyn_rows k_plan k_emit)
fi
timeout -k 10 120 rocprofv3 --output-format csv --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS GRBM_GUI_ACTIVE -d "$O/pmc" -o run -- python3 bench.py --workload $W --steps 2 --warmup 1 --no-cpu --no-verify --no-host > "$O/pmc.log" 2>&1
python3 h264-scroll-encoder_amd/tools/sq_summary.py "$O/pmc" "$O/sq.json" "${K[@]}" > /dev/null
