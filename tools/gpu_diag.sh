#!/bin/bash
# GPU box: ablation kernel-time table + PMC passes for the 128+128 x 64 KiB kernels.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
ABL="${ABL:-0 1 2 4 8 12 15 16}" KB_ARGS="${KB_ARGS:-128 128 65536 128 128 1048576}" bash tools/_prof_abl.sh > gpurun_out/abl.log 2>&1 || { tail -20 gpurun_out/abl.log; exit 1; }
cat gpurun_out/abl.log
[ -n "${NOPMC:-}" ] && exit 0
KB_ARGS="128 128 65536" bash tools/pmc.sh "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAVE_CYCLES" "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA" "FETCH_SIZE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" "WRITE_SIZE SQ_INSTS_BRANCH SQ_ACTIVE_INST_MISC"
python3 tools/pmc_summary.py gpurun_out/pmc1 gpurun_out/pmc2 gpurun_out/pmc3 gpurun_out/pmc4 2>&1 | tee gpurun_out/pmc_summary.txt
