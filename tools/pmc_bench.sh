#!/bin/bash
# GPU box: PMC counter sets over a short headline bench (LIB = library to load).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/pmcb}; rm -rf $OUT; mkdir -p $OUT
export LEOPARD_AMD_LIB=${LIB:-leopard_amd/lib/libleopard_amd.so}
CMD="python3 bench.py --steps 20 --warmup 2 --no-sharded --no-secondary --no-host --no-cpu-baseline ${BENCH_ARGS:-}"
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_SMEM" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE GRBM_COUNT" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $set --output-format csv -d $OUT/p$i -o p -- $CMD > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
python3 tools/pmc_summary.py $OUT/p*/ > $OUT/summary.txt; rm -rf $OUT/p1 $OUT/p2 $OUT/p3 $OUT/p4
python3 tools/pmc_derive.py $OUT/summary.txt
