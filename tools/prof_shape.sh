#!/bin/bash
# GPU box: kernel trace + PMC passes of tools/shape_time.py (the bench's
# ShuffleDeck16 loss pattern) at SHAPES (K,R,B,LOSS ...); OUT under gpurun_out.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/shape}
SHAPES=${SHAPES:-1000,200,65536,200}
rm -rf $OUT; mkdir -p $OUT
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o t -- python3 tools/shape_time.py $SHAPES > $OUT/kt.log 2>&1 || { echo "trace failed"; tail -20 $OUT/kt.log; exit 1; }
grep workload $OUT/kt.log
python3 tools/trace_summary.py $(find $OUT/kt -name "*kernel_trace.csv") | tee $OUT/trace_summary.txt
find $OUT/kt -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats.csv \;
[ -n "${NO_PMC:-}" ] && { rm -rf $OUT/kt; exit 0; }
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_SALU SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE GRBM_COUNT" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d $OUT/pmc$i -o p -- python3 tools/shape_time.py $SHAPES > $OUT/pmc$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 $OUT/pmc$i.log; exit 1; }
done
python3 tools/pmc_summary.py $OUT/pmc*/ > $OUT/pmc_summary.txt 2>&1
python3 tools/pmc_derive.py $OUT/pmc_summary.txt | tee $OUT/pmc_derived.txt
rm -rf $OUT/kt $OUT/pmc*/
echo done
