#!/bin/bash
# GPU box: FF16 kernel attribution at 32768+32768 x 64 KiB (and 1000+200):
# kernel trace, then PMC passes (one counter set per run, no tracing domains).
# OUT: directory under gpurun_out; KB_ARGS overrides the shapes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/ff16}
ARGS=${KB_ARGS:-32768 32768 65536 1000 200 65536}
rm -rf $OUT; mkdir -p $OUT
export KB_WARM=${KB_WARM:-3}
export KB_N=${KB_N:-10}
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o t -- python3 tools/kbench.py $ARGS > $OUT/kt.log 2>&1 || { echo "trace failed"; tail -20 $OUT/kt.log; exit 1; }
grep -E " x " $OUT/kt.log
python3 tools/trace_summary.py $(find $OUT/kt -name "*kernel_trace.csv") | tee $OUT/trace_summary.txt
find $OUT/kt -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats.csv \;
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT" \
           "FETCH_SIZE" "WRITE_SIZE" ${EXTRA_PMC:-}; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d $OUT/pmc$i -o p -- python3 tools/kbench.py $ARGS > $OUT/pmc$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 $OUT/pmc$i.log; exit 1; }
done
python3 tools/pmc_summary.py $OUT/pmc*/ > $OUT/pmc_summary.txt 2>&1; tail -60 $OUT/pmc_summary.txt
rm -rf $OUT/kt $OUT/pmc*/  # raw CSVs: too large to copy back
echo done
