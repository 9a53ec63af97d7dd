#!/bin/bash
# GPU box: rocprofv3 kernel trace + PMC passes (SQ issue/wait counters,
# instruction cache, HBM bytes) of one measurement command.
#   OUT=gpurun_out/x CMD="python3 tools/bbench.py 128 128 65536 16" bash tools/prof.sh
# Writes $OUT/kernel_stats.csv, trace_summary.txt, pmc_summary.txt, pmc_derived.txt.
# Each pass is its own run under its own time limit (no tracing domains with --pmc).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/prof}
CMD=${CMD:?set CMD}
rm -rf $OUT; mkdir -p $OUT
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o t -- $CMD > $OUT/kt.log 2>&1 || { echo "trace failed"; tail -20 $OUT/kt.log; exit 1; }
grep -v amdgpu.ids $OUT/kt.log | tail -5
python3 tools/trace_summary.py $(find $OUT/kt -name "*kernel_trace.csv") > $OUT/trace_summary.txt
find $OUT/kt -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats.csv \;
rm -rf $OUT/kt
[ -n "${NO_PMC:-}" ] && exit 0
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_SALU SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE GRBM_COUNT" \
           "SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQC_ICACHE_REQ" \
           ${PMC_EXTRA:-} "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d $OUT/pmc$i -o p -- $CMD > $OUT/pmc$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 $OUT/pmc$i.log; exit 1; }
done
python3 tools/pmc_summary.py $OUT/pmc*/ > $OUT/pmc_summary.txt 2>&1
python3 tools/pmc_derive.py $OUT/pmc_summary.txt > $OUT/pmc_derived.txt
rm -rf $OUT/pmc*/ $OUT/*.log
cat $OUT/pmc_derived.txt
echo done
