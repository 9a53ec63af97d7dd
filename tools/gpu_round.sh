#!/bin/bash
# GPU box: default bench line, the same bench under rocprofv3 --kernel-trace --stats,
# then the FETCH_SIZE / WRITE_SIZE passes for roofline.traffic.  Each step under its
# own time limit; stop at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
OUT=${OUT:-gpurun_out/round}
rm -rf $OUT; mkdir -p $OUT
timeout -k 10 600 python3 bench.py ${BENCH_ARGS:-} > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-host --no-secondary ${BENCH_ARGS:-} > $OUT/prof_bench.json 2> $OUT/prof.err || { tail -20 $OUT/prof.err; exit 1; }
cat $OUT/prof_bench.json
find $OUT/prof -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats.csv \;
python3 tools/trace_summary.py $(find $OUT/prof -name "*kernel_trace.csv") > $OUT/trace_summary.txt && grep "run of" $OUT/trace_summary.txt
KB_ARGS="${PMC_ARGS:-128 128 65536}" bash tools/pmc.sh FETCH_SIZE WRITE_SIZE || exit 1
python3 tools/pmc_traffic.py ${PMC_ARGS:-128 128 65536} gpurun_out/pmc1 gpurun_out/pmc2 > $OUT/pmc_traffic.json && cat $OUT/pmc_traffic.json
# the batch kernels of the headline (LAUNCH_OBJ objects per launch, the bench default 64)
rm -rf gpurun_out/pmc1 gpurun_out/pmc2
PMC_TOOL=bbench KB_ARGS="${PMC_ARGS:-128 128 65536} ${LAUNCH_OBJ:-64}" bash tools/pmc.sh FETCH_SIZE WRITE_SIZE || exit 1
python3 tools/pmc_traffic.py --objects ${LAUNCH_OBJ:-64} ${PMC_ARGS:-128 128 65536} gpurun_out/pmc1 gpurun_out/pmc2 > $OUT/pmc_traffic_batch.json && cat $OUT/pmc_traffic_batch.json
rm -rf gpurun_out/pmc1 gpurun_out/pmc2 $OUT/prof  # raw passes and traces: summarised above
