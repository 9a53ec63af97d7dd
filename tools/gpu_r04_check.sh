#!/bin/bash
# GPU box, round 4: the GPU test suite, the default bench line, and the bench
# launched with --gpus 2 (two ranks sharing the box's one GPU).  Each step
# under its own time limit; stop at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r04}
rm -rf $OUT; mkdir -p $OUT
timeout -k 10 ${TEST_LIMIT:-420} python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    ${TEST_ARGS:-} > $OUT/pytest_gpu.txt 2>&1 || { tail -40 $OUT/pytest_gpu.txt; exit 1; }
tail -3 $OUT/pytest_gpu.txt
[ -n "${NO_BENCH:-}" ] && exit 0
timeout -k 10 400 python3 bench.py ${BENCH_ARGS:-} > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
head -c 3000 $OUT/bench.json
[ -n "${NO_N2:-}" ] && exit 0
timeout -k 10 400 python3 bench.py --gpus 2 --steps 20 --warmup 5 --no-secondary --no-cpu-baseline --no-host \
    > $OUT/bench_n2.json 2> $OUT/bench_n2.err || { tail -30 $OUT/bench_n2.err; exit 1; }
head -c 3000 $OUT/bench_n2.json
