#!/bin/bash
# GPU box: selected GPU tests (PYTEST_K, all when empty), then bbench / kbench / bench as asked.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 ${PYTEST_TIMEOUT:-400} python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_q.log 2>&1; rc=$?
tail -4 gpurun_out/pytest_q.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/pytest_q.log | head -20; exit $rc; }
if [ -n "${BB_ARGS:-}" ]; then timeout -k 10 120 python3 tools/bbench.py $BB_ARGS 2>&1 | grep -v amdgpu.ids || exit 1; fi
if [ -n "${KB_ARGS:-}" ]; then timeout -k 10 200 python3 tools/kbench.py $KB_ARGS 2>&1 | grep -v amdgpu.ids || exit 1; fi
if [ -n "${BENCH:-}" ]; then timeout -k 10 500 python3 bench.py $BENCH_ARGS > gpurun_out/bench_q.json 2> gpurun_out/bench_q.err || { tail -20 gpurun_out/bench_q.err; exit 1; }; head -c 1500 gpurun_out/bench_q.json; echo; fi
