#!/bin/bash
# GPU box: smoke + parity suite (PYTEST_K filter) + quick kernel timings.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "SMOKE FAILED"; tail -30 gpurun_out/smoke.log; exit 1; }
timeout -k 10 ${PYTEST_TIMEOUT:-900} python -m pytest tests -x -q -m gpu -k "${PYTEST_K:-}" > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 300 python tools/kbench.py ${KB_ARGS:-128 128 65536 128 128 1048576 1000 200 65536 32768 32768 65536} 2>&1 | tee gpurun_out/kbench.log
