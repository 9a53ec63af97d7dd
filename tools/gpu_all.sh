#!/bin/bash
# GPU-box: parity tests (fast subset unless FULL=1) then the bench (+ optional profile).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
if [ -n "${FULL:-}" ]; then K=""; else K="not baseline"; fi
PYTEST_K="$K" bash tools/gpu_tests.sh || exit 1
bash tools/gpu_bench.sh
