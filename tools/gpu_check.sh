#!/bin/bash
# GPU box: selected GPU tests (PYTEST_K), then kbench on KB_ARGS.  Each step under its own limit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ -n "${PYTEST_K:-}" ]; then
  timeout -k 10 ${PYTEST_TIMEOUT:-600} python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$PYTEST_K" > gpurun_out/pytest_sel.log 2>&1; rc=$?
  tail -15 gpurun_out/pytest_sel.log
  [ $rc -eq 0 ] || exit $rc
fi
if [ -n "${KB_ARGS:-}" ]; then
  timeout -k 10 300 python3 tools/kbench.py $KB_ARGS || exit 1
fi
