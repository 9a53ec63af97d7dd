#!/bin/bash
# GPU box: rocprofv3 kernel trace of tools/dec_ab.py shapes (AB_SHAPES), per-kernel summary.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/dt
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/dt -o t -- python3 tools/dec_ab.py ${AB_SHAPES:-1000 200 65536 200} > gpurun_out/dt.log 2>&1 || { tail -20 gpurun_out/dt.log; exit 1; }
grep workload gpurun_out/dt.log | cut -c1-300
python3 tools/trace_summary.py $(find gpurun_out/dt -name "*kernel_trace.csv")
