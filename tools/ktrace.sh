#!/bin/bash
# GPU box: per-kernel durations (rocprofv3 kernel trace) of kbench for one or more
# library builds.  LIBS="name=path ..." (default: the product library).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
LIBS=${LIBS:-"main=leopard_amd/lib/libleopard_amd.so"}
for spec in $LIBS; do
  name=${spec%%=*}; lib=${spec#*=}
  rm -rf gpurun_out/kt_$name
  LEOPARD_AMD_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/kt_$name -o t -- python3 tools/kbench.py ${KB_ARGS:-128 128 65536 128 128 1048576} > gpurun_out/kt_$name.log 2>&1 || { echo "fail $name"; tail -20 gpurun_out/kt_$name.log; exit 1; }
  echo "== $name"; grep -E " x " gpurun_out/kt_$name.log
  python3 tools/trace_summary.py $(find gpurun_out/kt_$name -name "*kernel_trace.csv")
done
