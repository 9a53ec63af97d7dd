#!/bin/bash
# GPU box: rocprofv3 kernel trace of tools/shape_time.py at SHAPES for the
# shipped library and each leopard_amd/exp/<name> in VARIANTS (per-kernel
# averages: tools/trace_summary.py); OUT directory.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/tv}; rm -rf $OUT; mkdir -p $OUT
SHAPES=${SHAPES:-1000,200,65536,200}
for v in default $VARIANTS; do
  if [ $v = default ]; then L=leopard_amd/lib/libleopard_amd.so; else L=leopard_amd/exp/$v/libleopard_amd.so; fi
  LEOPARD_AMD_LIB=$L timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $OUT/$v -o t -- python3 tools/shape_time.py $SHAPES > $OUT/$v.log 2>&1 || { echo "trace $v failed"; tail -5 $OUT/$v.log; exit 1; }
  echo "== $v" >> $OUT/summary.txt
  python3 tools/trace_summary.py $(find $OUT/$v -name "*kernel_trace.csv") | grep -v "^gpurun\|^/" >> $OUT/summary.txt
  rm -rf $OUT/$v
done
cat $OUT/summary.txt
