#!/bin/bash
# GPU box: tools/shape_time.py at SHAPES on the shipped library and on each
# experiment library leopard_amd/exp/<name> in VARIANTS; OUT log file.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${OUT:-gpurun_out/ab_shapes.log}; : > $OUT
SHAPES=${SHAPES:-1000,200,65536,200}
for rep in ${REPS:-1 2}; do
for v in default $VARIANTS; do
  if [ $v = default ]; then L=leopard_amd/lib/libleopard_amd.so; else L=leopard_amd/exp/$v/libleopard_amd.so; fi
  echo "== $v" >> $OUT
  LEOPARD_AMD_LIB=$L timeout -k 10 100 python3 tools/shape_time.py $SHAPES >> $OUT 2>&1 || exit 1
done
done
cat $OUT
