#!/bin/bash
# GPU box: tools/bbench.py (batch launches) on the shipped library and on each
# experiment library leopard_amd/exp/<name> given in VARIANTS; OUT log file.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${OUT:-gpurun_out/ab.log}; : > $OUT
ARGS=${BB_ARGS:-128 128 65536 16}
for rep in ${REPS:-1 2}; do
for v in default $VARIANTS; do
  if [ $v = default ]; then L=leopard_amd/lib/libleopard_amd.so; else L=leopard_amd/exp/$v/libleopard_amd.so; fi
  echo "== $v" >> $OUT
  LEOPARD_AMD_LIB=$L timeout -k 10 100 python3 tools/bbench.py $ARGS >> $OUT 2>&1 || exit 1
done
done
cat $OUT
