#!/bin/bash
# GPU box: run one measurement command against several library builds (A/B).
#   LIBS="lib exp/bytes exp/x" CMD="python3 tools/bbench.py 128 128 65536 16" bash tools/gpu_ab.sh
# Each entry is a directory under leopard_amd/ holding libleopard_amd.so (built
# by make, or by tools/build_variant.sh NAME "-DFLAG=..." into exp/NAME);
# ENVS="A=1 B=2" instead runs the product library once per environment setting
# (experiment builds only read their switches, LAMD_EXPERIMENT_ENV=1); "A=1,B=2" sets both in one run.
# Every run has its own time limit; the first failure ends the script.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
CMD=${CMD:?set CMD}
if [ -n "${ENVS:-}" ]; then
  for e in $ENVS; do
    echo "== $e"
    env ${e//,/ } LEOPARD_AMD_LIB=leopard_amd/${LIB:-lib/exp}/libleopard_amd.so timeout -k 10 ${T:-200} $CMD 2>&1 | grep -v amdgpu.ids || exit 1
  done
  exit 0
fi
for v in ${LIBS:-lib}; do
  echo "== $v"
  LEOPARD_AMD_LIB=leopard_amd/$v/libleopard_amd.so timeout -k 10 ${T:-200} $CMD 2>&1 | grep -v amdgpu.ids || exit 1
done
