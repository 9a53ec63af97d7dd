#!/bin/bash
# GPU box: A/B of the in-tree library against leopard_amd/lib_base (the previous
# build): batched and single-call timings.  usage: tools/ab.sh [K R B]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
ARGS="${*:-128 128 65536}"
for lib in lib_base lib lib_base lib; do
  echo "== $lib"
  LEOPARD_AMD_LIB=leopard_amd/$lib/libleopard_amd.so timeout -k 10 120 python3 tools/bbench.py $ARGS 16 64 || exit 1
  LEOPARD_AMD_LIB=leopard_amd/$lib/libleopard_amd.so timeout -k 10 120 python3 tools/kbench.py $ARGS || exit 1
done
