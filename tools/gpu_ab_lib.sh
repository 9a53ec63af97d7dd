#!/bin/bash
# GPU box: bbench (16-object batches) and kbench (single calls) of 128+128 x 64 KiB for the
# product library and each variant under leopard_amd/exp/, alternating, twice.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for rep in 1 2; do for v in main ${VARIANTS:-$(ls leopard_amd/exp)}; do
  lib=leopard_amd/lib/libleopard_amd.so; [ $v = main ] || lib=leopard_amd/exp/$v/libleopard_amd.so
  echo "== $v"
  LEOPARD_AMD_LIB=$lib timeout -k 10 120 python3 tools/bbench.py ${SHAPE:-128 128 65536} 16 2>&1 | grep -v amdgpu.ids || exit 1
  LEOPARD_AMD_LIB=$lib timeout -k 10 120 python3 tools/kbench.py ${SHAPE:-128 128 65536} 2>&1 | grep -v amdgpu.ids || exit 1
done; done
