#!/bin/bash
# GPU box: kbench (KB_ARGS) for the product library and every variant under leopard_amd/exp/ (or VARIANTS).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export KB_WARM=${KB_WARM:-3} KB_N=${KB_N:-20}
echo "== main"; timeout -k 10 200 python3 tools/kbench.py $KB_ARGS || exit 1
for v in ${VARIANTS:-$(ls leopard_amd/exp)}; do
  echo "== $v"; LEOPARD_AMD_LIB=leopard_amd/exp/$v/libleopard_amd.so timeout -k 10 200 python3 tools/kbench.py $KB_ARGS || exit 1
done
