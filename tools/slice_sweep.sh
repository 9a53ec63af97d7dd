#!/bin/bash
# GPU box: FF16 32768+32768 x 64 KiB encode/decode time vs the multi-pass column slice (LEO_AMD_SLICE_MB).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for mb in ${SLICES:-96 192 384 1024 3072 8192}; do
  echo -n "SLICE_MB=$mb  "
  LEO_AMD_SLICE_MB=$mb KB_SETS=2 KB_N=${KB_N:-5} KB_WARM=2 timeout -k 10 120 python3 tools/kbench.py ${KB_ARGS:-32768 32768 65536} || exit 1
done
