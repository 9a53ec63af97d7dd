#!/bin/bash
# GPU box: parity subset and timing of the FF8 encoder lane-group forms (LEO_AMD_FF8_G = 0, 1, 2).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for G in ${GS:-2 1}; do
  LEO_AMD_FF8_G=$G timeout -k 10 300 python -m pytest tests -x -q -m gpu -k "not baseline" > gpurun_out/pt_g$G.log 2>&1 || { echo "G=$G tests failed"; tail -30 gpurun_out/pt_g$G.log; exit 1; }
  echo "G=$G: $(tail -1 gpurun_out/pt_g$G.log)"
done
for G in 0 1 2; do
  echo "== G=$G"
  LEO_AMD_FF8_G=$G timeout -k 10 120 python3 tools/kbench.py 128 128 65536 128 128 64000 100 20 65536 || exit 1
  LEO_AMD_FF8_G=$G timeout -k 10 120 python3 tools/conc.py 128 128 65536 1 2 3 || exit 1
done
