#!/bin/bash
# GPU box: launch floor of the GF(2^8) kernels -- the product library vs an
# LAMD_ABLATE=16 build whose kernels return at once (same arguments, grid and
# LDS), timed behind a spin kernel (bbench: GPU time only) and back to back
# without one (kbench: bounded by the host enqueue cost).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for lib in lib exp/abl16; do
  echo "== $lib"
  BB_NOCHECK=1 LEOPARD_AMD_LIB=leopard_amd/$lib/libleopard_amd.so timeout -k 10 120 python3 tools/bbench.py 128 128 65536 1 4 16 || exit 1
  LEOPARD_AMD_LIB=leopard_amd/$lib/libleopard_amd.so KB_SETS=16 timeout -k 10 120 python3 tools/kbench.py 128 128 65536 || exit 1
done
