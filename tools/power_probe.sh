#!/bin/bash
# GPU box: shader clock (in-kernel s_memtime / s_memrealtime) and board power
# (amd-smi / rocm-smi, read-only) while the bit-sliced slab kernel runs back to
# back (tools/bs_clock.py on the LAMD_CLOCK build).
#   bash tools/power_probe.sh [OBJ]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
BS_CLOCK_S=${BS_CLOCK_S:-6} BS_CLOCK_SMI=1 LEOPARD_AMD_LIB=${LIB:-leopard_amd/exp/clock/libleopard_amd.so} \
  timeout -k 10 150 python3 tools/bs_clock.py ${1:-64} 2>&1 | grep -v amdgpu.ids
