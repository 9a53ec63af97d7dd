#!/bin/bash
# Build ablated libraries (performance experiments only) into leopard_amd/ablate/N/.
cd "$(dirname "$0")/.."
for n in "$@"; do
  d=leopard_amd/ablate/$n; mkdir -p $d
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -fvisibility=hidden -DLAMD_ABLATE=$n -Iinclude -Ileopard_amd/csrc \
     -shared -o $d/libleopard_amd.so leopard_amd/csrc/gf_tables.cpp leopard_amd/csrc/leopard_amd.cpp leopard_amd/csrc/rs_kernels.hip leopard_amd/csrc/rs_ff8.hip &
done
wait
