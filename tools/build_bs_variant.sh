#!/bin/bash
# Build a library variant that differs from the product build only in
# rs_ff8_bs.hip (extra -D flags), reusing the product objects of every other
# file: leopard_amd/exp/<name>/libleopard_amd.so (experiments only).
# usage: tools/build_bs_variant.sh name "-DFOO=1 -DBAR=2"   (after make -C leopard_amd)
set -e
cd "$(dirname "$0")/.."
d=leopard_amd/exp/$1; mkdir -p $d
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -fvisibility=hidden -Iinclude -Ileopard_amd/csrc"
/opt/rocm/bin/hipcc $F -mllvm -amdgpu-sched-strategy=max-ilp -mllvm -amdgpu-atomic-optimizer-strategy=None $2 -c ${SRC:-leopard_amd/csrc/rs_ff8_bs.hip} -o $d/rs_ff8_bs.o
objs="leopard_amd/build/gf_tables.o leopard_amd/build/leopard_amd.o leopard_amd/build/rs_kernels.o leopard_amd/build/rs_ff8.o leopard_amd/build/rs_ff16_small.o leopard_amd/build/rs_ff8_mat.o"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $d/libleopard_amd.so $objs $d/rs_ff8_bs.o
rm -f $d/rs_ff8_bs.o
