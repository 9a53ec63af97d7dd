#!/bin/bash
# Build a library variant with extra -D flags into leopard_amd/exp/<name>/ (experiments only).
# usage: tools/build_variant.sh name "-DFOO=1 -DBAR=2"
cd "$(dirname "$0")/.."
d=leopard_amd/exp/$1; mkdir -p $d
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -fvisibility=hidden $2 -Iinclude -Ileopard_amd/csrc \
   -shared -o $d/libleopard_amd.so leopard_amd/csrc/*.cpp leopard_amd/csrc/*.hip
