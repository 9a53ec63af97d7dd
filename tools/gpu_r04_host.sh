#!/bin/bash
# GPU box: PCIe-inclusive host rates (bench host_e2e leg) of the product library
# (direct calls, one slice) and the 4-slice variant (leopard_amd/exp/slices4),
# alternating, at 128+128 and 512+512 x 64 KiB (full-loss decode: K <= R).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/host}
mkdir -p $OUT
for rep in 1 2; do for v in main ${HOST_VARIANTS:-slices4}; do
  lib=leopard_amd/lib/libleopard_amd.so; [ $v = main ] || lib=leopard_amd/exp/$v/libleopard_amd.so
  for shape in "128 128 65536" "512 512 65536"; do
    LEOPARD_AMD_LIB=$lib timeout -k 10 120 python3 tools/hoste2e.py $shape 2>/dev/null > $OUT/$v.tmp || exit 1
    python3 -c "
import json; d=json.load(open('$OUT/$v.tmp'))
print('$v', '$shape', 'step', d['value'], 'enc', d['encode_GBps'], 'dec', d['decode_GBps'], d['roundtrip_ok'], 'registered', d['registered']['value'])"
  done
done; done | tee $OUT/host.txt
