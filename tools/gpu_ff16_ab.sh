#!/bin/bash
# GPU box: FF16 encode/decode timings (tools/dec_ab.py shapes) for the product library and each
# variant under leopard_amd/exp/, alternating, twice.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for rep in 1 2; do for v in main ${VARIANTS:-$(ls leopard_amd/exp)}; do
  lib=leopard_amd/lib/libleopard_amd.so; [ $v = main ] || lib=leopard_amd/exp/$v/libleopard_amd.so
  LEOPARD_AMD_LIB=$lib AB_N=${AB_N:-10} timeout -k 10 200 python3 tools/dec_ab.py ${AB_SHAPES:-1000 200 65536 200 32768 32768 65536 32768} 2>&1 | grep workload | python3 -c "
import json, sys
for l in sys.stdin:
    d = json.loads(l); print('$v', d['workload'][:40], 'enc', d['encode_us'], 'dec', d['decode_us'])" || exit 1
done; done
