#!/bin/bash
# GPU box: headline-only bench line (modes) for the product library and each variant under leopard_amd/exp/.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in main ${VARIANTS:-$(ls leopard_amd/exp)}; do
  lib=leopard_amd/lib/libleopard_amd.so; [ $v = main ] || lib=leopard_amd/exp/$v/libleopard_amd.so
  LEOPARD_AMD_LIB=$lib timeout -k 10 200 python3 bench.py --steps ${STEPS:-100} --warmup 10 --no-sharded --no-secondary --no-host --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/bv_$v.json 2> gpurun_out/bv_$v.err || { echo "fail $v"; tail -5 gpurun_out/bv_$v.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('gpurun_out/bv_$v.json')); print('$v', {k: v['value'] for k, v in d['modes'].items()}, 'enc_us', d['encode_us'], 'dec_us', d['decode_us'])"
done
