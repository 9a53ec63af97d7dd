#!/bin/bash
# GPU box: order-only events (no system-scope fence) against the previous
# default events (leopard_amd/exp/evsys) and the round-2 build: per-call times
# of back-to-back decodes and the headline bench line (batch launches).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/ev}
mkdir -p $OUT
OUT=$OUT REPS=2 VARIANTS="evsys r02" SHAPES="128,128,65536,16 100,10,2560,10 100,20,2560,20 1000,200,65536,200 1000,200,2560,200" \
    bash tools/gpu_r04_ab.sh || exit 1
for v in main evsys; do
  lib=leopard_amd/lib/libleopard_amd.so; [ $v = main ] || lib=leopard_amd/exp/$v/libleopard_amd.so
  LEOPARD_AMD_LIB=$lib timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-host --no-secondary > $OUT/bench_$v.json 2> $OUT/bench_$v.err \
      || { tail -20 $OUT/bench_$v.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$OUT/bench_$v.json')); r=d['roofline']
print('$v', 'value', d['value'], 'launch_us', r['launch_us'], 'enc', r['batch_encode_us'], 'single', r['single_call_us'], 'frac', r['frac'], [ (k, m['value']) for k,m in d['modes'].items()])"
done
