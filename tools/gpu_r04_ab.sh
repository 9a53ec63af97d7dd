#!/bin/bash
# GPU box: per-call encode / decode times (bench.run_shape, HIP events behind a
# spin kernel) of SHAPES for the product library and each variant in VARIANTS
# (leopard_amd/exp/<name>), alternating, REPS times.  Optional: the GPU suite first.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/ab}
mkdir -p $OUT
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 ${TEST_LIMIT:-420} python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread $TESTS \
      > $OUT/pytest_gpu.txt 2>&1 || { tail -40 $OUT/pytest_gpu.txt; exit 1; }
  tail -2 $OUT/pytest_gpu.txt
fi
for rep in $(seq ${REPS:-2}); do for v in main ${VARIANTS:-}; do
  lib=leopard_amd/lib/libleopard_amd.so; [ $v = main ] || lib=leopard_amd/exp/$v/libleopard_amd.so
  LEOPARD_AMD_LIB=$lib timeout -k 10 180 python3 tools/shape_time.py $SHAPES > $OUT/$v.$rep.jsonl 2> $OUT/$v.$rep.err \
      || { tail -20 $OUT/$v.$rep.err; exit 1; }
  python3 - $v $OUT/$v.$rep.jsonl <<'PY'
import json, sys
for line in open(sys.argv[2]):
    d = json.loads(line)
    print(f"{sys.argv[1]:>10} {d['workload'][:44]:44} enc {d['encode_us']:8.2f} dec {d['decode_us']:8.2f} ok {d['roundtrip_ok']}")
PY
done; done
