#!/bin/bash
# GPU box, round 4: the one-pass GF(2^16) decoder variants (leopard_amd/exp/one,
# one_ne) — decode parity through them, per-call A/B against the product
# library's two-pass decoder, and phase stamps of the LAMD_STAMPS builds.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/onepass}
mkdir -p $OUT
LEOPARD_AMD_LIB=leopard_amd/exp/one/libleopard_amd.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py \
    tests/test_gpu_sweep.py -m gpu -x -q --timeout 120 --timeout-method thread -k "decode or batch or sweep or random or exhaustive" \
    > $OUT/pytest_one.txt 2>&1 || { tail -40 $OUT/pytest_one.txt; exit 1; }
tail -2 $OUT/pytest_one.txt
OUT=$OUT REPS=2 VARIANTS="${VARIANTS:-one}" SHAPES="1000,200,65536,200 1000,200,16384,200 2000,48,65536,48 600,400,65536,400" \
    bash tools/gpu_r04_ab.sh || exit 1
for v in ${STAMPS:-stamps}; do
  LEOPARD_AMD_LIB=leopard_amd/exp/$v/libleopard_amd.so timeout -k 10 120 python3 tools/stamps16one.py 1000 200 65536 200 \
      > $OUT/$v.txt 2> $OUT/$v.err || { tail -20 $OUT/$v.err; exit 1; }
  echo "== $v"; tail -12 $OUT/$v.txt
done
