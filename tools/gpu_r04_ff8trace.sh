#!/bin/bash
# GPU box: rocprofv3 kernel traces of the GF(2^8) partial-loss decode shapes,
# product library against the round-2 build (leopard_amd/exp/r02): which
# kernels each call launches and how long each runs.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/ff8trace}
mkdir -p $OUT
for v in main r02; do
  lib=leopard_amd/lib/libleopard_amd.so; [ $v = main ] || lib=leopard_amd/exp/$v/libleopard_amd.so
  LEOPARD_AMD_LIB=$lib timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$v -o kt -- \
      python3 tools/shape_time.py 100,10,2560,10 128,128,65536,16 > $OUT/$v.log 2>&1 || { tail -20 $OUT/$v.log; exit 1; }
  f=$(find $OUT/$v -name '*kernel_stats.csv' | head -1)
  echo "== $v"; python3 -c "
import csv,sys
for r in csv.DictReader(open('$f')):
    print(f\"{r['Name'][:60]:60} calls {r['Calls']:>6} avg_us {float(r['AverageNs'])/1e3:8.2f}\")" | tee $OUT/$v.stats.txt
  find $OUT/$v -name '*kernel_trace.csv' -exec cp {} $OUT/$v.kernel_trace.csv \;
  rm -rf $OUT/$v
done
