#!/bin/bash
# rocprofv3 kernel-trace stats of kbench for several ablation builds.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for n in ${ABL:-0 15 16}; do
  if [ $n = 0 ]; then lib=leopard_amd/lib/libleopard_amd.so; else lib=leopard_amd/ablate/$n/libleopard_amd.so; fi
  LEOPARD_AMD_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pa$n -o p -- python3 tools/kbench.py ${KB_ARGS:-128 128 65536 128 128 1048576} > gpurun_out/pa$n.log 2>&1 || { echo "fail $n"; tail gpurun_out/pa$n.log; exit 1; }
  echo "== ablate=$n"; grep -E "x " gpurun_out/pa$n.log
  f=$(find gpurun_out/pa$n -name "*kernel_stats.csv" | head -1)
  python3 -c "
import csv,sys
for r in csv.DictReader(open('$f')):
    if 'lamd' in r['Name']: print('  %-60s calls=%6s avg_us=%8.2f' % (r['Name'][:60].replace('lamd::(anonymous namespace)::',''), r['Calls'], float(r['AverageNs'])/1e3))
"
done
