#!/bin/bash
# PMC counters for the kernels of one kbench run (separate passes, no tracing domains);
# PMC_TOOL=bbench runs tools/bbench.py instead (KB_ARGS = "K R B OBJECTS": batched launches).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
ARGS=${KB_ARGS:-128 128 65536}
i=0
for set in "${@}"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set --output-format csv -d gpurun_out/pmc$i -o p -- python3 tools/${PMC_TOOL:-kbench}.py $ARGS > gpurun_out/pmc$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 gpurun_out/pmc$i.log; exit 1; }
done
echo done
