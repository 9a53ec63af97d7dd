# round 3: full GPU tier, then the round profile (bench line, rocprof stats, PMC traffic)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03_gpu_tests.log 2>&1 || { tail -30 gpurun_out/r03_gpu_tests.log; exit 1; }
tail -3 gpurun_out/r03_gpu_tests.log
timeout -k 10 100 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03_smoke.log 2>&1 || { tail gpurun_out/r03_smoke.log; exit 1; }
OUT=gpurun_out/${ROUND_OUT:-r03_v1} timeout -k 10 600 bash tools/gpu_round.sh
