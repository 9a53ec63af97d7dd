# round 3: full GPU tier, default bench line, FF16 small-code profile
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03_gpu_tests.log 2>&1 || { tail -30 gpurun_out/r03_gpu_tests.log; exit 1; }
tail -3 gpurun_out/r03_gpu_tests.log
timeout -k 10 300 python bench.py > gpurun_out/r03_bench.json 2> gpurun_out/r03_bench.err || { tail -20 gpurun_out/r03_bench.err; exit 1; }
cat gpurun_out/r03_bench.json
KB_ARGS="1000 200 65536" OUT=gpurun_out/r03_ff16s timeout -k 10 600 bash tools/ff16_prof.sh > gpurun_out/r03_ff16s.log 2>&1 || exit 1
timeout -k 10 120 python tools/hoste2e.py 128 128 65536 > gpurun_out/r03_host.json 2>&1
