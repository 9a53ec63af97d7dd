# round 3: GF(2^16) parity (every FF16 path), then A/B against leopard_amd/exp/base
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sweep.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r03_ff16_tests.log 2>&1 || { tail -30 gpurun_out/r03_ff16_tests.log; exit 1; }
tail -2 gpurun_out/r03_ff16_tests.log
SHAPES="1000,200,65536,200 600,300,65536,299 2000,2000,65536,2000 32768,32768,65536,32768 32768,2048,65536,2048" VARIANTS="base" OUT=gpurun_out/r03_ff16_ab.log REPS="1 2" bash tools/gpu_ab_shapes.sh > /dev/null && python3 tools/ab_table.py gpurun_out/r03_ff16_ab.log
