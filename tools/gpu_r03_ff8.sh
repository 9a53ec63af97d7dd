# round 3: FF8 parity subset, then batch-kernel A/B against leopard_amd/exp/base
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sweep.py -x -q --timeout 120 --timeout-method thread -k "encode or decode or batch or sweep or baseline" > gpurun_out/r03_ff8_tests.log 2>&1 || { tail -30 gpurun_out/r03_ff8_tests.log; exit 1; }
tail -2 gpurun_out/r03_ff8_tests.log
VARIANTS="${VARIANTS:-base}" OUT=gpurun_out/r03_ff8_ab.log REPS="1 2" BB_ARGS="128 128 65536 16" bash tools/gpu_ab_libs.sh | grep -v amdgpu.ids
SHAPES="128,128,65536,128 128,128,65536,16" VARIANTS="${VARIANTS:-base}" OUT=gpurun_out/r03_ff8_shapes.log REPS="1" bash tools/gpu_ab_shapes.sh > /dev/null && python3 tools/ab_table.py gpurun_out/r03_ff8_shapes.log
