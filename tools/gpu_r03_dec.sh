# round 3: FF16 decode parity subset, then pass-2 variants A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sweep.py -x -q --timeout 120 --timeout-method thread -k "decode or sweep or baseline or configs4 or host_layouts" > gpurun_out/r03_dec_tests.log 2>&1 || { tail -30 gpurun_out/r03_dec_tests.log; exit 1; }
tail -2 gpurun_out/r03_dec_tests.log
SHAPES="1000,200,65536,200 1000,200,65536,50 600,300,65536,299 2000,1000,16384,1000" VARIANTS="$VARIANTS" OUT=gpurun_out/r03_dec_ab.log bash tools/gpu_ab_shapes.sh | grep -v amdgpu.ids | cut -c1-240
