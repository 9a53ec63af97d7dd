# round 3: FF16 decode parity subset, A/B against leopard_amd/exp/base, stamps
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sweep.py tests/test_gpu_lifecycle.py -x -q --timeout 120 --timeout-method thread -k "decode or sweep or baseline or configs4 or host_layouts or scratch or fanout" > gpurun_out/r03_dec_tests.log 2>&1 || { tail -30 gpurun_out/r03_dec_tests.log; exit 1; }
tail -2 gpurun_out/r03_dec_tests.log
SHAPES="1000,200,65536,200 1000,200,65536,50 600,300,65536,299 2000,1000,16384,1000" VARIANTS="base" OUT=gpurun_out/r03_dec_ab.log REPS="1 2" bash tools/gpu_ab_shapes.sh > /dev/null && python3 tools/ab_table.py gpurun_out/r03_dec_ab.log
LEOPARD_AMD_LIB=leopard_amd/exp/stamps/libleopard_amd.so timeout -k 10 120 python3 tools/stamps16d.py 1000 200 65536 200 2>&1 | grep -v amdgpu.ids
