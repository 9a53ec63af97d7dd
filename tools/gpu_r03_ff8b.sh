# round 3: full parity + sweeps, then GF(2^8) general-path A/B against leopard_amd/exp/base
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sweep.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r03_ff8b_tests.log 2>&1 || { tail -30 gpurun_out/r03_ff8b_tests.log; exit 1; }
tail -2 gpurun_out/r03_ff8b_tests.log
SHAPES="128,128,65536,16 100,30,65536,17 200,55,65536,55 128,128,65536,128 60,40,65536,30" VARIANTS="base" OUT=gpurun_out/r03_ff8b_ab.log REPS="1 2" bash tools/gpu_ab_shapes.sh > /dev/null && python3 tools/ab_table.py gpurun_out/r03_ff8b_ab.log
for v in default base; do
  if [ $v = default ]; then L=leopard_amd/lib/libleopard_amd.so; else L=leopard_amd/exp/$v/libleopard_amd.so; fi
  echo "== $v"; LEOPARD_AMD_LIB=$L KB_N=200 KB_WARM=200 timeout -k 10 120 python3 tools/kbench.py 128 128 65536 100 20 65536 2>&1 | grep -v amdgpu.ids
done
