# round 3: full GPU suite on the build, then FF8 batch + FF16 shapes A/B against leopard_amd/exp/base
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03_late_tests.log 2>&1 || { tail -30 gpurun_out/r03_late_tests.log; exit 1; }
tail -2 gpurun_out/r03_late_tests.log
VARIANTS="base" OUT=gpurun_out/r03_late_bb.log REPS="1 2" BB_ARGS="128 128 65536 16" bash tools/gpu_ab_libs.sh | grep -v amdgpu.ids
SHAPES="1000,200,65536,200 32768,32768,65536,32768" VARIANTS="base" OUT=gpurun_out/r03_late_ab.log REPS="1" bash tools/gpu_ab_shapes.sh > /dev/null && python3 tools/ab_table.py gpurun_out/r03_late_ab.log
for v in default base; do
  if [ $v = default ]; then L=leopard_amd/lib/libleopard_amd.so; else L=leopard_amd/exp/$v/libleopard_amd.so; fi
  echo "== $v"; LEOPARD_AMD_LIB=$L KB_N=200 KB_WARM=200 timeout -k 10 120 python3 tools/kbench.py 128 128 65536 2>&1 | grep -v amdgpu.ids
done
