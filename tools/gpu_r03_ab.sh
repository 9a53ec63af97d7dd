set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "decode or encode or batch" > gpurun_out/r03_dec.log 2>&1
timeout -k 10 100 python tools/shape_time.py 1000,200,65536,200 1000,200,64000,200 1000,100,65536,100 600,300,65536,299 2000,1000,16384,1000 > gpurun_out/r03_shapes.log 2>&1
for v in default p0 p16; do
  if [ $v = default ]; then L=leopard_amd/lib/libleopard_amd.so; else L=leopard_amd/exp/$v/libleopard_amd.so; fi
  echo "== $v" >> gpurun_out/r03_ff8p.log
  LEOPARD_AMD_LIB=$L timeout -k 10 100 python tools/bbench.py 128 128 65536 16 64 >> gpurun_out/r03_ff8p.log 2>&1 || exit 1
done
LEOPARD_AMD_LIB=leopard_amd/exp/p0/libleopard_amd.so LEO_AMD_FF8_PERSIST=0 timeout -k 10 100 python tools/bbench.py 128 128 65536 16 64 > gpurun_out/r03_ff8p_off.log 2>&1
