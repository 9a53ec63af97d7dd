# round 3: host-memory paths (direct SDMA rows, gather ring) parity + rates
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_lifecycle.py -x -q --timeout 120 --timeout-method thread -k "host or fanout or registered or concurrent" > gpurun_out/r03_host_tests.log 2>&1 || { tail -30 gpurun_out/r03_host_tests.log; exit 1; }
tail -2 gpurun_out/r03_host_tests.log
for shape in "128 128 65536" "128 128 1048576" "512 512 65536"; do
  timeout -k 10 120 python tools/hoste2e.py $shape >> gpurun_out/r03_host.json 2>&1 || exit 1
done
cat gpurun_out/r03_host.json
