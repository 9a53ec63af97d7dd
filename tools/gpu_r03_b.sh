# round 3: decode parity, FF16 small-code profile, host-memory rates
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_lifecycle.py -x -q --timeout 120 --timeout-method thread -k "decode or fanout or scratch or release" > gpurun_out/r03_dec.log 2>&1 || exit 1
KB_ARGS="1000 200 65536" OUT=gpurun_out/r03_ff16s timeout -k 10 600 bash tools/ff16_prof.sh > gpurun_out/r03_ff16s.log 2>&1 || exit 1
timeout -k 10 120 python tools/hoste2e.py 128 128 65536 > gpurun_out/r03_host.json 2>&1
