set -o pipefail
mkdir -p gpurun_out
if [ -z "${NO_TESTS:-}" ]; then
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "decode or batch" > gpurun_out/pt_dec.log 2>&1 || { tail -30 gpurun_out/pt_dec.log; exit 1; }
tail -2 gpurun_out/pt_dec.log
fi
timeout -k 10 120 python3 tools/dec_ab.py ${AB_SHAPES:-128 128 65536 16 100 70 65536 30 128 128 65536 128 1000 200 65536 200} 2>&1 | grep -v amdgpu.ids
[ -n "${AB_ENV:-}" ] && env $AB_ENV timeout -k 10 120 python3 tools/dec_ab.py ${AB_SHAPES:-128 128 65536 16 100 70 65536 30} 2>&1 | grep -v amdgpu.ids
true
