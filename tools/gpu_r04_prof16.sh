#!/bin/bash
# GPU box: the GF(2^16) small decoder at 1000+200 x 64 KiB -- per-call times
# (main = one-pass, twopass variant), phase stamps of the one-pass kernel, and
# PMC passes (issue / wait / LDS counters, HBM traffic).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/prof16}
mkdir -p $OUT
SH=${SH:-1000,200,65536,200}
for v in main twopass main twopass; do
  lib=leopard_amd/lib/libleopard_amd.so; [ $v = main ] || lib=leopard_amd/exp/$v/libleopard_amd.so
  LEOPARD_AMD_LIB=$lib timeout -k 10 120 python3 tools/shape_time.py $SH 2>/dev/null | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print('$v', d['workload'][:40], 'enc', d['encode_us'], 'dec', d['decode_us'], d['roundtrip_ok'])" || exit 1
done | tee $OUT/times.txt
LEOPARD_AMD_LIB=leopard_amd/exp/stamps/libleopard_amd.so timeout -k 10 120 python3 tools/stamps16one.py ${SH//,/ } 2>&1 | grep -v amdgpu.ids | tee $OUT/stamps.txt || exit 1
rm -rf gpurun_out/pmc1 gpurun_out/pmc2 gpurun_out/pmc3 gpurun_out/pmc4
PMC_TOOL=shape_time KB_ARGS="$SH" bash tools/pmc.sh \
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE" \
  "SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM SQ_LDS_IDX_ACTIVE" \
  FETCH_SIZE WRITE_SIZE || exit 1
python3 tools/pmc_summary.py gpurun_out/pmc1 gpurun_out/pmc2 gpurun_out/pmc3 gpurun_out/pmc4 > $OUT/pmc_summary.txt
python3 tools/pmc_derive.py $OUT/pmc_summary.txt | tee $OUT/pmc_derived.txt
python3 tools/pmc_traffic.py $(echo $SH | cut -d, -f1-3 | tr , " ") gpurun_out/pmc3 gpurun_out/pmc4 > $OUT/pmc_traffic_${SH%%,*}x$(echo $SH | cut -d, -f2).json
cat $OUT/pmc_traffic_*.json
rm -rf gpurun_out/pmc1 gpurun_out/pmc2 gpurun_out/pmc3 gpurun_out/pmc4  # raw passes: summarised above
