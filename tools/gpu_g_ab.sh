# FF8 single-call encoder lane-group forms (LEO_AMD_FF8_G) at 128+128 x 64 KiB
set -o pipefail
cd $GRAFT_REPO_ROOT
for g in 0 1 2; do
  echo "== G=$g"
  LEO_AMD_FF8_G=$g timeout -k 10 120 python3 tools/shape_time.py 128,128,65536,128 128,128,65536,16 2>&1 | grep -v amdgpu.ids | python3 -c "
import sys,json
for l in sys.stdin:
    if l.startswith('{'): d=json.loads(l); print(d['workload'][:40], 'enc', d['encode_us'], 'dec', d['decode_us'])"
  LEO_AMD_FF8_G=$g KB_N=200 KB_WARM=200 timeout -k 10 120 python3 tools/kbench.py 128 128 65536 2>&1 | grep -v amdgpu.ids
done
