#!/bin/bash
# GPU box: host-memory e2e rate (tools/hoste2e.py) over host copy threads x ring slot sizes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for pm in ${MODES:-0}; do for th in ${THREADS:-4 8 16}; do for mb in ${SLOTS:-8 32 128}; do
  LEO_AMD_PIPE_MODE=$pm LEO_AMD_HOST_THREADS=$th LEO_AMD_SLOT_MB=$mb timeout -k 10 120 python3 tools/hoste2e.py ${SHAPE:-128 128 65536} > gpurun_out/hm.json 2>/dev/null || { echo "fail $th $mb"; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/hm.json')); print('mode=$pm threads=$th slot_mb=$mb pageable', d['value'], d['encode_GBps'], d['decode_GBps'], 'registered', d['registered']['value'])"
done; done; done
