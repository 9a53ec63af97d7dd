#!/bin/bash
# GPU box: PCIe probe, host-path tests, host_e2e under DMA slice counts, FF16 variants.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
#timeout -k 10 120 tools/bin/pcie_probe > gpurun_out/pcie.txt 2>&1 || { cat gpurun_out/pcie.txt; exit 1; }
#cat gpurun_out/pcie.txt
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "registered or host" > gpurun_out/pytest_host.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_host.log; [ $rc -eq 0 ] || exit $rc
for sl in 1 2 4 8; do
  echo "MAPPED_SLICES=$sl"; LEO_AMD_MAPPED_SLICES=$sl timeout -k 10 120 python3 tools/hoste2e.py || exit 1
done


