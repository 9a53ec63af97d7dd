cd "${GRAFT_REPO_ROOT}"; export TMPDIR=/tmp KB_WARM=2 KB_N=5
mkdir -p gpurun_out/ic
timeout -s KILL 90 rocprofv3 --pmc SQ_IFETCH SQ_IFETCH_LEVEL SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d gpurun_out/ic/p1 -o p -- python3 tools/kbench.py 32768 32768 65536 > gpurun_out/ic/p1.log 2>&1 || { tail -5 gpurun_out/ic/p1.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQC_ICACHE_REQ --output-format csv -d gpurun_out/ic/p2 -o p -- python3 tools/kbench.py 32768 32768 65536 > gpurun_out/ic/p2.log 2>&1 || { tail -5 gpurun_out/ic/p2.log; exit 1; }
python3 tools/pmc_summary.py gpurun_out/ic/p1 gpurun_out/ic/p2 > gpurun_out/ic/summary.txt; rm -rf gpurun_out/ic/p1 gpurun_out/ic/p2; cat gpurun_out/ic/summary.txt
