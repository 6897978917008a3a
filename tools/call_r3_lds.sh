# round 3: LDS counters of the transport kernels (config 2 pipelined ring, config 3 flattened, config 4 tiles):
# bank-conflict and unaligned-stall cycles against all LDS-array cycles; one pass per workload
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/lds; export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
for W in ${WS:-cfg2 cfg3 cfg4}; do
  timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_UNALIGNED_STALL SQ_LDS_ADDR_CONFLICT \
      SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_WAVES --kernel-trace --output-format csv -d gpurun_out/lds/${TAG:-base}_$W -o p -- \
      python3 bench.py --workload $W --steps 5 --warmup 2 --cpu-seconds 0 --no-cold --forged 0 --no-graph > gpurun_out/lds/${TAG:-base}_$W.log 2>&1 || exit 1
done
python3 tools/pmc_summary.py gpurun_out/lds/* > gpurun_out/lds_summary.txt 2>&1 || true
