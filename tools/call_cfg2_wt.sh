# cfg2: write-through ring stores (wt1) against the default build
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
RG_AEAD_LIB=tools/build/librg_wt1.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "full_config_digest or random_batches or open_failures or reference_framed" --timeout 120 --timeout-method thread > gpurun_out/wt_pytest.log 2>&1; rc=$?; tail -n 3 gpurun_out/wt_pytest.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 bash tools/ab.sh "base wt1" "cfg2" 3 --no-cold || exit $?
export RG_AEAD_LIB=tools/build/librg_wt1.so
timeout -k 10 120 python tools/stamps.py --workload cfg2 --plan 0 --mode 3 > gpurun_out/wt_stamps.log 2>&1 || exit $?
timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmcw_wt1 -o p -- python3 bench.py --workload cfg2 --steps 5 --warmup 2 --cpu-seconds 0 --no-cold > gpurun_out/pmcw_wt1.log 2>&1 || exit $?
