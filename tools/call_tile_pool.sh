# tile kernel global tail pool: GPU tests, A/B on cfg4/cfg5, stamps
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pool_pytest.log 2>&1; rc=$?; tail -n 3 gpurun_out/pool_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 bash tools/ab.sh "base pool0" "cfg4 cfg5" 3 --no-cold || exit $?
timeout -k 10 200 python tools/stamps.py --workload cfg4 > gpurun_out/cfg4_stamps_pool.log 2>&1 || exit $?
python3 - <<'PY'
import numpy as np
for op in ('seal','open'):
    d=np.load(f'gpurun_out/stamps_raw_cfg4_{op}.npy')[:2048]
    rt=d[:,7]/100.0; wg=rt.reshape(256,8)
    print(op,'dur pct', np.percentile(rt,[0,10,50,90,100]).round(1), 'per-CU max pct', np.percentile(wg.max(1),[0,50,100]).round(1))
PY
