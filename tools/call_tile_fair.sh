# tile kernel fair SIMD issue (s_setprio by progress): tile-path GPU tests, A/B on cfg4/cfg5, stamps
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/fair_pytest.log 2>&1; rc=$?; tail -n 3 gpurun_out/fair_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 bash tools/ab.sh "base fair0 dyn0" "cfg4 cfg5" 2 --no-cold || exit $?
timeout -k 10 200 python tools/stamps.py --workload cfg4 > gpurun_out/cfg4_stamps_fair.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/cfg4_stamps_fair.log | python3 -c "
import sys,json; d=json.loads(sys.stdin.read())
for k,v in d.items(): print(k, v['wave_us_pct_0_10_50_90_99_100'], v['shader_clock_ghz'], v['share'])"
