# flat kernel next-packet prefetch: flat GPU tests, A/B on cfg3, stamps
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -k "flat or auto or digest or malformed or keepalive" --timeout 120 --timeout-method thread > gpurun_out/npf_pytest.log 2>&1; rc=$?; tail -n 3 gpurun_out/npf_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 bash tools/ab.sh "base npf0" "cfg3" 4 --no-cold || exit $?
timeout -k 10 120 python tools/flat_stamps.py --workload cfg3 > gpurun_out/flat_stamps_npf.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/flat_stamps_npf.log | cut -c1-420
