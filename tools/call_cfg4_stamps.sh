# cfg4: tile kernel section stamps
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 200 python tools/stamps.py --workload cfg4 > gpurun_out/cfg4_stamps.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/cfg4_stamps.log
