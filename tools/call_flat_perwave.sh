set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 120 python tools/flat_stamps.py --workload cfg3 --per-wave > gpurun_out/flat_perwave.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/flat_perwave.log | tail -n 3 | cut -c1-1500
