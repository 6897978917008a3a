# cfg3: flattened kernel phase stamps with wall-clock start/end, and the bench line
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 120 python tools/flat_stamps.py --workload cfg3 > gpurun_out/flat_stamps.log 2>&1 || exit $?
cat gpurun_out/flat_stamps.log | grep -v amdgpu.ids
timeout -k 10 120 python bench.py --workload cfg3 --steps 20 --warmup 3 --cpu-seconds 0 --no-cold > gpurun_out/cfg3_bench.log 2>&1 || exit $?
grep '^{' gpurun_out/cfg3_bench.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["seal_ms"], d["open_ms"])'
