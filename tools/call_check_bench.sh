# quick check of the bench line fields (wire rate, copy ceiling) and smoke
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
tail -n 1 gpurun_out/smoke.log
timeout -k 10 200 python bench.py --steps 20 --warmup 3 --cpu-seconds 0 > gpurun_out/chk_cfg2.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --workload cfg5 --steps 5 --warmup 2 --cpu-seconds 0 > gpurun_out/chk_cfg5.log 2>&1 || exit $?
for f in gpurun_out/chk_cfg2.log gpurun_out/chk_cfg5.log; do grep '^{' $f | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["wire_gib_s"], d["roofline"])'; done
