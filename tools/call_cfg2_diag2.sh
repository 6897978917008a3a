# cfg2 diagnostics 2: compute-only / no-store modes at 1 and 2 lanes per packet, stamps at 2 lanes
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
for v in "base:--plan 0" "m1:--debug-mode 1 --no-verify --plan 0" "m7:--debug-mode 7 --no-verify --plan 0" "l2:--lanes 2 --plan 0" "l2m1:--lanes 2 --debug-mode 1 --no-verify --plan 0" "l2m7:--lanes 2 --debug-mode 7 --no-verify --plan 0" "l4m1:--lanes 4 --debug-mode 1 --no-verify --plan 0"; do
  n=${v%%:*}; f=${v#*:}
  timeout -k 10 120 python bench.py --workload cfg2 --steps 20 --warmup 3 --cpu-seconds 0 --no-cold $f > gpurun_out/diag2_$n.log 2>&1 || exit $?
  echo "$n $(grep '^{' gpurun_out/diag2_$n.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["seal_ms"], d["open_ms"], d["config"]["kernel"][:50])')"
done
for m in 1 7 0; do
timeout -k 10 120 python tools/stamps.py --workload cfg2 --plan 0 --lanes 2 --mode $m > gpurun_out/diag2_stamps_l2_m$m.log 2>&1 || exit $?
done
timeout -k 10 120 python tools/stamps.py --workload cfg2 --plan 0 --mode 1 > gpurun_out/diag2_stamps_l1_m1.log 2>&1 || exit $?
timeout -k 10 120 python tools/stamps.py --workload cfg2 --plan 0 --mode 7 > gpurun_out/diag2_stamps_l1_m7.log 2>&1 || exit $?
