# cfg2 diagnostics: per-wave stamps, compute-only / memory-only / store-to-one-block modes, lanes per packet
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 120 python tools/stamps.py --workload cfg2 --plan 0 > gpurun_out/diag_stamps.log 2>&1 || exit $?
tail -n 30 gpurun_out/diag_stamps.log
for v in "base:" "m1:--debug-mode 1 --no-verify" "m2:--debug-mode 2 --no-verify" "m8:--debug-mode 8 --no-verify" "l2:--lanes 2" "p0:--plan 0" "wg2:--wg-per-cu 2 --plan 0"; do
  n=${v%%:*}; f=${v#*:}
  timeout -k 10 120 python bench.py --workload cfg2 --steps 20 --warmup 3 --cpu-seconds 0 --no-cold $f > gpurun_out/diag_$n.log 2>&1 || exit $?
  echo "$n $(grep '^{' gpurun_out/diag_$n.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["seal_ms"], d["open_ms"], d["config"]["kernel"][:50])')"
done
