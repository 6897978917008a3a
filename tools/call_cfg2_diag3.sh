# cfg2 diagnostics 3: loads before stores (lf1), two waves per SIMD at 2 lanes per packet
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 300 bash tools/ab.sh "base lf1 d4 d4lf" "cfg2" 3 --no-cold || exit $?
for v in "l2w2:--lanes 2 --wg-per-cu 2 --plan 0" "l2w2m1:--lanes 2 --wg-per-cu 2 --plan 0 --debug-mode 1 --no-verify" "l2w2m7:--lanes 2 --wg-per-cu 2 --plan 0 --debug-mode 7 --no-verify" "l4w4:--lanes 4 --wg-per-cu 4 --plan 0"; do
  n=${v%%:*}; f=${v#*:}
  timeout -k 10 120 python bench.py --workload cfg2 --steps 20 --warmup 3 --cpu-seconds 0 --no-cold $f > gpurun_out/diag3_$n.log 2>&1 || exit $?
  echo "$n $(grep '^{' gpurun_out/diag3_$n.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["seal_ms"], d["open_ms"], d["config"]["kernel"][:50])')"
done
export RG_AEAD_LIB=tools/build/librg_d4lf.so
timeout -k 10 120 python tools/stamps.py --workload cfg2 --plan 0 --mode 3 > gpurun_out/diag3_stamps_lf1.log 2>&1 || exit $?
