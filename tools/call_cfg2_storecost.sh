# cfg2 store cost: default vs mode 8 (line stores to two cache-resident lines per frame) vs mode 7 (no payload stores), with stamps
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
for v in "base:" "m8:--debug-mode 8 --no-verify" "m7:--debug-mode 7 --no-verify"; do
  n=${v%%:*}; f=${v#*:}
  timeout -k 10 120 python bench.py --workload cfg2 --steps 20 --warmup 3 --cpu-seconds 0 --no-cold --plan 0 $f > gpurun_out/sc_$n.log 2>&1 || exit $?
  echo "$n $(grep '^{' gpurun_out/sc_$n.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["seal_ms"], d["open_ms"])')"
done
timeout -k 10 120 python tools/stamps.py --workload cfg2 --plan 0 --mode 8 > gpurun_out/sc_stamps_m8.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/sc_stamps_m8.log | python3 -c "
import sys,json; d=json.loads(sys.stdin.read())
for k,v in d.items(): print(k, round(v['cycles_per_wave_mean']), v['wave_us_pct_0_10_50_90_100'], v['shader_clock_ghz'], v['end_us_pct_0_50_90_100'])"
