set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
W=${W:-cfg2}
for v in ${VARIANTS:-"n:" "m1:--debug-mode_1" "m2:--debug-mode_2"}; do
  name=${v%%:*}; flags=${v#*:}; flags=${flags//_/ }
  timeout -k 10 200 python bench.py --workload $W --staged 4 $flags --steps 20 --warmup 3 --cpu-seconds 0 --no-verify > gpurun_out/diag_${W}_$name.log 2>&1 || exit 3
  python3 -c "import json,sys; d=json.loads([l for l in open('gpurun_out/diag_${W}_$name.log') if l.startswith('{')][-1]); print('$W $name', d['seal_ms'], d['open_ms'])"
done
[ -n "${NOSTAMPS:-}" ] && exit 0
timeout -k 10 200 python tools/stamps.py --workload $W --staged 4 > gpurun_out/diag_stamps_$W.log 2>&1 || exit 3
grep -v amdgpu.ids gpurun_out/diag_stamps_$W.log
