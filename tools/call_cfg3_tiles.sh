# cfg3 on the tile kernel (dynamic deal) against the automatic choice (flattened)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
for v in "auto:" "t2:--staged 2" "t1:--staged 1" "t2s1:--staged 2 --segments 1" "t2s2:--staged 2 --segments 2" "pipe:--staged 0"; do
  n=${v%%:*}; f=${v#*:}
  timeout -k 10 120 python bench.py --workload cfg3 --steps 20 --warmup 3 --cpu-seconds 0 --no-cold --forged 0 $f > gpurun_out/c3t_$n.log 2>&1 || exit $?
  echo "$n $(grep '^{' gpurun_out/c3t_$n.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["seal_ms"], d["open_ms"], d["config"]["kernel"][:60])')"
done
