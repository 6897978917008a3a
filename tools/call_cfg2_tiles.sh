# cfg2 on the LDS-staged tile kernel: windows 1/2 x segments 1/2/4, against the automatic choice
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
for v in "auto:" "t1s1:--staged 1 --segments 1" "t1s2:--staged 1 --segments 2" "t2s1:--staged 2 --segments 1" "t2s2:--staged 2 --segments 2" "t2s4:--staged 2 --segments 4" "t1s4:--staged 1 --segments 4" "c4auto:--workload cfg4" "c4t2s2:--workload cfg4 --staged 2 --segments 2"; do
  n=${v%%:*}; f=${v#*:}
  w=cfg2; case "$f" in *cfg4*) w=cfg4; f=${f/--workload cfg4/};; esac
  timeout -k 10 120 python bench.py --workload $w --steps 20 --warmup 3 --cpu-seconds 0 --no-cold $f > gpurun_out/tiles_$n.log 2>&1 || exit $?
  echo "$n $(grep '^{' gpurun_out/tiles_$n.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["seal_ms"], d["open_ms"], d["config"]["kernel"][:60])')"
done
