# forged-tag open cost on the final build (cfg2 pipelined, cfg4 tiles)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
for v in "cfg2:0.1" "cfg2:1.0" "cfg4:0.1" "cfg4:1.0"; do
  w=${v%%:*}; f=${v#*:}
  timeout -k 10 200 python bench.py --workload $w --steps 10 --warmup 2 --cpu-seconds 0 --no-cold --forged $f > gpurun_out/forged_${w}_$f.log 2>&1 || exit $?
  echo "$w $f $(grep '^{' gpurun_out/forged_${w}_$f.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["open_ms"], d["forged_open"])')"
done
