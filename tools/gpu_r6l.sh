# round 6: config 2 on every kernel family of the current build (the automatic choice is the pipelined kernel)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for r in 1 2; do
for v in "auto:" "tile2:--staged 2" "tile2s2:--staged 2 --segments 2" "tile1:--staged 1" "flat:--staged 3"; do
    n=${v%%:*}; f=${v#*:}
    timeout -k 10 200 python bench.py --workload cfg2 --steps 20 --warmup 3 --cpu-seconds 0 --no-cold --forged 0 $f > gpurun_out/fam_${n}_$r.log 2>&1 || exit $?
    echo "$n $r $(grep '"value"' gpurun_out/fam_${n}_$r.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["seal_ms"], d["open_ms"], d["config"]["kernel"][:60])')"
done
done
