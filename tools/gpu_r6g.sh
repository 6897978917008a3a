# round 6: the CPU baselines' placement study (no GPU), then the default bench line with the new placement
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
echo "== cpu study"; timeout -k 10 500 python bench.py --cpu-study --cpu-seconds 30 > gpurun_out/cpu_study.json 2> gpurun_out/cpu_study.err || exit $?
grep '^{' gpurun_out/cpu_study.err
grep -o '"cpus": \[[^]]*\]\|"cpus_compact": \[[^]]*\]' gpurun_out/cpu_study.json
echo "== default bench"; timeout -k 10 600 python bench.py > gpurun_out/bench_default.log 2>&1 || exit $?
grep '"value"' gpurun_out/bench_default.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['value']); print(json.dumps(d['cpu_baseline']['scaling'])); print(json.dumps(d['cpu_openssl']['scaling'])); print(d['cpu_baseline']['value'], d['cpu_openssl']['value'])"
