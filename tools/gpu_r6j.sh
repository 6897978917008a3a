# round 6 check: the whole GPU suite, smoke, and the default bench line as the driver runs them
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
bash tools/gpu_run.sh testall smoke || exit $?
echo "== default bench"; timeout -k 10 600 python bench.py > gpurun_out/bench_default.log 2>&1 || exit $?
grep '"value"' gpurun_out/bench_default.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['value'], d['seal_ms'], d['open_ms'], d['roofline']['frac'], d['roofline']['valu']['frac']); print(json.dumps(d['cpu_baseline']['scaling'])); print(json.dumps(d['cpu_openssl']['scaling'])); print(d['cpu_baseline']['value'], d['cpu_openssl']['value'])"
