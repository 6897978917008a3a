# round 3: what the driver runs at round end, on the final build -- every GPU test, smoke(), the default bench line
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/final_gpu.log 2>&1
rc=$?; tail -2 gpurun_out/final_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final_smoke.log 2>&1 || exit $?
tail -1 gpurun_out/final_smoke.log
timeout -k 10 400 python bench.py > gpurun_out/final_bench.log 2>&1 || exit $?
grep '^{' gpurun_out/final_bench.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["seal_ms"], d["open_ms"], d["roofline"]["frac"], d["valu_roofline"]["frac"], [f["ratio"] for f in d["forged_open"]])'
