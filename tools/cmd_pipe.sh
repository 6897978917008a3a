set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k pipe > gpurun_out/pipe_test.log 2>&1
rc=$?; tail -5 gpurun_out/pipe_test.log; [ $rc -eq 0 ] || exit $rc
for w in cfg2 cfg3 cfg4; do
  timeout -k 10 200 python bench.py --workload $w --staged 4 --steps 20 --warmup 3 --cpu-seconds 0 > gpurun_out/pipe_bench_$w.log 2>&1 || exit 3
  python3 -c "import json,sys; d=json.loads([l for l in open('gpurun_out/pipe_bench_$w.log') if l.startswith('{')][-1]); print('$w', d['value'], d['seal_ms'], d['open_ms'], d['roofline']['frac'])"
done
