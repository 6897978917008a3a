set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
if [ -z "${NOTEST:-}" ]; then
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/sweep_test.log 2>&1
rc=$?; tail -3 gpurun_out/sweep_test.log; [ $rc -eq 0 ] || exit $rc
fi
# each variant: name:workload:flags (flags with _ for spaces)
for v in ${VARIANTS}; do
  name=${v%%:*}; rest=${v#*:}; W=${rest%%:*}; flags=${rest#*:}; flags=${flags//_/ }
  timeout -k 10 200 python bench.py --workload $W $flags --steps 20 --warmup 3 --cpu-seconds 0 > gpurun_out/sweep_$name.log 2>&1 || exit 3
  python3 -c "import json,sys; d=json.loads([l for l in open('gpurun_out/sweep_$name.log') if l.startswith('{')][-1]); print('$name', d['value'], d['seal_ms'], d['open_ms'], d['roofline']['frac'])"
done
