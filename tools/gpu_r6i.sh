# round 6: the CPU baselines' placement study again, with OpenSSL keyed once per worker beside the per-packet re-key
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
echo "== cpu study"; timeout -k 10 600 python bench.py --cpu-study --cpu-seconds 24 > gpurun_out/cpu_study.json 2> gpurun_out/cpu_study.err || exit $?
grep '^{' gpurun_out/cpu_study.err
