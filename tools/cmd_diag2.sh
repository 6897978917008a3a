set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
W=${W:-cfg2}
for m in 3 1 2 5; do
  timeout -k 10 200 python tools/stamps.py --workload $W --staged 4 --mode $m > gpurun_out/st_${W}_m$m.log 2>&1 || exit 3
  python3 -c "
import json; t=open('gpurun_out/st_${W}_m$m.log').read(); d=json.loads(t[t.index('{'):])
s=d['seal']; print('$W m$m', s['wave_us_pct_0_10_50_90_100'], s['shader_clock_ghz'], s['cycles_per_wave_mean'], s['end_us_pct_0_50_90_100'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_pipe -o run -- python3 bench.py --workload $W --staged 4 --steps 20 --warmup 3 --cpu-seconds 0 > gpurun_out/prof_pipe.log 2>&1 || exit 3
grep -h "pipe\|Name" gpurun_out/prof_pipe/*kernel_stats.csv | cut -c1-200
