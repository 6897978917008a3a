# round 6 profile set, part 2: the CPU baselines' scaling study (no GPU), HBM counter passes, VALU issue
# counters, the bench rows of every config
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
echo "== cpu study"; timeout -k 10 400 python bench.py --cpu-study --cpu-seconds 24 > gpurun_out/cpu_study.json 2> gpurun_out/cpu_study.err || exit $?
cat gpurun_out/cpu_study.err
G="bash tools/gpu_run.sh"
for W in cfg2 cfg3 cfg4 cfg5; do RG_WORKLOAD=$W $G pmc_hbm || exit $?; done
RG_WORKLOADS="cfg2 cfg3 cfg4" $G valu || exit $?
RG_WORKLOADS="cfg2 cfg3 cfg4 cfg5" $G bench_all || exit $?
echo "profile set part 2 done"
