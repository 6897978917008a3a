# refresh after the dynamic tile deal: default line, bench rows, cfg4 stats, cfg4/cfg5 traffic
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
G="bash tools/gpu_run.sh"
$G default || exit $?
RG_WORKLOAD=cfg4 $G prof || exit $?
for W in cfg4 cfg5; do RG_WORKLOAD=$W $G pmc_hbm || exit $?; done
RG_WORKLOADS="cfg4" $G valu || exit $?
RG_WORKLOADS="cfg2 cfg3 cfg4 cfg5" $G bench_all || exit $?
