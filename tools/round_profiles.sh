#!/bin/bash
# Everything the committed profiles/ of a round come from, in one GPU call (each step under its own
# time limit; a step that faults or times out ends the run):
#   default bench line and rocprofv3 --kernel-trace --stats of that same command, rocprofv3 kernel stats per
#   config, FETCH/WRITE passes, VALU issue counters, and the bench rows of every config.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
G="bash tools/gpu_run.sh"
$G default defprof || exit $?
for W in cfg2 cfg3 cfg4; do RG_WORKLOAD=$W $G prof || exit $?; done
for W in cfg2 cfg3 cfg4 cfg5; do RG_WORKLOAD=$W $G pmc_hbm || exit $?; done
RG_WORKLOADS="cfg2 cfg3 cfg4" $G valu || exit $?
RG_WORKLOADS="cfg2 cfg3 cfg4 cfg5" $G bench_all || exit $?
echo "round profiles done"
