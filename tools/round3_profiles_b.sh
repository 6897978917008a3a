#!/bin/bash
# round 3 final profiles, part B: FETCH_SIZE / WRITE_SIZE passes per config and the VALU issue counters
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
G="bash tools/gpu_run.sh"
for W in cfg2 cfg3 cfg4 cfg5; do RG_WORKLOAD=$W $G pmc_hbm || exit $?; done
RG_WORKLOADS="cfg2 cfg3 cfg4" $G valu || exit $?
echo "round profiles B done"
