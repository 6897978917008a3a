#!/bin/bash
# round 3 final profiles, part A: default bench line, rocprofv3 kernel stats per config, bench rows of every config
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
G="bash tools/gpu_run.sh"
$G default || exit $?
for W in cfg2 cfg3 cfg4; do RG_WORKLOAD=$W $G prof || exit $?; done
RG_WORKLOADS="cfg2 cfg3 cfg4 cfg5" $G bench_all || exit $?
echo "round profiles A done"
