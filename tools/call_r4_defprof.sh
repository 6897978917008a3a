#!/bin/bash
# Round 4: rocprofv3 kernel stats of the default bench command itself (python bench.py, no flags).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_default -o run -- python3 bench.py > gpurun_out/prof_default.log 2>&1
rc=$?
grep '^{' gpurun_out/prof_default.log | cut -c1-200
find gpurun_out/prof_default -name "*kernel_stats.csv" | head -2
exit $rc
