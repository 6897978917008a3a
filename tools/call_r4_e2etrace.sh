#!/bin/bash
# Round 4: copy + kernel timeline of the host path (config 2, 8 MiB slices), to find where a seal call
# loses to the duplex ceiling (tools/e2e_timeline.py reads the CSVs).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/e2etrace -o run -- python3 tools/e2e_probe.py cfg2 8 > gpurun_out/e2etrace.log 2>&1
rc=$?
tail -3 gpurun_out/e2etrace.log
find gpurun_out/e2etrace -name "*.csv" | head
exit $rc
