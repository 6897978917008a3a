#!/bin/bash
# Round 4: host path (config 2, 8 MiB slices) with the HIP API trace beside copies and kernels, to see
# which host call waits (tools/e2e_timeline.py + the api CSV).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --hip-trace --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/e2etrace3 -o run -- python3 tools/e2e_probe.py cfg2 8 > gpurun_out/e2etrace3.log 2>&1
