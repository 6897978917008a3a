#!/bin/bash
# Round 4 diagnostic: the host path (config 2) with 4 (the box's default), 8 and 16 hardware queues per
# process, to see whether the pipeline streams share a queue.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for q in 4 8 16; do
    echo "== GPU_MAX_HW_QUEUES=$q"
    GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python tools/e2e_probe.py cfg2 8,16 || exit $?
done 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r4_e2e_hwq.txt
