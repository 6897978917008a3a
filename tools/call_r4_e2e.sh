#!/bin/bash
# Round 4: the host-memory path with one upload, one kernel and one download stream per context (the
# slices of a direction back to back, the two directions beside each other): the host-path GPU tests,
# the slice-size probe, and a copy/kernel timeline.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_sessions.py tests/test_gpu_group.py tests/test_gpu_sessions_dev.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r4_e2e_tests.log 2>&1
rc=$?
tail -2 gpurun_out/r4_e2e_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/e2e_probe.py cfg2 4,8,16,32 > gpurun_out/r4_e2e_probe2.jsonl && cat gpurun_out/r4_e2e_probe2.jsonl &&
timeout -k 10 120 tools/build/pcie 256 &&
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/r4_e2e_trace2 -o e2e -- python3 tools/e2e_probe.py cfg2 16 > gpurun_out/r4_e2e_trace2.log 2>&1
