#!/bin/bash
# Round 4: the flattened kernel's slowest waves at config 3 -- each wave's first sub-unit (packets, chunks,
# steps) and XCD beside its phase cycles (diag build) -- and the GPU tests after the device-restore change.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r4_gputest2.log 2>&1
rc=$?
tail -2 gpurun_out/r4_gputest2.log
[ $rc -eq 0 ] || exit $rc
RG_AEAD_LIB=tools/build/librg_diag.so timeout -k 10 200 python tools/flat_stamps.py --workload cfg3 --per-wave > gpurun_out/r4_cfg3_perwave.txt 2>&1 && cat gpurun_out/r4_cfg3_perwave.txt
