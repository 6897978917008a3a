#!/bin/bash
# Round 4: the flattened kernel's whole-group unit rule (> 1024 packets per unit) against the oracle.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v -m gpu -k "whole_groups" --timeout 400 --timeout-method thread > gpurun_out/r4_wholegroups.log 2>&1
rc=$?
tail -3 gpurun_out/r4_wholegroups.log
exit $rc
