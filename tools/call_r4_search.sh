#!/bin/bash
# Round 4: where the flattened kernel's cooperative unit search spends its ~10 k cycles (diag build, search
# sub-stamps), and the ADVICE r3 regrow test of the MAC key table on a busy stream.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "mac_verify" --timeout 120 --timeout-method thread > gpurun_out/r4_mac_tests.log 2>&1
rc=$?
tail -2 gpurun_out/r4_mac_tests.log
[ $rc -eq 0 ] || exit $rc
RG_AEAD_LIB=tools/build/librg_diag.so timeout -k 10 200 python tools/flat_stamps.py --workload cfg3 > gpurun_out/r4_cfg3_search_stamps.txt 2>&1 && cat gpurun_out/r4_cfg3_search_stamps.txt
