#!/bin/bash
# Round 4, final build: the flattened kernel's per-wave phases on config 3 (diag build), after the carry
# power's top-bit change and the dropped barrier.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
RG_AEAD_LIB=tools/build/librg_diag.so timeout -k 10 200 python tools/flat_stamps.py --workload cfg3 --per-wave > gpurun_out/r4_cfg3_perwave_final.txt 2>&1
rc=$?
head -3 gpurun_out/r4_cfg3_perwave_final.txt | cut -c1-600
exit $rc
