#!/bin/bash
# Round 4: the first lane-quad key-block group fused with the one-lane pass (flattened kernel, phase A):
# flat / forged / malformed / digest GPU tests, interleaved A/B against the committed build on config 3,
# and the per-wave stamps by unit packet count (diag build).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_forged.py -x -q -m gpu \
    -k "flat or open_failures or bad_descriptors or malformed or digest or auto" --timeout 300 --timeout-method thread \
    > gpurun_out/r4_quadfuse_tests.log 2>&1
rc=$?
tail -2 gpurun_out/r4_quadfuse_tests.log
[ $rc -eq 0 ] || exit $rc
bash tools/ab.sh "base head" "cfg3" 3 --no-cold --forged 0 &&
RG_AEAD_LIB=tools/build/librg_diag.so timeout -k 10 200 python tools/flat_stamps.py --workload cfg3 --per-wave > gpurun_out/r4_cfg3_perwave2.txt 2>&1 && grep -v "^slowest" gpurun_out/r4_cfg3_perwave2.txt
