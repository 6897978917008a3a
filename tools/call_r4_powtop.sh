#!/bin/bash
# Round 4: the flattened kernel with the carry power's top bit taken as a choice of 1 or r (one square-and-multiply step fewer):
# flat parity tests, then an interleaved A/B against the committed
# build on config 3.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_forged.py -x -q -m gpu \
    -k "flat or open_failures or bad_descriptors or malformed or digest or auto" --timeout 300 --timeout-method thread \
    > gpurun_out/r4_powtop_tests.log 2>&1
rc=$?
tail -2 gpurun_out/r4_powtop_tests.log
[ $rc -eq 0 ] || exit $rc
bash tools/ab.sh "base head" "cfg3" 4 --no-cold --forged 0 2>&1 | tee gpurun_out/r4_cfg3_powtop_ab.txt
