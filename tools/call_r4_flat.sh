#!/bin/bash
# Round 4: flattened-kernel changes (every packet >= 1 chunk step, no skip loops; the stream's first column
# round read from LDS at a packet switch; the last chunk's Horner blocks interleaved with the carry powers;
# descriptor fields kept in registers and counters loaded with them): the flat / forged parity tests, an
# interleaved A/B against the committed build (tools/build_rev.sh head) on config 3 and config 2, the new
# build's cfg3 stamps (diag build), and the host path by slice size again.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_forged.py -x -q -m gpu \
    -k "flat or open_failures or bad_descriptors or malformed or digest or auto" --timeout 300 --timeout-method thread \
    > gpurun_out/r4_flat_tests.log 2>&1
rc=$?
tail -2 gpurun_out/r4_flat_tests.log
[ $rc -eq 0 ] || exit $rc
bash tools/ab.sh "base head" "cfg3" 3 --no-cold --forged 0 &&
bash tools/ab.sh "base head" "cfg2" 1 --no-cold --forged 0 &&
RG_AEAD_LIB=tools/build/librg_diag.so timeout -k 10 200 python tools/flat_stamps.py --workload cfg3 > gpurun_out/r4_cfg3_flat_stamps4.txt 2>&1 && cat gpurun_out/r4_cfg3_flat_stamps4.txt &&
timeout -k 10 300 python tools/e2e_probe.py cfg2 8,16,32 > gpurun_out/r4_e2e_probe6.jsonl && cat gpurun_out/r4_e2e_probe6.jsonl
