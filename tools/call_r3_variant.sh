# round 3: one flattened-kernel build variant (tools/build/librg_$V.so): parity of the flat paths and the
# forged-frame tests on it, config-3 FETCH_SIZE / WRITE_SIZE passes, then an interleaved A/B against the
# in-tree build.   usage: V=align bash tools/call_r3_variant.sh
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
RG_AEAD_LIB=tools/build/librg_$V.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_forged.py -x -q -k "flat or imix or cfg3" --timeout 120 --timeout-method thread > gpurun_out/${V}_tests.log 2>&1
rc=$?; tail -2 gpurun_out/${V}_tests.log; [ $rc -ne 0 ] && exit $rc
[ "${TRAFFIC:-1}" = 1 ] && { VS="base $V" bash tools/call_r3_flattraffic.sh || exit 1; }
[ "${LDS:-0}" = 1 ] && { RG_AEAD_LIB=tools/build/librg_$V.so TAG=$V WS=cfg3 bash tools/call_r3_lds.sh || exit 1; }
bash tools/ab.sh "base $V" "${WS:-cfg3}" ${REPS:-3} --no-cold --forged 0
