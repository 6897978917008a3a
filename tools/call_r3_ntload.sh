# round 3: streaming (nt) payload loads in the flattened kernel -- do the partially written lines survive
# longer in L2 (config 3 WRITE_SIZE), and what does it do to the launch?  Parity on the variant first.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
RG_AEAD_LIB=tools/build/librg_ntload.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "flat" --timeout 120 --timeout-method thread > gpurun_out/nt_tests.log 2>&1
rc=$?; tail -2 gpurun_out/nt_tests.log; [ $rc -ne 0 ] && exit $rc
VS="ntload" bash tools/call_r3_flattraffic.sh || exit 1
bash tools/ab.sh "base ntload" "cfg3" 3 --no-cold --forged 0
