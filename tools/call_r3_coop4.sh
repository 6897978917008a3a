# round 3, config 3: cooperative search staging its first sub-units from a shared LDS window (base) vs from memory (prev)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_forged.py -x -q -k "flat or imix or digest or coop" --timeout 120 --timeout-method thread > gpurun_out/coop4_tests.log 2>&1
rc=$?; tail -1 gpurun_out/coop4_tests.log; [ $rc -ne 0 ] && exit $rc
bash tools/ab.sh "prev base" cfg3 4 --no-cold --forged 0 || exit $?
timeout -k 10 120 python tools/flat_stamps.py --workload cfg3 > gpurun_out/coop4_st.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/coop4_st.log | cut -c1-420
