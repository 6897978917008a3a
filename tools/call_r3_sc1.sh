# round 3: write-through (sc1) frame stores -- pipelined kernel's line-store waves through a buffer window, tile
# kernel's window stores.  Parity + forged-frame tests on the new build, then interleaved A/B:
# old = previous commit (plain stores), nosc1 = new code with RG_STORE_SC1=0, base = new (sc1)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_gpu_forged.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/sc1_tests.log 2>&1
rc=$?; tail -3 gpurun_out/sc1_tests.log; [ $rc -ne 0 ] && exit $rc
bash tools/ab.sh "old nosc1 base" "cfg2 cfg3 cfg4 cfg5" 2 --no-cold --forged 0
