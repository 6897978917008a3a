# round 3, config 3: workgroup-cooperative unit search over 4096-packet groups (default: work = 1 + 8 x chunks;
# coopw1: 1 + chunks; nocoop: the one-wave search over 1024-packet groups).  Flat-kernel tests, then A/B + phase stamps.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_forged.py -x -q -k "flat or imix or digest or coop" --timeout 120 --timeout-method thread > gpurun_out/coop_tests.log 2>&1
rc=$?; tail -3 gpurun_out/coop_tests.log; [ $rc -ne 0 ] && exit $rc
bash tools/ab.sh "nocoop base" cfg3 3 --no-cold --forged 0 || exit $?
for v in nocoop base; do
  if [ $v = base ]; then unset RG_AEAD_LIB; else export RG_AEAD_LIB=tools/build/librg_$v.so; fi
  timeout -k 10 120 python tools/flat_stamps.py --workload cfg3 > gpurun_out/coop_st_$v.log 2>&1 || exit $?
  echo "== $v"; grep -v amdgpu.ids gpurun_out/coop_st_$v.log | cut -c1-600
done
