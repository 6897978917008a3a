# round 3: config 2 without the LDS ring (lane-per-frame 64-byte frame-aligned stores), with and without the
# next chunk's loads issued ahead of the step's stores; parity of the pipelined paths on each build, then A/B
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
for V in nolines nolineslf; do
  RG_AEAD_LIB=tools/build/librg_$V.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_forged.py -x -q -k "pipe or cfg2 or auto" --timeout 120 --timeout-method thread > gpurun_out/${V}_tests.log 2>&1
  rc=$?; tail -1 gpurun_out/${V}_tests.log; [ $rc -ne 0 ] && exit $rc
done
bash tools/ab.sh "base nolines nolineslf" "cfg2" 3 --no-cold --forged 0
