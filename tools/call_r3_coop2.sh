# round 3, config 3: the workgroup-cooperative unit search (base) against the one-wave search (nocoop), 5 interleaved reps
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "coop or digest" --timeout 120 --timeout-method thread > gpurun_out/coop2_tests.log 2>&1
rc=$?; tail -1 gpurun_out/coop2_tests.log; [ $rc -ne 0 ] && exit $rc
bash tools/ab.sh "nocoop base" cfg3 5 --no-cold --forged 0
