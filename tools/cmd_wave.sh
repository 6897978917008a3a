set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "wave or pipe" > gpurun_out/wave_test.log 2>&1
rc=$?; tail -3 gpurun_out/wave_test.log; [ $rc -eq 0 ] || exit $rc
NOTEST=1 bash tools/cmd_sweep.sh
