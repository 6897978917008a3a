# tile pool prefetch: tests on the pool-from-2-rounds build, A/B base (pool from 16 rounds, ahead) / pmin2 / pmin2noahead
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
RG_AEAD_LIB=tools/build/librg_pmin2.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q -k "tile_dynamic_deal or digest or tile_g2" --timeout 120 --timeout-method thread > gpurun_out/pool2_pytest.log 2>&1; rc=$?; tail -n 2 gpurun_out/pool2_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 bash tools/ab.sh "base pmin2 pmin2noahead" "cfg4 cfg5" 3 --no-cold || exit $?
