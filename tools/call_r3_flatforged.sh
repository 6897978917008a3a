#!/bin/bash
# round 3: the flat kernel's cooperative restore -- forged-frame tests, flat parity, forged-open cost on config 3
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_forged.py tests/test_gpu_parity.py -k "forged or flat or untouched or imix" -x -q --timeout 120 --timeout-method thread > gpurun_out/r3_flat_tests.log 2>&1; rc=$?
tail -n 3 gpurun_out/r3_flat_tests.log
[ $rc -eq 0 ] || exit $rc
for f in 0.01 0.1 1.0; do
  timeout -k 10 150 python bench.py --workload cfg3 --steps 5 --warmup 2 --no-cold --cpu-seconds 0 --forged $f > gpurun_out/r3f_cfg3_$f.log 2>&1 || exit $?
  echo "cfg3 $f $(grep '^{' gpurun_out/r3f_cfg3_$f.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["open_ms"], d["forged_open"])')"
done
