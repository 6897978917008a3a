#!/bin/bash
# round 3: verify-then-decrypt open (RG_PIPE_MAC_FIRST) -- forged/parity tests, forged-tag open cost,
# interleaved A/B against decrypt-first (df) and staggered wave starts
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_forged.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r3_mf_tests.log 2>&1; rc=$?
tail -n 3 gpurun_out/r3_mf_tests.log
[ $rc -eq 0 ] || exit $rc
for f in 0.01 0.1 1.0; do
  timeout -k 10 120 python bench.py --steps 10 --warmup 3 --no-cold --cpu-seconds 0 --forged $f > gpurun_out/r3_forged_$f.log 2>&1 || exit $?
  echo "cfg2 forged $f $(grep '^{' gpurun_out/r3_forged_$f.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["open_ms"], d["forged_open"])')"
done
tools/ab.sh "base df stag16 stag32" "cfg2" 3 --no-cold || exit $?
