#!/bin/bash
# round 3: forged-frame restore with wavefront-scope ordering (tests + open cost), and config-2
# experiments against the lockstep memory bursts: line stores spread over the rounds, staggered wave starts
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_forged.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r3_forged_tests.log 2>&1; rc=$?
tail -n 3 gpurun_out/r3_forged_tests.log
[ $rc -le 1 ] || exit $rc
for f in 0.01 0.1 1.0; do
  timeout -k 10 120 python bench.py --steps 10 --warmup 3 --no-cold --cpu-seconds 0 --forged $f > gpurun_out/r3_forged_$f.log 2>&1 || exit $?
  echo "cfg2 forged $f $(grep '^{' gpurun_out/r3_forged_$f.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["open_ms"], d["forged_open"])')"
done
for f in 0.01 0.1; do
  timeout -k 10 120 python bench.py --workload cfg4 --steps 5 --warmup 2 --no-cold --cpu-seconds 0 --forged $f > gpurun_out/r3_forged_cfg4_$f.log 2>&1 || exit $?
  echo "cfg4 forged $f $(grep '^{' gpurun_out/r3_forged_cfg4_$f.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["open_ms"], d["forged_open"])')"
done
tools/ab.sh "base spread wt3 stag16 stag5" "cfg2" 2 --no-cold || exit $?
