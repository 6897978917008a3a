#!/bin/bash
# round 3: the staged (LDS-DMA) chunk stream of the pipelined kernel on config 2 -- per-wave stamps with
# and without it, interleaved A/B of staging depths, forged-tag open cost
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 120 python tools/stamps.py --workload cfg2 --plan 0 > gpurun_out/r3_stamps_dma.log 2>&1 || exit $?
RG_AEAD_LIB=tools/build/librg_nodma.so timeout -k 10 120 python tools/stamps.py --workload cfg2 --plan 0 > gpurun_out/r3_stamps_nodma.log 2>&1 || exit $?
grep -A3 '"seal"\|"open"' gpurun_out/r3_stamps_dma.log gpurun_out/r3_stamps_nodma.log | grep -v "^--$" | head -20
tools/ab.sh "base nodma d3 d6" "cfg2" 2 --no-cold || exit $?
for f in 0.01 0.1; do
  timeout -k 10 120 python bench.py --steps 10 --warmup 3 --no-cold --cpu-seconds 0 --forged $f > gpurun_out/r3_forged_$f.log 2>&1 || exit $?
  echo "forged $f $(grep '^{' gpurun_out/r3_forged_$f.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["open_ms"], d["forged_open"])')"
done
timeout -k 10 120 python bench.py --workload cfg4 --steps 5 --warmup 2 --no-cold --cpu-seconds 0 --forged 0.1 > gpurun_out/r3_forged_cfg4.log 2>&1 || exit $?
echo "cfg4 forged 0.1 $(grep '^{' gpurun_out/r3_forged_cfg4.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["open_ms"], d["forged_open"])')"
