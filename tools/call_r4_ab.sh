#!/bin/bash
# Round 4: config 2 against the round-3 pipelined kernel (tools/build/librg_r3pipe.so), config 3 against two
# flattened-kernel variants (flat2w: 64-packet sub-units and two workgroups = two waves per SIMD;
# flatpk64: 64-packet sub-units alone), and the host-memory path by pipeline slice size (tools/e2e_probe.py).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
bash tools/ab.sh "base r3pipe" "cfg2" 3 --no-cold --forged 0 &&
bash tools/ab.sh "base flat2w flatpk64" "cfg3" 3 --no-cold --forged 0 &&
timeout -k 10 300 python tools/e2e_probe.py cfg2 2,4,8,16,32 > gpurun_out/r4_e2e_probe.jsonl && cat gpurun_out/r4_e2e_probe.jsonl
