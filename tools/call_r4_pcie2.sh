#!/bin/bash
# Round 4: the bench line's e2e.pcie_ceiling with hipHostMalloc buffers (short bench run).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --e2e --steps 5 --warmup 2 --cpu-seconds 0 --forged 0 --no-cold > gpurun_out/r4_pcie2.jsonl 2>gpurun_out/r4_pcie2.err && python3 -c "import json; d=json.loads(open('gpurun_out/r4_pcie2.jsonl').read()); print(d['e2e'])"
