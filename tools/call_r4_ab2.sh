#!/bin/bash
# Round 4: config 3 with two waves per SIMD at 128-packet sub-units (flat2w128: -DRG_FLAT_WG_PER_CU=2, the
# LDS image trimmed to fit two workgroups per CU), and a copy/kernel timeline of the host-memory path
# (rocprofv3 memory-copy + kernel traces of tools/e2e_probe.py at 16 MiB slices).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/ab.sh "base flat2w128" "cfg3" 3 --no-cold --forged 0 &&
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/r4_e2e_trace -o e2e -- python3 tools/e2e_probe.py cfg2 16 > gpurun_out/r4_e2e_trace.log 2>&1
ls -R gpurun_out/r4_e2e_trace | head -20
