#!/bin/bash
# Round 4: GPU tests on the current build, the host-link ceilings (tools/pcie.hip), then config 2 against
# the round-3 pipelined kernel (tools/build/librg_r3pipe.so: commit e1c0e7c's rg_pipe.hip with today's
# other objects) and config 3 against two flattened-kernel variants (flat2w: 64-packet sub-units, two
# workgroups = two waves per SIMD; flatpk64: 64-packet sub-units alone).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r4_gputest.log 2>&1
rc=$?
tail -3 gpurun_out/r4_gputest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 tools/build/pcie 256 > gpurun_out/r4_pcie.json && cat gpurun_out/r4_pcie.json &&
bash tools/ab.sh "base r3pipe" "cfg2" 3 --no-cold --forged 0 &&
bash tools/ab.sh "base flat2w flatpk64" "cfg3" 3 --no-cold --forged 0
