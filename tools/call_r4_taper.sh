#!/bin/bash
# Round 4: the host-memory path with tapered slices (first and last a quarter of the span) and the small
# uploads moved off the frame stream: host-path GPU tests, then the slice-size probe for this build and the
# committed one (tools/build_rev.sh head) on the same box.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu -k "host or session or group or recv or send" --timeout 300 --timeout-method thread > gpurun_out/r4_taper_tests.log 2>&1
rc=$?
tail -2 gpurun_out/r4_taper_tests.log
[ $rc -eq 0 ] || exit $rc
for r in 1; do
    timeout -k 10 300 python tools/e2e_probe.py cfg2 4,8,16,32 > gpurun_out/r4_taper_new_$r.jsonl && echo "new $r" && cat gpurun_out/r4_taper_new_$r.jsonl || exit 1
    RG_AEAD_LIB=tools/build/librg_head.so timeout -k 10 300 python tools/e2e_probe.py cfg2 16 > gpurun_out/r4_taper_head_$r.jsonl && echo "head $r" && cat gpurun_out/r4_taper_head_$r.jsonl || exit 1
done
