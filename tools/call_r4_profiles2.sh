#!/bin/bash
# Round 4, the profile set again on the final build (tile seal fast path, flat barrier dropped):
# default line, kernel stats, FETCH/WRITE passes, VALU counters, bench rows of every config.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/round_profiles.sh > gpurun_out/r4_profiles2.log 2>&1
rc=$?
tail -8 gpurun_out/r4_profiles2.log
exit $rc
