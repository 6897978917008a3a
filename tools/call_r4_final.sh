#!/bin/bash
# Round 4 final check, as the driver runs it: every GPU test, smoke(), the default bench line; then the
# round's profile set again (kernel stats, FETCH/WRITE, VALU counters, bench rows) on the final build.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r4_final_gputest.log 2>&1
rc=$?
tail -2 gpurun_out/r4_final_gputest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r4_final_smoke.log 2>&1 && tail -1 gpurun_out/r4_final_smoke.log &&
bash tools/round_profiles.sh > gpurun_out/r4_final_profiles.log 2>&1 && tail -8 gpurun_out/r4_final_profiles.log
