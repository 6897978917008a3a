#!/bin/bash
# Round 4, final build (tile whole-chunk loops, flat carry top bit): every GPU test, smoke(), and the default bench line (with --e2e).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r4_check3_gputest.log 2>&1
rc=$?
tail -2 gpurun_out/r4_check3_gputest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r4_check3_smoke.log 2>&1 && tail -1 gpurun_out/r4_check3_smoke.log &&
timeout -k 10 400 python bench.py --e2e > gpurun_out/r4_check3_default.jsonl 2> gpurun_out/r4_check3_default.err && cut -c1-300 gpurun_out/r4_check3_default.jsonl
