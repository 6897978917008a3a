#!/bin/bash
# Round 4: the cooperative search's work weights at config 3 -- a packet's one-time-key block counted as 1
# (base), 2 or 3 eighths of a chunk step (kCoopWPkt, variant builds wp2 / wp3) -- interleaved A/B.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/ab.sh "base wp2 wp3" "cfg3" 3 --no-cold --forged 0
timeout -k 10 400 python -u -m pytest tests/test_gpu_bench_ranks.py -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/r4_bench_ranks_test.log 2>&1
rc=$?
tail -3 gpurun_out/r4_bench_ranks_test.log
exit $rc
