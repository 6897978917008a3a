#!/bin/bash
# Round 4: the cooperative search's work weights at config 3 -- a packet's one-time-key block counted as 1
# (base), 2 or 3 eighths of a chunk step (kCoopWPkt, variant builds wp2 / wp3) -- interleaved A/B.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/ab.sh "base wp2 wp3" "cfg3" 3 --no-cold --forged 0
