#!/bin/bash
# Round 4: how many cycles the pipelined kernel spends before its first unit (kernel-argument loads, the
# walk's setup, the first descriptor): config 2 seal, one lane per packet, one workgroup per CU, stamps of
# the diag build (tools/coresidency.py reports the prologue beside the wave's cycles).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
RG_AEAD_LIB=tools/build/librg_diag.so timeout -k 10 200 python tools/coresidency.py --workload cfg2 --lanes 1 --wg-per-cu 1 --mode 3 > gpurun_out/r4_pipe_prologue.json 2>gpurun_out/r4_pipe_prologue.err && cat gpurun_out/r4_pipe_prologue.json
