#!/bin/bash
# Round 4: instruction-cache and wait-state counters of the pipelined (config 2) and flattened (config 3)
# kernels: does instruction fetch explain the one-time phases' cycles?  One rocprofv3 pass per counter set
# (SQ issue/wait states + instruction fetch; SQC instruction-cache requests / hits / misses), each under
# its own kill timer.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for W in cfg3 cfg2; do
    timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_IFETCH SQ_IFETCH_LEVEL \
        --kernel-trace --output-format csv -d gpurun_out/icache_sq_$W -o p -- \
        python3 bench.py --workload $W --steps 3 --warmup 1 --cpu-seconds 0 --no-graph --no-cold --forged 0 \
        > gpurun_out/icache_sq_$W.log 2>&1 || exit $?
    timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE \
        --kernel-trace --output-format csv -d gpurun_out/icache_sqc_$W -o p -- \
        python3 bench.py --workload $W --steps 3 --warmup 1 --cpu-seconds 0 --no-graph --no-cold --forged 0 \
        > gpurun_out/icache_sqc_$W.log 2>&1 || exit $?
done
python3 tools/pmc_summary.py gpurun_out/icache_sq_* gpurun_out/icache_sqc_* > gpurun_out/icache_summary.txt 2>&1
cat gpurun_out/icache_summary.txt
