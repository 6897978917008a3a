#!/bin/bash
# Round 4, first look at real two-wave co-residency on config 2: the in-tree build against
# __launch_bounds__(256, 2) (tools/build_variant.sh lb2 -DRG_PIPE_LB2: the pipelined kernels forced
# into 256 VGPRs, so two 256-thread workgroups fit per CU), each with 1 and 2 lanes per packet.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
run() { # name lib flags...
    local name=$1 lib=$2
    shift 2
    if [ "$lib" = base ]; then unset RG_AEAD_LIB; else export RG_AEAD_LIB=tools/build/librg_$lib.so; fi
    timeout -k 10 200 python bench.py --workload cfg2 --steps 20 --warmup 3 --cpu-seconds 0 --no-cold --forged 0 "$@" \
        >gpurun_out/r4lb2_$name.log 2>&1 || { echo "$name FAILED $?"; tail -5 gpurun_out/r4lb2_$name.log; exit 1; }
    python3 -c "import json; d=json.loads([l for l in open('gpurun_out/r4lb2_$name.log') if l.startswith('{')][-1]); print('$name', d['value'], d['seal_ms'], d['open_ms'], d['config']['kernel'][:40])"
}
for rep in 1 2; do
    run base_l1_$rep base
    run lb2_l1_$rep lb2
    run base_l2w2_$rep base --lanes 2 --wg-per-cu 2
    run lb2_l2w2_$rep lb2 --lanes 2 --wg-per-cu 2
done
run base_l1_m1 base --debug-mode 1 --no-verify
run lb2_l2w2_m1 lb2 --lanes 2 --wg-per-cu 2 --debug-mode 1 --no-verify
run base_l2w2_m1 base --lanes 2 --wg-per-cu 2 --debug-mode 1 --no-verify
