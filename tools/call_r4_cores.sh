#!/bin/bash
# Round 4: per-wave HW_ID stamps of config 2's seal on the __launch_bounds__(256, 2) build
# (tools/build_variant.sh lb2 -DRG_PIPE_LB2): two lanes per packet, two workgroups per CU.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export RG_AEAD_LIB=tools/build/librg_lb2.so
timeout -k 10 120 python tools/coresidency.py --lanes 2 --wg-per-cu 2 --mode 3 > gpurun_out/r4_cores_l2w2.json &&
timeout -k 10 120 python tools/coresidency.py --lanes 2 --wg-per-cu 2 --mode 1 > gpurun_out/r4_cores_l2w2_m1.json &&
timeout -k 10 120 python tools/coresidency.py --lanes 1 --wg-per-cu 1 --mode 3 > gpurun_out/r4_cores_l1w1.json &&
timeout -k 10 120 python tools/coresidency.py --lanes 1 --wg-per-cu 1 --mode 1 > gpurun_out/r4_cores_l1w1_m1.json
