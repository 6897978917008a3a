#!/bin/bash
# Round 4, last measurement on the final build: the default bench line with the host path, and the N = 4
# launcher path as the driver runs it with the four ranks sharing the GPU (RG_BENCH_SHARE_GPU=1).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python bench.py --e2e > gpurun_out/r4_last_default.jsonl 2> gpurun_out/r4_last_default.err && cat gpurun_out/r4_last_default.jsonl | cut -c1-600 &&
RG_BENCH_SHARE_GPU=1 timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 4 --steps 5 --warmup 2 --cpu-seconds 2 > gpurun_out/r4_rehearse_torchrun4.jsonl 2> gpurun_out/r4_rehearse_torchrun4.err && cut -c1-400 gpurun_out/r4_rehearse_torchrun4.jsonl
