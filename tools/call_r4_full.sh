#!/bin/bash
# Round 4: every GPU test, the host-memory path by slice size (four slots), the default bench line, the
# single-process bench on one GPU (two contexts sharing it: a rehearsal), and the N = 2 launcher path as
# the driver runs it, both ranks sharing the GPU (RG_BENCH_SHARE_GPU=1; gloo bookkeeping).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r4_gputest.log 2>&1
rc=$?
tail -2 gpurun_out/r4_gputest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/e2e_probe.py cfg2 8,16,32 > gpurun_out/r4_e2e_probe3.jsonl && cat gpurun_out/r4_e2e_probe3.jsonl &&
timeout -k 10 400 python bench.py --e2e > gpurun_out/r4_bench_default.jsonl 2> gpurun_out/r4_bench_default.err && cat gpurun_out/r4_bench_default.jsonl &&
RG_BENCH_SHARE_GPU=1 timeout -k 10 300 python bench.py --single-process --gpus 2 --steps 5 --warmup 2 > gpurun_out/r4_single_share2.jsonl 2> gpurun_out/r4_single_share2.err && cat gpurun_out/r4_single_share2.jsonl &&
RG_BENCH_SHARE_GPU=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 --cpu-seconds 2 > gpurun_out/r4_rehearse_torchrun2.jsonl 2> gpurun_out/r4_rehearse_torchrun2.err && cat gpurun_out/r4_rehearse_torchrun2.jsonl
RG_AEAD_LIB=tools/build/librg_diag.so timeout -k 10 200 python tools/flat_stamps.py --workload cfg3 > gpurun_out/r4_cfg3_flat_stamps.txt 2>&1 && cat gpurun_out/r4_cfg3_flat_stamps.txt
