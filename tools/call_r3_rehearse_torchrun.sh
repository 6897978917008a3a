# round 3: the N > 1 bench path rehearsed on one GPU exactly as the driver launches it (torch.distributed.run,
# WORLD_SIZE set, bench.py does not spawn ranks itself); 2 ranks then 4 ranks sharing the GPU over gloo
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
for n in 2 4; do
  RG_BENCH_SHARE_GPU=1 timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
    --master-addr 127.0.0.1 --master-port $((29500 + n)) bench.py --gpus $n --steps 5 --warmup 2 --cpu-seconds 2 \
    > gpurun_out/rehearse_tr$n.log 2>&1
  rc=$?; grep '^{' gpurun_out/rehearse_tr$n.log | cut -c1-400; [ $rc -ne 0 ] && { tail -20 gpurun_out/rehearse_tr$n.log; exit $rc; }
done
exit 0
