# round 6: the N > 1 bench path rehearsed on one GPU (two ranks sharing it over gloo), with every leg the
# driver's 8-GPU run takes on rank 0: base_1gpu, single_process, e2e_multi (NUMA-placed frames), CPU baselines
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export RG_BENCH_SHARE_GPU=1
timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 5 --warmup 2 > gpurun_out/rehearse2.log 2>&1 || { tail -30 gpurun_out/rehearse2.log; exit 1; }
grep '"value"' gpurun_out/rehearse2.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['value'], d['n_gpus'], d.get('speedup'), json.dumps(d.get('e2e_multi'))[:900]); print(json.dumps(d['cpu_openssl']['scaling'])[:400])"
