# round 3: GPU tests on the current build, then the N > 1 bench path rehearsed on one GPU (2 ranks sharing it)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/allgpu.log 2>&1
rc=$?; tail -2 gpurun_out/allgpu.log; [ $rc -ne 0 ] && exit $rc
RG_BENCH_SHARE_GPU=1 timeout -k 10 400 python bench.py --gpus 2 --steps 5 --warmup 2 --cpu-seconds 2 > gpurun_out/rehearse2.log 2>&1
rc=$?; tail -c 3000 gpurun_out/rehearse2.log; exit $rc
