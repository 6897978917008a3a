cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
bash tools/gpu_run.sh test && \
RG_BENCH_SHARE_GPU=1 timeout -k 10 400 python bench.py --single-process --gpus 2 --steps 5 --warmup 2 > gpurun_out/sp2.log 2>&1; echo rc=$?; tail -c 3000 gpurun_out/sp2.log
