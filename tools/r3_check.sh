#!/bin/bash
# round-3 check: forged-frame tests, parity suite, default bench line, forged bench (one GPU call)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
step() { # name timeout cmd...
    local name=$1 to=$2; shift 2
    echo "== $name $(date +%T)"
    timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "rc=$rc"; tail -n 4 "gpurun_out/$name.log"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stop after $name"; exit $rc; fi
}
for s in "$@"; do
    case $s in
    forged) step forged 600 python -u -m pytest tests/test_gpu_forged.py -x -v --timeout 120 --timeout-method thread ;;
    parity) step parity 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sessions.py tests/test_gpu_sessions_dev.py -v --timeout 120 --timeout-method thread ;;
    allgpu) step allgpu 1000 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread ;;
    bench) step bench 300 python bench.py --steps 20 --warmup 5 --cpu-seconds 0 ;;
    bench_forged) step bench_forged 300 python bench.py --steps 10 --warmup 3 --no-cold --cpu-seconds 0 --forged 0.1 ;;
    bench_forged1) step bench_forged1 300 python bench.py --steps 10 --warmup 3 --no-cold --cpu-seconds 0 --forged 0.01 ;;
    bench_cfg4f) step bench_cfg4f 300 python bench.py --workload cfg4 --steps 5 --warmup 2 --no-cold --cpu-seconds 0 --forged 0.1 ;;
    bench_all) for w in cfg2 cfg3 cfg4 cfg5; do step bench_$w 300 python bench.py --workload $w --steps 10 --warmup 3 --no-cold --cpu-seconds 0; done ;;
    prof) step prof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python bench.py --steps 20 --warmup 5 --no-cold --cpu-seconds 0 ;;
    esac
done
