#!/bin/bash
# Runs a list of GPU steps on the gpurun box, each under its own time limit.
# Test failures (rc 1) do not stop the run; any other non-zero rc (fault,
# abort, timeout, signal) ends it immediately.
#   usage: tools/gpu_run.sh step1 [step2 ...]
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
export HSA_ENABLE_IPC_MODE_LEGACY=0

run() { # name timeout cmd...
    local name=$1 to=$2
    shift 2
    echo "== $name ($(date +%T))"
    timeout -k 10 "$to" "$@" >"gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "rc=$rc"
    tail -n 12 "gpurun_out/$name.log"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
        echo "stopping after $name (rc=$rc)"
        exit $rc
    fi
}

for s in "$@"; do
    case $s in
    micro) run micro 120 tools/build/microbench ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    test) run pytest_gpu 900 python -m pytest tests -m gpu -x -q ;;
    testall) run pytest_gpu 900 python -m pytest tests -m gpu -q ;;
    bench) run bench 400 python bench.py --steps 50 --warmup 10 --cpu-seconds 10 ;;
    benchq) run bench 300 python bench.py --steps 30 --warmup 5 --cpu-seconds 0 ;;
    bench_all)
        for w in cfg2 cfg3 cfg4 cfg5; do run bench_$w 300 python bench.py --workload $w --steps 30 --warmup 5 --cpu-seconds 0; done ;;
    lanes)
        for l in 1 2 4; do run bench_l$l 300 python bench.py --lanes $l --steps 30 --warmup 5 --cpu-seconds 0; done ;;
    e2e) run e2e 400 python bench.py --steps 10 --warmup 3 --cpu-seconds 0 --e2e ;;
    prof)
        run prof 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- \
            python3 bench.py --steps 30 --warmup 5 --cpu-seconds 0 ;;
    *) echo "unknown step $s"; exit 2 ;;
    esac
done
echo "all steps done"
