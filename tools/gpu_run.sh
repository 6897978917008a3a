#!/bin/bash
# Runs a list of GPU steps on the gpurun box, each under its own time limit.
# Test failures (rc 1) do not stop the run; any other non-zero rc (fault,
# abort, timeout, signal) ends it immediately.
#   usage: tools/gpu_run.sh step1 [step2 ...]
# VARIANTS="name:workload:flags ..." (flags with _ for spaces) drives the
# variants / stamps_v / pmc_clock steps, e.g.
#   VARIANTS="p2:cfg2:--staged_0 t4:cfg4:--staged_2" tools/gpu_run.sh variants
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

summ() { # print value / seal / open / roofline of bench logs
    grep -H '"value"' "$@" | python3 -c "import sys,json
for l in sys.stdin:
    f,j=l.split(':',1); d=json.loads(j); print(f.split('/')[-1], d['value'], d['seal_ms'], d['open_ms'], d['roofline']['frac'], d['config']['kernel'][:40])"
}

each_variant() { # callback name workload flags...
    for v in ${VARIANTS:-}; do
        local name=${v%%:*} rest=${v#*:}
        local W=${rest%%:*} flags=${rest#*:}
        "$1" "$name" "$W" ${flags//_/ }
    done
}

bench_variant() { local n=$1 W=$2; shift 2; run var_$n 200 python bench.py --workload $W "$@" --steps 20 --warmup 3 --cpu-seconds 0; }
stamp_variant() { local n=$1 W=$2; shift 2; run stv_$n 200 python tools/stamps.py --workload $W "$@"; }
pmc_variant() {
    local n=$1 W=$2; shift 2
    run pmcclk_$n 240 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_WAVES SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY \
        --kernel-trace --output-format csv -d gpurun_out/pmcclk_$n -o p -- python3 bench.py --workload $W "$@" --steps 5 --warmup 2 --cpu-seconds 0 --no-graph
}

for s in "$@"; do
    case $s in
    micro) run micro 120 tools/build/microbench ;;
    mempat) run mempat 120 tools/build/mempattern ;;
    aux) run bench_aux 300 python tools/bench_aux.py ;;
    prof_aux) run prof_aux 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_aux -o run -- \
        python3 tools/bench_aux.py ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    test) run pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread ;;
    testall) run pytest_gpu 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread ;;
    ktest) run pytest_k 900 python -u -m pytest tests -m gpu -x -v -k "${PYTEST_K}" --timeout 180 --timeout-method thread ;;
    bench) run bench 400 python bench.py --steps 50 --warmup 10 --cpu-seconds 10 ;;
    benchq) run bench 300 python bench.py --steps 30 --warmup 5 --cpu-seconds 0 ;;
    bench_all)
        for w in ${RG_WORKLOADS:-cfg2 cfg3 cfg4 cfg5}; do run bench_$w 300 python bench.py --workload $w --steps 30 --warmup 5 --cpu-seconds 0; done
        summ gpurun_out/bench_cfg[2-5].log ;;
    e2e) run e2e 400 python bench.py --steps 10 --warmup 3 --cpu-seconds 0 --e2e ;;
    default) run bench_default 600 python bench.py ;;
    defprof) run prof_default 700 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_default -o run -- \
        python3 bench.py ;;
    cfg1) run bench_cfg1 300 python bench.py --workload cfg1 ;;
    prof)
        W=${RG_WORKLOAD:-cfg2}
        run prof_$W 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$W -o run -- \
            python3 bench.py --workload $W --steps 30 --warmup 5 --cpu-seconds 0 --no-cold ;;
    pmc_hbm)
        # separate passes: FETCH_SIZE and WRITE_SIZE do not fit one pass; never combined with tracing domains
        W=${RG_WORKLOAD:-cfg2}
        run pmc_fetch_$W 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_fetch_$W -o p -- \
            python3 bench.py --workload $W --steps 5 --warmup 2 --cpu-seconds 0 --no-cold ${RG_BENCH_FLAGS:-}
        run pmc_write_$W 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_write_$W -o p -- \
            python3 bench.py --workload $W --steps 5 --warmup 2 --cpu-seconds 0 --no-cold ${RG_BENCH_FLAGS:-} ;;
    valu)
        # issue counters of the transport kernels (one pass: 8 SQ + 2 GRBM), per BASELINE config
        for W in ${RG_WORKLOADS:-cfg2 cfg3 cfg4}; do
            run valu_$W 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_INSTS_LDS \
                SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT \
                --kernel-trace --output-format csv -d gpurun_out/valu_$W -o p -- \
                python3 bench.py --workload $W --steps 5 --warmup 2 --cpu-seconds 0 --no-cold ${RG_BENCH_FLAGS:-}
        done ;;
    hbmcal)
        # FETCH_SIZE / WRITE_SIZE / raw EA requests against known byte counts (1 GiB working set)
        for k in rd_coal rd_frame wr_coal wr_frame wr_split; do
            run hbmcal_fetch_$k 60 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/hbmcal/fetch_$k -o p -- tools/build/hbmcal $k
            run hbmcal_write_$k 60 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/hbmcal/write_$k -o p -- tools/build/hbmcal $k
            run hbmcal_ea_$k 60 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum --kernel-trace --output-format csv -d gpurun_out/hbmcal/ea_$k -o p -- tools/build/hbmcal $k
        done
        python3 tools/pmc_summary.py gpurun_out/hbmcal/* > gpurun_out/hbmcal_summary.txt 2>&1 || true ;;
    variants) each_variant bench_variant; summ gpurun_out/var_*.log ;;
    stamps_v) each_variant stamp_variant ;;
    pmc_clock) each_variant pmc_variant; python3 tools/pmc_clock.py gpurun_out/pmcclk_* ;;
    *) echo "unknown step $s"; exit 2 ;;
    esac
done
echo "all steps done"
