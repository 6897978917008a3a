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
    mempat) run mempat 120 tools/build/mempattern ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    test) run pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread ;;
    testall) run pytest_gpu 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread ;;
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
    default) run bench_default 600 python bench.py ;;
    pmc_hbm)
        W=${RG_PMC_WORKLOAD:-cfg2}
        run pmc_fetch_$W 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_fetch_$W -o p -- \
            python3 bench.py --workload $W --steps 5 --warmup 2 --cpu-seconds 0
        run pmc_write_$W 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_write_$W -o p -- \
            python3 bench.py --workload $W --steps 5 --warmup 2 --cpu-seconds 0 ;;
    tiles)
        W=${RG_WORKLOAD:-cfg2}
        for v in ${RG_TILES:-"auto:" "p1k0:--plan 1" "p0k1:--plan 0 --segments 1" "p1k1:--plan 1 --segments 1" "p1k2:--plan 1 --segments 2" "g1auto:--staged 1"}; do
            name=${v%%:*}; flags=${v#*:}; flags=${flags//_/ }
            run tiles_${W}_$name 200 python bench.py --workload $W $flags --steps 20 --warmup 3 --cpu-seconds 0
        done
        grep -H '"value"' gpurun_out/tiles_${W}_*.log | python3 -c "import sys,json
for l in sys.stdin:
    f,j=l.split(':',1); d=json.loads(j); print(f.split('/')[-1], d['value'], d['seal_ms'], d['open_ms'])" ;;
    pmc_list) run pmc_list 120 rocprofv3 -L ;;
    pmc)
        # separate passes (TCC FETCH_SIZE and WRITE_SIZE do not fit one pass; never combined with tracing domains)
        W=${RG_PMC_WORKLOAD:-cfg2}
        run pmc_sq 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
            --kernel-trace --output-format csv -d gpurun_out/pmc_sq -o p -- python3 bench.py --workload $W --steps 5 --warmup 2 --cpu-seconds 0
        run pmc_wait 300 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_SCA SQ_INSTS_LDS SQ_WAVES \
            --kernel-trace --output-format csv -d gpurun_out/pmc_wait -o p -- python3 bench.py --workload $W --steps 5 --warmup 2 --cpu-seconds 0
        run pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_fetch -o p -- \
            python3 bench.py --workload $W --steps 5 --warmup 2 --cpu-seconds 0
        run pmc_write 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_write -o p -- \
            python3 bench.py --workload $W --steps 5 --warmup 2 --cpu-seconds 0 ;;
    pmc2)
        W=${RG_PMC_WORKLOAD:-cfg2}
        run pmc_a 300 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INST_LEVEL_VMEM SQ_BUSY_CYCLES \
            --kernel-trace --output-format csv -d gpurun_out/pmc_a -o p -- python3 bench.py --workload $W --steps 5 --warmup 2 --cpu-seconds 0
        run pmc_b 300 rocprofv3 --pmc TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum TA_TA_BUSY_sum GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INST_CYCLES_VMEM_RD \
            --kernel-trace --output-format csv -d gpurun_out/pmc_b -o p -- python3 bench.py --workload $W --steps 5 --warmup 2 --cpu-seconds 0
        run pmc_c 300 rocprofv3 --pmc TCP_PENDING_STALL_CYCLES_sum TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum \
            --kernel-trace --output-format csv -d gpurun_out/pmc_c -o p -- python3 bench.py --workload $W --steps 5 --warmup 2 --cpu-seconds 0 ;;
    sweep)
        W=${RG_WORKLOAD:-cfg2}
        for l in 1 2 4; do for g in -1 0 2 3 4; do
            run sweep_${W}_l${l}_g${g} 200 python bench.py --workload $W --lanes $l --wg-per-cu $g --steps 20 --warmup 3 --cpu-seconds 0
        done; done
        grep -h '"value"' gpurun_out/sweep_${W}_*.log | python3 -c "import sys,json
for l in sys.stdin:
    d=json.loads(l); c=d['config']; print(c['lanes_per_packet'], c['wg_per_cu'], d['value'], d['seal_ms'], d['open_ms'], d['gpu_ms_per_step'])" ;;
    diag)
        W=${RG_WORKLOAD:-cfg2}
        for m in 0 1 2; do for l in 1 2; do
            run diag_${W}_m${m}_l${l} 200 python bench.py --workload $W --lanes $l --debug-mode $m --steps 20 --warmup 3 --cpu-seconds 0
        done; done
        grep -H '"value"' gpurun_out/diag_${W}_*.log | python3 -c "import sys,json
for l in sys.stdin:
    f,j=l.split(':',1); d=json.loads(j); print(f.split('/')[-1], d['seal_ms'])" ;;
    staged)
        W=${RG_WORKLOAD:-cfg2}
        for g in 0 1 2 4; do for c in 1 2; do
            run st_${W}_g${g}_c${c} 200 python bench.py --workload $W --staged $g --wg-per-cu $c --steps 20 --warmup 3 --cpu-seconds 0
        done; done
        grep -H '"value"' gpurun_out/st_${W}_*.log | python3 -c "import sys,json
for l in sys.stdin:
    f,j=l.split(':',1); d=json.loads(j); print(f.split('/')[-1], d['value'], d['seal_ms'], d['open_ms'])" ;;
    pmc_clock)
        W=${RG_WORKLOAD:-cfg2}
        for v in ${RG_PMC_VARIANTS:-"l1:--lanes_1_--staged_0" "l1m1:--lanes_1_--staged_0_--debug-mode_1" "l1m2:--lanes_1_--staged_0_--debug-mode_2" "l2:--lanes_2_--staged_0" "g2:--staged_2"}; do
            name=${v%%:*}; flags=${v#*:}; flags=${flags//_/ }
            run pmcclk_$name 240 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_WAVES SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY \
                --kernel-trace --output-format csv -d gpurun_out/pmcclk_$name -o p -- python3 bench.py --workload $W $flags --steps 5 --warmup 2 --cpu-seconds 0 --no-graph
        done
        python3 tools/pmc_clock.py gpurun_out/pmcclk_* ;;
    pmc_sq)
        W=${RG_PMC_WORKLOAD:-cfg2}
        run pmcsq_$W 240 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_WAVES SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY \
            --kernel-trace --output-format csv -d gpurun_out/pmcsq_$W -o p -- python3 bench.py --workload $W --steps 5 --warmup 2 --cpu-seconds 0 --no-graph
        run pmcsq2_$W 240 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS \
            --kernel-trace --output-format csv -d gpurun_out/pmcsq2_$W -o p -- python3 bench.py --workload $W --steps 5 --warmup 2 --cpu-seconds 0 --no-graph ;;
    stamps) run stamps_${RG_WORKLOAD:-cfg2} 300 python tools/stamps.py --workload ${RG_WORKLOAD:-cfg2} --staged ${RG_G:-2} --wg-per-cu ${RG_WPC:-0} ${RG_STAMP_FLAGS:-} ;;
    *) echo "unknown step $s"; exit 2 ;;
    esac
done
echo "all steps done"
