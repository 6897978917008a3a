#!/bin/bash
# A/B of variant libraries (tools/build/librg_<name>.so; "base" = the in-tree library) on one workload,
# alternating, two rounds:  LIBS="base w8" W=cfg3 FLAGS="--staged 3" tools/ab_lib.sh
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for rep in 1 2; do
    for v in ${LIBS:-base}; do
        if [ $v = base ]; then L=""; else L="RG_AEAD_LIB=tools/build/librg_$v.so"; fi
        env $L timeout -k 10 200 python bench.py --workload ${W:-cfg3} ${FLAGS:-} --steps 20 --warmup 3 --cpu-seconds 0 --no-cold > gpurun_out/ab_${v}_$rep.log 2>&1 || exit 1
        python3 -c "import json; d=json.loads([l for l in open('gpurun_out/ab_${v}_$rep.log') if l.startswith('{')][-1]); print('$v', $rep, d['value'], d['seal_ms'], d['open_ms'])"
    done
done
