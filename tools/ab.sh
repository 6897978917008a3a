#!/bin/bash
# A/B of library builds on given workloads, interleaved, each run under its own limit.
#   usage: tools/ab.sh "base fence1 ..." "cfg2 cfg3" REPS [extra bench flags]
# "base" is the in-tree library, NAME is tools/build/librg_NAME.so (tools/build_variant.sh).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
LIBS=$1 WS=$2 REPS=${3:-2}
shift 3
for r in $(seq "$REPS"); do
    for w in $WS; do
        for v in $LIBS; do
            if [ "$v" = base ]; then unset RG_AEAD_LIB; else export RG_AEAD_LIB=tools/build/librg_$v.so; fi
            log=gpurun_out/ab_${v}_${w}_$r.log
            timeout -k 10 200 python bench.py --workload "$w" --steps 20 --warmup 3 --cpu-seconds 0 "$@" >"$log" 2>&1 || exit $?
            echo "$v $w $r $(grep '"value"' "$log" | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["seal_ms"], d["open_ms"], d.get("cold_cache", {}).get("gib_s"))')"
        done
    done
done
