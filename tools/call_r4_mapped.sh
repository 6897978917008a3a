#!/bin/bash
# Round 4: the host path with descriptors, counters and statuses in mapped host memory (working tree)
# against the committed build (tools/build/librg_head.so, three copies per slice): host-path GPU tests,
# then tools/e2e_probe.py on configs 2 and 3 by slice size, interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu -k "host or group or sessions" --timeout 120 --timeout-method thread > gpurun_out/r4_mapped_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r4_mapped_tests.log
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
    for v in head base; do
        if [ "$v" = base ]; then unset RG_AEAD_LIB; else export RG_AEAD_LIB=tools/build/librg_$v.so; fi
        for w in cfg2 cfg3; do
            echo "== $v $w run $r"
            timeout -k 10 240 python tools/e2e_probe.py $w 4,8,16 || exit $?
        done
    done
done 2>&1 | tee gpurun_out/r4_e2e_mapped_ab.txt
