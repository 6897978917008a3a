#!/bin/bash
# Round 4: host path with uploads read by a 128-workgroup host-load kernel (working tree)
# against the committed build (tools/build/librg_head.so): host-path GPU tests, interleaved
# tools/e2e_probe.py on configs 2 and 3, then a copy + kernel trace of the working tree.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu -k "host or group or sessions or pinned" --timeout 120 --timeout-method thread > gpurun_out/r4_hostload_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r4_hostload_tests.log
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
    for v in head base; do
        if [ "$v" = base ]; then unset RG_AEAD_LIB; else export RG_AEAD_LIB=tools/build/librg_$v.so; fi
        for w in cfg2 cfg3; do
            echo "== $v $w run $r"
            timeout -k 10 240 python tools/e2e_probe.py $w 4,8,16 || exit $?
        done
    done
done 2>&1 | tee gpurun_out/r4_e2e_hostload_ab.txt
unset RG_AEAD_LIB
timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/e2etrace8 -o run -- python3 tools/e2e_probe.py cfg2 8 > gpurun_out/e2etrace8.log 2>&1
