#!/bin/bash
# round 3: forged-tag open cost with the corrected harness (clean and forged opens both behind a spin kernel),
# default (decrypt + cooperative restore) and verify-then-decrypt (mf) builds; configs 2, 3, 4
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
for lib in base mf; do
  if [ $lib = base ]; then unset RG_AEAD_LIB; else export RG_AEAD_LIB=tools/build/librg_$lib.so; fi
  for w in cfg2 cfg3 cfg4; do
    for f in 0.01 0.1 1.0; do
      timeout -k 10 150 python bench.py --workload $w --steps 5 --warmup 2 --no-cold --cpu-seconds 0 --forged $f > gpurun_out/r3f_${lib}_${w}_$f.log 2>&1 || exit $?
      echo "$lib $w $f $(grep '^{' gpurun_out/r3f_${lib}_${w}_$f.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["open_ms"], d["forged_open"])')"
    done
  done
done
