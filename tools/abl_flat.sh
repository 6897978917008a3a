#!/bin/bash
# flat-kernel phase stamps under diagnostic ablation builds (tools/build/librg_<name>.so)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for v in base ${ABL:-nostore noload nopoly nomem}; do
    if [ $v = base ]; then L=""; else L="RG_AEAD_LIB=tools/build/librg_$v.so"; fi
    echo "== $v"
    env $L timeout -k 10 120 python tools/flat_stamps.py --workload ${W:-cfg3} --plan 1 | grep '^seal' || exit 1
done
