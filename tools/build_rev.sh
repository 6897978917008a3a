#!/bin/bash
# Builds the library of a committed revision into tools/build/librg_<name>.so, for an interleaved A/B of
# the working tree ("base" in tools/ab.sh) against it (load it with RG_AEAD_LIB=...).
#   usage: tools/build_rev.sh NAME [REV]     (REV defaults to HEAD)
set -eu
cd "$(dirname "$0")/.."
name=$1
rev=${2:-HEAD}
src=$(mktemp -d /tmp/rg_rev.XXXXXX)
git archive "$rev" rustyguard_amd/csrc include rustyguard_amd/build.py | tar -x -C "$src"
# that revision's per-file scheduler flags (rustyguard_amd/build.py FILE_FLAGS, round 5 on)
sched=()
grep -q "iterative-ilp" "$src/rustyguard_amd/build.py" && sched=(-mllvm -amdgpu-sched-strategy=iterative-ilp)
mkdir -p tools/build
objs=()
for s in rg_kernels.hip rg_tile.hip rg_pipe.hip rg_flat.hip rg_mac.hip rg_api.cpp; do
    x=()
    [[ $s == *.cpp ]] && x=(-x hip)
    [[ $s == rg_pipe.hip || $s == rg_flat.hip ]] && x+=("${sched[@]}")
    /opt/rocm/bin/hipcc "${x[@]}" --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -I "$src/include" \
        -c "$src/rustyguard_amd/csrc/$s" -o "$src/$s.o" &
    objs+=("$src/$s.o")
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o tools/build/librg_$name.so "${objs[@]}"
rm -rf "$src"
echo tools/build/librg_$name.so
