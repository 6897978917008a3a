#!/bin/bash
# Builds an experimental librg_aead.so with extra compile flags into
# tools/build/librg_<name>.so (load it with RG_AEAD_LIB=...).
#   usage: tools/build_variant.sh NAME [-DFLAG ...]
set -eu
cd "$(dirname "$0")/.."
name=$1
shift
out=tools/build/var_$name
mkdir -p "$out"
objs=()
for src in rg_kernels.hip rg_tile.hip rg_pipe.hip rg_flat.hip rg_mac.hip rg_api.cpp; do
    x=()
    [[ $src == *.cpp ]] && x=(-x hip)
    /opt/rocm/bin/hipcc "${x[@]}" --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall "$@" -I include \
        -c rustyguard_amd/csrc/$src -o "$out/$src.o" &
    objs+=("$out/$src.o")
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o tools/build/librg_$name.so "${objs[@]}"
rm -rf "$out"
echo tools/build/librg_$name.so
