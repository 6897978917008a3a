#!/bin/bash
# Builds an experimental librg_aead.so with extra compile flags into
# tools/build/librg_<name>.so (load it with RG_AEAD_LIB=...).
#   usage: tools/build_variant.sh NAME [-DFLAG ...]
#   VAR_ONLY="rg_pipe.hip rg_flat.hip" applies the extra flags to those sources only.
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
    extra=("$@")
    [[ -n "${VAR_ONLY:-}" && " $VAR_ONLY " != *" $src "* ]] && extra=()
    # the product's per-file flags (rustyguard_amd/build.py FILE_FLAGS), before the variant's own
    [[ $src == rg_pipe.hip || $src == rg_flat.hip ]] && extra=(-mllvm -amdgpu-sched-strategy=iterative-ilp "${extra[@]}")
    /opt/rocm/bin/hipcc "${x[@]}" --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall "${extra[@]}" -I include \
        -c rustyguard_amd/csrc/$src -o "$out/$src.o" &
    objs+=("$out/$src.o")
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o tools/build/librg_$name.so "${objs[@]}"
rm -rf "$out"
echo tools/build/librg_$name.so
