"""Build librg_aead.so (HIP kernels + C ABI) in-tree for gfx950.

``python -m rustyguard_amd.build`` or ``__graft_entry__.build()``.  The .so is
git-ignored but travels to the GPU box with the gpurun snapshot.
"""
from __future__ import annotations

import os
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
LIBDIR = os.path.join(PKG, "lib")
LIB = os.path.join(LIBDIR, "librg_aead.so")
SOURCES = ["rg_kernels.hip", "rg_tile.hip", "rg_pipe.hip", "rg_flat.hip", "rg_mac.hip", "rg_api.cpp"]
HEADERS = ["rg_device.h", "rg_internal.h"]
ARCH = os.environ.get("RG_OFFLOAD_ARCH", "gfx950")


def _inputs():
    return [os.path.join(CSRC, f) for f in SOURCES + HEADERS] + [os.path.join(REPO, "include", "rg_aead.h")]


def up_to_date() -> bool:
    if not os.path.exists(LIB):
        return False
    t = os.path.getmtime(LIB)
    return all(os.path.getmtime(p) <= t for p in _inputs())


def build(force: bool = False, verbose: bool = False) -> str:
    if not force and up_to_date():
        return LIB
    os.makedirs(LIBDIR, exist_ok=True)
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    objs = []
    for src in SOURCES:
        obj = os.path.join(LIBDIR, src + ".o")
        cmd = [hipcc, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-Wall",
               "-I", os.path.join(REPO, "include"), "-c", os.path.join(CSRC, src), "-o", obj]
        if src.endswith(".cpp"):
            cmd[1:1] = ["-x", "hip"]
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)
        objs.append(obj)
    tmp = LIB + ".tmp"
    subprocess.run([hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp] + objs, check=True)
    os.replace(tmp, LIB)
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
