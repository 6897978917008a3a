"""Build librg_aead.so (HIP kernels + C ABI) in-tree for gfx950.

``python -m rustyguard_amd.build`` or ``__graft_entry__.build()``.  The .so files are
git-ignored but travel to the GPU box with the gpurun snapshot.

Two libraries come out of one set of kernel objects:
  lib/librg_aead.so       the product: include/rg_aead.h, no diagnostics, no test hooks
  lib/librg_aead_test.so  the same kernels + rg_api.cpp with -DRG_TEST_HOOKS
                          (include/rg_aead_test.h), loaded only by the GPU tests that
                          check key wiping and allocation failures
Diagnostic builds (-DRG_DIAG: seal modes, per-wave stamps) are tools/build_variant.sh's.
"""
from __future__ import annotations

import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

PKG = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
LIBDIR = os.path.join(PKG, "lib")
LIB = os.path.join(LIBDIR, "librg_aead.so")
TEST_LIB = os.path.join(LIBDIR, "librg_aead_test.so")
KERNELS = ["rg_kernels.hip", "rg_tile.hip", "rg_pipe.hip", "rg_flat.hip", "rg_mac.hip"]
API = "rg_api.cpp"
SOURCES = KERNELS + [API]
HEADERS = ["rg_device.h", "rg_internal.h"]
ARCH = os.environ.get("RG_OFFLOAD_ARCH", "gfx950")
# Per-file code generation.  The pipelined and flattened kernels run one wave per SIMD, so nothing hides a
# hazard wait state: LLVM's iterative-ILP machine scheduler fills most of the s_nops the default strategy
# leaves between a carry-flag write and its read (pipelined seal 604 -> 159, flattened 425 -> 135) and
# needs fewer VGPRs there.  Config 2 +2-3 %, config 3 +0.6-1 % (profiles/r5_sched_ab.txt).  The tile kernel
# keeps the default: at G = 2 the ILP schedule spills (scratch 52 -> 104 bytes) and its open ran 1-2 % slower.
FILE_FLAGS = {
    "rg_pipe.hip": ("-mllvm", "-amdgpu-sched-strategy=iterative-ilp"),
    "rg_flat.hip": ("-mllvm", "-amdgpu-sched-strategy=iterative-ilp"),
}


def _inputs():
    return ([os.path.join(CSRC, f) for f in SOURCES + HEADERS] +
            [os.path.join(REPO, "include", h) for h in ("rg_aead.h", "rg_aead_test.h")] +
            [os.path.abspath(__file__)])  # the flags above


def up_to_date() -> bool:
    if not (os.path.exists(LIB) and os.path.exists(TEST_LIB)):
        return False
    t = min(os.path.getmtime(LIB), os.path.getmtime(TEST_LIB))
    return all(os.path.getmtime(p) <= t for p in _inputs())


def _compile(hipcc: str, src: str, obj: str, defines, verbose: bool):
    cmd = [hipcc, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-Wall", *FILE_FLAGS.get(src, ()), *defines,
           "-I", os.path.join(REPO, "include"), "-c", os.path.join(CSRC, src), "-o", obj]
    if src.endswith(".cpp"):
        cmd[1:1] = ["-x", "hip"]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    return obj


def _link(hipcc: str, out: str, objs):
    tmp = out + ".tmp"
    subprocess.run([hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp] + list(objs), check=True)
    os.replace(tmp, out)


def build(force: bool = False, verbose: bool = False) -> str:
    if not force and up_to_date():
        return LIB
    os.makedirs(LIBDIR, exist_ok=True)
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    jobs = [(src, os.path.join(LIBDIR, src + ".o"), ()) for src in SOURCES]
    jobs.append((API, os.path.join(LIBDIR, "rg_api_test.cpp.o"), ("-DRG_TEST_HOOKS=1",)))
    # the largest kernel files take ~50 s each: compile them side by side
    with ThreadPoolExecutor(max_workers=min(len(jobs), os.cpu_count() or 1)) as ex:
        objs = list(ex.map(lambda j: _compile(hipcc, j[0], j[1], j[2], verbose), jobs))
    kernel_objs = objs[:len(KERNELS)]
    _link(hipcc, LIB, kernel_objs + [objs[len(KERNELS)]])
    _link(hipcc, TEST_LIB, kernel_objs + [objs[-1]])
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
