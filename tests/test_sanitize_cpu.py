"""The library's host logic under AddressSanitizer + UBSan and ThreadSanitizer, on the CPU.

rg_api.cpp is compiled host-only (hipcc --cuda-host-only, the sanitizer flags after -Xarch_host) and linked
against tests/sanitize/hip_stub.cpp -- a CPU stand-in for the HIP runtime calls it makes and for the kernel
launchers, with the kernels' descriptor checks and status rules around a fake cipher -- and driven by
tests/sanitize/driver.cpp: the host slice pipeline with descriptors out of offset order, the session layer's
replay pass and side effects, a four-context group whose batches start one worker thread per context, the
device-frame session calls, the fail-closed paths (a lost planner hand-off, lost completions against the
bounded waits) and the per-message drop-in.  Each build runs the whole driver; any sanitizer report or a
failed functional check fails the test.  (GPU-side sanitizers are not available on the GPU pool.)"""
import os
import shutil
import subprocess

import pytest

from conftest import REPO

HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
CLANG = "/opt/rocm/lib/llvm/bin/clang++"
SAN = os.path.join(REPO, "tests", "sanitize")
FLAGS = {"asan": ["-fsanitize=address,undefined", "-fno-sanitize-recover=undefined"], "tsan": ["-fsanitize=thread"]}

pytestmark = pytest.mark.skipif(not (os.path.exists(HIPCC) and os.path.exists(CLANG)), reason="no ROCm clang")


def _build(kind, out):
    f = FLAGS[kind]
    inc = ["-I", os.path.join(REPO, "include")]
    host = [HIPCC, "-x", "hip", "--cuda-host-only", "-O1", "-g", "-std=c++17", "-fno-omit-frame-pointer", "-w"]
    for fl in f:
        host += ["-Xarch_host", fl]
    objs = []
    jobs = [(host + ["-DRG_TEST_HOOKS=1"] + inc, os.path.join(REPO, "rustyguard_amd", "csrc", "rg_api.cpp")),
            (host + inc, os.path.join(SAN, "hip_stub.cpp")),
            ([CLANG, "-O1", "-g", "-std=c++17", "-fno-omit-frame-pointer"] + f + inc, os.path.join(SAN, "driver.cpp"))]
    procs = []
    for cmd, src in jobs:
        o = os.path.join(out, os.path.basename(src) + f".{kind}.o")
        procs.append(subprocess.Popen(cmd + ["-c", src, "-o", o], stdout=subprocess.PIPE, stderr=subprocess.STDOUT))
        objs.append(o)
    for p in procs:
        log = p.communicate(timeout=600)[0].decode(errors="replace")
        assert p.returncode == 0, log[-3000:]
    exe = os.path.join(out, f"driver_{kind}")
    subprocess.run([CLANG] + f + ["-o", exe] + objs + ["-lpthread"], check=True, timeout=300)
    return exe


@pytest.mark.parametrize("kind", ["asan", "tsan"])
def test_host_logic_under_sanitizer(kind, tmp_path):
    exe = _build(kind, str(tmp_path))
    env = dict(os.environ, RG_STUB_DEVICES="2", ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:halt_on_error=1",
               TSAN_OPTIONS="halt_on_error=1 second_deadlock_stack=1")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=600, env=env)
    out = r.stdout + r.stderr
    assert "Sanitizer" not in out and "runtime error" not in out, out[-6000:]
    assert r.returncode == 0 and "all scenarios passed" in r.stdout, out[-6000:]
    shutil.rmtree(tmp_path, ignore_errors=True)
