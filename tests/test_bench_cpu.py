"""bench.py's launch contract, checked on CPU (no GPU work: --dry-run stops before it).

`python bench.py --gpus N` must start N ranks itself and report N (not silently one), a
WORLD_SIZE that disagrees with --gpus must fail, and N > 1 defaults to BASELINE config 5's
strong split.
"""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env_extra=None, timeout=240):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(REPO, "bench.py")] + args, env=env, cwd=REPO,
                          capture_output=True, text=True, timeout=timeout)


def test_gpus_n_launches_n_ranks():
    r = _run(["--gpus", "2", "--dry-run"])
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert sorted(x["rank"] for x in lines) == [0, 1]
    assert all(x["world"] == 2 and x["gpus"] == 2 and x["workload"] == "cfg5" for x in lines)
    assert sorted(x["local_rank"] for x in lines) == [0, 1]
    # the N > 1 line is self-contained: rank 0 also runs the same workload's 1-GPU base and the CPU baselines
    legs = {x["rank"]: x["legs"] for x in lines}
    assert legs[0] == ["timed", "base_1gpu", "single_process", "e2e_multi", "cpu_baseline"] and legs[1] == ["timed"]


def test_single_gpu_defaults_to_cfg2():
    r = _run(["--dry-run"])
    assert r.returncode == 0, r.stderr[-2000:]
    (line,) = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    # the default line also times the open with 1 % and 10 % forged tags (forged_open)
    assert line == {"rank": 0, "world": 1, "gpus": 1, "local_rank": 0, "workload": "cfg2", "forged": [0.01, 0.1]}
    r = _run(["--dry-run", "--forged", "0"])
    (line,) = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert line["forged"] == []
    r = _run(["--dry-run", "--forged", "1.5"])
    assert r.returncode != 0


def test_world_size_mismatch_is_an_error():
    r = _run(["--gpus", "4", "--dry-run"], {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode == 2
    assert "WORLD_SIZE=2" in r.stderr
    r = _run(["--gpus", "1", "--dry-run"], {"WORLD_SIZE": "8", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode == 2


def test_pcie_ceiling_reads_the_duplex_tool(monkeypatch):
    """`e2e.pcie_ceiling` takes tools/build/pcie's figures (run as a child process): the in-process copies on
    two torch streams ran the directions one after the other (28.5 GB/s per direction against 47.7)."""
    import importlib.util

    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(REPO, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    out = {"bytes": 100663296, "piece_bytes": 16777216,
           "gb_s_per_direction": {"h2d_copy": 56.8, "d2h_copy": 56.4, "both_copies": 47.7,
                                  "both_copies_16MiB_pieces": 46.7}}
    seen = {}

    def fake_run(cmd, **kw):
        seen["cmd"] = cmd
        return subprocess.CompletedProcess(cmd, 0, stdout="noise\n" + json.dumps(out) + "\n", stderr="")

    monkeypatch.setattr(os.path, "exists", lambda p: True)
    monkeypatch.setattr(subprocess, "run", fake_run)
    got = bench.pcie_ceiling(96 << 20)
    assert seen["cmd"][0].endswith(os.path.join("tools", "build", "pcie")) and seen["cmd"][1] == "96"
    assert got["h2d_gb_s"] == 56.8 and got["d2h_gb_s"] == 56.4 and got["bidir_gb_s_per_dir"] == 47.7
    assert got["bidir_16MiB_pieces_gb_s_per_dir"] == 46.7 and "lower_bound" not in got


def _bench_module():
    import importlib.util

    spec = importlib.util.spec_from_file_location("bench_mod_r", os.path.join(REPO, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    return bench


def test_roofline_reports_the_valu_bound():
    """the line names the bound the counters show (VALU issue, not HBM): roofline.bound is
    "valu", the contract's achieved / peak / frac / traffic stay the dominant kernel's HBM figures beside it,
    and roofline.valu carries the VALU-ceiling fraction at the microbenchmark clock and at the kernel's own,
    the latter labelled as an assumed (recorded, not measured) clock."""
    import numpy as np

    bench = _bench_module()
    lens = np.full(65536, 1504, np.uint32)
    ceil = bench.valu_ceiling_gbs(lens, False)
    roof, valu = bench.rooflines("seal", 2588.95, 199229440, 200972678, 1280.85, ceil, bench.KERNEL_CLOCK_GHZ["cfg2"])
    assert roof["bound"] == "valu"
    assert roof["unit"] == "GB/s" and roof["peak"] == bench.HBM_PEAK_GBS == 8000.0
    assert abs(roof["frac"] - 2588.95 / 8000.0) < 1e-4 and roof["traffic"] == 200972678
    assert abs(valu["frac"] - 1280.85 / ceil) < 1e-4 and 0.55 < valu["frac"] < 0.65
    assert valu["clock_assumed"] is True and valu["frac_at_kernel_clock"] > valu["frac"]
    assert roof["valu"]["frac"] == valu["frac"] and roof["valu"]["frac_at_kernel_clock"] == valu["frac_at_kernel_clock"]
    # no recorded clock for a workload: no kernel-clock fraction, and nothing claims one
    _, v2 = bench.rooflines("open", 1.0, 1, None, 1.0, ceil, None)
    assert "frac_at_kernel_clock" not in v2 and "clock_assumed" not in v2


def test_cpu_baseline_harness_reports_scaling_and_limits():
    """the CPU baselines run on a persistent pool (threads and OpenSSL contexts kept
    across rounds) over a >= 64 Ki-packet sample of the workload; each line names its thread count, the
    limits it came from (affinity, cgroup cpu.max, OMP_NUM_THREADS) and its scaling efficiency
    (N-thread / (N x 1-thread)).  Run here on a small workload with a short budget."""
    from rustyguard_amd import workloads

    bench = _bench_module()
    assert bench.CPU_SAMPLE >= 65536
    threads, limits = bench.all_core_threads(0)
    assert threads >= 1 and "affinity" in limits
    assert bench.all_core_threads(3)[0] == 3
    w = workloads.uniform(1024, 1500, name="t")
    port, ossl = bench.cpu_baselines(w, 1.2, (2, {"requested": 2}))
    for d in (port, ossl):
        if d is None:
            continue
        assert d["cores"] == 2 and d["n_sample"] == 1024 and d["value"] > 0 and d["one_thread"]["value"] > 0
        sc = d["scaling"]
        assert sc["threads"] == 2 and 0 < sc["efficiency"] and sc["thread_limits"] == {"requested": 2}
        assert abs(sc["speedup"] - d["value"] / d["one_thread"]["value"]) < 0.02
        assert "persistent pool" in d["sample"] and sc["placement"] in d["sample"]
        if sc["efficiency"] < 0.9:
            assert sc["limit"]  # the line says what stops the scaling


def test_pick_cpus_one_per_core_on_one_node():
    """The pinned baseline's CPUs: distinct, inside the affinity mask, at most one per physical core."""
    bench = _bench_module()
    aff = sorted(os.sched_getaffinity(0))
    cpus = bench.pick_cpus(2)
    if cpus is None:
        pytest.skip("the affinity mask has fewer than two cores on one node")
    assert len(cpus) == len(set(cpus)) == 2 and set(cpus) <= set(aff)
    assert bench.pick_cpus(len(aff) + 1) is None
    assert bench._cpulist("0-2,5,7-8") == [0, 1, 2, 5, 7, 8]


def test_private_slices_must_not_overlap():
    """rg_cpu_bench's private copies are written back whole, so slices whose frame spans overlap are
    refused (-4) instead of being corrupted."""
    from oracle import oracle
    from rustyguard_amd import workloads

    w = workloads.uniform(64, 64, name="t")
    desc = w.desc.copy()
    desc["offset"] = desc["offset"][::-1].copy()  # frames in reverse: the second worker's span lies below the first's
    buf = np.zeros(int(w.buf_bytes), np.uint8)
    with pytest.raises(RuntimeError, match="failed: -4"):
        oracle.cpu_bench("port", 2, w.keys, w.receivers, desc, w.counters, buf, 0.05, local=True)


def test_cgroup_quota_parser(monkeypatch, tmp_path):
    bench = _bench_module()
    real_open = open

    def fake_open(path, *a, **k):
        if path == "/sys/fs/cgroup/cpu.max":
            p = tmp_path / "cpu.max"
            p.write_text("1600000 100000\n")
            return real_open(p, *a, **k)
        return real_open(path, *a, **k)

    monkeypatch.setattr("builtins.open", fake_open)
    assert bench.cgroup_cpu_quota() == 16.0
