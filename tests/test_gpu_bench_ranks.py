"""The N > 1 bench path exactly as the driver launches it: `python -m
torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 ... bench.py --gpus 2`, one rank per GPU.
A one-GPU box cannot run RCCL with two ranks on one device, so both ranks share device 0 with the
bookkeeping collectives over gloo (RG_BENCH_SHARE_GPU=1); everything else -- the WORLD_SIZE check, the
per-rank engines and graphs, the barrier and the MAX reduction of the elapsed time, rank 0's JSON line --
is the driver's path.  Config 2 on every rank keeps it short (the config-5 split and its base_1gpu leg run
in the bench rehearsals, profiles/r4_rehearse_torchrun2.jsonl)."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_torchrun_two_ranks_sharing_one_gpu():
    env = dict(os.environ, RG_BENCH_SHARE_GPU="1", HSA_ENABLE_IPC_MODE_LEGACY="0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py", "--gpus", "2",
           "--workload", "cfg2", "--steps", "3", "--warmup", "1", "--cpu-seconds", "0", "--forged", "0", "--no-cold"]
    p = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [json.loads(x) for x in p.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]  # rank 0 alone prints
    d = lines[0]
    assert d["n_gpus"] == 2 and d["steps"] == 3 and d["value"] > 0
    assert "rehearsal" in d and d["config"]["packets_per_gpu"] == 65536
