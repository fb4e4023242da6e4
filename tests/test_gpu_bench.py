"""The benchmark's multi-rank path on the GPU box: a plain
`python bench.py --gpus 2` starts its own two ranks (torch.distributed.run on
127.0.0.1), each renders its interleaved-row shard of config 3, the shards
are gathered and de-interleaved on rank 0, and the gathered frame is checked
bit for bit against rank 0 rendering the whole frame alone.  With one GPU on
the box both ranks share it over gloo (BWRT_DIST_BACKEND=gloo); on an 8-GPU
node the same path runs one rank per GPU over RCCL."""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.gpu
@pytest.mark.timeout(300)
def test_bench_plain_launch_two_ranks_verified():
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")}
    env.update(BWRT_DIST_BACKEND="gloo", HSA_ENABLE_IPC_MODE_LEGACY="0")
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--steps", "3", "--warmup", "1"],
                       env=env, cwd=REPO, capture_output=True, text=True, timeout=280)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]  # rank 0 prints the one JSON line
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["world_size"] == 2 and out["backend"] == "gloo"
    assert out["verified"] is True, out.get("verify")
    assert out["value"] > 0 and out["config"]["parallelism"].startswith("pixel-rows/2")


@pytest.mark.gpu
@pytest.mark.timeout(300)
def test_bench_rccl_path_one_rank_verified():
    """The RCCL branch every N > 1 point of the headline takes (nccl process
    group with device_id, rooted gather of the row blocks on the gather
    stream, de-interleave kernel, verify against a solo render), run once at
    world size 1 under torch.distributed.run with the default backend."""
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT",
                        "BWRT_DIST_BACKEND")}
    env.update(HSA_ENABLE_IPC_MODE_LEGACY="0")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
                        "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.join(REPO, "bench.py"),
                        "--gpus", "1", "--dist", "--steps", "3", "--warmup", "1"],
                       env=env, cwd=REPO, capture_output=True, text=True, timeout=280)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    out = json.loads(lines[0])
    assert out["backend"] == "rccl" and out["world_size"] == 1 and out["n_gpus"] == 1
    assert out["verified"] is True, out.get("verify")
    assert "rccl gather" in out["config"]["parallelism"]
