"""bench.py's launch logic (CPU): a plain `python bench.py --gpus N` must
start its own N ranks (torch.distributed.run on 127.0.0.1) before anything
touches the GPU, forward their exit status, and never re-exec itself; a rank
started by torch.distributed.run (WORLD_SIZE set) runs the benchmark."""
import importlib.util
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def bench():
    spec = importlib.util.spec_from_file_location("bench_under_test", os.path.join(REPO, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_self_launch_command(bench, monkeypatch):
    # a stale rank identity in the caller's environment must not reach the
    # children; an IPC mode the caller chose is kept
    for k, v in (("RANK", "5"), ("LOCAL_RANK", "5"), ("WORLD_SIZE", "7"), ("MASTER_PORT", "1")):
        monkeypatch.setenv(k, v)
    monkeypatch.delenv("HSA_ENABLE_IPC_MODE_LEGACY", raising=False)
    argv = ["--gpus", "8", "--steps", "20", "--warmup", "5"]
    cmd, env = bench.self_launch_command(argv, 8, 29123)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nnodes=1" in cmd and "--nproc-per-node=8" in cmd
    assert "--master-addr=127.0.0.1" in cmd and "--master-port=29123" in cmd
    script = cmd.index(os.path.join(REPO, "bench.py"))
    assert cmd[script + 1:] == argv  # the same arguments reach every rank
    assert env["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_PORT"):
        assert k not in env, k
    monkeypatch.setenv("HSA_ENABLE_IPC_MODE_LEGACY", "1")
    assert bench.self_launch_command(argv, 8, 29123)[1]["HSA_ENABLE_IPC_MODE_LEGACY"] == "1"


def test_dist_flag_self_launches_one_rank(bench, monkeypatch):
    """`--gpus 1 --dist` without a launcher starts one torch.distributed.run
    rank (the multi-rank path at N = 1: RCCL group, gather, de-interleave)."""
    calls = []

    class Done:
        returncode = 0

    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(bench.subprocess, "run", lambda cmd, env=None, **kw: calls.append(cmd) or Done())
    monkeypatch.setattr(bench.torch.cuda, "set_device", lambda *a: pytest.fail("launcher touched the GPU"))
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "1", "--dist", "--steps", "3"])
    with pytest.raises(SystemExit) as e:
        bench.main()
    assert e.value.code == 0 and len(calls) == 1
    assert "--nproc-per-node=1" in calls[0] and calls[0][-5:] == ["--gpus", "1", "--dist", "--steps", "3"]


@pytest.mark.parametrize("rc", [0, 3])
def test_plain_launch_spawns_ranks_and_forwards_status(bench, monkeypatch, rc):
    calls = []

    class Done:
        returncode = rc

    def fake_run(cmd, env=None, **kw):
        calls.append((cmd, env))
        return Done()

    def no_gpu(*a, **k):
        raise AssertionError("the launcher process must not touch the GPU")

    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(bench.subprocess, "run", fake_run)
    monkeypatch.setattr(bench.torch.cuda, "set_device", no_gpu)
    monkeypatch.setattr(bench.os, "execv", no_gpu)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "2", "--steps", "3"])
    with pytest.raises(SystemExit) as e:
        bench.main()
    assert e.value.code == rc
    assert len(calls) == 1
    cmd, env = calls[0]
    assert "--nproc-per-node=2" in cmd and cmd[-4:] == ["--gpus", "2", "--steps", "3"]


def test_rank_under_torchrun_does_not_relaunch(bench, monkeypatch):
    """WORLD_SIZE set (a torch.distributed.run rank): no child launch; a
    mismatch with --gpus is an error, not a relaunch."""
    monkeypatch.setenv("WORLD_SIZE", "4")
    monkeypatch.setattr(bench.subprocess, "run", lambda *a, **k: pytest.fail("relaunched"))
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "2"])
    with pytest.raises(SystemExit) as e:
        bench.main()
    assert "WORLD_SIZE=4" in str(e.value.code)


def test_traffic_record_is_per_workload(bench, tmp_path):
    """The PMC record (tools/make_traffic_json.py) is looked up per config
    (profiles/traffic_<config>.json, then traffic_latest.json) and used only
    when its workload key is this run's."""
    import json
    a, b = tmp_path / "traffic_c5.json", tmp_path / "traffic_latest.json"
    a.write_text(json.dumps({"workload": "stress-1920x1080-32spp-8b-rows1", "l1": {"tag_accesses_per_launch": 1}}))
    b.write_text(json.dumps({"workload": "07-1920x1080-8spp-4b-rows1"}))
    assert bench.load_traffic([str(a), str(b)], "stress-1920x1080-32spp-8b-rows1")["l1"]
    assert bench.load_traffic([str(a), str(b)], "07-1920x1080-8spp-4b-rows1") == {"workload": "07-1920x1080-8spp-4b-rows1"}
    assert bench.load_traffic([str(a), str(b)], "07-1920x1080-8spp-4b-rows2") is None
    assert bench.load_traffic([str(tmp_path / "missing.json")], "x") is None
    paths = bench.traffic_paths(None, "c5")
    assert paths[0].endswith("profiles/traffic_c5.json") and paths[1].endswith("profiles/traffic_latest.json")
    assert bench.traffic_paths("/x.json", "c5") == ["/x.json"]
    # the L1 line peak: 256 CUs at the micro-benchmark's one L1-hit line per cycle
    assert 0.95 < bench.L1_HIT_CYCLES_PER_LINE < 1.05 and bench.L1_MISS_CYCLES_PER_LINE > 2


def test_oracle_check_leg(bench, bwrt_lib):
    """The bench's oracle check (CPU-baseline leg, checker only) on config 1:
    the renderer it is handed (here the product's CPU backend, on the GPU box
    the GPU context) against the oracle, RGBA8 + frameSum + RNG; config 5 is
    not checked there (the oracle's brute-force loop is minutes per row)."""
    from bwrt import Renderer
    with Renderer.cpu(2, lib=bwrt_lib) as r:
        oc = bench.oracle_check("c1", "01", 256, 256, 1, 1, r)
    assert oc["bit_exact"] is True and oc["rows"] == 256 and oc["row_stride"] == 1
    assert bench.oracle_check("c5", "stress", 1920, 1080, 32, 8, None) is None
    assert set(bench.ORACLE_ROW_STRIDE) == {"c1", "c2", "c3", "c4"}


def test_cpu_baseline_leg_repeats_sample(bench, bwrt_lib, monkeypatch):
    """The CPU-baseline leg renders its sample again from the same seeds
    (at least CPU_MIN_REPS times) and reports the median rep; handed a
    renderer (here the CPU backend standing in for the GPU context) it
    compares that renderer's frame with the sample, bit for bit."""
    from bwrt import Renderer
    monkeypatch.setattr(bench, "CPU_MIN_S", 0.0)
    with Renderer.cpu(2, lib=bwrt_lib) as other:
        other.set_scene(bench.scenes.SCENES["01"]())
        out = bench.cpu_baseline(bwrt_lib, "c1", "01", 256, 256, 1, 1, 2, gpu_renderer=other)
    assert out["reps"] == bench.CPU_MIN_REPS and out["cores"] == 2 and out["kind"] == "port"
    lo, hi = out["ms_per_sample_min_max"]
    assert lo <= out["ms_per_sample"] <= hi
    assert out["bit_exact_vs_gpu"] is True and out["ms_per_frame"] == out["ms_per_sample"]
