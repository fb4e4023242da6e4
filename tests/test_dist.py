"""Multi-rank path on CPU (world_size 2, 3 and 8, gloo): the interleaved-row
shard plan, the padded gather of RGBA8 row blocks to rank 0 and the
de-interleave that bench.py runs over RCCL.  Every rank renders its rows
with the product — libbwrt.so's CPU backend (rt_create_cpu / rt_render_cpu,
the kernels' per-ray arithmetic compiled for the host) with the rank's
row_offset / row_stride — and the gathered frame must equal one CPU context
rendering the whole frame and the oracle's frame; the GPU tests check that
libbwrt's device shards equal the full image row for row."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from bwrt.dist import ShardPlan, deinterleave_reference, gather_rows


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, w, h, spp, mb, q):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path[:0] = [os.path.join(os.path.dirname(here), "bwidman-raytracer_amd")]
    from bwrt import Renderer, scenes
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    plan = ShardPlan(h, world, rank)
    with Renderer.cpu(1) as c:  # the product's CPU backend, this rank's rows
        c.set_scene(scenes.scene_07())
        c.init_rand(w, h, plan.row_offset, plan.row_stride)
        rgba = c.render(w, h, spp, mb, first_frame=1, row_offset=plan.row_offset, row_stride=plan.row_stride)
    assert rgba.shape == (plan.rows, w, 4)
    block = np.zeros((plan.rows_per_shard, w), dtype=np.uint32)
    block[:plan.rows] = np.ascontiguousarray(rgba).view(np.uint32).reshape(plan.rows, w)
    gathered = gather_rows(torch.from_numpy(block.view(np.int32)).reshape(-1), plan)
    assert (gathered is None) == (rank != 0)
    if rank == 0:
        img = deinterleave_reference(gathered.numpy().view(np.uint32), plan, w)
        q.put(img.view(np.uint8).reshape(h, w, 4))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("h,world", [(54, 2), (55, 2), (55, 3), (30, 8)])
def test_multi_rank_gather_matches_single_render(oracle, h, world):
    w, spp, mb = 96, 2, 4
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, w, h, spp, mb, q)) for r in range(world)]
    for p in procs:
        p.start()
    img = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    from bwrt import Renderer, scenes
    with Renderer.cpu(2) as c:  # one context, the whole frame
        c.set_scene(scenes.scene_07())
        c.init_rand(w, h)
        single = c.render(w, h, spp, mb, first_frame=1)
    assert np.array_equal(img, single)
    full = oracle.render_image(scenes.scene_07(), w, h, spp, mb).rgba
    assert np.array_equal(img, full)


@pytest.mark.parametrize("h,world", [(1080, 8), (1080, 3), (7, 8), (2160, 8)])
def test_shard_plan_covers_every_row_once(h, world):
    rows = []
    for r in range(world):
        p = ShardPlan(h, world, r)
        assert p.rows <= p.rows_per_shard
        rows += p.global_rows()
    assert sorted(rows) == list(range(h))


def test_deinterleave_reference_layout():
    h, w, world = 10, 3, 4
    plan = ShardPlan(h, world, 0)
    g = np.full((world, plan.rows_per_shard, w, 1), -1, dtype=np.int32)
    for r in range(world):
        for j, y in enumerate(range(r, h, world)):
            g[r, j] = y
    img = deinterleave_reference(g, plan, w)
    assert (img[..., 0] == np.arange(h)[:, None]).all()
