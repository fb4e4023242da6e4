"""Multi-GPU frame partition and gather (one process per GPU).

The reference renders on one GPU (Main.cu:342, stream 0).  Pixels are
independent (the RNG seed is the global pixel index, Main.cu:377), so a frame
splits across G ranks by INTERLEAVED rows — rank r renders rows
y = r, r+G, r+2G, ... — which balances cheap sky rows against expensive floor
rows.  Frames (spp) are never split: a pixel's RNG stream is sequential across
frames.  After the render the ranks exchange ONE message: a gather of
equal-size RGBA8 row blocks (padded to ceil(H/G) rows) to rank 0 over
RCCL/xGMI, and rank 0 de-interleaves the blocks into the image (a HIP kernel
on the GPU path).
"""
from __future__ import annotations

from dataclasses import dataclass


@dataclass(frozen=True)
class ShardPlan:
    height: int
    world: int
    rank: int

    @property
    def row_offset(self) -> int:
        return self.rank

    @property
    def row_stride(self) -> int:
        return self.world

    @property
    def rows(self) -> int:
        """Rows this rank renders."""
        return len(range(self.rank, self.height, self.world))

    @property
    def rows_per_shard(self) -> int:
        """Padded block height of every rank in the gather."""
        return -(-self.height // self.world)

    def global_rows(self):
        return list(range(self.rank, self.height, self.world))


def deinterleave_reference(gathered, plan: ShardPlan, width: int):
    """Host (numpy/torch) version of rt_deinterleave_rows_device: gathered
    [world, rows_per_shard, width, ...] -> image [height, width, ...]."""
    import numpy as np
    g = np.asarray(gathered).reshape(plan.world, plan.rows_per_shard, width, -1)
    out = np.empty((plan.height, width, g.shape[-1]), dtype=g.dtype)
    for r in range(plan.world):
        ys = range(r, plan.height, plan.world)
        out[list(ys)] = g[r, :len(ys)]
    return out


def gather_rows(local_block, plan: ShardPlan, out=None, group=None, dst: int = 0):
    """Rooted gather of every rank's padded row block to rank `dst` (torch
    tensors, any backend: RCCL on GPUs, gloo in the CPU tests) into `out`
    ([world, *local_block.shape], allocated on `dst` when None).  Returns
    `out` on `dst` and None elsewhere.

    Only rank 0 needs the image, so this is a gather, not an all_gather: over
    RCCL each peer's block reaches the root on its own xGMI link (grouped
    send/recv), where a ring all_gather would move every block across all
    G - 1 links and keep RCCL kernels busy on every rank while the next frame
    renders."""
    import torch
    import torch.distributed as dist
    root = dist.get_rank(group) == dst if group is not None else dist.get_rank() == dst
    if root and out is None:
        out = torch.empty((plan.world,) + tuple(local_block.shape), dtype=local_block.dtype,
                          device=local_block.device)
    if dist.get_backend(group) == "gloo" and local_block.is_cuda:
        # rehearsal of the GPU path over gloo: stage through the host
        host = torch.empty((plan.world,) + tuple(local_block.shape), dtype=local_block.dtype) if root else None
        dist.gather(local_block.cpu(), gather_list=list(host.unbind(0)) if root else None, dst=dst, group=group)
        if root:
            out.copy_(host)
    else:
        dist.gather(local_block, gather_list=list(out.unbind(0)) if root else None, dst=dst, group=group)
    return out if root else None
