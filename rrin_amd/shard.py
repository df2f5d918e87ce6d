"""Frame-batch data parallelism: one process per GPU.

Replaces the single-device dispatch of the reference caller
(`/root/reference/convert.py:90-92,110,130`: ``model.cuda()`` and
``model(img1.cuda(), img2.cuda(), t)``).  Frame pairs are independent, so a
global batch of B pairs is split into contiguous shards of B/W pairs; each rank
runs the HIP ``Net`` on its shard and the only exchange is one all-gather that
reassembles the ``[B,3,H,W]`` output sequence in order (RCCL over xGMI with
backend "nccl" on ROCm; gloo in the CPU tests).
"""
from __future__ import annotations

import zlib

import torch
import torch.distributed as dist


def shard_bounds(global_batch: int, rank: int, world: int):
    """Contiguous shard [lo, hi) of rank ``rank``; B must divide evenly so the
    all-gather moves equal-size messages."""
    if global_batch % world:
        raise ValueError(f"global batch {global_batch} is not divisible by world size {world}")
    per = global_batch // world
    return rank * per, (rank + 1) * per


def gather_frames(local: torch.Tensor, group=None, out: torch.Tensor | None = None, async_op: bool = False):
    """All-gather equal shards ``local`` [b,...] into ``[world*b, ...]`` (rank order).
    ``async_op=True`` returns ``(out, work)``: on RCCL the gather runs on the
    communicator's stream and ``work.wait()`` orders the caller's stream after
    it; gloo (CPU tests / single-GPU rehearsal) completes before returning."""
    work = None
    if not (dist.is_available() and dist.is_initialized()):  # single process, no group: identity
        out = local if out is None else out.copy_(local)
        return (out, work) if async_op else out
    world = dist.get_world_size(group)   # world 1 still goes through the backend (RCCL rehearsal)
    local = local.contiguous()
    if out is None:
        out = torch.empty((world * local.shape[0],) + tuple(local.shape[1:]),
                          dtype=local.dtype, device=local.device)
    if dist.get_backend(group) == "gloo":
        # gather through host memory
        host = local.cpu()
        parts = [torch.empty_like(host) for _ in range(world)]
        dist.all_gather(parts, host, group=group)
        out.copy_(torch.cat(parts))
    else:
        work = dist.all_gather_into_tensor(out, local, group=group, async_op=async_op)
    return (out, work) if async_op else out


class GatherPipeline:
    """Overlap the all-gather of step k with the compute of step k+1 (SURVEY
    §8e: the gather is issued on a side stream while the next batch computes).
    ``depth`` output buffers are cycled; a buffer's previous gather is waited
    for before it is reused, and ``drain()`` waits for every gather in flight."""

    def __init__(self, shape, dtype, device, group=None, depth: int = 2):
        self.group = group
        self.bufs = [torch.empty(shape, dtype=dtype, device=device) for _ in range(depth)]
        self.inflight = [None] * depth  # (work, local) per buffer
        self.k = 0

    def submit(self, local: torch.Tensor):
        """Issue the gather of ``local``; returns ``(out, work)``.  ``out`` is only
        valid after ``work.wait()`` (RCCL: orders the caller's stream after the
        gather) or ``drain()``; ``work`` is None when the gather already completed
        (gloo, one rank)."""
        i = self.k % len(self.bufs)
        self.k += 1
        if self.inflight[i] is not None:
            work, _ = self.inflight[i]
            if work is not None:
                work.wait()
        out, work = gather_frames(local, group=self.group, out=self.bufs[i], async_op=True)
        self.inflight[i] = (work, local)  # keep the shard alive until its gather is done
        return out, work

    def drain(self):
        for i, f in enumerate(self.inflight):
            if f is not None and f[0] is not None:
                f[0].wait()
            self.inflight[i] = None


def _crc(t: torch.Tensor) -> int:
    return zlib.crc32(t.detach().contiguous().cpu().view(torch.uint8).numpy().tobytes()) & 0xFFFFFFFF


def verify_gather(local: torch.Tensor, gathered: torch.Tensor, group=None) -> dict:
    """Bitwise check of one all-gather: every rank's shard ``local`` [b,...] is the
    rank-order slice of ``gathered`` [world*b,...] -- on every rank, its own slice
    by exact equality, and every slice's CRC-32 against the CRC its owner computed
    of its shard (exchanged with ``all_gather_object``).  The verdict is reduced
    over the ranks, so every rank returns the same ``ok``."""
    inited = dist.is_available() and dist.is_initialized()
    world = dist.get_world_size(group) if inited else 1
    rank = dist.get_rank(group) if inited else 0
    b = local.shape[0]
    own = bool(torch.equal(gathered[rank * b:(rank + 1) * b], local))
    mine = _crc(local)
    crcs = [mine]
    if inited:
        crcs = [None] * world
        dist.all_gather_object(crcs, mine, group=group)
    seen = [_crc(gathered[r * b:(r + 1) * b]) for r in range(world)]
    ok = own and seen == crcs
    if inited:
        flag = torch.tensor([1 if ok else 0], dtype=torch.int32,
                            device=gathered.device if dist.get_backend(group) != "gloo" else "cpu")
        dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=group)
        ok = bool(flag.item())
    return {"ok": ok, "shard_crc32": [f"{c:08x}" for c in crcs],
            "what": "bitwise: each rank's own slice of the gathered output == its shard (torch.equal), and "
                    "the CRC-32 of every slice == the CRC-32 its owner computed of its shard; reduced over ranks"}


def interpolate_sharded(net, i0_local: torch.Tensor, i1_local: torch.Tensor, t=0.5, group=None,
                        out: torch.Tensor | None = None) -> torch.Tensor:
    """Run ``net`` on this rank's pairs and return the whole gathered batch."""
    with torch.no_grad():
        local = net(i0_local, i1_local, t)
    return gather_frames(local, group=group, out=out)
