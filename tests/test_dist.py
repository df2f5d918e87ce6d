"""CPU, world_size 2 over gloo: frame-batch sharding + all-gather reassembly
(rrin_amd.shard) returns the same output sequence as an unsharded run.  The
per-pair model here is the CPU oracle (the HIP kernels need a GPU); the code
under test is the sharding / gather plumbing that bench.py uses with RCCL."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from rrin_amd.shard import gather_frames, shard_bounds


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class _OracleNet:
    def __init__(self, sd):
        self.sd = sd

    def __call__(self, i0, i1, t=0.5):
        from oracle.ref_net import net_forward
        return net_forward(self.sd, i0, i1, t)


def _worker(rank, world, port, result_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(2)
    from rrin_amd import Net
    from rrin_amd.shard import interpolate_sharded
    from rrin_amd.synthetic import keyed_state_dict, synthetic_batch
    sd = keyed_state_dict(Net().state_dict(), stress=True)
    B, H, W = 4, 32, 48
    lo, hi = shard_bounds(B, rank, world)
    i0, i1 = synthetic_batch(hi - lo, H, W, first_index=lo)   # each rank makes only its pairs
    out = interpolate_sharded(_OracleNet(sd), i0, i1, 0.5)
    if rank == 0:
        torch.save(out, result_path)
    dist.barrier()
    dist.destroy_process_group()


def test_shard_bounds():
    assert [shard_bounds(8, r, 4) for r in range(4)] == [(0, 2), (2, 4), (4, 6), (6, 8)]
    with pytest.raises(ValueError):
        shard_bounds(6, 0, 4)


def test_gather_single_process_is_identity():
    port = _free_port()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=0, world_size=1)
    try:
        x = torch.randn(2, 3, 4, 4)
        assert torch.equal(gather_frames(x), x)
    finally:
        dist.destroy_process_group()


def test_sharded_equals_unsharded(tmp_path):
    from oracle.ref_net import net_forward
    from rrin_amd import Net
    from rrin_amd.synthetic import keyed_state_dict, synthetic_batch
    world = 2
    path = str(tmp_path / "out.pt")
    mp.start_processes(_worker, args=(world, _free_port(), path), nprocs=world, join=True,
                       start_method="spawn")
    got = torch.load(path, weights_only=True)
    sd = keyed_state_dict(Net().state_dict(), stress=True)
    i0, i1 = synthetic_batch(4, 32, 48, first_index=0)
    with torch.no_grad():
        ref = net_forward(sd, i0, i1, 0.5)
    assert got.shape == (4, 3, 32, 48)
    assert torch.allclose(got, ref, atol=1e-6, rtol=0)


def _pipeline_worker(rank, world, port, result_path):
    """GatherPipeline: three steps through two cycled buffers; every gather
    returns the rank-ordered concatenation of that step's shards."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from rrin_amd.shard import GatherPipeline
    pipe = GatherPipeline((world * 2, 3, 4, 5), torch.float32, "cpu")
    outs = []
    for k in range(3):
        local = torch.full((2, 3, 4, 5), float(10 * k + rank))
        out, work = pipe.submit(local)
        if work is not None:
            work.wait()
        outs.append(out.clone())
    pipe.drain()
    if rank == 0:
        torch.save(torch.stack(outs), result_path)
    dist.barrier()
    dist.destroy_process_group()


def test_gather_pipeline_gloo(tmp_path):
    world = 2
    path = str(tmp_path / "pipe.pt")
    mp.start_processes(_pipeline_worker, args=(world, _free_port(), path), nprocs=world, join=True,
                       start_method="spawn")
    got = torch.load(path, weights_only=True)
    for k in range(3):
        ref = torch.cat([torch.full((2, 3, 4, 5), float(10 * k + r)) for r in range(world)])
        assert torch.equal(got[k], ref)


def _verify_worker(rank, world, port, result_path):
    """verify_gather: an honest gather passes on every rank; one flipped bit in
    rank 0's slice of rank 1's gathered copy fails on every rank."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from rrin_amd.shard import gather_frames, verify_gather
    local = torch.rand(2, 3, 8, 10, generator=torch.Generator().manual_seed(rank))
    g = gather_frames(local)
    ok1 = verify_gather(local, g)["ok"]
    bad = g.clone()
    if rank == 1:
        bits = bad.view(torch.int32)
        bits[0, 1, 2, 3] ^= 1  # rank 0's slice, as rank 1 received it
    ok2 = verify_gather(local, bad)["ok"]
    torch.save(torch.tensor([ok1, ok2]), f"{result_path}.{rank}")
    dist.barrier()
    dist.destroy_process_group()


def test_verify_gather_bitwise_gloo(tmp_path):
    world = 2
    path = str(tmp_path / "v")
    mp.start_processes(_verify_worker, args=(world, _free_port(), path), nprocs=world, join=True,
                       start_method="spawn")
    for r in range(world):
        ok1, ok2 = torch.load(f"{path}.{r}", weights_only=True).tolist()
        assert ok1 and not ok2, (r, ok1, ok2)
