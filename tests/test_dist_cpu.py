"""world_size-2/4 gloo tests of the distributed plumbing on CPU: the z-slab
partition each rank computes tiles the grid exactly, and the bench's
max-over-ranks timing reduction and unique-id broadcast work over gloo."""
import os
import socket

import pytest
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, ncell, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import torch
    from meep_nl_amd import core
    lo, hi = core.slab_range(ncell, rank, world)
    t = torch.tensor([lo, hi], dtype=torch.int64)
    out = [torch.zeros(2, dtype=torch.int64) for _ in range(world)]
    dist.all_gather(out, t)
    el = torch.tensor([0.1 * (rank + 1)], dtype=torch.float64)
    dist.all_reduce(el, op=dist.ReduceOp.MAX)
    obj = [b"x" * 128 if rank == 0 else None]  # stand-in for mnl_comm_unique_id bytes
    dist.broadcast_object_list(obj, src=0)
    if rank == 0:
        q.put(([tuple(v.tolist()) for v in out], float(el.item()), obj[0]))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,ncell", [(2, 1024), (4, 1026), (3, 17)])
def test_slab_partition_over_gloo(world, ncell):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, ncell, q)) for r in range(world)]
    for p in procs:
        p.start()
    ranges, el, blob = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert ranges[0][0] == 0 and ranges[-1][1] == ncell
    for a, b in zip(ranges, ranges[1:]):
        assert a[1] == b[0]
    sizes = [h - l for l, h in ranges]
    assert max(sizes) - min(sizes) <= 1
    assert el == pytest.approx(0.1 * world)
    assert blob == b"x" * 128
