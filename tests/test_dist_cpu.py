"""world_size-2/3/4 gloo tests of the distributed plumbing on CPU: the z-slab
partition each rank computes tiles the grid exactly, the bench's
max-over-ranks timing reduction works over gloo, and the IPC transport's
control plane (shared-memory id broadcast over gloo, process-shared barrier,
rank-order allreduce, failure agreement) runs in separate processes through the
C-ABI (mnl_comm_ipc_id / mnl_comm_ipc_reduce -- no GPU call)."""
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
    obj = [core.ipc_id(world) if rank == 0 else None]
    dist.broadcast_object_list(obj, src=0)
    import ctypes
    import numpy as np
    from meep_nl_amd._lib import lib, ptr
    n = 20000  # > one 8192-double slot: chunked reduction
    v = np.arange(n, dtype=np.float64) * (rank + 1) + 0.25 * rank
    rc = lib().mnl_comm_ipc_reduce(obj[0], rank, world, ptr(v), n, 1)
    want = np.arange(n, dtype=np.float64) * sum(r + 1 for r in range(world)) + \
        0.25 * sum(range(world))
    ok1 = rc == 0 and np.array_equal(v, want)
    # one rank reports failure: every rank gets -1 (nobody waits in the data step)
    obj2 = [core.ipc_id(world) if rank == 0 else None]
    dist.broadcast_object_list(obj2, src=0)
    w = np.ones(4)
    rc2 = lib().mnl_comm_ipc_reduce(obj2[0], rank, world, ptr(w), 4, int(rank != world - 1))
    ok2 = rc2 != 0 and b"failure" in ctypes.string_at(lib().mnl_last_error())
    res = torch.tensor([int(ok1), int(ok2)], dtype=torch.int64)
    dist.all_reduce(res, op=dist.ReduceOp.MIN)
    if rank == 0:
        q.put(([tuple(v.tolist()) for v in out], float(el.item()), obj[0][:7], res.tolist()))
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
    ranges, el, blob, ipc_ok = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert ranges[0][0] == 0 and ranges[-1][1] == ncell
    for a, b in zip(ranges, ranges[1:]):
        assert a[1] == b[0]
    sizes = [h - l for l, h in ranges]
    assert max(sizes) - min(sizes) <= 1
    assert el == pytest.approx(0.1 * world)
    assert blob == b"MNLIPC1"
    assert ipc_ok == [1, 1]


def test_create_dist_error_paths():
    """mnl_fields_create_dist refuses bad ranks and a bad id before any GPU work,
    and without a HIP device it fails loudly (no CPU fallback)."""
    from meep_nl_amd import core
    from meep_nl_amd._lib import lib
    gv = core.GridVolume(3, [8, 8, 8], 10.0)
    s = core.Structure(gv)
    nid = core.ipc_id(2)
    try:
        for rank, nranks in ((2, 2), (-1, 2), (0, 0)):
            assert not lib().mnl_fields_create_dist(s.h, 0, rank, nranks, nid)
            assert b"rank" in lib().mnl_last_error()
        if core.device_count() == 0:
            with pytest.raises(RuntimeError, match="no HIP device"):
                core.Fields(s, rank=0, nranks=2, nccl_id=nid)
    finally:
        assert lib().mnl_comm_ipc_unlink(nid) == 0
    assert lib().mnl_comm_ipc_unlink(nid) != 0  # gone
