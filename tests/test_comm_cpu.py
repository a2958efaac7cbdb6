"""Collective semantics of the communicator layer (SURVEY §4.2 "Unit: comm"):
all_reduce (SUM / MAX), broadcast from a non-zero root, all_gather rank order,
the reference's ``reduce_tensor`` (main.py:173-177: clone, SUM, / W), the async
bucket average, and the cross-rank ``check_same`` guard -- at W = 2 and 4 over
gloo, one process per rank."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist
    from pytorch_multiprocessing_distributed_amd.parallel.comm import get_comm
    dist.init_process_group("gloo", rank=rank, world_size=world)
    comm = get_comm()
    assert comm is not None and comm.world_size == world and comm.rank == rank

    t = torch.full((5,), float(rank + 1))
    comm.all_reduce_(t)
    assert torch.equal(t, torch.full((5,), float(world * (world + 1) // 2)))

    t = torch.tensor([float(rank), -float(rank)])
    comm.all_reduce_(t, op=dist.ReduceOp.MAX)
    assert torch.equal(t, torch.tensor([float(world - 1), 0.0]))

    b = torch.arange(4, dtype=torch.float32) * (rank + 1)
    comm.broadcast_(b, src=1)
    assert torch.equal(b, torch.arange(4, dtype=torch.float32) * 2)

    g = comm.all_gather(torch.tensor([rank * 10, rank]))
    assert [int(x[0]) for x in g] == [r * 10 for r in range(world)]

    x = torch.tensor([2.0 * rank, 1.0])
    m = comm.reduce_mean(x)
    assert torch.equal(x, torch.tensor([2.0 * rank, 1.0]))          # input untouched (clone)
    torch.testing.assert_close(m, torch.tensor([float(world - 1), 1.0]))

    a = torch.full((3,), float(rank))
    comm.all_reduce_mean_async(a).wait()
    torch.testing.assert_close(a, torch.full((3,), (world - 1) / 2.0))

    comm.check_same("same on every rank")
    with pytest.raises(RuntimeError):
        comm.check_same(f"rank {rank} differs")
    comm.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_comm_collective_semantics(world):
    mp.spawn(_worker, args=(world, _free_port()), nprocs=world, join=True)
