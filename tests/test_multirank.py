"""bench.py's multi-rank aggregation (weak scaling over independent filters) on gloo, world size 2.

The GPU box runs the same function over RCCL (`torch.distributed.run ... bench.py --gpus N`); here
it runs on the CPU with two processes, as SURVEY.md §8(e) prescribes for the N>1 path.
"""
import os
import socket
import sys

import numpy as np
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    import torch.distributed as dist
    sys.path.insert(0, ROOT)
    import bench
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    F = 3  # filters per rank; rank r owns filters [3r, 3r+3)
    poses = np.arange(F * 3, dtype=np.float64).reshape(F, 3) + 100 * rank
    elapsed, total, gathered = bench.reduce_ranks(0.5 + rank, 10 * (rank + 1), poses, "cpu")
    q.put((rank, elapsed, total, gathered))
    dist.barrier()
    dist.destroy_process_group()


def test_reduce_ranks_gloo_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, elapsed, total, gathered in out:
        assert elapsed == 1.5            # MAX over ranks
        assert total == 30.0             # SUM of corrections
        assert gathered.shape == (6, 3)  # contiguous filter blocks, rank order
        np.testing.assert_array_equal(gathered[:3], np.arange(9.0).reshape(3, 3))
        np.testing.assert_array_equal(gathered[3:], np.arange(9.0).reshape(3, 3) + 100)
