"""Multi-rank path of bench.py on CPU: world_size 2 over gloo (127.0.0.1)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from openfl_amd.sharding import lpt_partition, max_over_ranks, shard_indices, throughput_gib_s
from openfl_amd.workloads import llama3_8b, numel


def test_lpt_partition_covers_and_balances():
    sizes = [numel(s) for _, s in llama3_8b()]
    for parts in (1, 2, 4, 8):
        shards = lpt_partition(sizes, parts)
        flat = sorted(i for s in shards for i in s)
        assert flat == list(range(len(sizes)))
        loads = [sum(sizes[i] for i in s) for s in shards]
        assert max(loads) / (sum(sizes) / parts) < 1.08  # >= 6x of 8 feasible at 8 GPUs


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sizes = [numel(s) for _, s in llama3_8b()]
    mine = shard_indices(sizes, rank, world, "strong")
    weak = shard_indices(sizes, rank, world, "weak")
    elapsed = 1.0 + rank  # rank 1 is the slowest
    slowest = max_over_ranks(elapsed)
    gathered = [None] * world
    dist.all_gather_object(gathered, mine)
    if rank == 0:
        q.put((gathered, len(weak), slowest))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(120)
def test_two_rank_gloo():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    gathered, nweak, slowest = q.get(timeout=100)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert sorted(gathered[0] + gathered[1]) == list(range(291))
    assert not set(gathered[0]) & set(gathered[1])
    assert nweak == 291 and slowest == 2.0
    assert throughput_gib_s(2 ** 30, 2, 10, 2.0, "weak") == 10.0
    assert throughput_gib_s(0, 2, 10, 2.0, "strong", 2 ** 31) == 10.0
