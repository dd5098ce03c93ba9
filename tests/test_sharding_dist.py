"""Multi-rank path of bench.py on CPU: world_size 2 over gloo (127.0.0.1)."""
import json
import os
import socket
import subprocess
import sys

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from openfl_amd.sharding import (imbalance, lpt_partition, max_over_ranks, shard_indices, slice_dims, tensor_cost,
                                 throughput_gib_s)
from openfl_amd.workloads import llama3_8b, numel

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_lpt_partition_covers_and_balances():
    sizes = [numel(s) for _, s in llama3_8b()]
    for parts in (1, 2, 4, 8):
        shards = lpt_partition(sizes, parts)
        flat = sorted(i for s in shards for i in s)
        assert flat == list(range(len(sizes)))
        loads = [sum(sizes[i] for i in s) for s in shards]
        assert max(loads) / (sum(sizes) / parts) < 1.08  # >= 6x of 8 feasible at 8 GPUs


def test_cost_weighted_lpt_balances_llama_at_8():
    """Shards weighted by the bytes each tensor's passes move (a 2^29 slice
    makes 5 passes per direction, 2^16..2^25 slices 3): < 1.1 imbalance."""
    sizes = [numel(s) for _, s in llama3_8b()]
    for parts in (2, 4, 8):
        shards = lpt_partition(sizes, parts, tensor_cost)
        assert sorted(i for s in shards for i in s) == list(range(len(sizes)))
        assert imbalance(sizes, shards) < 1.1
    embed = 128256 * 4096
    assert slice_dims(embed) == [(1 << 29, embed)]
    assert tensor_cost(embed) > 1.4 * tensor_cost(1 << 28)  # 5-pass slice weighs more per element


@pytest.mark.timeout(240)
def test_bench_spawns_ranks_dry_run():
    """bench.py --gpus 2 started directly spawns 2 ranks (torch.distributed.run,
    127.0.0.1) that shard ONE Llama-3-8B update (strong scaling, the default)."""
    env = dict(os.environ, PYTHONPATH=ROOT)
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dry-run"],
                       capture_output=True, text=True, timeout=220, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    out = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert out["n_gpus"] == 2 and out["gpus_arg"] == 2 and out["scaling"] == "strong"
    assert out["tensors"] == 291 and out["covered"] and sum(out["per_rank_tensors"]) == 291
    assert out["imbalance"] < 1.1 and out["imbalance_8"] < 1.1


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
