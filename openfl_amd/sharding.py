"""Per-tensor sharding of a codec batch over the GPUs of one node.

The Eden path has no cross-tensor dependency, so multi-GPU runs
need no data-path collective: each rank codes its own tensors.  The only
collectives are a barrier and the max of the timed region, used by bench.py.
"""


def lpt_partition(sizes, parts):
    """Longest-processing-time-first partition of tensor indices by size."""
    order = sorted(range(len(sizes)), key=lambda i: (-sizes[i], i))
    load = [0] * parts
    out = [[] for _ in range(parts)]
    for i in order:
        r = min(range(parts), key=lambda k: (load[k], k))
        out[r].append(i)
        load[r] += sizes[i]
    return [sorted(o) for o in out]


def shard_indices(sizes, rank, world, scaling):
    """'weak': every rank codes the whole set (its own update); 'strong': LPT share."""
    if scaling == "strong" and world > 1:
        return lpt_partition(sizes, world)[rank]
    return list(range(len(sizes)))


def max_over_ranks(value, device=None):
    """Max of a float over the process group (identity without one)."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return float(value)
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def throughput_gib_s(bytes_per_rank, world, steps, elapsed_s, scaling, total_set_bytes=None):
    """Whole-job GiB/s: all bytes all ranks coded / slowest rank's time."""
    total = bytes_per_rank * world if scaling == "weak" else total_set_bytes
    return total * steps / elapsed_s / 2 ** 30
