"""Per-tensor sharding of a codec batch over the GPUs of one node.

The Eden path has no cross-tensor dependency: the aggregator
codes every model tensor independently (aggregator.py:816 compress, :826
decompress, once per tensor), so multi-GPU runs need no data-path
collective -- each rank codes its own tensors.  The only collectives are a
barrier and the max of the timed region, used by bench.py.

Shards are balanced by the HBM bytes a tensor's encode+decode moves on this
implementation (`tensor_cost`), not by its element count: a slice of
P > 2^15 elements makes extra fp32 round trips through its intermediate
(two per direction for P <= 2^25, four for 2^26 <= P <= 2^29),
so the Llama-3-8B embed / lm_head (one 2^29 slice each) weigh ~1.5x their
size.
"""
_THRESH = 0.1  # Eden max_padding_overhead (eden_pipeline.py:397)


def slice_dims(n):
    """Reference slicing rule (eden_pipeline.py:588-602): [(P, valid len)]."""
    def low(v):
        return 1 << (v.bit_length() - 1) if v else 0

    def high(v):
        return 1 << (v - 1).bit_length() if v > 1 else v

    out, rem = [], int(n)
    while n and (high(rem) - rem) / n > _THRESH:
        lo = low(rem)
        out.append((max(lo, 8), lo))
        rem -= lo
    if n:
        out.append((max(high(rem), 8), rem))
    return out


def tensor_cost(n, n_bits=8):
    """HBM bytes one Eden encode + decode of an n-element tensor moves
    (fp32 in/out, bit planes, fp32 intermediates of the multi-pass FWHT)."""
    c = 0
    for P, ln in slice_dims(n):
        c += 8 * ln + n_bits * P // 4
        if P > 1 << 25:
            c += 64 * P
        elif P > 1 << 15:
            c += 32 * P
    return c


def lpt_partition(sizes, parts, cost=None):
    """Longest-processing-time-first partition of tensor indices, by
    cost(size) (default: the size itself)."""
    w = [cost(s) if cost else s for s in sizes]
    order = sorted(range(len(sizes)), key=lambda i: (-w[i], i))
    load = [0] * parts
    out = [[] for _ in range(parts)]
    for i in order:
        r = min(range(parts), key=lambda k: (load[k], k))
        out[r].append(i)
        load[r] += w[i]
    return [sorted(o) for o in out]


def imbalance(sizes, shards, cost=tensor_cost):
    """max rank cost / mean rank cost (1.0 = perfect)."""
    loads = [sum(cost(sizes[i]) for i in s) for s in shards]
    return max(loads) / (sum(loads) / len(loads)) if loads and sum(loads) else 1.0


def shard_indices(sizes, rank, world, scaling):
    """'weak': every rank codes the whole set (its own update);
    'strong': the rank's LPT share of ONE set, weighted by tensor_cost."""
    if scaling == "strong" and world > 1:
        return lpt_partition(sizes, world, tensor_cost)[rank]
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
