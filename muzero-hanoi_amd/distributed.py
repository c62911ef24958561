"""Multi-GPU sharding of independent roots.

Roots are independent, so the search shards with no data-path collective: rank r owns the
contiguous slice [r*B/W, (r+1)*B/W) of the global batch.  Every random draw is made for the
GLOBAL batch in global root order and then sliced, so results do not depend on the world size.
The single exchange is one all_gather of each root's search result -- what run_mcts returns
(MCTS/mcts.py:122-126): the visit histogram, the action and root Q (fp64) -- packed as 10 int32
words per root (RCCL over xGMI on the GPUs, gloo in the CPU tests); weights are broadcast once
at start-up.
"""
import numpy as np
import torch
import torch.distributed as dist


def shard_range(B, world, rank):
    """contiguous, balanced shards: the first B % world ranks get one extra root"""
    base, extra = divmod(B, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def shard(x, world, rank):
    if x is None:
        return None
    s, e = shard_range(len(x), world, rank)
    return x[s:e]


def broadcast_weights(flat, device, src=0):
    """weights broadcast once (~0.5 MB); returns a host numpy copy identical on every rank"""
    t = torch.as_tensor(np.ascontiguousarray(flat, np.float32)).to(device)
    dist.broadcast(t, src=src)
    return t.cpu().numpy()


def gather_rows(local, B, world):
    """all_gather of per-rank [b_r, k] rows -> global [B, k] in root order.  Even shards (every
    BASELINE config at N = 1, 2, 4, 8) gather straight into the result; uneven ones (they differ by
    one root) pad to the largest shard and drop the padding rows afterwards."""
    bmax = shard_range(B, world, 0)[1]  # rank 0 holds the largest shard
    out = torch.empty((world * bmax, local.shape[1]), dtype=local.dtype, device=local.device)
    if B % world == 0:
        dist.all_gather_into_tensor(out, local.contiguous())
        return out
    pad = torch.zeros((bmax, local.shape[1]), dtype=local.dtype, device=local.device)
    pad[: local.shape[0]] = local
    dist.all_gather_into_tensor(out, pad)
    parts = []
    for r in range(world):
        s, e = shard_range(B, world, r)
        parts.append(out[r * bmax: r * bmax + (e - s)])
    return torch.cat(parts)


def gather_visits(local, B, world):
    """all_gather of per-rank [b_r, 6] int32 visit histograms -> global [B, 6] in root order"""
    return gather_rows(local, B, world)


# packed result row: visits (6 int32), action (1), pad (1), root Q's fp64 bits (2) -- 40 B, so root Q
# sits 8-byte aligned in every row and the unpacked fields are views of the gathered rows
PACK_WORDS = 10


def pack_results(visits, action, root_q):
    """[b, 10] int32 rows for one collective per search (see PACK_WORDS)"""
    b = visits.shape[0]
    return torch.cat([visits.to(torch.int32).reshape(b, 6), action.to(torch.int32).reshape(b, 1),
                      torch.zeros((b, 1), dtype=torch.int32, device=visits.device),
                      root_q.to(torch.float64).contiguous().view(torch.int32).reshape(b, 2)], 1)


def unpack_results(packed):
    """views of the gathered rows (no copies): visits [B, 6], action [B], root_q [B] fp64"""
    b = packed.shape[0]
    return dict(visits=packed[:, :6], action=packed[:, 6], root_q=packed[:, 8:10].view(torch.float64).reshape(b))


def gather_results_async(out, B, world):
    """gather_results without waiting, for even shards (B % world == 0; None otherwise): returns
    (work, rows, packed).  The packing runs on the current stream and the collective on the backend's
    own stream after it, so the next search on the launch stream overlaps the all_gather; the caller
    keeps the tuple alive and calls work.wait() before reading unpack_results(rows)."""
    if B % world:
        return None
    packed = pack_results(out["visits"], out["action"], out["root_q"])
    rows = torch.empty((B, PACK_WORDS), dtype=torch.int32, device=packed.device)
    work = dist.all_gather_into_tensor(rows, packed, async_op=True)
    return work, rows, packed


def gather_results(out, B, world):
    """the global batch's visits [B, 6] int32, action [B] int32 and root_q [B] fp64 in root order,
    from every rank's search outputs (one all_gather of the packed rows)"""
    return unpack_results(gather_rows(pack_results(out["visits"], out["action"], out["root_q"]), B, world))
