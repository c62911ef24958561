"""World-size-2 gloo test of the sharding path on CPU: each rank searches its shard
of the roots (the oracle stands in for the GPU search here -- the sharding, global-order draws and
the result all_gather are what is under test), and the gathered visit histograms, actions and
root Q values must equal the single-process result bit for bit, for even and uneven shards."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from conftest import GOLDEN, ROOT


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, B, out_path):
    import sys

    sys.path.insert(0, ROOT)
    import torch
    import torch.distributed as dist

    from muzero_hanoi_amd import distributed as mdist
    from muzero_hanoi_amd import rng
    from oracle import oracle as orc

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    w, in_dim, sup = orc.load_weights_npz(f"{GOLDEN}/weights_N3_s0.npz")
    flat = orc.flat_weights(w) if rank == 0 else np.zeros_like(orc.flat_weights(w))
    flat = mdist.broadcast_weights(flat, "cpu")
    n, S = 3, 12
    g = np.random.default_rng(11)
    st = g.integers(0, 3, (B, n))
    obs = np.zeros((B, 3 * n), np.float32)
    obs[np.arange(B)[:, None], np.arange(n) * 3 + st] = 1
    noise, tie, u = rng.synthetic_draws(B, deterministic=False, alpha=0.25, seed=3)  # GLOBAL order
    sl = lambda x: mdist.shard(x, world, rank)
    o = orc.search(n, S, sl(obs), flat=flat, support=sup, noise=sl(noise), tie_idx=sl(tie), action_u=sl(u))
    mine = dict(visits=torch.from_numpy(o["visits"]), action=torch.from_numpy(o["action"]),
                root_q=torch.from_numpy(o["rootQ"]))
    res = mdist.gather_results(mine, B, world)
    # the overlapped form bench.py times (even shards only): the same rows once its work completes
    pend = mdist.gather_results_async(mine, B, world)
    if B % world:
        assert pend is None
    else:
        pend[0].wait()
        for k, v in mdist.unpack_results(pend[1]).items():
            assert torch.equal(v, res[k]), k
    if rank == 0:
        np.savez(out_path, **{k: v.numpy() for k, v in res.items()})
    dist.destroy_process_group()


@pytest.mark.parametrize("B", [40, 37])
def test_sharded_equals_single(tmp_path, oracle, B):
    from muzero_hanoi_amd import distributed as mdist
    from muzero_hanoi_amd import rng

    out = str(tmp_path / "res.npz")
    mp.spawn(_worker, args=(2, _free_port(), B, out), nprocs=2, join=True)
    got = np.load(out)
    w, in_dim, sup = oracle.load_weights_npz(f"{GOLDEN}/weights_N3_s0.npz")
    g = np.random.default_rng(11)
    st = g.integers(0, 3, (B, 3))
    obs = np.zeros((B, 9), np.float32)
    obs[np.arange(B)[:, None], np.arange(3) * 3 + st] = 1
    noise, tie, u = rng.synthetic_draws(B, deterministic=False, alpha=0.25, seed=3)
    ref = oracle.search(3, 12, obs, flat=oracle.flat_weights(w), support=sup, noise=noise, tie_idx=tie, action_u=u)
    assert np.array_equal(got["visits"], ref["visits"])
    assert np.array_equal(got["action"], ref["action"])
    assert got["root_q"].dtype == np.float64 and np.array_equal(got["root_q"], ref["rootQ"])
    assert [mdist.shard_range(B, 2, r) for r in range(2)] == ([(0, 20), (20, 40)] if B == 40 else [(0, 19), (19, 37)])
