"""Whole-batch oracle outputs for the BASELINE.json search configs at their full per-GPU sizes,
on the exact inputs bench.py searches (seed 0): the GPU test (tests/test_gpu_parity.py::
test_search_full_batch_equals_oracle) compares EVERY root of the HIP search with these.

    python tests/golden/gen_fullbatch.py [TAG ...]        # ~10 min on 8 host cores

configs[1] is also stored for seeds 1-4 and in the deterministic mode (alpha 0, no noise, the
action the argmax of the visits) -- the seeds and mode SURVEY.md 8d names for the parity runs.

Inputs, as bench.py builds them (bench.random_roots + rng.predraw on RandomState(seed), global
root order, then the rank's contiguous shard); weights tests/golden/weights_N{n}_s0.npz (the
reference's MuZeroNet(TD_return=True) after torch.manual_seed(0), identical to bench.py's
random-init network -- checked below).  The outputs come from the C oracle (oracle/mzh_oracle.c,
pinned on the reference's own fixtures), run one process per host core over root chunks (roots are
independent: each has its own fresh MinMaxStats, MCTS/mcts.py:23).

Stored per config (np.savez_compressed): visits uint8 [B,6], action uint8 [B], sel_steps uint16 [B],
extra_ties uint8 [B]; root Q and the (max, min) MinMaxStats as SHA-256 digests of 256-root blocks
of their float64 bytes (rootq_minmax_sha [B/256, 32] uint8) -- exact, 1/64 the size -- and for the
4,096-root config the float64 arrays themselves; inputs_sha: digest of the regenerated inputs.
"""
import hashlib
import multiprocessing as mp
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

# tag: (disks, global roots, sims, world, rank) -- BASELINE.json configs[1..4] as bench.py runs them
CONFIGS = {
    "c1_4096": (4, 4096, 50, 1, 0),          # configs[1]
    "c3_16384": (4, 16384, 200, 1, 0),       # configs[3]
    "c2_65536": (4, 65536, 50, 1, 0),        # configs[2], the metric's batch on one GPU
    "c2_shard7of8": (4, 65536, 50, 8, 7),    # configs[2], rank 7's 8,192-root shard at N=8 (the 8-GPU headline)
    "c4_shard0of8": (7, 262144, 100, 8, 0),  # configs[4], rank 0's 32,768-root shard at N=8
}
# configs[4]'s other seven shards: with rank 0's, every root of the 262,144-root batch (the GPU test
# runs the whole batch as one launch and compares it with the eight shards' outputs in root order)
CONFIGS.update({f"c4_shard{r}of8": (7, 262144, 100, 8, r) for r in range(1, 8)})
SEED = 0
BLOCK = 256
# further draws of configs[1] (seeds 0..4; the parity runs' deterministic mode with alpha 0):
# tag: (config tag, seed, deterministic)
VARIANTS = {f"c1_4096_s{k}": ("c1_4096", k, False) for k in range(1, 5)}
VARIANTS["c1_4096_det"] = ("c1_4096", 0, True)


def _spec(tag):
    """(n, global roots, sims, world, rank, seed, deterministic) of a fixture tag"""
    base, seed, det = VARIANTS.get(tag, (tag, SEED, False))
    return (*CONFIGS[base], seed, det)


def inputs(tag):
    """(obs f32 [B,3N], noise f64 [B,6], tie i32 [B], u f64 [B]) exactly as bench.py makes them"""
    import bench
    from muzero_hanoi_amd import distributed as mdist
    from muzero_hanoi_amd import rng

    n, GB, S, W, r, seed, det = _spec(tag)
    obs = bench.random_roots(n, GB, seed)
    noise, tie, u = rng.predraw(GB, deterministic=det, alpha=0.0 if det else 0.25, rng=np.random.RandomState(seed))
    return tuple(None if x is None else np.ascontiguousarray(mdist.shard(x, W, r)) for x in (obs, noise, tie, u))


def deterministic(tag):
    return _spec(tag)[6]


def inputs_sha(obs, noise, tie, u):
    h = hashlib.sha256()
    for x, t in ((obs, np.float32), (noise, np.float64), (tie, np.int32), (u, np.float64)):
        if x is not None:  # the deterministic mode draws no noise and no action uniform
            h.update(np.ascontiguousarray(x, t).tobytes())
    return np.frombuffer(h.digest(), np.uint8)


def block_sha(root_q, mm):
    """SHA-256 of each 256-root block's float64 root Q then (max, min) bytes"""
    B = len(root_q)
    out = np.zeros((-(-B // BLOCK), 32), np.uint8)
    for k in range(out.shape[0]):
        sl = slice(k * BLOCK, min(B, (k + 1) * BLOCK))
        h = hashlib.sha256(np.ascontiguousarray(root_q[sl], np.float64).tobytes())
        h.update(np.ascontiguousarray(mm[sl], np.float64).tobytes())
        out[k] = np.frombuffer(h.digest(), np.uint8)
    return out


def weights(n):
    from oracle import oracle

    w, in_dim, sup = oracle.load_weights_npz(os.path.join(HERE, f"weights_N{n}_s0.npz"))
    return oracle.flat_weights(w), sup


def _chunk(args):
    n, S, obs, noise, tie, u, det = args
    from oracle import oracle

    flat, sup = weights(n)
    r = oracle.search(n, S, obs, flat=flat, support=sup, noise=noise, tie_idx=tie, action_u=u, temperature=1.0,
                      deterministic=det, discount=0.8)
    return {k: r[k] for k in ("visits", "rootQ", "mm_max", "mm_min", "action", "sel_steps", "extra_ties")}


def generate(tag, procs):
    import torch

    n, GB, S, W, r, seed, det = _spec(tag)
    obs, noise, tie, u = inputs(tag)
    B = len(obs)
    # bench.py's network is MuZeroNet after torch.manual_seed(0): the same weights as the fixture
    from muzero_hanoi_amd import engine
    from muzero_hanoi_amd.networks import MuZeroNet

    torch.manual_seed(SEED)
    net = MuZeroNet(3 * n, 6, 0.002, "cpu", TD_return=True)
    assert np.array_equal(engine.flat_weights(net.state_dict()), weights(n)[0]), "bench weights != fixture weights"
    step = 512
    sl = lambda x, i: None if x is None else x[i:i + step]
    jobs = [(n, S, obs[i:i + step], sl(noise, i), tie[i:i + step], sl(u, i), det) for i in range(0, B, step)]
    with mp.get_context("spawn").Pool(procs) as pool:
        parts = pool.map(_chunk, jobs)
    cat = {k: np.concatenate([p[k] for p in parts]) for k in parts[0]}
    mm = np.stack([cat["mm_max"], cat["mm_min"]], 1)
    assert cat["sel_steps"].max() < 65536 and cat["visits"].max() < 256
    out = dict(n_disks=n, n_sims=S, global_roots=GB, world=W, rank=r, seed=seed, deterministic=det,
               visits=cat["visits"].astype(np.uint8), action=cat["action"].astype(np.uint8),
               sel_steps=cat["sel_steps"].astype(np.uint16), extra_ties=cat["extra_ties"].astype(np.uint8),
               rootq_minmax_sha=block_sha(cat["rootQ"], mm), inputs_sha=inputs_sha(obs, noise, tie, u))
    if B <= 4096:
        out.update(root_q=cat["rootQ"], minmax=mm)
    np.savez_compressed(os.path.join(HERE, f"full_{tag}.npz"), **out)
    print(tag, B, "roots:", "visits sum ok" if (cat["visits"].sum(1) == S).all() else "BAD", flush=True)


if __name__ == "__main__":
    tags = sys.argv[1:] or list(CONFIGS) + list(VARIANTS)
    procs = min(8, os.cpu_count() or 1)
    for t in tags:
        generate(t, procs)
