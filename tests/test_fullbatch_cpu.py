"""CPU checks of the whole-batch fixtures (tests/golden/full_*.npz, gen_fullbatch.py) that the GPU
test compares every root with: the bench inputs regenerate to the recorded digest here, and a sample
of roots re-run through the oracle reproduces the recorded outputs."""
import os
import sys

import numpy as np
import pytest

from conftest import GOLDEN, golden

sys.path.insert(0, GOLDEN)


@pytest.fixture(scope="module")
def gf():
    from muzero_hanoi_amd import build

    build.build()  # rng.predraw runs libmzh's host code
    import gen_fullbatch

    return gen_fullbatch


TAGS = sorted(f[len("full_"):-len(".npz")] for f in os.listdir(GOLDEN) if f.startswith("full_") and f.endswith(".npz"))


def test_every_config_has_its_fixture():
    import gen_fullbatch as gf

    assert sorted(list(gf.CONFIGS) + list(gf.VARIANTS)) == TAGS


@pytest.mark.parametrize("tag", TAGS)
def test_full_batch_fixture(gf, oracle, tag):
    z = golden(f"full_{tag}.npz")
    n, S = int(z["n_disks"]), int(z["n_sims"])
    obs, noise, tie, u = gf.inputs(tag)
    assert np.array_equal(gf.inputs_sha(obs, noise, tie, u), z["inputs_sha"])
    B = len(obs)
    assert z["visits"].shape == (B, 6) and (z["visits"].astype(np.int64).sum(1) == S).all()
    assert z["rootq_minmax_sha"].shape == (-(-B // gf.BLOCK), 32)
    # 4 roots of the first block, re-run through the oracle: the block's digest needs the whole block,
    # so the sampled roots are checked field by field (visits, action, selection steps)
    idx = np.r_[0:2, B - 2:B]
    flat, sup = gf.weights(n)
    sel = lambda x: None if x is None else x[idx]
    r = oracle.search(n, S, obs[idx], flat=flat, support=sup, noise=sel(noise), tie_idx=tie[idx], action_u=sel(u),
                      temperature=1.0, deterministic=gf.deterministic(tag), discount=0.8)
    assert np.array_equal(r["visits"], z["visits"][idx].astype(np.int32))
    assert np.array_equal(r["action"], z["action"][idx].astype(np.int32))
    assert np.array_equal(r["sel_steps"], z["sel_steps"][idx].astype(np.int64))
    if "root_q" in z:
        assert np.array_equal(r["rootQ"], z["root_q"][idx])
    assert os.path.exists(os.path.join(GOLDEN, "gen_fullbatch.py"))
