"""Checkpoint / ablation compatibility with the reference."""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN


def test_load_reference_checkpoint_and_ablate(tmp_path):
    from muzero_hanoi_amd.checkpoint import ablate_networks, load_model, save_model

    path = os.path.join(GOLDEN, "muzero_model_N3.pt")
    net = load_model(path)
    ref = torch.load(path, map_location="cpu", weights_only=True)
    for k, v in ref["Muzero_net"].items():
        assert torch.equal(net.state_dict()[k], v), k
    assert net.TD_return and net.support_size == 33
    st = net.optimiser.state_dict()
    assert len(st["state"]) == len(ref["Net_optim"]["state"]) > 0
    # round trip in the same format
    out = tmp_path / "m.pt"
    save_model(net, out)
    again = torch.load(out, map_location="cpu", weights_only=True)
    assert set(again) == {"Muzero_net", "Net_optim"}
    # the reference's head ablation under the same torch seed gives the same weights
    torch.manual_seed(123)
    ablate_networks(True, False, True, net)
    ab = np.load(os.path.join(GOLDEN, "ablated_N3.npz"))
    for k in ab.files:
        assert np.array_equal(net.state_dict()[k].numpy(), ab[k]), k


@pytest.mark.gpu
def test_engine_repacks_after_ablation(oracle):
    """The search engine follows in-place parameter changes (ablation / optimiser steps)."""
    from muzero_hanoi_amd.checkpoint import ablate_networks, load_model
    from muzero_hanoi_amd.engine import flat_weights

    net = load_model(os.path.join(GOLDEN, "muzero_model_N3.pt"))
    x = torch.zeros(9)
    x[[0, 3, 6]] = 1
    h0, _, pi0, v0 = net.initial_inference(x)
    o = oracle.initial_inference(flat_weights(net.state_dict()), 9, 33, x[None].numpy())
    assert np.array_equal(pi0, o["pi"][0]) and v0 == float(o["value"][0])
    torch.manual_seed(123)
    ablate_networks(True, False, False, net)
    h1, _, pi1, v1 = net.initial_inference(x)
    o = oracle.initial_inference(flat_weights(net.state_dict()), 9, 33, x[None].numpy())
    assert np.array_equal(pi1, o["pi"][0]) and not np.array_equal(pi0, pi1)
    assert np.array_equal(h0, h1)  # representation untouched by a policy-head ablation
