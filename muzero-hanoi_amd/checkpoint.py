"""Checkpoint / ablation compatibility.

The reference stores `{"Muzero_net": state_dict, "Net_optim": optimiser.state_dict()}` in
stats/<env>/<timestamp>/muzero_model.pt (training_main.py:91-103) and the acting experiments load
it and optionally re-initialise heads (acting_experiments/acting_ablations.py:29-45, 357-362).
MuZeroNet keeps the reference's parameter names, so these files load unchanged; the search engine
re-packs the weights into the MFMA layout the next time the network is used (networks.engine_for
tracks parameter versions).  Loading uses torch.load(weights_only=True): nothing in the file is
executed.
"""
import torch

from .networks import MuZeroNet


def save_model(networks, path):
    """training_main.py:91-103"""
    sd = networks._orig_mod.state_dict() if hasattr(networks, "_orig_mod") else networks.state_dict()
    torch.save({"Muzero_net": sd, "Net_optim": networks.optimiser.state_dict()}, path)


def load_model(path, lr=0.002, device="cpu", load_optimiser=True):
    """acting_ablations.py:349-360: rebuild MuZeroNet from the state_dict shapes and load it."""
    d = torch.load(path, map_location="cpu", weights_only=True)
    sd = d["Muzero_net"]
    in_dim = sd["representation_net.0.weight"].shape[1]
    n_action = sd["policy_net.2.weight"].shape[0]
    td = sd["value_net.2.weight"].shape[0] != 1
    net = MuZeroNet(rpr_input_s=in_dim, action_s=n_action, lr=lr, TD_return=td, device=device).to(device)
    net.load_state_dict(sd)
    if load_optimiser and "Net_optim" in d:
        net.optimiser.load_state_dict(d["Net_optim"])
    return net


def ablate_networks(reset_latent_policy, reset_latent_values, reset_latent_rwds, networks):
    """acting_ablations.py:29-45: re-initialise heads (uses the global torch RNG like the reference)"""
    if reset_latent_policy:
        networks.policy_net.apply(networks.reset_param)
    if reset_latent_values:
        networks.value_net.apply(networks.reset_param)
    if reset_latent_rwds:
        networks.rwd_net.apply(networks.reset_param)
    return networks
