"""MuZeroNet drop-in (reference: networks.py:11-205).

Same constructor, same submodules and state_dict keys (so `torch.manual_seed(s); MuZeroNet(...)`
gives the reference's weights and checkpoints load unchanged), same torch methods for the
training / analysis paths (represent, dynamics, prediction, the value transform, update).
`initial_inference` / `recurrent_inference` -- the search-time entry points (networks.py:71-116)
-- run on the MI355X through libmzh (batched MFMA MLP), never through torch on the CPU.
"""
import weakref

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F
import torch.optim as opt

from . import engine as _engine


class MuZeroNet(nn.Module):
    def __init__(self, rpr_input_s, action_s, lr, device, reward_s=1, h1_s=256, reprs_output_size=64,
                 weight_decay=1e-4, TD_return=False):
        super().__init__()
        self.dev = device
        self.num_actions = action_s
        self.TD_return = TD_return
        self.reprs_output_size = reprs_output_size
        self.support_size = 33 if TD_return else 1  # networks.py:34-37

        # construction order == reference (networks.py:39-67): identical init under one seed
        self.representation_net = nn.Sequential(nn.Linear(rpr_input_s, h1_s), nn.ReLU(),
                                                nn.Linear(h1_s, reprs_output_size))
        self.dynamic_net = nn.Sequential(nn.Linear(reprs_output_size + action_s, h1_s), nn.ReLU(),
                                         nn.Linear(h1_s, reprs_output_size))
        self.rwd_net = nn.Sequential(nn.Linear(reprs_output_size, h1_s), nn.ReLU(),
                                     nn.Linear(h1_s, self.support_size))
        self.policy_net = nn.Sequential(nn.Linear(reprs_output_size, h1_s), nn.ReLU(), nn.Linear(h1_s, action_s))
        self.value_net = nn.Sequential(nn.Linear(reprs_output_size, h1_s), nn.ReLU(),
                                       nn.Linear(h1_s, self.support_size))
        self.optimiser = opt.Adam(self.parameters(), lr)

    # ------------------------------------------------------------------ search-time inference (HIP)
    @torch.no_grad()
    def initial_inference(self, x):
        """networks.py:71-94 -> (h np.float32[64], rwd 0.0, pi np.float32[6], value float).
        A [B, D] batch with B > 1 returns arrays ([B,64], [B], [B,6], [B])."""
        eng = engine_for(self, 0, _rows(x))
        xb = _as_rows(x, eng.device)
        out = eng.initial_inference(xb)
        return _unpack(out, x, recurrent=False)

    @torch.no_grad()
    def recurrent_inference(self, h_state, action):
        """networks.py:96-116; `action` is the one-hot float vector the reference passes."""
        eng = engine_for(self, 0, _rows(h_state))
        hb = _as_rows(h_state, eng.device)
        ab = _as_rows(action, eng.device)
        ones = (ab == 1).sum(-1)
        zeros = (ab == 0).sum(-1)
        if not bool(((ones == 1) & (ones + zeros == ab.shape[-1])).all()):
            raise ValueError("recurrent_inference expects one-hot actions (the search path's contract, "
                             "MCTS/mcts.py:92-99); use dynamics()/prediction() for arbitrary inputs")
        out = eng.recurrent_inference(hb, ab.argmax(-1).to(torch.int32))
        return _unpack(out, h_state, recurrent=True)

    # ------------------------------------------------------------------ torch paths (training / analysis)
    def update(self, loss):
        self.optimiser.zero_grad()
        loss.backward()
        self.optimiser.step()

    def represent(self, x):
        return self.normalize_h_state(self.representation_net(x))

    def dynamics(self, h_state, action):
        x = torch.cat([h_state, action], dim=-1)
        new_h_state = self.dynamic_net(x)
        rwd_prediction = self.rwd_net(new_h_state)
        if self.TD_return:
            rwd_prediction = self.logits_to_transformed_expected_value(rwd_prediction)
        return self.normalize_h_state(new_h_state), rwd_prediction

    def prediction(self, h):
        pi_logits = self.policy_net(h)
        value_logits = self.value_net(h)
        if self.TD_return:
            value_logits = self.logits_to_transformed_expected_value(value_logits)
        return pi_logits, value_logits

    def logits_to_transformed_expected_value(self, logits):
        max_value = (self.support_size - 1) // 2
        probs = torch.softmax(logits, dim=-1)
        x = self._transform_from_2hot(probs, -max_value, max_value)
        return self._signed_parabolic(x)

    def _transform_from_2hot(self, probs, min_value, max_value):
        support = torch.linspace(min_value, max_value, self.support_size, device=probs.device)
        return torch.sum(probs * support.expand_as(probs), dim=-1, keepdim=True)

    def _signed_parabolic(self, x, eps=1e-3):
        z = torch.sqrt(1 + 4 * eps * (eps + 1 + torch.abs(x))) / 2 / eps - 1 / 2 / eps
        return torch.sign(x) * (torch.square(z) - 1)

    def normalize_h_state(self, h_state):
        _min = h_state.min(dim=-1, keepdim=True)[0]
        _max = h_state.max(dim=-1, keepdim=True)[0]
        return (h_state - _min) / (_max - _min + 1e-8)

    def set_pol_pertubation(self, pertub_magnitude):
        self.perturb_p_magnitude = pertub_magnitude

    def reset_param(self, l):
        k = np.sqrt(1 / self.reprs_output_size)
        if isinstance(l, nn.Linear):
            nn.init.uniform_(l.weight, a=-k, b=k)
            nn.init.uniform_(l.bias, a=-k, b=k)


# ---------------------------------------------------------------------- binding to libmzh engines
def _rows(t):
    return 1 if t.dim() == 1 else int(t.shape[0])


def _as_rows(t, device):
    t = torch.as_tensor(t)
    if t.dim() == 1:
        t = t[None]
    return t.to(device, torch.float32).contiguous()


def _unpack(out, like, recurrent):
    if like.dim() == 1 or like.shape[0] == 1:
        h = out["h"][0].cpu().numpy()
        pi = out["pi"][0].cpu().numpy()
        v = float(out["value"][0].item())
        r = float(out["reward"][0].item()) if recurrent else 0.0
        return h, r, pi, v
    r = out["reward"].cpu().numpy() if recurrent else np.zeros(out["h"].shape[0], np.float32)
    return out["h"].cpu().numpy(), r, out["pi"].cpu().numpy(), out["value"].cpu().numpy()


_CACHE = weakref.WeakKeyDictionary()  # network -> {"engine", "sig"}


def _param_signature(net):
    return tuple((p.data_ptr(), p._version) for p in net.parameters())


def _param_refs(net):
    """(module, name) of every parameter, in state_dict order: the signature reads them through the module each
    call, so a replaced Parameter object is seen as well as an in-place update"""
    refs = []
    for mname, mod in net.named_modules():
        for pname, prm in mod._parameters.items():
            if prm is not None:
                refs.append((mod, pname))
    return refs


def _fast_signature(refs):
    return tuple([x for mod, name in refs for p in (mod._parameters[name],) for x in (p.data_ptr(), p._version)])


def engine_for(net, max_sims, max_roots, device=None):
    """The libmzh engine bound to `net` (ours or any module with MuZeroNet's state_dict keys),
    with capacity >= (max_sims, max_roots) and the network's CURRENT weights loaded.

    Per call (MCTS.run_mcts makes one per environment step) only the capacity and the parameters' storage /
    version counters are checked: the shape validation and the parameter list are cached per network."""
    cache = _CACHE.get(net)
    if cache is not None and "refs" in cache:
        eng = cache.get("engine")
        if eng is not None and eng.max_sims >= max_sims and eng.max_roots >= max_roots:
            if cache.get("sig") == _fast_signature(cache["refs"]):
                return eng
    sd_keys = set(net.state_dict().keys())
    missing = [k for k in _engine.WEIGHT_KEYS if k not in sd_keys]
    if missing:
        raise TypeError(f"network lacks MuZeroNet parameters {missing}")
    in_dim = net.representation_net[0].in_features
    support = net.value_net[2].out_features
    if (in_dim % 3 or net.representation_net[2].out_features != 64 or net.representation_net[0].out_features != 256
            or net.policy_net[2].out_features != 6 or support not in (1, 33)):
        raise NotImplementedError("libmzh supports the Hanoi MuZeroNet shape (3N -> 256 -> 64, 6 actions, "
                                  "support 33 or 1)")
    cache = _CACHE.setdefault(net, {})
    eng = cache.get("engine")
    if eng is None or eng.max_sims < max_sims or eng.max_roots < max_roots:
        if eng is not None:
            eng.close()
        eng = _engine.Engine(in_dim // 3, max(max_sims, 64 if eng is None else eng.max_sims),
                             max(max_roots, 1 if eng is None else eng.max_roots), support, device=device)
        cache["engine"] = eng
        cache["sig"] = None
    if "refs" not in cache:
        cache["refs"] = _param_refs(net)
    sig = _fast_signature(cache["refs"])
    if cache.get("sig") != sig:
        eng.load_weights(_engine.flat_weights(net.state_dict()))
        cache["sig"] = sig
    return eng
