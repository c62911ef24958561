"""Engine: one libmzh engine (device workspace + packed weights) driven with torch tensors.

All tensors are device tensors on the engine's GPU; calls are asynchronous on torch's current
stream.  This is the layer the drop-in classes (env.py, networks.py, mcts.py) and bench.py use.
"""
import ctypes

import numpy as np
import torch

from . import _lib
from ._lib import check, ptr

WEIGHT_KEYS = [
    f"{net}.{layer}.{kind}"
    for net in ("representation_net", "dynamic_net", "rwd_net", "policy_net", "value_net")
    for layer in (0, 2)
    for kind in ("weight", "bias")
]

ACTIONS = 6
LATENT = 64


def flat_weights(state_dict):
    """MuZeroNet.state_dict() (or a dict of arrays) -> canonical flat fp32 numpy vector."""
    parts = []
    for k in WEIGHT_KEYS:
        v = state_dict[k]
        if isinstance(v, torch.Tensor):
            v = v.detach().to("cpu", torch.float32).numpy()
        parts.append(np.asarray(v, np.float32).reshape(-1))
    return np.ascontiguousarray(np.concatenate(parts))


def require_device():
    if not torch.cuda.is_available() or _lib.device_count() == 0:
        raise RuntimeError("muzero_hanoi_amd needs a HIP device (MI355X); there is no CPU fallback")


class Engine:
    def __init__(self, n_disks, max_sims, max_roots, support=33, device=None):
        require_device()
        if device is None:
            device = torch.cuda.current_device()
        self.device = torch.device("cuda", device if isinstance(device, int) else torch.device(device).index or 0)
        self.n_disks = int(n_disks)
        self.max_sims = int(max_sims)
        self.max_roots = int(max_roots)
        self.support = int(support)
        h = ctypes.c_void_p()
        check(_lib.lib().mzh_create(self.device.index, self.n_disks, self.max_sims, self.max_roots,
                                     self.support, ctypes.byref(h)), "mzh_create")
        self._h = h
        self.weights_loaded = False

    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            torch.cuda.synchronize(self.device)
            _lib.lib().mzh_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _stream(self):
        return _lib.stream_handle(self.device)

    # ---------------------------------------------------------------- weights
    def load_weights(self, flat):
        flat = np.ascontiguousarray(flat, np.float32)
        n = ctypes.c_size_t()
        check(_lib.lib().mzh_weights_size(self.n_disks, self.support, ctypes.byref(n)), "mzh_weights_size")
        if flat.size != n.value:
            raise ValueError(f"expected {n.value} weights, got {flat.size}")
        torch.cuda.synchronize(self.device)
        check(_lib.lib().mzh_load_weights(self._h, flat.ctypes.data_as(ctypes.c_void_p), flat.size),
              "mzh_load_weights")
        self.weights_loaded = True

    # ---------------------------------------------------------------- inference
    def _f32(self, *shape):
        return torch.empty(shape, dtype=torch.float32, device=self.device)

    def initial_inference(self, obs):
        obs = obs.to(self.device, torch.float32).contiguous()
        B = obs.shape[0]
        out = dict(h=self._f32(B, LATENT), reward=self._f32(B), pi=self._f32(B, ACTIONS), value=self._f32(B),
                   policy_logits=self._f32(B, ACTIONS), value_logits=self._f32(B, self.support))
        check(_lib.lib().mzh_initial_inference(self._h, B, ptr(obs), ptr(out["h"]), ptr(out["reward"]),
                                               ptr(out["pi"]), ptr(out["value"]), ptr(out["policy_logits"]),
                                               ptr(out["value_logits"]), self._stream()), "mzh_initial_inference")
        return out

    def recurrent_inference(self, h, action):
        h = h.to(self.device, torch.float32).contiguous()
        a = action.to(self.device, torch.int32).contiguous()
        B = h.shape[0]
        out = dict(h=self._f32(B, LATENT), reward=self._f32(B), pi=self._f32(B, ACTIONS), value=self._f32(B),
                   policy_logits=self._f32(B, ACTIONS), value_logits=self._f32(B, self.support),
                   reward_logits=self._f32(B, self.support))
        check(_lib.lib().mzh_recurrent_inference(self._h, B, ptr(h), ptr(a), ptr(out["h"]), ptr(out["reward"]),
                                                 ptr(out["pi"]), ptr(out["value"]), ptr(out["policy_logits"]),
                                                 ptr(out["value_logits"]), ptr(out["reward_logits"]),
                                                 self._stream()), "mzh_recurrent_inference")
        return out

    # ---------------------------------------------------------------- search
    def alloc_search_outputs(self, B, n_sims, lockstep=False):
        """lockstep=True adds lockstep_levels (zeroed, one entry per group of roots that advance together: at most
        one per root -- the latency kernel's groups are single roots)"""
        d = self.device
        extra = {"lockstep_levels": torch.zeros(B + 1, dtype=torch.int32, device=d)} if lockstep else {}
        return dict(**extra,
            visits=torch.empty((B, ACTIONS), dtype=torch.int32, device=d),
            root_q=torch.empty(B, dtype=torch.float64, device=d),
            minmax=torch.empty((B, 2), dtype=torch.float64, device=d),
            extra_ties=torch.empty(B, dtype=torch.int32, device=d),
            action=torch.empty(B, dtype=torch.int32, device=d),
            pi=torch.empty((B, ACTIONS), dtype=torch.float64, device=d),
            latent=torch.empty((B, n_sims + 1), dtype=torch.int32, device=d),
            latent_len=torch.empty(B, dtype=torch.int32, device=d),
            sel_steps=torch.empty(B, dtype=torch.int32, device=d),
        )

    def pow_table(self, n_sims, temperature):
        """play-policy power table for a non-integer exponent (None otherwise): np.power over
        arange(n_sims + 1) as int64 with the Python-float exponent, exactly the call
        generate_play_policy makes on the visit counts (MCTS/mcts.py:168-174), on the device"""
        if not 0.0 < temperature <= 1.0:
            return None
        e = max(1.0, min(5.0, 1.0 / temperature))
        if e == int(e):
            return None
        cache = self.__dict__.setdefault("_pow_tables", {})
        key = (int(n_sims), float(temperature))
        if key not in cache:
            tab = np.power(np.arange(n_sims + 1, dtype=np.int64), e)
            cache[key] = torch.from_numpy(tab).to(self.device)
        return cache[key]

    def search(self, n_sims, *, obs=None, replay=None, tie_idx, noise=None, action_u=None, minmax_in=None,
               temperature=1.0, deterministic=False, discount=0.8, eps=0.25, np1_ucb=False, out=None,
               kernel=None, tile=None):
        """Batched search. Tensors must already be on the device (bench: inputs resident in HBM).
        replay = dict(root_pi, pi, reward, value) -> tree-only mode (mzh_search_replay).
        kernel = None (automatic by batch size) | "coop" | "occ2" | "wave" | "wave16" | "one" (all give identical
        results; "one" = the latency kernel, MLP searches only);
        tile = None | 16 | 32: the cooperative kernel's roots per workgroup (default by batch size)."""
        B = int(tie_idx.shape[0])
        if out is None:
            out = self.alloc_search_outputs(B, n_sims)
        keep = []

        def dev(t, dtype):
            if t is None:
                return None
            t = t.to(self.device, dtype).contiguous()
            keep.append(t)
            return t

        a = _lib.SearchArgs()
        a.B = B
        a.n_sims = int(n_sims)
        a.discount = float(discount)
        a.eps = float(eps)
        a.temperature = float(temperature)
        a.deterministic = 1 if deterministic else 0
        a.flags = search_flags(kernel, tile, np1_ucb)
        a.obs = ptr(dev(obs, torch.float32))
        a.noise = ptr(dev(noise, torch.float64))
        a.tie_idx = ptr(dev(tie_idx, torch.int32))
        a.action_u = ptr(dev(action_u, torch.float64))
        a.minmax_in = ptr(dev(minmax_in, torch.float64))
        if replay is not None:
            a.rp_root_pi = ptr(dev(replay["root_pi"], torch.float32))
            a.rp_sim = ptr(dev(replay["sim"] if "sim" in replay else pack_replay(replay), torch.float32))
        a.visits = ptr(out["visits"])
        a.root_q = ptr(out.get("root_q"))
        a.minmax_out = ptr(out.get("minmax"))
        a.extra_ties = ptr(out.get("extra_ties"))
        a.action = ptr(out.get("action"))
        a.pi = ptr(out.get("pi"))
        a.latent = ptr(out.get("latent"))
        a.latent_len = ptr(out.get("latent_len"))
        a.sel_steps = ptr(out.get("sel_steps"))
        pt = self.pow_table(n_sims, float(temperature)) if (out.get("pi") is not None or
                                                              out.get("action") is not None) else None
        if pt is not None:
            keep.append(pt)
        a.pow_table = ptr(pt)
        a.lockstep_levels = ptr(out.get("lockstep_levels"))
        plan = _lib.SearchPlan()
        a.plan_out = ctypes.pointer(plan)
        fn = _lib.lib().mzh_search_replay if replay is not None else _lib.lib().mzh_search
        check(fn(self._h, ctypes.byref(a), self._stream()), "mzh_search")
        out["_keep"] = keep  # inputs stay alive until the caller is done with the async call
        out["_plan"] = plan.as_dict()  # the instantiation the library launched
        return out


def search_flags(kernel=None, tile=None, np1_ucb=False):
    """mzh_search_args.flags for a kernel choice (None | "coop" | "occ2" | "wave" | "wave16" | "one") and coop
    tile ("occ2": the cooperative kernel's two-workgroups-per-CU 16-root form; "one": the latency kernel)"""
    f = _lib.MZH_FLAG_NP1_UCB if np1_ucb else 0
    f |= {None: 0, "auto": 0, "coop": _lib.MZH_FLAG_KERNEL_COOP, "wave": _lib.MZH_FLAG_KERNEL_WAVE,
          "wave16": _lib.MZH_FLAG_KERNEL_WAVE16,
          "occ2": _lib.MZH_FLAG_KERNEL_COOP | _lib.MZH_FLAG_COOP_OCC2, "one": _lib.MZH_FLAG_KERNEL_ONE}[kernel]
    return f | {None: 0, 16: _lib.MZH_FLAG_COOP_TILE16, 32: _lib.MZH_FLAG_COOP_TILE32}[tile]


def pack_replay(replay):
    """recorded network outputs pi [B,S,6], reward [B,S], value [B,S] -> the kernel's replay records
    [S,B,8] (6 priors, reward, value per simulation and root; simulation-major, mzh_search_args.rp_sim)"""
    pi = torch.as_tensor(replay["pi"], dtype=torch.float32)
    rw = torch.as_tensor(replay["reward"], dtype=torch.float32).to(pi.device)
    va = torch.as_tensor(replay["value"], dtype=torch.float32).to(pi.device)
    return torch.cat([pi, rw[..., None], va[..., None]], -1).transpose(0, 1).contiguous()


# ---------------------------------------------------------------- environment (no engine needed)
def env_step(n_disks, max_steps, state, action, step_ctr, active, goal_peg=2, moved=None, obs=None, err=None,
             reward=None, done=None, illegal=None):
    """Batched TowersOfHanoi.step on device tensors (state/step_ctr/active updated in place;
    reward codes / done / illegal written to the given tensors or fresh ones)."""
    B = state.shape[0]
    dev = state.device
    reward = torch.empty(B, dtype=torch.int8, device=dev) if reward is None else reward
    done = torch.empty(B, dtype=torch.uint8, device=dev) if done is None else done
    illegal = torch.empty(B, dtype=torch.uint8, device=dev) if illegal is None else illegal
    check(_lib.lib().mzh_env_step(n_disks, goal_peg, max_steps, B, ptr(state), ptr(action), ptr(moved), ptr(obs),
                                  ptr(reward), ptr(done), ptr(illegal), ptr(step_ctr), ptr(active), ptr(err),
                                  _lib.stream_handle(dev)), "mzh_env_step")
    return reward, done, illegal


def legal_mask(n_disks, state):
    mask = torch.empty(state.shape[0], dtype=torch.uint8, device=state.device)
    check(_lib.lib().mzh_legal_mask(n_disks, state.shape[0], ptr(state), ptr(mask), _lib.stream_handle(state.device)),
          "mzh_legal_mask")
    return mask


def encode_obs(n_disks, state):
    obs = torch.empty((state.shape[0], 3 * n_disks), dtype=torch.float32, device=state.device)
    check(_lib.lib().mzh_encode_obs(n_disks, state.shape[0], ptr(state), ptr(obs), _lib.stream_handle(state.device)),
          "mzh_encode_obs")
    return obs


def hanoi_solver_batch(n_disks, state, goal_peg=2):
    moves = torch.empty(state.shape[0], dtype=torch.int32, device=state.device)
    check(_lib.lib().mzh_hanoi_solver(n_disks, goal_peg, state.shape[0], ptr(state), ptr(moves),
                                      _lib.stream_handle(state.device)), "mzh_hanoi_solver")
    return moves
