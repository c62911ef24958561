"""MCTS drop-in (reference: MCTS/mcts.py:8-176, MCTS/node.py, MCTS/utils_mcts.py).

`MCTS.run_mcts(state, network, temperature, deterministic)` keeps the reference's signature,
return types, RNG consumption (global legacy NumPy stream, see rng.py), MinMaxStats persistence
across calls on one instance (mcts.py:23) and `return_latent_actions`.  The whole search -- root
inference, every simulation's select / MLP expansion / backup, and the play policy -- is one
fused libmzh kernel launch on the GPU (mzh_search).

`MCTS.run_batch(states, ...)` runs B independent searches in one launch (each root with its own
MinMaxStats, i.e. B fresh single-root searches), the form the bench and batched self-play use.
"""
import ctypes
import warnings

import numpy as np
import torch

from . import _lib
from . import rng as _rng
from .networks import engine_for
from .staging import Packed

_ENV_REWARD = {0: 0, 1: 100, -1: -100 / 1000}  # mzh_env_step codes -> the reference's rewards (env.py)


_REPLAY_ENGINES = {}


def _replay_engine(n_disks, n_sims):
    from .engine import Engine

    eng = _REPLAY_ENGINES.get(n_disks)
    if eng is None or eng.max_sims < n_sims:
        eng = Engine(n_disks, max(n_sims, 64), 1, 33)
        _REPLAY_ENGINES[n_disks] = eng
    return eng


class MinMaxStats(object):
    """utils_mcts.py:1-16 (host mirror; the device carries the same two doubles)."""

    def __init__(self, min_value_bound=None, max_value_bound=None):
        self.maximum = min_value_bound if min_value_bound else -float("inf")
        self.minimum = max_value_bound if max_value_bound else float("inf")

    def update(self, value):
        self.maximum = max(self.maximum, value)
        self.minimum = min(self.minimum, value)

    def normalize(self, value):
        if self.maximum > self.minimum:
            return (value - self.minimum) / (self.maximum - self.minimum)
        return value


class RecordedNetwork:
    """Network duck type whose outputs were recorded (tree-only mode, mzh_search_replay).

    calls: list of dicts, one per run_mcts call, each with root_pi [6] and, per simulation,
    pi [S,6], reward [S], value [S] (fp32 values, exactly what the network returned)."""

    def __init__(self, calls, n_disks, num_actions=6):
        self.calls = list(calls)
        self.n_disks = n_disks
        self.num_actions = num_actions
        self.cursor = 0

    def next_call(self):
        c = self.calls[self.cursor]
        self.cursor += 1
        return c


class MCTS:
    def __init__(self, discount, root_dirichlet_alpha, n_simulations, batch_s, device, h_dim=64, clip_grad=True,
                 root_exploration_eps=0.25, known_bounds=[]):
        self.min_max_stats = MinMaxStats()
        self.pb_c_base = 19652  # baked into the kernel's UCB table (mzh_create)
        self.pb_c_init = 1.25
        self.discount = discount
        self.root_dirichlet_alpha = root_dirichlet_alpha
        self.root_exploration_eps = root_exploration_eps
        self.n_simulations = n_simulations
        self.batch_s = batch_s
        self.dev = device
        self.latent_actions = []
        self.np1_ucb = False  # True: NumPy-1.x UCB rounding (the reference's numpy==1.25.2 pin)
        self.last_extra_ties = 0

    # ------------------------------------------------------------------ reference API
    def run_mcts(self, state, network, temperature, deterministic):
        """mcts.py:34-126 -> (action int, pi np.float64[6], root Q float)."""
        if self.pb_c_base != 19652 or self.pb_c_init != 1.25:
            raise NotImplementedError("libmzh bakes pb_c_base=19652, pb_c_init=1.25 (mcts.py:24-25)")
        S = int(self.n_simulations)
        # the reference raises for a bad temperature inside generate_play_policy (mcts.py:113,
        # 163-166): after the whole search (Dirichlet draw, argmax tie draws, MinMaxStats updates,
        # latent_actions) and before the action draw (mcts.py:120).  So the search runs, its state
        # is kept, no action uniform is drawn, then the ValueError.
        bad_t = not 0.0 <= temperature <= 1.0
        if not isinstance(network, RecordedNetwork):
            return self._run_mcts_fast(state, network, temperature, deterministic, S, bad_t)
        noise, tie, u = _rng.predraw(1, deterministic=deterministic, alpha=self.root_dirichlet_alpha,
                                     eps=self.root_exploration_eps, draw_action=not bad_t)
        if bad_t:
            deterministic, temperature_k = True, 0.0  # the kernel's policy output is discarded
        else:
            temperature_k = temperature
        replay = None
        if isinstance(network, RecordedNetwork):
            eng = _replay_engine(network.n_disks, S)
            call = network.next_call()
            replay = {k: torch.as_tensor(np.asarray(call[k], np.float32)).to(eng.device)[None]
                      for k in ("root_pi", "pi", "reward", "value")}
        else:
            eng = engine_for(network, S, 1)
        dev = eng.device
        x = np.asarray(state).reshape(-1)
        # inputs down in one copy, every output back in one copy (staging.Packed)
        pin, pout = self._packed(eng, S, x.size, replay is not None)
        h = pin.h
        h["obs"][0] = x
        h["mm"][0] = (self.min_max_stats.maximum, self.min_max_stats.minimum)
        h["tie"][:] = tie
        if noise is not None:
            h["noise"][:] = noise
        if u is not None:
            h["u"][:] = u
        pin.to_device()
        d = pin.d
        out = eng.search(S, obs=None if replay else d["obs"], replay=replay, tie_idx=d["tie"],
                         noise=None if noise is None else d["noise"], action_u=None if u is None else d["u"],
                         minmax_in=d["mm"], temperature=float(temperature_k), deterministic=bool(deterministic),
                         discount=float(self.discount), eps=float(self.root_exploration_eps), np1_ucb=self.np1_ucb,
                         out=dict(pout.d))
        pout.to_host()
        host = pout.h
        self.min_max_stats.maximum = float(host["minmax"][0, 0])
        self.min_max_stats.minimum = float(host["minmax"][0, 1])
        L = int(host["latent_len"][0])
        self._latent_host = [int(m) for m in host["latent"][0, :L]]  # tensors made on first access
        self.last_extra_ties = int(host["extra_ties"][0])
        if self.last_extra_ties:
            warnings.warn("search met an argmax tie beyond the root's first selection: the NumPy RNG stream "
                          "now differs from the reference's", RuntimeWarning)
        if bad_t:
            raise ValueError(f"Expect `temperature` to be in the range [0.0, 1.0], got {temperature}")
        return int(host["action"][0]), host["pi"][0].astype(np.float64), float(host["root_q"][0])

    def _run_mcts_fast(self, state, network, temperature, deterministic, S, bad_t):
        """run_mcts for a network: the draws go straight into the pinned staging buffer (rng.predraw_into),
        and the search arguments -- every device pointer of the staging buffers fixed -- are built once per
        (engine, S, observation width) and only their scalars and optional pointers set per call"""
        eng, pout = self._launch_fast(state, network, temperature, deterministic, S, bad_t)
        pout.to_host()
        return self._finish_fast(pout, temperature, bad_t)

    def _launch_fast(self, state, network, temperature, deterministic, S, bad_t):
        eng = engine_for(network, S, 1)
        x = np.asarray(state).reshape(-1)
        pin, pout, a, addrs = self._prepared(eng, S, x.size)
        h = pin.h
        noisy, drew_u = _rng.predraw_into(h["noise"], h["tie"], h["u"], deterministic=deterministic,
                                          alpha=self.root_dirichlet_alpha, eps=self.root_exploration_eps,
                                          draw_action=not bad_t, addrs=addrs)
        if bad_t:
            deterministic, temperature_k = True, 0.0  # the kernel's policy output is discarded
        else:
            temperature_k = temperature
        h["obs"][0] = x
        mm = h["mm"][0]
        mm[0] = self.min_max_stats.maximum
        mm[1] = self.min_max_stats.minimum
        pin.to_device()
        a.n_sims = S
        a.discount = float(self.discount)
        a.eps = float(self.root_exploration_eps)
        a.temperature = float(temperature_k)
        a.deterministic = 1 if deterministic else 0
        a.flags = _lib.MZH_FLAG_NP1_UCB if self.np1_ucb else 0
        d = self._pk_ptrs
        a.noise = d["noise"] if noisy else None
        a.action_u = d["u"] if drew_u else None
        pt = eng.pow_table(S, float(temperature_k))
        a.pow_table = None if pt is None else pt.data_ptr()
        _lib.check(_lib.lib().mzh_search(eng._h, ctypes.byref(a), _lib.stream_handle(eng.device)), "mzh_search")
        return eng, pout

    def _finish_fast(self, pout, temperature, bad_t):
        host = pout.h
        self.min_max_stats.maximum = float(host["minmax"][0, 0])
        self.min_max_stats.minimum = float(host["minmax"][0, 1])
        L = int(host["latent_len"][0])
        self._latent_host = [int(m) for m in host["latent"][0, :L]]  # tensors made on first access
        self.last_extra_ties = int(host["extra_ties"][0])
        if self.last_extra_ties:
            warnings.warn("search met an argmax tie beyond the root's first selection: the NumPy RNG stream "
                          "now differs from the reference's", RuntimeWarning)
        if bad_t:
            raise ValueError(f"Expect `temperature` to be in the range [0.0, 1.0], got {temperature}")
        return int(host["action"][0]), host["pi"][0].astype(np.float64), float(host["root_q"][0])

    def run_mcts_step(self, state, network, temperature, deterministic, env):
        """run_mcts(state, ...) followed by env.step(action) (Muzero._play_game's pair of calls,
        Muzero.py:165-175) as two chained launches and ONE synchronisation: the env kernel reads the
        action the search kernel wrote.  The same draws, results and env state as the two calls.
        Returns (action, pi, root_Q, env.step's tuple), or None where run_mcts itself must run (a replayed
        network, a temperature it refuses, an env not reset, other UCB constants) -- the caller then makes
        the two calls; with staging through copies or the env on another device the two run one after
        the other here."""
        S = int(self.n_simulations)
        if (isinstance(network, RecordedNetwork) or not 0.0 <= temperature <= 1.0 or not env.reset_check
                or self.pb_c_base != 19652 or self.pb_c_init != 1.25):
            return None
        eng, pout = self._launch_fast(state, network, temperature, deterministic, S, False)
        pk = env._packed()
        if pout.zero_copy and pk.zero_copy and torch.device(eng.device) == env._dev:
            env._launch_step(action_ptr=pout.dptr["action"])
            _lib.synchronize(eng.device)
            action, pi, q = self._finish_fast(pout, temperature, False)
            return action, pi, q, env._finish_step()
        pout.to_host()  # staging with copies: the two calls one after the other
        action, pi, q = self._finish_fast(pout, temperature, False)
        return action, pi, q, env.step(action)

    def play_episode(self, env, network, temperature, deterministic):
        """Muzero._play_game's decision loop (run_mcts then env.step until done, Muzero.py:165-186) with the
        decisions pipelined on the device: decision k+1's search reads its observation from decision k's env
        kernel and its MinMaxStats from decision k's search, so it is launched (with its env step) BEFORE the
        host waits for decision k -- the GPU runs decision after decision while the host records the last one.
        When decision k ends the episode, the speculative decision k+1 is discarded: its env step meets an
        inactive env (left untouched, as the kernel's AssertionError path does) and the NumPy stream is put back
        to where decision k left it.  The same draws, results, MinMaxStats and env state as the per-decision calls
        (tests/test_selfplay.py).  Returns (steps, obs list, actions, rewards, pis, root Qs) or None where the
        pipeline does not apply (then the caller makes the per-decision calls)."""
        S = int(self.n_simulations)
        rs = np.random.mtrand._rand
        bg = rs._bit_generator
        if (isinstance(network, RecordedNetwork) or not 0.0 <= temperature <= 1.0 or not env.reset_check
                or self.pb_c_base != 19652 or self.pb_c_init != 1.25 or type(bg).__name__ != "MT19937"
                or (_rng.uses_noise(deterministic, self.root_dirichlet_alpha, self.root_exploration_eps)
                    and not 0.0 < float(self.root_dirichlet_alpha) <= 1.0)):
            return None
        eng = engine_for(network, S, 1)
        x0 = np.asarray(env.oneH_c_state if hasattr(env, "oneH_c_state") else None)
        sets = self._prepared2(eng, S, env.discs * 3)
        ek, eo = env._packed(), env._packed_out2()
        if not all(p.zero_copy for st in sets for p in st[:2]) or not (ek.zero_copy and eo.zero_copy) \
                or torch.device(eng.device) != env._dev or x0.shape != (env.discs * 3,):
            return None
        stream = _lib.stream_handle(eng.device)
        L = _lib.lib()
        pt = eng.pow_table(S, float(temperature))
        flags = _lib.MZH_FLAG_NP1_UCB if self.np1_ucb else 0
        outs = [(ek.h, ek.dptr), (eo.h, eo.dptr)]  # env output records, alternating
        q = ek.dptr  # state / ctr / active: one record, updated in place decision after decision
        eh = ek.h
        eh["state"][0] = env.c_state
        eh["ctr"][0] = env.step_counter
        eh["active"][0] = 1
        mt = ctypes.c_char * 2500  # struct mt19937_state {uint32 key[624]; int pos}
        saved = mt()
        st_addr = bg.ctypes.state_address
        evs = [torch.cuda.Event(), torch.cuda.Event()]

        def launch(k):
            pin, pout, a, addrs = sets[k % 2]
            h = pin.h
            noisy, drew_u = _rng.predraw_into(h["noise"], h["tie"], h["u"], deterministic=deterministic,
                                              alpha=self.root_dirichlet_alpha, eps=self.root_exploration_eps,
                                              draw_action=True, addrs=addrs)
            if k == 0:
                h["obs"][0] = x0
                h["mm"][0] = (self.min_max_stats.maximum, self.min_max_stats.minimum)
                a.obs, a.minmax_in = pin.dptr["obs"], pin.dptr["mm"]
            else:  # the previous decision's env observation and search MinMaxStats, on the device
                a.obs = outs[(k - 1) % 2][1]["obs"]
                a.minmax_in = sets[(k - 1) % 2][1].dptr["minmax"]
            a.n_sims, a.discount, a.eps = S, float(self.discount), float(self.root_exploration_eps)
            a.temperature, a.deterministic, a.flags = float(temperature), 1 if deterministic else 0, flags
            a.noise = pin.dptr["noise"] if noisy else None
            a.action_u = pin.dptr["u"] if drew_u else None
            a.pow_table = None if pt is None else pt.data_ptr()
            _lib.check(L.mzh_search(eng._h, ctypes.byref(a), stream), "mzh_search")
            o = outs[k % 2][1]
            _lib.check(L.mzh_env_step(env.discs, env.goal_peg, env.max_steps, 1, q["state"], pout.dptr["action"],
                                      o["moved"], o["obs"], o["code"], o["done"], o["illegal"], q["ctr"], q["active"],
                                      None, stream), "mzh_env_step")
            evs[k % 2].record(torch.cuda.current_stream(eng.device))

        obs_l, act_l, rwd_l, pi_l, q_l = [x0.astype(np.float64)], [], [], [], []
        launch(0)
        k = 0
        while True:
            ctypes.memmove(saved, st_addr, 2500)  # the stream before the speculative next decision's draws
            launch(k + 1)
            evs[k % 2].synchronize()
            pout = sets[k % 2][1]
            ph, oh = pout.h, outs[k % 2][0]
            self.min_max_stats.maximum = float(ph["minmax"][0, 0])
            self.min_max_stats.minimum = float(ph["minmax"][0, 1])
            n = int(ph["latent_len"][0])
            self._latent_host = [int(m) for m in ph["latent"][0, :n]]
            self.last_extra_ties = int(ph["extra_ties"][0])
            if self.last_extra_ties:
                warnings.warn("search met an argmax tie beyond the root's first selection: the NumPy RNG stream "
                              "now differs from the reference's", RuntimeWarning)
            act_l.append(int(ph["action"][0]))
            pi_l.append(ph["pi"][0].astype(np.float64))
            q_l.append(float(ph["root_q"][0]))
            rwd_l.append(_ENV_REWARD[int(oh["code"][0])])
            done = bool(oh["done"][0])
            if done:
                ctypes.memmove(st_addr, saved, 2500)  # the discarded decision's draws never happened
                evs[(k + 1) % 2].synchronize()  # it ran on an inactive env: state, counter untouched
                break
            obs_l.append(oh["obs"][0].astype(np.float64))
            k += 1
        env.c_state = tuple(int(v) for v in eh["state"][0])
        env.step_counter, env.reset_check = int(eh["ctr"][0]), bool(eh["active"][0])
        return k + 1, obs_l, act_l, rwd_l, pi_l, q_l

    def _prepared2(self, eng, S, in_dim):
        """two sets of zero-copy staging buffers and SearchArgs (play_episode's pipeline alternates them)"""
        key = (id(eng), S, in_dim)
        if getattr(self, "_args2_key", None) != key:
            sets = []
            for _ in range(2):
                fin = [("obs", torch.float32, (1, in_dim)), ("noise", torch.float64, (1, 6)),
                       ("tie", torch.int32, (1,)), ("u", torch.float64, (1,)), ("mm", torch.float64, (1, 2))]
                fout = [("visits", torch.int32, (1, 6)), ("root_q", torch.float64, (1,)),
                        ("minmax", torch.float64, (1, 2)), ("extra_ties", torch.int32, (1,)),
                        ("action", torch.int32, (1,)), ("pi", torch.float64, (1, 6)),
                        ("latent", torch.int32, (1, S + 1)), ("latent_len", torch.int32, (1,)),
                        ("sel_steps", torch.int32, (1,))]
                try:
                    pin, pout = Packed(fin, eng.device, zero_copy=True), Packed(fout, eng.device, zero_copy=True)
                except RuntimeError:
                    pin, pout = Packed(fin, eng.device), Packed(fout, eng.device)
                a = _lib.SearchArgs()
                a.B = 1
                a.tie_idx = pin.dptr["tie"]
                o = pout.dptr
                for k, f in (("visits", "visits"), ("root_q", "root_q"), ("minmax_out", "minmax"),
                             ("extra_ties", "extra_ties"), ("action", "action"), ("pi", "pi"), ("latent", "latent"),
                             ("latent_len", "latent_len"), ("sel_steps", "sel_steps")):
                    setattr(a, k, o[f])
                h = pin.h
                sets.append((pin, pout, a, (h["noise"].ctypes.data, h["tie"].ctypes.data, h["u"].ctypes.data)))
            self._sets2 = sets
            self._args2_key = key
        return self._sets2

    def _prepared(self, eng, S, in_dim):
        """zero-copy staging buffers (the search kernel reads its inputs from and writes its outputs to pinned
        host memory: a call is one launch and one synchronisation) and a SearchArgs holding their device
        addresses, cached per (engine, S, observation width)"""
        key = (id(eng), S, in_dim)
        if getattr(self, "_args_key", None) != key:
            fin = [("obs", torch.float32, (1, in_dim)), ("noise", torch.float64, (1, 6)), ("tie", torch.int32, (1,)),
                   ("u", torch.float64, (1,)), ("mm", torch.float64, (1, 2))]
            fout = [("visits", torch.int32, (1, 6)), ("root_q", torch.float64, (1,)), ("minmax", torch.float64, (1, 2)),
                    ("extra_ties", torch.int32, (1,)), ("action", torch.int32, (1,)), ("pi", torch.float64, (1, 6)),
                    ("latent", torch.int32, (1, S + 1)), ("latent_len", torch.int32, (1,)),
                    ("sel_steps", torch.int32, (1,))]
            try:
                pin, pout = Packed(fin, eng.device, zero_copy=True), Packed(fout, eng.device, zero_copy=True)
            except RuntimeError:  # no device address for pinned memory here: one copy each way
                pin, pout = Packed(fin, eng.device), Packed(fout, eng.device)
            d, o = pin.dptr, pout.dptr
            self._pk_ptrs = d
            a = _lib.SearchArgs()
            a.B = 1
            a.obs = d["obs"]
            a.tie_idx = d["tie"]
            a.minmax_in = d["mm"]
            for k, f in (("visits", "visits"), ("root_q", "root_q"), ("minmax_out", "minmax"),
                         ("extra_ties", "extra_ties"), ("action", "action"), ("pi", "pi"), ("latent", "latent"),
                         ("latent_len", "latent_len"), ("sel_steps", "sel_steps")):
                setattr(a, k, o[f])
            h = pin.h
            self._prep = (pin, pout)
            self._args = a
            self._addrs = (h["noise"].ctypes.data, h["tie"].ctypes.data, h["u"].ctypes.data)
            self._args_key = key
        return self._prep[0], self._prep[1], self._args, self._addrs

    def return_latent_actions(self):
        return self.latent_actions

    @property
    def latent_actions(self):
        """mcts.py:79, 84-86: the last simulation's path as [LongTensor[1]] on the MCTS device"""
        if self._latent_host is not None:
            self._latent = [torch.tensor([m], dtype=torch.long, device=self.dev) for m in self._latent_host]
            self._latent_host = None
        return self._latent

    @latent_actions.setter
    def latent_actions(self, value):
        self._latent = value
        self._latent_host = None

    def _packed(self, eng, S, in_dim, replay):
        key = (id(eng), S, in_dim, replay)
        if getattr(self, "_pk_key", None) != key:
            dev = eng.device
            self._pk_in = Packed([("obs", torch.float32, (1, in_dim)), ("noise", torch.float64, (1, 6)),
                                  ("tie", torch.int32, (1,)), ("u", torch.float64, (1,)),
                                  ("mm", torch.float64, (1, 2))], dev)
            self._pk_out = Packed([("visits", torch.int32, (1, 6)), ("root_q", torch.float64, (1,)),
                                   ("minmax", torch.float64, (1, 2)), ("extra_ties", torch.int32, (1,)),
                                   ("action", torch.int32, (1,)), ("pi", torch.float64, (1, 6)),
                                   ("latent", torch.int32, (1, S + 1)), ("latent_len", torch.int32, (1,)),
                                   ("sel_steps", torch.int32, (1,))], dev)
            self._pk_key = key
        return self._pk_in, self._pk_out

    def add_dirichlet_noise(self, prob, eps=0.25, alpha=0.25):
        """mcts.py:132-152 (host form, for callers that use it directly)."""
        if not isinstance(prob, np.ndarray) or prob.dtype not in (np.float32, np.float64):
            raise ValueError(f"Expect `prob` to be a numpy.array, got {prob}")
        noise = np.random.dirichlet(np.ones_like(prob) * alpha)
        return (1 - eps) * prob + eps * noise

    def generate_play_policy(self, visits_count, temperature):
        """mcts.py:154-176 (host form; the search kernel computes the same policy on device)."""
        if not 0.0 <= temperature <= 1.0:
            raise ValueError(f"Expect `temperature` to be in the range [0.0, 1.0], got {temperature}")
        visits_count = np.asarray(visits_count, dtype=np.int64)
        if temperature > 0.0:
            visits_count = np.power(visits_count, max(1.0, min(5.0, 1.0 / temperature)))
        return visits_count / np.sum(visits_count)

    # ------------------------------------------------------------------ batched form
    def run_batch(self, states, network, temperature, deterministic, *, legacy_rng=True, seed=None, minmax=None,
                  out=None):
        """B independent run_mcts calls in one kernel launch.

        states: [B, 3N] observations (numpy or tensor).  With legacy_rng the draws come from the
        global NumPy stream in the order B sequential run_mcts calls would consume them (each
        root with a fresh MinMaxStats, unless `minmax` [B,2] is given); otherwise a vectorised
        Generator(seed) is used.  Returns device tensors (visits, action, pi, root_q, minmax, ...).
        """
        S = int(self.n_simulations)
        obs = torch.as_tensor(states)
        B = obs.shape[0]
        if legacy_rng:
            noise, tie, u = _rng.predraw(B, deterministic=deterministic, alpha=self.root_dirichlet_alpha,
                                         eps=self.root_exploration_eps)
        else:
            noise, tie, u = _rng.synthetic_draws(B, deterministic=deterministic, alpha=self.root_dirichlet_alpha,
                                                 eps=self.root_exploration_eps, seed=seed or 0)
        eng = engine_for(network, S, B)
        dev = eng.device
        t = lambda a: None if a is None else torch.as_tensor(a).to(dev)
        return eng.search(S, obs=obs.to(dev, torch.float32), tie_idx=t(tie), noise=t(noise), action_u=t(u),
                          minmax_in=t(minmax), temperature=float(temperature), deterministic=bool(deterministic),
                          discount=float(self.discount), eps=float(self.root_exploration_eps),
                          np1_ucb=self.np1_ucb, out=out)
