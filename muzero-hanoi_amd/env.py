"""TowersOfHanoi drop-in (reference: env/hanoi.py:11-151) + a batched form.

The public surface is the reference's: constructor, `states`, `moves`, `goal`, `oneH_s_size`,
`n_pegs`, `discs`, `max_steps`, `init_state_idx`, `c_state` / `oneH_c_state` (assignable, as
noise_injection_comparison.py:20-21 and permutation_importance.py:46-47 do), `step`, `reset`,
`random_reset`, `current_state`, `_move_allowed`.  Transitions, legality and the observation are
computed by the libmzh integer kernels (mzh_env_step / mzh_legal_mask / mzh_encode_obs).

`HanoiBatch` keeps B environments resident on the GPU for batched self-play.
"""
import itertools

import numpy as np
import torch

from . import _lib, engine
from .engine import require_device
from .staging import Packed

_REWARD = {0: 0, 1: 100, -1: -100 / 1000}  # codes of mzh_env_step -> the reference's rewards


class TowersOfHanoi:
    def __init__(self, N, max_steps, init_state_idx=0, goal_peg=2):
        require_device()
        self.discs = N
        self.n_pegs = 3
        self.states = list(itertools.product(list(range(self.n_pegs)), repeat=self.discs))
        self.oneH_s_size = self.discs * self.n_pegs
        self.goal = tuple([goal_peg] * self.discs)
        self.goal_peg = goal_peg
        self.init_state_idx = init_state_idx
        self.moves = list(itertools.permutations(list(range(self.n_pegs)), 2))
        self.max_steps = max_steps
        self.reset_check = False
        self.step_counter = 0
        self._dev = torch.device("cuda", torch.cuda.current_device())
        self._pk = None

    # ------------------------------------------------------------------ reference API
    def step(self, action):
        """env/hanoi.py:47-84 -> (one-hot obs float64[3N], rwd, done, illegal_move)."""
        assert self.reset_check, "Need to reset env before taking a step"
        action = int(action)
        if not 0 <= action < 6:
            raise IndexError("list index out of range")
        pk = self._launch_step(action=action)
        pk.to_host()
        return self._finish_step()

    def _launch_step(self, action=None, action_ptr=None):
        """stage the env's state and launch mzh_env_step on the current stream; the action either goes into
        the staging record or is read by the kernel from `action_ptr` (device-readable int32, e.g. the search's
        own action output: MCTS.run_mcts_step chains the two launches)"""
        pk = self._packed()
        h = pk.h
        h["state"][0] = self.c_state
        if action_ptr is None:
            h["action"][0] = action
        h["ctr"][0] = self.step_counter
        h["active"][0] = 1
        pk.to_device()
        q = self._ptrs
        _lib.check(_lib.lib().mzh_env_step(self.discs, self.goal_peg, self.max_steps, 1, q["state"],
                                           q["action"] if action_ptr is None else action_ptr, q["moved"], q["obs"],
                                           q["code"], q["done"], q["illegal"], q["ctr"], q["active"], None,
                                           _lib.stream_handle(self._dev)), "mzh_env_step")
        return pk

    def _finish_step(self):
        """the step's results from the staging record (after the synchronisation)"""
        h = self._pk.h
        self.c_state = tuple(int(x) for x in h["state"][0])
        self.step_counter, self.reset_check = int(h["ctr"][0]), bool(h["active"][0])
        rwd, done_b, illegal_b = _REWARD[int(h["code"][0])], bool(h["done"][0]), bool(h["illegal"][0])
        return h["obs"][0].astype(np.float64), rwd, done_b, illegal_b

    def reset(self):
        self.reset_check = True
        self.c_state = self.states[self.init_state_idx]
        self.oneH_c_state = self._encode(self.c_state)
        return self.oneH_c_state

    def random_reset(self):
        """env/hanoi.py:103-115: draws from the global NumPy RNG exactly like the reference."""
        self.reset_check = True
        while True:
            random_indx = np.random.randint(len(self.states))
            self.c_state = self.states[random_indx]
            if self.c_state != self.goal:
                break
        self.oneH_c_state = self._encode(self.c_state)
        return self.oneH_c_state

    def current_state(self):
        return list(self.c_state)

    def _discs_on_peg(self, peg):
        return [disc for disc in range(self.discs) if self.c_state[disc] == peg]

    def _move_allowed(self, move):
        mask = engine.legal_mask(self.discs, torch.tensor([list(self.c_state)], dtype=torch.uint8, device=self._dev))
        return bool((int(mask.item()) >> self.moves.index(tuple(move))) & 1)

    # ------------------------------------------------------------------ helpers
    def _packed(self):
        if self._pk is None:
            n = self.discs
            fields = [("state", torch.uint8, (1, n)), ("action", torch.int32, (1,)), ("ctr", torch.int32, (1,)),
                      ("active", torch.uint8, (1,)), ("moved", torch.uint8, (1, n)), ("obs", torch.float32, (1, 3 * n)),
                      ("code", torch.int8, (1,)), ("done", torch.uint8, (1,)), ("illegal", torch.uint8, (1,))]
            try:  # the kernel reads and writes the pinned staging buffer itself: one launch + one sync per step
                self._pk = Packed(fields, self._dev, zero_copy=True)
            except RuntimeError:  # no device address for pinned memory here: one copy each way
                self._pk = Packed(fields, self._dev)
            self._ptrs = self._pk.dptr  # fixed: the call passes them as is
        return self._pk

    def _packed_out2(self):
        """a second record of the step's outputs (MCTS.play_episode alternates output records between decisions)"""
        if getattr(self, "_pk2", None) is None:
            n = self.discs
            fields = [("moved", torch.uint8, (1, n)), ("obs", torch.float32, (1, 3 * n)), ("code", torch.int8, (1,)),
                      ("done", torch.uint8, (1,)), ("illegal", torch.uint8, (1,))]
            try:
                self._pk2 = Packed(fields, self._dev, zero_copy=True)
            except RuntimeError:
                self._pk2 = Packed(fields, self._dev)
        return self._pk2

    def _encode(self, state):
        st = torch.tensor([list(state)], dtype=torch.uint8, device=self._dev)
        return engine.encode_obs(self.discs, st)[0].to(torch.float64).cpu().numpy()


class HanoiBatch:
    """B independent TowersOfHanoi envs resident on one GPU (state [B,N] uint8, step counters,
    reset flags).  step() is one mzh_env_step launch; nothing leaves the device."""

    def __init__(self, N, max_steps, B, goal_peg=2, device=None):
        require_device()
        self.N, self.max_steps, self.B, self.goal_peg = N, max_steps, B, goal_peg
        self.device = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
        self.state = torch.zeros((B, N), dtype=torch.uint8, device=self.device)
        self.step_ctr = torch.zeros(B, dtype=torch.int32, device=self.device)
        self.active = torch.zeros(B, dtype=torch.uint8, device=self.device)
        self.err = torch.zeros(1, dtype=torch.int32, device=self.device)

    def reset(self, state_idx):
        """state_idx [B] -> reference state tuples (index = sum s[i] * 3^(N-1-i))."""
        idx = torch.as_tensor(state_idx, device=self.device).to(torch.int64)
        pw = 3 ** torch.arange(self.N - 1, -1, -1, device=self.device)
        self.state.copy_(((idx[:, None] // pw) % 3).to(torch.uint8))
        self.step_ctr.zero_()
        self.active.fill_(1)
        return self.obs()

    def obs(self):
        return engine.encode_obs(self.N, self.state)

    def step(self, action):
        obs = torch.empty((self.B, 3 * self.N), dtype=torch.float32, device=self.device)
        code, done, illegal = engine.env_step(self.N, self.max_steps, self.state, action.to(torch.int32).contiguous(),
                                              self.step_ctr, self.active, goal_peg=self.goal_peg, obs=obs, err=self.err)
        return obs, code, done, illegal

    def legal_mask(self):
        return engine.legal_mask(self.N, self.state)

    @staticmethod
    def reward_value(code):
        """int8 codes -> the reference's float rewards (0, 100, -0.1)"""
        out = torch.zeros(code.shape, dtype=torch.float64, device=code.device)
        out[code == 1] = 100.0
        out[code == -1] = -100 / 1000
        return out
