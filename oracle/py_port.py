"""Python restatement of the reference's per-node MCTS -- TEST INFRASTRUCTURE / CPU BASELINE ONLY.

The reference's Python files do not travel to the GPU box, so bench.py's `cpu_baseline` times
this from-scratch restatement of the same algorithm with the same costs: a pointer tree of Python
`Node` objects (MCTS/node.py:6-141), one batch-1 torch-CPU MLP call per simulation
(networks.py:71-116), fp64 Python-float statistics and NumPy's global RNG (MCTS/mcts.py:34-176).
tests/test_py_port.py pins it against the golden replay traces (bit-exact visits) and against the
reference's own end-to-end visit counts.
"""
import math

import numpy as np
import torch
import torch.nn.functional as F

WEIGHT_KEYS = [
    f"{net}.{layer}.{kind}"
    for net in ("representation_net", "dynamic_net", "rwd_net", "policy_net", "value_net")
    for layer in (0, 2)
    for kind in ("weight", "bias")
]


class PortNet:
    """Batch-1 torch-CPU MuZero network (networks.py:71-196) over a state_dict of arrays."""

    def __init__(self, weights, td=True):
        self.w = {k: torch.as_tensor(np.asarray(weights[k], np.float32)) for k in WEIGHT_KEYS}
        self.td = td
        self.support_size = 33 if td else 1
        self.num_actions = 6

    def _mlp(self, name, x):
        w = self.w
        return F.linear(F.relu(F.linear(x, w[f"{name}.0.weight"], w[f"{name}.0.bias"])),
                        w[f"{name}.2.weight"], w[f"{name}.2.bias"])

    @staticmethod
    def _norm(h):
        mn = h.min(dim=-1, keepdim=True)[0]
        mx = h.max(dim=-1, keepdim=True)[0]
        return (h - mn) / (mx - mn + 1e-8)

    def _to_value(self, logits):
        if not self.td:
            return logits
        probs = torch.softmax(logits, dim=-1)
        support = torch.linspace(-16, 16, 33)
        x = torch.sum(probs * support.expand_as(probs), dim=-1, keepdim=True)
        eps = 1e-3
        z = torch.sqrt(1 + 4 * eps * (eps + 1 + torch.abs(x))) / 2 / eps - 1 / 2 / eps
        return torch.sign(x) * (torch.square(z) - 1)

    @torch.no_grad()
    def initial_inference(self, x):
        h = self._norm(self._mlp("representation_net", x))
        pi = F.softmax(self._mlp("policy_net", h), dim=-1)
        v = self._to_value(self._mlp("value_net", h))
        return h.numpy(), 0.0, pi.numpy(), v.squeeze(0).item()

    @torch.no_grad()
    def recurrent_inference(self, h, a):
        hr = self._mlp("dynamic_net", torch.cat([h, a], dim=-1))
        r = self._to_value(self._mlp("rwd_net", hr))
        h2 = self._norm(hr)
        pi = F.softmax(self._mlp("policy_net", h2), dim=-1)
        v = self._to_value(self._mlp("value_net", h2))
        return h2.numpy(), r.squeeze(0).item(), pi.numpy(), v.squeeze(0).item()


class ReplayNet:
    """Replays recorded network outputs (tree-only parity)."""

    def __init__(self, root_pi, pi, rwd, value):
        self.root_pi, self.pi, self.rwd, self.value = root_pi, pi, rwd, value
        self.num_actions = 6
        self.k = 0

    def initial_inference(self, x):
        self.k = 0
        return None, 0.0, np.asarray(self.root_pi, np.float32), 0.0

    def recurrent_inference(self, h, a):
        k = self.k
        self.k += 1
        return None, float(self.rwd[k]), np.asarray(self.pi[k], np.float32), float(self.value[k])


class MinMaxStats:
    def __init__(self):
        self.maximum = -float("inf")
        self.minimum = float("inf")

    def update(self, value):
        self.maximum = max(self.maximum, value)
        self.minimum = min(self.minimum, value)

    def normalize(self, value):
        if self.maximum > self.minimum:
            return (value - self.minimum) / (self.maximum - self.minimum)
        return value


class Node:
    __slots__ = ("prior", "move", "parent", "is_expanded", "N", "W", "rwd", "h_state", "children")

    def __init__(self, prior=None, move=None, parent=None):
        self.prior, self.move, self.parent = prior, move, parent
        self.is_expanded = False
        self.N = 0
        self.W = 0.0
        self.rwd = 0.0
        self.h_state = None
        self.children = []

    def expand(self, prior, h_state, reward):
        self.h_state = h_state
        self.rwd = reward
        self.children = [Node(prior=prior[a], move=a, parent=self) for a in range(prior.shape[0])]
        self.is_expanded = True

    def Q(self):
        return 0.0 if self.N == 0 else self.W / self.N

    def backup(self, value, discount, mm):
        cur = self
        while cur is not None:
            cur.W += value
            cur.N += 1
            mm.update(cur.rwd + discount * cur.Q())
            value = cur.rwd + discount * value
            cur = cur.parent

    def best_child(self, pb_c_base, pb_c_init, discount, mm):
        q = np.array([mm.normalize(c.rwd + discount * c.Q()) if c.N > 0 else 0 for c in self.children], np.float32)
        u = np.array([c.prior * ((math.log((self.N + pb_c_base + 1) / pb_c_base) + pb_c_init)
                                 * math.sqrt(self.N) / (c.N + 1)) for c in self.children], np.float32)
        ucb = q + u
        return self.children[np.random.choice(np.where(ucb == ucb.max())[0])]


class PortMCTS:
    def __init__(self, discount, root_dirichlet_alpha, n_simulations, root_exploration_eps=0.25):
        self.mm = MinMaxStats()
        self.discount = discount
        self.alpha = root_dirichlet_alpha
        self.eps = root_exploration_eps
        self.n_simulations = n_simulations

    def run_mcts(self, state, network, temperature, deterministic):
        x = torch.from_numpy(state).to(dtype=torch.float32)
        h, rwd, prior, _ = network.initial_inference(x)
        root = Node(prior=0.0)
        if not deterministic and self.alpha > 0.0 and self.eps > 0.0:
            noise = np.random.dirichlet(np.ones_like(prior) * self.alpha)
            prior = (1 - self.eps) * prior + self.eps * noise
        root.expand(prior, h, rwd)
        for _ in range(self.n_simulations):
            node = root
            while node.is_expanded:
                node = node.best_child(19652, 1.25, self.discount, self.mm)
            hp = None if node.parent.h_state is None else torch.from_numpy(node.parent.h_state)
            a = F.one_hot(torch.tensor([node.move]), num_classes=6).squeeze().float()
            h, r, pi, v = network.recurrent_inference(hp, a)
            node.expand(pi, h, r)
            node.backup(v, self.discount, self.mm)
        visits = np.array([c.N for c in root.children], np.int32)
        vc = visits.astype(np.int64)
        if temperature > 0.0:
            vc = np.power(vc, max(1.0, min(5.0, 1.0 / temperature)))
        pi = vc / np.sum(vc)
        if deterministic:
            action = int(np.argmax(visits))
        else:
            action = int(np.random.choice(np.arange(6), p=pi))
        return action, pi, root.Q(), visits


class PortHanoi:
    """env/hanoi.py:11-151 + utils.py:9-25 restated in the reference's own form (tuples, list scans, NumPy one-hot):
    the host-side TowersOfHanoi.step the reference runs, as the CPU baseline of the env step
    (tools/bench_env.py).  tests/test_py_port.py checks it against the exhaustive env fixtures."""

    def __init__(self, N, max_steps, init_state_idx=0, goal_peg=2):
        import itertools

        self.discs, self.n_pegs = N, 3
        self.states = list(itertools.product(list(range(3)), repeat=N))
        self.goal = tuple([goal_peg] * N)
        self.init_state_idx = init_state_idx
        self.moves = list(itertools.permutations(list(range(3)), 2))
        self.max_steps = max_steps
        self.reset_check = False
        self.step_counter = 0

    @staticmethod
    def one_hot(x, n):
        m = np.zeros((len(x), n))
        m[np.arange(len(x)), x] = 1
        return m.reshape(-1)

    def reset(self):
        self.reset_check = True
        self.c_state = self.states[self.init_state_idx]
        return self.one_hot(self.c_state, 3)

    def _discs_on_peg(self, peg):
        return [d for d in range(self.discs) if self.c_state[d] == peg]

    def _move_allowed(self, move):
        f, t = self._discs_on_peg(move[0]), self._discs_on_peg(move[1])
        if f:
            return (min(t) > min(f)) if t else True
        return False

    def _get_moved_state(self, move):
        if self._move_allowed(move):
            d = min(self._discs_on_peg(move[0]))
        s = list(self.c_state)
        s[d] = move[1]
        return tuple(s)

    def step(self, action):
        assert self.reset_check, "Need to reset env before taking a step"
        move = self.moves[action]
        illegal = not self._move_allowed(move)
        self.step_counter += 1
        if not illegal:
            moved = self._get_moved_state(move)
            if moved != self.goal:
                rwd, done = 0, False
                self.c_state = moved
            else:
                rwd, done = 100, True
                self.reset_check = False
                self.step_counter = 0
        else:
            rwd, moved, done = -100 / 1000, self.c_state, False
        if self.step_counter == self.max_steps:
            done = True
            self.reset_check = False
            self.step_counter = 0
        return self.one_hot(moved, 3), rwd, done, illegal
