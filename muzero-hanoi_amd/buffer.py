"""Replay buffer drop-in (reference: buffer.py:5-139, `Buffer`).

Transitions are already organised for `unroll_n_steps` (Muzero.organise_transitions). The
reference keeps them in host NumPy arrays and copies every sampled batch to the device; here the
five transition arrays live on the training device (HBM on the MI355X: a ring of 10^8 transitions
is a few GB of 288) and a sampled batch is an on-device gather.  Only what the reference's RNG
stream depends on stays on the host: the priorities, from which `np.random.choice` draws the
indices exactly as the reference does (same global legacy stream, same calls), so a seeded run
samples the same transitions.
"""
import numpy as np
import torch


class Buffer:
    def __init__(self, size, unroll_n_steps, d_state, n_action, device, priority_exponent=1,
                 importance_sampling_exponent=0):
        self.dev = torch.device(device)
        self._priority_exponent = priority_exponent
        self._importance_sampling_exponent = importance_sampling_exponent
        self.size = size
        self.unroll_n_steps = unroll_n_steps
        self.n_action = n_action
        self.d_state = d_state
        U, dev = unroll_n_steps, self.dev
        self.states = torch.zeros((size, d_state), dtype=torch.float32, device=dev)  # initial state only
        self.rwds = torch.zeros((size, U), dtype=torch.float32, device=dev)
        self.actions = torch.zeros((size, U), dtype=torch.int64, device=dev)
        self.pi_probs = torch.zeros((size, U, n_action), dtype=torch.float32, device=dev)
        self.mc_returns = torch.zeros((size, U), dtype=torch.float32, device=dev)
        self.priorities = np.zeros((size,), dtype=np.float32)  # host: drives np.random.choice
        self.ptr = 0
        self.is_full = False

    def _ring_write(self, dst, src):
        """buffer.py:44-60: write n rows at ptr, the overflow wrapping to the start"""
        n = src.shape[0]
        head = min(n, self.size - self.ptr)
        dst[self.ptr:self.ptr + head] = src[:head]
        if head < n:
            dst[:n - head] = src[head:]

    def add(self, states, rwds, actions, pi_probs, mc_returns, priorities):
        """buffer.py:62-77"""
        n = states.shape[0]
        assert n <= self.size
        as_dev = lambda x, dt: torch.as_tensor(np.asarray(x), dtype=dt).to(self.dev)
        self._ring_write(self.states, as_dev(states, torch.float32))
        self._ring_write(self.rwds, as_dev(rwds, torch.float32))
        self._ring_write(self.actions, as_dev(actions, torch.int64))
        self._ring_write(self.pi_probs, as_dev(pi_probs, torch.float32))
        self._ring_write(self.mc_returns, as_dev(mc_returns, torch.float32))
        self._ring_write(self.priorities, np.asarray(priorities, np.float32))
        if self.ptr + n >= self.size:
            self.is_full = True
        self.ptr = (self.ptr + n) % self.size

    def _gather(self, indx):
        i = torch.as_tensor(indx, dtype=torch.int64).to(self.dev)
        return self.states[i], self.rwds[i], self.actions[i], self.pi_probs[i], self.mc_returns[i]

    def uniform_sample(self, batch_s):
        """buffer.py:79-87.  np.random.choice(np.arange(n), batch_s, replace=True) draws
        RandomState.randint(0, n, batch_s); the same call without building the index array."""
        indx = np.random.randint(0, len(self), size=batch_s).astype(np.int64)
        return self._gather(indx)

    def priority_sample(self, batch_s):
        """buffer.py:89-112: P(i) = p_i^a / sum_j p_j^a, importance weights ((1/size)/P(i))^b / max"""
        num = len(self)
        p = self.priorities[:num] ** self._priority_exponent
        probs = p / np.sum(p)
        # np.random.choice(np.arange(num), batch_s, replace=True, p=probs) as RandomState.choice
        # computes it -- float64 cdf, cdf /= cdf[-1], one random_sample per index, right-sided
        # searchsorted -- without its input validation and index-array gather: the same indices
        # from the same stream position (tests/test_training.py checks them against the reference)
        cdf = probs.astype(np.float64).cumsum()
        cdf /= cdf[-1]
        indx = cdf.searchsorted(np.random.random_sample(batch_s), side="right").astype(np.int64)
        w = ((1.0 / self.size) / probs[indx]) ** self._importance_sampling_exponent
        w /= np.max(w)
        return (*self._gather(indx), indx, torch.from_numpy(w).to(self.dev, dtype=torch.float32))

    def update_priorities(self, indx, new_priorities):
        """buffer.py:127-134"""
        if indx is None:
            return
        assert np.isfinite(new_priorities).all() and (new_priorities > 0.0).any(), \
            "Priorities must be finite and positive."
        self.priorities[indx] = new_priorities

    def __len__(self):
        return self.size if self.is_full else self.ptr
