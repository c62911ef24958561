"""Replay buffer drop-in (reference: buffer.py:5-139, `Buffer`).

Transitions are already organised for `unroll_n_steps` (Muzero.organise_transitions). The
reference keeps them in host NumPy arrays and copies every sampled batch to the device; here the
five transition arrays live on the training device (HBM on the MI355X: a ring of 10^8 transitions
is a few GB of 288) and a sampled batch is an on-device gather.  Only what the reference's RNG
stream depends on stays on the host: the priorities, from which `np.random.choice` draws the
indices exactly as the reference does (same global legacy stream, same calls), so a seeded run
samples the same transitions.

With `device_sampling=True` (what Muzero(update_impl="fused") uses on a GPU) the priorities live in HBM
as well and the whole draw runs on the device (csrc/mzh_replay.hip: P = p / np.sum(p), the float64 cdf,
searchsorted, the row gather -- the same indices as NumPy's choice for the same uniforms, which are
still np.random.random_sample(batch_s) on the global stream), as does update_priorities.  Then
`priority_sample` returns the indices as a device tensor, the batch tensors are new device tensors as
before, and `update_priorities` waits for its write-back and raises the reference's AssertionError
(non-finite or no positive priority) from the same call; a probability vector NumPy's choice would
refuse (NaN or negative) raises ValueError from the update_priorities of that draw (or from the next
draw or read of `priorities`, whichever comes first).  `priorities` then returns a read-only host copy.
Only the reference's defaults are supported there (priority_exponent 1, importance_sampling_exponent
0: the importance weights are ones).
"""
import ctypes

import numpy as np
import torch


class Buffer:
    def __init__(self, size, unroll_n_steps, d_state, n_action, device, priority_exponent=1,
                 importance_sampling_exponent=0, device_sampling=False):
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
        self.device_sampling = bool(device_sampling)
        if self.device_sampling:
            self._dev_replay = _DeviceReplay(self)
            self._prio = self._dev_replay.prio
        else:
            self._prio = np.zeros((size,), dtype=np.float32)  # host: drives np.random.choice
        self.ptr = 0
        self.is_full = False

    @property
    def priorities(self):
        """the priority array (host mode); with device_sampling a read-only host copy of the device array"""
        if self.device_sampling:
            return self._dev_replay.host_priorities()
        return self._prio

    @priorities.setter
    def priorities(self, value):
        if self.device_sampling:
            self._dev_replay.check_pending(block=True)
            self._prio.copy_(torch.as_tensor(np.asarray(value, np.float32)))
        else:
            self._prio[...] = value

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
        self._ring_write(self._prio, as_dev(priorities, torch.float32) if self.device_sampling
                         else np.asarray(priorities, np.float32))
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
        if self.device_sampling:
            return self._dev_replay.sample(batch_s)
        num = len(self)
        p = self._prio[:num] ** self._priority_exponent
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
        if self.device_sampling:
            return self._dev_replay.set_priorities(indx, new_priorities)
        assert np.isfinite(new_priorities).all() and (new_priorities > 0.0).any(), \
            "Priorities must be finite and positive."
        self._prio[indx] = new_priorities

    def __len__(self):
        return self.size if self.is_full else self.ptr


class _DeviceReplay:
    """The device half of Buffer(device_sampling=True): priorities and cdf workspace in HBM, the draw's
    uniforms and the kernels' status words in mapped page-locked memory (read by the kernels directly;
    RING slots, each reused only after the draw that used it has finished)."""

    RING = 4

    def __init__(self, buf):
        from . import _lib

        if buf.dev.type != "cuda":
            raise ValueError("Buffer(device_sampling=True) needs a GPU device")
        if buf._priority_exponent != 1 or buf._importance_sampling_exponent != 0:
            raise ValueError("Buffer(device_sampling=True) implements priority_exponent=1, "
                             "importance_sampling_exponent=0 (the reference's defaults) only")
        self.L = _lib
        self.buf = buf
        self.prio = torch.zeros((buf.size,), dtype=torch.float32, device=buf.dev)
        self.cdf = torch.empty((buf.size,), dtype=torch.float64, device=buf.dev)
        # status words: [slot][0..1] of a draw, [RING][0] of update_priorities
        self.status = torch.zeros((self.RING + 1, 2), dtype=torch.int32, pin_memory=True)
        self.status_np = self.status.numpy()
        self.status_dev = _lib.host_device_pointer(self.status.data_ptr())
        self.m = 0
        self.slot = 0
        self.pending = [None] * self.RING  # the event of the draw in each slot, until its status is read
        self.events = [torch.cuda.Event() for _ in range(self.RING)]
        self.ones = None

    def _stream(self):
        return self.L.stream_handle(self.buf.dev)

    def _alloc_u(self, m):
        self.u = torch.zeros((self.RING, m), dtype=torch.float64, pin_memory=True)
        self.u_np = self.u.numpy()
        self.u_dev = self.L.host_device_pointer(self.u.data_ptr())
        self.ones = torch.ones(m, dtype=torch.float32, device=self.buf.dev)
        self.m = m
        buf = self.buf
        a = self.L.ReplayArgs()
        a.m, a.d_state, a.U, a.A = m, buf.d_state, buf.unroll_n_steps, buf.n_action
        a.prio, a.cdf = self.prio.data_ptr(), self.cdf.data_ptr()
        a.states, a.rwds, a.actions = buf.states.data_ptr(), buf.rwds.data_ptr(), buf.actions.data_ptr()
        a.pi, a.returns = buf.pi_probs.data_ptr(), buf.mc_returns.data_ptr()
        self.args = a
        self.args_ptr = ctypes.byref(a)

    def check_pending(self, block):
        """raise NumPy's ValueError for a finished draw whose probabilities it would have refused"""
        for s, ev in enumerate(self.pending):
            if ev is None:
                continue
            if block:
                ev.synchronize()
            elif not ev.query():
                continue
            self.pending[s] = None
            if self.status_np[s, 0] != 0:
                raise ValueError("probabilities contain NaN or are not non-negative "
                                 "(np.random.choice's check of the priorities, buffer.py:89-112)")

    def sample(self, m):
        buf = self.buf
        n = len(buf)
        if n == 0:
            raise ValueError("a cannot be empty unless no samples are taken")
        if m != self.m:
            self.check_pending(block=True)
            self._alloc_u(m)
        self.check_pending(block=False)
        s = self.slot
        self.slot = (s + 1) % self.RING
        if self.pending[s] is not None:  # the draw that used this slot must be done with its uniforms
            self.check_pending(block=True)
        self.u_np[s] = np.random.random_sample(m)  # the reference's stream: choice draws random_sample(m)
        dev, U, A = buf.dev, buf.unroll_n_steps, buf.n_action
        indx = torch.empty(m, dtype=torch.int64, device=dev)
        out = (torch.empty((m, buf.d_state), dtype=torch.float32, device=dev),
               torch.empty((m, U), dtype=torch.float32, device=dev),
               torch.empty((m, U), dtype=torch.int64, device=dev),
               torch.empty((m, U, A), dtype=torch.float32, device=dev),
               torch.empty((m, U), dtype=torch.float32, device=dev))
        a = self.args  # the fixed fields were set by _alloc_u
        a.n = n
        a.u = self.u_dev + s * m * 8
        a.indx = indx.data_ptr()
        a.out_states, a.out_rwds, a.out_actions, a.out_pi, a.out_returns = (t.data_ptr() for t in out)
        a.status = self.status_dev + s * 8
        self.L.check(self.L.lib().mzh_replay_sample(self.args_ptr, self._stream()), "mzh_replay_sample")
        ev = self.events[s]
        ev.record(torch.cuda.current_stream(dev))
        self.pending[s] = ev
        return (*out, indx, self.ones)

    def set_priorities(self, indx, new_priorities):
        dev = self.buf.dev
        idx = torch.as_tensor(indx).to(dev, torch.int64).contiguous()
        val = torch.as_tensor(new_priorities).to(dev, torch.float32).contiguous()
        if idx.numel() != val.numel():
            raise ValueError(f"update_priorities: {idx.numel()} indices, {val.numel()} priorities")
        st = self.status_dev + self.RING * 8
        self.L.check(self.L.lib().mzh_replay_set_priorities(self.prio.data_ptr(), self.buf.size, idx.data_ptr(),
                                                            val.data_ptr(), idx.numel(), st, self._stream()),
                     "mzh_replay_set_priorities")
        self.L.synchronize(dev)
        self.check_pending(block=True)
        code = int(self.status_np[self.RING, 0])
        if code == 1:
            raise AssertionError("Priorities must be finite and positive.")
        if code == 2:
            raise IndexError(f"update_priorities: an index is outside [0, {self.buf.size})")

    def host_priorities(self):
        self.check_pending(block=True)
        out = self.prio.cpu().numpy()
        out.flags.writeable = False
        return out
