"""Packed host<->device transfers for the one-root drop-in calls (MCTS.run_mcts, TowersOfHanoi.step).

The reference's training loop makes one search and one env step per decision (Muzero._play_game,
Muzero.py:153-207); each carries a handful of tiny inputs and outputs.  Moving them as separate
tensors costs one copy (and, for reads, one synchronisation) each.  A `Packed` is one device
buffer and one pinned host buffer carved into the same typed fields, so a call's inputs go down in
one copy and its outputs come back in one copy and one synchronisation.
"""
import numpy as np
import torch

from . import _lib


class Packed:
    def __init__(self, fields, device, zero_copy=False):
        """fields: [(name, torch dtype, shape)] -- each field 16-byte aligned.

        zero_copy: no device buffer -- the kernels read and write the pinned host buffer itself through its
        device address (`dptr`: field -> device address; mzh_host_device_pointer), so to_device does nothing and
        to_host only synchronises."""
        self.layout = {}
        off = 0
        for name, dt, shape in fields:
            n = int(np.prod(shape)) * torch.empty((), dtype=dt).element_size()
            self.layout[name] = (off, dt, tuple(shape), n)
            off += (n + 15) & ~15
        self.nbytes = max(off, 16)
        self.zero_copy = zero_copy
        self.device = torch.device(device)
        self.host = torch.zeros(self.nbytes, dtype=torch.uint8, pin_memory=True)
        self.h = {k: self._view(self.host, k).numpy() for k in self.layout}  # numpy views of pinned memory
        if zero_copy:
            base = _lib.host_device_pointer(self.host.data_ptr())
            self.dev = None
            self.d = None
            self.dptr = {k: base + self.layout[k][0] for k in self.layout}
        else:
            self.dev = torch.zeros(self.nbytes, dtype=torch.uint8, device=device)
            self.d = {k: self._view(self.dev, k) for k in self.layout}  # device tensors
            self.dptr = {k: v.data_ptr() for k, v in self.d.items()}

    def _view(self, buf, k):
        off, dt, shape, n = self.layout[k]
        return buf[off:off + n].view(dt).view(shape)

    def to_device(self):
        """host fields -> device fields, ordered on the current stream"""
        if not self.zero_copy:
            self.dev.copy_(self.host, non_blocking=True)

    def to_host(self):
        """device fields -> host fields; returns once they are there"""
        if not self.zero_copy:
            self.host.copy_(self.dev, non_blocking=True)
        _lib.synchronize(self.device)
