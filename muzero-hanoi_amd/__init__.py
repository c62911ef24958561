"""muzero_hanoi_amd -- MI355X-native batched MuZero-MCTS + Tower-of-Hanoi search.

Drop-in for the reference's hot path (A-Andrews/Muzero-Hanoi):
  TowersOfHanoi   env/hanoi.py          -> muzero_hanoi_amd.env.TowersOfHanoi
  MuZeroNet       networks.py           -> muzero_hanoi_amd.networks.MuZeroNet
  MCTS            MCTS/mcts.py          -> muzero_hanoi_amd.mcts.MCTS   (+ batched run_batch)
  Muzero          Muzero.py             -> muzero_hanoi_amd.muzero.Muzero (self-play on the GPU search,
                                           training update on PyTorch-ROCm)
  Buffer          buffer.py             -> muzero_hanoi_amd.buffer.Buffer (device-resident storage)
The compute runs in libmzh.so (hand-written gfx950 HIP behind the C ABI in include/mzh.h).
Importing this package does not load the library; the first device call does, and fails
loudly if it is missing.
"""
__all__ = ["TowersOfHanoi", "MuZeroNet", "MCTS", "MinMaxStats", "Muzero", "Buffer", "hanoi_solver", "oneHot_encoding"]


def __getattr__(name):
    if name == "TowersOfHanoi":
        from .env import TowersOfHanoi
        return TowersOfHanoi
    if name == "MuZeroNet":
        from .networks import MuZeroNet
        return MuZeroNet
    if name in ("MCTS", "MinMaxStats"):
        from . import mcts
        return getattr(mcts, name)
    if name == "Muzero":
        from .muzero import Muzero
        return Muzero
    if name == "Buffer":
        from .buffer import Buffer
        return Buffer
    if name == "hanoi_solver":
        from .hanoi_utils import hanoi_solver
        return hanoi_solver
    if name == "oneHot_encoding":
        from .utils import oneHot_encoding
        return oneHot_encoding
    raise AttributeError(name)
