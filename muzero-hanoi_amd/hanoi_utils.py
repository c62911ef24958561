"""hanoi_solver drop-in (env/hanoi_utils.py:4-26).  The batched device form is
engine.hanoi_solver_batch / mzh_hanoi_solver; this scalar form keeps the reference's signature
(tuple state -> int) for the acting scripts and runs through the same kernel."""
from functools import lru_cache

import torch

from . import engine


@lru_cache(maxsize=None)
def hanoi_solver(state: tuple, goal_peg: int = 2) -> int:
    st = torch.tensor([list(state)], dtype=torch.uint8, device="cuda")
    return int(engine.hanoi_solver_batch(len(state), st, goal_peg).item())
