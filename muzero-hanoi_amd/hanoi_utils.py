"""hanoi_solver drop-in (env/hanoi_utils.py:4-26): the fewest moves from any legal configuration
to all disks on `goal_peg`.

The acting scripts call it once per episode with one state (acting_experiments/
acting_ablations.py:96-98), so the scalar form runs on the host -- a device launch + sync per
call would cost more than the whole computation.  Batches of states (evaluation sweeps) use the
device kernel, engine.hanoi_solver_batch / mzh_hanoi_solver, which computes the same closed form.
"""
from functools import lru_cache


@lru_cache(maxsize=None)
def hanoi_solver(state: tuple, goal_peg: int = 2) -> int:
    """state[i] in {0, 1, 2} is the peg of disk i (disk 0 the smallest).  Walk the disks from the
    largest down: a disk that is not on the peg its stack must end on costs 2^i moves (it moves
    once, after the i smaller disks have been parked on the third peg, which then becomes where
    they must go); a disk already there costs nothing and leaves the target unchanged."""
    total, peg = 0, goal_peg
    for disk in range(len(state) - 1, -1, -1):
        on = state[disk]
        if on != peg:
            total += 1 << disk
            peg = 3 - peg - on  # the third peg (pegs are 0, 1, 2)
    return total
