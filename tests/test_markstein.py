"""The search kernel divides with y = RN(1/b) and one fma correction step (csrc/mzh_search.hip
mzh_div, Markstein's theorem) instead of the long IEEE division sequence; the reference divides
with Python floats (node.py:98-121, utils_mcts.py:12-16).  The two must agree bit for bit on the
operand domains the search produces."""


def test_markstein_division_is_ieee(oracle):
    assert oracle.lib().orc_markstein_mismatches(20_000_000, 12345) == 0
