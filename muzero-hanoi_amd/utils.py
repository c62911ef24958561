"""Host helpers of the reference's utils.py used around the hot path."""
import numpy as np


def oneHot_encoding(x, n_integers):
    """utils.py:9-25: per-dimension one-hot of an integer vector, flattened (float64).
    (The batched device form is engine.encode_obs / mzh_encode_obs.)"""
    x_dim = len(x)
    oneH_mat = np.zeros((x_dim, n_integers))
    oneH_mat[np.arange(x_dim), x] = 1
    return oneH_mat.reshape(-1)


def adjust_temperature(episode):
    """utils.py:89-96: temperature schedule used by Muzero._play_game."""
    if episode < 500:
        return 1.0
    elif episode < 750:
        return 0.5
    return 0.1


def compute_n_step_returns(rwds, root_values, n_step, discount):
    """utils.py:28-69: n-step TD targets (host bookkeeping of an episode)."""
    assert n_step > 0, "the n_step return must be greater than zero"
    assert len(rwds) == len(root_values), "`rewards` and `root_values` don have the same length."
    T = len(rwds)
    _rwds = list(rwds) + [0] * n_step
    _root_values = list(root_values) + [0] * n_step
    td_returns = []
    for t in range(T):
        bootstrap_idx = t + n_step
        dis_rwd_sum = sum([discount**i * r for i, r in enumerate(_rwds[t:bootstrap_idx])])
        td_returns.append(dis_rwd_sum + discount**n_step * _root_values[bootstrap_idx])
    return td_returns


def compute_MCreturns(rwds, discount):
    """utils.py:72-86: Monte-Carlo returns."""
    rwds = np.array(rwds)
    discounts = discount ** (np.array(range(len(rwds))))
    return list(np.flip(np.cumsum(np.flip(discounts * rwds, axis=(0,)), axis=0), axis=(0,)) / discounts)


def organise_transitions(episode_state, episode_rwd, episode_action, episode_piProb, episode_returns,
                         unroll_n_steps, n_action):
    """Muzero.py:276-323: per-state unroll targets; pads with absorbing steps and draws ONE
    np.random.randint for the padding actions (global RNG, like the reference)."""
    n_states = len(episode_state)
    episode_rwd = list(episode_rwd) + [0] * unroll_n_steps
    episode_action = list(episode_action) + [np.random.randint(0, n_action)] * unroll_n_steps
    episode_returns = list(episode_returns) + [0] * unroll_n_steps
    absorbing_policy = np.ones_like(episode_piProb[-1]) / len(episode_piProb[-1])
    episode_piProb = list(episode_piProb) + [absorbing_policy] * unroll_n_steps
    rwds = np.zeros((n_states, unroll_n_steps), dtype=np.float32)
    actions = np.zeros((n_states, unroll_n_steps), dtype=np.int64)
    pi_probs = np.zeros((n_states, unroll_n_steps, len(episode_piProb[0])), dtype=np.float32)
    returns = np.zeros((n_states, unroll_n_steps), dtype=np.float32)
    for i in range(n_states):
        rwds[i, :] = episode_rwd[i:i + unroll_n_steps]
        actions[i, :] = episode_action[i:i + unroll_n_steps]
        pi_probs[i, :, :] = episode_piProb[i:i + unroll_n_steps]
        returns[i, :] = episode_returns[i:i + unroll_n_steps]
    return np.array(episode_state), rwds, actions, pi_probs, returns
