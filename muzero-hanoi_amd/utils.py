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
