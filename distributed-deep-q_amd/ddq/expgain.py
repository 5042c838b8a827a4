"""Experience gainer: the acting loop of expgain.py (reference) with the same
interface -- ε-greedy action selection, 4-frame history, gray-scale +
nearest-neighbour resampling, one environment step + ``add_experience`` per
``generate_experience`` call.  Greedy actions come from the GPU Q tower
(``BaristaNet.select_action`` -> ``ddq_select_action``), batch n instead of the
reference's full-batch forward.
"""
from __future__ import annotations

import random
from collections import deque

import numpy as np

FRAME_LIMIT = 50000     # expgain.py:6
EPSILON_MAX = 1.0       # expgain.py:7
EPSILON_MIN = 0.1       # expgain.py:8
NFRAME = 4              # expgain.py:9


def resampler(size):
    """Nearest-neighbour zoom of a (C, nx, ny) stack to (C, size[0], size[1])
    (expgain.py:12-18: scipy.ndimage.zoom(order=0))."""
    import scipy.ndimage

    def func(state):
        zoom = (1.0, float(size[0]) / state.shape[1], float(size[1]) / state.shape[2])
        return scipy.ndimage.zoom(state, zoom, order=0)

    return func


def generate_preprocessor(size, gray_scale):
    """expgain.py:21-27."""
    resamp = resampler(size)

    def preprocessor(state):
        return resamp(gray_scale(state))

    return preprocessor


def epsilon(iter_num):
    """Linear ε schedule 1.0 -> 0.1 over 50 000 iterations (expgain.py:55-60)."""
    if iter_num > FRAME_LIMIT:
        return EPSILON_MIN
    return EPSILON_MIN + (EPSILON_MAX - EPSILON_MIN) * max(FRAME_LIMIT - iter_num, 0) / FRAME_LIMIT


class ExpGain:
    """Same constructor and methods as the reference ExpGain (expgain.py:30-111)."""

    def __init__(self, net, actions, preprocessor, game, dataset, init_state, rng=None):
        self.net = net
        self.actions = list(actions)
        self.preprocessor = preprocessor
        self.game = game
        self.dataset = dataset
        self.init_state = init_state
        self.rng = rng or random.Random()
        self.game_over = False
        self.sequence = deque([init_state] * NFRAME)

    def reset_game(self):
        self.sequence = deque([self.init_state] * NFRAME)
        self.game_over = False

    def get_epsilon(self, iter_num):
        return epsilon(iter_num)

    def select_action(self, pstate, eps):
        if self.rng.random() < eps:
            return self.rng.choice(self.actions)
        return self.actions[int(self.net.select_action(pstate))]

    def arrayify_frames(self):
        return np.stack(list(self.sequence)[:NFRAME]).astype(np.int64)

    def get_preprocessed_state(self):
        return self.preprocessor(self.arrayify_frames())

    def generate_experience(self, iter_num):
        pstate = self.preprocessor(self.arrayify_frames())
        action = self.select_action(pstate, self.get_epsilon(iter_num))
        new_state, reward, gameover = self.game(self.sequence[-1], action)
        self.sequence.popleft()
        self.sequence.append(new_state)
        exp_frame = None if gameover else self.preprocessor(self.arrayify_frames())
        self.dataset.add_experience(self.actions.index(action), reward, exp_frame)
        if gameover:
            self.reset_game()

    def play_policy(self):
        pstate = self.preprocessor(self.arrayify_frames())
        action = self.actions[int(self.net.select_action(pstate))]
        return self.play_action(action)

    def play_action(self, action):
        new_state, reward, gameover = self.game(self.sequence[-1], action)
        self.sequence.popleft()
        self.sequence.append(new_state)
        if gameover:
            self.game_over = True
        return reward


def synthetic_transitions(n, frame, seed=0):
    """n transitions of random-policy Snake (ε = 1), preprocessed to frame x
    frame 4-stacks: returns (states u8 (n,4,S,S), actions u8, rewards i16,
    non_terminal bool) in add_experience order (SURVEY.md 8(d) frames)."""
    from .snake import SnakeGame, gray_scale

    rng = random.Random(seed)
    game = SnakeGame(rng)
    pre = generate_preprocessor((frame, frame), gray_scale)
    init = game.encode_state()
    seq = deque([init] * NFRAME)
    states = np.zeros((n, NFRAME, frame, frame), np.uint8)
    acts = np.zeros(n, np.uint8)
    rews = np.zeros(n, np.int16)
    nts = np.zeros(n, bool)
    moves = "wasd"
    for i in range(n):
        a = rng.randrange(4)
        new, r, over = game.cpu_play(seq[-1], moves[a])
        seq.popleft()
        seq.append(new)
        acts[i], rews[i], nts[i] = a, r, not over
        if not over:
            states[i] = pre(np.stack(seq))
        else:
            seq = deque([init] * NFRAME)
    return states, acts, rews, nts
