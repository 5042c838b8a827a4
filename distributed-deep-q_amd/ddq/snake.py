"""Snake emulator used as the synthetic frame source (host side, not on the
GPU path).  Restates the game rules of gamesim/SnakeGame.py (reference):

* 10x10 board, no wrap-around: leaving the board or hitting the body ends the
  game (SnakeGame.py:163-165, :220-226);
* reward +1 when an apple is eaten (the snake grows and a new apple appears on
  a random empty cell), 0 for a plain move, -1 on game over (:19-21, :227-237);
* a move opposite to the current heading keeps the heading (:74-81);
* the start position is head (6,5), tail (5,5), heading east, one apple
  (:149-154; Snake.__init__ :53-57 places the "neck" one cell east and pushes
  it to the front, so it becomes the head);
* ``encode_state`` board codes: -1 empty, -2 apple, k = k-th snake cell from
  the head (:186-196); ``gray_scale``: body/head 200, apple 255, empty 0
  (:22-24, :268-292).

Directions are 'w' (y+1), 's' (y-1), 'd' (x+1), 'a' (x-1) (SnakeGame.py:8-12,
:117-136).
"""
from __future__ import annotations

import random

import numpy as np

NX = NY = 10
EMPTY, APPLE = -1, -2
APPLE_COLOR, BODY_COLOR = 255, 200
SCORE_GROW, SCORE_MOVE, SCORE_OVER = 1, 0, -1
_STEP = {"w": (0, 1), "s": (0, -1), "d": (1, 0), "a": (-1, 0)}
_OPPOSITE = {"w": "s", "s": "w", "d": "a", "a": "d"}


class SnakeGame:
    """cpu_play(state_array, direction) -> (new_state, reward, game_over)."""

    def __init__(self, rng=None):
        self.rng = rng or random.Random()
        self.body = [(6, 5), (5, 5)]      # head first
        self.heading = "d"
        self.apples = set()
        self._add_apple()

    def _empty_cells(self):
        occupied = set(self.body) | self.apples
        return [(x, y) for x in range(NX) for y in range(NY) if (x, y) not in occupied]

    def _add_apple(self):
        cells = self._empty_cells()
        if cells:
            self.apples.add(cells[self.rng.randrange(len(cells))])

    def encode_state(self):
        s = np.full((NX, NY), EMPTY, np.int64)
        for (x, y) in self.apples:
            s[x, y] = APPLE
        for k, (x, y) in enumerate(self.body):
            s[x, y] = k
        return s

    def set_state(self, s):
        cells = {}
        self.apples = set()
        for x in range(NX):
            for y in range(NY):
                v = int(s[x, y])
                if v == APPLE:
                    self.apples.add((x, y))
                elif v != EMPTY:
                    cells[v] = (x, y)
        self.body = [cells[k] for k in range(len(cells))]
        (hx, hy), (nx_, ny_) = self.body[0], self.body[1]
        dx = (hx - nx_) % NX
        dy = (hy - ny_) % NY
        dx = -1 if dx > 1 else dx
        dy = -1 if dy > 1 else dy
        self.heading = {(1, 0): "d", (-1, 0): "a", (0, 1): "w", (0, -1): "s"}[(dx, dy)]

    def update(self, direction):
        if _OPPOSITE[direction] == self.heading:
            direction = self.heading
        dx, dy = _STEP[direction]
        hx, hy = self.body[0]
        new = (hx + dx, hy + dy)
        if new in self.body or not (0 <= new[0] < NX and 0 <= new[1] < NY):
            return SCORE_OVER
        self.heading = direction
        self.body.insert(0, new)
        if new in self.apples:
            self.apples.discard(new)
            self._add_apple()
            return SCORE_GROW
        self.body.pop()
        return SCORE_MOVE

    def cpu_play(self, state_array, direction):
        self.set_state(state_array)
        r = self.update(direction)
        return self.encode_state(), r, r == SCORE_OVER


def gray_scale(state_array):
    """(nc, nx, ny) board codes -> uint8 gray levels (SnakeGame.py:268-292)."""
    g = np.zeros(state_array.shape, np.uint8)
    g[state_array != EMPTY] = BODY_COLOR
    g[state_array == APPLE] = APPLE_COLOR
    return g
