"""7x7 toroidal hex "Infexion" as a Game plugin (reference inflexion/InflexionGame.py).

Host-side mirror of the plugin the engine accelerates: same constructor,
attributes (`_board`, `_curr_turn`, `_max_turns`, ...) and methods, so code
written against the reference (Coach, Arena, players) runs unchanged, and the
engine can take its state (board, turn, player) from any instance.

Rules (restated; pinned by tests/golden/rules_kat.npz):
  actions a = move * n*n + r*n + q, moves 0-5 SPREAD along R1 (1,0), R2 (-1,0),
  Q1 (0,1), Q2 (0,-1), P1 (1,-1), P2 (-1,1), move 6 SPAWN (InflexionGame.py:14-36);
  SPREAD of power p moves onto the next p cells (wrapping), each becoming the
  mover's with power |x|+1 (0 if it exceeds 6), the origin empties; SPAWN puts
  power 1 on an empty cell while total power <= 48 (:273-291); the game ends
  when a spread leaves the opponent no piece (WON), when turn >= max_turns
  (power difference >= 2 WON, <= -2 LOST, else DRAW) or on an empty board
  (DRAW), checked before the turn counter advances (:293-310).
"""
import copy
from enum import Enum
from itertools import product

import numpy as np

from .flags import GameOutcome, PlayerColour
from .game import Game

MAX_POWER_AT_SPAWN = 48
MAX_CELL_POWER = 6


class Move(Enum):
    SPREAD_R1 = 0, (1, 0)
    SPREAD_R2 = 1, (-1, 0)
    SPREAD_Q1 = 2, (0, 1)
    SPREAD_Q2 = 3, (0, -1)
    SPREAD_P1 = 4, (1, -1)
    SPREAD_P2 = 5, (-1, 1)
    SPAWN = 6, (0, 0)

    def __init__(self, num, direction):
        self.num = num
        self.direction = direction

    @classmethod
    def from_num(cls, num):
        for m in cls:
            if m.num == num:
                return m
        raise IndexError(f"Move number {num} is not valid.")

    @classmethod
    def all_spreads(cls):
        return tuple(m for m in cls if m is not cls.SPAWN)


_SPREADS = Move.all_spreads()


def hex_rotation_source(n, k):
    """Source (row, col) of every output cell for a rotation by 60*k degrees.

    With s = (r + q) mod n the axial triple (r, q, s) is cycled by k and sign
    flipped (InflexionGame.py:124-168), negative indices wrapping."""
    r, q = np.indices((n, n))
    s = (r + q) % n
    k %= 6
    src = {0: (r, q), 1: (-s, r), 2: (-q, s), 3: (-r, -q), 4: (s, -r), 5: (q, -s)}[k]
    return src[0] % n, src[1] % n


class InflexionGame(Game):
    def __init__(self, n, first_mover=PlayerColour.RED, curr_player=None, board=None, curr_turn=0,
                 max_turns=100, max_power=6):
        super().__init__(board_shape=(n, n), policy_shape=(7, n, n), first_mover=first_mover)
        if not (isinstance(n, int) and n > 0):
            raise AssertionError("n must be a positive int")
        if board is not None and board.shape != (n, n):
            raise AssertionError("board must be n x n")
        self._n = n
        if curr_player is not None:
            self._player = curr_player
        self._board = np.zeros((n, n), dtype=int) if board is None else board
        self._curr_turn = curr_turn
        self._max_turns = max_turns
        self._max_power = max_power
        self._planes_shape = (4, n, n)
        self._max_power_at_spawn = MAX_POWER_AT_SPAWN

    # ------------------------------------------------------------------ lifecycle
    def restarted(self):
        return InflexionGame(self._n, first_mover=self._firstMover, max_turns=self._max_turns,
                             max_power=self._max_power)

    def to_next_state(self, action):
        if not (0 <= action < self.max_actions):
            raise AssertionError(f"action {action} out of range")
        nxt = copy.deepcopy(self)
        nxt.execute_move(self.action_to_move(action))
        return nxt

    # ------------------------------------------------------------------ features
    def total_power(self):
        return int(np.abs(self._board).sum())

    def to_planes(self):
        me = self._player.num
        mine = (self._board * me > 0).astype(int)
        theirs = (self._board * me < 0).astype(int)
        turn = np.full(self._board_shape, self._curr_turn, dtype=int)
        spawn = np.full(self._board_shape, int(self.total_power() <= MAX_POWER_AT_SPAWN), dtype=int)
        return np.stack([mine, theirs, turn, spawn])

    def valid_actions_mask(self):
        me = self._player.num
        mask = np.zeros((7, self._n, self._n), dtype=int)
        mask[:6] = (self._board * me > 0)[None]
        if self.total_power() <= MAX_POWER_AT_SPAWN:
            mask[6] = self._board == 0
        return mask.ravel()

    # ------------------------------------------------------------------ symmetries
    def rotate(self, board_like, k=1):
        rr, qq = hex_rotation_source(self._n, int(k))
        return board_like[:, rr, qq].copy()

    def translate(self, board_like, shift, axis):
        if axis == "r":
            return np.roll(board_like, shift, axis=1)
        if axis == "q":
            return np.roll(board_like, shift, axis=2)
        if axis == "s":
            return np.roll(np.roll(board_like, shift, axis=2), -shift, axis=1)
        raise ValueError(f"unknown axis {axis!r}")

    def symmetries(self, board_like):
        """36 forms: identity, 5 rotations, then each rotation shifted 1..n-1 along r."""
        rots = [self.rotate(board_like, k) for k in range(1, 6)]
        shifted = [self.translate(b, j, "r") for b in rots for j in range(1, self._n)]
        return [board_like.copy()] + rots + shifted

    def random_symmetry(self, board_like):
        """Draw order on numpy's global RandomState: randint(0,6), randint(0,n), choice(r,q,s)."""
        k = np.random.randint(0, 6)
        shift = np.random.randint(0, self._n)
        axis = np.random.choice(["r", "q", "s"])
        return self.translate(self.rotate(board_like, k), shift, axis=axis)

    # ------------------------------------------------------------------ moves
    def move_to_action(self, move):
        kind, r, q = move
        if not (0 <= r < self._n and 0 <= q < self._n and kind in Move):
            raise AssertionError("bad move")
        return int((kind.num * self._n + r) * self._n + q)

    def action_to_move(self, action):
        if not (0 <= action < self.max_actions):
            raise AssertionError("bad action")
        kind, rest = divmod(int(action), self._n * self._n)
        r, q = divmod(rest, self._n)
        return Move.from_num(kind), r, q

    def execute_move(self, move):
        kind, r, q = move
        b, me, n = self._board, self._player.num, self._n
        if kind is Move.SPAWN and self.total_power() <= MAX_POWER_AT_SPAWN:
            if b[r, q] != 0:
                raise AssertionError("spawn on an occupied cell")
            b[r, q] = me
        elif kind in _SPREADS:
            if not b[r, q] * me > 0:
                raise AssertionError("spread from a cell the player does not own")
            dr, dq = kind.direction
            for k in range(1, abs(int(b[r, q])) + 1):
                rr, qq = (r + k * dr) % n, (q + k * dq) % n
                x = abs(int(b[rr, qq])) + 1
                b[rr, qq] = (0 if x > MAX_CELL_POWER else x) * me
            b[r, q] = 0
        else:
            raise ValueError("Invalid move")

        if kind in _SPREADS and not np.any(b * me < 0):
            self._outcome = GameOutcome.WON
        elif self._curr_turn >= self._max_turns:
            diff = self.power_diff(self._player)
            self._outcome = GameOutcome.WON if diff >= 2 else GameOutcome.LOST if diff <= -2 else GameOutcome.DRAW
        elif not b.any():
            self._outcome = GameOutcome.DRAW
        self._curr_turn += 1
        self.player = self._player.opponent

    # ------------------------------------------------------------------ scores
    def power_diff(self, player):
        return int(player.num * self._board.sum())

    def piece_count_diff(self, player):
        me = player.num
        return int(np.count_nonzero(self._board * me > 0) - np.count_nonzero(self._board * me < 0))

    def score(self):
        return self.piece_count_diff(self._player)

    def render(self, ansi=False):
        n, out = self._n, []
        for row in range(2 * n - 1):
            line = "    " * abs((n - 1) - row)
            for col in range(n - abs(row - (n - 1))):
                r, q = max((n - 1) - row, 0) + col, max(row - (n - 1), 0) + col
                x = int(self._board[r, q])
                line += (f"{PlayerColour.from_piece(x).token}{abs(x)}".center(4) if x else " .. ") + "    "
            out.append(line)
        print("\n".join(out))
