"""Othello as a Game plugin of this fork's API (builder-authored: the reference
fork has no Othello code, SURVEY.md finding 1).

Board n x n (6 or 8), +1 = RED (moves first), -1 = BLUE.  Standard rules: a
move places a piece that brackets a straight line of opponent pieces in at
least one of the 8 directions and flips them; a player with no such move must
pass (action n*n, legal only then); the game ends when neither player can move,
the side with more pieces WINS (equal: DRAW).

Fork-API choices (mirroring InflexionGame):
  * actions: r*n + q for placements, n*n for pass; policy_shape = (1, 1, n*n+1);
  * to_planes() = [own pieces, opponent pieces] (2, n, n), player-relative;
  * symmetries: the 8 dihedral symmetries of the square (identity first); on a
    policy vector the pass entry stays in place;
  * random_symmetry draws one np.random.randint(0, 8) from numpy's global RNG;
  * _curr_turn counts moves (passes included); there is no turn limit.
"""
import copy

import numpy as np

from .flags import GameOutcome, PlayerColour
from .game import Game

DIRECTIONS = ((-1, -1), (-1, 0), (-1, 1), (0, -1), (0, 1), (1, -1), (1, 0), (1, 1))


def dihedral_source(n, k):
    """Source (row, col) for output cell (r, q) under dihedral symmetry k (0..7):
    k & 3 = number of 90-degree rotations (np.rot90 convention), k & 4 = then mirror left-right."""
    r, q = np.indices((n, n))
    idx = r * n + q
    t = np.rot90(idx, k & 3)
    if k & 4:
        t = np.fliplr(t)
    return t // n, t % n


class OthelloGame(Game):
    def __init__(self, n=8, first_mover=PlayerColour.RED, curr_player=None, board=None, curr_turn=0,
                 max_turns=None):
        if n % 2 or not 4 <= n <= 8:
            raise AssertionError("n must be even, 4..8")
        super().__init__(board_shape=(n, n), policy_shape=(1, 1, n * n + 1), first_mover=first_mover)
        self._n = n
        if curr_player is not None:
            self._player = curr_player
        if board is None:
            board = np.zeros((n, n), dtype=int)
            h = n // 2
            board[h - 1, h - 1] = board[h, h] = PlayerColour.BLUE.num
            board[h - 1, h] = board[h, h - 1] = PlayerColour.RED.num
        self._board = board
        self._curr_turn = curr_turn
        self._max_turns = (n * n) * 2 if max_turns is None else max_turns  # unused bound, API parity
        self._planes_shape = (2, n, n)

    # ------------------------------------------------------------------ lifecycle
    def restarted(self):
        return OthelloGame(self._n, first_mover=self._firstMover)

    def to_next_state(self, action):
        if not 0 <= action < self.max_actions:
            raise AssertionError(f"action {action} out of range")
        nxt = copy.deepcopy(self)
        nxt.execute_move(self.action_to_move(action))
        return nxt

    # ------------------------------------------------------------------ rules
    def _flips(self, r, q, me):
        b, n, out = self._board, self._n, []
        if b[r, q] != 0:
            return out
        for dr, dq in DIRECTIONS:
            line = []
            rr, qq = r + dr, q + dq
            while 0 <= rr < n and 0 <= qq < n and b[rr, qq] == -me:
                line.append((rr, qq))
                rr += dr
                qq += dq
            if line and 0 <= rr < n and 0 <= qq < n and b[rr, qq] == me:
                out += line
        return out

    def _legal(self, me):
        n = self._n
        return [(r, q) for r in range(n) for q in range(n) if self._flips(r, q, me)]

    def valid_actions_mask(self):
        n = self._n
        mask = np.zeros(n * n + 1, dtype=int)
        legal = self._legal(self._player.num)
        for r, q in legal:
            mask[r * n + q] = 1
        if not legal:
            mask[n * n] = 1
        return mask

    def execute_move(self, move):
        kind, r, q = move
        me, n = self._player.num, self._n
        if kind == "pass":
            if self._legal(me):
                raise ValueError("Invalid move: pass with a legal placement available")
        else:
            flips = self._flips(r, q, me)
            if not flips:
                raise ValueError("Invalid move")
            self._board[r, q] = me
            for rr, qq in flips:
                self._board[rr, qq] = me
        self._curr_turn += 1
        if not self._legal(-me) and not self._legal(me):
            diff = int(np.sum(self._board)) * me
            self._outcome = GameOutcome.WON if diff > 0 else GameOutcome.LOST if diff < 0 else GameOutcome.DRAW
        self.player = self._player.opponent

    # ------------------------------------------------------------------ features
    def to_planes(self):
        me = self._player.num
        return np.stack([(self._board * me > 0).astype(int), (self._board * me < 0).astype(int)])

    def _sym(self, board_like, k):
        rr, qq = dihedral_source(self._n, k)
        if board_like.shape == self.policy_shape:
            flat = board_like.reshape(-1)
            n2 = self._n * self._n
            out = flat.copy()
            out[:n2] = flat[:n2].reshape(self._n, self._n)[rr, qq].reshape(-1)
            return out.reshape(self.policy_shape)
        return board_like[..., rr, qq].copy()

    def symmetries(self, board_like):
        return [self._sym(board_like, k) for k in range(8)]

    def random_symmetry(self, board_like):
        return self._sym(board_like, np.random.randint(0, 8))

    # ------------------------------------------------------------------ moves
    def move_to_action(self, move):
        kind, r, q = move
        return self._n * self._n if kind == "pass" else int(r * self._n + q)

    def action_to_move(self, action):
        n = self._n
        if not 0 <= action <= n * n:
            raise AssertionError("bad action")
        if action == n * n:
            return "pass", 0, 0
        return "place", int(action) // n, int(action) % n

    def score(self):
        me = self._player.num
        return int(np.count_nonzero(self._board == me) - np.count_nonzero(self._board == -me))

    def render(self):
        sym = {1: "R", -1: "B", 0: "."}
        print("\n".join(" ".join(sym[int(x)] for x in row) for row in self._board))
