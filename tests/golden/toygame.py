"""A third Game plugin with no native rules: four in a row on a 6 x 6 board.

TEST INFRASTRUCTURE for the generic plugin path (azg_amd/hostsearch.py): the engine has no
kernels for this game, so MCTS / Coach run it through the host search, which calls these
methods exactly as the reference MCTS does (MCTS.py:62-145 over Game.py:8-181).
tests/golden/make_golden.py drives the REFERENCE MCTS / Coach with this class to pin the
host search (mcts_toy*.json.gz); this file is the plugin, not reference code.

Rules: players alternately place a stone on an empty cell (action r * n + q); four of one
colour in a row (row, column or diagonal) wins for the player who placed the last stone; a
full board without one is a draw.  Fork-API choices:
  * to_planes() = [own stones, opponent stones, ones] (3, n, n), player-relative;
  * symmetries: the 8 dihedral symmetries (identity first);
  * random_symmetry draws np.random.randint(0, 4) (quarter turns) then np.random.randint(0, 2)
    (mirror) from numpy's global stream -- two draws, unlike the other plugins.
"""
import copy

import numpy as np

from azg_amd.flags import GameOutcome, PlayerColour
from azg_amd.game import Game

LINES = ((0, 1), (1, 0), (1, 1), (1, -1))


class FourInARowGame(Game):
    def __init__(self, n=6, first_mover=PlayerColour.RED, need=4):
        super().__init__(board_shape=(n, n), policy_shape=(1, n, n), first_mover=first_mover)
        self._n, self._need = n, need
        self._board = np.zeros((n, n), dtype=int)
        self._curr_turn = 0
        self._max_turns = n * n

    def restarted(self):
        return FourInARowGame(self._n, self._firstMover, self._need)

    def to_next_state(self, action):
        if not 0 <= action < self.max_actions:
            raise AssertionError(f"action {action} out of range")
        nxt = copy.deepcopy(self)
        nxt.execute_move(self.action_to_move(action))
        return nxt

    def _wins(self, r, q, me):
        b, n = self._board, self._n
        for dr, dq in LINES:
            run = 1
            for s in (1, -1):
                rr, qq = r + s * dr, q + s * dq
                while 0 <= rr < n and 0 <= qq < n and b[rr, qq] == me:
                    run += 1
                    rr += s * dr
                    qq += s * dq
            if run >= self._need:
                return True
        return False

    def execute_move(self, move):
        r, q = move
        me = self._player.num
        if self._board[r, q] != 0:
            raise ValueError("Invalid move: occupied")
        self._board[r, q] = me
        self._curr_turn += 1
        if self._wins(r, q, me):
            self._outcome = GameOutcome.WON
        elif not (self._board == 0).any():
            self._outcome = GameOutcome.DRAW
        self.player = self._player.opponent

    def valid_actions_mask(self):
        return (self._board.reshape(-1) == 0).astype(int)

    def to_planes(self):
        me = self._player.num
        return np.stack([(self._board * me > 0).astype(int), (self._board * me < 0).astype(int),
                         np.ones_like(self._board)])

    def _sym(self, x, k, flip):
        y = np.rot90(x, k, axes=(-2, -1))
        return np.flip(y, axis=-1).copy() if flip else y.copy()

    def symmetries(self, board_like):
        return [self._sym(board_like, k & 3, k >> 2) for k in range(8)]

    def random_symmetry(self, board_like):
        k = np.random.randint(0, 4)
        flip = np.random.randint(0, 2)
        return self._sym(board_like, k, flip)

    def move_to_action(self, move):
        return int(move[0] * self._n + move[1])

    def action_to_move(self, action):
        return int(action) // self._n, int(action) % self._n

    def score(self):
        return 0

    def render(self):
        sym = {1: "R", -1: "B", 0: "."}
        print("\n".join(" ".join(sym[int(x)] for x in row) for row in self._board))
