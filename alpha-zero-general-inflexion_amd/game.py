"""Abstract two-player game plugin (reference Game.py:8-181).

Same surface: board_shape, policy_shape, player (+ setter that flips the
outcome, Game.py:49-62), outcome, max_actions, restarted, to_next_state,
to_planes, valid_actions_mask, symmetries, random_symmetry, score,
move_to_action, action_to_move, render.
"""
from math import prod

from .flags import GameOutcome, PlayerColour


class Game:
    def __init__(self, board_shape, policy_shape, first_mover):
        if not (isinstance(board_shape, tuple) and len(board_shape) == 2):
            raise AssertionError("board_shape must be a 2-tuple of ints")
        if not (isinstance(policy_shape, tuple) and len(policy_shape) == 3):
            raise AssertionError("policy_shape must be a 3-tuple of ints")
        if not isinstance(first_mover, PlayerColour):
            raise AssertionError("first_mover must be a PlayerColour")
        self._board_shape = board_shape
        self._policy_shape = policy_shape
        self._firstMover = first_mover
        self._player = first_mover
        self._outcome = GameOutcome.ONGOING

    @property
    def board_shape(self):
        return self._board_shape

    @property
    def policy_shape(self):
        return self._policy_shape

    @property
    def player(self):
        return self._player

    @player.setter
    def player(self, player):
        """Switching to the other player also switches the outcome's point of view."""
        if not isinstance(player, PlayerColour):
            raise AssertionError("player must be a PlayerColour")
        if player != self._player:
            self._player = player
            self._outcome = self._outcome.opposite()

    @property
    def outcome(self):
        return self._outcome

    @property
    def max_actions(self):
        return int(prod(self._policy_shape))

    def restarted(self):
        raise NotImplementedError

    def to_next_state(self, action):
        raise NotImplementedError

    def to_planes(self):
        raise NotImplementedError

    def valid_actions_mask(self):
        raise NotImplementedError

    def symmetries(self, board_like):
        raise NotImplementedError

    def random_symmetry(self, board_like):
        raise NotImplementedError

    def score(self):
        raise NotImplementedError

    def move_to_action(self, move):
        raise NotImplementedError

    def action_to_move(self, action):
        raise NotImplementedError

    def render(self):
        raise NotImplementedError
