"""Player colours and game outcomes of the plugin API (reference flags.py:6-44).

Values are part of the hot path's arithmetic: a terminal state backs up
-outcome.value (MCTS.py:87), DRAW counts 1e-4 (flags.py:34).
"""
from enum import Enum

import numpy as np


class PlayerColour(Enum):
    RED = 1, "R"
    BLUE = -1, "B"

    def __init__(self, num, token):
        self.num = num
        self.token = token

    @classmethod
    def from_piece(cls, piece):
        if piece > 0:
            return cls.RED
        if piece < 0:
            return cls.BLUE
        raise IndexError(f"No player owns piece {piece}")

    @property
    def opponent(self):
        return PlayerColour.BLUE if self is PlayerColour.RED else PlayerColour.RED

    def owns(self, piece):
        """piece * num > 0, elementwise for arrays."""
        return np.multiply(piece, self.num) > 0


class GameOutcome(Enum):
    ONGOING = 0
    DRAW = 1e-4
    WON = 1
    LOST = -1

    def opposite(self):
        if self is GameOutcome.WON:
            return GameOutcome.LOST
        if self is GameOutcome.LOST:
            return GameOutcome.WON
        return self


def ongoing(outcome):
    """outcome == ONGOING for this module's GameOutcome or any enum with the same values (a
    plugin written against the reference's flags.py compares with ITS enum, whose members
    are not this one's)."""
    return getattr(outcome, "value", outcome) == 0
