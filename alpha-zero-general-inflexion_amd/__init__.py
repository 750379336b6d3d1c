"""azg_amd -- MI355X-native batched self-play engine for alpha-zero-general-inflexion.

Hot path replaced: Coach.executeEpisode -> MCTS.getActionProb -> MCTS.search
(reference Coach.py:41-90, MCTS.py:33-145), run for thousands of games at once
by the HIP kernels of libazg.so (csrc/), with the leaf evaluations batched
through a PyTorch-ROCm network.  Import as `import azg_amd` from the repo root.
"""
PACKAGE_DIR = __path__[0]

from . import _lib  # noqa: E402,F401
