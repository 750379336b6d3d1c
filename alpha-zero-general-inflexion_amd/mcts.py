"""Drop-in MCTS (reference MCTS.py:16-148) whose search runs on the GPU engine.

    mcts = MCTS(nnet, args)                 # args.numMCTSSims, args.cpuct
    pi = mcts.getActionProb(game, temp)     # same result as the reference, bit for bit

The tree lives in the engine (one game slot, no node GC, so the tree persists
across calls exactly like the reference's dicts; the node pool holds a whole
game's tree, and a search that still fills it raises AzgError).  The reference draws its
random symmetries from numpy's *global* RandomState (InflexionGame.py:120-121);
this class hands that stream to the engine before the simulations and takes it
back afterwards, so interleaving with the caller's own np.random use
(Coach.py:81) is preserved draw for draw.  The root policy and the temp-0 tie
break (MCTS.py:48-60) run here on the host from the engine's root counts.

`nnet` may be a NNetWrapper-like object (its `.nnet` torch module is used on
the GPU, batched), a torch module returning (log_softmax, tanh), or the string
"stub" (hash evaluator used by the parity tests).
"""
import warnings

import numpy as np
import torch

from .engine import SelfPlayEngine, game_spec
from .flags import GameOutcome


def _evaluator_of(nnet, device):
    if isinstance(nnet, str):
        return nnet
    ev = getattr(nnet, "azg_evaluator", None)
    if ev is not None:
        return ev
    module = getattr(nnet, "nnet", nnet)
    if isinstance(module, torch.nn.Module):
        module = module.to(device)
        module.eval()
        return module
    if callable(module):
        return module
    raise TypeError("nnet must be a NNetWrapper-like object, a torch module or 'stub'")


MAX_NODE_CAPACITY = (1 << 21) - 1  # azg_create's limit


def whole_game_capacity(sims, game):
    """Nodes a whole game's tree can reach: one expansion per simulation, sims per
    move, at most max_turns + 1 moves (2n^2 for Othello: every move fills a cell or
    passes, and two passes end it).  The reference keeps every node for the game
    (MCTS.py:24-30), so the drop-in sizes its pool to hold them all."""
    name, n, max_turns = game_spec(game)
    moves = 2 * n * n if name == "othello" or max_turns <= 0 else max_turns + 1
    return min(int(sims) * moves + 64, MAX_NODE_CAPACITY)


class MCTS:
    def __init__(self, nnet, args, device=None, node_capacity=None, graph=True):
        self.nnet = nnet
        self.args = args
        self.device = torch.device(device) if device is not None else torch.device("cuda")
        self.node_capacity = node_capacity  # None: whole_game_capacity
        # graph: after one eager getActionProb, the numMCTSSims simulations of a call are
        # captured once as a HIP graph and replayed (the search is launch-bound at one
        # leaf per simulation); an evaluator that cannot be captured stays eager
        self.graph = bool(graph)
        self._sims_graph = None
        self._graph_sims = 0
        self._warm = False
        self._engine = None
        self._max_turns = None

    def _engine_for(self, game):
        spec = game_spec(game)
        if self._engine is None or self._max_turns != spec:
            if self._engine is not None:
                self._engine.close()
            name, n, max_turns = spec
            cap = self.node_capacity or whole_game_capacity(self.args.numMCTSSims, game)
            self._engine = SelfPlayEngine(1, sims=int(self.args.numMCTSSims), cpuct=self.args.cpuct,
                                          temp_threshold=1, max_turns=max_turns, game=name, n=n,
                                          evaluator=_evaluator_of(self.nnet, self.device), device=self.device,
                                          node_capacity=cap, max_depth=1024, gc=False, record=False)
            self._max_turns = spec
            self._sims_graph, self._warm = None, False
        return self._engine

    def _capture(self, eng, sims):
        """Record `sims` simulations (select, network, expand/backup) as one graph.
        Capturing launches nothing, so the tree is unchanged."""
        g = torch.cuda.CUDAGraph()
        torch.cuda.synchronize(self.device)
        try:
            with torch.cuda.device(self.device), torch.cuda.graph(g):
                for _ in range(sims):
                    eng.simulate()
        except RuntimeError as e:
            warnings.warn(f"MCTS: evaluator not graph-capturable ({e}); searching eagerly")
            self.graph = False
            torch.cuda.synchronize(self.device)
            return None
        self._sims_graph, self._graph_sims = g, sims
        return g

    def _simulate(self, eng, sims):
        if not self.graph or sims != int(self.args.numMCTSSims):
            for _ in range(sims):
                eng.simulate()
            return
        g = self._sims_graph
        if g is not None and self._graph_sims != sims:  # args.numMCTSSims changed since the capture
            g = self._sims_graph = None
        if g is None and self._warm:
            g = self._capture(eng, sims)
        if g is not None:
            g.replay()
            return
        for _ in range(sims):  # first call: eager, initialises the evaluator's libraries
            eng.simulate()
        self._warm = True

    def _run(self, game, sims):
        if game.outcome != GameOutcome.ONGOING:
            raise ValueError("search from a finished game")
        eng = self._engine_for(game)
        state = np.random.get_state()
        eng.set_rng(0, state[1], state[2])
        eng.set_root(0, game._board, game._curr_turn, game.player.num)
        self._simulate(eng, sims)
        # a full node pool (or any engine error) stops the slot's search: raise rather
        # than return counts from a truncated search (azg_active_games reports it)
        eng.active()
        eng.check_evaluator()
        mt, pos = eng.get_rng(0)
        np.random.set_state((state[0], mt, pos, state[3], state[4]))
        return eng

    def search(self, game):
        """One simulation from `game` (MCTS.py:62-145); updates the tree."""
        self._run(game, 1)

    def getActionProb(self, game, temp=1):
        if not (isinstance(temp, (int, float)) and temp >= 0):
            raise AssertionError("temp must be a number >= 0")
        eng = self._run(game, int(self.args.numMCTSSims))
        counts = eng.root_counts(0).astype(np.int64)
        if temp == 0:
            best = np.argwhere(counts == np.max(counts)).ravel()
            pick = np.random.choice(best)
            probs = np.zeros(len(counts), dtype=np.int8)
            probs[pick] = 1
            return probs
        counts = counts ** (1.0 / temp)
        return counts / counts.sum()

    def stats(self):
        return self._engine.stats() if self._engine is not None else {}

    def reset(self):
        return MCTS(self.nnet, self.args, self.device, self.node_capacity, self.graph)
