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

A Game plugin the engine has no kernels for (engine.game_spec raises: a new plugin, a
subclass of a known one, unsupported parameters) is searched by hostsearch.HostSearch
instead: the reference's search on the host over the plugin's own methods, the leaves
evaluated by the network on the GPU ("unknown Game subclasses fall back to a
CPU path that calls the Python methods").
"""
import itertools
import warnings
import weakref

import numpy as np
import torch

from ._lib import AzgError
from .engine import SelfPlayEngine, game_spec
from .flags import ongoing


# InflexionNNet module -> [weights version, its InferenceNet] (fast_evaluator)
_FAST = weakref.WeakKeyDictionary()


def _weights_version(module):
    """Sum of the autograd version counters of every parameter and buffer: it moves with
    every in-place update (optimizer steps, load_state_dict, dist.broadcast_weights)."""
    return sum(t._version for t in itertools.chain(module.parameters(), module.buffers()))


def fast_evaluator(module, device):
    """The drop-in's leaf evaluator for an InflexionNNet: its InferenceNet (BN folded; at the
    drop-in's one leaf per simulation the small-batch kernels of azg_small.hip),
    cached per module and re-folded in place whenever the module's weights have changed since
    (training between episodes), so captured graphs stay valid."""
    from .nnet import InferenceNet
    ver = _weights_version(module)
    hit = _FAST.get(module)
    if hit is None:
        with torch.cuda.device(device):
            ev = InferenceNet(module.to(device), conv="miopen", gemm="f32")
        _FAST[module] = [ver, ev]
        # the pooled engines keep `ev` (~50 MB of folded weights) alive: drop them with the module
        weakref.finalize(module, _drop_pooled, id(ev))
        return ev
    if hit[0] != ver:
        hit[1].refresh_from(module)
        hit[0] = ver
    return hit[1]


def _evaluator_of(nnet, device, fast=True):
    if isinstance(nnet, str):
        return nnet
    ev = getattr(nnet, "azg_evaluator", None)
    if ev is not None:
        return ev
    module = getattr(nnet, "nnet", nnet)
    if isinstance(module, torch.nn.Module):
        from .nnet import InflexionNNet
        if fast and type(module) is InflexionNNet:
            return fast_evaluator(module, device)
        module = module.to(device)
        module.eval()
        return module
    if callable(module):
        return module
    raise TypeError("nnet must be a NNetWrapper-like object, a torch module or 'stub'")


MAX_NODE_CAPACITY = (1 << 21) - 1  # azg_create's limit

# Engines (and their captured simulation graphs) of MCTS instances that are gone, for the
# next instance with the same evaluator and configuration.  The reference's Coach builds a
# fresh MCTS per episode (Coach.py:110) and Arena per game; each would otherwise create an
# engine, run an eager call and capture a new graph (with its own graph memory pool).  A
# reused engine is reset (empty tree, as a new MCTS's dicts are) before it is handed out,
# and an entry is checked out by one live MCTS at a time.
_POOL = {}
_POOL_MAX = 2  # idle engines kept per key
_POOL_TOTAL_MAX = 4  # idle engines kept over all keys: the least recently released go first
_POOL_ORDER = []  # keys of the idle entries, in release order (one per entry)


def clear_pool():
    """Free the idle engines (and the evaluators and graphs they keep alive)."""
    for idle in _POOL.values():
        for eng, *_ in idle:
            eng.close()
    _POOL.clear()
    _POOL_ORDER.clear()


def _drop_pooled(ev_id):
    """Close the idle engines of an evaluator whose module is gone (weakref.finalize)."""
    for key in [k for k in _POOL if k[0] == ev_id]:
        for eng, *_ in _POOL.pop(key):
            eng.close()
    _POOL_ORDER[:] = [k for k in _POOL_ORDER if k[0] != ev_id]


def _pool_put(key, entry):
    """Keep an idle entry (at most _POOL_MAX per key, _POOL_TOTAL_MAX in all, LRU)."""
    idle = _POOL.setdefault(key, [])
    if len(idle) >= _POOL_MAX:
        entry[0].close()
        return
    idle.append(entry)
    _POOL_ORDER.append(key)
    while len(_POOL_ORDER) > _POOL_TOTAL_MAX:
        old = _POOL_ORDER.pop(0)
        eng = _POOL[old].pop(0)[0]
        if not _POOL[old]:
            del _POOL[old]
        eng.close()


def _pool_get(key):
    idle = _POOL.get(key)
    if not idle:
        return None
    entry = idle.pop()
    if not idle:
        del _POOL[key]
    # this key's most recent release (the entry just taken) leaves the LRU order
    i = len(_POOL_ORDER) - 1 - _POOL_ORDER[::-1].index(key)
    del _POOL_ORDER[i]
    return entry


def whole_game_capacity(sims, game):
    """Nodes a whole game's tree can reach: one expansion per simulation, sims per
    move, at most max_turns + 1 moves (2n^2 for Othello: every move fills a cell or
    passes, and two passes end it).  The reference keeps every node for the game
    (MCTS.py:24-30), so the drop-in sizes its pool to hold them all."""
    name, n, max_turns = game_spec(game)
    moves = 2 * n * n if name == "othello" or max_turns <= 0 else max_turns + 1
    return min(int(sims) * moves + 64, MAX_NODE_CAPACITY)


class MCTS:
    def __init__(self, nnet, args, device=None, node_capacity=None, graph=True, fast=True):
        self.nnet = nnet
        self.args = args
        # fast: an InflexionNNet (e.g. a NNetWrapper's .nnet) is evaluated through its
        # InferenceNet (fast_evaluator); False evaluates the module itself, as the reference does
        self.fast = bool(fast)
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
        self._host = None  # hostsearch.HostSearch for plugins without native rules

    @staticmethod
    def native(game):
        """Whether the engine has rules kernels for this Game instance (engine.game_spec)."""
        try:
            game_spec(game)
            return True
        except AzgError:
            return False

    def _host_search(self):
        if self._host is None:
            from .hostsearch import HostSearch
            self._host = HostSearch(self.nnet, self.args, 1, self.device)
        return self._host

    def _pool_key(self, spec, ev, cap):
        return (id(ev), spec, int(self.args.numMCTSSims), float(self.args.cpuct), cap, str(self.device))

    def _release(self):
        """Hand this instance's engine (and graph) back to the pool."""
        if self._engine is None:
            return
        _pool_put(self._key, (self._engine, self._sims_graph, self._graph_sims, self._warm))
        self._engine, self._sims_graph, self._warm = None, None, False

    def __del__(self):
        try:
            self._release()
        except Exception:
            pass

    def _engine_for(self, game):
        spec = game_spec(game)
        if self._engine is None or self._max_turns != spec:
            self._release()
            name, n, max_turns = spec
            cap = self.node_capacity or whole_game_capacity(self.args.numMCTSSims, game)
            ev = _evaluator_of(self.nnet, self.device, self.fast)
            self._key = self._pool_key(spec, ev, cap)
            entry = _pool_get(self._key)
            if entry is not None:
                self._engine, self._sims_graph, self._graph_sims, self._warm = entry
                self._engine.reset()  # a fresh tree, as a new MCTS's empty dicts
            else:
                self._engine = SelfPlayEngine(1, sims=int(self.args.numMCTSSims), cpuct=self.args.cpuct,
                                              temp_threshold=1, max_turns=max_turns, game=name, n=n,
                                              evaluator=ev, device=self.device, node_capacity=cap, max_depth=1024,
                                              gc=False, record=False)
                self._sims_graph, self._warm = None, False
            self._max_turns = spec
        return self._engine

    def _capture(self, eng, sims):
        """Record `sims` simulations (select, then per simulation the network and the
        backup fused with the next select) as one graph.
        Capturing launches nothing, so the tree is unchanged."""
        g = torch.cuda.CUDAGraph()
        torch.cuda.synchronize(self.device)
        try:
            with torch.cuda.device(self.device), torch.cuda.graph(g):
                eng.simulate_many(sims)
        except AzgError:
            raise  # an engine error is an error, not a capture limitation
        except RuntimeError as e:
            warnings.warn(f"MCTS: evaluator not graph-capturable ({e}); searching eagerly")
            self.graph = False
            torch.cuda.synchronize(self.device)
            return None
        self._sims_graph, self._graph_sims = g, sims
        return g

    def _simulate(self, eng, sims):
        if not self.graph or sims != int(self.args.numMCTSSims):
            eng.simulate_many(sims)
            return
        g = self._sims_graph
        if g is not None and self._graph_sims != sims:  # args.numMCTSSims changed since the capture
            g = self._sims_graph = None
        if g is None and self._warm:
            g = self._capture(eng, sims)
        if g is not None:
            g.replay()
            return
        eng.simulate_many(sims)  # first call: eager, initialises the evaluator's libraries
        self._warm = True

    def _run(self, game, sims):
        if not ongoing(game.outcome):
            raise ValueError("search from a finished game")
        if self._engine is not None and self.fast:
            _evaluator_of(self.nnet, self.device, True)  # re-fold the weights if they were trained since
        if not self.native(game):  # the generic plugin path: numpy's global stream, as the reference
            hs = self._host_search()
            for _ in range(sims):
                hs.simulate([game])
            return None
        eng = self._engine_for(game)
        state = np.random.get_state()
        eng.slot_begin(0, game._board, game._curr_turn, game.player.num, state[1], state[2])
        self._simulate(eng, sims)
        # a full node pool (or any engine error) stops the slot's search: slot_end raises
        # rather than return counts from a truncated search
        counts, mt, pos, _ = eng.slot_end(0)
        eng.check_evaluator()
        np.random.set_state((state[0], mt, pos, state[3], state[4]))
        return counts

    def search(self, game):
        """One simulation from `game` (MCTS.py:62-145); updates the tree."""
        self._run(game, 1)

    def getActionProb(self, game, temp=1):
        if not (isinstance(temp, (int, float)) and temp >= 0):
            raise AssertionError("temp must be a number >= 0")
        counts = self._run(game, int(self.args.numMCTSSims))
        counts = counts.astype(np.int64) if counts is not None else self._host.root_counts(0, game)
        if temp == 0:
            best = np.argwhere(counts == np.max(counts)).ravel()
            pick = np.random.choice(best)
            probs = np.zeros(len(counts), dtype=np.int8)
            probs[pick] = 1
            return probs
        counts = counts ** (1.0 / temp)
        return counts / counts.sum()

    def stats(self):
        if self._host is not None:
            h = self._host
            return {"expansions": h.expansions, "terminal_hits": h.terminal_hits, "fallbacks": h.fallbacks,
                    "nodes": h.nodes(0), "error": 0}
        return self._engine.stats() if self._engine is not None else {}

    def reset(self):
        return MCTS(self.nnet, self.args, self.device, self.node_capacity, self.graph, self.fast)
