"""The generic plugin path: MCTS over any Game plugin the engine has no kernels for.

The engine's kernels restate the rules of the games it knows (InflexionGame(7),
OthelloGame(6|8); engine.game_spec).  Any other Game subclass (Game.py:8-181) -- a new
plugin, or a subclass of a known one that may override its rules -- is searched here, on
the host, by calling the plugin's own methods exactly where the reference search does
(MCTS.py:62-145: to_planes, outcome, random_symmetry, valid_actions_mask, to_next_state),
while the leaves of all games in flight are evaluated as ONE batch by the network on the
GPU (one forward per simulation step instead of one per leaf).

Per game the search is the reference's, operation for operation:
  * node key = to_planes().tobytes(); a finished game returns -outcome.value (a Python
    number, MCTS.py:83-87);
  * a new key: P, v = network(random_symmetry(planes)); P *= valid mask; s = P.sum()
    (numpy's own f32 pairwise sum); P /= s, or the uniform fallback over the valid actions
    when s == 0 (MCTS.py:89-112); the value returned up is -v (f32);
  * otherwise PUCT over the valid actions in action order, strict > (first index wins a
    tie, NaN never wins): with an edge u = Q + cpuct P sqrt(Ns) / (1 + N), without one
    u = cpuct P sqrt(Ns + 1e-8) (MCTS.py:114-131), evaluated for all valid actions at once
    in f32 with the same rounding steps as numpy's scalar expression under NEP 50
    (f32(cpuct) P, times f32(sqrt_f64(Ns)), over f32(1 + N), plus f32(Q));
  * backup with the reference's own arithmetic on the same Python / numpy types
    (MCTS.py:136-145): Q = (N Q + v) / (N + 1) -- f32 where an f32 value took part, f64
    where only Python numbers (terminal values) did.
The tree persists across moves (MCTS.py:24-31).  Each game draws from its own numpy stream
(the reference's global RandomState, seeded per game as np.random.seed(seed) would), which
is swapped into numpy's global state around every plugin call that draws, so a game's
draws and results are those of the reference's single-game run with that seed
(tests/test_generic_plugin.py against reference traces, tests/golden/toygame.py).
"""
import math

import numpy as np
import torch

from .flags import ongoing

EPS = 1e-8


class _Node:
    """One expanded state: priors and edge statistics over its valid actions (action order)."""
    __slots__ = ("acts", "P", "Ns", "N", "Q", "Qv")

    def __init__(self, acts, P):
        self.acts = acts                       # valid actions, ascending (int64)
        self.P = P                             # f32 priors of those actions
        self.Ns = 0
        self.N = np.zeros(len(acts), np.int64)
        self.Q = np.zeros(len(acts), np.float64)   # f32(Q) is what PUCT reads (exact for f32-typed Q)
        self.Qv = [None] * len(acts)               # the Q objects themselves (np.float32 or Python float)


def _as_evaluator(nnet, device=None):
    """A batched leaf evaluator planes [L, C, n, n] (numpy ints) -> (P f32 [L, A], v f32 [L]).

    nnet: a NNetWrapper-like object (its .nnet torch module), a torch module returning
    (log_softmax, tanh) or (probabilities, tanh) with `outputs_probs`, or a plain callable
    taking and returning numpy arrays (e.g. a test evaluator).  A torch module runs on the
    GPU -- there is no CPU fallback for the network."""
    module = getattr(nnet, "azg_evaluator", None) or getattr(nnet, "nnet", nnet)
    if isinstance(module, torch.nn.Module) or (callable(module) and getattr(module, "outputs_probs", False)):
        if not torch.cuda.is_available():
            raise RuntimeError("the generic plugin path evaluates its leaves on the GPU (no CPU fallback)")
        dev = torch.device(device) if device is not None else torch.device("cuda")
        if isinstance(module, torch.nn.Module):
            module = module.to(dev).eval()
        probs = getattr(module, "outputs_probs", False)

        def evaluate(planes):
            # NNet.py:86-94: board.astype(float64) -> f32 tensor; exp(log_softmax), tanh
            x = torch.as_tensor(np.asarray(planes).astype(np.float64), dtype=torch.float32, device=dev)
            with torch.no_grad():
                pi, v = module(x)
                P = pi if probs else torch.exp(pi)
            return P.float().cpu().numpy(), v.float().reshape(-1).cpu().numpy()
        return evaluate
    if callable(module):
        return module
    raise TypeError("nnet must be a NNetWrapper-like object, a torch module or a callable evaluator")


class _Slot:
    """One game's search state: tree, root, RNG stream (None: numpy's global stream)."""
    __slots__ = ("tree", "rng", "path", "game", "planes", "valid", "key")

    def __init__(self, rng=None):
        self.tree = {}
        self.rng = rng
        self.path = None


class HostSearch:
    """MCTS (MCTS.py:16-148) for any number of games of any Game plugin, the leaves of one
    simulation step of all games evaluated together (module docstring)."""

    def __init__(self, nnet, args, num_games=1, device=None, rngs=None):
        self.evaluate = _as_evaluator(nnet, device)
        self.args = args
        self.cpuct = args.cpuct
        self.slots = [_Slot(rngs[i] if rngs is not None else None) for i in range(num_games)]
        self.expansions = 0
        self.terminal_hits = 0
        self.fallbacks = 0

    # ---------------------------------------------------------------- numpy stream per game
    def _draw(self, slot, fn):
        """fn() with numpy's global stream set to the slot's own (if it has one)."""
        if slot.rng is None:
            return fn()
        saved = np.random.get_state()
        np.random.set_state(slot.rng)
        try:
            return fn()
        finally:
            slot.rng = np.random.get_state()
            np.random.set_state(saved)

    # ---------------------------------------------------------------- PUCT (MCTS.py:114-131)
    def _select(self, node):
        cp = np.float32(self.cpuct) * node.P
        has = node.N > 0
        u = cp * np.float32(math.sqrt(node.Ns + EPS))
        if has.any():
            t = (cp * np.float32(math.sqrt(node.Ns))) / (1 + node.N).astype(np.float32)
            u = np.where(has, node.Q.astype(np.float32) + t, u)
        u = np.where(np.isnan(u), np.float32(-np.inf), u)
        i = int(np.argmax(u))
        if not u[i] > -np.inf:
            raise RuntimeError("MCTS: no action beats -inf at a searched node (the reference's best_act = -1)")
        return i

    # ---------------------------------------------------------------- one simulation per game
    def _descend(self, slot, game):
        """Walk from `game` to a leaf (or a finished game).  Returns ("leaf", None) with
        the leaf stored on the slot, or ("value", v) for a terminal value to back up."""
        path = []
        while True:
            planes = game.to_planes()
            key = planes.tobytes()
            status = game.outcome
            if not ongoing(status):
                self.terminal_hits += 1
                slot.path = path
                return -status.value
            node = slot.tree.get(key)
            if node is None:
                slot.path = path
                slot.key = key
                slot.planes = self._draw(slot, lambda: game.random_symmetry(planes))
                slot.valid = game.valid_actions_mask()
                return None
            i = self._select(node)
            path.append((node, i))
            game = game.to_next_state(int(node.acts[i]))

    def _expand(self, slot, P, v):
        """MCTS.py:89-112 for the slot's pending leaf; returns the value backed up (-v, f32)."""
        valid = slot.valid
        P = np.asarray(P, np.float32) * valid
        P = P.astype(np.float32)
        s = P.sum()
        if s > 0:
            P = P / s
        else:
            self.fallbacks += 1
            P = P + valid
            P = P.astype(np.float32)
            P = P / P.sum()
        acts = np.nonzero(valid)[0]
        slot.tree[slot.key] = _Node(acts, P[acts].astype(np.float32))
        self.expansions += 1
        return -np.float32(v)

    @staticmethod
    def _backup(path, v):
        """MCTS.py:136-145 from the leaf's parent up to the root; v is the leaf's return value."""
        for node, i in reversed(path):
            n = int(node.N[i])
            if n:
                q = (n * node.Qv[i] + v) / (n + 1)
            else:
                q = v
            node.Qv[i] = q
            node.Q[i] = float(q)
            node.N[i] = n + 1
            node.Ns += 1
            v = -v

    def simulate(self, games):
        """One MCTS.search from games[k] for every slot k whose game is not None."""
        pending = []
        for k, g in enumerate(games):
            if g is None:
                continue
            slot = self.slots[k]
            val = self._descend(slot, g)
            if val is None:
                pending.append(k)
            else:
                self._backup(slot.path, val)
        if not pending:
            return
        planes = np.stack([self.slots[k].planes for k in pending])
        P, v = self.evaluate(planes)
        for j, k in enumerate(pending):
            slot = self.slots[k]
            self._backup(slot.path, self._expand(slot, P[j], v[j]))

    def root_counts(self, k, game):
        """Nsa of every action at the root (MCTS.py:48-49), int64 [max_actions]."""
        counts = np.zeros(game.max_actions, np.int64)
        node = self.slots[k].tree.get(game.to_planes().tobytes())
        if node is not None:
            counts[node.acts] = node.N
        return counts

    def nodes(self, k):
        return len(self.slots[k].tree)


def action_probs(counts, temp):
    """getActionProb's policy from root counts (MCTS.py:51-60): the temperature-0 one-hot
    (ties broken by np.random.choice on the current global stream) or counts^(1/temp)."""
    if temp == 0:
        best = np.argwhere(counts == np.max(counts)).ravel()
        pick = np.random.choice(best)
        probs = np.zeros(len(counts), dtype=np.int8)
        probs[pick] = 1
        return probs
    c = counts ** (1.0 / temp)
    return c / c.sum()


class HostSelfPlay:
    """Coach.executeEpisode (Coach.py:41-90) for G games of a plugin at once on HostSearch:
    game i seeded as np.random.seed(seed_base + first_game + i), so its examples are the
    reference's single-game episode with that seed."""

    def __init__(self, template, nnet, args, num_games, seed_base=0, first_game=0, device=None):
        self.template = template
        self.args = args
        self.G = int(num_games)
        rngs = []
        for i in range(self.G):
            rs = np.random.RandomState((int(seed_base) + int(first_game) + i) & 0xFFFFFFFF)
            rngs.append(rs.get_state())
        self.search = HostSearch(nnet, args, self.G, device, rngs)

    def play(self, label_mode="reference"):
        """Play every game to its end; returns (examples per game, records per game)."""
        from .coach import build_examples
        G, sims = self.G, int(self.args.numMCTSSims)
        tt = int(self.args.tempThreshold)
        games = [self.template.restarted() for _ in range(G)]
        steps = [0] * G
        hist = [([], [], [], [], []) for _ in range(G)]  # planes, pis, players, actions, root counts
        out = [None] * G
        while any(g is not None for g in games):
            for _ in range(sims):
                self.search.simulate(games)
            for k, g in enumerate(games):
                if g is None:
                    continue
                slot = self.search.slots[k]
                steps[k] += 1
                temp = int(steps[k] < tt)
                counts = self.search.root_counts(k, g)
                pi = self.search._draw(slot, lambda: action_probs(counts, temp))
                action = self.search._draw(slot, lambda: np.random.choice(len(pi), p=pi))
                planes, pis, players, actions, cnts = hist[k]
                cnts.append(counts)
                planes.append(g.to_planes())
                pis.append(pi)
                players.append(g.player.num)
                actions.append(int(action))
                g = g.to_next_state(action)
                if not ongoing(g.outcome):
                    out[k] = (build_examples(g, planes, pis, players, g, label_mode),
                              {"actions": actions, "counts": cnts, "moves": len(actions), "final": g})
                    games[k] = None
                else:
                    games[k] = g
        return out

    def rng_state(self, k):
        return self.search.slots[k].rng


__all__ = ["HostSearch", "HostSelfPlay", "action_probs"]
