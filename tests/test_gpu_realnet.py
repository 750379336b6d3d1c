"""Search parity with the PRODUCTION evaluator: the engine driven by the real
network reproduces the reference's visit counts with the reference's own network.

Fixtures (tests/golden/make_golden.py `realnet`, `realnet_othello`): the reference
Coach.executeEpisode (Coach.py:41-90) + MCTS (MCTS.py:33-145) with the reference
NNetWrapper (inflexion/pytorch/NNet.py:78-94, batch-1 CPU f32) over the 512-channel
InflexionNNet built under torch.manual_seed(0) -- whole 344-move Inflexion episodes at
main.py's 25 sims (4 seeds), 40-turn games at C3's 100 sims (2 seeds), and whole games
of the builder's Othello plugin: 6x6 at 25 sims (C1, 4 seeds), 8x8 at 25 sims (2) and
at C5's 200 sims (1).

Each is replayed by:
  * the drop-in MCTS + Coach.executeEpisode with an NNetWrapper (batch-1 forward of
    the reference module on the GPU), and with InferenceNet(conv="miopen", gemm="f32")
    as its evaluator (the form INTEGRATION.md recommends for the drop-in) -- all 8
    realnet_main seeds;
  * SelfPlayEngine with InferenceNet(gemm="split") at 4096 concurrent games -- the
    benchmarked path (Winograd transforms, split-fp16 MFMA GEMMs, split-K fc1) -- and at
    C2's 256 and 512 games (the split GEMM's 128 / 64-row schedules; below FC1_SPLIT_MIN_BATCH
    the small-batch libazg FC tail, fc1 transposed: InferenceNet.fc_tail_small, the default since
    round 5);
  * the same with InferenceNet(gemm="f32") (f32 hipBLASLt GEMMs) at 1024 games.
pi returned by getActionProb is a function of the counts (MCTS.py:48-60), so equal
counts give pi exactly (tolerance 0, inside the north_star's 1e-5).

What is asserted, per seed, against the reference's visit counts:
  * the first 40 moves identical, count for count (the 40-move traces SURVEY hard
    part 5 measured as robust to 1e-6 perturbations of the network; 16 for the
    32-60-move Othello games; the sims100 games must match entirely);
  * every later move identical up to the first difference, if any, and that
    difference a single search decision (one simulation of the move that took
    another action: two counts differing by one) AT A MOVE WHERE THE REFERENCE'S
    OWN TRACE CHANGES when its network's weights move by 1e-7 or 1e-6 relative
    (tests/golden/realnet_sensitivity.json.gz: seed 0 at move 222, seed 3 at move
    197 -- the very moves where the GPU runs differ).  A GPU network agrees with the
    CPU one to ~1e-6 relative (root priors here: ~5e-9 absolute), and over a whole
    344-move game the search meets PUCT ties closer than that: the reference's OWN
    traces diverge the same way when its network's weights (or outputs) move by
    1e-7 or 1e-6 relative.  Every flip is reported with its move and the root's prior
    error and smallest prior gap; a mismatch of any other shape -- more than one
    decision, inside the first 40 moves, or at a move the reference's own perturbed
    runs do not certify as a near-tie -- fails;
  * after a certified flip the game goes on being compared: the flipped move's counts
    must equal those of the reference's own perturbed run that diverges there
    (tests/golden/realnet_branches.json.gz), and every later move is compared with that
    run (final board, outcome and RNG position included) -- the game the reference
    itself plays when its rounding falls the other way.  Each test prints how many of
    its moves were compared (all of them, on MI355X).
The sims100 games (40 turns) must match entirely.

The peaked-prior network (fc3 x 16: logits 16x larger, so every f32 evaluation -- the reference's own
module on a GPU included -- moves its priors by up to ~6e-5 in log space, test_leaf_parity_peaked) is
held to a sharper certificate: tests/golden/paths_peaked_*.npz record, for every simulation of the
reference's traces (and of its weight-perturbed branch runs), the leaf it evaluated and the closest PUCT
decision on its way down.  The engine's leaf sequence is recorded too; a mismatch of any shape, at any
move, passes only when the first simulation whose leaf differs descends through a decision the reference
itself makes by less than DECISION_TAU (2 x the leaf error bound) -- about 20 of a game's 8,600
simulations, so it certifies the located near-tie, not the game.
"""
import numpy as np
import pytest
import torch

import oracle_lib as ol

pytestmark = pytest.mark.gpu

G_ENGINE = 4096  # the benchmarked leaf batch (split-K fc1 needs >= 1024 leaves)


class Args(dict):
    __getattr__ = dict.__getitem__


# per fixture set: game, board side, moves that must match before a certified near-tie may flip
SETS = {"realnet_main": ("inflexion", 7, 40), "realnet_sims100": ("inflexion", 7, None),
        "realnet_othello6": ("othello", 6, 16), "realnet_othello8": ("othello", 8, 16),
        "realnet_othello8_s200": ("othello", 8, 16),
        # the network the reference trains on its own self-play (make_golden.py trained_net):
        # Coach.learn's second iteration searches with it (Coach.py:110, :152)
        "trained_main": ("inflexion", 7, 40), "trained_sims100": ("inflexion", 7, None),
        # the peaked-prior network (make_golden.py peaked_net: the trained network's fc3 x 16; median
        # root top prior 0.66 vs 0.038): deep trees, near-ties between a few strong actions
        "peaked_main": ("inflexion", 7, 40), "peaked_sims100": ("inflexion", 7, None)}


def _trained(name):
    return name.startswith("trained") or name.startswith("peaked")


def _family(name):
    return "peaked" if name.startswith("peaked") else "trained" if name.startswith("trained") else "realnet"


def _ref_net(game="inflexion", n=7, name="realnet_main"):
    """The reference's network for the game, as NNetWrapper(game) builds it under manual_seed(0)
    (trained / peaked sets: with the weights of tests/golden/trained_net.npz, fc3 scaled for peaked)."""
    import azg_amd  # noqa: F401
    from azg_amd.nnet import InflexionNNet
    torch.manual_seed(0)
    if game == "inflexion":
        return ol.golden_net(InflexionNNet(), name).cuda().eval()
    return InflexionNNet(n=n, depth=2, action_size=n * n + 1).cuda().eval()


def _game(name, cfg):
    from azg_amd.inflexion import InflexionGame
    from azg_amd.othello import OthelloGame
    kind, n, _ = SETS[name]
    return InflexionGame(7, max_turns=cfg["max_turns"], max_power=6) if kind == "inflexion" else OthelloGame(n)


def _margin_report(net, evaluator, board, turn, player, template, batch=G_ENGINE):
    """Root priors at a failing move: the evaluator on the GPU (at the batch size
    it ran at) against the reference's arithmetic (the module on the CPU, batch 1)."""
    import copy
    from azg_amd.flags import PlayerColour
    g = template.restarted()
    n = g._n
    g._board = np.asarray(board).reshape(n, n).astype(int)
    g._curr_turn = turn
    g._player = PlayerColour.RED if player == 1 else PlayerColour.BLUE
    x = torch.as_tensor(g.to_planes(), dtype=torch.float32).unsqueeze(0)
    with torch.no_grad():
        p_ref = torch.exp(copy.deepcopy(net).cpu()(x)[0][0]).numpy()
        if isinstance(evaluator, str) or evaluator is None:  # the drop-in: the module, batch 1
            p_ev = torch.exp(net(x.cuda())[0][0]).cpu().numpy()
        else:
            xb = x.cuda().expand(batch, *x.shape[1:]).contiguous()
            p_ev = evaluator(xb)[0][0].cpu().numpy()
    valid = g.valid_actions_mask().astype(bool)
    pv = np.sort(p_ref[valid])
    gap = float(np.min(np.diff(pv))) if len(pv) > 1 else float("inf")
    return f"root prior error {float(np.max(np.abs(p_ev - p_ref)[valid])):.3g}, smallest prior gap {gap:.3g}"


def _sensitivity(name):
    fname = ("realnet_sensitivity_othello.json.gz" if "othello" in name else
             f"{_family(name)}_sensitivity.json.gz")
    try:
        d = ol.load_json(fname)
    except FileNotFoundError:
        return {}
    return {(r["kind"], r["eps"], r["seed"]): r["first_divergent_move"] for r in d["runs"]
            if r.get("set", "realnet_main") == name}


def _branches(name):
    """The perturbed reference's traces past its divergent moves (make_golden.py `branches`):
    {(seed, move): [branch, ...]}."""
    if name not in ("realnet_main", "trained_main", "peaked_main"):
        return {}
    try:
        d = ol.load_json(f"{_family(name)}_branches.json.gz")
    except FileNotFoundError:
        return {}
    out = {}
    for b in d["branches"]:
        out.setdefault((b["seed"], b["from_move"]), []).append(b)
    return out


# Decision certificate (tests/golden/paths_<set>.npz, make_golden.py gen_peaked_paths): a run whose leaf
# sequence first leaves the reference's at simulation k took another branch at one of simulation k's
# PUCT decisions; that is rounding, not a bug, when the reference's own closest decision on simulation
# k's way down is nearer a tie than the evaluator's error can move it: the evaluators' priors agree with
# the reference's to LEAF_LOG_ERR in log space on the reference's own leaves (test_leaf_parity_peaked),
# so two upper confidence bounds can swap when they are within 2 x that of each other.
LEAF_LOG_ERR = 6.25e-5
DECISION_TAU = 2 * LEAF_LOG_ERR


def _paths(name, weights_eps=None):
    """{seed: (leaf keys, decision gaps)} of the reference's trace (or, with weights_eps, of its
    weight-perturbed branch runs), one entry per simulation."""
    import os
    tag = "" if weights_eps is None else f"_w{weights_eps:g}"
    path = os.path.join(os.path.dirname(__file__), "golden", f"paths_{name}{tag}.npz")
    if not os.path.exists(path):
        return None
    d = np.load(path)
    return {int(sd): (d["leaf"][d["offsets"][j]:d["offsets"][j + 1]], d["gap"][d["offsets"][j]:d["offsets"][j + 1]])
            for j, sd in enumerate(d["seeds"])}


def _leaf_keys(rows):
    """leaf_key (make_golden.py) of each recorded planes row (int8, [4 * n * n])."""
    import hashlib
    return np.array([int.from_bytes(hashlib.sha256(r.tobytes()).digest()[:8], "little", signed=True) for r in rows],
                    np.int64)


class LeafRecorder:
    """The evaluator with the planes of the first `slots` leaf rows of every call kept (as int8, on the
    device) -- the engine's leaf sequence of the fixture's game slots, for the decision certificate.
    The row index is a device counter, so calls replayed from a captured HIP graph (the drop-in MCTS)
    are recorded too."""

    def __init__(self, ev, slots, max_calls):
        self.ev, self.slots, self.max_calls = ev, slots, max_calls
        self.buf = self.idx = None

    def __getattr__(self, name):
        return getattr(self.ev, name)

    def __call__(self, planes):
        if self.buf is None:
            self.buf = torch.zeros((self.max_calls, self.slots, planes[0].numel()), dtype=torch.int8,
                                   device=planes.device)
            self.idx = torch.zeros(1, dtype=torch.long, device=planes.device)
        rows = planes[:self.slots].reshape(1, self.slots, -1).to(torch.int8)
        self.buf.index_copy_(0, self.idx.clamp(max=self.max_calls - 1), rows)
        self.idx += 1
        return self.ev(planes)

    def rows(self, slot, n):
        k = int(self.idx.item()) if self.idx is not None else 0
        return self.buf[:min(n, k, self.max_calls), slot].cpu().numpy() if k else np.zeros((0, 0), np.int8)


def _leaf_certificate(paths, name, seed, rec, slot, sims):
    """leaf_cert for _check_episode: (first simulation whose leaf differs, sims per move, the reference's
    closest decision on it) against the reference's trace, or -- br, a weight-perturbed branch the run
    has followed -- against that branch's run from the run's first departure from the trace on."""
    def cert(m, br=None):
        got = _leaf_keys(rec.rows(slot, (m + 1) * sims))

        def first(keys, gaps, start):
            for k in range(start, min(len(got), len(keys))):
                if keys[k] != 0 and keys[k] != got[k]:
                    return k, sims, float(gaps[k])
            return None
        c0 = first(*paths[seed], 0)
        if br is None:
            return c0
        bp = _paths(name, br["eps"])
        if bp is None or seed not in bp or c0 is None:
            return None
        return first(*bp[seed], c0[0])
    return cert


def _first_mismatch(moves, counts, actions, n_moves, start, A):
    """First move index m >= start at which (counts, action) differ from `moves` (a list
    indexed from `start`), or None if they agree through the end of `moves`."""
    for j, mv in enumerate(moves):
        m = start + j
        if m < n_moves and np.array_equal(counts[m], ol.golden_counts(mv, A)) and actions[m] == mv["action"]:
            continue
        return m
    return None


def _hidden_flip(cert, where, seed):
    """A game whose every move's counts equal the reference's may still have taken another branch inside
    its tree (a subtree later discarded): its leaf sequence says so.  Such a departure must sit on a
    certified near-tie like any other."""
    if cert is None:
        return
    k, sims, gap = cert
    assert gap < DECISION_TAU, (where, seed, f"leaf sequence leaves the reference's at simulation {k % sims} of "
                                f"move {k // sims}, closest decision {gap:.3g} relative: not a near-tie")
    print(f"HIDDEN FLIP {where}: seed {seed}: counts equal the reference's on every move; the leaf sequence leaves "
          f"it at simulation {k % sims} of move {k // sims} (closest decision {gap:.3g} relative), inside a subtree "
          "the game did not take")


def _check_episode(ep, counts, actions, n_moves, where, report, name, final=None, leaf_cert=None):
    """Compare one episode with the reference.  Returns (first divergent move from the
    reference's own trace or None, moves compared, branch followed or None).

    After a certified near-tie flip the comparison does not stop: if the flipped move's
    counts equal those of the reference's own perturbed run that diverges at that move
    (realnet_branches.json.gz: the same reference search with its weights moved by 1e-7 /
    1e-6), the rest of the game is compared move for move against that branch -- the
    game the reference plays when its arithmetic takes the other side of the tie.  A
    mismatch on the branch fails unless it too is a single search decision (reported)."""
    min_prefix = SETS[name][2]
    whole = min_prefix is None
    A = len(counts[0]) if n_moves else 0

    def shape(m, want_moves, off):
        mv = want_moves[m - off]
        want = ol.golden_counts(mv, A)
        got = counts[m] if m < n_moves else None
        diff = np.nonzero(got != want)[0].tolist() if got is not None else []
        msg = (f"{where}: seed {ep['seed']} move {m} (turn {mv['turn']}): counts differ at actions {diff[:8]} "
               f"(engine {got[diff[:8]].tolist() if got is not None else None}, reference {want[diff[:8]].tolist()})")
        single = (got is not None and len(diff) == 2 and int(np.abs(got - want).sum()) == 2
                  and int(got.sum()) == int(want.sum()))
        return msg, single, mv

    m = _first_mismatch(ep["moves"], counts, actions, n_moves, 0, A)
    if m is None:
        assert n_moves == ep["n_moves"], (where, ep["seed"])
        return None, n_moves, None
    msg, single_flip, mv = shape(m, ep["moves"], 0)
    sens = _sensitivity(name)
    certified = any(sens.get(("weights", eps, ep["seed"])) == m for eps in (1e-7, 1e-6))
    cert = leaf_cert(m) if leaf_cert is not None else None
    # the peaked network: the decision certificate alone (its f32 error scale makes near-ties common);
    # the others keep the weight-perturbation rule, and where the leaf record exists the flip must also
    # sit on a near-tie decision
    peaked = _family(name) == "peaked"
    if peaked and cert is not None and cert[2] < DECISION_TAU:
        k, sims, gap = cert
        print(f"DECISION-CERTIFIED FLIP {msg}; {report(mv)}; identical counts through move {m - 1}; the leaf "
              f"sequence first leaves the reference's at simulation {k % sims} of move {k // sims}, whose closest "
              f"PUCT decision in the reference is {gap:.3g} relative (< {DECISION_TAU:.3g} = 2 x the evaluators' "
              f"leaf prior error bound)")
    elif peaked or whole or m < min_prefix or not single_flip or not certified or (
            cert is not None and cert[2] >= DECISION_TAU):
        raise AssertionError(msg + "; " + report(mv) + ("" if certified else "; the reference's own trace does "
                             "not diverge at this move when its weights move by 1e-7 or 1e-6")
                             + (f"; leaf sequence first differs at simulation {cert[0]}, closest decision there "
                                f"{cert[2]:.3g} relative (not below {DECISION_TAU:.3g})" if cert is not None else ""))
    else:
        print(f"NEAR-TIE FLIP {msg}; {report(mv)}; identical through move {m - 1}; the reference's own trace with "
              f"its weights moved by 1e-7 / 1e-6 first diverges at move "
              f"{sens.get(('weights', 1e-7, ep['seed']), '?')} / {sens.get(('weights', 1e-6, ep['seed']), '?')} "
              "(None: never)" + (f"; leaf sequence first leaves the reference's at simulation {cert[0] % cert[1]} "
                                 f"of move {cert[0] // cert[1]}, closest decision {cert[2]:.3g} relative"
                                 if cert is not None else ""))
    for br in _branches(name).get((ep["seed"], m), []):
        if not (m < n_moves and np.array_equal(counts[m], ol.golden_counts(br["moves"][0], A))):
            continue
        m2 = _first_mismatch(br["moves"], counts, actions, n_moves, m, A)
        if m2 is None:
            assert n_moves == br["n_moves"], (where, ep["seed"], "branch length")
            if final is not None:
                final(br)
            print(f"BRANCH {where}: seed {ep['seed']} follows the reference's eps={br['eps']:g} branch from move {m} "
                  f"to the end of the game ({n_moves} moves, final board / outcome / RNG position equal)")
            return m, n_moves, br
        msg2, single2, mv2 = shape(m2, br["moves"], m)
        cert2 = leaf_cert(m2, br) if leaf_cert is not None else None
        if cert2 is not None and cert2[2] < DECISION_TAU:
            print(f"BRANCH {where}: seed {ep['seed']} follows the reference's eps={br['eps']:g} branch from move {m} "
                  f"through move {m2 - 1}; at {m2}: DECISION-CERTIFIED {msg2}; {report(mv2)}; the leaf sequence "
                  f"first leaves the branch's at simulation {cert2[0] % cert2[1]} of move {cert2[0] // cert2[1]}, "
                  f"closest decision there {cert2[2]:.3g} relative")
            return m, m2, br
        if not single2:
            raise AssertionError(f"on the reference's eps={br['eps']:g} branch from move {m}: " + msg2 + "; "
                                 + report(mv2) + (f"; leaf sequence first leaves the branch's at simulation "
                                                  f"{cert2[0]}, closest decision {cert2[2]:.3g}" if cert2 else ""))
        print(f"BRANCH {where}: seed {ep['seed']} follows the reference's eps={br['eps']:g} branch from move {m} "
              f"through move {m2 - 1}; at {m2} a second single-decision flip: {msg2}; {report(mv2)}")
        return m, m2, br
    print(f"BRANCH {where}: seed {ep['seed']}: no reference branch from move {m} matches the flipped counts")
    return m, m, None


@pytest.mark.parametrize("form", ["split:4096", "split:256", "f32:1024", "small:1", "module:1"])
def test_leaf_parity_peaked(form):
    """The evaluator on the reference's own leaves (tests/golden/peaked_leaves_peaked_sims100_s10.npz:
    the 800 leaves the reference search evaluates in its first 8 moves of peaked_sims100 seed 10, planes
    as NNetWrapper.predict got them, with its P and v): every GPU form's priors within LEAF_LOG_ERR of the
    reference's in log space wherever both are normal floats, v within 1e-6.  The bound the decision
    certificate (DECISION_TAU) rests on.  Forms: the split-fp16 form at the benchmarked 4096 leaves and at
    C2's 256, the f32-GEMM form, the drop-in's batch-1 small-batch kernels, the module itself."""
    import os
    import azg_amd  # noqa: F401
    from azg_amd.nnet import InferenceNet
    d = np.load(os.path.join(os.path.dirname(__file__), "golden", "peaked_leaves_peaked_sims100_s10.npz"))
    kind, B = form.split(":")
    B = int(B)
    net = _ref_net("inflexion", 7, "peaked_main")
    ev = None if kind == "module" else InferenceNet(net, conv="miopen", gemm="f32") if kind == "small" \
        else InferenceNet(net, gemm=kind)
    x = torch.tensor(d["x"].astype(np.float32), device="cuda")
    n = x.shape[0]
    pg, vg = [], []
    with torch.no_grad():
        for i in range(0, n, B):
            xb = x[i:i + B]
            k = xb.shape[0]
            if k < B:
                xb = torch.cat([xb, xb[:1].expand(B - k, -1, -1, -1)])
            if ev is None:
                a, b = net(xb)
                a = torch.exp(a)
            else:
                a, b = ev(xb)
            pg.append(a[:k].double().cpu().numpy())
            vg.append(b.reshape(-1)[:k].double().cpu().numpy())
    pg, vg = np.concatenate(pg), np.concatenate(vg)
    pr, vr = d["p"].astype(np.float64), d["v"].astype(np.float64)
    normal = (pr >= 2.0 ** -126) & (pg >= 2.0 ** -126)
    lerr = np.abs(np.log(np.where(normal, pg, 1.0)) - np.log(np.where(normal, pr, 1.0)))
    # below the normal range both sides round exp() onto the subnormal grid: the forms agree there too
    # to within a few of its steps, and the reference's zeros stay (near) zero
    sub = ~normal & ((pr > 0) | (pg > 0))
    print(f"{form}: {n} leaves, prior log error max {lerr.max():.3g} (normal range), {int(sub.sum())} subnormal "
          f"entries (max |diff| {np.abs(pg - pr)[sub].max() if sub.any() else 0:.3g}), v error max "
          f"{np.abs(vg - vr).max():.3g}")
    assert lerr.max() <= LEAF_LOG_ERR
    assert np.abs(vg - vr).max() <= 1e-6
    assert (np.abs(pg - pr)[sub] <= 2.0 ** -126).all()


DROPIN_CASES = ([("realnet_main", k) for k in range(8)] + [("realnet_sims100", 0)]
                + [("realnet_othello6", i) for i in range(8)] + [("realnet_othello8", 0)]
                + [("trained_main", k) for k in range(8)] + [("trained_sims100", 0), ("trained_sims100", 1)]
                + [("peaked_main", k) for k in range(8)] + [("peaked_sims100", 0), ("peaked_sims100", 1)])


@pytest.mark.parametrize("form", ["module", "inference"])
@pytest.mark.parametrize("name,k", DROPIN_CASES)
def test_dropin_mcts_real_net(name, k, form):
    """Drop-in MCTS + Coach.executeEpisode, whole episodes (for the 6x6 Othello sets:
    BASELINE configs[0], C1, the reference main.py path on one game), with the leaf
    evaluator as the reference wires it (form="module": the NNetWrapper's own torch module,
    batch 1 on the GPU, MCTS(fast=False)) and in the drop-in's default form (form="inference":
    InferenceNet(nnet.nnet, conv="miopen", gemm="f32"), BN folded, which at one leaf runs on
    libazg's small-batch kernels, azg_small.hip -- what MCTS(fast=True) builds itself)."""
    import hashlib
    import azg_amd  # noqa: F401
    from azg_amd.coach import Coach
    from azg_amd.mcts import MCTS
    from azg_amd.nnet import InferenceNet, NNetWrapper

    data = ol.load_json(f"mcts_{name}.json.gz")
    cfg, ep = data["config"], data["episodes"][k]
    args = Args(numMCTSSims=cfg["sims"], cpuct=cfg["cpuct"], tempThreshold=cfg["temp_threshold"])
    game = _game(name, cfg)
    torch.manual_seed(0)
    wrapper = NNetWrapper(game, device="cuda")
    ol.golden_net(wrapper.nnet, name)
    ev = None
    if form == "inference":
        ev = InferenceNet(wrapper.nnet.eval(), conv="miopen", gemm="f32")
        wrapper.azg_evaluator = ev
    paths = _paths(name)
    rec = None
    if paths is not None:  # the leaf sequence, for the decision certificate
        rec = LeafRecorder(ev if ev is not None else wrapper.nnet.eval(), 1, ep["n_moves"] * cfg["sims"] + 64)
        wrapper.azg_evaluator = rec
    counts, actions = [], []

    class RecMCTS(MCTS):
        def getActionProb(self, g, temp=1):
            p = super().getActionProb(g, temp)
            counts.append(self._engine.root_counts(0))
            return p

    cls = type(game)
    orig = cls.to_next_state

    def tns(self, a):
        actions.append(int(a))
        return orig(self, a)
    np.random.seed(ep["seed"])
    cls.to_next_state = tns
    try:
        ex = Coach(game, wrapper, args).executeEpisode((game.restarted(),
                                                        RecMCTS(wrapper, args, fast=form != "module")))
    finally:
        cls.to_next_state = orig
    net = wrapper.nnet.eval()
    pol = hashlib.sha256(np.array([e[1] for e in ex], np.float64).tobytes()).hexdigest()
    rng_pos = np.random.get_state()[2]

    def final(ref):  # the same game as the reference's (or its branch): same examples and RNG position
        assert pol == ref["policy_sha256"] and len(ex) == ref["n_examples"]
        assert rng_pos == ref["rng_pos"]
    flip, upto, br = _check_episode(ep, counts, actions, len(counts), f"drop-in MCTS ({form})",
                                    lambda mv: _margin_report(net, ev, mv["board"], mv["turn"],
                                                              1 - 2 * (mv["turn"] % 2), game, batch=1),
                                    name, final=final,
                                    leaf_cert=_leaf_certificate(paths, name, ep["seed"], rec, 0, cfg["sims"])
                                    if rec is not None else None)
    if flip is None:
        final(ep)
        if rec is not None:
            _hidden_flip(_leaf_certificate(paths, name, ep["seed"], rec, 0, cfg["sims"])(len(counts) - 1),
                         f"drop-in MCTS ({form})", ep["seed"])


ENGINE_CASES = ([(name, "split", G_ENGINE) for name in SETS] + [(name, "f32", G_ENGINE // 4) for name in SETS]
                # C2's leaf batch (and twice it): the split GEMM's 128 / 64-row schedules and the small-batch
                # libazg FC tail (fc1 transposed, InferenceNet.fc_tail_small)
                + [(name, "split", g) for g in (256, 512) for name in SETS])


@pytest.mark.parametrize("name,gemm,G", ENGINE_CASES)
def test_engine_real_net(name, gemm, G):
    """The batched engine with the production evaluator: the fixture's seeds are game
    slots of a G-game run (seed = slot index + first_game), the other slots are ordinary
    games in the same leaf batches.  G = 4096 (C4 / C3 shapes, C5's 8x8 x 200 sims; the
    split form, benchmarked), 1024 (the f32-GEMM form, a fallback: same kernels, a quarter of
    the leaves keeps the suite short), and 256 / 512 (C2's batch: the split GEMM's 128- and
    64-row tile schedules, and below FC1_SPLIT_MIN_BATCH the small-batch libazg FC tail, fc1
    transposed -- InferenceNet.fc_tail_small)."""
    import azg_amd  # noqa: F401
    from azg_amd.engine import SelfPlayEngine
    from azg_amd.nnet import InferenceNet

    data = ol.load_json(f"mcts_{name}.json.gz")
    cfg, eps = data["config"], data["episodes"]
    kind, n, _ = SETS[name]
    seeds = [ep["seed"] for ep in eps]
    assert seeds == list(range(seeds[0], seeds[0] + len(seeds)))
    net = _ref_net(kind, n, name)
    ev = InferenceNet(net, gemm=gemm)
    paths = _paths(name)
    evaluator = ev
    if paths is not None:
        evaluator = LeafRecorder(ev, len(seeds), max(ep["n_moves"] for ep in eps) * cfg["sims"])
    game = _game(name, cfg)
    e = SelfPlayEngine(G, sims=cfg["sims"], cpuct=cfg["cpuct"], temp_threshold=cfg["temp_threshold"],
                       max_turns=cfg.get("max_turns", 343), seed_base=0, first_game=seeds[0], evaluator=evaluator,
                       game=kind, n=n)
    e.play()
    st = e.stats()
    assert st["error"] == 0
    rec = e.read_moves()
    state = e.state()
    whole = compared = total = 0
    for i, ep in enumerate(eps):
        def final(ref, i=i):
            assert state["boards"][i].tolist() == ref["final_board"]
            assert ol.OUTCOME_VALUE[int(state["outcomes"][i])] == ref["final_outcome"]
            assert e.get_rng(i)[1] == ref["rng_pos"]
        flip, upto, br = _check_episode(
            ep, rec["counts"][i], rec["actions"][i], int(rec["moves"][i]), f"engine gemm={gemm} G={G}",
            lambda mv: _margin_report(net, ev, mv["board"], mv["turn"], 1 - 2 * (mv["turn"] % 2), game, batch=G),
            name, final=final,
            leaf_cert=_leaf_certificate(paths, name, ep["seed"], evaluator, i, cfg["sims"]) if paths else None)
        if flip is None:
            whole += 1
            final(ep)
            if paths:
                _hidden_flip(_leaf_certificate(paths, name, ep["seed"], evaluator, i, cfg["sims"])(
                    int(rec["moves"][i]) - 1), f"engine gemm={gemm} G={G}", ep["seed"])
        compared += upto
        total += int(rec["moves"][i])
    print(f"{name} gemm={gemm} G={G}: {whole} of {len(eps)} games identical to the reference move for move; "
          f"{compared} of {total} moves compared against the reference or its certified branch")
    e.close()


@pytest.mark.parametrize("G", [4093, 1500, 1024])
def test_real_net_batch_composition_invariance(G):
    """Every leaf's evaluation depends on its own planes only: the production evaluator's
    GEMMs, transforms and split-K FC tail never mix rows, whatever the batch size and
    whichever GEMM schedule (persistent 256-row tiles, 128 / 64-row tiles) the size picks.
    So the games a G-game run shares with the 4096-game run -- ragged last tiles and the
    highest slots included -- have the same visit counts and actions bit for bit.  (At
    least 1024 leaves: below FC1_SPLIT_MIN_BATCH the FC tail is the small-batch one, other bits.)"""
    import azg_amd  # noqa: F401
    from azg_amd.engine import SelfPlayEngine
    from azg_amd.nnet import InferenceNet

    net = _ref_net()
    ev = InferenceNet(net)
    recs = {}
    for g in (G_ENGINE, G):
        e = SelfPlayEngine(g, sims=25, cpuct=1, temp_threshold=30, max_turns=343, seed_base=0, first_game=0,
                           evaluator=ev)
        for _ in range(3):
            e.move()
        e.check_evaluator()
        assert e.stats()["error"] == 0
        recs[g] = e.read_moves()
        e.close()
    a, b = recs[G_ENGINE], recs[G]
    assert np.array_equal(a["moves"][:G], b["moves"])
    assert np.array_equal(a["actions"][:G, :3], b["actions"][:, :3])
    assert np.array_equal(a["counts"][:G, :3], b["counts"][:, :3])
