/*
 * oracle.c -- plain-C restatement of the reference self-play hot path.
 *
 * TEST INFRASTRUCTURE ONLY (see oracle.h).  Each block cites the reference
 * file:line it restates.  Parity of this restatement is pinned against the
 * fixtures under tests/golden/ that were produced by importing the reference
 * (tests/golden/make_golden.py); tests/test_oracle_golden.py checks it.
 *
 * Float semantics follow NumPy 2.x (NEP 50) as the reference experiences them
 * (SURVEY.md 8(a) a4-a6): numpy f32 arrays mixed with weak Python scalars stay
 * f32, math.sqrt is double, terminal values are Python numbers (double).
 */
#include "oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------------ RNG
 * numpy/random/src/legacy + mt19937: RandomState.seed(int) = init_genrand,
 * randint(lo, hi) = masked rejection on one u32 when hi-1-lo < 2^32,
 * random_sample = 53-bit double from two u32, choice(p) = cumsum/searchsorted.
 * Callers: InflexionGame.py:120-121 (random_symmetry), MCTS.py:53 (temp-0 tie
 * break), Coach.py:81 (action sampling). */
void orc_rng_seed(orc_rng* r, uint32_t seed) {
    r->mt[0] = seed;
    for (int i = 1; i < 624; ++i)
        r->mt[i] = 1812433253u * (r->mt[i - 1] ^ (r->mt[i - 1] >> 30)) + (uint32_t)i;
    r->pos = 624;
}

static void rng_twist(orc_rng* r) {
    uint32_t* mt = r->mt;
    for (int i = 0; i < 624; ++i) {
        uint32_t y = (mt[i] & 0x80000000u) | (mt[(i + 1) % 624] & 0x7fffffffu);
        mt[i] = mt[(i + 397) % 624] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
    }
    r->pos = 0;
}

uint32_t orc_rng_u32(orc_rng* r) {
    if (r->pos >= 624) rng_twist(r);
    uint32_t y = r->mt[r->pos++];
    y ^= y >> 11;
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= y >> 18;
    return y;
}

int64_t orc_rng_randint(orc_rng* r, int64_t lo, int64_t hi) {
    uint32_t rng = (uint32_t)(hi - 1 - lo);
    if (rng == 0) return lo; /* no draw */
    uint32_t mask = rng;
    mask |= mask >> 1; mask |= mask >> 2; mask |= mask >> 4;
    mask |= mask >> 8; mask |= mask >> 16;
    for (;;) {
        uint32_t v = orc_rng_u32(r) & mask;
        if (v <= rng) return lo + (int64_t)v;
    }
}

double orc_rng_random_sample(orc_rng* r) {
    uint32_t a = orc_rng_u32(r) >> 5, b = orc_rng_u32(r) >> 6;
    return ((double)a * 67108864.0 + (double)b) / 9007199254740992.0;
}

int orc_rng_choice_p(orc_rng* r, const double* p, int n) {
    double cdf[ORC_MAXA];
    double acc = 0.0;
    for (int i = 0; i < n; ++i) { acc += p[i]; cdf[i] = acc; } /* sequential cumsum */
    double last = cdf[n - 1];
    for (int i = 0; i < n; ++i) cdf[i] /= last;
    double u = orc_rng_random_sample(r);
    for (int i = 0; i < n; ++i) /* searchsorted(side='right') on a monotone cdf */
        if (cdf[i] > u) return i;
    return n;
}

/* -------------------------------------------------------------- pairwise sum
 * numpy umath loops_utils pairwise sum for float32 add.reduce (MCTS.py:96,107). */
static float pw_rec(const float* a, int n) {
    if (n < 8) {
        float res = 0.0f;
        for (int i = 0; i < n; ++i) res += a[i];
        return res;
    }
    if (n <= 128) {
        float r[8];
        for (int j = 0; j < 8; ++j) r[j] = a[j];
        int i;
        for (i = 8; i < n - (n % 8); i += 8)
            for (int j = 0; j < 8; ++j) r[j] += a[i + j];
        float res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
        for (; i < n; ++i) res += a[i];
        return res;
    }
    int n2 = n / 2;
    n2 -= n2 % 8;
    return pw_rec(a, n2) + pw_rec(a + n2, n - n2);
}

float orc_pairwise_sum_f32(const float* a, int n) { return 0.0f + pw_rec(a, n); }

/* ---------------------------------------------------------------------- rules
 * InflexionGame.py: Move directions :15-20, valid_actions_mask :93-100,
 * to_planes :84-91, execute_move :273-310, power_diff :312-317; outcome flip
 * on player change Game.py:49-62; values flags.py:32-36. */
static const int DIRS[6][2] = {{1, 0}, {-1, 0}, {0, 1}, {0, -1}, {1, -1}, {-1, 1}};
#define MAX_POWER_AT_SPAWN 48

double orc_outcome_value(int o) {
    switch (o) {
        case ORC_DRAW: return 1e-4;
        case ORC_WON: return 1.0;
        case ORC_LOST: return -1.0;
        default: return 0.0;
    }
}

static int flip_outcome(int o) { return o == ORC_WON ? ORC_LOST : o == ORC_LOST ? ORC_WON : o; }

static int total_power(const orc_game* g) {
    int s = 0;
    for (int c = 0; c < g->n * g->n; ++c) s += abs(g->board[c]);
    return s;
}

void orc_game_init(orc_game* g, int n, int max_turns) {
    memset(g, 0, sizeof(*g));
    g->n = n;
    g->max_turns = max_turns;
    g->player = 1;
}

/* ------------------------------------------------------------------- Othello
 * builder-authored rules (azg_amd/othello.py), restated independently. */
static const int ODIR[8][2] = {{-1, -1}, {-1, 0}, {-1, 1}, {0, -1}, {0, 1}, {1, -1}, {1, 0}, {1, 1}};

int orc_actions(const orc_game* g) { return g->kind == ORC_OTHELLO ? g->n * g->n + 1 : 7 * g->n * g->n; }
int orc_channels(const orc_game* g) { return g->kind == ORC_OTHELLO ? 2 : 4; }

void orc_othello_init(orc_game* g, int n) {
    memset(g, 0, sizeof(*g));
    g->n = n;
    g->max_turns = 2 * n * n;
    g->player = 1;
    g->kind = ORC_OTHELLO;
    int h = n / 2;
    g->board[(h - 1) * n + h - 1] = g->board[h * n + h] = -1;
    g->board[(h - 1) * n + h] = g->board[h * n + h - 1] = 1;
}

/* flips of a placement by `me` at (r, q): count, and marks them in flip[] when given */
static int oth_flips(const orc_game* g, int r, int q, int me, uint8_t* flip) {
    int n = g->n, total = 0;
    if (g->board[r * n + q] != 0) return 0;
    for (int d = 0; d < 8; ++d) {
        int rr = r + ODIR[d][0], qq = q + ODIR[d][1], k = 0;
        while (rr >= 0 && rr < n && qq >= 0 && qq < n && g->board[rr * n + qq] == -me) {
            rr += ODIR[d][0];
            qq += ODIR[d][1];
            ++k;
        }
        if (k > 0 && rr >= 0 && rr < n && qq >= 0 && qq < n && g->board[rr * n + qq] == me) {
            total += k;
            if (flip)
                for (int s = 1; s <= k; ++s) flip[(r + s * ODIR[d][0]) * n + q + s * ODIR[d][1]] = 1;
        }
    }
    return total;
}

static int oth_has_move(const orc_game* g, int me) {
    for (int c = 0; c < g->n * g->n; ++c)
        if (oth_flips(g, c / g->n, c % g->n, me, NULL)) return 1;
    return 0;
}

static int oth_valid(const orc_game* g, uint8_t* valid) {
    int nn = g->n * g->n, cnt = 0;
    for (int c = 0; c < nn; ++c) {
        valid[c] = oth_flips(g, c / g->n, c % g->n, g->player, NULL) > 0;
        cnt += valid[c];
    }
    valid[nn] = cnt == 0;
    return cnt + valid[nn];
}

static int oth_apply(orc_game* g, int action) {
    int n = g->n, nn = n * n, me = g->player;
    if (action < 0 || action > nn) return -1;
    if (action == nn) {
        if (oth_has_move(g, me)) return -2;
    } else {
        uint8_t flip[ORC_MAXC] = {0};
        if (!oth_flips(g, action / n, action % n, me, flip)) return -3;
        g->board[action] = (int8_t)me;
        for (int c = 0; c < nn; ++c)
            if (flip[c]) g->board[c] = (int8_t)me;
    }
    g->turn += 1;
    int outcome = ORC_ONGOING;
    if (!oth_has_move(g, -me) && !oth_has_move(g, me)) {
        int sum = 0;
        for (int c = 0; c < nn; ++c) sum += g->board[c];
        int diff = sum * me;
        outcome = diff > 0 ? ORC_WON : diff < 0 ? ORC_LOST : ORC_DRAW;
    }
    g->player = -me;
    g->outcome = outcome == ORC_WON ? ORC_LOST : outcome == ORC_LOST ? ORC_WON : outcome;
    return 0;
}

void orc_dihedral_gather(int n, int k, int* src) {
    for (int r = 0; r < n; ++r)
        for (int q = 0; q < n; ++q) {
            int i = r, j = (k & 4) ? n - 1 - q : q; /* fliplr after the rotations */
            int sr, sq;
            switch (k & 3) {
                case 0: sr = i; sq = j; break;
                case 1: sr = j; sq = n - 1 - i; break;
                case 2: sr = n - 1 - i; sq = n - 1 - j; break;
                default: sr = n - 1 - j; sq = i; break;
            }
            src[r * n + q] = sr * n + sq;
        }
}

int orc_valid_mask(const orc_game* g, uint8_t* valid) {
    if (g->kind == ORC_OTHELLO) return oth_valid(g, valid);
    int nn = g->n * g->n, cnt = 0;
    int can_spawn = total_power(g) <= MAX_POWER_AT_SPAWN;
    for (int m = 0; m < 7; ++m)
        for (int c = 0; c < nn; ++c) {
            int v = (m < 6) ? (g->board[c] * g->player > 0) : (can_spawn && g->board[c] == 0);
            valid[m * nn + c] = (uint8_t)v;
            cnt += v;
        }
    return cnt;
}

int orc_apply(orc_game* g, int action) {
    if (g->kind == ORC_OTHELLO) return oth_apply(g, action);
    int n = g->n, nn = n * n;
    if (action < 0 || action >= 7 * nn) return -1;
    int m = action / nn, c = action % nn, r = c / n, q = c % n;
    int spread = m < 6;
    if (!spread) {
        if (total_power(g) > MAX_POWER_AT_SPAWN || g->board[c] != 0) return -2;
        g->board[c] = (int8_t)g->player;
    } else {
        if (g->board[c] * g->player <= 0) return -3;
        int power = abs(g->board[c]);
        for (int k = 1; k <= power; ++k) {
            int rr = ((r + k * DIRS[m][0]) % n + n) % n;
            int qq = ((q + k * DIRS[m][1]) % n + n) % n;
            int x = abs(g->board[rr * n + qq]) + 1;
            g->board[rr * n + qq] = (int8_t)((x > 6 ? 0 : x) * g->player);
        }
        g->board[c] = 0;
    }
    int outcome = ORC_ONGOING;
    int opp_pieces = 0, sum = 0, any = 0;
    for (int i = 0; i < nn; ++i) {
        opp_pieces += g->board[i] * g->player < 0;
        sum += g->board[i];
        any |= g->board[i] != 0;
    }
    if (spread && opp_pieces == 0) {
        outcome = ORC_WON;
    } else if (g->turn >= g->max_turns) {
        int diff = g->player * sum;
        outcome = diff >= 2 ? ORC_WON : diff <= -2 ? ORC_LOST : ORC_DRAW;
    } else if (!any) {
        outcome = ORC_DRAW;
    }
    g->turn += 1;
    g->player = -g->player;
    g->outcome = flip_outcome(outcome);
    return 0;
}

void orc_planes(const orc_game* g, int32_t* planes) {
    int nn = g->n * g->n;
    int can_spawn = total_power(g) <= MAX_POWER_AT_SPAWN;
    for (int c = 0; c < nn; ++c) {
        planes[c] = g->board[c] * g->player > 0;
        planes[nn + c] = g->board[c] * g->player < 0;
        if (g->kind == ORC_OTHELLO) continue; /* othello.py to_planes: [own, opp] */
        planes[2 * nn + c] = g->turn;
        planes[3 * nn + c] = can_spawn;
    }
}

/* rotate (InflexionGame.py:124-168) then translate (:170-196): out[c] = in[src[c]].
 * axis 0 'r', 1 'q', 2 's' (order of np.random.choice(['r','q','s'])). */
void orc_sym_gather(int n, int k, int shift, int axis, int* src) {
    for (int r = 0; r < n; ++r)
        for (int q = 0; q < n; ++q) {
            int tr = r, tq = q; /* translate: position read from the rotated board */
            if (axis == 0) tr = r - shift;
            else if (axis == 1) tq = q - shift;
            else { tr = r + shift; tq = q - shift; }
            tr = ((tr % n) + n) % n;
            tq = ((tq % n) + n) % n;
            int s = (tr + tq) % n, rr, qq;
            switch (k % 6) {
                case 0: rr = tr; qq = tq; break;
                case 1: rr = -s; qq = tr; break;
                case 2: rr = -tq; qq = s; break;
                case 3: rr = -tr; qq = -tq; break;
                case 4: rr = s; qq = -tr; break;
                default: rr = tq; qq = -s; break;
            }
            rr = ((rr % n) + n) % n;
            qq = ((qq % n) + n) % n;
            src[r * n + q] = rr * n + qq;
        }
}

/* ------------------------------------------------------------- stub evaluator */
static uint64_t mix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

void orc_stub_eval(const int32_t* planes, int n, float* P, float* v) {
    orc_stub_eval_c(planes, 4, n, 7 * n * n, P, v);
}

void orc_stub_eval_c(const int32_t* planes, int channels, int n, int A, float* P, float* v) {
    int nn = n * n;
    uint64_t own = 0, opp = 0;
    for (int c = 0; c < nn; ++c) {
        if (planes[c]) own |= 1ull << c;
        if (planes[nn + c]) opp |= 1ull << c;
    }
    uint64_t t = channels > 2 ? (uint64_t)(int64_t)planes[2 * nn] : 0;
    uint64_t k = channels > 3 ? (uint64_t)(int64_t)planes[3 * nn] : 0;
    uint64_t h = mix64(own ^ mix64(opp ^ mix64((t << 1) | k)));
    int all_zero = (h >> 56) < 4;
    for (int a = 0; a < A; ++a) {
        uint64_t ha = mix64(h ^ ((uint64_t)(a + 1) * 0xD1B54A32D192ED03ull));
        float p = (float)(uint32_t)(ha & 0xFFFFFFu) * 0x1p-24f;
        P[a] = (all_zero || (ha >> 59) == 0) ? 0.0f : p;
    }
    *v = (float)((int)((h >> 20) & 2047) - 1024) / 1024.0f;
}

/* ----------------------------------------------------------------------- MCTS
 * MCTS.py: dict tables Qsa/Nsa/Ns/Ps/Vs (:25-31) restated as a node table keyed
 * by the state key to_planes().tobytes() == (own, opp, turn, can_spawn). */
typedef struct {
    uint64_t own, opp;
    int32_t turn, can_spawn;
    int32_t Ns;
    float* P;       /* [A] */
    int32_t* N;     /* [A] */
    double* Q;      /* [A] exact value */
    uint8_t* qf32;  /* [A] 1: Q is a numpy f32 array, 0: Python number */
} orc_node;

typedef struct {
    int n, A, max_turns, sims, temp_threshold;
    float cpuct_f;
    orc_node* nodes;
    int n_nodes, cap_nodes;
    int32_t* table;
    int table_cap;
    orc_rng rng;
    orc_eval_fn eval;
    void* user;
    int64_t expansions, terminal_hits, fallbacks, max_depth;
} orc_mcts;

static uint64_t key_hash(uint64_t own, uint64_t opp, int turn, int cs) {
    return mix64(own ^ mix64(opp ^ (((uint64_t)turn << 1) | (uint64_t)cs)));
}

/* The key is the information in to_planes().tobytes() (MCTS.py:83): Inflexion
 * (own, opp, turn, can_spawn); Othello (own, opp), with the disc count -- a
 * function of the planes -- in the turn slot so that nodes can be aged. */
static void state_key(const orc_game* g, uint64_t* own, uint64_t* opp, int* cs, int* kt) {
    uint64_t o = 0, p = 0;
    for (int c = 0; c < g->n * g->n; ++c) {
        if (g->board[c] * g->player > 0) o |= 1ull << c;
        if (g->board[c] * g->player < 0) p |= 1ull << c;
    }
    *own = o;
    *opp = p;
    if (g->kind == ORC_OTHELLO) {
        *cs = 0;
        *kt = __builtin_popcountll(o | p);
    } else {
        *cs = total_power(g) <= MAX_POWER_AT_SPAWN;
        *kt = g->turn;
    }
}

static int table_find(orc_mcts* m, uint64_t own, uint64_t opp, int turn, int cs, int* slot) {
    uint32_t mask = (uint32_t)m->table_cap - 1;
    uint32_t i = (uint32_t)key_hash(own, opp, turn, cs) & mask;
    for (;;) {
        int32_t id = m->table[i];
        if (id < 0) { *slot = (int)i; return -1; }
        orc_node* nd = &m->nodes[id];
        if (nd->own == own && nd->opp == opp && nd->turn == turn && nd->can_spawn == cs) return id;
        i = (i + 1) & mask;
    }
}

static void table_grow(orc_mcts* m) {
    int cap = m->table_cap * 2;
    int32_t* t = (int32_t*)malloc(sizeof(int32_t) * (size_t)cap);
    for (int i = 0; i < cap; ++i) t[i] = -1;
    free(m->table);
    m->table = t;
    m->table_cap = cap;
    for (int id = 0; id < m->n_nodes; ++id) {
        orc_node* nd = &m->nodes[id];
        int slot;
        table_find(m, nd->own, nd->opp, nd->turn, nd->can_spawn, &slot);
        m->table[slot] = id;
    }
}

typedef struct { double v; int f32; } pyval; /* value returned by search() */

/* MCTS.py:89-112 */
static pyval expand(orc_mcts* m, const orc_game* g, uint64_t own, uint64_t opp, int cs, int kt, int slot) {
    int n = g->n, nn = n * n, A = m->A, C = orc_channels(g);
    int32_t planes[4 * ORC_MAXC], sym[4 * ORC_MAXC];
    int src[ORC_MAXC];
    orc_planes(g, planes);
    if (g->kind == ORC_OTHELLO) { /* othello.py random_symmetry: one randint(0, 8) */
        orc_dihedral_gather(n, (int)orc_rng_randint(&m->rng, 0, 8), src);
    } else {
        int k = (int)orc_rng_randint(&m->rng, 0, 6);
        int shift = (int)orc_rng_randint(&m->rng, 0, n);
        int axis = (int)orc_rng_randint(&m->rng, 0, 3);
        orc_sym_gather(n, k, shift, axis, src);
    }
    for (int ch = 0; ch < C; ++ch)
        for (int c = 0; c < nn; ++c) sym[ch * nn + c] = planes[ch * nn + src[c]];

    float P[ORC_MAXA], v;
    if (m->eval) {
        float fp[4 * ORC_MAXC];
        for (int i = 0; i < C * nn; ++i) fp[i] = (float)sym[i];
        m->eval(fp, P, &v, m->user);
    } else {
        orc_stub_eval_c(sym, C, n, A, P, &v);
    }
    uint8_t valid[ORC_MAXA];
    orc_valid_mask(g, valid);
    for (int a = 0; a < A; ++a) P[a] = valid[a] ? P[a] : P[a] * 0.0f;
    float s = orc_pairwise_sum_f32(P, A);
    if (s > 0.0f) {
        for (int a = 0; a < A; ++a) P[a] = P[a] / s;
    } else {
        m->fallbacks++;
        for (int a = 0; a < A; ++a) P[a] = (float)((double)P[a] + (double)valid[a]);
        float s2 = orc_pairwise_sum_f32(P, A);
        for (int a = 0; a < A; ++a) P[a] = P[a] / s2;
    }
    if (m->n_nodes == m->cap_nodes) {
        m->cap_nodes = m->cap_nodes ? m->cap_nodes * 2 : 1024;
        m->nodes = (orc_node*)realloc(m->nodes, sizeof(orc_node) * (size_t)m->cap_nodes);
    }
    int id = m->n_nodes++;
    orc_node* nd = &m->nodes[id];
    nd->own = own; nd->opp = opp; nd->turn = kt; nd->can_spawn = cs; nd->Ns = 0;
    nd->P = (float*)malloc(sizeof(float) * (size_t)A);
    nd->N = (int32_t*)calloc((size_t)A, sizeof(int32_t));
    nd->Q = (double*)calloc((size_t)A, sizeof(double));
    nd->qf32 = (uint8_t*)calloc((size_t)A, 1);
    memcpy(nd->P, P, sizeof(float) * (size_t)A);
    m->table[slot] = id;
    if (2 * m->n_nodes > m->table_cap) table_grow(m);
    m->expansions++;
    pyval r = {(double)(-v), 1};
    return r;
}

/* MCTS.py:62-145 (recursion made explicit; a path never revisits a node
 * because the key contains the turn). */
static pyval search(orc_mcts* m, const orc_game* root) {
    orc_game g = *root;
    int path_node[1024], path_act[1024], depth = 0;
    pyval ret;
    for (;;) {
        if (g.outcome != ORC_ONGOING) { /* MCTS.py:85-87 */
            ret.v = -orc_outcome_value(g.outcome);
            ret.f32 = 0;
            m->terminal_hits++;
            break;
        }
        uint64_t own, opp;
        int cs, kt, slot;
        state_key(&g, &own, &opp, &cs, &kt);
        int id = table_find(m, own, opp, kt, cs, &slot);
        if (id < 0) {
            ret = expand(m, &g, own, opp, cs, kt, slot);
            break;
        }
        /* select: MCTS.py:114-131 */
        orc_node* nd = &m->nodes[id];
        uint8_t valid[ORC_MAXA];
        orc_valid_mask(&g, valid);
        float sq_edge = (float)sqrt((double)nd->Ns);
        float sq_new = (float)sqrt((double)nd->Ns + 1e-8);
        float best = -INFINITY;
        int best_a = -1;
        for (int a = 0; a < m->A; ++a) {
            if (!valid[a]) continue;
            float cp = m->cpuct_f * nd->P[a];
            float u;
            if (nd->N[a] > 0) {
                float t = (cp * sq_edge) / (float)(1 + nd->N[a]);
                u = (float)nd->Q[a] + t;
            } else {
                u = cp * sq_new;
            }
            if (u > best) { best = u; best_a = a; }
        }
        if (best_a < 0) abort(); /* reference: best_act = -1 crashes (SURVEY hard part 7) */
        if (depth >= 1024) abort();
        path_node[depth] = id;
        path_act[depth] = best_a;
        depth++;
        orc_apply(&g, best_a);
    }
    if (depth > m->max_depth) m->max_depth = depth;
    /* backup MCTS.py:136-145, deepest edge first */
    for (int d = depth - 1; d >= 0; --d) {
        orc_node* nd = &m->nodes[path_node[d]];
        int a = path_act[d];
        int N = nd->N[a];
        if (N == 0) {
            nd->Q[a] = ret.v;
            nd->qf32[a] = (uint8_t)ret.f32;
        } else if (nd->qf32[a] || ret.f32) {
            float prod = nd->qf32[a] ? (float)N * (float)nd->Q[a] : (float)((double)N * nd->Q[a]);
            float num = prod + (float)ret.v;
            nd->Q[a] = (double)(num / (float)(N + 1));
            nd->qf32[a] = 1;
        } else {
            nd->Q[a] = ((double)N * nd->Q[a] + ret.v) / (double)(N + 1);
        }
        nd->N[a] = N + 1;
        nd->Ns += 1;
        ret.v = -ret.v;
    }
    return ret;
}

static void mcts_free(orc_mcts* m) {
    for (int i = 0; i < m->n_nodes; ++i) {
        free(m->nodes[i].P); free(m->nodes[i].N); free(m->nodes[i].Q); free(m->nodes[i].qf32);
    }
    free(m->nodes);
    free(m->table);
}

/* Coach.executeEpisode (Coach.py:41-90) + MCTS.getActionProb (MCTS.py:33-60) */
int orc_episode(int n, int max_turns, int sims, double cpuct, int temp_threshold,
                uint32_t seed, orc_eval_fn eval, void* user,
                int32_t* actions, int32_t* counts, int8_t* temps, int max_moves,
                int64_t* stats) {
    return orc_episode_kind(ORC_INFLEXION, n, max_turns, sims, cpuct, temp_threshold, seed, eval, user,
                            actions, counts, temps, max_moves, stats);
}

int orc_episode_kind(int kind, int n, int max_turns, int sims, double cpuct, int temp_threshold,
                     uint32_t seed, orc_eval_fn eval, void* user,
                     int32_t* actions, int32_t* counts, int8_t* temps, int max_moves,
                     int64_t* stats) {
    orc_game g;
    if (kind == ORC_OTHELLO) {
        orc_othello_init(&g, n);
    } else {
        orc_game_init(&g, n, max_turns);
        g.kind = ORC_INFLEXION;
    }
    orc_mcts m;
    memset(&m, 0, sizeof(m));
    m.n = n; m.A = orc_actions(&g); m.max_turns = max_turns; m.sims = sims;
    m.temp_threshold = temp_threshold;
    m.cpuct_f = (float)cpuct;
    m.eval = eval; m.user = user;
    m.table_cap = 4096;
    m.table = (int32_t*)malloc(sizeof(int32_t) * (size_t)m.table_cap);
    for (int i = 0; i < m.table_cap; ++i) m.table[i] = -1;
    orc_rng_seed(&m.rng, seed);

    int moves = 0;
    int32_t cnt[ORC_MAXA];
    double pi[ORC_MAXA];
    while (1) {
        int step = moves + 1;
        int temp = step < temp_threshold;
        for (int i = 0; i < sims; ++i) search(&m, &g);
        uint64_t own, opp;
        int cs, slot;
        int kt;
        state_key(&g, &own, &opp, &cs, &kt);
        int id = table_find(&m, own, opp, kt, cs, &slot);
        for (int a = 0; a < m.A; ++a) cnt[a] = id >= 0 ? m.nodes[id].N[a] : 0;
        if (temp == 0) { /* MCTS.py:51-56 */
            int mx = cnt[0], nb = 0, best[ORC_MAXA];
            for (int a = 1; a < m.A; ++a) if (cnt[a] > mx) mx = cnt[a];
            for (int a = 0; a < m.A; ++a) if (cnt[a] == mx) best[nb++] = a;
            int b = best[orc_rng_randint(&m.rng, 0, nb)];
            for (int a = 0; a < m.A; ++a) pi[a] = a == b;
        } else { /* MCTS.py:58-60, temp == 1 */
            double tot = 0.0;
            for (int a = 0; a < m.A; ++a) tot += (double)cnt[a];
            for (int a = 0; a < m.A; ++a) pi[a] = (double)cnt[a] / tot;
        }
        int action = orc_rng_choice_p(&m.rng, pi, m.A);
        if (moves < max_moves) {
            if (actions) actions[moves] = action;
            if (counts) memcpy(counts + (size_t)moves * m.A, cnt, sizeof(int32_t) * (size_t)m.A);
            if (temps) temps[moves] = (int8_t)temp;
        }
        moves++;
        if (orc_apply(&g, action) != 0) abort();
        if (g.outcome != ORC_ONGOING) break;
        if (moves >= max_moves) break; /* bounded sample (cpu_baseline) */
    }
    if (stats) {
        stats[0] = moves; stats[1] = m.expansions; stats[2] = m.n_nodes;
        stats[3] = g.outcome; stats[4] = g.player; stats[5] = m.rng.pos;
        for (int i = 0; i < 4; ++i) stats[6 + i] = orc_rng_u32(&m.rng);
        stats[10] = m.terminal_hits; stats[11] = m.max_depth; stats[12] = m.fallbacks;
    }
    mcts_free(&m);
    return moves;
}
