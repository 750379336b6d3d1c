// azg_kernels.hip -- CDNA4 (gfx950) kernels of the batched self-play engine.
//
// Launch geometry: one 64-thread workgroup (= one wavefront) per game slot.
// The tree work per simulation is latency-bound pointer chasing over a handful
// of node rows, so the design goal is: every HBM access is a
// coalesced wave-wide row read, every reduction is an in-register __shfl_xor
// butterfly or a __ballot, no atomics on the tree (the slot is owned by its
// wave), and no host synchronisation between kernels (a whole move can be
// captured in a hipGraph).
//
// The search kernels are templates over a game's rules (struct Inflexion,
// struct Othello<N>): key, valid-action context, move application and the
// randomly symmetrised NN planes are wave-collective device functions with
// one lane per board cell.
//
// Numerics restate the reference bit-exactly (oracle/oracle.c is the CPU
// checker): f32 ops are single-rounded (-ffp-contract=off
// for this file), math.sqrt is a correctly rounded f64 sqrt, Q values that the
// reference holds as Python numbers are kept in f64 with a type bit.
#include <hip/hip_runtime.h>
#include <math.h>

#include "azg_engine.h"
#include "azg_launch.h"

namespace azg {

// ---------------------------------------------------------------- wave utils
__device__ __forceinline__ int lane_id() { return threadIdx.x; }

__device__ __forceinline__ int wave_sum(int x) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) x += __shfl_xor(x, o);
    return x;
}

__device__ __forceinline__ int wave_max(int x) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) x = max(x, __shfl_xor(x, o));
    return x;
}

__device__ __forceinline__ uint64_t mix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

__device__ __forceinline__ uint64_t key_hash(uint64_t own, uint64_t opp, int turn, int cs) {
    return mix64(own ^ mix64(opp ^ (((uint64_t)(uint32_t)turn << 1) | (uint64_t)cs)));
}

__device__ __forceinline__ double outcome_value(int o) {
    return o == DRAW ? 1e-4 : o == WON ? 1.0 : o == LOST ? -1.0 : 0.0;  // flags.py:32-36
}

__device__ __forceinline__ int flip_outcome(int o) {  // GameOutcome.opposite, Game.py:49-62
    return o == WON ? LOST : o == LOST ? WON : o;
}

// ------------------------------------------------------------------- MT19937
// numpy RandomState (legacy) stream of one game.  A kernel draws a handful of
// words, so the 64 words from the current position are prefetched into one
// register per lane (one coalesced 256-B load, issued as early as the kernel
// knows the slot) and served by __shfl; only a draw past them or past the end
// of the state (the twist) stages the whole 2.5 KB state in LDS.
struct BlockRng {
    uint32_t* g;   // global [624]
    int32_t* gpos;
    uint32_t* s;   // LDS [624]
    int pos;
    bool loaded, dirty;
    int pre_base;  // position of lane 0's prefetched word (-1: none)
    uint32_t pre;  // this lane's prefetched word g[pre_base + lane]
};

__device__ __forceinline__ BlockRng rng_open(uint32_t* g, int32_t* gpos, uint32_t* s) {
    BlockRng r{g, gpos, s, *gpos, false, false, -1, 0u};
    const int i = r.pos + (int)threadIdx.x;
    if (r.pos < MT_N) {
        r.pre_base = r.pos;
        r.pre = i < MT_N ? g[i] : 0u;
    }
    return r;
}

__device__ __forceinline__ uint32_t mt_temper(uint32_t y) {
    y ^= y >> 11;
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= y >> 18;
    return y;
}

__device__ __forceinline__ uint32_t mt_mix(uint32_t cur, uint32_t nxt, uint32_t far) {
    uint32_t y = (cur & 0x80000000u) | (nxt & 0x7fffffffu);
    return far ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
}

// In-place sequential twist restated as three wave-parallel phases:
// i < 227 reads only old words; 227 <= i < 623 reads new[i-227]; i = 623 last.
__device__ void mt_twist(uint32_t* s) {
    const int lane = lane_id();
    for (int b = 0; b < 227; b += WAVE) {
        int i = b + lane;
        uint32_t v = 0;
        if (i < 227) v = mt_mix(s[i], s[i + 1], s[i + 397]);
        __syncthreads();
        if (i < 227) s[i] = v;
        __syncthreads();
    }
    for (int b = 227; b < 623; b += WAVE) {
        int i = b + lane;
        uint32_t v = 0;
        if (i < 623) v = mt_mix(s[i], s[i + 1], s[i - 227]);
        __syncthreads();
        if (i < 623) s[i] = v;
        __syncthreads();
    }
    if (lane == 0) s[623] = mt_mix(s[623], s[0], s[396]);
    __syncthreads();
}

__device__ uint32_t rng_u32(BlockRng& R) {
    if (!R.loaded && R.pre_base >= 0 && R.pos < MT_N && R.pos - R.pre_base < WAVE)
        return mt_temper(__shfl(R.pre, R.pos++ - R.pre_base));
    if (!R.loaded) {
        for (int i = lane_id(); i < MT_N; i += WAVE) R.s[i] = R.g[i];
        __syncthreads();
        R.loaded = true;
    }
    if (R.pos >= MT_N) {
        mt_twist(R.s);
        R.pos = 0;
        R.dirty = true;
    }
    return mt_temper(R.s[R.pos++]);
}

__device__ int rng_randint(BlockRng& R, int lo, int hi) {  // legacy masked rejection
    uint32_t rng = (uint32_t)(hi - 1 - lo);
    if (rng == 0) return lo;
    uint32_t mask = rng;
    mask |= mask >> 1; mask |= mask >> 2; mask |= mask >> 4; mask |= mask >> 8; mask |= mask >> 16;
    for (;;) {
        uint32_t v = rng_u32(R) & mask;
        if (v <= rng) return lo + (int)v;
    }
}

__device__ double rng_random_sample(BlockRng& R) {
    uint32_t a = rng_u32(R) >> 5, b = rng_u32(R) >> 6;
    return ((double)a * 67108864.0 + (double)b) / 9007199254740992.0;
}

__device__ void rng_store(BlockRng& R) {
    if (R.dirty)
        for (int i = lane_id(); i < MT_N; i += WAVE) R.g[i] = R.s[i];
    if (lane_id() == 0) *R.gpos = R.pos;
}

// ------------------------------------------------------------ numpy pairwise
struct PW {
    int nleaf = 0, nops = 0;
    int off[16] = {}, len[16] = {}, ops[32] = {};
};
constexpr void pw_build(PW& p, int off, int n) {
    if (n <= 128) {
        p.ops[p.nops++] = p.nleaf;
        p.off[p.nleaf] = off;
        p.len[p.nleaf] = n;
        p.nleaf++;
        return;
    }
    int n2 = n / 2;
    n2 -= n2 % 8;
    pw_build(p, off, n2);
    pw_build(p, off + n2, n - n2);
    p.ops[p.nops++] = -1;
}
constexpr PW make_pw(int n) {
    PW p{};
    pw_build(p, 0, n);
    return p;
}

// float32 add.reduce over NA values in numpy's exact association (MCTS.py:96,
// :107).  x: LDS [NA]; acc: LDS [64]; leaf: LDS [16].  Sum in every lane.
template <int NA>
__device__ float pairwise_sum(const float* x, float* acc, float* leaf) {
    constexpr PW kPW = make_pw(NA);
    static_assert(kPW.nleaf <= 8, "one pass of 8 lanes per leaf");
    const int lane = lane_id();
    const int l = lane >> 3, j = lane & 7;
#pragma unroll
    for (int q = 0; q < kPW.nleaf; ++q) {
        if (l == q && kPW.len[q] >= 8) {
            const int off = kPW.off[q], full = kPW.len[q] - kPW.len[q] % 8;
            float r = x[off + j];
            for (int i = 8; i < full; i += 8) r = r + x[off + i + j];
            acc[lane] = r;
        }
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < kPW.nleaf; ++q) {
        if (lane == q) {
            const int off = kPW.off[q], len = kPW.len[q];
            float res;
            int i;
            if (len < 8) {
                res = 0.0f;
                i = 0;
            } else {
                const float* r = acc + q * 8;
                res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
                i = len - len % 8;
            }
            for (; i < len; ++i) res = res + x[off + i];
            leaf[q] = res;
        }
    }
    __syncthreads();
    float st[8];
    int sp = 0;
#pragma unroll
    for (int k = 0; k < kPW.nops; ++k) {
        if (kPW.ops[k] >= 0) {
            st[sp++] = leaf[kPW.ops[k]];
        } else {
            float b = st[--sp];
            float a = st[--sp];
            st[sp++] = a + b;
        }
    }
    __syncthreads();
    return 0.0f + st[0];
}

// ------------------------------------------------------------------- games
// One lane per cell (lanes 0..CELLS-1).  Pos: this lane's cell value, and the
// wave-uniform turn, player to move (+1 RED / -1 BLUE), outcome w.r.t. it.
struct Pos {
    int cell, turn, player, outcome;
};

// --- InflexionGame(7) (InflexionGame.py) ---------------------------------
struct Inflexion {
    static constexpr int N = 7, CELLS = 49, A = 7 * CELLS, AP = 384, AJ = AP / WAVE, PLANES = 4;
    static constexpr uint64_t FULL = (1ull << CELLS) - 1ull;
    static __device__ __forceinline__ int mod_n(int x) { return ((x % N) + N) % N; }

    __device__ static int initial_cell(int) { return 0; }

    // key = to_planes() information (InflexionGame.py:84-91): own, opp, turn, can_spawn
    __device__ static void key(const Pos& p, uint64_t& own, uint64_t& opp, int& kt, int& cs) {
        const bool on = lane_id() < CELLS;
        own = __ballot(on && p.cell * p.player > 0);
        opp = __ballot(on && p.cell * p.player < 0);
        cs = wave_sum(on ? abs(p.cell) : 0) <= MAX_POWER_AT_SPAWN;
        kt = p.turn;
    }

    // valid_actions_mask (InflexionGame.py:93-100) from the key
    struct VCtx {
        uint64_t own, spawn;
    };
    __device__ static VCtx vctx(uint64_t own, uint64_t opp, int cs) { return {own, cs ? (~(own | opp) & FULL) : 0ull}; }
    __device__ static bool valid(int a, const VCtx& v) {
        const int m = a / CELLS, c = a - m * CELLS;
        return m < 6 ? ((v.own >> c) & 1ull) : ((v.spawn >> c) & 1ull);
    }

    // execute_move (:273-310) + player setter (Game.py:49-62)
    __device__ static void apply(Pos& p, int a, int max_turns) {
        const int lane = lane_id();
        const int m = a / CELLS, c = a - m * CELLS, r = c / N, q = c - (c / N) * N;
        const int orig = __shfl(p.cell, c);
        const bool spread = m < 6;
        if (!spread) {
            if (lane == c) p.cell = p.player;
        } else if (lane < CELLS) {
            const int dr = (m == 0 || m == 4) ? 1 : (m == 1 || m == 5) ? -1 : 0;
            const int dq = (m == 2 || m == 5) ? 1 : (m == 3 || m == 4) ? -1 : 0;
            const int power = abs(orig);
            const int lr = lane / N, lq = lane - (lane / N) * N;
            const int k = dr != 0 ? mod_n((lr - r) * dr) : mod_n((lq - q) * dq);
            const bool hit = k >= 1 && k <= power && mod_n(r + k * dr) == lr && mod_n(q + k * dq) == lq;
            if (hit) {
                int x = abs(p.cell) + 1;
                p.cell = (x > 6 ? 0 : x) * p.player;
            }
            if (lane == c) p.cell = 0;
        }
        const bool on = lane < CELLS;
        const uint64_t oppb = __ballot(on && p.cell * p.player < 0);
        const int sum = wave_sum(on ? p.cell : 0);
        const uint64_t anyb = __ballot(on && p.cell != 0);
        int out = ONGOING;
        if (spread && oppb == 0) {
            out = WON;
        } else if (p.turn >= max_turns) {
            const int diff = p.player * sum;
            out = diff >= 2 ? WON : diff <= -2 ? LOST : DRAW;
        } else if (anyb == 0) {
            out = DRAW;
        }
        p.turn += 1;
        p.player = -p.player;
        p.outcome = flip_outcome(out);
    }

    // rotate(k) then translate(shift, axis): source cell of output cell c
    __device__ static int sym_src(int c, int k, int shift, int axis) {
        int r = c / N, q = c - (c / N) * N;
        int tr = r, tq = q;
        if (axis == 0) tr = r - shift;
        else if (axis == 1) tq = q - shift;
        else { tr = r + shift; tq = q - shift; }
        tr = mod_n(tr);
        tq = mod_n(tq);
        const int s = (tr + tq) % N;
        int rr, qq;
        switch (k) {
            case 0: rr = tr; qq = tq; break;
            case 1: rr = -s; qq = tr; break;
            case 2: rr = -tq; qq = s; break;
            case 3: rr = -tr; qq = -tq; break;
            case 4: rr = s; qq = -tr; break;
            default: rr = tq; qq = -s; break;
        }
        return mod_n(rr) * N + mod_n(qq);
    }

    // random_symmetry (InflexionGame.py:115-122): randint(0,6), randint(0,n), choice(r,q,s)
    __device__ static void write_planes(float* out, uint64_t own, uint64_t opp, int kt, int cs, BlockRng& R) {
        const int k = rng_randint(R, 0, 6);
        const int shift = rng_randint(R, 0, N);
        const int axis = rng_randint(R, 0, 3);
        const int lane = lane_id();
        if (lane < CELLS) {
            const int src = sym_src(lane, k, shift, axis);
            out[lane] = (float)((own >> src) & 1ull);
            out[CELLS + lane] = (float)((opp >> src) & 1ull);
            out[2 * CELLS + lane] = (float)kt;
            out[3 * CELLS + lane] = (float)cs;
        }
    }

    // symmetries() (InflexionGame.py:102-113), form s: identity, rotate(s) for
    // s = 1..5, then translate(rotate(k), j, 'r') for k = 1..5, j = 1..n-1
    static constexpr int NSYM = 6 + 5 * (N - 1);
    static constexpr int SYM_ACTIONS = A;  // every action is a (move kind, cell)
    __device__ static int form_src(int s, int c) {
        if (s < 6) return sym_src(c, s, 0, 0);
        return sym_src(c, 1 + (s - 6) / (N - 1), 1 + (s - 6) % (N - 1), 0);
    }
    // the policy plane (7, n, n) moves its cells; the move kinds stay put
    __device__ static int form_action_src(int s, int a) {
        const int m = a / CELLS;
        return m * CELLS + form_src(s, a - m * CELLS);
    }
    // to_planes() value of plane pl at (source) cell src (InflexionGame.py:84-91)
    __device__ static float plane(int pl, int src, uint64_t own, uint64_t opp, int kt, int cs) {
        return pl == 0 ? (float)((own >> src) & 1ull)
                       : pl == 1 ? (float)((opp >> src) & 1ull) : pl == 2 ? (float)kt : (float)cs;
    }
};

// --- OthelloGame(n) (azg_amd/othello.py; builder-authored) ----------------
template <int NB>
struct Othello {
    static constexpr int N = NB, CELLS = NB * NB, A = CELLS + 1, AP = ((A + WAVE - 1) / WAVE) * WAVE,
                         AJ = AP / WAVE, PLANES = 2;
    static constexpr uint64_t FULL = CELLS == 64 ? ~0ull : (1ull << CELLS) - 1ull;

    static constexpr uint64_t col_mask(int q) {
        uint64_t m = 0;
        for (int r = 0; r < N; ++r) m |= 1ull << (r * N + q);
        return m;
    }
    static constexpr uint64_t FIRST = col_mask(0), LAST = col_mask(NB - 1);

    __device__ static int initial_cell(int c) {
        const int h = N / 2, r = c / N, q = c % N;
        if ((r == h - 1 && q == h - 1) || (r == h && q == h)) return -1;
        if ((r == h - 1 && q == h) || (r == h && q == h - 1)) return 1;
        return 0;
    }

    // one step of direction d = (dr, dq) in {-1,0,1}^2 \ (0,0) on a bitboard
    __device__ static __forceinline__ uint64_t step(uint64_t b, int dr, int dq) {
        if (dq == 1) b &= ~LAST;
        if (dq == -1) b &= ~FIRST;
        const int s = dr * N + dq;
        return (s > 0 ? (b << s) : (b >> (-s))) & FULL;
    }

    __device__ static uint64_t legal(uint64_t own, uint64_t opp) {
        const uint64_t empty = ~(own | opp) & FULL;
        uint64_t moves = 0;
#pragma unroll
        for (int d = 0; d < 9; ++d) {
            const int dr = d / 3 - 1, dq = d % 3 - 1;
            if (dr == 0 && dq == 0) continue;
            uint64_t x = step(own, dr, dq) & opp;
#pragma unroll
            for (int i = 0; i < N - 3; ++i) x |= step(x, dr, dq) & opp;
            moves |= step(x, dr, dq) & empty;
        }
        return moves;
    }

    __device__ static uint64_t flips(uint64_t own, uint64_t opp, int c) {
        uint64_t f = 0;
        const uint64_t m = 1ull << c;
#pragma unroll
        for (int d = 0; d < 9; ++d) {
            const int dr = d / 3 - 1, dq = d % 3 - 1;
            if (dr == 0 && dq == 0) continue;
            uint64_t run = 0, x = step(m, dr, dq);
            while (x & opp) {
                run |= x;
                x = step(x, dr, dq);
            }
            if (x & own) f |= run;
        }
        return f;
    }

    // key = to_planes() information: (own, opp); disc count in the turn slot (for node ageing)
    __device__ static void key(const Pos& p, uint64_t& own, uint64_t& opp, int& kt, int& cs) {
        const bool on = lane_id() < CELLS;
        own = __ballot(on && p.cell * p.player > 0);
        opp = __ballot(on && p.cell * p.player < 0);
        kt = __popcll(own | opp);
        cs = 0;
    }

    struct VCtx {
        uint64_t legal;
    };
    __device__ static VCtx vctx(uint64_t own, uint64_t opp, int) { return {legal(own, opp)}; }
    __device__ static bool valid(int a, const VCtx& v) {
        return a < CELLS ? ((v.legal >> a) & 1ull) : (v.legal == 0ull);
    }

    __device__ static void apply(Pos& p, int a, int) {
        const int lane = lane_id();
        const bool on = lane < CELLS;
        const uint64_t own = __ballot(on && p.cell * p.player > 0);
        const uint64_t opp = __ballot(on && p.cell * p.player < 0);
        uint64_t own2 = own, opp2 = opp;
        if (a < CELLS) {
            const uint64_t f = flips(own, opp, a);
            own2 = own | f | (1ull << a);
            opp2 = opp & ~f;
            if (on && ((own2 >> lane) & 1ull)) p.cell = p.player;
        }
        int out = ONGOING;
        if (legal(opp2, own2) == 0 && legal(own2, opp2) == 0) {
            const int diff = __popcll(own2) - __popcll(opp2);
            out = diff > 0 ? WON : diff < 0 ? LOST : DRAW;
        }
        p.turn += 1;
        p.player = -p.player;
        p.outcome = flip_outcome(out);
    }

    // random_symmetry: one randint(0, 8); k&3 rot90s then fliplr if k&4 (othello.py dihedral_source)
    __device__ static void write_planes(float* out, uint64_t own, uint64_t opp, int, int, BlockRng& R) {
        const int k = rng_randint(R, 0, 8);
        const int lane = lane_id();
        if (lane < CELLS) {
            const int src = form_src(k, lane);
            out[lane] = (float)((own >> src) & 1ull);
            out[CELLS + lane] = (float)((opp >> src) & 1ull);
        }
    }

    // symmetries(): the 8 dihedral forms k (k & 3 rot90s, then fliplr if k & 4);
    // source cell of output cell c
    static constexpr int NSYM = 8;
    static constexpr int SYM_ACTIONS = CELLS;  // the pass action is not moved
    __device__ static int form_src(int k, int c) {
        const int i = c / N, j = (k & 4) ? N - 1 - c % N : c % N;
        int sr, sq;
        switch (k & 3) {
            case 0: sr = i; sq = j; break;
            case 1: sr = j; sq = N - 1 - i; break;
            case 2: sr = N - 1 - i; sq = N - 1 - j; break;
            default: sr = N - 1 - j; sq = i; break;
        }
        return sr * N + sq;
    }
    __device__ static int form_action_src(int k, int a) { return a < CELLS ? form_src(k, a) : a; }  // pass stays
    __device__ static float plane(int pl, int src, uint64_t own, uint64_t opp, int, int) {
        return pl == 0 ? (float)((own >> src) & 1ull) : (float)((opp >> src) & 1ull);
    }
};

// ------------------------------------------------------------------- tree
template <class R>
__device__ __forceinline__ size_t node_row(const Dev& E, int g, int id) {
    return ((size_t)g * E.M + id) * R::AP;
}

// Compact edge slots.  A node's row holds its edges (P, N, Q) only for the valid
// actions of its key, packed in action order: the edge of valid action a sits at
// slot ci = #(valid actions < a).  The valid set is a function of the key, which
// every kernel that addresses a row already holds, so the mapping costs a ballot
// and a popcount per 64 actions and no memory; a wave's reads of a row are then
// nv contiguous elements (87 at a mean 7x7 Inflexion node: 3 + 3 + 6 lines of P, N,
// Q) instead of scattered elements of all 12 + 12 + 24 lines of the 384-wide row.
// Edge order equals action order, so first-index tie-breaks are unchanged.
// Lane's action lane + 64 j gets slot ci[j] (-1: not valid); returns nv.
template <class R>
__device__ __forceinline__ int edge_slots(const typename R::VCtx& vc, int (&ci)[R::AJ]) {
    const int lane = lane_id();
    const uint64_t below = (1ull << lane) - 1ull;
    int base = 0;
#pragma unroll
    for (int j = 0; j < R::AJ; ++j) {
        const int a = lane + WAVE * j;
        const bool v = a < R::A && R::valid(a, vc);
        const uint64_t b = __ballot(v);
        ci[j] = v ? base + __popcll(b & below) : -1;
        base += __popcll(b);
    }
    return base;
}

template <class R>
__device__ __forceinline__ Pos load_root(const Dev& E, int g) {
    Pos p;
    const int lane = lane_id();
    p.cell = lane < R::CELLS ? (int)E.board[(size_t)g * 64 + lane] : 0;
    p.turn = E.turn[g];
    p.player = E.player[g];
    p.outcome = E.outcome[g];
    return p;
}

// Wave-cooperative open-addressing lookup: 64 consecutive slots per probe.
// Returns node id or -1 (then *slot = first empty slot in probe order).
__device__ int table_lookup(const Dev& E, int g, uint64_t own, uint64_t opp, int turn, int cs, int* slot);

__device__ int table_lookup(const Dev& E, int g, uint64_t own, uint64_t opp, int turn, int cs, int* slot) {
    const int lane = lane_id();
    const uint64_t h = key_hash(own, opp, turn, cs);
    const uint32_t tag = (uint32_t)(h >> 32);
    const uint64_t* T = E.table + (size_t)g * E.H;
    const uint32_t hm = (uint32_t)E.H - 1;
    const uint32_t base = (uint32_t)h & hm;
    // The first probe covers 16 slots (128 B: the table is at most half full, so a
    // lookup almost always ends there), later ones 64; slots are visited in the same
    // order either way, so the first match-or-empty is the same.
    for (int probe = 0, width = 16; probe < E.H; probe += width, width = WAVE) {
        const bool in = lane < width;
        const uint32_t s = (base + (uint32_t)probe + (uint32_t)lane) & hm;
        const uint64_t e = in ? T[s] : ~0ull;
        const bool empty = e == 0;
        int id = -1;
        bool match = false;
        if (in && !empty && (uint32_t)(e >> 32) == tag) {
            id = (int)(uint32_t)e - 1;
            const size_t ni = (size_t)g * E.M + id;
            const NodeKey& k = E.node_key[ni];
            match = k.own == own && k.opp == opp && k.turn == turn && k.cs == cs;
        }
        const uint64_t stop = __ballot(match || empty);
        if (stop) {
            const int l = __ffsll((unsigned long long)stop) - 1;
            const int found = __shfl(match ? id : -1, l);
            *slot = (int)((base + (uint32_t)probe + (uint32_t)l) & hm);
            return found;
        }
    }
    *slot = -1;
    return -1;
}

// A node's edges as the PUCT scan reads them: the lane's compact slots, P, N and the
// f32 Q per valid action, and the node's visit count.  Loaded together (one round trip),
// and by the descent below the root together with the node's key check.
template <class R>
struct EdgeRow {
    int ci[R::AJ];
    float P[R::AJ], Qf[R::AJ];
    uint32_t N[R::AJ];
    int Ns;
};
template <class R>
__device__ __forceinline__ void load_edges(const Dev& E, int g, int id, const typename R::VCtx& vc, EdgeRow<R>& er) {
    const size_t row = node_row<R>(E, g, id);
    er.Ns = E.node_key[(size_t)g * E.M + id].Ns;
    edge_slots<R>(vc, er.ci);
#pragma unroll
    for (int j = 0; j < R::AJ; ++j) {
        // the f32 Q loaded with P and N (not after N says the edge exists): one
        // dependent round trip less per level; used only where N > 0
        if (er.ci[j] >= 0) {
            er.P[j] = E.node_P[row + er.ci[j]];
            er.N[j] = E.node_N[row + er.ci[j]];
            er.Qf[j] = E.node_Qf[row + er.ci[j]];
        }
    }
}

// The descent's lookup below the root: the first probe's slots, then -- for the first
// slot whose tag matches, if no empty slot comes before it -- the node's key check and its
// edges in ONE round trip (the edges speculatively: a tag match is almost always the node).
// Same result as table_lookup (+ load_edges when found): a key that does not match, or no
// decision in the first probe, falls back to table_lookup.
template <class R>
__device__ int lookup_with_edges(const Dev& E, int g, uint64_t own, uint64_t opp, int turn, int cs, int* slot,
                                 const typename R::VCtx& vc, EdgeRow<R>& er) {
    const int lane = lane_id();
    const uint64_t h = key_hash(own, opp, turn, cs);
    const uint32_t tag = (uint32_t)(h >> 32);
    const uint64_t* T = E.table + (size_t)g * E.H;
    const uint32_t hm = (uint32_t)E.H - 1;
    const uint32_t base = (uint32_t)h & hm;
    constexpr int W = 16;  // table_lookup's first probe
    const bool in = lane < W && lane < E.H;
    const uint64_t e = in ? T[(base + (uint32_t)lane) & hm] : ~0ull;
    const uint64_t empty = __ballot(in && e == 0);
    const uint64_t tagm = __ballot(in && e != 0 && (uint32_t)(e >> 32) == tag);
    const int fe = empty ? __ffsll((unsigned long long)empty) - 1 : 64;
    const int ft = tagm ? __ffsll((unsigned long long)tagm) - 1 : 64;
    if (ft < fe) {  // a candidate before any empty slot
        const int id = __shfl((int)(uint32_t)e - 1, ft);
        const NodeKey k = E.node_key[(size_t)g * E.M + id];
        load_edges<R>(E, g, id, vc, er);  // (speculative: with the key's round trip)
        if (k.own == own && k.opp == opp && k.turn == turn && k.cs == cs) {
            *slot = (int)((base + (uint32_t)ft) & hm);
            return id;
        }
    } else if (fe < 64) {  // empty before any tag match: not in the table
        *slot = (int)((base + (uint32_t)fe) & hm);
        return -1;
    }
    const int id = table_lookup(E, g, own, opp, turn, cs, slot);
    if (id >= 0) load_edges<R>(E, g, id, vc, er);
    return id;
}

// PUCT argmax (MCTS.py:114-131): strict '>' scan in action order == max u,
// ties to the lowest action; NaN never wins.  Returns the action; *edge gets its
// compact edge slot (edge_slots).
template <class R>
__device__ int puct_select(const Dev& E, int g, int id, const EdgeRow<R>& er, int* edge) {
    const int lane = lane_id();
    const size_t row = node_row<R>(E, g, id);
    const int Ns = er.Ns;
    const float sq_edge = (float)sqrt((double)Ns);
    const float sq_new = (float)sqrt((double)Ns + 1e-8);
    const int(&ci)[R::AJ] = er.ci;
    float best = -INFINITY;
    int besta = 0x7fffffff, besti = -1;
#pragma unroll
    for (int j = 0; j < R::AJ; ++j) {
        const int a = lane + WAVE * j;
        if (ci[j] >= 0) {
            const float cp = E.cpuct_f * er.P[j];
            const uint32_t nr = er.N[j];
            // an edge whose Q is still a Python float (only terminal values backed into
            // it) reads its f64 Q after N: rare, near the end of a game
            const float qf = er.Qf[j];
            const int n = (int)(nr & 0x7fffffffu);
            float u;
            if (n > 0) {
                const float q = (nr >> 31) ? qf : (float)E.node_Q[row + ci[j]];
                const float t = (cp * sq_edge) / (float)(1 + n);
                u = q + t;
            } else {
                u = cp * sq_new;
            }
            if (u > best) {
                best = u;
                besta = a;
                besti = ci[j];
            }
        }
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
        const float ou = __shfl_xor(best, o);
        const int oa = __shfl_xor(besta, o);
        const int oi = __shfl_xor(besti, o);
        if (ou > best || (ou == best && oa < besta)) {
            best = ou;
            besta = oa;
            besti = oi;
        }
    }
    *edge = besti;
    return besta == 0x7fffffff ? -1 : besta;
}

// arena slots search only on their own colour's turns (searcher 0 = self-play)
__device__ __forceinline__ bool searching(const Dev& E, int g) {
    return E.searcher[g] == 0 || E.searcher[g] == E.player[g];
}

__device__ __forceinline__ void set_err(const Dev& E, int g, int code) {
    if (lane_id() == 0 && E.err[g] == 0) E.err[g] = code;
}

// --------------------------------------------------------------- kernels
// What a descent reads before its first tree access and no expansion / backup writes
// (slot state, root position, the next random words): loaded together, and in the
// fused expand_select kernel before the expansion, so none of it waits behind the
// backup's round trips (the drop-in's one-game search is a chain of dependent loads).
// The slot's error code and cached root id are loaded here too: in the fused kernel the expansion
// hands over what it changes of them (ExpandOut) instead of the descent re-reading them.
template <class R>
struct SelPre {
    int active, searcher, err, root_id;
    Pos root;
    BlockRng rg;
};
struct ExpandOut {
    int err;      // error code the expansion set (0: none)
    int root_id;  // node id the expansion made the root (-1: none)
};
template <class R>
__device__ __forceinline__ SelPre<R> select_prefetch(const Dev& E) {
    __shared__ uint32_t s_mt[MT_N];
    const int g = blockIdx.x;
    SelPre<R> q;
    q.active = E.active[g];
    q.searcher = E.searcher[g];
    q.err = E.err[g];
    q.root_id = E.root_id[g];
    q.root = load_root<R>(E, g);
    q.rg = rng_open(E.mt + (size_t)g * MT_N, E.mt_pos + g, s_mt);  // the slot's next random words
    return q;
}

// sim_begin: MCTS.search down to a leaf (MCTS.py:83-132), writing the leaf's
// randomly symmetrised planes (MCTS.py:91-92) as f32 into the NN batch.
template <class R>
__device__ __forceinline__ void select_body(const Dev& E, float* __restrict__ planes, SelPre<R>& q) {
    const int g = blockIdx.x, lane = lane_id();
    float* out = planes + (size_t)g * R::PLANES * R::CELLS;
    // (searching(): searcher 0 = self-play, else the searcher's colour to move)
    if (!q.active || q.err || !(q.searcher == 0 || q.searcher == q.root.player)) {
        for (int i = lane; i < R::PLANES * R::CELLS; i += WAVE) out[i] = 0.0f;
        if (lane == 0) E.leaf_kind[g] = LEAF_NONE;
        return;
    }
    BlockRng& rg = q.rg;
    const int root_id = q.root_id;
    Pos p = q.root;
    int depth = 0, kind = LEAF_NONE, slot = -1, cs = 0, kt = 0;
    uint64_t own = 0, opp = 0;
    double tval = 0.0;
    int32_t* path = E.path + (size_t)g * E.DMAX;
    for (;;) {
        if (p.outcome != ONGOING) {  // MCTS.py:85-87
            kind = LEAF_TERMINAL;
            tval = -outcome_value(p.outcome);
            break;
        }
        R::key(p, own, opp, kt, cs);
        const typename R::VCtx vc = R::vctx(own, opp, cs);
        EdgeRow<R> er;
        // the root's node id is cached for the rest of the move (ids are stable;
        // commit_move / set_root invalidate it): one hash probe less per simulation
        int id = depth == 0 ? root_id : -1;
        if (id >= 0) {
            load_edges<R>(E, g, id, vc, er);
        } else {
            id = lookup_with_edges<R>(E, g, own, opp, kt, cs, &slot, vc, er);
            if (depth == 0 && id >= 0 && lane == 0) E.root_id[g] = id;
        }
        if (id < 0) {
            if (slot < 0) set_err(E, g, -3);
            kind = slot < 0 ? LEAF_NONE : LEAF_EXPAND;
            break;
        }
        int ei;
        const int a = puct_select<R>(E, g, id, er, &ei);
        if (a < 0) {
            set_err(E, g, -5);
            kind = LEAF_NONE;
            break;
        }
        if (depth >= E.DMAX) {
            set_err(E, g, -4);
            kind = LEAF_NONE;
            break;
        }
        if (lane == 0) path[depth] = (id << 10) | ei;  // the edge's slot in the node's row
        depth++;
        R::apply(p, a, E.max_turns);
    }
    if (lane == 0) {
        E.leaf_kind[g] = kind;
        E.leaf_depth[g] = depth;
        E.leaf_value[g] = tval;
        E.leaf_own[g] = own;
        E.leaf_opp[g] = opp;
        E.leaf_turn[g] = kt;
        E.leaf_cs[g] = cs;
        E.leaf_slot[g] = slot;
        if (depth > E.st_depth[g]) E.st_depth[g] = depth;
        E.st_sims[g] += 1;
    }
    if (kind != LEAF_EXPAND) {
        for (int i = lane; i < R::PLANES * R::CELLS; i += WAVE) out[i] = 0.0f;
        return;
    }
    R::write_planes(out, own, opp, kt, cs, rg);
    rng_store(rg);
}

// Test evaluator: tests/golden/stubnet.py on the symmetrised planes.
template <class R>
__global__ __launch_bounds__(WAVE) void stub_eval_kernel(const float* __restrict__ planes, float* __restrict__ P,
                                                         float* __restrict__ v) {
    const int g = blockIdx.x, lane = lane_id();
    const float* in = planes + (size_t)g * R::PLANES * R::CELLS;
    const bool on = lane < R::CELLS;
    const uint64_t own = __ballot(on && in[lane] != 0.0f);
    const uint64_t opp = __ballot(on && in[R::CELLS + lane] != 0.0f);
    const uint64_t t = R::PLANES > 2 ? (uint64_t)(int64_t)(int)in[2 * R::CELLS] : 0ull;
    const uint64_t kk = R::PLANES > 3 ? (uint64_t)(int64_t)(int)in[3 * R::CELLS] : 0ull;
    const uint64_t h = mix64(own ^ mix64(opp ^ mix64((t << 1) | kk)));
    const bool all_zero = (h >> 56) < 4;
    for (int a = lane; a < R::A; a += WAVE) {
        const uint64_t ha = mix64(h ^ ((uint64_t)(a + 1) * 0xD1B54A32D192ED03ull));
        const float pa = (float)(uint32_t)(ha & 0xFFFFFFu) * 0x1p-24f;
        P[(size_t)g * R::A + a] = (all_zero || (ha >> 59) == 0) ? 0.0f : pa;
    }
    if (lane == 0) v[g] = (float)((int)((h >> 20) & 2047) - 1024) / 1024.0f;
}

// sim_end: expand the leaf (MCTS.py:89-112) and back the value up the path
// (MCTS.py:136-145).  The path holds distinct nodes, so lanes update one edge
// each with no atomics.
template <class R>
__device__ __forceinline__ ExpandOut expand_backup_body(const Dev& E, const float* __restrict__ Pin, int p_stride,
                                                        const float* __restrict__ vin) {
    ExpandOut xo{0, -1};
    __shared__ float s_p[R::AP];
    __shared__ float s_acc[WAVE];
    __shared__ float s_leaf[16];
    const int g = blockIdx.x, lane = lane_id();
    // Every per-slot field the expansion and the backup read and the path entries are
    // loaded before the first branch on any of them: one memory round trip instead of a
    // chain (kind, then depth, then the path, ...).  The leaf's P row follows the kind
    // check (no slot without a leaf reads it), in the round trip of the path edges' N / Q.
    const int kind = E.leaf_kind[g];
    const int depth = E.leaf_depth[g];
    const int32_t* path = E.path + (size_t)g * E.DMAX;
    constexpr int PATH0 = 16;  // path entries loaded with the record (one 64-B segment; deeper: below)
    const int pk = lane < PATH0 && lane < E.DMAX ? path[lane] : 0;
    const int top_ld = E.free_top[g];
    const uint64_t l_own = E.leaf_own[g], l_opp = E.leaf_opp[g];
    const int l_cs = E.leaf_cs[g], l_kt = E.leaf_turn[g], l_slot = E.leaf_slot[g];
    const double l_value = E.leaf_value[g];
    const float l_v = vin[g];
    if (kind == LEAF_NONE) return xo;
    float praw[R::AJ];
#pragma unroll
    for (int j = 0; j < R::AJ; ++j) {
        const int a = lane + WAVE * j;
        praw[j] = a < R::A && kind == LEAF_EXPAND ? Pin[(size_t)g * p_stride + a] : 0.0f;
    }
    // Everything the backup reads (path entry, edge N and Q; one level per lane) and
    // the free-stack top are fetched up front, so they travel with the leaf's P
    // row instead of after the expansion (the path's edges are never the new node).
    const int packed0 = lane < depth ? (lane < PATH0 ? pk : path[lane]) : 0;
    const int top0 = kind == LEAF_EXPAND ? top_ld : 0;
    uint32_t nr0 = 0u;
    float qf0 = 0.0f;
    if (lane < depth) {
        const size_t erow = ((size_t)g * E.M + (packed0 >> 10)) * R::AP + (packed0 & 1023);
        nr0 = E.node_N[erow];
        qf0 = E.node_Qf[erow];  // used only where N > 0 and Q is f32-typed
    }
    double ret;
    bool ret_f32;
    if (kind == LEAF_EXPAND) {
        const uint64_t own = l_own, opp = l_opp;
        const int cs = l_cs, kt = l_kt;
        const typename R::VCtx vc = R::vctx(own, opp, cs);
        float pv[R::AJ];
        bool vv[R::AJ];
        int ci[R::AJ];
        edge_slots<R>(vc, ci);
#pragma unroll
        for (int j = 0; j < R::AJ; ++j) {
            const int a = lane + WAVE * j;
            vv[j] = ci[j] >= 0;
            float x = praw[j];
            x = vv[j] ? x : x * 0.0f;  // policies *= valids
            pv[j] = x;
            s_p[a] = x;
        }
        __syncthreads();
        const float sum = pairwise_sum<R::A>(s_p, s_acc, s_leaf);
        if (sum > 0.0f) {
#pragma unroll
            for (int j = 0; j < R::AJ; ++j) pv[j] = pv[j] / sum;
        } else {  // MCTS.py:100-107 fallback: policies += valids; policies /= policies.sum()
            if (lane == 0) E.st_fallback[g] += 1;
#pragma unroll
            for (int j = 0; j < R::AJ; ++j) {
                pv[j] = (float)((double)pv[j] + (vv[j] ? 1.0 : 0.0));
                s_p[lane + WAVE * j] = pv[j];
            }
            __syncthreads();
            const float s2 = pairwise_sum<R::A>(s_p, s_acc, s_leaf);
#pragma unroll
            for (int j = 0; j < R::AJ; ++j) pv[j] = pv[j] / s2;
        }
        int id = -1;
        if (lane == 0) {
            const int top = top0;
            if (top > 0) {
                id = E.free_stack[(size_t)g * E.M + top - 1];
                E.free_top[g] = top - 1;
                const int lv = E.live[g] + 1;
                E.live[g] = lv;
                if (lv > E.st_live_max[g]) E.st_live_max[g] = lv;
            }
        }
        id = __shfl(id, 0);
        if (id < 0) {
            set_err(E, g, -3);
            xo.err = -3;
            return xo;
        }
        if (depth == 0) xo.root_id = id;
        const size_t ni = (size_t)g * E.M + id, row = ni * R::AP;
        // the valid actions' edges only, in their compact slots (edge_slots); Q is read
        // only where N > 0: no init
#pragma unroll
        for (int j = 0; j < R::AJ; ++j) {
            if (ci[j] >= 0) {
                E.node_P[row + ci[j]] = pv[j];
                E.node_N[row + ci[j]] = 0u;
            }
        }
        if (lane == 0) {
            if (depth == 0) E.root_id[g] = id;
            E.node_key[ni] = NodeKey{own, opp, kt, cs, 0, 0};
            E.node_turn[ni] = kt;
            const uint64_t h = key_hash(own, opp, kt, cs);
            E.table[(size_t)g * E.H + l_slot] = ((h >> 32) << 32) | (uint64_t)(uint32_t)(id + 1);
            E.st_exp[g] += 1;
        }
        ret = -(double)l_v;  // `return -v`, a float32 array (MCTS.py:112)
        ret_f32 = true;
    } else {
        ret = l_value;  // Python number (MCTS.py:87)
        ret_f32 = false;
        if (lane == 0) E.st_term[g] += 1;
    }
    for (int d = lane; d < depth; d += WAVE) {
        const int packed = d < WAVE ? packed0 : path[d];
        const int id = packed >> 10, a = packed & 1023;
        const double v = ((depth - 1 - d) & 1) ? -ret : ret;
        const size_t ni = (size_t)g * E.M + id, row = ni * R::AP + a;
        const uint32_t nr = d < WAVE ? nr0 : E.node_N[row];
        const int n = (int)(nr & 0x7fffffffu);
        const bool qf = (nr >> 31) != 0;
        double q = 0.0;
        if (n > 0) q = qf ? (double)(d < WAVE ? qf0 : E.node_Qf[row]) : E.node_Q[row];
        bool nf;
        if (n == 0) {  // an edge's first backup defines Q
            q = v;
            nf = ret_f32;
        } else if (qf || ret_f32) {  // numpy f32 arithmetic with weak Python scalars
            const float prod = qf ? (float)n * (float)q : (float)((double)n * q);
            const float num = prod + (float)v;
            q = (double)(num / (float)(n + 1));
            nf = true;
        } else {  // both Python numbers: double arithmetic
            q = ((double)n * q + v) / (double)(n + 1);
            nf = false;
        }
        if (nf)
            E.node_Qf[row] = (float)q;  // exact: an f32-typed Q is an f32 value
        else
            E.node_Q[row] = q;
        E.node_N[row] = (uint32_t)(n + 1) | (nf ? 0x80000000u : 0u);
        E.node_key[ni].Ns += 1;
    }
    return xo;
}

// (the descents' kernels held to 128 VGPRs, 4 waves per SIMD: 131 otherwise since the edge rows are
// loaded with the key check; no spill, +0.7% at C4 alternating on one box, tools/ab_bench.sh)
template <class R>
__global__ __launch_bounds__(WAVE) __attribute__((amdgpu_waves_per_eu(4))) void select_kernel(Dev E, float* __restrict__ planes) {
    SelPre<R> q = select_prefetch<R>(E);
    select_body<R>(E, planes, q);
}

template <class R>
__global__ __launch_bounds__(WAVE) void expand_backup_kernel(Dev E, const float* __restrict__ Pin, int p_stride,
                                                             const float* __restrict__ vin) {
    expand_backup_body<R>(E, Pin, p_stride, vin);
}

// sim_end of one simulation and sim_begin of the next in one launch (same wave, same
// order of operations as the two kernels: the tree writes of the backup are visible to
// the next descent through the workgroup barrier): one kernel boundary less per
// simulation where the search is launch-bound (one leaf per simulation, the drop-in).
template <class R>
__global__ __launch_bounds__(WAVE) __attribute__((amdgpu_waves_per_eu(4))) void expand_select_kernel(Dev E, const float* __restrict__ Pin, int p_stride,
                                                             const float* __restrict__ vin,
                                                             float* __restrict__ planes) {
    SelPre<R> q = select_prefetch<R>(E);  // (the expansion's changes to err / root_id come back in xo)
    const ExpandOut xo = expand_backup_body<R>(E, Pin, p_stride, vin);
    if (xo.err && !q.err) q.err = xo.err;  // (set_err keeps the first code)
    if (xo.root_id >= 0) q.root_id = xo.root_id;
    __syncthreads();
    select_body<R>(E, planes, q);
}

// move_end: MCTS.getActionProb root policy (MCTS.py:48-60), Coach.executeEpisode
// temperature + np.random.choice + step (Coach.py:68-84), record, node GC.
// Game.to_next_state for slot g's root (Coach.py:82 / Arena.py:69): apply the
// action, store the new root, and (AZG_FLAG_GC) free the nodes no later
// search can reach and rebuild the slot's hash table.
template <class R>
__device__ void commit_move(const Dev& E, int g, Pos p, int action, int m) {
    const int lane = lane_id();
    R::apply(p, action, E.max_turns);
    if (lane < R::CELLS) E.board[(size_t)g * 64 + lane] = (int8_t)p.cell;
    if (lane == 0) {
        E.turn[g] = p.turn;
        E.player[g] = p.player;
        E.outcome[g] = p.outcome;
        E.moves[g] = m + 1;
        E.root_id[g] = -1;  // the next search looks the new root up (and caches it)
        if (p.outcome != ONGOING) E.active[g] = 0;
    }
    if (!(E.flags & 1)) return;  // AZG_FLAG_GC
    // Node GC: a search from a root whose key-turn is T only reaches key-turns
    // >= T (Inflexion: the turn, in the key; Othello: the disc count, which
    // never decreases), so nodes below T are dead; keep all others
    // (transpositions may still reach them).  Finished game: free everything.
    uint64_t o2, p2;
    int cs2, T;
    R::key(p, o2, p2, T, cs2);
    if (p.outcome != ONGOING) T = 0x7fffffff;
    const size_t nb0 = (size_t)g * E.M;
    int top = 0, live = 0;
    for (int b = 0; b < E.M; b += WAVE) {
        const int i = b + lane;
        bool fr = false;
        if (i < E.M) {
            int t = E.node_turn[nb0 + i];
            if (t >= 0 && t < T) {
                E.node_turn[nb0 + i] = -1;
                t = -1;
            }
            fr = t < 0;
        }
        const uint64_t fb = __ballot(fr);
        if (fr) E.free_stack[nb0 + top + __popcll(fb & ((1ull << lane) - 1ull))] = i;
        top += __popcll(fb);
        live += __popcll(__ballot(i < E.M && !fr));
    }
    if (lane == 0) {
        E.free_top[g] = top;
        E.live[g] = live;
    }
    uint64_t* T64 = E.table + (size_t)g * E.H;
    for (int s = lane; s < E.H; s += WAVE) T64[s] = 0ull;
    __threadfence_block();
    __syncthreads();
    const uint32_t hm = (uint32_t)E.H - 1;
    for (int b = 0; b < E.M; b += WAVE) {
        const int i = b + lane;
        if (i < E.M && E.node_turn[nb0 + i] >= 0) {
            const NodeKey& k = E.node_key[nb0 + i];
            const uint64_t h = key_hash(k.own, k.opp, k.turn, k.cs);
            const unsigned long long ent = ((h >> 32) << 32) | (uint64_t)(uint32_t)(i + 1);
            uint32_t s = (uint32_t)h & hm;
            while (atomicCAS((unsigned long long*)&T64[s], 0ull, ent) != 0ull) s = (s + 1) & hm;
        }
    }
}

template <class R>
__global__ __launch_bounds__(WAVE) void move_end_kernel(Dev E) {
    __shared__ uint32_t s_mt[MT_N];
    __shared__ int s_cnt[R::AP];
    __shared__ double s_cdf[R::AP];
    const int g = blockIdx.x, lane = lane_id();
    if (!E.active[g] || E.err[g] || !searching(E, g)) return;
    Pos p = load_root<R>(E, g);
    uint64_t own, opp;
    int cs, kt, slot;
    R::key(p, own, opp, kt, cs);
    const int id = table_lookup(E, g, own, opp, kt, cs, &slot);
    int cnt[R::AJ], ci[R::AJ];
    edge_slots<R>(R::vctx(own, opp, cs), ci);
#pragma unroll
    for (int j = 0; j < R::AJ; ++j) {
        const int a = lane + WAVE * j;
        cnt[j] = (id >= 0 && ci[j] >= 0) ? (int)(E.node_N[node_row<R>(E, g, id) + ci[j]] & 0x7fffffffu) : 0;
        s_cnt[a] = cnt[j];
    }
    const int m = E.moves[g];
    const int temp = (m + 1) < E.temp_threshold;  // episodeStep < tempThreshold
    BlockRng rg = rng_open(E.mt + (size_t)g * MT_N, E.mt_pos + g, s_mt);
    int action = -1;
    if (temp == 0) {
        int mx = cnt[0];
#pragma unroll
        for (int j = 1; j < R::AJ; ++j) mx = max(mx, cnt[j]);
        mx = wave_max(mx);
        uint64_t tie[R::AJ];
        int nb = 0;
#pragma unroll
        for (int j = 0; j < R::AJ; ++j) {
            const int a = lane + WAVE * j;
            tie[j] = __ballot(a < R::A && cnt[j] == mx);
            nb += __popcll(tie[j]);
        }
        int pick = rng_randint(rg, 0, nb);  // np.random.choice(bestAs), draws only if nb > 1
#pragma unroll
        for (int j = 0; j < R::AJ; ++j) {
            const int c = __popcll(tie[j]);
            if (action < 0 && pick < c) {
                uint64_t b = tie[j];
                for (int k = 0; k < pick; ++k) b &= b - 1ull;
                action = WAVE * j + __ffsll((unsigned long long)b) - 1;
            }
            if (action < 0) pick -= c;
        }
        // Coach.py:81 np.random.choice(len(pi), p=one-hot) still draws; the arena's
        // MCTSPlayer takes the argmax instead (InflexionPlayers.py:88)
        if (!(E.flags & 4)) (void)rng_random_sample(rg);
    } else {
        __syncthreads();
        if (lane == 0) {  // probs = counts / counts.sum(); cdf = cumsum (sequential f64)
            long long tot = 0;
            for (int a = 0; a < R::A; ++a) tot += s_cnt[a];
            double acc = 0.0;
            for (int a = 0; a < R::A; ++a) {
                acc += (double)s_cnt[a] / (double)tot;
                s_cdf[a] = acc;
            }
        }
        __syncthreads();
        const double last = s_cdf[R::A - 1];
        const double u = rng_random_sample(rg);
        int first = 0x7fffffff;
#pragma unroll
        for (int j = 0; j < R::AJ; ++j) {
            const int a = lane + WAVE * j;
            if (a < R::A && s_cdf[a] / last > u) first = min(first, a);
        }
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) first = min(first, __shfl_xor(first, o));
        action = first == 0x7fffffff ? R::A : first;
    }
    rng_store(rg);
    if (m < E.max_moves) {
        if (lane == 0) {
            E.rec_action[(size_t)g * E.max_moves + m] = action;
            E.rec_temp[(size_t)g * E.max_moves + m] = (int8_t)temp;
        }
        if (E.rec_counts) {
            int32_t* rc = E.rec_counts + ((size_t)g * E.max_moves + m) * R::A;
#pragma unroll
            for (int j = 0; j < R::AJ; ++j) {
                const int a = lane + WAVE * j;
                if (a < R::A) rc[a] = cnt[j];
            }
        }
    }
    if (action < 0 || action >= R::A || !R::valid(action, R::vctx(own, opp, cs))) {
        set_err(E, g, -5);
        return;
    }
    commit_move<R>(E, g, p, action, m);
}

// The arena's baseline players (InflexionPlayers.py:24-77) for the slots whose
// colour to move is not the searcher's: RandomPlayer = np.random.choice over
// the valid actions (the slot's numpy stream); GreedyPlayer = the valid action
// whose next state has the best piece_count_diff for the mover, ties to the
// larger action (candidates.sort(reverse=True)).
template <class R>
__global__ __launch_bounds__(WAVE) void opponent_kernel(Dev E, int kind) {
    __shared__ uint32_t s_mt[MT_N];
    const int g = blockIdx.x, lane = lane_id();
    if (!E.active[g] || E.err[g] || E.searcher[g] == 0 || searching(E, g)) return;
    Pos p = load_root<R>(E, g);
    uint64_t own, opp;
    int cs, kt;
    R::key(p, own, opp, kt, cs);
    const typename R::VCtx vc = R::vctx(own, opp, cs);
    uint64_t vb[R::AJ];
    int nv = 0;
#pragma unroll
    for (int j = 0; j < R::AJ; ++j) {
        const int a = lane + WAVE * j;
        vb[j] = __ballot(a < R::A && R::valid(a, vc));
        nv += __popcll(vb[j]);
    }
    if (nv == 0) {
        set_err(E, g, -5);
        return;
    }
    int action = -1;
    if (kind == 1) {
        BlockRng rg = rng_open(E.mt + (size_t)g * MT_N, E.mt_pos + g, s_mt);
        int pick = rng_randint(rg, 0, nv);
        rng_store(rg);
#pragma unroll
        for (int j = 0; j < R::AJ; ++j) {
            const int c = __popcll(vb[j]);
            if (action < 0 && pick < c) {
                uint64_t b = vb[j];
                for (int k = 0; k < pick; ++k) b &= b - 1ull;
                action = WAVE * j + __ffsll((unsigned long long)b) - 1;
            }
            if (action < 0) pick -= c;
        }
    } else {
        int best = -0x7fffffff;
        const bool on = lane < R::CELLS;
        for (int j = 0; j < R::AJ; ++j) {
            for (uint64_t b = vb[j]; b; b &= b - 1ull) {
                const int a = WAVE * j + __ffsll((unsigned long long)b) - 1;
                Pos q = p;
                R::apply(q, a, E.max_turns);
                const int sc = __popcll(__ballot(on && q.cell * p.player > 0)) -
                               __popcll(__ballot(on && q.cell * p.player < 0));
                if (sc >= best) {
                    best = sc;
                    action = a;
                }
            }
        }
    }
    const int m = E.moves[g];
    if (m < E.max_moves && lane == 0) {
        E.rec_action[(size_t)g * E.max_moves + m] = action;
        E.rec_temp[(size_t)g * E.max_moves + m] = 0;
    }
    commit_move<R>(E, g, p, action, m);
}

// Arena between two searchers (Arena.playGame, Arena.py:54-69, with two MCTSPlayers): two
// arena engines hold the same games, each searching for its own colour.  After the leader
// S has moved in slot g, the follower E plays the same action in its copy of the game and
// takes over S's numpy stream for the slot (the reference's two players draw from one
// process-wide stream).  The action is checked against E's valid mask (Arena.py:64-67).
template <class R>
__global__ __launch_bounds__(WAVE) void follow_kernel(Dev E, Dev S) {
    const int g = blockIdx.x, lane = lane_id();
    if (!E.active[g] || E.err[g] || E.searcher[g] == 0 || searching(E, g)) return;
    const int m = E.moves[g];
    if (S.moves[g] != m + 1) return;  // the leader has not moved in this slot
    if (S.err[g] || m >= S.max_moves) {
        set_err(E, g, -6);  // AZG_ERR_STATE
        return;
    }
    const int action = S.rec_action[(size_t)g * S.max_moves + m];
    Pos p = load_root<R>(E, g);
    uint64_t own, opp;
    int cs, kt;
    R::key(p, own, opp, kt, cs);
    const typename R::VCtx vc = R::vctx(own, opp, cs);
    const bool ok = __ballot(lane == 0 && action >= 0 && action < R::A && R::valid(action, vc)) != 0ull;
    if (!ok) {
        set_err(E, g, -7);  // AZG_ERR_ACTION
        return;
    }
    for (int i = lane; i < MT_N; i += WAVE) E.mt[(size_t)g * MT_N + i] = S.mt[(size_t)g * MT_N + i];
    if (lane == 0) E.mt_pos[g] = S.mt_pos[g];
    if (m < E.max_moves && lane == 0) {
        E.rec_action[(size_t)g * E.max_moves + m] = action;
        E.rec_temp[(size_t)g * E.max_moves + m] = 0;
    }
    commit_move<R>(E, g, p, action, m);
}

// The drop-in's per-call slot I/O in one launch each way (MCTS.getActionProb on one
// game, numpy's global stream handed over and back).  in: board as 16 words of int8,
// turn, player, mt_pos, mt[624] (SLOT_IN_WORDS); out: root visit counts [A], mt[624],
// mt_pos, err, active (A + SLOT_OUT_EXTRA words).
template <class R>
__global__ __launch_bounds__(WAVE) void slot_begin_kernel(Dev E, int g, const int32_t* __restrict__ in) {
    const int lane = lane_id();
    if (lane < 16) ((int32_t*)(E.board + (size_t)g * 64))[lane] = in[lane];
    for (int i = lane; i < MT_N; i += WAVE) E.mt[(size_t)g * MT_N + i] = (uint32_t)in[19 + i];
    if (lane == 0) {
        E.turn[g] = in[16];
        E.player[g] = in[17];
        E.mt_pos[g] = in[18];
        E.outcome[g] = ONGOING;
        E.active[g] = 1;
        E.moves[g] = in[16];
        E.err[g] = 0;
        E.root_id[g] = -1;  // look the new root up
    }
}

template <class R>
__global__ __launch_bounds__(WAVE) void slot_end_kernel(Dev E, int g, int32_t* __restrict__ out) {
    const int lane = lane_id();
    Pos p = load_root<R>(E, g);
    uint64_t own, opp;
    int cs, kt, slot;
    R::key(p, own, opp, kt, cs);
    const int id = table_lookup(E, g, own, opp, kt, cs, &slot);
    int ci[R::AJ];
    edge_slots<R>(R::vctx(own, opp, cs), ci);
#pragma unroll
    for (int j = 0; j < R::AJ; ++j) {
        const int a = lane + WAVE * j;
        if (a < R::A)
            out[a] = (id >= 0 && ci[j] >= 0) ? (int)(E.node_N[node_row<R>(E, g, id) + ci[j]] & 0x7fffffffu) : 0;
    }
    for (int i = lane; i < MT_N; i += WAVE) out[R::A + i] = (int32_t)E.mt[(size_t)g * MT_N + i];
    if (lane == 0) {
        out[R::A + MT_N] = E.mt_pos[g];
        out[R::A + MT_N + 1] = E.err[g];
        out[R::A + MT_N + 2] = E.active[g];
    }
}

// Root visit counts of one slot (drop-in MCTS.getActionProb, MCTS.py:48-49).
template <class R>
__global__ __launch_bounds__(WAVE) void root_counts_kernel(Dev E, int g, int32_t* out) {
    const int lane = lane_id();
    Pos p = load_root<R>(E, g);
    uint64_t own, opp;
    int cs, kt, slot;
    R::key(p, own, opp, kt, cs);
    const int id = table_lookup(E, g, own, opp, kt, cs, &slot);
    int ci[R::AJ];
    edge_slots<R>(R::vctx(own, opp, cs), ci);
#pragma unroll
    for (int j = 0; j < R::AJ; ++j) {
        const int a = lane + WAVE * j;
        if (a < R::A)
            out[a] = (id >= 0 && ci[j] >= 0) ? (int)(E.node_N[node_row<R>(E, g, id) + ci[j]] & 0x7fffffffu) : 0;
    }
}

// A fresh game in slot g (Coach.py:110-111): initial board, RED to move, numpy
// RandomState(seed), empty tree; global game index gid.  Per-slot counters are
// cleared only by a full reset (refilled slots keep accumulating them).
template <class R>
__device__ void reset_slot(const Dev& E, int g, uint32_t seed, long long gid, bool clear_stats) {
    const int lane = lane_id();
    E.board[(size_t)g * 64 + lane] = lane < R::CELLS ? (int8_t)R::initial_cell(lane) : (int8_t)0;
    if (lane == 0) {
        E.turn[g] = 0;
        E.player[g] = 1;
        E.searcher[g] = 0;
        E.root_id[g] = -1;
        E.outcome[g] = ONGOING;
        E.active[g] = 1;
        E.moves[g] = 0;
        E.err[g] = 0;
        E.game_id[g] = gid;
        E.harvested[g] = 0;
        E.free_top[g] = E.M;
        E.live[g] = 0;
        if (clear_stats) {
            E.st_exp[g] = E.st_term[g] = E.st_fallback[g] = E.st_sims[g] = 0;
            E.st_depth[g] = E.st_live_max[g] = 0;
        }
        E.leaf_kind[g] = LEAF_NONE;
        // init_genrand (RandomState.seed): sequential recurrence, one lane
        uint32_t* mt = E.mt + (size_t)g * MT_N;
        uint32_t x = seed;
        mt[0] = x;
        for (int i = 1; i < MT_N; ++i) {
            x = 1812433253u * (x ^ (x >> 30)) + (uint32_t)i;
            mt[i] = x;
        }
        E.mt_pos[g] = MT_N;
    }
    const size_t nb0 = (size_t)g * E.M;
    for (int i = lane; i < E.M; i += WAVE) {
        E.node_turn[nb0 + i] = -1;
        E.free_stack[nb0 + i] = E.M - 1 - i;
    }
    uint64_t* T64 = E.table + (size_t)g * E.H;
    for (int s = lane; s < E.H; s += WAVE) T64[s] = 0ull;
}

// Every slot: the game with global index first_game + g, seeded seed_base + index.
template <class R>
__global__ __launch_bounds__(WAVE) void reset_kernel(Dev E, uint32_t seed_base, long long first_game) {
    const int g = blockIdx.x;
    reset_slot<R>(E, g, seed_base + (uint32_t)(first_game + g), first_game + g, true);
}

// Continuous batching: a slot whose game has ended hands its
// record (game index, moves, actions, temps, root counts) to row j of the
// completed-game buffers (j from a device counter, so rows are in completion
// order) and starts the next global game index at once; past end_game it goes
// idle.  Each game is still seeded by its global index, so its record equals the
// one-game-per-slot run's, whatever slot or moment it ran in.
template <class R>
__global__ __launch_bounds__(WAVE) void refill_kernel(Dev E, RefillArgs X) {
    const int g = blockIdx.x, lane = lane_id();
    if (E.active[g] || E.harvested[g] || E.err[g]) return;
    const long long gid = E.game_id[g];
    unsigned j = 0xffffffffu, klo = 0, khi = 0;
    if (lane == 0) {
        if (gid < X.end_game) j = (unsigned)atomicAdd(X.count, 1ull);
        const unsigned long long k = atomicAdd(X.next_game, 1ull);
        klo = (unsigned)k;
        khi = (unsigned)(k >> 32);
    }
    j = __shfl(j, 0);
    const long long k = (long long)(((unsigned long long)__shfl(khi, 0) << 32) | __shfl(klo, 0));
    if (j != 0xffffffffu && (long long)j < X.cap) {
        const int m = E.moves[g], mm = m < E.max_moves ? m : E.max_moves;
        const size_t src = (size_t)g * E.max_moves, dst = (size_t)j * E.max_moves;
        if (lane == 0) {
            X.ids[j] = gid;
            X.moves[j] = m;
        }
        for (int i = lane; i < mm; i += WAVE) {
            X.actions[dst + i] = E.rec_action[src + i];
            X.temps[dst + i] = E.rec_temp[src + i];
        }
        if (X.counts && E.rec_counts) {  // rows of A (odd for Inflexion): dword copies
            const int32_t* sc = E.rec_counts + src * R::A;
            int32_t* dc = X.counts + dst * R::A;
            const size_t n = (size_t)mm * R::A;
            for (size_t i = lane; i < n; i += WAVE) dc[i] = sc[i];
        }
    }
    if (k < X.end_game)
        reset_slot<R>(E, g, X.seed_base + (uint32_t)k, k, false);
    else if (lane == 0)
        E.harvested[g] = 1;
}

// [0] active slots, [1] first error code
__global__ __launch_bounds__(256) void summary_kernel(Dev E, int32_t* out) {
    int act = 0, err = 0;
    for (int g = threadIdx.x; g < E.G; g += blockDim.x) {
        act += E.active[g] && !E.err[g];
        if (E.err[g] && !err) err = E.err[g];
    }
    __shared__ int s_a[256], s_e[256];
    s_a[threadIdx.x] = act;
    s_e[threadIdx.x] = err;
    __syncthreads();
    if (threadIdx.x == 0) {
        int a = 0, e = 0;
        for (int i = 0; i < (int)blockDim.x; ++i) {
            a += s_a[i];
            if (!e) e = s_e[i];
        }
        out[0] = a;
        out[1] = e;
    }
}

__global__ __launch_bounds__(256) void stats_kernel(Dev E, long long* out) {
    __shared__ long long s[256][8];
    long long v[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int g = threadIdx.x; g < E.G; g += blockDim.x) {
        v[0] += E.st_exp[g];
        v[1] += E.st_term[g];
        v[2] += E.st_fallback[g];
        v[3] = max(v[3], (long long)E.st_depth[g]);
        v[4] = max(v[4], (long long)E.st_live_max[g]);
        if (!v[5] && E.err[g]) v[5] = E.err[g];
        v[6] += E.st_sims[g];
    }
    for (int i = 0; i < 8; ++i) s[threadIdx.x][i] = v[i];
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int t = 1; t < (int)blockDim.x; ++t) {
            v[0] += s[t][0];
            v[1] += s[t][1];
            v[2] += s[t][2];
            v[3] = max(v[3], s[t][3]);
            v[4] = max(v[4], s[t][4]);
            if (!v[5]) v[5] = s[t][5];
            v[6] += s[t][6];
        }
        for (int i = 0; i < 8; ++i) out[i] = v[i];
    }
}

// ------------------------------------------------------ training examples
// Coach.executeEpisode's example list (Coach.py:74-90) rebuilt from compact
// move records (moves, actions, root counts): replay_kernel re-plays every
// game from the initial position (one wave per game), keeping each move's
// root key and player and the final outcome; emit_kernel then writes the
// game.symmetries() forms of each move's planes and policy with its label.

// per-game status: > 0 finished game of that many moves, 0 unfinished/empty, -1 bad record
template <class R>
__global__ __launch_bounds__(WAVE) void replay_kernel(ExampleArgs X) {
    const int g = blockIdx.x, lane = lane_id();
    Pos p;
    p.cell = lane < R::CELLS ? R::initial_cell(lane) : 0;
    p.turn = 0;
    p.player = 1;
    p.outcome = ONGOING;
    const int L = X.moves[g];
    int status = (L < 0 || L > X.MM) ? -1 : L;
    for (int m = 0; m < L && status > 0; ++m) {
        if (p.outcome != ONGOING) {  // record runs past the end of the game
            status = -1;
            break;
        }
        uint64_t own, opp;
        int kt, cs;
        R::key(p, own, opp, kt, cs);
        const int a = X.actions[(size_t)g * X.MM + m];
        if (a < 0 || a >= R::A || !R::valid(a, R::vctx(own, opp, cs))) {
            status = -1;
            break;
        }
        if (lane == 0) X.keys[(size_t)g * X.MM + m] = MoveKey{own, opp, kt, cs | (p.player > 0 ? 2 : 0)};
        R::apply(p, a, X.max_turns);
    }
    if (status > 0 && p.outcome == ONGOING) status = 0;
    if (lane == 0) {
        X.status[g] = status;
        X.zval[g] = (float)outcome_value(p.outcome);  // result.value (flags.py:32-36)
        X.zplayer[g] = p.player;                      // game.player after the last move
    }
}

// Coach.py:79 player list: after move m (0-based) it holds S (m+1)(m+2)/2
// entries, so example el of the game is labelled with the player of move mb,
// the first with S (mb+1)(mb+2)/2 > el
__device__ __forceinline__ int label_move(long long el, int S) {
    int mb = (int)((sqrt(8.0 * (double)el / S + 1.0) - 1.0) * 0.5);
    while ((long long)S * (mb + 1) * (mb + 2) / 2 <= el) ++mb;
    while (mb > 0 && (long long)S * mb * (mb + 1) / 2 > el) --mb;
    return mb;
}

// one 256-thread block per (game g >= g0, move m); writes the move's R::NSYM examples
// that fall inside the kept window [skip, skip + maxlen)
template <class R>
__global__ __launch_bounds__(256) void emit_kernel(ExampleArgs X) {
    __shared__ float s_pi[R::AP];
    __shared__ long long s_part[4];
    __shared__ uint8_t s_src[R::NSYM * R::CELLS];
    const int g = X.g0 + blockIdx.x, m = blockIdx.y, tid = threadIdx.x;
    const int L = X.status[g];
    if (L <= 0 || m >= L) return;
    const long long e0 = X.base[g] + (long long)R::NSYM * m;
    if (e0 + R::NSYM <= X.skip) return;
    const size_t row = (size_t)g * X.MM + m;
    const int temp = (m + 1) < X.temp_threshold;  // episodeStep < tempThreshold (Coach.py:68)
    const int action = X.actions[row];
    long long part = 0;
    const size_t crow = (size_t)g * X.CR + m;  // the move's count row (moves past CR: zero counts)
    for (int a = tid; a < R::A; a += 256) {
        const int c = m >= X.CR ? 0 : X.counts16 ? (int)X.counts16[crow * R::A + a] : X.counts32[crow * R::A + a];
        s_pi[a] = (float)c;  // exact: counts < 2^24
        part += c;
    }
    if (temp) {
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) part += __shfl_xor(part, o);
        if ((tid & 63) == 0) s_part[tid >> 6] = part;
    }
    __syncthreads();
    // getActionProb (MCTS.py:51-60): counts / counts.sum() in f64, or the one-hot
    // of the sampled action; the trainer reads it as f32 (NNet.py:55)
    if (temp) {
        const double tot = (double)(s_part[0] + s_part[1] + s_part[2] + s_part[3]);
        float v[(R::A + 255) / 256];
#pragma unroll
        for (int i = 0; i < (R::A + 255) / 256; ++i) {
            const int a = tid + 256 * i;
            if (a < R::A) v[i] = (float)((double)s_pi[a] / tot);
        }
        __syncthreads();
#pragma unroll
        for (int i = 0; i < (R::A + 255) / 256; ++i) {
            const int a = tid + 256 * i;
            if (a < R::A) s_pi[a] = v[i];
        }
    } else {
        for (int a = tid; a < R::A; a += 256) s_pi[a] = a == action ? 1.0f : 0.0f;
    }
    __syncthreads();
    const MoveKey k = X.keys[row];
    const int cs = k.cp & 1;
    const float zv = X.zval[g];
    const int zp = X.zplayer[g];
    // the move's examples e0 + s (s = s_lo..NSYM-1 inside the window) are
    // consecutive rows of planes / pis / vs: write them as three flat,
    // fully coalesced ranges, gathering through an LDS table of symmetry sources
    const int s_lo = e0 < X.skip ? (int)(X.skip - e0) : 0;
    const long long o0 = e0 + s_lo - X.skip;
    for (int t = tid; t < (R::NSYM - s_lo) * R::CELLS; t += 256) {
        const int s = s_lo + t / R::CELLS;
        s_src[t] = (uint8_t)R::form_src(s, t - (t / R::CELLS) * R::CELLS);
    }
    __syncthreads();
    constexpr int PC = R::PLANES * R::CELLS;
    float* pl = X.planes + o0 * PC;
    for (int t = tid; t < (R::NSYM - s_lo) * PC; t += 256) {
        const int j = t / PC, r = t - j * PC, q = r / R::CELLS, c = r - q * R::CELLS;
        pl[t] = R::plane(q, s_src[j * R::CELLS + c], k.own, k.opp, k.kt, cs);
    }
    float* pi = X.pis + o0 * R::A;
    for (int t = tid; t < (R::NSYM - s_lo) * R::A; t += 256) {
        const int j = t / R::A, a = t - j * R::A;
        const int mv = a / R::CELLS, c = a - mv * R::CELLS;
        pi[t] = s_pi[a < R::SYM_ACTIONS ? mv * R::CELLS + s_src[j * R::CELLS + c] : a];
    }
    for (int j = tid; j < R::NSYM - s_lo; j += 256) {
        const long long el = (long long)R::NSYM * m + s_lo + j;
        const int mb = X.label_mode == 0 ? label_move(el, R::NSYM) : m;
        const int player = (X.keys[(size_t)g * X.MM + mb].cp & 2) ? 1 : -1;
        X.vs[o0 + j] = player == zp ? zv : -zv;
    }
}

// ------------------------------------------------------------- launchers
template <class R>
struct Impl {
    static hipError_t replay(const ExampleArgs& X, hipStream_t st) {
        hipLaunchKernelGGL(replay_kernel<R>, dim3(X.G), dim3(WAVE), 0, st, X);
        return hipGetLastError();
    }
    static hipError_t emit(const ExampleArgs& X, hipStream_t st) {
        if (X.G - X.g0 <= 0) return hipSuccess;
        hipLaunchKernelGGL(emit_kernel<R>, dim3(X.G - X.g0, X.MM), dim3(256), 0, st, X);
        return hipGetLastError();
    }
    static hipError_t select(const Dev& E, float* planes, hipStream_t st) {
        hipLaunchKernelGGL(select_kernel<R>, dim3(E.G), dim3(WAVE), 0, st, E, planes);
        return hipGetLastError();
    }
    static hipError_t stub_eval(const Dev& E, const float* planes, float* P, float* v, hipStream_t st) {
        hipLaunchKernelGGL(stub_eval_kernel<R>, dim3(E.G), dim3(WAVE), 0, st, planes, P, v);
        return hipGetLastError();
    }
    static hipError_t expand_backup(const Dev& E, const float* P, int p_stride, const float* v, hipStream_t st) {
        hipLaunchKernelGGL(expand_backup_kernel<R>, dim3(E.G), dim3(WAVE), 0, st, E, P, p_stride, v);
        return hipGetLastError();
    }
    static hipError_t expand_select(const Dev& E, const float* P, int p_stride, const float* v, float* planes,
                                    hipStream_t st) {
        hipLaunchKernelGGL(expand_select_kernel<R>, dim3(E.G), dim3(WAVE), 0, st, E, P, p_stride, v, planes);
        return hipGetLastError();
    }
    static hipError_t move_end(const Dev& E, hipStream_t st) {
        hipLaunchKernelGGL(move_end_kernel<R>, dim3(E.G), dim3(WAVE), 0, st, E);
        return hipGetLastError();
    }
    static hipError_t opponent(const Dev& E, int kind, hipStream_t st) {
        hipLaunchKernelGGL(opponent_kernel<R>, dim3(E.G), dim3(WAVE), 0, st, E, kind);
        return hipGetLastError();
    }
    static hipError_t follow(const Dev& E, const Dev& S, hipStream_t st) {
        hipLaunchKernelGGL(follow_kernel<R>, dim3(E.G), dim3(WAVE), 0, st, E, S);
        return hipGetLastError();
    }
    static hipError_t slot_begin(const Dev& E, int g, const int32_t* in, hipStream_t st) {
        hipLaunchKernelGGL(slot_begin_kernel<R>, dim3(1), dim3(WAVE), 0, st, E, g, in);
        return hipGetLastError();
    }
    static hipError_t slot_end(const Dev& E, int g, int32_t* out, hipStream_t st) {
        hipLaunchKernelGGL(slot_end_kernel<R>, dim3(1), dim3(WAVE), 0, st, E, g, out);
        return hipGetLastError();
    }
    static hipError_t root_counts(const Dev& E, int g, int32_t* out, hipStream_t st) {
        hipLaunchKernelGGL(root_counts_kernel<R>, dim3(1), dim3(WAVE), 0, st, E, g, out);
        return hipGetLastError();
    }
    static hipError_t reset(const Dev& E, uint32_t seed_base, long long first_game, hipStream_t st) {
        hipLaunchKernelGGL(reset_kernel<R>, dim3(E.G), dim3(WAVE), 0, st, E, seed_base, first_game);
        return hipGetLastError();
    }
    static hipError_t refill(const Dev& E, const RefillArgs& X, hipStream_t st) {
        hipLaunchKernelGGL(refill_kernel<R>, dim3(E.G), dim3(WAVE), 0, st, E, X);
        return hipGetLastError();
    }
};

template <class R>
static GameOps make_ops() {
    GameOps o;
    o.cells = R::CELLS;
    o.actions = R::A;
    o.row = R::AP;
    o.planes = R::PLANES;
    o.nsym = R::NSYM;
    o.select = &Impl<R>::select;
    o.stub_eval = &Impl<R>::stub_eval;
    o.expand_backup = &Impl<R>::expand_backup;
    o.move_end = &Impl<R>::move_end;
    o.expand_select = &Impl<R>::expand_select;
    o.root_counts = &Impl<R>::root_counts;
    o.slot_begin = &Impl<R>::slot_begin;
    o.slot_end = &Impl<R>::slot_end;
    o.reset = &Impl<R>::reset;
    o.refill = &Impl<R>::refill;
    o.opponent = &Impl<R>::opponent;
    o.follow = &Impl<R>::follow;
    o.replay = &Impl<R>::replay;
    o.emit = &Impl<R>::emit;
    return o;
}

bool game_ops(int kind, int n, GameOps* out) {
    if (kind == 1 && n == 7) {
        *out = make_ops<Inflexion>();
        return true;
    }
    if (kind == 2 && n == 6) {
        *out = make_ops<Othello<6>>();
        return true;
    }
    if (kind == 2 && n == 8) {
        *out = make_ops<Othello<8>>();
        return true;
    }
    return false;
}

hipError_t launch_summary(const Dev& E, int32_t* out, hipStream_t st) {
    hipLaunchKernelGGL(summary_kernel, dim3(1), dim3(256), 0, st, E, out);
    return hipGetLastError();
}
hipError_t launch_stats(const Dev& E, long long* out, hipStream_t st) {
    hipLaunchKernelGGL(stats_kernel, dim3(1), dim3(256), 0, st, E, out);
    return hipGetLastError();
}

}  // namespace azg
