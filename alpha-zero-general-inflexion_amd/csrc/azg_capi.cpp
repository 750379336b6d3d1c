// azg_capi.cpp -- the C ABI (include/azg.h) over the engine kernels.
//
// Owns every device allocation of an engine (one arena per engine, sized once
// at azg_create for G slots x node_capacity nodes) and forwards each call to a
// kernel on the caller's stream.  Calls that hand data to the host synchronise
// that stream; the per-simulation calls never do.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <string.h>

#include <string>
#include <vector>

#include "../../include/azg.h"
#include "azg_engine.h"
#include "azg_launch.h"

using azg::Dev;

namespace {
thread_local std::string g_err;

int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}

#define HIP_TRY(expr)                                                                   \
    do {                                                                                \
        hipError_t _e = (expr);                                                         \
        if (_e != hipSuccess)                                                           \
            return fail(AZG_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(_e)); \
    } while (0)

int next_pow2(int x) {
    int p = 1;
    while (p < x) p <<= 1;
    return p;
}
}  // namespace

// the thread-local error message for the host-only helpers (azg_host.cpp)
int azg_host_fail(int code, const std::string& msg) { return fail(code, msg); }

struct azg_engine {
    azg_config cfg;
    Dev d;
    azg::GameOps ops;
    int device;
    std::vector<void*> allocs;
    int32_t* summary;   // device [2]
    long long* stats;   // device [8]
    int32_t* counts1;   // device [A]
    size_t bytes;
    // drop-in slot I/O (azg_slot_begin / azg_slot_end), allocated at first use
    int32_t* io_dev = nullptr;   // device [SLOT_IN_WORDS + A + SLOT_OUT_EXTRA]
    int32_t* io_host = nullptr;  // pinned, same layout
    hipEvent_t io_copied = nullptr;  // the last slot_begin's upload has been read
};

namespace {
constexpr int SLOT_IN_WORDS = 19 + azg::MT_N, SLOT_OUT_EXTRA = azg::MT_N + 3;
}

// Zeroed on the caller's stream, ahead of azg_reset's kernels on that stream: a plain
// hipMemset runs on the null stream, which a non-blocking stream (every torch side
// stream) does not wait for, so the reset kernels could run first and be zeroed after.
template <typename T>
static int dalloc(azg_engine* e, T** p, size_t n, hipStream_t st) {
    void* q = nullptr;
    size_t b = n * sizeof(T);
    if (b == 0) b = 16;
    HIP_TRY(hipMalloc(&q, b));
    HIP_TRY(hipMemsetAsync(q, 0, b, st));
    e->allocs.push_back(q);
    e->bytes += b;
    *p = (T*)q;
    return 0;
}

#define ALLOC(ptr, n)                          \
    do {                                       \
        int _r = dalloc(e, &(ptr), (size_t)(n), (hipStream_t)stream); \
        if (_r) {                              \
            azg_destroy(e);                    \
            return _r;                         \
        }                                      \
    } while (0)

extern "C" {

const char* azg_last_error(void) { return g_err.c_str(); }

int azg_abi_version(void) { return AZG_ABI_VERSION; }

int azg_create(const azg_config* cfg, void* stream, azg_engine** out) {
    if (!cfg || !out) return fail(AZG_ERR_ARG, "null argument");
    azg::GameOps ops;
    if (!azg::game_ops(cfg->game_kind, cfg->n, &ops))
        return fail(AZG_ERR_ARG, "unsupported game: built for InflexionGame(7), OthelloGame(6), OthelloGame(8)");
    if (cfg->num_games <= 0 || cfg->sims <= 0 || cfg->max_turns < 0)
        return fail(AZG_ERR_ARG, "num_games, sims must be > 0 and max_turns >= 0");
    int device = 0;
    HIP_TRY(hipGetDevice(&device));
    auto* e = new azg_engine();
    memset(&e->d, 0, sizeof(Dev));
    e->cfg = *cfg;
    e->ops = ops;
    e->device = device;
    const size_t A = (size_t)ops.actions, ROW = (size_t)ops.row;
    e->bytes = 0;
    Dev& d = e->d;
    d.G = cfg->num_games;
    d.M = cfg->node_capacity > 0 ? cfg->node_capacity : 16 * cfg->sims + 128;
    if (d.M >= (1 << 21)) {
        delete e;
        return fail(AZG_ERR_ARG, "node_capacity must be < 2^21");
    }
    d.H = next_pow2(2 * d.M < 64 ? 64 : 2 * d.M);
    d.DMAX = cfg->max_depth > 0 ? cfg->max_depth : 256;
    d.max_moves = cfg->max_moves > 0 ? cfg->max_moves : cfg->max_turns + 1;
    d.max_turns = cfg->max_turns;
    d.sims = cfg->sims;
    d.temp_threshold = cfg->temp_threshold;
    d.flags = cfg->flags;
    d.cpuct_f = (float)cfg->cpuct;
    const size_t G = (size_t)d.G, GM = G * (size_t)d.M;
    ALLOC(d.board, G * 64);
    ALLOC(d.turn, G);
    ALLOC(d.player, G);
    ALLOC(d.outcome, G);
    ALLOC(d.active, G);
    ALLOC(d.searcher, G);
    ALLOC(d.root_id, G);
    ALLOC(d.mt, G * azg::MT_N);
    ALLOC(d.mt_pos, G);
    ALLOC(d.node_key, GM);
    ALLOC(d.node_turn, GM);
    ALLOC(d.node_P, GM * ROW);
    ALLOC(d.node_N, GM * ROW);
    ALLOC(d.node_Qf, GM * ROW);
    ALLOC(d.node_Q, GM * ROW);
    ALLOC(d.free_stack, GM);
    ALLOC(d.free_top, G);
    ALLOC(d.live, G);
    ALLOC(d.table, G * (size_t)d.H);
    ALLOC(d.path, G * (size_t)d.DMAX);
    ALLOC(d.leaf_kind, G);
    ALLOC(d.leaf_depth, G);
    ALLOC(d.leaf_value, G);
    ALLOC(d.leaf_own, G);
    ALLOC(d.leaf_opp, G);
    ALLOC(d.leaf_turn, G);
    ALLOC(d.leaf_cs, G);
    ALLOC(d.leaf_slot, G);
    ALLOC(d.moves, G);
    ALLOC(d.game_id, G);
    ALLOC(d.harvested, G);
    ALLOC(d.rec_action, G * (size_t)d.max_moves);
    ALLOC(d.rec_temp, G * (size_t)d.max_moves);
    if (cfg->flags & AZG_FLAG_RECORD) ALLOC(d.rec_counts, G * (size_t)d.max_moves * A);
    ALLOC(d.st_exp, G);
    ALLOC(d.st_term, G);
    ALLOC(d.st_fallback, G);
    ALLOC(d.st_sims, G);
    ALLOC(d.st_depth, G);
    ALLOC(d.st_live_max, G);
    ALLOC(d.err, G);
    ALLOC(e->summary, 2);
    ALLOC(e->stats, 8);
    ALLOC(e->counts1, A);
    *out = e;
    int r = azg_reset(e, cfg->seed_base, cfg->first_game, stream);
    if (r) {
        azg_destroy(e);
        *out = nullptr;
        return r;
    }
    return 0;
}

void azg_destroy(azg_engine* e) {
    if (!e) return;
    if (e->io_copied) (void)hipEventSynchronize(e->io_copied), (void)hipEventDestroy(e->io_copied);
    if (e->io_host) (void)hipHostFree(e->io_host);
    for (void* p : e->allocs) (void)hipFree(p);
    delete e;
}

int azg_reset(azg_engine* e, uint32_t seed_base, int64_t first_game, void* stream) {
    if (!e) return fail(AZG_ERR_ARG, "null engine");
    e->cfg.seed_base = seed_base;
    e->cfg.first_game = first_game;
    HIP_TRY(e->ops.reset(e->d, seed_base, (long long)first_game, (hipStream_t)stream));
    return 0;
}

int azg_refill(azg_engine* e, int64_t* next_game, int64_t end_game, uint32_t seed_base, int64_t* count,
               int64_t cap, int64_t* ids, int32_t* moves, int32_t* actions, int8_t* temps, int32_t* counts,
               void* stream) {
    if (!e || !next_game || !count || cap < 0 || (cap > 0 && (!ids || !moves || !actions || !temps)))
        return fail(AZG_ERR_ARG, "null argument or negative cap");
    if (counts && !e->d.rec_counts) return fail(AZG_ERR_ARG, "counts requested but the engine records none");
    azg::RefillArgs X;
    X.next_game = (unsigned long long*)next_game;
    X.end_game = (long long)end_game;
    X.seed_base = seed_base;
    X.count = (unsigned long long*)count;
    X.cap = (long long)cap;
    X.ids = ids;
    X.moves = moves;
    X.actions = actions;
    X.temps = temps;
    X.counts = counts;
    HIP_TRY(e->ops.refill(e->d, X, (hipStream_t)stream));
    return 0;
}

int azg_sim_begin(azg_engine* e, float* leaf_planes, void* stream) {
    if (!e || !leaf_planes) return fail(AZG_ERR_ARG, "null argument");
    HIP_TRY(e->ops.select(e->d, leaf_planes, (hipStream_t)stream));
    return 0;
}

int azg_sim_end(azg_engine* e, const float* P, int32_t p_stride, const float* v, void* stream) {
    if (!e || !P || !v || p_stride < e->ops.actions) return fail(AZG_ERR_ARG, "bad P/v");
    HIP_TRY(e->ops.expand_backup(e->d, P, p_stride, v, (hipStream_t)stream));
    return 0;
}

int azg_sim_end_begin(azg_engine* e, const float* P, int32_t p_stride, const float* v, float* leaf_planes,
                      void* stream) {
    if (!e || !P || !v || !leaf_planes || p_stride < e->ops.actions) return fail(AZG_ERR_ARG, "bad P/v/planes");
    HIP_TRY(e->ops.expand_select(e->d, P, p_stride, v, leaf_planes, (hipStream_t)stream));
    return 0;
}

int azg_stub_eval(azg_engine* e, const float* leaf_planes, float* P, float* v, void* stream) {
    if (!e || !leaf_planes || !P || !v) return fail(AZG_ERR_ARG, "null argument");
    HIP_TRY(e->ops.stub_eval(e->d, leaf_planes, P, v, (hipStream_t)stream));
    return 0;
}

int azg_move_end(azg_engine* e, void* stream) {
    if (!e) return fail(AZG_ERR_ARG, "null engine");
    HIP_TRY(e->ops.move_end(e->d, (hipStream_t)stream));
    return 0;
}

static const char* err_name(int code) {
    switch (code) {
        case AZG_ERR_NODE_POOL: return "node pool or hash table full (raise node_capacity)";
        case AZG_ERR_PATH: return "search path deeper than max_depth";
        case AZG_ERR_NO_ACTION: return "no valid action at a searched node";
        case AZG_ERR_STATE: return "arena: the leader engine failed in this slot";
        case AZG_ERR_ACTION: return "arena: the leader's action is not valid in the follower's game";
        default: return "engine error";
    }
}

int azg_active_games(azg_engine* e, int32_t* out, void* stream) {
    if (!e || !out) return fail(AZG_ERR_ARG, "null argument");
    hipStream_t st = (hipStream_t)stream;
    int32_t h[2];
    HIP_TRY(azg::launch_summary(e->d, e->summary, st));
    HIP_TRY(hipMemcpyAsync(h, e->summary, sizeof(h), hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    *out = h[0];
    if (h[1]) return fail(h[1], err_name(h[1]));
    return 0;
}

int azg_get_state(azg_engine* e, int8_t* boards, int32_t* turns, int32_t* players, int32_t* outcomes,
                  int32_t* active, void* stream) {
    if (!e) return fail(AZG_ERR_ARG, "null engine");
    hipStream_t st = (hipStream_t)stream;
    const int G = e->d.G, nn = e->ops.cells;
    if (boards) {
        std::vector<int8_t> tmp((size_t)G * 64);
        HIP_TRY(hipMemcpyAsync(tmp.data(), e->d.board, tmp.size(), hipMemcpyDeviceToHost, st));
        HIP_TRY(hipStreamSynchronize(st));
        for (int g = 0; g < G; ++g) memcpy(boards + (size_t)g * nn, tmp.data() + (size_t)g * 64, nn);
    }
    if (turns) HIP_TRY(hipMemcpyAsync(turns, e->d.turn, G * 4, hipMemcpyDeviceToHost, st));
    if (players) HIP_TRY(hipMemcpyAsync(players, e->d.player, G * 4, hipMemcpyDeviceToHost, st));
    if (outcomes) HIP_TRY(hipMemcpyAsync(outcomes, e->d.outcome, G * 4, hipMemcpyDeviceToHost, st));
    if (active) HIP_TRY(hipMemcpyAsync(active, e->d.active, G * 4, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    return 0;
}

int azg_set_root(azg_engine* e, int32_t slot, const int8_t* board, int32_t turn, int32_t player, void* stream) {
    if (!e || !board || slot < 0 || slot >= e->d.G || (player != 1 && player != -1))
        return fail(AZG_ERR_ARG, "bad set_root argument");
    hipStream_t st = (hipStream_t)stream;
    int8_t b[64] = {0};
    memcpy(b, board, (size_t)e->ops.cells);
    const int32_t ongoing = azg::ONGOING, one = 1, zero = 0;
    HIP_TRY(hipMemcpyAsync(e->d.board + (size_t)slot * 64, b, 64, hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemcpyAsync(e->d.turn + slot, &turn, 4, hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemcpyAsync(e->d.player + slot, &player, 4, hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemcpyAsync(e->d.outcome + slot, &ongoing, 4, hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemcpyAsync(e->d.active + slot, &one, 4, hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemcpyAsync(e->d.moves + slot, &turn, 4, hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemcpyAsync(e->d.err + slot, &zero, 4, hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemsetAsync(e->d.root_id + slot, 0xff, 4, st));  // -1: look the new root up
    HIP_TRY(hipStreamSynchronize(st));
    return 0;
}

static int slot_io(azg_engine* e, void* stream) {
    if (e->io_dev) return 0;
    const size_t words = (size_t)SLOT_IN_WORDS + e->ops.actions + SLOT_OUT_EXTRA;
    int r = dalloc(e, &e->io_dev, words, (hipStream_t)stream);
    if (r) return r;
    HIP_TRY(hipHostMalloc((void**)&e->io_host, words * 4, hipHostMallocDefault));
    HIP_TRY(hipEventCreateWithFlags(&e->io_copied, hipEventDisableTiming));
    return 0;
}

int azg_slot_begin(azg_engine* e, int32_t slot, const int8_t* board, int32_t turn, int32_t player,
                   const uint32_t* mt, int32_t pos, void* stream) {
    if (!e || !board || !mt || slot < 0 || slot >= e->d.G || (player != 1 && player != -1) || pos < 0 ||
        pos > azg::MT_N)
        return fail(AZG_ERR_ARG, "bad slot_begin argument");
    int r = slot_io(e, stream);
    if (r) return r;
    hipStream_t st = (hipStream_t)stream;
    HIP_TRY(hipEventSynchronize(e->io_copied));  // the previous upload has left the staging buffer
    int32_t* h = e->io_host;
    memset(h, 0, 64);
    memcpy(h, board, (size_t)e->ops.cells);
    h[16] = turn;
    h[17] = player;
    h[18] = pos;
    memcpy(h + 19, mt, azg::MT_N * 4);
    HIP_TRY(hipMemcpyAsync(e->io_dev, h, (size_t)SLOT_IN_WORDS * 4, hipMemcpyHostToDevice, st));
    HIP_TRY(hipEventRecord(e->io_copied, st));
    HIP_TRY(e->ops.slot_begin(e->d, slot, e->io_dev, st));
    return 0;
}

int azg_slot_end(azg_engine* e, int32_t slot, int32_t* counts, uint32_t* mt, int32_t* pos, int32_t* active,
                 void* stream) {
    if (!e || !counts || !mt || !pos || slot < 0 || slot >= e->d.G) return fail(AZG_ERR_ARG, "bad slot_end argument");
    int r = slot_io(e, stream);
    if (r) return r;
    hipStream_t st = (hipStream_t)stream;
    const int A = e->ops.actions;
    int32_t* dout = e->io_dev + SLOT_IN_WORDS;
    int32_t* hout = e->io_host + SLOT_IN_WORDS;
    HIP_TRY(e->ops.slot_end(e->d, slot, dout, st));
    HIP_TRY(hipMemcpyAsync(hout, dout, (size_t)(A + SLOT_OUT_EXTRA) * 4, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    memcpy(counts, hout, (size_t)A * 4);
    memcpy(mt, hout + A, azg::MT_N * 4);
    *pos = hout[A + azg::MT_N];
    if (active) *active = hout[A + azg::MT_N + 2];
    const int err = hout[A + azg::MT_N + 1];
    if (err) return fail(err, err_name(err));
    return 0;
}

int azg_get_rng(azg_engine* e, int32_t slot, uint32_t* mt, int32_t* pos, void* stream) {
    if (!e || !mt || !pos || slot < 0 || slot >= e->d.G) return fail(AZG_ERR_ARG, "bad get_rng argument");
    hipStream_t st = (hipStream_t)stream;
    HIP_TRY(hipMemcpyAsync(mt, e->d.mt + (size_t)slot * azg::MT_N, azg::MT_N * 4, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipMemcpyAsync(pos, e->d.mt_pos + slot, 4, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    return 0;
}

int azg_set_rng(azg_engine* e, int32_t slot, const uint32_t* mt, int32_t pos, void* stream) {
    if (!e || !mt || slot < 0 || slot >= e->d.G || pos < 0 || pos > azg::MT_N)
        return fail(AZG_ERR_ARG, "bad set_rng argument");
    hipStream_t st = (hipStream_t)stream;
    HIP_TRY(hipMemcpyAsync(e->d.mt + (size_t)slot * azg::MT_N, mt, azg::MT_N * 4, hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemcpyAsync(e->d.mt_pos + slot, &pos, 4, hipMemcpyHostToDevice, st));
    HIP_TRY(hipStreamSynchronize(st));
    return 0;
}

int azg_root_counts(azg_engine* e, int32_t slot, int32_t* counts, void* stream) {
    if (!e || !counts || slot < 0 || slot >= e->d.G) return fail(AZG_ERR_ARG, "bad root_counts argument");
    hipStream_t st = (hipStream_t)stream;
    HIP_TRY(e->ops.root_counts(e->d, slot, e->counts1, st));
    HIP_TRY(hipMemcpyAsync(counts, e->counts1, (size_t)e->ops.actions * 4, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    return 0;
}

int azg_read_moves(azg_engine* e, int32_t* actions, int8_t* temps, int32_t* counts, int32_t* moves,
                   void* stream) {
    if (!e) return fail(AZG_ERR_ARG, "null engine");
    hipStream_t st = (hipStream_t)stream;
    const size_t G = (size_t)e->d.G, MM = (size_t)e->d.max_moves;
    if (actions) HIP_TRY(hipMemcpyAsync(actions, e->d.rec_action, G * MM * 4, hipMemcpyDeviceToHost, st));
    if (temps) HIP_TRY(hipMemcpyAsync(temps, e->d.rec_temp, G * MM, hipMemcpyDeviceToHost, st));
    if (counts) {
        if (!e->d.rec_counts) return fail(AZG_ERR_STATE, "engine created without AZG_FLAG_RECORD");
        HIP_TRY(hipMemcpyAsync(counts, e->d.rec_counts, G * MM * (size_t)e->ops.actions * 4, hipMemcpyDeviceToHost,
                               st));
    }
    if (moves) HIP_TRY(hipMemcpyAsync(moves, e->d.moves, G * 4, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    return 0;
}

int azg_stats(azg_engine* e, int64_t* out, void* stream) {
    if (!e || !out) return fail(AZG_ERR_ARG, "null argument");
    hipStream_t st = (hipStream_t)stream;
    HIP_TRY(azg::launch_stats(e->d, e->stats, st));
    HIP_TRY(hipMemcpyAsync(out, e->stats, 8 * 8, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    return 0;
}

int azg_device_ptrs(azg_engine* e, void** out) {
    if (!e || !out) return fail(AZG_ERR_ARG, "null argument");
    out[0] = e->d.board;
    out[1] = e->d.turn;
    out[2] = e->d.player;
    out[3] = e->d.outcome;
    out[4] = e->d.active;
    out[5] = e->d.rec_action;
    out[6] = e->d.rec_counts;
    out[7] = e->d.moves;
    return 0;
}

int azg_set_arena(azg_engine* e, const int32_t* searcher, const int32_t* first_player, void* stream) {
    if (!e || !searcher || !first_player) return fail(AZG_ERR_ARG, "null argument");
    if (!(e->cfg.flags & AZG_FLAG_ARENA)) return fail(AZG_ERR_STATE, "engine created without AZG_FLAG_ARENA");
    const size_t G = (size_t)e->d.G;
    for (size_t g = 0; g < G; ++g)
        if ((searcher[g] != 1 && searcher[g] != -1) || (first_player[g] != 1 && first_player[g] != -1))
            return fail(AZG_ERR_ARG, "searcher / first_player must be +1 (RED) or -1 (BLUE)");
    hipStream_t st = (hipStream_t)stream;
    HIP_TRY(hipMemcpyAsync(e->d.searcher, searcher, G * 4, hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemcpyAsync(e->d.player, first_player, G * 4, hipMemcpyHostToDevice, st));
    HIP_TRY(hipStreamSynchronize(st));
    return 0;
}

int azg_opponent_move(azg_engine* e, int32_t kind, void* stream) {
    if (!e) return fail(AZG_ERR_ARG, "null engine");
    if (kind != AZG_OPPONENT_RANDOM && kind != AZG_OPPONENT_GREEDY) return fail(AZG_ERR_ARG, "unknown opponent");
    HIP_TRY(e->ops.opponent(e->d, kind, (hipStream_t)stream));
    return 0;
}

int azg_arena_follow(azg_engine* e, const azg_engine* leader, void* stream) {
    if (!e || !leader || e == leader) return fail(AZG_ERR_ARG, "need two distinct engines");
    if (!(e->cfg.flags & AZG_FLAG_ARENA) || !(leader->cfg.flags & AZG_FLAG_ARENA))
        return fail(AZG_ERR_STATE, "engines created without AZG_FLAG_ARENA");
    if (e->cfg.game_kind != leader->cfg.game_kind || e->cfg.n != leader->cfg.n || e->d.G != leader->d.G ||
        e->d.max_turns != leader->d.max_turns || e->device != leader->device)
        return fail(AZG_ERR_ARG, "engines differ in game, size, slot count, max_turns or device");
    HIP_TRY(e->ops.follow(e->d, leader->d, (hipStream_t)stream));
    return 0;
}

int azg_game_info(int32_t game_kind, int32_t n, int32_t* out) {
    azg::GameOps ops;
    if (!out || !azg::game_ops(game_kind, n, &ops)) return fail(AZG_ERR_ARG, "unsupported game kind / size");
    out[0] = ops.cells;
    out[1] = ops.actions;
    out[2] = ops.planes;
    out[3] = ops.nsym;
    return 0;
}

int azg_examples(int32_t game_kind, int32_t n, int32_t max_turns, int32_t temp_threshold, int32_t num_games,
                 int32_t max_moves, const int32_t* moves, const int32_t* actions, const void* counts,
                 int32_t counts_bytes, int32_t label_mode, int64_t maxlen, float* planes, float* pis, float* vs,
                 int64_t* count, void* stream) {
    return azg_examples_rows(game_kind, n, max_turns, temp_threshold, num_games, max_moves, moves, actions, counts,
                             max_moves, counts_bytes, label_mode, maxlen, planes, pis, vs, count, stream);
}

int azg_examples_rows(int32_t game_kind, int32_t n, int32_t max_turns, int32_t temp_threshold, int32_t num_games,
                      int32_t max_moves, const int32_t* moves, const int32_t* actions, const void* counts,
                      int32_t count_rows, int32_t counts_bytes, int32_t label_mode, int64_t maxlen, float* planes,
                      float* pis, float* vs, int64_t* count, void* stream) {
    azg::GameOps ops;
    if (!azg::game_ops(game_kind, n, &ops)) return fail(AZG_ERR_ARG, "unsupported game kind / size");
    if (count_rows < 0 || count_rows > max_moves || (count_rows < max_moves && count_rows < temp_threshold - 1))
        return fail(AZG_ERR_ARG, "azg_examples_rows: count_rows must cover the temperature-1 moves");
    if (num_games < 0 || max_moves <= 0 || max_moves > 65535 || !moves || !actions || (!counts && count_rows) || !count ||
        (counts_bytes != 2 && counts_bytes != 4) || (label_mode != 0 && label_mode != 1) || maxlen < 0 ||
        (maxlen > 0 && (!planes || !pis || !vs)))
        return fail(AZG_ERR_ARG, "bad azg_examples argument");
    *count = 0;
    if (num_games == 0 || maxlen == 0) return 0;
    hipStream_t st = (hipStream_t)stream;
    const size_t G = (size_t)num_games, MM = (size_t)max_moves;
    azg::ExampleArgs X{};
    X.G = num_games;
    X.MM = max_moves;
    X.max_turns = max_turns;
    X.temp_threshold = temp_threshold;
    X.label_mode = label_mode;
    X.moves = moves;
    X.actions = actions;
    X.counts16 = counts_bytes == 2 ? (const int16_t*)counts : nullptr;
    X.counts32 = counts_bytes == 4 ? (const int32_t*)counts : nullptr;
    X.CR = count_rows;
    X.planes = planes;
    X.pis = pis;
    X.vs = vs;
    // one scratch block: keys [G*MM] | base [G] | status [G] | zplayer [G] | zval [G]
    const size_t bytes = G * MM * sizeof(azg::MoveKey) + G * 8 + G * 4 * 3;
    char* scratch = nullptr;
    HIP_TRY(hipMallocAsync((void**)&scratch, bytes, st));
    X.keys = (azg::MoveKey*)scratch;
    long long* base = (long long*)(scratch + G * MM * sizeof(azg::MoveKey));
    X.base = base;
    X.status = (int32_t*)(base + G);
    X.zplayer = X.status + G;
    X.zval = (float*)(X.zplayer + G);
    int rc = 0;
    std::vector<int32_t> status(G);
    std::vector<long long> hbase(G);
    long long total = 0;
    hipError_t he = ops.replay(X, st);
    if (he == hipSuccess) he = hipMemcpyAsync(status.data(), X.status, G * 4, hipMemcpyDeviceToHost, st);
    if (he == hipSuccess) he = hipStreamSynchronize(st);
    if (he != hipSuccess) {
        rc = fail(AZG_ERR_HIP, std::string("examples replay: ") + hipGetErrorString(he));
    } else {
        for (size_t g = 0; g < G && !rc; ++g) {
            if (status[g] < 0) rc = fail(AZG_ERR_ARG, "move record " + std::to_string(g) + " is not a legal game");
            hbase[g] = total;
            total += (long long)ops.nsym * (status[g] > 0 ? status[g] : 0);
        }
    }
    if (!rc) {
        // deque(maxlen) keeps the last maxlen examples (Coach.py:107)
        X.skip = total > maxlen ? total - maxlen : 0;
        int g0 = 0;
        while (g0 < (int)G && hbase[g0] + (long long)ops.nsym * (status[g0] > 0 ? status[g0] : 0) <= X.skip) ++g0;
        X.g0 = g0;
        he = hipMemcpyAsync(base, hbase.data(), G * 8, hipMemcpyHostToDevice, st);
        if (he == hipSuccess) he = ops.emit(X, st);
        if (he == hipSuccess) he = hipStreamSynchronize(st);  // hbase must outlive the copy
        if (he != hipSuccess) rc = fail(AZG_ERR_HIP, std::string("examples emit: ") + hipGetErrorString(he));
        else *count = total - X.skip;
    }
    hipError_t fe = hipFreeAsync(scratch, st);
    if (!rc && fe != hipSuccess) rc = fail(AZG_ERR_HIP, std::string("hipFreeAsync: ") + hipGetErrorString(fe));
    return rc;
}

}  // extern "C"
