// azg_launch.h -- host launchers of the engine kernels (azg_kernels.hip).
//
// The search kernels are instantiated per game (Inflexion 7x7, Othello 6x6 /
// 8x8); azg_create picks one GameOps table and every later call dispatches
// through it.
#pragma once
#include <hip/hip_runtime.h>

#include "azg_engine.h"

namespace azg {

// root key + player of one recorded move (examples pipeline)
struct MoveKey {
    uint64_t own, opp;
    int32_t kt;  // turn (Inflexion) / disc count (Othello)
    int32_t cp;  // bit0 can_spawn, bit1 player to move is RED (+1)
};

// arguments of the replay / emit kernels (azg_examples)
struct ExampleArgs {
    int G, MM, max_turns, temp_threshold, label_mode, g0;
    const int32_t* moves;     // [G]
    const int32_t* actions;   // [G*MM]
    const int16_t* counts16;  // [G*CR*A] (one of the two)
    const int32_t* counts32;
    int CR;                   // count rows per game (<= MM: moves from CR on are read as zero counts)
    MoveKey* keys;            // [G*MM] scratch
    int32_t* status;          // [G]
    float* zval;              // [G]
    int32_t* zplayer;         // [G]
    const long long* base;    // [G] first example index of each game
    long long skip;           // examples before the kept window
    float* planes;            // [maxlen, PLANES*CELLS]
    float* pis;               // [maxlen, A]
    float* vs;                // [maxlen]
};

// arguments of the refill kernel (azg_refill, continuous batching)
struct RefillArgs {
    unsigned long long* next_game;  // device counter: next global game index to start
    long long end_game;             // games below end_game are started / handed off
    uint32_t seed_base;
    unsigned long long* count;      // device counter: games handed off so far
    long long cap;                  // rows of the completed-game buffers
    int64_t* ids;                   // [cap]
    int32_t* moves;                 // [cap]
    int32_t* actions;               // [cap * max_moves]
    int8_t* temps;                  // [cap * max_moves]
    int32_t* counts;                // [cap * max_moves * A] or null
};

struct GameOps {
    int cells;    // board cells (lanes in use)
    int actions;  // A = max_actions
    int row;      // per-node action stride (A rounded up to 64)
    int planes;   // NN input planes per cell
    int nsym;     // forms in game.symmetries()
    hipError_t (*select)(const Dev&, float* planes, hipStream_t);
    hipError_t (*stub_eval)(const Dev&, const float* planes, float* P, float* v, hipStream_t);
    hipError_t (*expand_backup)(const Dev&, const float* P, int p_stride, const float* v, hipStream_t);
    hipError_t (*move_end)(const Dev&, hipStream_t);
    hipError_t (*expand_select)(const Dev&, const float* P, int p_stride, const float* v, float* planes,
                                hipStream_t);
    hipError_t (*root_counts)(const Dev&, int g, int32_t* out, hipStream_t);
    hipError_t (*slot_begin)(const Dev&, int g, const int32_t* in, hipStream_t);
    hipError_t (*slot_end)(const Dev&, int g, int32_t* out, hipStream_t);
    hipError_t (*reset)(const Dev&, uint32_t seed_base, long long first_game, hipStream_t);
    hipError_t (*refill)(const Dev&, const RefillArgs&, hipStream_t);
    hipError_t (*opponent)(const Dev&, int kind, hipStream_t);
    hipError_t (*follow)(const Dev&, const Dev& leader, hipStream_t);
    hipError_t (*replay)(const ExampleArgs&, hipStream_t);
    hipError_t (*emit)(const ExampleArgs&, hipStream_t);
};

// kind: AZG_GAME_INFLEXION (n = 7) or AZG_GAME_OTHELLO (n = 6, 8)
bool game_ops(int kind, int n, GameOps* out);

hipError_t launch_summary(const Dev& E, int32_t* out, hipStream_t st);
hipError_t launch_stats(const Dev& E, long long* out, hipStream_t st);
}  // namespace azg
