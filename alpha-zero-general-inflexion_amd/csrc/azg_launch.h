// azg_launch.h -- host launchers of the engine kernels (azg_kernels.hip).
//
// The search kernels are instantiated per game (Inflexion 7x7, Othello 6x6 /
// 8x8); azg_create picks one GameOps table and every later call dispatches
// through it.
#pragma once
#include <hip/hip_runtime.h>

#include "azg_engine.h"

namespace azg {

struct GameOps {
    int cells;    // board cells (lanes in use)
    int actions;  // A = max_actions
    int row;      // per-node action stride (A rounded up to 64)
    int planes;   // NN input planes per cell
    hipError_t (*select)(const Dev&, float* planes, hipStream_t);
    hipError_t (*stub_eval)(const Dev&, const float* planes, float* P, float* v, hipStream_t);
    hipError_t (*expand_backup)(const Dev&, const float* P, int p_stride, const float* v, hipStream_t);
    hipError_t (*move_end)(const Dev&, hipStream_t);
    hipError_t (*root_counts)(const Dev&, int g, int32_t* out, hipStream_t);
    hipError_t (*reset)(const Dev&, uint32_t seed_base, long long first_game, hipStream_t);
};

// kind: AZG_GAME_INFLEXION (n = 7) or AZG_GAME_OTHELLO (n = 6, 8)
bool game_ops(int kind, int n, GameOps* out);

hipError_t launch_summary(const Dev& E, int32_t* out, hipStream_t st);
hipError_t launch_stats(const Dev& E, long long* out, hipStream_t st);
}  // namespace azg
