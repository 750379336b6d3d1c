// azg_launch.h -- host launchers of the engine kernels (azg_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>

#include "azg_engine.h"

namespace azg {
hipError_t launch_select(const Dev& E, float* planes, hipStream_t st);
hipError_t launch_stub_eval(const Dev& E, const float* planes, float* P, float* v, hipStream_t st);
hipError_t launch_expand_backup(const Dev& E, const float* P, int p_stride, const float* v, hipStream_t st);
hipError_t launch_move_end(const Dev& E, hipStream_t st);
hipError_t launch_root_counts(const Dev& E, int g, int32_t* out, hipStream_t st);
hipError_t launch_reset(const Dev& E, uint32_t seed_base, long long first_game, hipStream_t st);
hipError_t launch_summary(const Dev& E, int32_t* out, hipStream_t st);
hipError_t launch_stats(const Dev& E, long long* out, hipStream_t st);
}  // namespace azg
