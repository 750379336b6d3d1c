// azg_ptr.h -- boundary check for flags the kernels set with device atomics.
#pragma once
#include <hip/hip_runtime.h>

namespace {
// true if the GPU may write p with a device atomic: device (or managed) memory.  The
// Winograd transforms and FC epilogues set the caller's range flag this way the first
// time an operand leaves fp16's range; a pageable host pointer there would fault the
// GPU at that moment, so the C ABI rejects it up front.  The last 8 accepted pointers are
// remembered per thread (one attribute query per new flag, not per launch, also when several
// networks -- the arena's two, the multi-stream engines' -- alternate).
inline bool azg_device_writable(const void* p) {
    constexpr int NCACHE = 8;
    static thread_local const void* ok_ring[NCACHE] = {};
    static thread_local unsigned next = 0;
    if (!p) return false;
    for (int i = 0; i < NCACHE; ++i)
        if (ok_ring[i] == p) return true;
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();  // clear the query's own error
        return false;
    }
    const bool ok = a.type == hipMemoryTypeDevice || a.type == hipMemoryTypeManaged;
    if (ok) ok_ring[next++ % NCACHE] = p;
    return ok;
}
}  // namespace
