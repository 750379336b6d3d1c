// azg_ptr.h -- boundary check for flags the kernels set with device atomics.
#pragma once
#include <hip/hip_runtime.h>

namespace {
// true if the GPU may write p with a device atomic: device (or managed) memory.  The
// Winograd transforms and FC epilogues set the caller's range flag this way the first
// time an operand leaves fp16's range; a pageable host pointer there would fault the
// GPU at that moment, so the C ABI rejects it up front.  The last accepted pointer is
// remembered (one attribute query per new flag, not per launch).
inline bool azg_device_writable(const void* p) {
    static thread_local const void* last_ok = nullptr;
    if (!p) return false;
    if (p == last_ok) return true;
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();  // clear the query's own error
        return false;
    }
    const bool ok = a.type == hipMemoryTypeDevice || a.type == hipMemoryTypeManaged;
    if (ok) last_ok = p;
    return ok;
}
}  // namespace
