// azg_host.cpp -- host-side helpers of the learn loop (no device code).
//
// azg_py_shuffle: Coach.learn's `shuffle(trainExamples)` (Coach.py:149, Python's random.shuffle)
// over a steady-state history of 20 windows x 200,000 examples (main.py:19,27) costs ~1.8 s of
// interpreter time per iteration plus ~0.4 s to turn the shuffled list into an index tensor.
// This restates the interpreter's algorithm on the MT19937 state of its `random` module
// (random.getstate()), so the permutation and the stream position afterwards are the ones
// random.shuffle(list(range(n))) gives:
//   Lib/random.py  shuffle:  for i in reversed(range(1, len(x))): j = _randbelow(i + 1); swap
//                  _randbelow_with_getrandbits(n): k = n.bit_length(); r = getrandbits(k)
//                                                  while r >= n: r = getrandbits(k)
//   Modules/_randommodule.c  getrandbits(k <= 32) = genrand_uint32() >> (32 - k)
// (tests/test_examples_file_cpu.py checks it against random.shuffle itself).
#include <cstdint>
#include <string>

#include "../../include/azg.h"

namespace {
constexpr int MT_N = 624, MT_M = 397;

struct MT {
    uint32_t* mt;
    int32_t idx;
    uint32_t next() {
        if (idx >= MT_N) {
            for (int k = 0; k < MT_N; ++k) {
                uint32_t y = (mt[k] & 0x80000000u) | (mt[(k + 1) % MT_N] & 0x7fffffffu);
                mt[k] = mt[(k + MT_M) % MT_N] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
            }
            idx = 0;
        }
        uint32_t y = mt[idx++];
        y ^= y >> 11;
        y ^= (y << 7) & 0x9d2c5680u;
        y ^= (y << 15) & 0xefc60000u;
        y ^= y >> 18;
        return y;
    }
};

int bit_length(uint64_t n) {
    int k = 0;
    while (n) {
        ++k;
        n >>= 1;
    }
    return k;
}
}  // namespace

int azg_host_fail(int code, const std::string& msg);  // azg_capi.cpp (thread-local message)

extern "C" int azg_py_shuffle(int64_t* x, int64_t n, uint32_t* mt, int32_t* pos) {
    if (n < 0 || (n > 0 && x == nullptr) || mt == nullptr || pos == nullptr)
        return azg_host_fail(AZG_ERR_ARG, "azg_py_shuffle: null pointer or negative length");
    if (n >= (int64_t(1) << 32))
        return azg_host_fail(AZG_ERR_ARG, "azg_py_shuffle: 2^32 or more elements (getrandbits above 32 bits)");
    if (*pos < 0 || *pos > MT_N) return azg_host_fail(AZG_ERR_ARG, "azg_py_shuffle: state index out of range");
    MT g{mt, *pos};
    for (int64_t i = n - 1; i >= 1; --i) {
        uint64_t m = uint64_t(i) + 1;
        int k = bit_length(m);
        uint64_t r;
        do {
            r = g.next() >> (32 - k);
        } while (r >= m);
        int64_t t = x[i];
        x[i] = x[r];
        x[r] = t;
    }
    *pos = g.idx;
    return AZG_OK;
}
