// Philox4x32-10 (Salmon et al., SC'11), host+device.
// Same algorithm and counter/key convention as oracle/philox.py; pinned by the
// Random123 known-answer vectors in tests/test_philox_kat.py.
//
// Layout draw (SURVEY.md App. A S14 [DECISION], replaces MPE's np.random in
// scenario.reset_world): counter = (entity, episode, global env id, TAG),
// key = (seed lo32, seed hi32); u = (x >> 8) * 2^-24 in [0,1).
#pragma once
#include <stdint.h>

#ifndef GSM_HD
#define GSM_HD __host__ __device__ __forceinline__
#endif

namespace gsm {

enum : uint32_t { kTagLayout = 0u, kTagActions = 1u, kTagShape = 2u };

struct Philox4 { uint32_t x0, x1, x2, x3; };

GSM_HD Philox4 philox4x32_10(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                             uint32_t k0, uint32_t k1) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        if (r) { k0 += 0x9E3779B9u; k1 += 0xBB67AE85u; }
        const uint64_t p0 = (uint64_t)0xD2511F53u * c0;
        const uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
        const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
        const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
        c0 = hi1 ^ c1 ^ k0;
        c1 = lo1;
        c2 = hi0 ^ c3 ^ k1;
        c3 = lo0;
    }
    return Philox4{c0, c1, c2, c3};
}

// (x >> 8) * 2^-24: exact in fp32.
GSM_HD float u01(uint32_t x) { return (float)(x >> 8) * 5.9604644775390625e-08f; }

}  // namespace gsm
