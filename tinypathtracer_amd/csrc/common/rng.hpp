// rng.hpp -- cuRAND-compatible XORWOW (host + device).
//
// The reference draws every random number through curand_uniform on a
// per-pixel curandStateXORWOW (include/sampler.h:12-15, path_tracer.cu:34-40).
// cuRAND is not vendored in the reference; this restates its published
// generator: Marsaglia xorwow (5 x 32-bit xorshift words + Weyl counter d,
// step 362437), seed salting, 2^67-draw subsequences, and
// curand_uniform(x) = x * 2^-32 + 2^-33 in fp32 (range (0, 1]).
#pragma once

#include <stdint.h>

#include "tpt_math.hpp"

namespace tpt {

TPT_HD void xorwow_seed(uint64_t seed, uint32_t st[6]) {
    const uint32_t s0 = ((uint32_t)seed) ^ 0xaad26b49u;
    const uint32_t s1 = ((uint32_t)(seed >> 32)) ^ 0xf7dcefddu;
    const uint32_t t0 = 1099087573u * s0;
    const uint32_t t1 = 2591861531u * s1;
    st[0] = 123456789u + t0;
    st[1] = 362436069u ^ t0;
    st[2] = 521288629u + t1;
    st[3] = 88675123u ^ t1;
    st[4] = 5783321u + t0;
    st[5] = 6615241u + t1 + t0;   // Weyl counter d
}

TPT_HD uint32_t xorwow_next(uint32_t st[6]) {
    const uint32_t t = st[0] ^ (st[0] >> 2);
    st[0] = st[1];
    st[1] = st[2];
    st[2] = st[3];
    st[3] = st[4];
    st[4] = (st[4] ^ (st[4] << 4)) ^ (t ^ (t << 1));
    st[5] += 362437u;
    return st[4] + st[5];
}

TPT_HD float xorwow_uniform(uint32_t st[6]) {
    return (float)xorwow_next(st) * 2.3283064e-10f + (2.3283064e-10f / 2.0f);
}

// Jump matrices J_k = A^(2^67 * 4^k), k < n: row b (input bit b) = 5 words (host).
void xorwow_jump_matrices(int n, uint32_t* out);

}  // namespace tpt
