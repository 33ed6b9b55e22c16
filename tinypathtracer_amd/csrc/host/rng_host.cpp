// rng_host.cpp -- XORWOW jump matrices for curand_init's subsequence skip.
//
// One xorwow step is linear over GF(2) on the 160-bit state v0..v4 (the Weyl
// counter d is untouched by a 2^67-step jump: 2^67 * 362437 == 0 mod 2^32).
// J_0 = A^(2^67) by 67 squarings of the one-step matrix A, J_k = J_{k-1}^4.
// Row b of a matrix is the image of input bit b (word b/32, bit b%32).
#include <cstdint>
#include <cstring>
#include <vector>

#include "../common/rng.hpp"

namespace tpt {
namespace {

constexpr int kBits = 160, kWords = 5;

void apply(const uint32_t* m, const uint32_t* v, uint32_t* out) {
    uint32_t acc[kWords] = {0, 0, 0, 0, 0};
    for (int b = 0; b < kBits; ++b)
        if ((v[b >> 5] >> (b & 31)) & 1u)
            for (int k = 0; k < kWords; ++k) acc[k] ^= m[b * kWords + k];
    std::memcpy(out, acc, sizeof acc);
}

void compose(const uint32_t* m, const uint32_t* n, uint32_t* out) {   // out = m * n
    for (int b = 0; b < kBits; ++b) apply(m, n + b * kWords, out + b * kWords);
}

}  // namespace

void xorwow_jump_matrices(int count, uint32_t* out) {
    std::vector<uint32_t> a(kBits * kWords), t(kBits * kWords);
    for (int b = 0; b < kBits; ++b) {
        uint32_t st[6] = {0, 0, 0, 0, 0, 0};
        st[b >> 5] = 1u << (b & 31);
        xorwow_next(st);                       // d is ignored (linear part only)
        std::memcpy(&a[b * kWords], st, kWords * sizeof(uint32_t));
    }
    for (int s = 0; s < 67; ++s) {
        compose(a.data(), a.data(), t.data());
        a.swap(t);
    }
    for (int k = 0; k < count; ++k) {
        std::memcpy(out + (size_t)k * kBits * kWords, a.data(), a.size() * sizeof(uint32_t));
        compose(a.data(), a.data(), t.data());
        compose(t.data(), t.data(), a.data());
    }
}

}  // namespace tpt
