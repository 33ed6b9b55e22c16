// rng.hip -- per-pixel XORWOW initialisation (setupRandSeed, path_tracer.cu:34-40).
//
// curand_init(seed, subsequence = pixel index x + y*W, offset 0): salted seed
// words, then subsequence * 2^67 draws skipped by applying the GF(2) jump
// matrices J_k = A^(2^67 * 4^k) once per unit of the k-th base-4 digit.  The
// matrix rows are wave-uniform, so they stream through the scalar cache while
// each lane folds them into its own 160-bit state.
#include <hip/hip_runtime.h>

#include "../common/device_api.hpp"
#include "../common/rng.hpp"

namespace tpt {

__device__ __forceinline__ void jump_apply(const uint32_t* __restrict__ m, uint32_t v[5]) {
    uint32_t a0 = 0, a1 = 0, a2 = 0, a3 = 0, a4 = 0;
#pragma unroll
    for (int w = 0; w < 5; ++w) {
        const uint32_t word = v[w];
#pragma unroll 8
        for (int b = 0; b < 32; ++b) {
            const uint32_t mask = 0u - ((word >> b) & 1u);
            const uint32_t* row = m + (w * 32 + b) * 5;
            a0 ^= row[0] & mask;
            a1 ^= row[1] & mask;
            a2 ^= row[2] & mask;
            a3 ^= row[3] & mask;
            a4 ^= row[4] & mask;
        }
    }
    v[0] = a0; v[1] = a1; v[2] = a2; v[3] = a3; v[4] = a4;
}

__device__ void xorwow_init_device(const uint32_t* __restrict__ jumps, uint64_t seed, uint64_t subseq,
                                   uint32_t st[6]) {
    xorwow_seed(seed, st);
    for (int k = 0; k < kRngJumps && subseq; ++k) {
        const uint32_t digit = (uint32_t)(subseq & 3u);
        for (uint32_t i = 0; i < digit; ++i) jump_apply(jumps + k * kJumpWords, st);
        subseq >>= 2;
    }
}

__global__ __launch_bounds__(256) void k_rng_init(const uint32_t* __restrict__ jumps, uint64_t seed,
                                                  int32_t width, int32_t band_rows, int32_t band_count,
                                                  int32_t band_index, const int32_t* __restrict__ band_list,
                                                  int32_t band_height, int32_t height,
                                                  uint32_t* __restrict__ rng) {
    const int x = blockIdx.x * 64 + (threadIdx.x & 63);
    const int ly = blockIdx.y * 4 + (threadIdx.x >> 6);
    if (x >= width || ly >= band_height) return;
    // (trace_dev.hpp band_row: the interleaved deal, or an explicit band list)
    const int lb = ly / band_rows;
    const int y = (band_list ? band_list[lb] : lb * band_count + band_index) * band_rows + (ly % band_rows);
    if (y >= height) return;
    const size_t npix = (size_t)width * (size_t)height;
    const size_t off = (size_t)x + (size_t)y * (size_t)width;
    uint32_t st[6];
    xorwow_init_device(jumps, seed, (uint64_t)off, st);
#pragma unroll
    for (int i = 0; i < 6; ++i) rng[i * npix + off] = st[i];
}

__global__ void k_rng_init_linear(const uint32_t* __restrict__ jumps, uint64_t seed, uint64_t first, uint32_t n,
                                  uint32_t* __restrict__ out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint32_t st[6];
    xorwow_init_device(jumps, seed, first + i, st);
#pragma unroll
    for (int k = 0; k < 6; ++k) out[6 * (size_t)i + k] = st[k];
}

hipError_t launch_rng_init(const uint32_t* jumps, uint64_t seed, int32_t width, int32_t band_rows,
                           int32_t band_count, int32_t band_index, const int32_t* band_list, int32_t band_height,
                           int32_t height, uint32_t* rng, hipStream_t s) {
    dim3 grid((width + 63) / 64, (band_height + 3) / 4);
    hipLaunchKernelGGL(k_rng_init, grid, dim3(256), 0, s, jumps, seed, width, band_rows, band_count, band_index,
                       band_list, band_height, height, rng);
    return hipGetLastError();
}

hipError_t launch_rng_init_linear(const uint32_t* jumps, uint64_t seed, uint64_t first, uint32_t n,
                                  uint32_t* states_aos, hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_rng_init_linear, dim3((n + 255) / 256), dim3(256), 0, s, jumps, seed, first, n, states_aos);
    return hipGetLastError();
}

}  // namespace tpt
