// tri_rec.hpp -- the leaf triangle record (`tri`).
//
// Leaf slot j holds rayHitTriangle's operands (geometry_queries.h:65-86) for the
// triangle at sorted position j: v0, e1 = v1 - v0, e2 = v2 - v0 (pre-subtracted,
// the same rounding) and the face id.  Default: three float4 at byte 48 j,
//   (v0.xyz, bits(fid)) (e1.xyz, 0) (e2.xyz, 0).
// TPT_TRI40=1 (A/B build): 10 floats at byte 40 j,
//   (v0.x, v0.y, v0.z, bits(fid)) (e1.x, e1.y, e1.z, e2.x) (e2.y, e2.z),
// read as two 16-byte and one 8-byte load (8-byte aligned): 17 % fewer bytes
// for the leaf tests of a scene larger than an XCD's L2 to re-read.  Measured
// (round 5, 2 interleaved reps): C5 +0.3 %, C2 -0.6 %, C4 within noise -- the
// triangle bytes are not what C5 waits on, so the aligned records stay.
#pragma once

#include <hip/hip_runtime.h>
#include <stddef.h>

#ifndef TPT_TRI40
#define TPT_TRI40 0
#endif

namespace tpt {

constexpr int kTriFloats = TPT_TRI40 ? 10 : 12;

// float4 units that hold n records
constexpr size_t tri_float4s(size_t n) { return (n * (size_t)kTriFloats + 3) / 4; }

// the record as rayHitTriangle's operands: q0 = (v0, bits(fid)), q1.xyz = e1, q2.xyz = e2
struct TriQ {
    float4 q0, q1, q2;
};

__device__ __forceinline__ TriQ tri_load(const float4* __restrict__ tri, int pos) {
    if constexpr (TPT_TRI40) {
        typedef float f4a8 __attribute__((ext_vector_type(4), aligned(8)));
        typedef float f2 __attribute__((ext_vector_type(2)));
        const float* p = reinterpret_cast<const float*>(tri) + 10 * (size_t)pos;
        const f4a8 a = *reinterpret_cast<const f4a8*>(p);
        const f4a8 b = *reinterpret_cast<const f4a8*>(p + 4);
        const f2 c = *reinterpret_cast<const f2*>(p + 8);
        return TriQ{make_float4(a.x, a.y, a.z, a.w), make_float4(b.x, b.y, b.z, 0.0f), make_float4(b.w, c.x, c.y, 0.0f)};
    } else {
        const float4* t = tri + 3 * (size_t)pos;
        return TriQ{t[0], t[1], t[2]};
    }
}

__device__ __forceinline__ void tri_store(float4* tri, int pos, float v0x, float v0y, float v0z, int fid, float e1x,
                                          float e1y, float e1z, float e2x, float e2y, float e2z) {
    if constexpr (TPT_TRI40) {
        float* p = reinterpret_cast<float*>(tri) + 10 * (size_t)pos;
        const float w[10] = {v0x, v0y, v0z, __int_as_float(fid), e1x, e1y, e1z, e2x, e2y, e2z};
#pragma unroll
        for (int k = 0; k < 10; ++k) p[k] = w[k];
    } else {
        float4* t = tri + 3 * (size_t)pos;
        t[0] = make_float4(v0x, v0y, v0z, __int_as_float(fid));
        t[1] = make_float4(e1x, e1y, e1z, 0.0f);
        t[2] = make_float4(e2x, e2y, e2z, 0.0f);
    }
}

}  // namespace tpt
