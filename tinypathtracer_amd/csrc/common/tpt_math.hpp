// tpt_math.hpp -- float math of the hot path, host + device.
//
// Every operation keeps the reference's evaluation order so the HIP kernels
// round exactly where the reference rounds (the library is built with
// -ffp-contract=off and correctly rounded fp32 div/sqrt):
//   include/math/vec.h:73-192, include/math/mat.h:37-51,
//   include/geometry_queries.h:18-86.
#pragma once

#include <stdint.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstring>
#define TPT_HD __host__ __device__ __forceinline__
#else
#include <cmath>
#include <cstring>
#define TPT_HD inline
#endif

namespace tpt {

constexpr float kPi = 3.141592653589793f;       // vec.h:66
constexpr float kDelta = 2e-4f;                  // vec.h:70
constexpr float kRealMax = 3.402823466e+38f;     // FLT_MAX (vec.h:61)

struct V3 {
    float x, y, z;
};

TPT_HD V3 v3(float x, float y, float z) { return V3{x, y, z}; }
TPT_HD V3 operator+(V3 a, V3 b) { return V3{a.x + b.x, a.y + b.y, a.z + b.z}; }
TPT_HD V3 operator-(V3 a, V3 b) { return V3{a.x - b.x, a.y - b.y, a.z - b.z}; }
TPT_HD V3 operator-(V3 a) { return V3{-a.x, -a.y, -a.z}; }
TPT_HD V3 operator*(V3 a, V3 b) { return V3{a.x * b.x, a.y * b.y, a.z * b.z}; }
// Real * Vec3 == Vec3 * Real (IEEE products commute), vec.h:140-141
TPT_HD V3 operator*(float s, V3 a) { return V3{s * a.x, s * a.y, s * a.z}; }
// Vec3 / Real == (1 / rhs) * lhs, vec.h:143
TPT_HD V3 vdiv(V3 a, float s) { return (1.0f / s) * a; }
TPT_HD float dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
TPT_HD float norm2(V3 a) { return a.x * a.x + a.y * a.y + a.z * a.z; }
TPT_HD V3 cross(V3 l, V3 r) {
    return V3{l.y * r.z - l.z * r.y, l.z * r.x - l.x * r.z, l.x * r.y - l.y * r.x};
}
// template max/min/clamp (vec.h:73-78): plain ternaries, NaN behaviour as written
TPT_HD float fmx(float x, float y) { return x > y ? x : y; }
TPT_HD float fmn(float x, float y) { return x < y ? x : y; }
TPT_HD float fclamp(float x, float hi, float lo) { return fmx(fmn(x, hi), lo); }
TPT_HD float fsat(float x) { return fclamp(x, 1.0f, 0.0f); }
TPT_HD float fsq(float x) { return x * x; }
TPT_HD V3 vmin(V3 a, V3 b) { return V3{fmn(a.x, b.x), fmn(a.y, b.y), fmn(a.z, b.z)}; }
TPT_HD V3 vmax(V3 a, V3 b) { return V3{fmx(a.x, b.x), fmx(a.y, b.y), fmx(a.z, b.z)}; }

TPT_HD int32_t f2i_bits(float f) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __float_as_int(f);
#else
    int32_t i;
    std::memcpy(&i, &f, 4);
    return i;
#endif
}
TPT_HD float i2f_bits(int32_t i) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __int_as_float(i);
#else
    float f;
    std::memcpy(&f, &i, 4);
    return f;
#endif
}

// Quake inverse sqrt with one Newton step (vec.h:25-38)
TPT_HD float frsqrt(float num) {
    float x2 = num * 0.5f;
    float y = i2f_bits(0x5f3759df - (f2i_bits(num) >> 1));
    return y * (1.5f - (x2 * y * y));
}
TPT_HD V3 normalize(V3 v) { return frsqrt(norm2(v)) * v; }

TPT_HD float fsqrt(float x) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_sqrtf(x);   // correctly rounded (-fhip-fp32-correctly-rounded-divide-sqrt)
#else
    return std::sqrt(x);
#endif
}
TPT_HD float fabs_(float x) { return __builtin_fabsf(x); }   // std::abs(float)

// Column-major Mat4 * Vec4 (mat.h:37-51): r[i] = sum_j m[j][i] * v[j], from 0
TPT_HD void mat4_vec4(const float* m, float v0, float v1, float v2, float v3_, float* r) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        float acc = 0.0f;
        acc += m[i] * v0;
        acc += m[4 + i] * v1;
        acc += m[8 + i] * v2;
        acc += m[12 + i] * v3_;
        r[i] = acc;
    }
}

// Transcendentals: (float) f((double) x).  The reference calls CUDA's fp32
// sinf/cosf/acosf/atan2f/tanf (<= 2 ulp); rounding the double-precision
// result gives the correctly rounded value in all but ~2^-29 of inputs and is
// evaluated identically by the CPU oracle (trig_mode 1).
TPT_HD float psin(float x) { return (float)sin((double)x); }
TPT_HD float pcos(float x) { return (float)cos((double)x); }
TPT_HD float pacos(float x) { return (float)acos((double)x); }
TPT_HD float patan2(float y, float x) { return (float)atan2((double)y, (double)x); }
TPT_HD float ptan(float x) { return (float)tan((double)x); }

}  // namespace tpt
