// ptrig.hpp -- the transcendentals of the hot path ("parity trig").
//
// The reference calls CUDA's fp32 sinf/cosf/atan2f/acosf (<= 2 ulp, not
// reproducible off NVIDIA hardware).  This build fixes one evaluation that the
// HIP kernel and the CPU oracle (trig_mode 1) perform bit-identically:
//  * sin/cos of the diffuse sampler's phi (per bounce, hot): fsincos_2pi, an
//    all-fp32 Cody-Waite + minimax evaluation with explicit fmaf, <= 1 ulp;
//  * atan2/acos of the env lookup (cold): (float) of a double evaluation
//    (fdlibm-style kernels below, < 1 ulp of double), which equals the oracle's
//    (float)atan2((double)..) from libm except within ~2^-29 of a float
//    rounding boundary.  tests/test_cpu_math.py measures both.
#pragma once

#include "tpt_math.hpp"

namespace tpt {

TPT_HD double dfma(double a, double b, double c) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_fma(a, b, c);
#else
    return std::fma(a, b, c);
#endif
}

// sin and cos of x, |x| <= ~8 (phi in (0, 2*pi])
TPT_HD void dsincos_small(double x, double& s, double& c) {
    const double kInvPio2 = 6.36619772367581382433e-01;
    const double kPio2_1 = 1.57079632673412561417e+00;    // first 33 bits of pi/2
    const double kPio2_1t = 6.07710050650619224932e-11;   // pi/2 - kPio2_1
    const double kd = rint(x * kInvPio2);
    const int q = (int)kd & 3;
    const double r = (x - kd * kPio2_1) - kd * kPio2_1t;
    const double z = r * r;
    // sin kernel (|r| <= pi/4)
    double ps = dfma(z, 1.58969099521155010221e-10, -2.50507602534068634195e-08);
    ps = dfma(z, ps, 2.75573137070700676789e-06);
    ps = dfma(z, ps, -1.98412698298579493134e-04);
    ps = dfma(z, ps, 8.33333333332248946124e-03);
    ps = dfma(z, ps, -1.66666666666666324348e-01);
    const double sr = dfma(r * z, ps, r);
    // cos kernel
    double pc = dfma(z, -1.13596475577881948265e-11, 2.08757232129817482790e-09);
    pc = dfma(z, pc, -2.75573143513906633035e-07);
    pc = dfma(z, pc, 2.48015872894767294178e-05);
    pc = dfma(z, pc, -1.38888888888741095749e-03);
    pc = dfma(z, pc, 4.16666666666666019037e-02);
    const double hz = 0.5 * z;
    const double w = 1.0 - hz;
    const double cr = w + (((1.0 - w) - hz) + z * z * pc);
    switch (q) {
        case 0: s = sr; c = cr; break;
        case 1: s = cr; c = -sr; break;
        case 2: s = -sr; c = -cr; break;
        default: s = -cr; c = sr; break;
    }
}

// atan(t) for t >= 0 (fdlibm s_atan.c reduction + polynomial)
TPT_HD double datan_pos(double t) {
    double hi = 0.0, lo = 0.0;
    int id;
    if (t < 0.4375) {
        id = -1;
    } else if (t < 1.1875) {
        if (t < 0.6875) { id = 0; t = (2.0 * t - 1.0) / (2.0 + t); }
        else { id = 1; t = (t - 1.0) / (t + 1.0); }
    } else if (t < 2.4375) {
        id = 2; t = (t - 1.5) / (1.0 + 1.5 * t);
    } else {
        id = 3; t = -1.0 / t;
    }
    if (id == 0) { hi = 4.63647609000806093515e-01; lo = 2.26987774529616870924e-17; }
    if (id == 1) { hi = 7.85398163397448278999e-01; lo = 3.06161699786838301793e-17; }
    if (id == 2) { hi = 9.82793723247329054082e-01; lo = 1.39033110312309984516e-17; }
    if (id == 3) { hi = 1.57079632679489655800e+00; lo = 6.12323399573676603587e-17; }
    const double z = t * t;
    const double w = z * z;
    double s1 = dfma(w, 1.62858201153657823623e-02, 4.97687799461593236017e-02);
    s1 = dfma(w, s1, 6.66107313738753120669e-02);
    s1 = dfma(w, s1, 9.09088713343650656196e-02);
    s1 = dfma(w, s1, 1.42857142725034663711e-01);
    s1 = dfma(w, s1, 3.33333333333329318027e-01);
    s1 = z * s1;
    double s2 = dfma(w, -3.65315727442169155270e-02, -5.83357013379057348645e-02);
    s2 = dfma(w, s2, -7.69187620504482999495e-02);
    s2 = dfma(w, s2, -1.11111104054623557880e-01);
    s2 = dfma(w, s2, -1.99999999998764832476e-01);
    s2 = w * s2;
    if (id < 0) return t - t * (s1 + s2);
    return hi - ((t * (s1 + s2) - lo) - t);
}

TPT_HD double datan2(double y, double x) {
    const double kPi = 3.1415926535897931160e+00, kPiLo = 1.2246467991473531772e-16;
    if (x != x || y != y) return x + y;
    const double ax = x < 0.0 ? -x : x, ay = y < 0.0 ? -y : y;
    const bool yneg = __builtin_signbit(y);
    if (ay == 0.0) {   // atan2(+-0, x): +-0 for x > 0 or +0, +-pi for x < 0 or -0
        if (__builtin_signbit(x)) return yneg ? -kPi : kPi;
        return y;
    }
    if (ax == 0.0) return yneg ? -1.57079632679489655800e+00 : 1.57079632679489655800e+00;
    double a;
    if (ax == ay && ax > 1.0e308) a = 7.85398163397448278999e-01;   // inf/inf
    else a = datan_pos(ay / ax);
    if (x < 0.0) a = (kPi - (a - kPiLo));
    return yneg ? -a : a;
}

TPT_HD double dacos(double y) {
    if (y != y || y > 1.0 || y < -1.0) return (y - y) / (y - y);
    return datan2(sqrt((1.0 - y) * (1.0 + y)), y);
}

TPT_HD float ffma(float a, float b, float c) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_fmaf(a, b, c);
#else
    return std::fma(a, b, c);
#endif
}

// fp32 sin and cos of x in [0, 2*pi] (the diffuse sampler's phi = 2*pi*u,
// sampler.h:81).  Cody-Waite reduction by pi/2 in three parts and minimax
// polynomials on [-pi/4, pi/4]; every step is an explicit, correctly rounded
// fmaf / mul / add, so the CPU oracle (trig_mode 1, tpt_oracle.c) evaluates the
// very same bits.  Max error <= 1 ulp against the correctly rounded sin/cos
// (tests/test_cpu_math.py), the accuracy class of CUDA's sinf/cosf.
TPT_HD void fsincos_2pi(float x, float& s, float& c) {
    const float k = rintf(x * 0.636619772f);
    const int q = (int)k & 3;
    float r = ffma(-k, 1.57079637f, x);          // pi/2 = 1.57079637 - 4.37113883e-8 + ...
    r = ffma(-k, -4.37113883e-08f, r);
    r = ffma(-k, -1.71512489e-15f, r);
    const float z = r * r;
    float ps = ffma(z, 2.71808875e-06f, -1.98393362e-04f);
    ps = ffma(z, ps, 8.33332464e-03f);
    ps = ffma(z, ps, -1.66666657e-01f);
    const float sr = ffma(r * z, ps, r);
    float pc = ffma(z, 2.43904487e-05f, -1.38867637e-03f);
    pc = ffma(z, pc, 4.16666418e-02f);
    pc = ffma(z, pc, -0.5f);
    const float cr = ffma(z, pc, 1.0f);
    switch (q) {
        case 0: s = sr; c = cr; break;
        case 1: s = cr; c = -sr; break;
        case 2: s = -sr; c = -cr; break;
        default: s = -cr; c = sr; break;
    }
}

// Parity trig for the hot path (see tpt_math.hpp psin/pcos/...).
TPT_HD void psincos2pi(float phi, float& s, float& c) {
    double ds, dc;
    dsincos_small((double)phi, ds, dc);
    s = (float)ds;
    c = (float)dc;
}
TPT_HD float patan2_fast(float y, float x) { return (float)datan2((double)y, (double)x); }
TPT_HD float pacos_fast(float y) { return (float)dacos((double)y); }

// ---------------------------------------------------------------------------
// The env lookup's texel indices without the double evaluation where it cannot
// matter.  The lookup (env_light.cuh:72-78 via Vec2UV) only keeps
//   ix = clamp(floor(fl(u * w))), u = fl(A / fl(2 pi)) (+ 1 when < 0), A = (float)atan2_d(z, x)
//   iy = clamp(floor(fl(v * h))), v = 1 - fl(C / pi),                  C = (float)acos_d(y)
// and every step after A (or C) is monotonic in it (IEEE rounding is monotonic;
// the +1 only applies on one side of 0).  An fp32 approximation a with
// |a - A| <= kEnvTrigBound puts A in [a - bound, a + bound]; when both ends of
// that interval give the same index (and the same side of u = 0), so does A,
// exactly.  Otherwise (about 0.1 % of lookups: within ~1e-3 of a texel edge)
// the caller evaluates the double path.  tests/test_cpu_math.py measures the
// approximations' error (< 4e-7 rad) against the 4e-6 bound and checks the
// indices against the double path on adversarial and random directions.
constexpr float kEnvTrigBound = 4.0e-6f;

// atan(t) for t in [0, 1] (Cephes atanf reduction at tan(pi/8) and minimax
// polynomial; every step an explicit fmaf, mul or correctly rounded divide)
TPT_HD float fatan01(float t) {
    float off = 0.0f;
    if (t > 0.414213562f) {
        t = (t - 1.0f) / (t + 1.0f);
        off = 0.785398163f;
    }
    const float z = t * t;
    float p = ffma(z, 8.05374449538e-2f, -1.38776856032e-1f);
    p = ffma(z, p, 1.99777106478e-1f);
    p = ffma(z, p, -3.33329491539e-1f);
    return off + ffma(p * z, t, t);
}
// atan2(y, x) for finite y, x with max(|x|, |y|) >= 1e-18 (else: no bound claimed)
TPT_HD float fatan2_approx(float y, float x) {
    const float ax = x < 0.0f ? -x : x, ay = y < 0.0f ? -y : y;
    const float mx = ax > ay ? ax : ay, mn = ax > ay ? ay : ax;
    float a = fatan01(mn / mx);
    if (ay > ax) a = 1.57079633f - a;
    if (x < 0.0f) a = 3.14159265f - a;
    return __builtin_signbit(y) ? -a : a;   // atan2(-0, x < 0) = -pi
}
TPT_HD bool env_fast_ok(float v) { return v == v && v - v == 0.0f; }   // finite

// The lookup's column of direction (x, z) in a w-texel row, or -1 if undecided.
TPT_HD int env_col_fast(float z, float x, int w) {
    const float ax = x < 0.0f ? -x : x, az = z < 0.0f ? -z : z;
    if (!env_fast_ok(x) || !env_fast_ok(z) || !((ax > az ? ax : az) >= 1e-18f)) return -1;
    const float a = fatan2_approx(z, x);
    float ul = (a - kEnvTrigBound) / (2.0f * kPi), uh = (a + kEnvTrigBound) / (2.0f * kPi);
    if ((ul < 0.0f) != (uh < 0.0f)) return -1;
    if (ul < 0.0f) {
        ul += 1.0f;
        uh += 1.0f;
    }
    int il = (int)floorf(ul * (float)w), ih = (int)floorf(uh * (float)w);
    il = il < 0 ? 0 : (il > w - 1 ? w - 1 : il);
    ih = ih < 0 ? 0 : (ih > w - 1 ? w - 1 : ih);
    return il == ih ? il : -1;
}
// The lookup's row of direction component y (clamped to [-1, 1]) in h rows, or -1.
TPT_HD int env_row_fast(float y, int h) {
    if (!env_fast_ok(y)) return -1;
    const float c = y > 1.0f ? 1.0f : (y < -1.0f ? -1.0f : y);
    const float s = sqrtf((1.0f - c) * (1.0f + c));
    const float a = fatan2_approx(s, c);   // acos(c) = atan2(sqrt(1 - c^2), c), c = 0 included
    const float vh = 1.0f - (a - kEnvTrigBound) / kPi, vl = 1.0f - (a + kEnvTrigBound) / kPi;
    int il = (int)floorf(vl * (float)h), ih = (int)floorf(vh * (float)h);
    il = il < 0 ? 0 : (il > h - 1 ? h - 1 : il);
    ih = ih < 0 ? 0 : (ih > h - 1 ? h - 1 : ih);
    return il == ih ? il : -1;
}

}  // namespace tpt
