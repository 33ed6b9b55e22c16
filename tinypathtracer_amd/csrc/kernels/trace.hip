// trace.hip -- the per-pixel path-tracing megakernel (src/path_tracer.cu:296-435)
// and the framebuffer resolve (copyToFB, :451-471).
//
// MI355X design (DESIGN.md "Trace kernel"):
//  * one lane per pixel, 16x16 pixel tile per 256-thread workgroup, each wave an
//    8x8 sub-tile (coherent primary rays);
//  * the reference's nested spp -> depth -> {extension, shadow*, probe} loops are
//    flattened into a per-lane state machine that issues exactly ONE BVH
//    traversal per iteration from a single call site.  A lane whose path ends
//    immediately regenerates its next sample, so a wave stays full across
//    samples and bounces while every pixel still consumes its own XORWOW stream
//    in the reference's order;
//  * the traversal stack lives in LDS, [slot][lane] (conflict-free, sized to the
//    built tree's depth); the per-depth path records (attenuation, 1/p, direct)
//    are private arrays; RNG state and the running total live in registers and
//    are persisted to HBM (SoA) between spp chunks;
//  * node records are 64 B (both child AABBs + links: one visit = four 16-B
//    loads), triangles are pre-gathered (v0, e1, e2, fid: three 16-B loads).
#include <hip/hip_runtime.h>

#include "../common/device_api.hpp"
#include "../common/rng.hpp"
#include "../common/ptrig.hpp"
#include "../common/tpt_math.hpp"
#include "tpt.h"

namespace tpt {

struct Hit {
    int fid;
    float t, u, v;
};

// rayHitBBox (geometry_queries.h:18-46) with 1/dir hoisted per ray (same values).
// Returns the reference's hit/miss verdict and the slab interval [t0, t1] for
// the ordered traversal (NaN slabs propagate exactly as in the reference).
__device__ __forceinline__ bool box_hit(const V3& o, const V3& inv, float nx, float ny, float nz, float xx,
                                        float xy, float xz, float& t0, float& t1) {
    float a, b, s;
    t0 = -kRealMax;
    t1 = kRealMax;
    a = (nx - o.x) * inv.x;
    b = (xx - o.x) * inv.x;
    if (a > b) { s = b; b = a; a = s; }
    if (t0 > b || a > t1) return false;
    t0 = fmx(t0, a);
    t1 = fmn(t1, b);
    a = (ny - o.y) * inv.y;
    b = (xy - o.y) * inv.y;
    if (a > b) { s = b; b = a; a = s; }
    if (t0 > b || a > t1) return false;
    t0 = fmx(t0, a);
    t1 = fmn(t1, b);
    a = (nz - o.z) * inv.z;
    b = (xz - o.z) * inv.z;
    if (a > b) { s = b; b = a; a = s; }
    if (t0 > b || a > t1) return false;
    t0 = fmx(t0, a);
    t1 = fmn(t1, b);
    return true;
}

// traverseBVH (path_tracer.cu:61-107).  The current node stays in a register;
// the LDS stack ([slot][lane]) only holds deferred siblings.
//  ORDERED == false: the reference's order exactly (both children hit -> the
//    right child first, left deferred) -- same visit sequence as :95-104.
//  ORDERED == true: nearer child first and a child is skipped when its slab
//    entry lies beyond the best hit (with a 1e-4 relative margin) or its exit
//    lies before Delta/2: boxes that cannot hold an accepted hit.  Exact ties
//    (t == best) resolve to the larger leaf position, which is the triangle the
//    reference's right-first DFS finds first, so the winner is the reference's.
// any_hit: shadow rays stop at the first accepted triangle (only hitIdx == -1
// matters, :279).
template <bool ORDERED>
__device__ __forceinline__ Hit traverse(const float4* __restrict__ inner, const float4* __restrict__ tri, int nint,
                                        int* stk, int stack_depth, V3 o, V3 d, bool any_hit, uint32_t& c_inner,
                                        uint32_t& c_leaf, uint32_t& c_ovf) {
    const V3 inv = v3(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
    Hit h{-1, kRealMax, 0.0f, 0.0f};
    int hpos = -1;
    int sp = 0;
    int node = 0;
    for (;;) {
        if (node < nint) {
            ++c_inner;
            const float4* nd = inner + 4 * node;
            const float4 q0 = nd[0], q1 = nd[1], q2 = nd[2], q3 = nd[3];
            float l0, l1, r0, r1;
            bool hl = box_hit(o, inv, q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, l0, l1);
            bool hr = box_hit(o, inv, q1.z, q1.w, q2.x, q2.y, q2.z, q2.w, r0, r1);
            const int lc = __float_as_int(q3.x), rc = __float_as_int(q3.y);
            if (ORDERED) {
                const float lim = h.t * 1.0001f;
                hl = hl && !(l0 > lim) && !(l1 < 0.5f * kDelta);
                hr = hr && !(r0 > lim) && !(r1 < 0.5f * kDelta);
            }
            if (hl && hr) {
                int first = rc, second = lc;
                if (ORDERED && l0 < r0) { first = lc; second = rc; }
                if (sp >= stack_depth) { ++c_ovf; break; }
                stk[(sp++) * 256] = second;
                node = first;
                continue;
            }
            if (hl) { node = lc; continue; }
            if (hr) { node = rc; continue; }
        } else {
            ++c_leaf;
            const int pos = node - nint;
            const float4* tr = tri + 3 * pos;
            const float4 q0 = tr[0], q1 = tr[1], q2 = tr[2];
            const V3 v0 = v3(q0.x, q0.y, q0.z), e1 = v3(q1.x, q1.y, q1.z), e2 = v3(q2.x, q2.y, q2.z);
            const V3 tv = o - v0;
            const V3 p = cross(d, e2);
            const V3 q = cross(tv, e1);
            const float denom = dot(p, e1);
            if (denom != 0.0f) {
                const float id = 1.0f / denom;
                const float u = dot(p, tv) * id;
                const float v = dot(q, d) * id;
                if (!(u < 0.0f || v < 0.0f || u + v > 1.0f)) {
                    const float t = dot(q, e2) * id;
                    const bool better = ORDERED ? (t < h.t || (t == h.t && hpos >= 0 && pos > hpos)) : (t < h.t);
                    if (better && t > kDelta) {
                        h.t = t;
                        h.fid = __float_as_int(q0.w);
                        h.u = u;
                        h.v = v;
                        hpos = pos;
                        if (any_hit) break;
                    }
                }
            }
        }
        if (sp == 0) break;
        node = stk[(--sp) * 256];
    }
    return h;
}

__device__ __forceinline__ V3 reflect_dir(V3 d, V3 n) { return d - (2.0f * dot(d, n)) * n; }   // :137-141

// getNewDirection (path_tracer.cu:187-225) for a material (eta, metallic).
// Returns the pdf; consumes 1 (dielectric), 0 (metal) or 2 (diffuse) uniforms.
__device__ __forceinline__ float new_direction(V3 d, V3 n, float eta_m, float metallic, uint32_t st[6], V3& next,
                                               float& atten) {
    if (eta_m > 0.0f) {
        // refract (:143-163)
        float cos_i = dot(d, n);
        const float eta = cos_i > 0.0f ? eta_m : 1.0f / eta_m;
        const V3 nn = cos_i > 0.0f ? -n : n;
        cos_i = fabs_(cos_i);
        const float sin2i = 1.0f - cos_i * cos_i;
        const float sin2t = eta * eta * sin2i;
        const bool tir = sin2t >= 1.0f;
        V3 rf = v3(0.0f, 0.0f, 0.0f);
        float fr = 1.0f;
        if (!tir) {
            const float cos_t = fsqrt(1.0f - sin2t);
            rf = (eta * d) + ((cos_i * eta - cos_t) * nn);
            float f0 = (1.0f - eta) / (1.0f + eta);   // shlickFresnel (:165-173)
            f0 *= f0;
            const float m = fclamp(1.0f - cos_i, 1.0f, 0.0f);
            const float m2 = m * m;
            fr = f0 + (1.0f - f0) * m2 * m2 * m;
        }
        const V3 rl = reflect_dir(d, n);
        next = xorwow_uniform(st) < fr ? rl : rf;   // CoinFlip (sampler.h:98-101)
        atten = 1.0f;
        return 1.0f;
    } else if (metallic > 0.0f) {
        atten = 1.0f;
        next = reflect_dir(d, n);
        return 1.0f;
    }
    const float sign = dot(d, n) > 0.0f ? -1.0f : 1.0f;
    n = sign * n;
    // HemisphereCosine (sampler.h:75-89)
    V3 xb = n.z == 0.0f ? v3(0.0f, 0.0f, 1.0f) : v3(1.0f, 0.0f, -n.x / n.z);
    xb = vdiv(xb, fsqrt(norm2(xb)));
    const V3 zb = cross(xb, n);
    const float phi = 2.0f * kPi * xorwow_uniform(st);
    const float cos_t = fsqrt(xorwow_uniform(st));
    const float sin_t = fsqrt(1.0f - cos_t * cos_t);
    float sp, cp;
    psincos2pi(phi, sp, cp);
    const float x = cp * sin_t;
    const float z = sp * sin_t;
    next = ((x * xb) + (cos_t * n)) + (z * zb);
    const float c = dot(next, n);
    atten = fabs_(c) / kPi;
    return (c / kPi) * (c > 0.0f ? 1.0f : 0.0f);   // HemishpereCosinePDF (sampler.h:91-96)
}

// DeltaLight::sample + CalcDistAttenuation (delta_light.h:25-130)
__device__ __forceinline__ void light_sample(const DevLight* __restrict__ Ls, int li, V3 p, V3& dir, V3& rad) {
    const DevLight& L = Ls[li];
    float dist = 0.0f;
    const V3 color = v3(L.color[0], L.color[1], L.color[2]);
    dir = v3(0.0f, 0.0f, 0.0f);
    rad = v3(0.0f, 0.0f, 0.0f);
    if (L.type == 0 || L.type == 2) {
        const V3 dd = v3(L.pos[0], L.pos[1], L.pos[2]) - p;
        dist = fsqrt(norm2(dd));
        dir = vdiv(dd, dist);
        rad = L.intensity * color;
        if (L.type == 2) {
            const float cos_t = dot(-dir, v3(L.dir[0], L.dir[1], L.dir[2]));
            const float fall = fsq(fsat(cos_t - L.cos_outer) * L.inv_cos_cone_diff);
            rad = fall * rad;
        }
    } else if (L.type == 1) {
        dir = -v3(L.dir[0], L.dir[1], L.dir[2]);
        rad = L.intensity * color;
    }
    const float d2 = dist * dist;
    float att = 1.0f / (d2 + 1.0f);
    att *= fsq(fsat(1.0f - fsq(d2 * 0.01f)));
    rad = att * rad;
}

// sampleEnvLights (:288-294): Vec2UV (env_light.cuh:72-78) + point/clamp fetch
// (texture.cu:156-170) of the RGBA8 equirect, row 0 = bottom.
__device__ __noinline__ V3 env_lookup(const uint32_t* __restrict__ env, int w, int h, V3 d) {
    float u = patan2_fast(d.z, d.x) / (2.0f * kPi);
    if (u < 0.0f) u += 1.0f;
    const float v = 1.0f - pacos_fast(fclamp(d.y, 1.0f, -1.0f)) / kPi;
    int ix = (int)floorf(u * (float)w);
    int iy = (int)floorf(v * (float)h);
    ix = ix < 0 ? 0 : (ix > w - 1 ? w - 1 : ix);
    iy = iy < 0 ? 0 : (iy > h - 1 ? h - 1 : iy);
    const uint32_t t = env[(size_t)iy * (size_t)w + (size_t)ix];
    return (1.0f / 255.0f) * v3((float)(t & 0xffu), (float)((t >> 8) & 0xffu), (float)((t >> 16) & 0xffu));
}

__device__ __forceinline__ int band_row(int ly, int band_rows, int band_count, int band_index) {
    return ((ly / band_rows) * band_count + band_index) * band_rows + (ly % band_rows);
}

__device__ __forceinline__ unsigned long long wave_sum(uint32_t v) {
    unsigned long long s = v;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
    return s;
}

enum : int { PH_CAMERA = 0, PH_EXT = 1, PH_SHADOW = 2, PH_PROBE = 3 };

// Per-lane path records, one per depth (path_tracer.cu:315-318): attenuation
// (baseColor * atten), 1/p and the direct term, consumed by the unwind.
template <int MAXD>
struct PathRecords {
    V3 att[MAXD], dst[MAXD];
    float ivp[MAXD];
};

#ifndef TPT_TRACE_WAVES
#define TPT_TRACE_WAVES 5   // min waves per SIMD requested from the register allocator (96 VGPRs)
#endif

template <int MAXD, bool ORDERED>
__global__ __launch_bounds__(256, TPT_TRACE_WAVES) void k_trace(TraceArgs a) {
    extern __shared__ int lds_stack[];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int x = blockIdx.x * 16 + (wave & 1) * 8 + (lane & 7);
    const int ly = blockIdx.y * 16 + (wave >> 1) * 8 + (lane >> 3);
    const int y = band_row(ly, a.band_rows, a.band_count, a.band_index);
    const bool active = x < a.width && ly < a.band_height && y < a.height;
    uint32_t c_trav = 0, c_inner = 0, c_leaf = 0, c_shade = 0, c_ovf = 0;

    if (active) {
        const size_t npix = (size_t)a.width * (size_t)a.height;
        const size_t off = (size_t)x + (size_t)y * (size_t)a.width;
        const int nint = a.n_faces - 1;
        int* stk = lds_stack + tid;
        uint32_t st[6];
#pragma unroll
        for (int i = 0; i < 6; ++i) st[i] = a.rng[i * npix + off];
        V3 total = v3(a.accum[off], a.accum[npix + off], a.accum[2 * npix + off]);
        PathRecords<MAXD> rec;

        int remaining = a.samples;
        int phase = PH_CAMERA;
        int depth = 0, li = 0, mtl = 0;
        V3 ro = v3(0.0f, 0.0f, 0.0f), rd = ro, td = ro, nd = ro, nrm = ro, direct = ro;

        for (;;) {
            if (phase == PH_CAMERA) {
                if (remaining == 0) break;
                --remaining;
                // sampleRays (path_tracer.cu:42-59)
                const float ju = xorwow_uniform(st);
                const float jv = xorwow_uniform(st);
                float lx = ju * 1.0f, lyf = jv * 1.0f;
                lx = lx + (float)x;
                lyf = lyf + (float)y;
                lx = lx * a.inv_w;
                lyf = lyf * a.inv_h;
                lx = lx * a.sensor_w;
                lyf = lyf * a.sensor_h;
                float r4[4];
                mat4_vec4(a.c2w, lx - a.half_sw, lyf - a.half_sh, 0.0f - 1.0f, 0.0f, r4);
                rd = normalize(v3(r4[0], r4[1], r4[2]));
                ro = v3(a.origin[0], a.origin[1], a.origin[2]);
                td = rd;
                depth = 0;
                phase = PH_EXT;
            }

            ++c_trav;
            const Hit h = traverse<ORDERED>(a.inner, a.tri, nint, stk, a.stack_depth, ro, td, phase == PH_SHADOW,
                                            c_inner, c_leaf, c_ovf);

            bool finish = false, lights_next = false, after = false;
            V3 L = v3(0.0f, 0.0f, 0.0f);
            if (phase == PH_EXT) {
                if (h.fid < 0) {
                    if (a.env) L = env_lookup(a.env, a.env_w, a.env_h, rd);
                    finish = true;
                } else {
                    ++c_shade;
                    const float4* sh = a.shade + 3 * h.fid;
                    const float4 s0 = sh[0], s1 = sh[1], s2 = sh[2];
                    const float w = 1.0f - h.u - h.v;
                    nrm = normalize(((w * v3(s0.x, s0.y, s0.z)) + (h.u * v3(s1.x, s1.y, s1.z))) +
                                    (h.v * v3(s2.x, s2.y, s2.z)));
                    ro = ro + (h.t * rd);
                    mtl = __float_as_int(s0.w);
                    const float4 m0 = a.mtl[2 * mtl], m1 = a.mtl[2 * mtl + 1];
                    float af;
                    const float prob = new_direction(rd, nrm, m1.x, m1.y, st, nd, af);
                    rec.att[depth] = af * v3(m0.x, m0.y, m0.z);
                    rec.ivp[depth] = 1.0f / prob;
                    direct = v3(0.0f, 0.0f, 0.0f);
                    li = 0;
                    lights_next = true;
                }
            } else if (phase == PH_SHADOW) {
                if (h.fid < 0) {   // sampleDeltaLights :279-282 (light re-sampled: deterministic)
                    V3 ldir, lrad;
                    light_sample(a.lights, li, ro, ldir, lrad);
                    const float4 m0 = a.mtl[2 * mtl];
                    direct = direct + (v3(m0.x, m0.y, m0.z) * lrad);
                }
                ++li;
                lights_next = true;
            } else {   // PH_PROBE (:390-400)
                V3 dl = direct;
                if (h.fid >= 0) {
                    const int pm = __float_as_int(a.shade[3 * h.fid].w);
                    const float e = a.mtl[2 * pm].w;
                    dl = (v3(1.0f, 1.0f, 1.0f) * v3(e, e, e)) + direct;
                }
                rec.dst[depth] = dl;
                after = true;
            }

            if (lights_next) {
                const float4 m1 = a.mtl[2 * mtl + 1];
                if (li < a.n_lights) {
                    V3 lrad;
                    light_sample(a.lights, li, ro, td, lrad);
                    phase = PH_SHADOW;
                } else if (!(m1.x >= 1.0f || m1.y > 0.0f)) {   // direct probe (:387-389)
                    float af2;
                    new_direction(rd, nrm, m1.x, m1.y, st, td, af2);
                    phase = PH_PROBE;
                } else {
                    rec.dst[depth] = direct;
                    after = true;
                }
            }
            if (after) {
                const float e = a.mtl[2 * mtl].w;
                if (e > 0.0f) {   // an emitter ends the path (:408-412); the unwind starts from e
                    L = e * v3(1.0f, 1.0f, 1.0f);
                    finish = true;
                } else {
                    rd = nd;
                    td = rd;
                    ++depth;
                    if (depth == a.max_depth) finish = true;
                    else phase = PH_EXT;
                }
            }
            if (finish) {   // unwind (:416-431): levels depth-1 .. 0
                for (int k = depth - 1; k >= 0; --k) L = rec.ivp[k] * ((rec.dst[k] + L) * rec.att[k]);
                total = total + L;
                phase = PH_CAMERA;
            }
        }
#pragma unroll
        for (int i = 0; i < 6; ++i) a.rng[i * npix + off] = st[i];
        a.accum[off] = total.x;
        a.accum[npix + off] = total.y;
        a.accum[2 * npix + off] = total.z;
    }

    const unsigned long long s_trav = wave_sum(c_trav), s_inner = wave_sum(c_inner), s_leaf = wave_sum(c_leaf),
                             s_shade = wave_sum(c_shade), s_ovf = wave_sum(c_ovf);
    if (lane == 0) {
        atomicAdd(&a.counters[0], s_trav);
        atomicAdd(&a.counters[1], s_inner);
        atomicAdd(&a.counters[2], s_leaf);
        atomicAdd(&a.counters[3], s_shade);
        if (s_ovf) atomicAdd(&a.counters[4], s_ovf);
    }
}

// ---------------------------------------------------------------------------
// v3 megakernel: ballot-driven traversal with postponed shading.
//
// A wave keeps stepping its lanes through BVH nodes while at least
// `a.refill` of them are still traversing; once fewer are, it leaves the loop
// and the finished lanes shade their hit, advance their path state machine and
// set up their next ray (next bounce, shadow, probe or next sample), while the
// unfinished lanes keep their traversal state (node, stack, best hit) in
// registers and resume afterwards.  The wave therefore pays for the average
// traversal length of its lanes instead of the longest one.
// ---------------------------------------------------------------------------
struct Trav {
    V3 o, d, inv;
    int node, sp, hpos, fid;
    float t, u, v;
    bool any_hit;
};

__device__ __forceinline__ void trav_begin(Trav& r, V3 o, V3 d, bool any_hit) {
    r.o = o;
    r.d = d;
    r.inv = v3(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
    r.node = 0;
    r.sp = 0;
    r.hpos = -1;
    r.fid = -1;
    r.t = kRealMax;
    r.u = 0.0f;
    r.v = 0.0f;
    r.any_hit = any_hit;
}

// One node of traverseBVH (path_tracer.cu:61-107), same semantics as
// traverse<ORDERED> above.  Returns false once the traversal has finished.
template <bool ORDERED>
__device__ __forceinline__ bool trav_step(Trav& r, const float4* __restrict__ inner, const float4* __restrict__ tri,
                                          int nint, int* stk, int stack_depth, uint32_t& c_inner, uint32_t& c_leaf,
                                          uint32_t& c_ovf) {
    if (r.node < nint) {
        ++c_inner;
        const float4* nd = inner + 4 * r.node;
        const float4 q0 = nd[0], q1 = nd[1], q2 = nd[2], q3 = nd[3];
        float l0, l1, r0, r1;
        bool hl = box_hit(r.o, r.inv, q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, l0, l1);
        bool hr = box_hit(r.o, r.inv, q1.z, q1.w, q2.x, q2.y, q2.z, q2.w, r0, r1);
        const int lc = __float_as_int(q3.x), rc = __float_as_int(q3.y);
        if (ORDERED) {
            const float lim = r.t * 1.0001f;
            hl = hl && !(l0 > lim) && !(l1 < 0.5f * kDelta);
            hr = hr && !(r0 > lim) && !(r1 < 0.5f * kDelta);
        }
        if (hl && hr) {
            int first = rc, second = lc;
            if (ORDERED && l0 < r0) { first = lc; second = rc; }
            if (r.sp >= stack_depth) { ++c_ovf; return false; }
            stk[(r.sp++) * 256] = second;
            r.node = first;
            return true;
        }
        if (hl) { r.node = lc; return true; }
        if (hr) { r.node = rc; return true; }
    } else {
        ++c_leaf;
        const int pos = r.node - nint;
        const float4* tr = tri + 3 * pos;
        const float4 q0 = tr[0], q1 = tr[1], q2 = tr[2];
        const V3 v0 = v3(q0.x, q0.y, q0.z), e1 = v3(q1.x, q1.y, q1.z), e2 = v3(q2.x, q2.y, q2.z);
        const V3 tv = r.o - v0;
        const V3 p = cross(r.d, e2);
        const V3 q = cross(tv, e1);
        const float denom = dot(p, e1);
        if (denom != 0.0f) {
            const float id = 1.0f / denom;
            const float u = dot(p, tv) * id;
            const float v = dot(q, r.d) * id;
            if (!(u < 0.0f || v < 0.0f || u + v > 1.0f)) {
                const float t = dot(q, e2) * id;
                const bool better = ORDERED ? (t < r.t || (t == r.t && r.hpos >= 0 && pos > r.hpos)) : (t < r.t);
                if (better && t > kDelta) {
                    r.t = t;
                    r.fid = __float_as_int(q0.w);
                    r.u = u;
                    r.v = v;
                    r.hpos = pos;
                    if (r.any_hit) return false;
                }
            }
        }
    }
    if (r.sp == 0) return false;
    r.node = stk[(--r.sp) * 256];
    return true;
}

enum : int { TS_DONE = 0, TS_TRAV = 1, TS_DEAD = 2 };

template <int MAXD, bool ORDERED>
__global__ __launch_bounds__(256, TPT_TRACE_WAVES) void k_trace3(TraceArgs a) {
    extern __shared__ int lds_stack[];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int x = blockIdx.x * 16 + (wave & 1) * 8 + (lane & 7);
    const int ly = blockIdx.y * 16 + (wave >> 1) * 8 + (lane >> 3);
    const int y = band_row(ly, a.band_rows, a.band_count, a.band_index);
    const bool active = x < a.width && ly < a.band_height && y < a.height;
    uint32_t c_trav = 0, c_inner = 0, c_leaf = 0, c_shade = 0, c_ovf = 0;
    const size_t npix = (size_t)a.width * (size_t)a.height;
    const size_t off = active ? (size_t)x + (size_t)y * (size_t)a.width : 0;
    const int nint = a.n_faces - 1;
    int* stk = lds_stack + tid;

    uint32_t st[6];
    V3 total = v3(0.0f, 0.0f, 0.0f);
    if (active) {
#pragma unroll
        for (int i = 0; i < 6; ++i) st[i] = a.rng[i * npix + off];
        total = v3(a.accum[off], a.accum[npix + off], a.accum[2 * npix + off]);
    }
    PathRecords<MAXD> rec;
    int remaining = a.samples;
    int phase = PH_CAMERA;
    int depth = 0, li = 0, mtl = 0;
    V3 rd = v3(0.0f, 0.0f, 0.0f), nd = rd, nrm = rd, direct = rd;
    Trav r;
    trav_begin(r, rd, v3(1.0f, 1.0f, 1.0f), false);
    int ts = active ? TS_DONE : TS_DEAD;
    const int refill = a.refill;

    for (;;) {
        if (ts == TS_DONE) {
            // ---- consume the finished traversal (none for a fresh sample) ----
            bool finish = false, lights_next = false, after = false;
            V3 L = v3(0.0f, 0.0f, 0.0f);
            if (phase == PH_EXT) {
                if (r.fid < 0) {
                    if (a.env) L = env_lookup(a.env, a.env_w, a.env_h, rd);
                    finish = true;
                } else {
                    ++c_shade;
                    const float4* sh = a.shade + 3 * r.fid;
                    const float4 s0 = sh[0], s1 = sh[1], s2 = sh[2];
                    const float w = 1.0f - r.u - r.v;
                    nrm = normalize(((w * v3(s0.x, s0.y, s0.z)) + (r.u * v3(s1.x, s1.y, s1.z))) +
                                    (r.v * v3(s2.x, s2.y, s2.z)));
                    r.o = r.o + (r.t * rd);
                    mtl = __float_as_int(s0.w);
                    const float4 m0 = a.mtl[2 * mtl], m1 = a.mtl[2 * mtl + 1];
                    float af;
                    const float prob = new_direction(rd, nrm, m1.x, m1.y, st, nd, af);
                    rec.att[depth] = af * v3(m0.x, m0.y, m0.z);
                    rec.ivp[depth] = 1.0f / prob;
                    direct = v3(0.0f, 0.0f, 0.0f);
                    li = 0;
                    lights_next = true;
                }
            } else if (phase == PH_SHADOW) {
                if (r.fid < 0) {   // sampleDeltaLights :279-282 (light re-sampled: deterministic)
                    V3 ldir, lrad;
                    light_sample(a.lights, li, r.o, ldir, lrad);
                    const float4 m0 = a.mtl[2 * mtl];
                    direct = direct + (v3(m0.x, m0.y, m0.z) * lrad);
                }
                ++li;
                lights_next = true;
            } else if (phase == PH_PROBE) {   // :390-400
                V3 dl = direct;
                if (r.fid >= 0) {
                    const int pm = __float_as_int(a.shade[3 * r.fid].w);
                    const float e = a.mtl[2 * pm].w;
                    dl = (v3(1.0f, 1.0f, 1.0f) * v3(e, e, e)) + direct;
                }
                rec.dst[depth] = dl;
                after = true;
            }
            V3 td = rd;
            bool shadow = false;
            if (lights_next) {
                const float4 m1 = a.mtl[2 * mtl + 1];
                if (li < a.n_lights) {
                    V3 lrad;
                    light_sample(a.lights, li, r.o, td, lrad);
                    phase = PH_SHADOW;
                    shadow = true;
                } else if (!(m1.x >= 1.0f || m1.y > 0.0f)) {   // direct probe (:387-389)
                    float af2;
                    new_direction(rd, nrm, m1.x, m1.y, st, td, af2);
                    phase = PH_PROBE;
                } else {
                    rec.dst[depth] = direct;
                    after = true;
                }
            }
            if (after) {
                const float e = a.mtl[2 * mtl].w;
                if (e > 0.0f) {   // an emitter ends the path (:408-412); the unwind starts from e
                    L = e * v3(1.0f, 1.0f, 1.0f);
                    finish = true;
                } else {
                    rd = nd;
                    td = rd;
                    ++depth;
                    if (depth == a.max_depth) finish = true;
                    else phase = PH_EXT;
                }
            }
            if (finish) {   // unwind (:416-431): levels depth-1 .. 0
                for (int k = depth - 1; k >= 0; --k) L = rec.ivp[k] * ((rec.dst[k] + L) * rec.att[k]);
                total = total + L;
                phase = PH_CAMERA;
            }
            V3 to = r.o;
            if (phase == PH_CAMERA) {
                if (remaining == 0) {
                    ts = TS_DEAD;
                } else {
                    --remaining;
                    // sampleRays (path_tracer.cu:42-59)
                    const float ju = xorwow_uniform(st);
                    const float jv = xorwow_uniform(st);
                    float lx = ju * 1.0f, lyf = jv * 1.0f;
                    lx = lx + (float)x;
                    lyf = lyf + (float)y;
                    lx = lx * a.inv_w;
                    lyf = lyf * a.inv_h;
                    lx = lx * a.sensor_w;
                    lyf = lyf * a.sensor_h;
                    float r4[4];
                    mat4_vec4(a.c2w, lx - a.half_sw, lyf - a.half_sh, 0.0f - 1.0f, 0.0f, r4);
                    rd = normalize(v3(r4[0], r4[1], r4[2]));
                    td = rd;
                    to = v3(a.origin[0], a.origin[1], a.origin[2]);
                    depth = 0;
                    phase = PH_EXT;
                }
            }
            if (ts != TS_DEAD) {
                ++c_trav;
                trav_begin(r, to, td, shadow);
                ts = TS_TRAV;
            }
        }
        if (__ballot(ts != TS_DEAD) == 0ull) break;
        // ---- traversal: step while enough lanes of the wave are still traversing ----
        for (;;) {
            const unsigned long long tm = __ballot(ts == TS_TRAV);
            const int cnt = __popcll(tm);
            if (cnt == 0) break;
            if (cnt < refill && __ballot(ts == TS_DONE) != 0ull) break;
            if (ts == TS_TRAV) {
                if (!trav_step<ORDERED>(r, a.inner, a.tri, nint, stk, a.stack_depth, c_inner, c_leaf, c_ovf))
                    ts = TS_DONE;
            }
        }
    }
    if (active) {
#pragma unroll
        for (int i = 0; i < 6; ++i) a.rng[i * npix + off] = st[i];
        a.accum[off] = total.x;
        a.accum[npix + off] = total.y;
        a.accum[2 * npix + off] = total.z;
    }
    const unsigned long long s_trav = wave_sum(c_trav), s_inner = wave_sum(c_inner), s_leaf = wave_sum(c_leaf),
                             s_shade = wave_sum(c_shade), s_ovf = wave_sum(c_ovf);
    if (lane == 0) {
        atomicAdd(&a.counters[0], s_trav);
        atomicAdd(&a.counters[1], s_inner);
        atomicAdd(&a.counters[2], s_leaf);
        atomicAdd(&a.counters[3], s_shade);
        if (s_ovf) atomicAdd(&a.counters[4], s_ovf);
    }
}

// copyToFB (path_tracer.cu:451-471) + the radiance readout (color / spp).
__global__ void k_resolve(ResolveArgs a) {
    const int x = blockIdx.x * blockDim.x + threadIdx.x;
    const int ly = blockIdx.y;
    if (x >= a.width || ly >= a.band_height) return;
    const int y = band_row(ly, a.band_rows, a.band_count, a.band_index);
    if (y >= a.height) return;
    const size_t npix = (size_t)a.width * (size_t)a.height;
    const size_t off = (size_t)x + (size_t)y * (size_t)a.width;
    const float inv = 1.0f / (float)a.spp;
    const float r = (0.0f + a.accum[off]) * inv;
    const float g = (0.0f + a.accum[npix + off]) * inv;
    const float b = (0.0f + a.accum[2 * npix + off]) * inv;
    if (a.radiance) {
        a.radiance[3 * off] = r;
        a.radiance[3 * off + 1] = g;
        a.radiance[3 * off + 2] = b;
    }
    if (a.bgra) {   // Spectrum::toUChar (material.h:74-81): truncating clamp
        uint8_t* px = a.bgra + 4 * ((size_t)(a.height - y - 1) * (size_t)a.width + (size_t)x);
        px[0] = (uint8_t)fclamp(b * 255.0f, 255.0f, 0.0f);
        px[1] = (uint8_t)fclamp(g * 255.0f, 255.0f, 0.0f);
        px[2] = (uint8_t)fclamp(r * 255.0f, 255.0f, 0.0f);
    }
}

__global__ __launch_bounds__(256) void k_trace_rays(TraceArgs a, uint32_t n, const float* __restrict__ o,
                                                    const float* __restrict__ d, int32_t* hit, float* t, float* uv) {
    extern __shared__ int lds_stack[];
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    uint32_t c0 = 0, c1 = 0, c2 = 0;
    if (i < n) {
        const Hit h = traverse<false>(a.inner, a.tri, a.n_faces - 1, lds_stack + threadIdx.x, a.stack_depth,
                               v3(o[3 * i], o[3 * i + 1], o[3 * i + 2]), v3(d[3 * i], d[3 * i + 1], d[3 * i + 2]),
                               false, c0, c1, c2);
        hit[i] = h.fid;
        t[i] = h.t;
        uv[2 * i] = h.u;
        uv[2 * i + 1] = h.v;
    }
}

template <bool ORDERED, bool V3K>
static void launch_trace_t(const TraceArgs& a, dim3 grid, size_t lds, hipStream_t s) {
    if (V3K) {
        if (a.max_depth <= 8)
            hipLaunchKernelGGL((k_trace3<8, ORDERED>), grid, dim3(256), lds, s, a);
        else if (a.max_depth <= 16)
            hipLaunchKernelGGL((k_trace3<16, ORDERED>), grid, dim3(256), lds, s, a);
        else if (a.max_depth <= 32)
            hipLaunchKernelGGL((k_trace3<32, ORDERED>), grid, dim3(256), lds, s, a);
        else
            hipLaunchKernelGGL((k_trace3<64, ORDERED>), grid, dim3(256), lds, s, a);
        return;
    }
    if (a.max_depth <= 8)
        hipLaunchKernelGGL((k_trace<8, ORDERED>), grid, dim3(256), lds, s, a);
    else if (a.max_depth <= 16)
        hipLaunchKernelGGL((k_trace<16, ORDERED>), grid, dim3(256), lds, s, a);
    else if (a.max_depth <= 32)
        hipLaunchKernelGGL((k_trace<32, ORDERED>), grid, dim3(256), lds, s, a);
    else
        hipLaunchKernelGGL((k_trace<64, ORDERED>), grid, dim3(256), lds, s, a);
}

hipError_t launch_trace(const TraceArgs& a, hipStream_t s) {
    dim3 grid((a.width + 15) / 16, (a.band_height + 15) / 16);
    const size_t lds = (size_t)a.stack_depth * 256 * sizeof(int);
    const bool legacy = (a.flags & TPT_FLAG_LEGACY_LOOP) != 0;
    if (a.flags & TPT_FLAG_REF_ORDER) {
        if (legacy) launch_trace_t<false, false>(a, grid, lds, s);
        else launch_trace_t<false, true>(a, grid, lds, s);
    } else {
        if (legacy) launch_trace_t<true, false>(a, grid, lds, s);
        else launch_trace_t<true, true>(a, grid, lds, s);
    }
    return hipGetLastError();
}

hipError_t launch_resolve(const ResolveArgs& a, hipStream_t s) {
    dim3 grid((a.width + 255) / 256, a.band_height);
    hipLaunchKernelGGL(k_resolve, grid, dim3(256), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_trace_rays(const TraceArgs& a, uint32_t n, const float* o, const float* d, int32_t* hit, float* t,
                             float* uv, hipStream_t s) {
    if (n == 0) return hipSuccess;
    const size_t lds = (size_t)a.stack_depth * 256 * sizeof(int);
    hipLaunchKernelGGL(k_trace_rays, dim3((n + 255) / 256), dim3(256), lds, s, a, n, o, d, hit, t, uv);
    return hipGetLastError();
}

}  // namespace tpt
