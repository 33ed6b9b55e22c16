/*
 * tpt_oracle.c -- CPU restatement of the TinyPathTracer hot path.
 *
 * TEST INFRASTRUCTURE ONLY (see tpt_oracle.h).  Compiled with
 * -ffp-contract=off so every float expression rounds exactly where the
 * reference's C++ rounds.  References are to /root/reference/.
 */
#include "tpt_oracle.h"

#include <float.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* ------------------------------------------------------------------------ */
/* L0 math: include/math/vec.h                                               */
/* ------------------------------------------------------------------------ */
typedef struct { float x, y, z; } v3;

static inline v3 V3(float x, float y, float z) { v3 r = {x, y, z}; return r; }
static inline v3 vadd(v3 a, v3 b) { return V3(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline v3 vsub(v3 a, v3 b) { return V3(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline v3 vneg(v3 a) { return V3(-a.x, -a.y, -a.z); }
static inline v3 vmul(v3 a, v3 b) { return V3(a.x * b.x, a.y * b.y, a.z * b.z); }
/* Real * Vec3 and Vec3 * Real (vec.h:140-141); IEEE products commute. */
static inline v3 vscale(float s, v3 a) { return V3(s * a.x, s * a.y, s * a.z); }
/* Vec3 / Real == (1/rhs) * lhs (vec.h:143) */
static inline v3 vdiv(v3 a, float s) { return vscale(1.0f / s, a); }
/* dot, cross (vec.h:151-152), left-to-right sums */
static inline float vdot(v3 a, v3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
static inline v3 vcross(v3 l, v3 r) {
    return V3(l.y * r.z - l.z * r.y, l.z * r.x - l.x * r.z, l.x * r.y - l.y * r.x);
}
static inline float vnorm2(v3 a) { return a.x * a.x + a.y * a.y + a.z * a.z; }
/* template max/min/clamp (vec.h:73-78): ternaries, NaN-propagating as written */
static inline float fmx(float x, float y) { return x > y ? x : y; }
static inline float fmn(float x, float y) { return x < y ? x : y; }
static inline float fclamp(float x, float hi, float lo) { return fmx(fmn(x, hi), lo); }
static inline float fsat(float x) { return fclamp(x, 1.0f, 0.0f); }
static inline float fsq(float x) { return x * x; }
static inline v3 vmin(v3 a, v3 b) { return V3(fmn(a.x, b.x), fmn(a.y, b.y), fmn(a.z, b.z)); }
static inline v3 vmax(v3 a, v3 b) { return V3(fmx(a.x, b.x), fmx(a.y, b.y), fmx(a.z, b.z)); }

/* Quake inverse square root with one Newton step (vec.h:44-57). */
static inline float frsqrt(float num) {
    float x2 = num * 0.5f;
    float y = num;
    int32_t i;
    memcpy(&i, &y, 4);
    i = 0x5f3759df - (i >> 1);
    memcpy(&y, &i, 4);
    y = y * (1.5f - (x2 * y * y));
    return y;
}
/* normalize(v) = v * frsqrt(v.norm2()) (vec.h:155) */
static inline v3 vnormalize(v3 v) { return vscale(frsqrt(vnorm2(v)), v); }

static const float PI_F = 3.141592653589793f;   /* vec.h:66 */
static const float DELTA_F = 2e-4f;              /* vec.h:70 */

/* Column-major Mat4 * Vec4 (mat.h:37-51): res[i] += m[j][i] * v[j], j=0..3 */
static inline void mat4_vec4(const float* m, const float v[4], float r[4]) {
    for (int i = 0; i < 4; ++i) {
        float acc = 0.0f;
        for (int j = 0; j < 4; ++j) acc += m[4 * j + i] * v[j];
        r[i] = acc;
    }
}

/* ------------------------------------------------------------------------ */
/* Transcendentals.  trig_mode 0: libm float (the survey's host harness);     */
/* trig_mode 1: the HIP kernel's parity trig (ptrig.hpp): fp32 sincos below,  */
/* (float)f((double)x) for atan2/acos/tan                                     */
/* ------------------------------------------------------------------------ */
float orc_parity_sinf(float x) { return (float)sin((double)x); }
float orc_parity_cosf(float x) { return (float)cos((double)x); }
/* fsincos_2pi: the HIP kernel's fp32 sin/cos of phi in [0, 2pi]
 * (tinypathtracer_amd/csrc/common/ptrig.hpp) restated step for step: Cody-Waite
 * reduction by pi/2 in three fmaf steps, minimax polynomials, quadrant swap. */
static void parity_sincos(float x, float* s, float* c) {
    const float k = rintf(x * 0.636619772f);
    const int q = (int)k & 3;
    float r = fmaf(-k, 1.57079637f, x);
    r = fmaf(-k, -4.37113883e-08f, r);
    r = fmaf(-k, -1.71512489e-15f, r);
    const float z = r * r;
    float ps = fmaf(z, 2.71808875e-06f, -1.98393362e-04f);
    ps = fmaf(z, ps, 8.33332464e-03f);
    ps = fmaf(z, ps, -1.66666657e-01f);
    const float sr = fmaf(r * z, ps, r);
    float pc = fmaf(z, 2.43904487e-05f, -1.38867637e-03f);
    pc = fmaf(z, pc, 4.16666418e-02f);
    pc = fmaf(z, pc, -0.5f);
    const float cr = fmaf(z, pc, 1.0f);
    switch (q) {
        case 0: *s = sr; *c = cr; break;
        case 1: *s = cr; *c = -sr; break;
        case 2: *s = -sr; *c = -cr; break;
        default: *s = -cr; *c = sr; break;
    }
}
void orc_parity_sincos(float x, float* s, float* c) { parity_sincos(x, s, c); }
static inline float t_sin(int m, float x) {
    if (!m) return sinf(x);
    float s, c;
    parity_sincos(x, &s, &c);
    return s;
}
static inline float t_cos(int m, float x) {
    if (!m) return cosf(x);
    float s, c;
    parity_sincos(x, &s, &c);
    return c;
}
static inline float t_acos(int m, float x) { return m ? (float)acos((double)x) : acosf(x); }
static inline float t_atan2(int m, float y, float x) {
    return m ? (float)atan2((double)y, (double)x) : atan2f(y, x);
}
static inline float t_tan(int m, float x) { return m ? (float)tan((double)x) : tanf(x); }

/* ------------------------------------------------------------------------ */
/* cuRAND XORWOW (CUDA toolkit curand_kernel.h; call sites path_tracer.cu:39, */
/* sampler.h:14).  Not vendored in the reference: restated from its published */
/* algorithm (Marsaglia xorwow + Weyl counter, 2^67 subsequence spacing).     */
/* ------------------------------------------------------------------------ */
#define XW_WORDS 5
#define XW_BITS 160
#define XW_NJUMP 32
static uint32_t g_jump[XW_NJUMP][XW_BITS * XW_WORDS];
static int g_jump_ready = 0;

static void xw_step_raw(uint32_t v[5]) {
    uint32_t t = v[0] ^ (v[0] >> 2);
    v[0] = v[1]; v[1] = v[2]; v[2] = v[3]; v[3] = v[4];
    v[4] = (v[4] ^ (v[4] << 4)) ^ (t ^ (t << 1));
}
/* r = M v where row b of M is the image of input bit b */
static void xw_matvec(const uint32_t* m, const uint32_t v[5], uint32_t r[5]) {
    uint32_t acc[5] = {0, 0, 0, 0, 0};
    for (int b = 0; b < XW_BITS; ++b) {
        if ((v[b >> 5] >> (b & 31)) & 1u) {
            const uint32_t* row = m + b * XW_WORDS;
            for (int k = 0; k < 5; ++k) acc[k] ^= row[k];
        }
    }
    memcpy(r, acc, sizeof acc);
}
/* out = M * M */
static void xw_square(const uint32_t* m, uint32_t* out) {
    for (int b = 0; b < XW_BITS; ++b) xw_matvec(m, m + b * XW_WORDS, out + b * XW_WORDS);
}
static void xw_build_jumps(void) {
    static uint32_t a[XW_BITS * XW_WORDS], tmp[XW_BITS * XW_WORDS];
    for (int b = 0; b < XW_BITS; ++b) {       /* one-step matrix A */
        uint32_t v[5] = {0, 0, 0, 0, 0};
        v[b >> 5] = 1u << (b & 31);
        xw_step_raw(v);
        memcpy(a + b * XW_WORDS, v, sizeof v);
    }
    for (int s = 0; s < 67; ++s) {            /* A^(2^67) */
        xw_square(a, tmp);
        memcpy(a, tmp, sizeof a);
    }
    memcpy(g_jump[0], a, sizeof a);
    for (int k = 1; k < XW_NJUMP; ++k) {      /* J_k = J_{k-1}^4 */
        xw_square(g_jump[k - 1], tmp);
        xw_square(tmp, g_jump[k]);
    }
    g_jump_ready = 1;
}
const uint32_t* orc_xorwow_jump_matrices(void) {
#pragma omp critical(orc_jump)
    {
        if (!g_jump_ready) xw_build_jumps();
    }
    return &g_jump[0][0];
}

/* state = {v0..v4, d} */
void orc_xorwow_init(uint64_t seed, uint64_t subsequence, uint32_t st[6]) {
    orc_xorwow_jump_matrices();
    uint32_t s0 = ((uint32_t)seed) ^ 0xaad26b49u;
    uint32_t s1 = ((uint32_t)(seed >> 32)) ^ 0xf7dcefddu;
    uint32_t t0 = 1099087573u * s0;
    uint32_t t1 = 2591861531u * s1;
    st[5] = 6615241u + t1 + t0;
    st[0] = 123456789u + t0;
    st[1] = 362436069u ^ t0;
    st[2] = 521288629u + t1;
    st[3] = 88675123u ^ t1;
    st[4] = 5783321u + t0;
    /* skip subsequence * 2^67 draws: base-4 digits apply J_k (d unchanged: 2^67*n = 0 mod 2^32) */
    int k = 0;
    while (subsequence && k < XW_NJUMP) {
        unsigned digit = (unsigned)(subsequence & 3u);
        for (unsigned i = 0; i < digit; ++i) xw_matvec(g_jump[k], st, st);
        subsequence >>= 2;
        ++k;
    }
}

uint32_t orc_xorwow_next(uint32_t st[6]) {
    xw_step_raw(st);
    st[5] += 362437u;
    return st[4] + st[5];
}

/* curand_uniform: x * 2^-32 + 2^-33 in float, result in (0, 1] */
float orc_uniform(uint32_t st[6]) {
    uint32_t x = orc_xorwow_next(st);
    return (float)x * 2.3283064e-10f + (2.3283064e-10f / 2.0f);
}

/* ------------------------------------------------------------------------ */
/* transform kernel (path_tracer.cu:227-263)                                 */
/* ------------------------------------------------------------------------ */
static int find_object(int fid, const orc_interval* lut, int n) {
    int i = n - 1;                        /* findIdxOfTrans / mtlLinearSearch */
    for (; i >= 0; --i)
        if (fid >= lut[i].begin) return i;
    return i;
}

void orc_transform(const orc_scene* s, float* wv, float* wn) {
    for (uint32_t f = 0; f < s->n_faces; ++f) {
        int obj = find_object((int)f, s->lut, (int)s->n_objects);
        const float* vt = s->vert_trans + 16 * obj;
        const float* nt = s->normal_trans + 16 * obj;
        for (int c = 0; c < 3; ++c) {
            uint32_t vid = s->indices[3 * f + c];
            float in[4] = {s->vertices[3 * vid], s->vertices[3 * vid + 1], s->vertices[3 * vid + 2], 1.0f};
            float out[4];
            mat4_vec4(vt, in, out);
            wv[3 * vid] = out[0]; wv[3 * vid + 1] = out[1]; wv[3 * vid + 2] = out[2];
        }
        for (int c = 0; c < 3; ++c) {
            uint32_t vid = s->indices[3 * f + c];
            float in[4] = {s->normals[3 * vid], s->normals[3 * vid + 1], s->normals[3 * vid + 2], 0.0f};
            float out[4];
            mat4_vec4(nt, in, out);
            v3 n = vnormalize(V3(out[0], out[1], out[2]));
            wn[3 * vid] = n.x; wn[3 * vid + 1] = n.y; wn[3 * vid + 2] = n.z;
        }
    }
}

/* ------------------------------------------------------------------------ */
/* LBVH (src/bvh.cu)                                                         */
/* ------------------------------------------------------------------------ */
static int g_x86_shift = 0;
void orc_set_x86_shift(int on) { g_x86_shift = on; }

/* floatTo21Int (bvh.cu:23-46).  Defined choices: a right
 * shift by >= 32 yields 0 (PTX semantics), signed overflow wraps. */
int64_t orc_float_to_21int(float x) {
    int32_t ix;
    memcpy(&ix, &x, 4);
    int32_t exponent = (ix >> 23) & 0xff;
    int32_t mantissa = (ix & 0x00ffffff) | 0x00800000;
    exponent -= 127;
    uint32_t signbit = ((uint32_t)ix & 0x80000000u) >> 30;
    int32_t sign = -1 * ((int32_t)signbit - 1);
    uint32_t value;
    if (exponent >= 8) {
        value = 0x7fffffffu;
    } else if (exponent >= 0) {
        value = (uint32_t)mantissa << exponent;
    } else {
        int sh = -exponent;
        if (sh >= 32) sh = g_x86_shift ? (sh & 31) : 32;   /* UB in C++: PTX clamps, x86 masks */
        value = sh >= 32 ? 0u : (uint32_t)(mantissa >> sh);
    }
    value = value * (uint32_t)sign;
    value = value + 0x7fffffffu;
    return (int64_t)((value & 0xfffff800u) >> 11);
}

static inline int64_t expand_bits(int64_t b) {       /* bvh.cu:14-21 */
    uint64_t u = (uint64_t)b;
    u = (u | u << 32) & 0x1f00000000ffffull;
    u = (u | u << 16) & 0x1f0000ff0000ffull;
    u = (u | u << 8) & 0x100f00f00f00f00full;
    u = (u | u << 4) & 0x10c30c30c30c30c3ull;
    u = (u | u << 2) & 0x1249249249249249ull;
    return (int64_t)u;
}

int64_t orc_morton(float x, float y, float z) {       /* bvh.cu:48-62 */
    int64_t ix = expand_bits(orc_float_to_21int(x));
    int64_t iy = expand_bits(orc_float_to_21int(y));
    int64_t iz = expand_bits(orc_float_to_21int(z));
    return ix | (iy << 1) | (iz << 2);
}

static inline int clz64(int64_t v) {                  /* __clzll, 0 -> 64 */
    return v == 0 ? 64 : __builtin_clzll((unsigned long long)v);
}

/* getTheOtherEnd (bvh.cu:64-99) */
static int other_end(const int64_t* keys, int idx, int size, int* dir, int* lmax) {
    int64_t left = idx == 0 ? -1 : keys[idx - 1];
    int64_t right = keys[idx + 1];
    int64_t self = keys[idx];
    int lc = clz64(left ^ self), rc = clz64(right ^ self);
    *dir = lc > rc ? -1 : 1;
    int minr = lc < rc ? lc : rc;
    *lmax = 2;
    int e = idx + *dir * *lmax;
    while (e >= 0 && e < size && clz64(self ^ keys[e]) > minr) {
        *lmax <<= 1;
        e = idx + *dir * *lmax;
    }
    int range = 0;
    for (int step = *lmax >> 1; step > 0; step >>= 1) {
        e = idx + (range + step) * *dir;
        if (e < 0 || e >= size) continue;
        if (clz64(self ^ keys[e]) > minr) range += step;
    }
    return idx + range * *dir;
}

/* findSplitPosition (bvh.cu:101-120) */
static int split_position(const int64_t* keys, int idx, int oe, int dir, int lmax) {
    int l = dir == -1 ? oe : idx, r = dir == -1 ? idx : oe;
    int delta = clz64(keys[l] ^ keys[r]);
    int split = 0;
    for (int t = lmax >> 1; t > 0; t >>= 1) {
        int pos = idx + dir * (split + t);
        if (pos < l || pos > r) continue;
        if (clz64(keys[idx] ^ keys[pos]) > delta) split += t;
    }
    return idx + split * dir;
}

typedef struct { int64_t key; int32_t fid; } key_fid;
static int cmp_key_fid(const void* a, const void* b) {  /* stable: tie -> fid order */
    const key_fid* x = (const key_fid*)a;
    const key_fid* y = (const key_fid*)b;
    if (x->key != y->key) return x->key < y->key ? -1 : 1;
    return x->fid < y->fid ? -1 : (x->fid > y->fid);
}

static void union_box(orc_node* nodes, int i, int n_int) {
    /* exact recursive union == computeBBox's level sweep (bvh.cu:219-302):
     * box = left.box; box.enclose(right.box) */
    int l = nodes[i].a, r = nodes[i].b;
    if (l < n_int) union_box(nodes, l, n_int);
    if (r < n_int) union_box(nodes, r, n_int);
    v3 lmin = V3(nodes[l].bmin[0], nodes[l].bmin[1], nodes[l].bmin[2]);
    v3 lmax = V3(nodes[l].bmax[0], nodes[l].bmax[1], nodes[l].bmax[2]);
    v3 rmin = V3(nodes[r].bmin[0], nodes[r].bmin[1], nodes[r].bmin[2]);
    v3 rmax = V3(nodes[r].bmax[0], nodes[r].bmax[1], nodes[r].bmax[2]);
    v3 mn = vmin(lmin, rmin), mx = vmax(lmax, rmax);
    nodes[i].bmin[0] = mn.x; nodes[i].bmin[1] = mn.y; nodes[i].bmin[2] = mn.z;
    nodes[i].bmax[0] = mx.x; nodes[i].bmax[1] = mx.y; nodes[i].bmax[2] = mx.z;
}

int orc_build_bvh(uint32_t nf, const float* wv, const uint32_t* idx, orc_node* nodes, int64_t* keys) {
    if (nf == 0) return -1;
    int n = (int)nf, n_int = n - 1;
    orc_node* leaves = nodes + n_int;
    key_fid* kf = (key_fid*)malloc(sizeof(key_fid) * (size_t)n);
    orc_node* tmp = (orc_node*)malloc(sizeof(orc_node) * (size_t)n);
    if (!kf || !tmp) { free(kf); free(tmp); return -2; }
    for (int i = 0; i < n_int; ++i) {                 /* BVHNode() ctor + initNodes box reset */
        memset(&nodes[i], 0, sizeof(orc_node));
        nodes[i].bmin[0] = nodes[i].bmin[1] = nodes[i].bmin[2] = FLT_MAX;
        nodes[i].bmax[0] = nodes[i].bmax[1] = nodes[i].bmax[2] = -FLT_MAX;
    }
    for (int f = 0; f < n; ++f) {                     /* initNodes (bvh.cu:128-148) */
        const float* p0 = wv + 3 * idx[3 * f];
        const float* p1 = wv + 3 * idx[3 * f + 1];
        const float* p2 = wv + 3 * idx[3 * f + 2];
        v3 a = V3(p0[0], p0[1], p0[2]), b = V3(p1[0], p1[1], p1[2]), c = V3(p2[0], p2[1], p2[2]);
        v3 mn = vmin(vmin(a, b), c), mx = vmax(vmax(a, b), c);
        v3 ctr = vscale(0.5f, vadd(mn, mx));          /* BBox::center (bvh.cuh:24) */
        kf[f].key = orc_morton(ctr.x, ctr.y, ctr.z);
        kf[f].fid = f;
        memset(&tmp[f], 0, sizeof(orc_node));
        tmp[f].a = f;
        tmp[f].bmin[0] = mn.x; tmp[f].bmin[1] = mn.y; tmp[f].bmin[2] = mn.z;
        tmp[f].bmax[0] = mx.x; tmp[f].bmax[1] = mx.y; tmp[f].bmax[2] = mx.z;
    }
    /* thrust::sort_by_key (bvh.cu:326), stable */
    qsort(kf, (size_t)n, sizeof(key_fid), cmp_key_fid);
    for (int j = 0; j < n; ++j) {
        keys[j] = kf[j].key;
        leaves[j] = tmp[kf[j].fid];
    }
    /* computeNodeRange (bvh.cu:150-217) */
    for (int i = 0; i < n_int; ++i) {
        int dir, lmax;
        int oe = other_end(keys, i, n, &dir, &lmax);
        int sp = split_position(keys, i, oe, dir, lmax);
        int hi = i > oe ? i : oe, lo = i < oe ? i : oe;
        if (dir == 1) {
            if (hi == sp + 1) { leaves[sp + 1].parent = (uint32_t)i; nodes[i].b = sp + n; }
            else              { nodes[sp + 1].parent = (uint32_t)i;  nodes[i].b = sp + 1; }
            if (lo == sp)     { leaves[sp].parent = (uint32_t)i;     nodes[i].a = sp + n - 1; }
            else              { nodes[sp].parent = (uint32_t)i;      nodes[i].a = sp; }
        } else {
            if (lo == sp - 1) { leaves[sp - 1].parent = (uint32_t)i; nodes[i].a = sp + n - 2; }
            else              { nodes[sp - 1].parent = (uint32_t)i;  nodes[i].a = sp - 1; }
            if (hi == sp)     { leaves[sp].parent = (uint32_t)i;     nodes[i].b = sp + n - 1; }
            else              { nodes[sp].parent = (uint32_t)i;      nodes[i].b = sp; }
        }
    }
    /* a parent chain that does not reach the root (runs of duplicate keys split
     * without a tie-break: a cycle) -- the library refuses it too (build.hip
     * kMaxLbvhDepth); the recursive union would not terminate */
    for (int i = 1; i < 2 * n - 1; ++i) {
        int cur = i, d = 0;
        while (cur != 0 && d < 4096) { cur = (int)nodes[cur].parent; ++d; }
        if (d >= 4096) { free(kf); free(tmp); return -3; }
    }
    if (n_int > 0) union_box(nodes, 0, n_int);
    free(kf);
    free(tmp);
    return 0;
}

/* ------------------------------------------------------------------------ */
/* Geometry queries (include/geometry_queries.h)                             */
/* ------------------------------------------------------------------------ */
typedef struct { v3 o, d; } ray_t;

/* rayHitBBox (:18-46): slab test on the infinite line; 1/dir per call */
static inline int hit_box(const ray_t* r, const float* bmin, const float* bmax) {
    v3 inv = V3(1.0f / r->d.x, 1.0f / r->d.y, 1.0f / r->d.z);
    float t0 = -FLT_MAX, t1 = FLT_MAX, a, b, s;
    a = (bmin[0] - r->o.x) * inv.x; b = (bmax[0] - r->o.x) * inv.x;
    if (a > b) { s = b; b = a; a = s; }
    if (t0 > b || a > t1) return 0;
    t0 = fmx(t0, a); t1 = fmn(t1, b);
    a = (bmin[1] - r->o.y) * inv.y; b = (bmax[1] - r->o.y) * inv.y;
    if (a > b) { s = b; b = a; a = s; }
    if (t0 > b || a > t1) return 0;
    t0 = fmx(t0, a); t1 = fmn(t1, b);
    a = (bmin[2] - r->o.z) * inv.z; b = (bmax[2] - r->o.z) * inv.z;
    if (a > b) { s = b; b = a; a = s; }
    if (t0 > b || a > t1) return 0;
    return 1;
}

/* rayHitTriangle (:65-86), Moller-Trumbore */
static inline int hit_tri(const ray_t* r, v3 v0, v3 v1, v3 v2, float* dist, float* u_o, float* v_o) {
    v3 e1 = vsub(v1, v0), e2 = vsub(v2, v0), t = vsub(r->o, v0);
    v3 p = vcross(r->d, e2), q = vcross(t, e1);
    float denom = vdot(p, e1);
    if (denom == 0.0f) return 0;
    float inv = 1.0f / denom;
    float u = vdot(p, t) * inv;
    float v = vdot(q, r->d) * inv;
    if (u < 0.0f || v < 0.0f || u + v > 1.0f) return 0;
    *u_o = u; *v_o = v;
    *dist = vdot(q, e2) * inv;
    return 1;
}

typedef struct {
    const orc_node* nodes;
    const float* wv;
    const float* wn;
    const uint32_t* idx;
    int n_faces;
} bvh_ctx;

typedef struct { int hit; float t, u, v; } hit_t;
typedef struct { uint64_t trav, inner, leaf, shade; } cnt_t;

/* traverseBVH (path_tracer.cu:61-107) */
static void traverse(const bvh_ctx* c, const ray_t* r, hit_t* h, cnt_t* cnt) {
    int stack[64];
    int sp = 1;
    stack[0] = 0;
    h->hit = -1; h->t = FLT_MAX; h->u = 0.0f; h->v = 0.0f;
    cnt->trav++;
    while (sp > 0) {
        int cur = stack[--sp];
        const orc_node* nd = &c->nodes[cur];
        if (cur >= c->n_faces - 1) {
            cnt->leaf++;
            int fid = nd->a;
            const float* p0 = c->wv + 3 * c->idx[3 * fid];
            const float* p1 = c->wv + 3 * c->idx[3 * fid + 1];
            const float* p2 = c->wv + 3 * c->idx[3 * fid + 2];
            float dist, u, v;
            if (hit_tri(r, V3(p0[0], p0[1], p0[2]), V3(p1[0], p1[1], p1[2]), V3(p2[0], p2[1], p2[2]), &dist, &u, &v)) {
                if (dist < h->t && dist > DELTA_F) {
                    h->t = dist; h->hit = fid; h->u = u; h->v = v;
                }
            }
        } else {
            cnt->inner++;
            int l = nd->a, rr = nd->b;
            if (hit_box(r, c->nodes[l].bmin, c->nodes[l].bmax)) stack[sp++] = l;
            if (hit_box(r, c->nodes[rr].bmin, c->nodes[rr].bmax)) stack[sp++] = rr;
        }
    }
}

int orc_trace_ray(const orc_node* nodes, uint32_t nf, const float* wv, const uint32_t* idx,
                  const float o[3], const float d[3], float* t_out, float uv_out[2]) {
    bvh_ctx c = {nodes, wv, NULL, idx, (int)nf};
    ray_t r = {V3(o[0], o[1], o[2]), V3(d[0], d[1], d[2])};
    hit_t h;
    cnt_t cnt = {0, 0, 0, 0};
    traverse(&c, &r, &h, &cnt);
    *t_out = h.t; uv_out[0] = h.u; uv_out[1] = h.v;
    return h.hit;
}

/* ------------------------------------------------------------------------ */
/* Shading (path_tracer.cu:137-225, sampler.h, delta_light.h, env_light.cuh) */
/* ------------------------------------------------------------------------ */
static inline v3 reflect_dir(v3 d, v3 n) {           /* :137-141 */
    return vsub(d, vscale(2.0f * vdot(d, n), n));
}

/* refract (:143-163) */
static inline v3 refract_dir(v3 d, v3 n, float ior, float* cos_i, float* eta, int* tir) {
    *cos_i = vdot(d, n);
    *eta = *cos_i > 0.0f ? ior : 1.0f / ior;
    n = *cos_i > 0.0f ? vneg(n) : n;
    *cos_i = fabsf(*cos_i);
    float sin2i = 1.0f - *cos_i * *cos_i;
    float sin2t = *eta * *eta * sin2i;
    if (sin2t >= 1.0f) { *tir = 1; return V3(0.0f, 0.0f, 0.0f); }
    float cos_t = sqrtf(1.0f - sin2t);
    return vadd(vscale(*eta, d), vscale(*cos_i * *eta - cos_t, n));
}

static inline float schlick(float cos_i, float eta) { /* :165-173 */
    float f0 = (1.0f - eta) / (1.0f + eta);
    f0 *= f0;
    float m = fclamp(1.0f - cos_i, 1.0f, 0.0f);
    float m2 = m * m;
    return f0 + (1.0f - f0) * m2 * m2 * m;
}

/* HemisphereCosine (sampler.h:75-89) */
static inline v3 hemisphere_cosine(uint32_t st[6], v3 n, int tm) {
    v3 xb = n.z == 0.0f ? V3(0.0f, 0.0f, 1.0f) : V3(1.0f, 0.0f, -n.x / n.z);
    xb = vdiv(xb, sqrtf(vnorm2(xb)));
    v3 zb = vcross(xb, n);
    float phi = 2.0f * PI_F * orc_uniform(st);
    float cos_t = sqrtf(orc_uniform(st));
    float sin_t = sqrtf(1.0f - cos_t * cos_t);
    float x = t_cos(tm, phi) * sin_t;
    float z = t_sin(tm, phi) * sin_t;
    float y = cos_t;
    return vadd(vadd(vscale(x, xb), vscale(y, n)), vscale(z, zb));
}

/* getNewDirection (:187-225); returns probability */
static inline float new_direction(v3 d, v3 n, const orc_material* m, uint32_t st[6], int tm,
                                  v3* next, float* atten) {
    if (m->eta > 0.0f) {
        int tir = 0;
        float eta, cos_i;
        v3 rf = refract_dir(d, n, m->eta, &cos_i, &eta, &tir);
        v3 rl = reflect_dir(d, n);
        float fr = tir ? 1.0f : schlick(cos_i, eta);
        *next = orc_uniform(st) < fr ? rl : rf;       /* CoinFlip (sampler.h:98-101) */
        *atten = 1.0f;
        return 1.0f;
    } else if (m->metallic > 0.0f) {
        *atten = 1.0f;
        *next = reflect_dir(d, n);
        return 1.0f;
    } else {
        float sign = vdot(d, n) > 0.0f ? -1.0f : 1.0f;
        n = vscale(sign, n);
        *next = hemisphere_cosine(st, n, tm);
        *atten = fabsf(vdot(*next, n)) / PI_F;
        float c = vdot(*next, n);                      /* HemishpereCosinePDF (sampler.h:91-96) */
        float f = c > 0.0f ? 1.0f : 0.0f;
        return (c / PI_F) * f;
    }
}

/* CalcDistAttenuation (delta_light.h:25-33) */
static inline v3 dist_atten(float dist, v3 rad) {
    float d2 = dist * dist;
    float att = 1.0f / (d2 + 1.0f);
    att *= fsq(fsat(1.0f - fsq(d2 * 0.01f)));
    return vscale(att, rad);
}

/* DeltaLight::sample + CalcDistAttenuation (delta_light.h:25-33, 35-130) */
static inline void light_sample(const orc_light* L, v3 p, v3* dir, v3* rad) {
    v3 color = V3(L->color[0], L->color[1], L->color[2]);
    float dist = 0.0f;
    *dir = V3(0.0f, 0.0f, 0.0f);
    *rad = V3(0.0f, 0.0f, 0.0f);
    if (L->type == 0) {
        v3 dd = vsub(V3(L->pos[0], L->pos[1], L->pos[2]), p);
        dist = sqrtf(vnorm2(dd));
        *dir = vdiv(dd, dist);
        *rad = vscale(L->intensity, color);
    } else if (L->type == 1) {
        *dir = vneg(V3(L->direction[0], L->direction[1], L->direction[2]));
        *rad = vscale(L->intensity, color);
        dist = 0.0f;
    } else if (L->type == 2) {
        v3 dd = vsub(V3(L->pos[0], L->pos[1], L->pos[2]), p);
        dist = sqrtf(vnorm2(dd));
        *dir = vdiv(dd, dist);
        float cos_t = vdot(vneg(*dir), V3(L->direction[0], L->direction[1], L->direction[2]));
        float fall = fsq(fsat(cos_t - L->cos_outer) * L->inv_cos_cone_diff);
        *rad = vscale(fall, vscale(L->intensity, color));
    }
    *rad = dist_atten(dist, *rad);
}

/* sampleEnvLights (:288-294) + Vec2UV (env_light.cuh:72-78) + point/clamp
 * tex2DLod level 0 (texture.cu:156-170). NULL env -> black (defined choice). */
static inline v3 env_lookup(const orc_env* env, v3 d, int tm) {
    if (!env || !env->rgba) return V3(0.0f, 0.0f, 0.0f);
    float u = t_atan2(tm, d.z, d.x) / (2.0f * PI_F);
    if (u < 0.0f) u += 1.0f;
    float v = 1.0f - t_acos(tm, fclamp(d.y, 1.0f, -1.0f)) / PI_F;
    int ix = (int)floorf(u * (float)env->w);
    int iy = (int)floorf(v * (float)env->h);
    ix = ix < 0 ? 0 : (ix > env->w - 1 ? env->w - 1 : ix);
    iy = iy < 0 ? 0 : (iy > env->h - 1 ? env->h - 1 : iy);
    const uint8_t* px = env->rgba + 4 * ((size_t)iy * (size_t)env->w + (size_t)ix);
    return vscale(1.0f / 255.0f, V3((float)px[0], (float)px[1], (float)px[2]));
}

/* Env importance sampling: the build's A15 re-derivation (env_light.cu:10-54
 * intends a 2-D piecewise-constant distribution), restating
 * libtpt's format (api.cpp build_env_is, trace.hip env_is_sample): piecewise
 * constant over blocks of B x B texels, B = 1 up to 2^17 texels and doubled
 * until the block grid has at most 2^17 cells.  Block weight = sum over its
 * texels (texel rows, then columns) of luma * sin(theta at the texel row's
 * centre), rows iy = 0 (bottom) .. h-1 as the lookup reads them; sequential
 * float prefix sums per block row and over block rows. */
typedef struct {
    float *cond, *row, *marg;
    float total;
    int b, bw, bh;
} env_is_t;

static int env_is_block(int w, int h) {
    int b = 1;
    while ((long long)((w + b - 1) / b) * (long long)((h + b - 1) / b) > (1ll << 17)) b *= 2;
    return b;
}

static void env_is_free(env_is_t* t) {
    free(t->cond);
    free(t->row);
    free(t->marg);
}

static void env_is_build(const orc_env* env, env_is_t* t) {
    const int w = env->w, h = env->h;
    const int b = env_is_block(w, h), bw = (w + b - 1) / b, bh = (h + b - 1) / b;
    t->b = b;
    t->bw = bw;
    t->bh = bh;
    t->cond = (float*)malloc(sizeof(float) * (size_t)bw * bh);
    t->row = (float*)malloc(sizeof(float) * (size_t)bh);
    t->marg = (float*)malloc(sizeof(float) * (size_t)bh);
    float* sw = (float*)malloc(sizeof(float) * (size_t)h);
    for (int iy = 0; iy < h; ++iy) {
        const float theta = PI_F * (1.0f - ((float)iy + 0.5f) / (float)h);
        float cw;
        parity_sincos(theta, &sw[iy], &cw);
    }
    float acc_rows = 0.0f;
    for (int by = 0; by < bh; ++by) {
        float acc = 0.0f;
        for (int bx = 0; bx < bw; ++bx) {
            float wb = 0.0f;
            const int ye = by * b + b < h ? by * b + b : h, xe = bx * b + b < w ? bx * b + b : w;
            for (int iy = by * b; iy < ye; ++iy)
                for (int ix = bx * b; ix < xe; ++ix) {
                    const uint8_t* px = env->rgba + 4 * ((size_t)iy * w + ix);
                    const float luma = (0.2126f * (float)px[0] + 0.7152f * (float)px[1]) + 0.0722f * (float)px[2];
                    wb = wb + luma * sw[iy];
                }
            acc = acc + wb;
            t->cond[(size_t)by * bw + bx] = acc;
        }
        t->row[by] = acc;
        acc_rows = acc_rows + acc;
        t->marg[by] = acc_rows;
    }
    t->total = acc_rows;
    free(sw);
}

static int lower_bound_f(const float* a, int n, float t) {
    int lo = 0, hi = n - 1;
    while (lo < hi) {
        int mid = (lo + hi) >> 1;
        if (a[mid] >= t) hi = mid; else lo = mid + 1;
    }
    return lo;
}

/* One env sample for a diffuse hit with incident-side normal nf: a block by
 * the two CDFs, a point uniformly inside it, the direction and the
 * contribution factor Le * cos / (pi * pdf) with pdf = (p_block * W * H /
 * block texels) / (2 pi^2 sin(theta)), p_block from the CDF steps; 0 when it
 * cannot contribute (the two uniforms are drawn either way). */
static int env_is_sample(const orc_env* env, const env_is_t* t, v3 nf, uint32_t st[6], int tm, v3* dir, v3* k_le) {
    const float x1 = orc_uniform(st);
    const float x2 = orc_uniform(st);
    const int W = env->w, H = env->h, B = t->b, BW = t->bw, BH = t->bh;
    const float t1 = x1 * t->total;
    const int by = lower_bound_f(t->marg, BH, t1);
    const float lo1 = by > 0 ? t->marg[by - 1] : 0.0f;
    const float hi1 = t->marg[by];
    const float f1 = fminf((t1 - lo1) / (hi1 - lo1), 0.99999994f);
    const float* cond = t->cond + (size_t)by * BW;
    const float rs = t->row[by];
    const float t2 = x2 * rs;
    const int bx = lower_bound_f(cond, BW, t2);
    const float lo2 = bx > 0 ? cond[bx - 1] : 0.0f;
    const float hi2 = cond[bx];
    const float f2 = fminf((t2 - lo2) / (hi2 - lo2), 0.99999994f);
    const int x0 = bx * B, y0 = by * B;
    const int wb = B < W - x0 ? B : W - x0, hb = B < H - y0 ? B : H - y0;
    const float u = ((float)x0 + f2 * (float)wb) / (float)W;
    const float v = ((float)y0 + f1 * (float)hb) / (float)H;
    float sp, cp, sth, cth;
    parity_sincos((2.0f * PI_F) * u, &sp, &cp);
    parity_sincos(PI_F * (1.0f - v), &sth, &cth);
    *dir = V3(sth * cp, cth, sth * sp);
    const float c = vdot(*dir, nf);
    const float pb = ((hi2 - lo2) / rs) * ((hi1 - lo1) / t->total);
    const float pdf = (pb * (((float)W * (float)H) / (float)(wb * hb))) / ((2.0f * PI_F * PI_F) * sth);
    if (!(sth > 0.0f) || !(c > 0.0f) || !(pdf > 0.0f) || !(pdf < 3.40282347e+38f)) return 0;
    /* Le: the texel the sample lies in (the lookup of dir up to rounding at texel edges) */
    (void)tm;
    const int fx = (int)(f2 * (float)wb), fy = (int)(f1 * (float)hb);
    const int ix = x0 + (fx < wb - 1 ? fx : wb - 1), iy = y0 + (fy < hb - 1 ? fy : hb - 1);
    const uint8_t* px = env->rgba + 4 * ((size_t)iy * (size_t)W + (size_t)ix);
    const v3 le = vscale(1.0f / 255.0f, V3((float)px[0], (float)px[1], (float)px[2]));
    const float k = c / (PI_F * pdf);
    *k_le = vscale(k, le);
    return 1;
}

/* Test hook: n env samples for normal nf from stream (seed, subsequence 0):
 * directions and contribution factors (zero when a sample cannot contribute). */
int orc_env_is_samples(const uint8_t* rgba, int w, int h, const float nf[3], uint64_t seed, int n,
                       float* dirs, float* k_le) {
    orc_env env = {rgba, w, h};
    env_is_t t;
    env_is_build(&env, &t);
    if (!(t.total > 0.0f)) { env_is_free(&t); return -1; }
    orc_xorwow_jump_matrices();
    uint32_t st[6];
    orc_xorwow_init(seed, 0, st);
    for (int i = 0; i < n; ++i) {
        v3 d = V3(0.0f, 0.0f, 0.0f), k = V3(0.0f, 0.0f, 0.0f);
        if (!env_is_sample(&env, &t, V3(nf[0], nf[1], nf[2]), st, 1, &d, &k)) k = V3(0.0f, 0.0f, 0.0f);
        dirs[3 * i] = d.x; dirs[3 * i + 1] = d.y; dirs[3 * i + 2] = d.z;
        k_le[3 * i] = k.x; k_le[3 * i + 1] = k.y; k_le[3 * i + 2] = k.z;
    }
    env_is_free(&t);
    return 0;
}

static const orc_material k_default_material = {
    {0.82f, 0.67f, 0.16f}, 0.0f, 0.0f, 0.0f, 0.0f, 0.5f, 0.5f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 1.0f};

typedef struct {
    bvh_ctx b;
    const orc_scene* s;
    const orc_env* env;
    const float* c2w;
    float vfov, aspect, tan_half;
    int W, H, spp, max_depth, tm;
    const env_is_t* is;   /* non-NULL: env next-event estimation (opt-in A15) */
} trace_ctx;

static inline const orc_material* mtl_of(const trace_ctx* c, int fid) {
    int obj = find_object(fid, c->s->lut, (int)c->s->n_objects);   /* mtlLinearSearch :125-135 */
    int mi = c->s->lut[obj].mtl;
    if (mi < 0 || (uint32_t)mi >= c->s->n_materials) return &k_default_material; /* App. A.9 */
    return &c->s->materials[mi];
}

/* One pixel of the trace kernel (path_tracer.cu:296-435). */
static void trace_pixel(const trace_ctx* c, int px, int py, uint32_t st[6], float out[3], cnt_t* cnt) {
    float sw, sh;
    sh = 2.0f * c->tan_half;                           /* sampleRays :50-52 */
    sw = c->aspect * sh;
    float p_st[64];
    v3 dir_st[64], att_st[64];
    const orc_material* m_st[64];
    v3 total = V3(0.0f, 0.0f, 0.0f);
    for (int s = 0; s < c->spp; ++s) {
        /* sampleRays (:42-59) */
        float ju = orc_uniform(st);
        float jv = orc_uniform(st);
        float lx = ju * 1.0f, ly = jv * 1.0f;          /* RectUniform * size(1,1) */
        lx = lx + (float)px; ly = ly + (float)py;
        lx = lx * (1.0f / (float)c->W); ly = ly * (1.0f / (float)c->H);
        lx = lx * sw; ly = ly * sh;
        v3 cd = vsub(V3(lx, ly, 0.0f), V3(0.5f * sw, 0.5f * sh, 1.0f));
        float in4[4] = {cd.x, cd.y, cd.z, 0.0f}, o4[4];
        mat4_vec4(c->c2w, in4, o4);
        ray_t ray;
        ray.d = vnormalize(V3(o4[0], o4[1], o4[2]));
        float org[4] = {0.0f, 0.0f, 0.0f, 1.0f};
        mat4_vec4(c->c2w, org, o4);
        ray.o = V3(o4[0], o4[1], o4[2]);

        int depth = 0;
        v3 rad = V3(0.0f, 0.0f, 0.0f);
        for (; depth < c->max_depth; ++depth) {
            hit_t h;
            traverse(&c->b, &ray, &h, cnt);
            if (h.hit < 0) {
                rad = env_lookup(c->env, ray.d, c->tm);
                break;
            }
            cnt->shade++;
            const uint32_t* tri = c->b.idx + 3 * h.hit;
            const float* n0 = c->b.wn + 3 * tri[0];
            const float* n1 = c->b.wn + 3 * tri[1];
            const float* n2 = c->b.wn + 3 * tri[2];
            float w = 1.0f - h.u - h.v;
            v3 nrm = vnormalize(vadd(vadd(vscale(w, V3(n0[0], n0[1], n0[2])),
                                          vscale(h.u, V3(n1[0], n1[1], n1[2]))),
                                     vscale(h.v, V3(n2[0], n2[1], n2[2]))));
            ray.o = vadd(ray.o, vscale(h.t, ray.d));
            const orc_material* m = mtl_of(c, h.hit);
            v3 ndir;
            float af;
            float prob = new_direction(ray.d, nrm, m, st, c->tm, &ndir, &af);
            v3 base = V3(m->base_color[0], m->base_color[1], m->base_color[2]);
            att_st[depth] = vscale(af, base);
            p_st[depth] = prob;
            /* sampleDeltaLights (:265-286) */
            v3 direct = V3(0.0f, 0.0f, 0.0f);
            for (uint32_t li = 0; li < c->s->n_lights; ++li) {
                v3 ldir, lrad;
                light_sample(&c->s->lights[li], ray.o, &ldir, &lrad);
                ray_t sr = {ray.o, ldir};
                hit_t sh2;
                traverse(&c->b, &sr, &sh2, cnt);
                if (sh2.hit == -1) direct = vadd(direct, vmul(base, lrad));
            }
            if (c->is && !(m->eta > 0.0f) && !(m->metallic > 0.0f)) {   /* env NEE (opt-in) */
                float sgn = vdot(ray.d, nrm) > 0.0f ? -1.0f : 1.0f;     /* getNewDirection's flip */
                v3 edir, ek;
                if (env_is_sample(c->env, c->is, vscale(sgn, nrm), st, c->tm, &edir, &ek)) {
                    ray_t sr = {ray.o, edir};
                    hit_t sh3;
                    traverse(&c->b, &sr, &sh3, cnt);
                    if (sh3.hit == -1) direct = vadd(direct, ek);
                }
            }
            if (!(m->eta >= 1.0f || m->metallic > 0.0f)) {  /* direct probe :387-401 */
                v3 pdir;
                float af2;
                new_direction(ray.d, nrm, m, st, c->tm, &pdir, &af2);
                ray.d = pdir;
                hit_t ph;
                traverse(&c->b, &ray, &ph, cnt);
                if (ph.hit >= 0) {
                    const orc_material* dm = mtl_of(c, ph.hit);
                    float e = dm->emission_factor;
                    dir_st[depth] = vadd(vmul(V3(1.0f, 1.0f, 1.0f), V3(e, e, e)), direct);
                } else {
                    dir_st[depth] = direct;
                }
            } else {
                dir_st[depth] = direct;
            }
            m_st[depth] = m;
            if (m->emission_factor > 0.0f) { depth++; break; }
            ray.d = ndir;
        }
        /* unwind (:416-430) */
        depth -= 1;
        while (depth >= 0) {
            const orc_material* m = m_st[depth];
            if (m->emission_factor > 0.0f) {
                float e = m->emission_factor;
                rad = vscale(e, V3(1.0f, 1.0f, 1.0f));
            } else {
                rad = vscale(1.0f / p_st[depth], vmul(vadd(dir_st[depth], rad), att_st[depth]));
            }
            depth -= 1;
        }
        total = vadd(total, rad);
    }
    out[0] = total.x; out[1] = total.y; out[2] = total.z;
}

static double now_ms(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec * 1e3 + (double)ts.tv_nsec * 1e-6;
}

static inline uint8_t to_uchar(float c) {           /* Spectrum::toUChar (material.h:74-81) */
    return (uint8_t)(fclamp(c * 255.0f, 255.0f, 0.0f));
}

int orc_render(const orc_scene* s, const orc_env* env, const orc_camera* cam, const orc_params* p,
               float* radiance, uint8_t* bgra, orc_counters* out) {
    if (!s || !cam || !p || s->n_faces == 0 || p->width <= 0 || p->height <= 0 || p->spp <= 0 ||
        p->max_depth <= 0 || p->max_depth > 64)
        return -1;
    orc_xorwow_jump_matrices();
    int W = p->width, H = p->height;
    int band_rows = p->band_rows > 0 ? p->band_rows : H;
    int band_count = p->band_count > 0 ? p->band_count : 1;
    int band_index = p->band_index;
    size_t nv = s->n_vertices, nf = s->n_faces;
    float* wv = (float*)malloc(sizeof(float) * 3 * nv);
    float* wn = (float*)malloc(sizeof(float) * 3 * nv);
    orc_node* nodes = (orc_node*)malloc(sizeof(orc_node) * (2 * nf - 1));
    int64_t* keys = (int64_t*)malloc(sizeof(int64_t) * nf);
    uint32_t* states = (uint32_t*)malloc(sizeof(uint32_t) * 6 * (size_t)W * (size_t)H);
    if (!wv || !wn || !nodes || !keys || !states) {
        free(wv); free(wn); free(nodes); free(keys); free(states);
        return -2;
    }
    memset(wv, 0, sizeof(float) * 3 * nv);
    memset(wn, 0, sizeof(float) * 3 * nv);
    orc_transform(s, wv, wn);
    {
        const int brc = orc_build_bvh((uint32_t)nf, wv, s->indices, nodes, keys);
        if (brc != 0) {
            free(wv); free(wn); free(nodes); free(keys); free(states);
            return brc;
        }
    }

    trace_ctx c;
    c.b.nodes = nodes; c.b.wv = wv; c.b.wn = wn; c.b.idx = s->indices; c.b.n_faces = (int)nf;
    c.s = s; c.env = env; c.c2w = cam->c2w; c.vfov = cam->vfov; c.aspect = cam->aspect;
    c.W = W; c.H = H; c.spp = p->spp; c.max_depth = p->max_depth; c.tm = p->trig_mode;
    c.tan_half = t_tan(p->trig_mode, cam->vfov * 0.5f);
    env_is_t is_tab = {NULL, NULL, NULL, 0.0f, 1, 0, 0};
    c.is = NULL;
    if (p->env_is && env && env->rgba) {
        env_is_build(env, &is_tab);
        if (is_tab.total > 0.0f) c.is = &is_tab;
    }

#ifdef _OPENMP
    if (p->threads > 0) omp_set_num_threads(p->threads);
#endif
    double t0 = now_ms();
    long npix = (long)W * (long)H;
#pragma omp parallel for schedule(static)
    for (long i = 0; i < npix; ++i) {
        int y = (int)(i / W);
        if ((y / band_rows) % band_count != band_index) continue;
        orc_xorwow_init(p->seed, (uint64_t)i, states + 6 * i);   /* setupRandSeed (:34-40) */
    }
    double t1 = now_ms();

    int tiles_x = (W + 15) / 16, tiles_y = (H + 15) / 16;
    uint64_t trav = 0, inner = 0, leaf = 0, shade = 0, pix = 0;
#pragma omp parallel for schedule(dynamic, 1) reduction(+ : trav, inner, leaf, shade, pix)
    for (long t = 0; t < (long)tiles_x * tiles_y; ++t) {
        int bx = (int)(t % tiles_x), by = (int)(t / tiles_x);
        cnt_t cnt = {0, 0, 0, 0};
        for (int ly = 0; ly < 16; ++ly) {
            int y = by * 16 + ly;
            if (y >= H || (y / band_rows) % band_count != band_index) continue;
            for (int lx = 0; lx < 16; ++lx) {
                int x = bx * 16 + lx;
                if (x >= W) continue;
                size_t off = (size_t)x + (size_t)y * (size_t)W;
                float tot[3];
                trace_pixel(&c, x, y, states + 6 * off, tot, &cnt);
                /* color[offset] += totalRad onto a zeroed buffer, then copyToFB's /spp */
                float col[3] = {0.0f + tot[0], 0.0f + tot[1], 0.0f + tot[2]};
                float inv = 1.0f / (float)p->spp;
                float r = col[0] * inv, g = col[1] * inv, b = col[2] * inv;
                if (radiance) { radiance[3 * off] = r; radiance[3 * off + 1] = g; radiance[3 * off + 2] = b; }
                if (bgra) {                             /* copyToFB (:451-471): flip, BGR, alpha untouched */
                    size_t fo = ((size_t)(H - y - 1) * (size_t)W + (size_t)x) * 4;
                    bgra[fo] = to_uchar(b); bgra[fo + 1] = to_uchar(g); bgra[fo + 2] = to_uchar(r);
                }
                pix++;
            }
        }
        trav += cnt.trav; inner += cnt.inner; leaf += cnt.leaf; shade += cnt.shade;
    }
    double t2 = now_ms();
    if (out) {
        out->traversals = trav; out->internal_visits = inner; out->leaf_tests = leaf;
        out->shade_hits = shade; out->pixels = pix;
        out->init_ms = t1 - t0; out->trace_ms = t2 - t1;
    }
    free(wv); free(wn); free(nodes); free(keys); free(states);
    env_is_free(&is_tab);
    return 0;
}

/* ------------------------------------------------------------------------ */
/* KAT entry points: the hot-path functions one at a time, pinned against the */
/* reference's own headers compiled here (oracle/_ref/ref_hot_kat,           */
/* tests/golden/ref_hot_kat.json).                                           */
/* ------------------------------------------------------------------------ */
int orc_kat_box_hit(const float o[3], const float d[3], const float bmin[3], const float bmax[3]) {
    ray_t r;
    r.o = V3(o[0], o[1], o[2]);
    r.d = V3(d[0], d[1], d[2]);
    return hit_box(&r, bmin, bmax);
}

int orc_kat_tri(const float o[3], const float d[3], const float v0[3], const float v1[3], const float v2[3],
                float out[3]) {
    ray_t r;
    r.o = V3(o[0], o[1], o[2]);
    r.d = V3(d[0], d[1], d[2]);
    return hit_tri(&r, V3(v0[0], v0[1], v0[2]), V3(v1[0], v1[1], v1[2]), V3(v2[0], v2[1], v2[2]), &out[0], &out[1],
                   &out[2]);
}

void orc_kat_light(const orc_light* L, const float p[3], float dir[3], float rad[3]) {
    v3 dd, rr;
    light_sample(L, V3(p[0], p[1], p[2]), &dd, &rr);
    dir[0] = dd.x; dir[1] = dd.y; dir[2] = dd.z;
    rad[0] = rr.x; rad[1] = rr.y; rad[2] = rr.z;
}

void orc_kat_dist_atten(float dist, float rgb[3]) {
    v3 r = dist_atten(dist, V3(rgb[0], rgb[1], rgb[2]));
    rgb[0] = r.x; rgb[1] = r.y; rgb[2] = r.z;
}

void orc_kat_to_uchar(const float rgb[3], uint8_t out[3]) {
    for (int i = 0; i < 3; ++i) out[i] = to_uchar(rgb[i]);
}

void orc_kat_default_material(orc_material* m) { *m = k_default_material; }
