// trace_dev.hpp -- device functions of the path-tracing hot path shared by the
// megakernel (trace.hip, k_trace) and the wavefront variant (wavefront.hip):
// the traversal (traverseBVH, path_tracer.cu:61-107) with its exactness guards,
// the triangle / box tests (geometry_queries.h:18-86), getNewDirection
// (path_tracer.cu:187-225), the delta lights (delta_light.h), the env lookup
// (path_tracer.cu:288-294) and env importance sampling (A15, opt-in).
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>

#include "../common/device_api.hpp"
#include "../common/ptrig.hpp"
#include "../common/rng.hpp"
#include "../common/tri_rec.hpp"
#include "../common/tpt_math.hpp"
#include "tpt.h"

#ifndef TPT_FAST
// 1: the tolerance-mode build of this file (Makefile trace_fast.hip.o, namespace
// tpt_fast, TPT_FLAG_FAST; DESIGN.md section 4 "Tolerance mode"): FMA
// contraction, FMA slab tests, the hardware's approximate reciprocal, sqrt and
// sin/cos, no culling guards.  The images then match the reference within SURVEY
// 8(d)'s per-channel tolerance, not bit for bit.
#define TPT_FAST 0
#endif
#ifndef TPT_FAST_SINCOS   // tolerance build: hardware v_sin/v_cos in the hemisphere sampler (0: the parity sincos)
#define TPT_FAST_SINCOS 1
#endif
#ifndef TPT_FAST_RCP      // tolerance build: v_rcp_f32 for 1/d and the triangle test's 1/denom (0: IEEE divides)
#define TPT_FAST_RCP 1
#endif
#ifndef TPT_PROBE_SHORTCUT
#define TPT_PROBE_SHORTCUT 1   // no emissive triangle: resolve direct probes in the shading pass
#endif
#ifndef TPT_PK_SLAB   // 4-wide visits: slab products as packed fp32 pairs (v_pk_add_f32 / v_pk_mul_f32)
#define TPT_PK_SLAB 0
#endif
typedef float f32x2 __attribute__((ext_vector_type(2)));
#ifndef TPT_PACKED_SORT   // 4-wide visits with 16-bit node ids: children sorted by packed (entry, link) keys
#define TPT_PACKED_SORT 0   // measured: C2 -1.6 %, C4 +1.5 %
#endif
#ifndef TPT_LEAF_KP
#define TPT_LEAF_KP 24    // run the triangle branch once this many lanes hold a parked leaf (or a.leaf_kb are blocked)
#endif
// Top 4-wide nodes staged in LDS (breadth-first prefix of inner4).  Off by
// default: measured on box 256 spp, 14 staged nodes cost 10 % (the per-visit
// LDS/global branch and LDS reads outweigh the shorter latency of the first
// levels); build with -DTPT_LDS_NODES_MAX=4096 to stage up to 32.
#ifndef TPT_LDS_NODES_MAX
#define TPT_LDS_NODES_MAX 0
#endif
#ifndef TPT_TRACE_WAVES
#define TPT_TRACE_WAVES 5   // min waves per SIMD requested from the register allocator
#endif

#ifndef TPT_TRACE_WAVES_IS
// The env importance-sampling variants (A15) carry the env sample's state across
// the shading pass: at 96 VGPRs (5 waves) they spilled 121 VGPRs to scratch;
// 4 waves give them 128.
#define TPT_TRACE_WAVES_IS 4
#endif
#ifndef TPT_TRACE_WAVES_PAIR
// pair-mode (delta-light) variants: at 5 waves (96 VGPRs) they spilled 38 VGPRs;
// C3 4096 spp, 4 waves: +6.4 % (7,220 -> 7,685 Mrays/s, 2 interleaved reps)
#define TPT_TRACE_WAVES_PAIR 4
#endif
#ifndef TPT_TRACE_WAVES_DRAIN
// DRAIN variants (launches that cannot fill the chip: a few waves per SIMD anyway)
#define TPT_TRACE_WAVES_DRAIN 4
#endif
#ifndef TPT_TRACE_WAVES_QUAD
#define TPT_TRACE_WAVES_QUAD 4   // four lanes per pixel (k_trace QUAD)
#endif
#ifndef TPT_GRAZE_HIT   // the grazing-hit rule (Culling: "Grazing hits"); 0 only to measure its cost
#define TPT_GRAZE_HIT 1
#endif
#ifndef TPT_TILE_POOL
// 1: one-lane-per-pixel, full-occupancy launches give each workgroup two
// adjacent 16x16 tiles; the second is a pixel pool its finished lanes draw
// from ("Round 4: N1").  0 (default): one tile per
// workgroup -- the pool measured C2 -15 %, C4 -39 %, C5 -5 % (workgroups live
// twice as long, so a launch's tail of heavy workgroups grows, while lanes
// without work were only 7.6 % of C2's lane-steps).
#define TPT_TILE_POOL 0
#endif
#ifndef TPT_ENV_FAST
#define TPT_ENV_FAST 1     // env texel indices from fp32 bounds, double trig only near texel edges (0: A/B builds)
#endif
#ifndef TPT_PROBE_INLINE
// 1: probe pass 1 inside the shading pass for <= 4 emitters (INL variants,
// emit_probe_inline; round 3).  0 (default): the conservative slab pre-test
// (probe_misses_emitters) resolves the probes that can hit no emitter in the
// shading pass and the others trace pass 1 as a traversal.
#define TPT_PROBE_INLINE 0
#endif
#ifndef TPT_SHARE_HEMI
#define TPT_SHARE_HEMI 0   // 1: the direct probe reuses the extension sample's hemisphere frame (new_direction)
#endif
#ifndef TPT_FMA_SLAB_UB
#define TPT_FMA_SLAB_UB 0   // 1: A/B builds only -- every slab as one FMA per bound (NOT exact: the
                            // upper bound of the inner-box FMA cut, DESIGN.md section 5 "Round 6")
#endif
#ifndef TPT_ENV_INLINE
#define TPT_ENV_INLINE 0   // 1: env_lookup inlined in every variant (A/B builds)
#endif

namespace tpt {

// LDS-typed pointers: the compiler then always emits ds_* accesses; a plain
// (generic) pointer that may meet a private or global one in a select is
// lowered to slower flat accesses.
#define TPT_LDS __attribute__((address_space(3)))
struct alignas(16) LdsF4 {   // float4 stand-in usable in LDS address space
    float x, y, z, w;
};

// rayHitBBox (geometry_queries.h:18-46) with 1/dir hoisted per ray (same
// values), written without branches: the reference returns false at the first
// axis whose slab misses the running interval; a sticky `miss` flag gives the
// same verdict (later axes cannot undo it) and the interval [t0, t1] -- used
// only by the ordered traversal, only on a hit -- is the reference's sequence
// of max/min updates.  NaN slabs propagate exactly as in the reference.
__device__ __forceinline__ bool box_hit(const V3& o, const V3& inv, float nx, float ny, float nz, float xx,
                                        float xy, float xz, float& t0, float& t1) {
    bool miss;
    float a, b, lo, hi;
    t0 = -kRealMax;
    t1 = kRealMax;
    a = (nx - o.x) * inv.x;
    b = (xx - o.x) * inv.x;
    lo = a > b ? b : a;
    hi = a > b ? a : b;
    miss = (t0 > hi) | (lo > t1);
    t0 = fmx(t0, lo);
    t1 = fmn(t1, hi);
    a = (ny - o.y) * inv.y;
    b = (xy - o.y) * inv.y;
    lo = a > b ? b : a;
    hi = a > b ? a : b;
    miss = miss | (t0 > hi) | (lo > t1);
    t0 = fmx(t0, lo);
    t1 = fmn(t1, hi);
    a = (nz - o.z) * inv.z;
    b = (xz - o.z) * inv.z;
    lo = a > b ? b : a;
    hi = a > b ? a : b;
    miss = miss | (t0 > hi) | (lo > t1);
    t0 = fmx(t0, lo);
    t1 = fmn(t1, hi);
    return !miss;
}

// ---------------------------------------------------------------------------
// Traversal (traverseBVH, path_tracer.cu:61-107), one node per step.  The
// current node is in a register; the LDS stack only holds deferred siblings.
//  ORDERED == false: the reference's visit order exactly (both children hit ->
//    right first, left deferred: :95-104), no culling.
//  ORDERED == true (default): nearer child first; on the 4-wide path a child is
//    skipped when its slab entry lies beyond the best hit or its exit lies
//    before Delta/2 -- boxes that cannot hold an accepted hit (Culling, below).
//    Exact ties (t == best) resolve to the larger leaf position, the triangle
//    the reference's right-first DFS meets first, so the winner is the
//    reference's.  The binary path (non-finite rays or boxes) does not cull.
//
//  Culling.  The reference tests every leaf whose box the infinite line passes
//  and keeps the least Moller-Trumbore t > Delta (geometry_queries.h:65-86,
//  path_tracer.cu:61-107), so a culled box must not hold a triangle whose
//  *computed* t would win -- and the computed t can lie outside the leaf box's
//  slab interval:
//   * sliver triangles (sin of the angle at v0 below 1e-3, e.g. the ball's
//     near-degenerate cap triangles; one with an edge of exactly zero length
//     has a determinant of exactly 0 and is never accepted, so it is not one):
//     the determinant is rounding noise and t is
//     arbitrary (measured: a hit at t = 2.15 on a leaf box spanning
//     [2.89, 2.95]).  The host lists them in up to 8 groups under a union
//     box; after every culled traversal, sliver_pass tests each sliver whose
//     exact leaf box the ray's line passes (the reference's rayHitBBox
//     verdict, no culling) under the same acceptance and tie rules -- exact
//     for any ray, one box test per ray in scenes with slivers (ball: 54 pole
//     triangles), nothing otherwise;
//   * hits on a shared edge accepted by barycentric rounding lie a few ulps
//     outside the triangle, which is a large t offset when the ray crosses the
//     box face at a grazing angle (measured: 5e-6 before the box entry at
//     |d.y| = 1e-3): the entry cull carries an absolute slack of cull_eps (4
//     ulps of the largest world coordinate) per unit of max |1/d|, on top of
//     a 1e-4 relative margin for t's own rounding.  (The same slack on the
//     exit cull found no further ray in the verification runs and cost tir
//     28 %: boxes just behind a secondary ray's origin are entered again.);
//   * rays grazing a triangle's plane (|cos| < ~1e-4) have the same
//     ill-conditioned t; origins exactly on an edge or vertex with such
//     directions diverge at ~1e-3 of adversarial rays (tests/test_gpu_cull.py):
//     a ray leaving a face within 1e-3 of its plane takes the uncull'd binary
//     path from the start;
//   * grazing hits (round 4): a ray that meets a shared edge at a grazing
//     angle to both faces gets a neighbour's t a long way outside that
//     neighbour's box (C5 at 2048 spp: 2 rays of 105 G, |cos| 4e-5 and 1e-4,
//     t 1.5e-4 and 3.9e-4 relative before the box); a closest hit (or probe
//     emitter hit) found by the culled walk on a face met within 1e-3 of its
//     plane sends the ray again through the uncull'd binary path.
//  Modes:
//   TM_CLOSEST  closest hit (extension and camera rays; probes in reference order)
//   TM_ANY      shadow rays stop at the first accepted triangle (only
//               hitIdx == -1 matters, :279)
//   TM_EMIT     direct probe, pass 1: the closest hit among emissive triangles
//               only -- the 4-wide path walks the tree over the emissive
//               triangles alone (a.emit_root); the binary path does not enter
//               children whose subtree holds no emitter (bit 30 of the link)
//   TM_OCCL     direct probe, pass 2 (after an emitter hit): any triangle that
//               beats that hit (t, then leaf position) ends the ray as
//               TM_OCCLUDED.  The probe only reads the closest hit's emission
//               (:394-396): an emitter hit nothing beats is the closest hit; if
//               something beats it, that triangle's emission is 0 and adds
//               exactly like a miss (the direct term is never -0).
// ---------------------------------------------------------------------------
enum : int { TM_CLOSEST = 0, TM_ANY = 1, TM_EMIT = 2, TM_OCCL = 3, TM_OCCLUDED = 4 };
constexpr int kLinkMask = 0x3fffffff;   // child link without its emitter bit

struct Trav {
    V3 o, d, inv;
    int node, sp, hpos, fid;
    int pend;   // parked leaf position (speculative traversal), -1: none
    float t, u, v;
    float lim;     // entry-cull bound: min(R, t * 1.0001 + cull_eps * max |1/d|) (Culling), kept with t
    int mode;      // TM_*
    bool fin;      // origin and 1/dir finite: no slab product can be NaN
};

__device__ __forceinline__ void trav_begin(Trav& r, V3 o, V3 d, int mode, bool boxes_finite = false,
                                           int emit_root = -1, float cull_eps = 0.0f, bool graze = false) {
    r.o = o;
    r.d = d;
    if (TPT_FAST && TPT_FAST_RCP)
        r.inv = v3(__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y), __builtin_amdgcn_rcpf(d.z));
    else
        r.inv = v3(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);   // rayHitBBox :20, hoisted
    r.node = 0;
    r.sp = 0;
    r.pend = -1;
    r.hpos = -1;
    r.fid = -1;
    r.t = kRealMax;
    r.u = 0.0f;
    r.v = 0.0f;
    r.mode = mode;
    // (graze: a ray leaving a surface within 1e-3 of its plane takes the uncull'd
    // binary path, "Culling" above)
    r.fin = boxes_finite & !graze & __builtin_isfinite(o.x) & __builtin_isfinite(o.y) & __builtin_isfinite(o.z) &
            __builtin_isfinite(r.inv.x) & __builtin_isfinite(r.inv.y) & __builtin_isfinite(r.inv.z);
    r.lim = kRealMax;   // t = FLT_MAX: nothing to cull against yet
    (void)cull_eps;
    if (mode == TM_EMIT && r.fin) {
        // probe pass 1 on the 4-wide path walks the emissive-triangle tree; without
        // one it becomes a plain closest-hit probe (the reference's own probe,
        // whose closest hit may then be a non-emitter adding +0)
        if (emit_root >= 0) r.node = emit_root;
        else r.mode = TM_CLOSEST;
    }
}

// Rays leaving a surface almost in its plane (Culling, "rays grazing a
// triangle's plane"): |cos(d, n)| < kGraze against the geometric unit normal of
// the face the ray leaves (shade record: n.x, n.y, the sign of n.z in n.x's
// lowest bit).  Adversarial rays that the culled walk resolves differently from
// the reference all leave their face at sin < 1e-4 (origins on its vertices and
// edges; tools/cull_diag.py); such rays take the binary path, which tests every
// leaf whose box the line passes (no culls), so they find the reference's hit.
// A face is carried as the pair (n.x bits, n.y); NaN n.x: no surface (camera
// rays, degenerate faces).
constexpr float kGraze = 1e-3f;
struct Surf {
    float x, y;
};
__device__ __forceinline__ Surf no_surface() { return Surf{__builtin_nanf(""), 0.0f}; }
__device__ __forceinline__ bool grazing(Surf g, V3 d) {
    if (!(g.x == g.x)) return false;
    const float zz = fmaxf(0.0f, 1.0f - g.x * g.x - g.y * g.y);
    const float z = (__float_as_uint(g.x) & 1u) ? -__builtin_amdgcn_sqrtf(zz) : __builtin_amdgcn_sqrtf(zz);
    const float dn = d.x * g.x + d.y * g.y + d.z * z;
    const float dd = d.x * d.x + d.y * d.y + d.z * d.z;
    return dn * dn < (kGraze * kGraze) * dd;   // (|n| = 1 to ~1e-7)
}

// Visit of inner node r.node: the child to descend into (-1: none) and, when
// both children are entered, the deferred one to push.
template <bool ORDERED>
__device__ __forceinline__ void inner_visit(const Trav& r, const float4* __restrict__ inner, int& next, bool& push,
                                            int& deferred) {
    const float4* nd = inner + 4 * r.node;
    const float4 q0 = nd[0], q1 = nd[1], q2 = nd[2], q3 = nd[3];
    float l0, l1, r0, r1;
    bool hl = box_hit(r.o, r.inv, q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, l0, l1);
    bool hr = box_hit(r.o, r.inv, q1.z, q1.w, q2.x, q2.y, q2.z, q2.w, r0, r1);
    const int lraw = __float_as_int(q3.x), rraw = __float_as_int(q3.y);
    const int lc = lraw & kLinkMask, rc = rraw & kLinkMask;
    if (ORDERED && r.mode == TM_EMIT) {   // probe pass 1: emitter subtrees only
        hl = hl & ((lraw >> 30) != 0);
        hr = hr & ((rraw >> 30) != 0);
    }
    const bool lfirst = ORDERED && (l0 < r0);   // reference order: right child first
    push = hl & hr;
    deferred = lfirst ? rc : lc;
    next = push ? (lfirst ? lc : rc) : (hl ? lc : (hr ? rc : -1));
}

// The same ordered visit through min/max slab arithmetic, for rays and boxes
// whose slab products cannot be NaN (finite origin, 1/dir and box bounds).
// Then lo <= hi on every axis and the reference's sequential test (miss as soon
// as max(-R, lo..) > min(R, hi..) for the axes seen so far) reduces to
// T0 = max(lo_x, lo_y, lo_z) <= T1 = min(R, hi_x, hi_y, hi_z) -- any crossed
// pair (lo_i > hi_j) is caught at the later of the two axes -- and the two
// culls fold in: hit & T0 <= lim & T1 >= Delta/2  <=>  max(T0, Delta/2) <=
// min(T1, R, lim), since Delta/2 > -R and lim > Delta/2.  Signed zeros may
// differ from the ternaries; only comparisons consume T0/T1.
__device__ __forceinline__ void slab_minmax(const V3& o, const V3& inv, float nx, float ny, float nz, float xx,
                                            float xy, float xz, float& t0, float& t1) {
#if TPT_FAST || TPT_FMA_SLAB_UB
    // (n - o) / d as one FMA per bound: n * (1/d) - o * (1/d) (the o * (1/d) terms
    // are common to every box a visit tests)
    const float ox = -(o.x * inv.x), oy = -(o.y * inv.y), oz = -(o.z * inv.z);
    const float ax = __builtin_fmaf(nx, inv.x, ox), bx = __builtin_fmaf(xx, inv.x, ox);
    const float ay = __builtin_fmaf(ny, inv.y, oy), by = __builtin_fmaf(xy, inv.y, oy);
    const float az = __builtin_fmaf(nz, inv.z, oz), bz = __builtin_fmaf(xz, inv.z, oz);
#else
    const float ax = (nx - o.x) * inv.x, bx = (xx - o.x) * inv.x;
    const float ay = (ny - o.y) * inv.y, by = (xy - o.y) * inv.y;
    const float az = (nz - o.z) * inv.z, bz = (xz - o.z) * inv.z;
#endif
    t0 = fmaxf(fmaxf(fminf(ax, bx), fminf(ay, by)), fminf(az, bz));
    t1 = fminf(fminf(fmaxf(ax, bx), fmaxf(ay, by)), fmaxf(az, bz));
}


// Traversal stack of one lane: slots [0, nlds) in LDS ([slot][lane], shared
// memory of the workgroup), deeper slots in private memory.  Deep stacks are
// rare (the ordered traversal keeps few deferred siblings), so scenes whose
// worst-case capacity exceeds the LDS budget (large trees, 32-bit ids) keep
// the LDS fast path for all but the deepest moments.
constexpr int kMaxStackSlots = 160 + 3;

// LDS slot addressing: [slot][lane].  TPT_STACK_PAIRED=1 pairs two 16-bit
// slots in one dword per lane ([slot/2][lane][slot%2]) so the 32 lanes of a
// ds_read/ds_write group touch 32 distinct banks instead of two lanes per bank
// (2-way conflicts whenever neighbouring lanes' stack depths differ).  Measured
// (3 interleaved reps): box 256 spp -2.5 %, C3 +2 %, C5 0 -- the extra
// address arithmetic costs more than the conflicts, so it is off.
#ifndef TPT_STACK_PAIRED
#define TPT_STACK_PAIRED 0
#endif
template <typename StackT>
__device__ __forceinline__ int stack_slot_offset(int i) {
    if (TPT_STACK_PAIRED && sizeof(StackT) == 2) return (i >> 1) * 512 + (i & 1);
    return i * 256;
}

// QS (four lanes per ray): one stack per quad, in its four lanes' columns --
// slot i at row i / 4, column 4q + i % 4 -- a quarter of the rows
template <typename StackT, bool QS = false>
struct LaneStack {
    TPT_LDS StackT* lds;   // this lane's (QS: its quad's first lane's) base: slot i at lds[off(i)]
    int nlds;
    StackT deep[kMaxStackSlots];
    __device__ static __forceinline__ int off(int i) {
        if constexpr (QS) return (i >> 2) * 256 + (i & 3);
        else return stack_slot_offset<StackT>(i);
    }
    __device__ __forceinline__ void put(int i, int v) {
        if (i < nlds) lds[off(i)] = (StackT)v;
        else deep[i - nlds] = (StackT)v;
    }
    __device__ __forceinline__ int get(int i) const {
        return i < nlds ? (int)lds[off(i)] : (int)deep[i - nlds];
    }
};

// 4-wide visit (ordered traversal, finite rays and boxes): tests the up to 4
// grandchildren of node r.node (inner4 layout, device_api.hpp) with the
// min/max slab test.  A grandchild's box lies inside its parent's (exact
// min/max unions) and the slab arithmetic is monotonic in the bounds, so a
// grandchild that passes implies its parent passes: the set of leaves reached
// is the binary traversal's.  Hit children are sorted by slab entry; the
// nearest is returned, the others (up to 3) are pushed farthest-first.  The
// stack region has 3 spare slots so all three writes are unconditional.
__device__ __forceinline__ float4 lds_f4(const TPT_LDS LdsF4* p) { return make_float4(p->x, p->y, p->z, p->w); }

// (packed v_pk_add/v_pk_mul slab math was measured 17 % slower: register-pair
// constraints outweigh the halved instruction count)

template <typename StackT, bool QS>
__device__ __forceinline__ int inner_visit4_q(const Trav& r, float4 q0, float4 q1, float4 q2, float4 q3, float4 q4,
                                              float4 q5, float4 q6, LaneStack<StackT, QS>& stk, int& sp);
template <typename StackT, bool QS>
__device__ __forceinline__ int inner_visit4(const Trav& r, const float4* __restrict__ inner4,
                                            const TPT_LDS LdsF4* snodes, int nlds_nodes, LaneStack<StackT, QS>& stk,
                                            int& sp) {
    float4 q0, q1, q2, q3, q4, q5, q6;
    if (TPT_LDS_NODES_MAX > 0 && r.node < nlds_nodes) {   // top levels, staged in LDS at kernel start
        const TPT_LDS LdsF4* nd = snodes + 8 * r.node;
        q0 = lds_f4(nd);
        q1 = lds_f4(nd + 1);
        q2 = lds_f4(nd + 2);
        q3 = lds_f4(nd + 3);
        q4 = lds_f4(nd + 4);
        q5 = lds_f4(nd + 5);
        q6 = lds_f4(nd + 6);
    } else {
        const float4* nd = inner4 + 8 * r.node;
        q0 = nd[0];
        q1 = nd[1];
        q2 = nd[2];
        q3 = nd[3];
        q4 = nd[4];
        q5 = nd[5];
        q6 = nd[6];
    }
    return inner_visit4_q(r, q0, q1, q2, q3, q4, q5, q6, stk, sp);
}
// the visit's arithmetic on the node's seven float4 (from global memory or LDS)
template <typename StackT, bool QS>
__device__ __forceinline__ int inner_visit4_q(const Trav& r, float4 q0, float4 q1, float4 q2, float4 q3, float4 q4,
                                              float4 q5, float4 q6, LaneStack<StackT, QS>& stk, int& sp) {
    float k0, k1, k2, k3, e0, e1, e2, e3;
#if TPT_PK_SLAB && !TPT_FAST
    // The slab products as packed fp32 pairs (v_pk_add_f32 / v_pk_mul_f32: two IEEE
    // operations per lane per instruction, the same rounding as the scalar ones, so
    // the same verdicts): a child's six bounds are three register pairs of the
    // loaded node -- (min.x, min.y), (min.z, max.x), (max.y, max.z) -- against the
    // ray's origin and 1/dir arranged the same way.
    {
        const f32x2 oa = {r.o.x, r.o.y}, ob = {r.o.z, r.o.x}, oc = {r.o.y, r.o.z};
        const f32x2 ia = {r.inv.x, r.inv.y}, ib = {r.inv.z, r.inv.x}, ic = {r.inv.y, r.inv.z};
        auto slab2 = [&](f32x2 pa, f32x2 pb, f32x2 pc, float& t0, float& t1) {
            const f32x2 a = (pa - oa) * ia, b = (pb - ob) * ib, c = (pc - oc) * ic;
            // a = (lo.x, lo.y), b = (lo.z, hi.x), c = (hi.y, hi.z) in slab-time units
            t0 = fmaxf(fmaxf(fminf(a.x, b.y), fminf(a.y, c.x)), fminf(b.x, c.y));
            t1 = fminf(fminf(fmaxf(a.x, b.y), fmaxf(a.y, c.x)), fmaxf(b.x, c.y));
        };
        slab2(f32x2{q0.x, q0.y}, f32x2{q0.z, q0.w}, f32x2{q1.x, q1.y}, k0, e0);
        slab2(f32x2{q1.z, q1.w}, f32x2{q2.x, q2.y}, f32x2{q2.z, q2.w}, k1, e1);
        slab2(f32x2{q3.x, q3.y}, f32x2{q3.z, q3.w}, f32x2{q4.x, q4.y}, k2, e2);
        slab2(f32x2{q4.z, q4.w}, f32x2{q5.x, q5.y}, f32x2{q5.z, q5.w}, k3, e3);
    }
#else
    slab_minmax(r.o, r.inv, q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, k0, e0);
    slab_minmax(r.o, r.inv, q1.z, q1.w, q2.x, q2.y, q2.z, q2.w, k1, e1);
    slab_minmax(r.o, r.inv, q3.x, q3.y, q3.z, q3.w, q4.x, q4.y, k2, e2);
    slab_minmax(r.o, r.inv, q4.z, q4.w, q5.x, q5.y, q5.z, q5.w, k3, e3);
#endif
    const float hi = r.lim;
    int i0 = __float_as_int(q6.x), i1 = __float_as_int(q6.y), i2 = __float_as_int(q6.z), i3 = __float_as_int(q6.w);
    const float hd = 0.5f * kDelta;
    // a link is -1 (no child) or an id with a flag in bit 30 (unused here)
    const bool h0 = (i0 >= 0) & (fmaxf(k0, hd) <= fminf(e0, hi));
    const bool h1 = (i1 >= 0) & (fmaxf(k1, hd) <= fminf(e1, hi));
    const bool h2 = (i2 >= 0) & (fmaxf(k2, hd) <= fminf(e2, hi));
    const bool h3 = (i3 >= 0) & (fmaxf(k3, hd) <= fminf(e3, hi));
    const int m = (int)h0 + (int)h1 + (int)h2 + (int)h3;
    if constexpr (TPT_PACKED_SORT && sizeof(StackT) == 2 && !QS) {
        // 16-bit node ids: one sort key per child, the clamped slab entry's top 16 bits
        // (sign, exponent, 7 mantissa bits; >= Delta/2, so never a denormal) over the
        // link's 16 bits, sorted as floats with one min and one max per comparator.
        // Entries within 1/128 of each other, and the children holding the origin
        // (entry < Delta/2), order by link instead -- the visit order only steers:
        // the walk's hit is the least t, then the larger leaf position, whatever the
        // order (Culling), so the frame is the same.
        const float inf = __builtin_inff();
        auto pk = [inf](bool h, float k, int i, float hd_) {
            return h ? __uint_as_float((__float_as_uint(fmaxf(k, hd_)) & 0xffff0000u) | ((uint32_t)i & 0xffffu)) : inf;
        };
        float p0 = pk(h0, k0, i0, hd), p1 = pk(h1, k1, i1, hd), p2 = pk(h2, k2, i2, hd), p3 = pk(h3, k3, i3, hd);
#define TPT_CXP(a, b)                    \
    {                                    \
        const float lo_ = fminf(a, b);   \
        b = fmaxf(a, b);                 \
        a = lo_;                         \
    }
        TPT_CXP(p0, p1)
        TPT_CXP(p2, p3)
        TPT_CXP(p0, p2)
        TPT_CXP(p1, p3)
        TPT_CXP(p1, p2)
#undef TPT_CXP
        const int np = m > 0 ? m - 1 : 0;
        const uint32_t u0 = __float_as_uint(np == 3 ? p3 : (np == 2 ? p2 : p1)), u1 = __float_as_uint(np == 3 ? p2 : p1),
                       u2 = __float_as_uint(p1);
        if (sp + 3 <= stk.nlds) {   // (StackT)u: the low 16 bits, the link
            stk.lds[stk.off(sp)] = (StackT)u0;
            stk.lds[stk.off(sp + 1)] = (StackT)u1;
            stk.lds[stk.off(sp + 2)] = (StackT)u2;
        } else {
            stk.put(sp, (int)(u0 & 0xffffu));
            stk.put(sp + 1, (int)(u1 & 0xffffu));
            stk.put(sp + 2, (int)(u2 & 0xffffu));
        }
        sp += np;
        return m > 0 ? (int)(__float_as_uint(p0) & 0xffffu) : -1;   // -1 when no child was entered
    }
    i0 &= kLinkMask;
    i1 &= kLinkMask;
    i2 &= kLinkMask;
    i3 &= kLinkMask;
    const float inf = __builtin_inff();
    k0 = h0 ? k0 : inf;
    k1 = h1 ? k1 : inf;
    k2 = h2 ? k2 : inf;
    k3 = h3 ? k3 : inf;
    i0 = h0 ? i0 : -1;
    i1 = h1 ? i1 : -1;
    i2 = h2 ? i2 : -1;
    i3 = h3 ? i3 : -1;
#define TPT_CX(ka, ia, kb, ib)          \
    {                                   \
        const bool sw = kb < ka;        \
        const float tk = sw ? kb : ka;  \
        kb = sw ? ka : kb;              \
        ka = tk;                        \
        const int ti = sw ? ib : ia;    \
        ib = sw ? ia : ib;              \
        ia = ti;                        \
    }
    TPT_CX(k0, i0, k1, i1)
    TPT_CX(k2, i2, k3, i3)
    TPT_CX(k0, i0, k2, i2)
    TPT_CX(k1, i1, k3, i3)
    TPT_CX(k1, i1, k2, i2)
#undef TPT_CX
    // push sorted[m-1] .. sorted[1] (m-1 entries), farthest at the bottom
    const int np = m > 0 ? m - 1 : 0;
    const int v0 = np == 3 ? i3 : (np == 2 ? i2 : i1), v1 = np == 3 ? i2 : i1;
    if (sp + 3 <= stk.nlds) {
        stk.lds[stk.off(sp)] = (StackT)v0;
        stk.lds[stk.off(sp + 1)] = (StackT)v1;
        stk.lds[stk.off(sp + 2)] = (StackT)i1;
    } else {
        stk.put(sp, v0);
        stk.put(sp + 1, v1);
        stk.put(sp + 2, i1);
    }
    sp += np;
    return i0;   // -1 when no child was entered
}

// rayHitTriangle (geometry_queries.h:65-86) on leaf position pos, e1/e2
// pre-gathered.  Returns true when an any-hit ray may stop.
// Moller-Trumbore core: rayHitTriangle's verdict (denom != 0, u, v >= 0,
// u + v <= 1) and its dist/u/v, branch-free (t/u/v are computed either way).
__device__ __forceinline__ bool tri_core(const V3& o, const V3& d, const V3& v0, const V3& e1, const V3& e2, float& t,
                                         float& u, float& v) {
    const V3 tv = o - v0;
    const V3 p = cross(d, e2);
    const V3 q = cross(tv, e1);
    const float denom = dot(p, e1);
    const float id = (TPT_FAST && TPT_FAST_RCP) ? __builtin_amdgcn_rcpf(denom) : 1.0f / denom;
    u = dot(p, tv) * id;
    v = dot(q, d) * id;
    t = dot(q, e2) * id;
    return (denom != 0.0f) & !((u < 0.0f) | (v < 0.0f) | (u + v > 1.0f));
}

__device__ __forceinline__ float cull_slack(const V3& inv, float cull_eps) {
    return cull_eps * fmaxf(fmaxf(fabsf(inv.x), fabsf(inv.y)), fabsf(inv.z));
}
template <bool ORDERED>
__device__ __forceinline__ bool leaf_test_q(Trav& r, const float4 q0, const float4 q1, const float4 q2, int pos,
                                            float cull_eps) {
    const V3 v0 = v3(q0.x, q0.y, q0.z), e1 = v3(q1.x, q1.y, q1.z), e2 = v3(q2.x, q2.y, q2.z);
    float t, u, v;
    const bool inside = tri_core(r.o, r.d, v0, e1, e2, t, u, v);
    const bool better = ORDERED ? ((t < r.t) | ((t == r.t) & (r.hpos >= 0) & (pos > r.hpos))) : (t < r.t);
    const bool take = inside & better & (t > kDelta);   // :83
    r.t = take ? t : r.t;
    if (ORDERED) r.lim = take ? fminf(kRealMax, t * 1.0001f + cull_slack(r.inv, cull_eps)) : r.lim;
    r.fid = take ? __float_as_int(q0.w) : r.fid;
    r.u = take ? u : r.u;
    r.v = take ? v : r.v;
    r.hpos = take ? pos : r.hpos;
    const bool occl = r.mode == TM_OCCL;
    r.mode = (take & occl) ? TM_OCCLUDED : r.mode;
    return take & ((r.mode == TM_ANY) | occl);
}
template <bool ORDERED>
__device__ __forceinline__ bool leaf_test(Trav& r, const float4* __restrict__ tri, int pos, float cull_eps) {
    const TriQ tq = tri_load(tri, pos);
    return leaf_test_q<ORDERED>(r, tq.q0, tq.q1, tq.q2, pos, cull_eps);
}

// Four lanes per ray (k_trace QUAD variants, tpt_debug_step_latency mode 2;
// DESIGN.md section 6, "Four lanes per ray").  The ray's traversal state is
// replicated on lanes 4q..4q+3 (every lane computes the same path); a 4-wide
// visit is split over them: lane k loads and tests child k alone (its 24-byte
// box, its link), leaf children are tested at once, each by its own lane, and
// the quad keeps the best hit under the tie rule (least t, then the larger leaf
// position: the order-independent result of the one-lane walk, so the hit is
// the same); the internal children that pass -- against the bound the leaves
// left -- are ranked by slab entry across the quad (DPP), the nearest is
// returned and the others are pushed farthest-first, each by its own lane, into
// the quad's stack (LaneStack QS).  A node passes the culls of the final
// bound whenever it passes them in the one-lane walk, so the sliver pass's
// premise holds.
template <int CTRL>
__device__ __forceinline__ int quad_mov(int v) {
    return __builtin_amdgcn_update_dpp(0, v, CTRL, 0xf, 0xf, false);
}
template <int CTRL>
__device__ __forceinline__ float quad_mov(float v) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xf, 0xf, false));
}
constexpr int kQuadXor1 = 0xb1, kQuadXor2 = 0x4e;   // quad_perm [1,0,3,2], [2,3,0,1]
// one butterfly step of the quad's best-hit reduction
template <int CTRL>
__device__ __forceinline__ void quad_best(Trav& r) {
    const float t2 = quad_mov<CTRL>(r.t), u2 = quad_mov<CTRL>(r.u), v2 = quad_mov<CTRL>(r.v), l2 = quad_mov<CTRL>(r.lim);
    const int p2 = quad_mov<CTRL>(r.hpos), f2 = quad_mov<CTRL>(r.fid), m2 = quad_mov<CTRL>(r.mode);
    const bool take = (t2 < r.t) | ((t2 == r.t) & (r.hpos >= 0) & (p2 > r.hpos));
    r.t = take ? t2 : r.t;
    r.u = take ? u2 : r.u;
    r.v = take ? v2 : r.v;
    r.lim = take ? l2 : r.lim;
    r.hpos = take ? p2 : r.hpos;
    r.fid = take ? f2 : r.fid;
    r.mode = take ? m2 : r.mode;
}
// The split visit of 4-wide node r.node (finite rays): returns the child to
// descend into (-1: none); stop when a leaf test ends an any-hit / occlusion walk.
template <typename StackT, bool QS>
__device__ __forceinline__ int inner_visit4_quad(Trav& r, const float4* __restrict__ inner4,
                                                 const float4* __restrict__ tri, int nint, float cull_eps,
                                                 LaneStack<StackT, QS>& stk, int& sp, bool& stop, uint32_t& c_leaf) {
    const int lane = (int)__lane_id(), k = lane & 3;
    const float* nf = (const float*)(inner4 + 8 * (size_t)r.node);
    const float2 b0 = *(const float2*)(nf + 6 * k), b1 = *(const float2*)(nf + 6 * k + 2),
                 b2 = *(const float2*)(nf + 6 * k + 4);
    const int link = ((const int*)nf)[24 + k];
    float kk, ee;
    slab_minmax(r.o, r.inv, b0.x, b0.y, b1.x, b1.y, b2.x, b2.y, kk, ee);
    const float hd = 0.5f * kDelta;
    const int id = link & kLinkMask;
    const bool h = (link >= 0) & (fmaxf(kk, hd) <= fminf(ee, r.lim));
    const bool lf = h & (id >= nint);
    stop = false;
#ifndef TPT_QUAD_EARLY
#define TPT_QUAD_EARLY 1
#endif
#if TPT_QUAD_EARLY
    // the leaf children's triangles in flight while the internal children are ranked
    // against the bound the node was entered with (strong-scaled C2 at N = 8, 2
    // interleaved reps: 245.0 / 245.7 ms against 249.8 / 250.1 with the ranking after
    // the leaf tests, which culls siblings beyond a leaf hit at the cost of the wait)
    TriQ tq = TriQ{make_float4(0.0f, 0.0f, 0.0f, 0.0f), make_float4(0.0f, 0.0f, 0.0f, 0.0f),
                   make_float4(0.0f, 0.0f, 0.0f, 0.0f)};
    if (lf) tq = tri_load(tri, id - nint);
    const bool in = h & (id < nint);
#else
    if (__ballot(lf) != 0ull) {
        int s = 0;
        if (lf) {
            ++c_leaf;
            s = leaf_test<true>(r, tri, id - nint, cull_eps) ? 1 : 0;
        }
        quad_best<kQuadXor1>(r);
        quad_best<kQuadXor2>(r);
        s |= quad_mov<kQuadXor1>(s);
        s |= quad_mov<kQuadXor2>(s);
        stop = s != 0;
    }
    // internal children against the bound the leaves left
    const bool in = !stop & h & (id < nint) & (fmaxf(kk, hd) <= fminf(ee, r.lim));
#endif
    const float key = in ? kk : __builtin_inff();
    const float c0 = quad_mov<0x00>(key), c1 = quad_mov<0x55>(key), c2 = quad_mov<0xaa>(key), c3 = quad_mov<0xff>(key);
    const int rank = ((c0 < key) | ((c0 == key) & (0 < k))) + ((c1 < key) | ((c1 == key) & (1 < k))) +
                     ((c2 < key) | ((c2 == key) & (2 < k))) + ((c3 < key) | ((c3 == key) & (3 < k)));
    const int n_in = __popcll((__ballot(in) >> (lane & ~3)) & 0xfull);
    if (in & (rank > 0)) stk.put(sp + n_in - 1 - rank, id);
    int near = (in & (rank == 0)) ? id : -1;
    near = max(near, quad_mov<kQuadXor1>(near));
    near = max(near, quad_mov<kQuadXor2>(near));
    sp += n_in > 0 ? n_in - 1 : 0;
#if TPT_QUAD_EARLY
    if (__ballot(lf) != 0ull) {
        int s = 0;
        if (lf) {
            ++c_leaf;
            s = leaf_test_q<true>(r, tq.q0, tq.q1, tq.q2, id - nint, cull_eps) ? 1 : 0;
        }
        quad_best<kQuadXor1>(r);
        quad_best<kQuadXor2>(r);
        s |= quad_mov<kQuadXor1>(s);
        s |= quad_mov<kQuadXor2>(s);
        stop = s != 0;
    }
#endif
    return near;
}

// Probe pass 1 over an emissive-triangle tree that is a single 4-wide node of
// leaves (<= 4 emitters), run inside the shading pass instead of a traversal:
// the node's leaf boxes by the same min/max slab test, then the triangle test
// of every passing leaf.  The closest hit under the ordered tie rule does not
// depend on the order the leaves are tested in, so r ends as the traversal
// would leave it.
template <bool HOIST = false>
__device__ __forceinline__ void emit_probe_inline(Trav& r, const float4* __restrict__ nd,
                                                  const float4* __restrict__ tri, int nint, uint32_t& c_leaf,
                                                  float cull_eps) {
    const float4 q0 = nd[0], q1 = nd[1], q2 = nd[2], q3 = nd[3], q4 = nd[4], q5 = nd[5], q6 = nd[6];
    if constexpr (HOIST) {
        // (DRAIN variants) the leaves' triangles are loaded together, before any
        // test: the node's links are the same for every lane, so these are
        // uniform loads issued at once instead of one round trip per leaf
        const float hi = kRealMax, hd = 0.5f * kDelta;
        const int i0 = __float_as_int(q6.x), i1 = __float_as_int(q6.y), i2 = __float_as_int(q6.z),
                  i3 = __float_as_int(q6.w);
        // (empty slots -- uniform -- skip their slab test; their verdict below is false)
        float k0 = 0.0f, k1 = 0.0f, k2 = 0.0f, k3 = 0.0f, e0 = 0.0f, e1 = 0.0f, e2 = 0.0f, e3 = 0.0f;
        if (i0 >= 0) slab_minmax(r.o, r.inv, q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, k0, e0);
        if (i1 >= 0) slab_minmax(r.o, r.inv, q1.z, q1.w, q2.x, q2.y, q2.z, q2.w, k1, e1);
        if (i2 >= 0) slab_minmax(r.o, r.inv, q3.x, q3.y, q3.z, q3.w, q4.x, q4.y, k2, e2);
        if (i3 >= 0) slab_minmax(r.o, r.inv, q4.z, q4.w, q5.x, q5.y, q5.z, q5.w, k3, e3);
        const int p0 = i0 >= 0 ? (i0 & kLinkMask) - nint : 0, p1 = i1 >= 0 ? (i1 & kLinkMask) - nint : 0,
                  p2 = i2 >= 0 ? (i2 & kLinkMask) - nint : 0, p3 = i3 >= 0 ? (i3 & kLinkMask) - nint : 0;
        const TriQ ta = tri_load(tri, p0), tb = tri_load(tri, p1);
        const float4 a0 = ta.q0, a1 = ta.q1, a2 = ta.q2;
        const float4 b0 = tb.q0, b1 = tb.q1, b2 = tb.q2;
        float4 c0 = a0, c1 = a1, c2 = a2, d0 = a0, d1 = a1, d2 = a2;
        if (i2 >= 0) {
            const TriQ tc = tri_load(tri, p2);
            c0 = tc.q0;
            c1 = tc.q1;
            c2 = tc.q2;
        }
        if (i3 >= 0) {
            const TriQ td = tri_load(tri, p3);
            d0 = td.q0;
            d1 = td.q1;
            d2 = td.q2;
        }
        if ((i0 >= 0) & (fmaxf(k0, hd) <= fminf(e0, hi))) { ++c_leaf; leaf_test_q<true>(r, a0, a1, a2, p0, cull_eps); }
        if ((i1 >= 0) & (fmaxf(k1, hd) <= fminf(e1, hi))) { ++c_leaf; leaf_test_q<true>(r, b0, b1, b2, p1, cull_eps); }
        if ((i2 >= 0) & (fmaxf(k2, hd) <= fminf(e2, hi))) { ++c_leaf; leaf_test_q<true>(r, c0, c1, c2, p2, cull_eps); }
        if ((i3 >= 0) & (fmaxf(k3, hd) <= fminf(e3, hi))) { ++c_leaf; leaf_test_q<true>(r, d0, d1, d2, p3, cull_eps); }
        return;
    }
    const float hi = kRealMax;   // nothing hit yet: r.t = FLT_MAX
    const float hd = 0.5f * kDelta;
    // the node is the same for every lane (links uniform): a child slot that is
    // empty (-1, fewer than 4 emitters) skips its slab test as a whole wave
    const int i0 = __float_as_int(q6.x), i1 = __float_as_int(q6.y), i2 = __float_as_int(q6.z),
              i3 = __float_as_int(q6.w);
    float k, e;
    if (i0 >= 0) {
        slab_minmax(r.o, r.inv, q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, k, e);
        if (fmaxf(k, hd) <= fminf(e, hi)) { ++c_leaf; leaf_test<true>(r, tri, (i0 & kLinkMask) - nint, cull_eps); }
    }
    if (i1 >= 0) {
        slab_minmax(r.o, r.inv, q1.z, q1.w, q2.x, q2.y, q2.z, q2.w, k, e);
        if (fmaxf(k, hd) <= fminf(e, hi)) { ++c_leaf; leaf_test<true>(r, tri, (i1 & kLinkMask) - nint, cull_eps); }
    }
    if (i2 >= 0) {
        slab_minmax(r.o, r.inv, q3.x, q3.y, q3.z, q3.w, q4.x, q4.y, k, e);
        if (fmaxf(k, hd) <= fminf(e, hi)) { ++c_leaf; leaf_test<true>(r, tri, (i2 & kLinkMask) - nint, cull_eps); }
    }
    if (i3 >= 0) {
        slab_minmax(r.o, r.inv, q4.z, q4.w, q5.x, q5.y, q5.z, q5.w, k, e);
        if (fmaxf(k, hd) <= fminf(e, hi)) { ++c_leaf; leaf_test<true>(r, tri, (i3 & kLinkMask) - nint, cull_eps); }
    }
}

// Direct-probe pre-test (path_tracer.cu:382-405; DESIGN.md section 5 "Probe
// pre-test").  The probe only adds the emission of its closest hit, and an
// emissive triangle can be that hit only if the probe's line passes its leaf
// box (rayHitBBox, :61-107), which lies inside one of the boxes a.emit_box
// (api.cpp emitter_boxes).  This is the slab test of those boxes with the
// hardware's approximate reciprocal (v_rcp_f32, 1 ulp) instead of the
// correctly rounded 1/d, and it answers "miss" only when the slab intervals
// fail to overlap by more than 2^-16 (|T0| + |T1|).  Every t it computes is
// within ~2^-21 relative of the exact (n - o) / d, and so is every t of the
// reference's float test (1/d rounded, then two roundings); the max/min over
// axes keeps that bound relative to |T0|, |T1| themselves, and an enclosing
// box's interval contains a leaf box's (a factor 2 on the |T| sum at most):
// a line whose leaf box the reference enters always fails this miss test, with
// a 30x margin.  A probe that misses every box has no emitter hit -- exactly
// the traversal's "no hit" of pass 1 (kNoProbe), whatever path or culls the
// traversal would take.  Non-finite reciprocals or products: traced.
__device__ __forceinline__ bool probe_misses_emitters(const TraceArgs& a, V3 o, V3 d) {
    if (a.n_emit_box <= 0) return false;
    const V3 inv = v3(__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y), __builtin_amdgcn_rcpf(d.z));
    bool miss = __builtin_isfinite(inv.x) & __builtin_isfinite(inv.y) & __builtin_isfinite(inv.z) &
                __builtin_isfinite(o.x) & __builtin_isfinite(o.y) & __builtin_isfinite(o.z);
    for (int k = 0; k < a.n_emit_box; ++k) {   // (uniform trip count)
        const float4 lo = a.emit_box[2 * k], hi = a.emit_box[2 * k + 1];
        float t0, t1;
        slab_minmax(o, inv, lo.x, lo.y, lo.z, hi.x, hi.y, hi.z, t0, t1);
        miss = miss & ((t0 - t1) > 0x1p-16f * (fabs_(t0) + fabs_(t1)));
    }
    return miss;
}

// Slivers (Culling): the triangles the culled traversal cannot be trusted to
// reach when they matter, re-tested after it against their exact leaf boxes.
// Group g: sliver_groups[2g] = (lo.xyz, first), [2g + 1] = (hi.xyz, count)
// over sliver_list, whose entry i is the sliver's exact leaf box (lo.xyz,
// leaf position | emissive << 30), (hi.xyz, 0) -- no dependent loads; groups
// 1.. are tested only when the ray passes group 0, the union of all of them.  Finite rays only (the
// binary path does not cull).  A sliver the traversal already tested is
// rejected by the tie rule the second time (same t and position).
// (Out of line and by value: a reference to the lane's traversal state would
// pin it to scratch memory for the whole kernel.)
struct SliverHit {
    float t, u, v;
    int fid, hpos, mode, tests;
};
__device__ __forceinline__ SliverHit sliver_scan(const float4* __restrict__ groups, const float4* __restrict__ list,
                                              int n_groups, const float4* __restrict__ tri, V3 o, V3 d, V3 inv,
                                              float cull_eps, SliverHit h) {
    Trav r;
    r.o = o;
    r.d = d;
    r.inv = inv;
    r.t = h.t;
    r.u = h.u;
    r.v = h.v;
    r.fid = h.fid;
    r.hpos = h.hpos;
    r.mode = h.mode;
    r.lim = fminf(kRealMax, h.t * 1.0001f + cull_slack(inv, cull_eps));
    int tests = 0;
    float t0, t1;
    // A sliver whose slab interval [t0, t1] has t1 >= hd and t0 <= lim (the
    // traversal's final cull bounds) was reached and tested by the traversal
    // itself; only the others can have been culled.
    const float hd = 0.5f * kDelta, lim = r.lim;
    {
        const float4 lo = groups[0], hi = groups[1];   // the union box
        if (!box_hit(o, inv, lo.x, lo.y, lo.z, hi.x, hi.y, hi.z, t0, t1) || (t0 >= hd && t1 <= lim)) n_groups = 0;
    }
    for (int g = 1; g < n_groups; ++g) {
        const float4 lo = groups[2 * g], hi = groups[2 * g + 1];
        if (!box_hit(o, inv, lo.x, lo.y, lo.z, hi.x, hi.y, hi.z, t0, t1)) continue;
        const int first = __float_as_int(lo.w), count = __float_as_int(hi.w);
        bool stop = false;
        for (int i = first; i < first + count && !stop; ++i) {
            const float4 bl = list[2 * i], bh = list[2 * i + 1];
            const int e = __float_as_int(bl.w);
            if (r.mode == TM_EMIT && !((e >> 30) & 1)) continue;   // probe pass 1: emitters only
            const int pos = e & kLinkMask;
            if (!box_hit(o, inv, bl.x, bl.y, bl.z, bh.x, bh.y, bh.z, t0, t1)) continue;   // rayHitBBox
            if (t1 >= hd && t0 <= lim) continue;   // not culled: already tested
            ++tests;
            stop = leaf_test<true>(r, tri, pos, cull_eps);   // any-hit / occluding: done
        }
        if (stop) break;
    }
    return SliverHit{r.t, r.u, r.v, r.fid, r.hpos, r.mode, tests};
}
__device__ __forceinline__ void sliver_pass(Trav& r, const TraceArgs& a, uint32_t& c_leaf) {
    if (!r.fin || r.mode == TM_OCCLUDED || (r.mode == TM_ANY && r.fid >= 0)) return;
    const SliverHit h = sliver_scan(a.sliver_groups, a.sliver_list, a.n_sliver_groups, a.tri, r.o, r.d, r.inv, a.cull_eps,
                                    SliverHit{r.t, r.u, r.v, r.fid, r.hpos, r.mode, 0});
    r.t = h.t;
    r.u = h.u;
    r.v = h.v;
    r.fid = h.fid;
    r.hpos = h.hpos;
    r.mode = h.mode;
    r.lim = fminf(kRealMax, r.t * 1.0001f + cull_slack(r.inv, a.cull_eps));
    c_leaf += (uint32_t)h.tests;
}

__device__ __forceinline__ V3 reflect_dir(V3 d, V3 n) { return d - (2.0f * dot(d, n)) * n; }   // :137-141

// HemisphereCosine's frame (sampler.h:75-89) for the incident-side normal:
// getNewDirection flips n toward the incident side (path_tracer.cu:216-218),
// then xBase = (1, 0, -n.x / n.z) / |.| (or (0, 0, 1)), zBase = xBase x n.
// The direct probe (:387-389) samples the same hemisphere as the bounce's
// extension ray (same incident direction and normal), so a shading pass
// computes the frame once and both samples use it (the same values as two
// evaluations: bit-identical).
// TPT_SHARE_HEMI 1 keeps the whole frame (6 floats) for the probe; 2 keeps
// only the two values that cost divides and a sqrt -- q = -n.x / n.z and
// r = 1 / |xBase| -- and rebuilds n, xBase = r * (1, 0, q) (or r * (0, 0, 1))
// from them: the same values, two live registers instead of six.
struct Hemi {
    V3 n, xb;
    float q, r;
};
__device__ __forceinline__ Hemi hemi_basis(V3 d, V3 n) {
    const float sign = dot(d, n) > 0.0f ? -1.0f : 1.0f;
    n = sign * n;
    const float q = n.z == 0.0f ? 0.0f : -n.x / n.z;
    V3 xb = n.z == 0.0f ? v3(0.0f, 0.0f, 1.0f) : v3(1.0f, 0.0f, q);
    const float r = 1.0f / fsqrt(norm2(xb));   // vdiv(xb, s) == (1 / s) * xb
    xb = r * xb;
    return Hemi{n, xb, q, r};
}
__device__ __forceinline__ Hemi hemi_rebuild(V3 d, V3 n, float q, float r) {
    const float sign = dot(d, n) > 0.0f ? -1.0f : 1.0f;
    n = sign * n;
    const V3 xb = r * (n.z == 0.0f ? v3(0.0f, 0.0f, 1.0f) : v3(1.0f, 0.0f, q));
    return Hemi{n, xb, q, r};
}

// getNewDirection (path_tracer.cu:187-225) for a material (eta, metallic).
// Returns the pdf; consumes 1 (dielectric), 0 (metal) or 2 (diffuse) uniforms.
// hb / hb_ok: the pass's hemisphere frame for (d, n), computed on first use.
__device__ __forceinline__ float new_direction(V3 d, V3 n, float eta_m, float metallic, uint32_t st[6], V3& next,
                                               float& atten, Hemi& hb, bool& hb_ok) {
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
    if (TPT_SHARE_HEMI == 2 && hb_ok) {
        hb = hemi_rebuild(d, n, hb.q, hb.r);
    } else if (!hb_ok) {
        hb = hemi_basis(d, n);
        hb_ok = true;
    }
    n = hb.n;
    const V3 xb = hb.xb;
    // HemisphereCosine (sampler.h:75-89)
    const V3 zb = cross(xb, n);
    float sp, cp;
#if TPT_FAST && TPT_FAST_SINCOS
    // v_sin_f32 / v_cos_f32 take revolutions: sin(2 pi u) directly
    const float u_phi = xorwow_uniform(st);
    const float cos_t = __builtin_amdgcn_sqrtf(xorwow_uniform(st));
    const float sin_t = __builtin_amdgcn_sqrtf(1.0f - cos_t * cos_t);
    sp = __builtin_amdgcn_sinf(u_phi);
    cp = __builtin_amdgcn_cosf(u_phi);
#else
    const float phi = 2.0f * kPi * xorwow_uniform(st);
    const float cos_t = fsqrt(xorwow_uniform(st));
    const float sin_t = fsqrt(1.0f - cos_t * cos_t);
    fsincos_2pi(phi, sp, cp);
#endif
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
// the texel indices of Vec2UV (env_light.cuh:72-78) through the double-precision
// atan2 / acos (ptrig.hpp): the exact path, cold (near texel edges only)
__device__ __forceinline__ int env_col_exact(float z, float x, int w) {
    float u = patan2_fast(z, x) / (2.0f * kPi);
    if (u < 0.0f) u += 1.0f;
    const int ix = (int)floorf(u * (float)w);
    return ix < 0 ? 0 : (ix > w - 1 ? w - 1 : ix);
}
__device__ __forceinline__ int env_row_exact(float y, int h) {
    const float v = 1.0f - pacos_fast(fclamp(y, 1.0f, -1.0f)) / kPi;
    const int iy = (int)floorf(v * (float)h);
    return iy < 0 ? 0 : (iy > h - 1 ? h - 1 : iy);
}
// Out of line where the lookup itself is inlined (the env importance-sampling
// variants): the double path's constants and temporaries then stay out of the
// kernel's register allocation (IS pair variant: 28 -> 8 spilled VGPRs at 128;
// the one-lane IS variants 12 -> 0).  COLD = false: inline (the out-of-line
// env_lookup_call of the other variants).
static __device__ __noinline__ int env_col_exact_call(float z, float x, int w) { return env_col_exact(z, x, w); }
static __device__ __noinline__ int env_row_exact_call(float y, int h) { return env_row_exact(y, h); }
#ifndef TPT_ENV_COLD_CALL
#define TPT_ENV_COLD_CALL 1
#endif
template <bool COLD>
__device__ __forceinline__ V3 env_lookup_inl(const uint32_t* __restrict__ env, int w, int h, V3 d) {
    // the texel indices from fp32 bounds (ptrig.hpp env_col_fast / env_row_fast:
    // the same indices as the double evaluation wherever they decide); the
    // double path only within ~1e-3 texel of an edge
    int ix = TPT_ENV_FAST ? env_col_fast(d.z, d.x, w) : -1;
    int iy = TPT_ENV_FAST ? env_row_fast(d.y, h) : -1;
    if (ix < 0) ix = (COLD && TPT_ENV_COLD_CALL) ? env_col_exact_call(d.z, d.x, w) : env_col_exact(d.z, d.x, w);
    if (iy < 0) iy = (COLD && TPT_ENV_COLD_CALL) ? env_row_exact_call(d.y, h) : env_row_exact(d.y, h);
    const uint32_t t = env[(size_t)iy * (size_t)w + (size_t)ix];
    return (1.0f / 255.0f) * v3((float)(t & 0xffu), (float)((t >> 8) & 0xffu), (float)((t >> 16) & 0xffu));
}
// Out of line in the variants without env importance sampling: inlined, its
// double-precision trig raised the register pressure of the whole kernel (C3
// 17 % slower at 5 waves; at 4 waves, 128 VGPRs, within 1-3 %).  The A15
// variants inline it (and env_is_sample): C3 with IS +25 % -- the calls'
// register saves went to scratch.
static __device__ __noinline__ V3 env_lookup_call(const uint32_t* __restrict__ env, int w, int h, V3 d) {
    return env_lookup_inl<false>(env, w, h, d);
}
template <bool INLINE>
__device__ __forceinline__ V3 env_lookup(const uint32_t* __restrict__ env, int w, int h, V3 d) {
    if constexpr (INLINE || TPT_ENV_INLINE) return env_lookup_inl<true>(env, w, h, d);
    else return env_lookup_call(env, w, h, d);
}

// Local row ly of this call's bands -> frame row.  Interleaved deal: local band
// k is global band k * band_count + band_index; an explicit deal (band_list,
// tpt_params.band_list) names local band k's global band.
__device__ __forceinline__ int band_of(int lb, int band_count, int band_index, const int32_t* band_list) {
    return band_list ? band_list[lb] : lb * band_count + band_index;
}
__device__ __forceinline__ int band_row(int ly, int band_rows, int band_count, int band_index,
                                        const int32_t* band_list) {
    return band_of(ly / band_rows, band_count, band_index, band_list) * band_rows + (ly % band_rows);
}

__device__ __forceinline__ unsigned long long wave_sum(uint32_t v) {
    unsigned long long s = v;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
    return s;
}

enum : int { PH_CAMERA = 0, PH_EXT = 1, PH_SHADOW = 2, PH_PROBE = 3, PH_ENVSHADOW = 4 };

// A15 env importance sampling, re-derived (TPT_FLAG_ENV_IS): a
// texel by the marginal (rows) then conditional (columns) CDF, the remapped
// uniforms as the position inside it, a direction by the inverse of Vec2UV
// (env_light.cuh:72-78) and its solid-angle pdf.  Returns the contribution
// factor Le * cos / (pi * pdf) for a diffuse hit with incident-side normal nf,
// or false when the sample cannot contribute (the two uniforms are drawn
// either way).  The oracle's env_is_sample is the same arithmetic.
// lower_bound (first i with a[i] >= t; n - 1 if none) of t = x * total over a
// nondecreasing prefix array a[0, n) whose last entry is total, through a guide
// table: g[k] = lower_bound(a, fl((k / K) * total)), k = 0..K, K a power of two.
// k = floor(x * K) is exact (a power-of-two scale) and x >= k / K, so t >=
// fl((k / K) * total) by monotone rounding: every a[j] with j < g[k] is < t, and
// the answer lies in [g[k], g[k + 1]].  The same index as a plain binary search
// over the whole array (the oracle's), in about two dependent loads instead of
// log2(n): the range's entries are loaded together and counted.
__device__ __forceinline__ int lower_bound_guided(const float* __restrict__ a, int n, float t, float x,
                                                  const int32_t* __restrict__ g, int K) {
    int k = (int)(x * (float)K);
    k = k < 0 ? 0 : (k > K ? K : k);
    int lo = g[k];
    int hi = k < K ? g[k + 1] : n - 1;
    hi = hi > n - 1 ? n - 1 : hi;
    while (hi - lo > 8) {   // rare: a bucket spanning many entries of tiny weight
        const int mid = (lo + hi) >> 1;
        if (a[mid] >= t) hi = mid;
        else lo = mid + 1;
    }
    int cnt = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const int i = lo + j;
        const float v = i < hi ? a[i] : t;
        cnt += v < t ? 1 : 0;
    }
    return lo + cnt;
}

// x1, x2: the two uniforms, drawn by the pixel's path lane in RNG order (pair
// mode hands them to the side lane with the bounce's shadow job).  The
// distribution is piecewise constant over blocks of B x B texels (api.cpp
// build_env_is): a block row by the marginal CDF, a block by that row's CDF,
// the remapped uniforms as the position inside the block (x0 + f2 * width,
// y0 + f1 * height in texels), and the pdf from the CDF steps the two
// searches stood on (the block's probability; no per-texel weight table, so
// the tables are 0.5 MB for a 2048 x 1024 map -- L2-resident):
// pdf = (p_block * W * H / (block texels)) / (2 pi^2 sin(theta)).
__device__ __forceinline__ bool env_is_sample(const TraceArgs& a, V3 nf, float x1, float x2, V3& dir, V3& k_le) {
    const int W = a.env_w, H = a.env_h, B = a.is_b, BW = a.is_bw, BH = a.is_bh;
    const float t1 = x1 * a.is_total;
    const int by = lower_bound_guided(a.is_marg, BH, t1, x1, a.is_guide_r, a.is_kr);
    const float lo1 = by > 0 ? a.is_marg[by - 1] : 0.0f;
    const float hi1 = a.is_marg[by];
    const float f1 = fminf((t1 - lo1) / (hi1 - lo1), 0.99999994f);
    const float* cond = a.is_cond + (size_t)by * (size_t)BW;
    const float rs = a.is_row[by];
    const float t2 = x2 * rs;
    const int bx = lower_bound_guided(cond, BW, t2, x2, a.is_guide_c + (size_t)by * (size_t)(a.is_kc + 1), a.is_kc);
    const float lo2 = bx > 0 ? cond[bx - 1] : 0.0f;
    const float hi2 = cond[bx];
    const float f2 = fminf((t2 - lo2) / (hi2 - lo2), 0.99999994f);
    const int x0 = bx * B, y0 = by * B;
    const int wb = min(B, W - x0), hb = min(B, H - y0);
    const float u = ((float)x0 + f2 * (float)wb) / (float)W;
    const float v = ((float)y0 + f1 * (float)hb) / (float)H;
    float sp, cp, sth, cth;
    fsincos_2pi((2.0f * kPi) * u, sp, cp);
    fsincos_2pi(kPi * (1.0f - v), sth, cth);
    dir = v3(sth * cp, cth, sth * sp);
    const float c = dot(dir, nf);
    const float pb = ((hi2 - lo2) / rs) * ((hi1 - lo1) / a.is_total);
    const float pdf = (pb * (((float)W * (float)H) / (float)(wb * hb))) / ((2.0f * kPi * kPi) * sth);
    if (!(sth > 0.0f) || !(c > 0.0f) || !(pdf > 0.0f) || !(pdf < kRealMax)) return false;
    // Le: the texel the sample lies in, (x0 + f2 * wb, y0 + f1 * hb) -- the texel the
    // lookup of dir (Vec2UV, env_light.cuh:72-78) finds, which inverts the same angles,
    // up to rounding at texel edges -- read without the atan2 / acos of the lookup
    const int ix = x0 + min((int)(f2 * (float)wb), wb - 1);
    const int iy = y0 + min((int)(f1 * (float)hb), hb - 1);
    const uint32_t tx = a.env[(size_t)iy * (size_t)W + (size_t)ix];
    const V3 le = (1.0f / 255.0f) * v3((float)(tx & 0xffu), (float)((tx >> 8) & 0xffu), (float)((tx >> 16) & 0xffu));
    const float k = c / (kPi * pdf);
    k_le = k * le;
    return true;
}
// TS_IDLE (pair mode): a side lane without a job, or a path lane waiting for
// its side lane's direct sum before the unwind -- neither traverses nor shades
enum : int { TS_DONE = 0, TS_TRAV = 1, TS_DEAD = 2, TS_IDLE = 3 };
enum : int { PH_WAIT = 5 };   // pair mode: path lane waiting to unwind

// Per-lane path records (path_tracer.cu:315-318), consumed by the unwind
// (:416-430).  The reference keeps attenuation = baseColor * atten (3 floats),
// p and the direct term (3) per depth.  Stored here, bit-equivalently:
//   w0 atten -- attenuation = atten * base is recomputed at unwind (same op);
//   p is atten itself (dielectric and metal: 1 and 1; diffuse with c > 0:
//     |c|/pi == (c/pi)*1) or a signed zero (c <= 0): a 2-bit kind in w1 bits
//     30-31 (a NaN c keeps its NaN, only the NaN's sign may differ);
//   w1 bits 0-14 material id;
//   no delta lights (rec_words == 2): the direct term is exactly
//     (1*e) + 0 of the material the probe ray hit, or 0 -- its id in w1 bits
//     15-29 (0x7fff: none);
//   delta lights (rec_words == 5): material id in bits 0-29, w2..w4 direct.
// Levels < a.rec_lds_levels live in LDS ([level][word][lane]); deeper ones in
// private memory.
constexpr uint32_t kNoProbe = 0x7fffu;

__device__ __forceinline__ uint32_t p_kind(float prob) {
    const uint32_t pb = __float_as_uint(prob);
    return pb == 0x80000000u ? 1u : (pb == 0u ? 2u : 0u);
}

// RS: LDS columns per workgroup (256: one per lane; 128 in pair mode, one per
// pixel -- the side lanes keep no records).
template <int MAXD, int RS = 256>
struct PathRecords {
    TPT_LDS float* lds;                        // this lane's column: word at lds[(level*words + w) * RS]
    int nlds, words;
    float deep[MAXD * 5];

    __device__ __forceinline__ void put(int level, int w, float v) {
        if (level < nlds) lds[(level * words + w) * RS] = v;
        else deep[level * 5 + w] = v;
    }
    __device__ __forceinline__ float get(int level, int w) const {
        return level < nlds ? lds[(level * words + w) * RS] : deep[level * 5 + w];
    }
    // word w of a level known to live in LDS (level < nlds), for records of
    // WORDS words per level (the caller's variant fixes it)
    template <int WORDS>
    __device__ __forceinline__ float lds_at(int level, int w) const {
        return lds[(level * WORDS + w) * RS];
    }
    // mk = material id | p-kind << 30; probe = material the probe hit (kNoProbe: none).
    // Pair mode (5 words, PACKED_PROBE): w1 = mk | probe << 15 as in the 2-word
    // records and w2..w4 = the delta lights' direct sum alone, written by whichever
    // lane traced the shadow rays; the unwind adds the probe's emission to it.
    template <bool PACKED_PROBE = false>
    __device__ __forceinline__ void put_dst(int level, uint32_t mk, uint32_t probe, V3 dst) {
        if (words == 2 || PACKED_PROBE) {
            put(level, 1, __uint_as_float(mk | (probe << 15)));
        } else {
            put(level, 1, __uint_as_float(mk));
            put(level, 2, dst.x);
            put(level, 3, dst.y);
            put(level, 4, dst.z);
        }
    }
};

}  // namespace tpt
