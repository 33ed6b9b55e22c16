// trace.hip -- the per-pixel path-tracing megakernel (src/path_tracer.cu:296-435)
// and the framebuffer resolve (copyToFB, :451-471).
//
// MI355X design (DESIGN.md "Trace kernel"):
//  * one lane per pixel, 16x16 pixel tile per 256-thread workgroup, each wave an
//    8x8 sub-tile (coherent primary rays);
//  * the reference's nested spp -> depth -> {extension, shadow*, probe} loops
//    become a per-lane state machine; every ray (primary, extension, shadow,
//    probe) is one traversal that the wave steps node by node;
//  * ballot-driven postponed shading: a wave keeps stepping while at least
//    `refill` of its lanes are still traversing, then the finished lanes shade,
//    advance their path and set up their next ray while the others keep their
//    traversal state in registers -- the wave pays the average traversal length
//    of its lanes, not the longest, and every pixel still consumes its own
//    XORWOW stream in the reference's order;
//  * ordered traversal over 4-wide nodes (an SAH tree over the reference's
//    exact leaf boxes, host/wide_bvh.cpp; 128 B: seven 16-B loads per visit)
//    with an exact min/max slab test for finite rays, the exactness guards of
//    "Culling" below, and speculative leaf postponement; the binary nodes and
//    the reference's ternary slab test serve the reference visit order and
//    rays with a non-finite origin or 1/dir;
//  * LDS per workgroup: the material table, the traversal stack ([slot][lane],
//    16-bit ids when the tree allows; deepest slots private when it does not
//    fit) and as many path-record levels as fit (2 words per bounce without
//    delta lights); deeper records in private memory;
//  * kernel variants by template: no-lights / delta lights, material table in
//    LDS or not, 16/32-bit stack ids, record depth 8/64; the reference order
//    and the opt-in env importance sampling have one general variant each;
//  * triangles are pre-gathered (v0, e1, e2, fid: three 16-B loads).
#include "trace_dev.hpp"

namespace tpt {
#ifdef TPT_VERIFY_CULL
template <bool ORDERED>
__device__ __forceinline__ void trav_lane(Trav& r, const TraceArgs& a, LaneStack<int>& stk, uint32_t& c_ovf);
// Diagnostic builds (-DTPT_VERIFY_CULL): every ray the render traversed is traced
// again in the reference's visit order (no culling) and compared with what the
// render used -- closest hit (fid, t, u, v bits), shadow verdict, or the probe's
// emission.  Mismatches go to a.debug_waves, 16 words each, counted in
// counters[24] (at most kVerifyCap logged).  The image is the render's.
constexpr unsigned long long kVerifyCap = 4096;
__device__ __noinline__ void verify_ray(const TraceArgs& a, const Trav& r, int phase, const float4* mtl) {
    Trav q;
    trav_begin(q, r.o, r.d, TM_CLOSEST);
    LaneStack<int> vs;
    vs.lds = nullptr;
    vs.nlds = 0;
    uint32_t ovf = 0;
    trav_lane<false>(q, a, vs, ovf);
    bool bad;
    if (r.mode == TM_ANY) {
        bad = (q.fid >= 0) != (r.fid >= 0);
    } else if (r.mode == TM_CLOSEST && phase != 3) {
        bad = (q.fid != r.fid) || (__float_as_uint(q.t) != __float_as_uint(r.t)) ||
              (__float_as_uint(q.u) != __float_as_uint(r.u)) || (__float_as_uint(q.v) != __float_as_uint(r.v));
    } else {   // probe: only the closest hit's emission is read (:394-396)
        const float er = q.fid >= 0 ? mtl[2 * __float_as_int(a.shade[3 * q.fid].w)].w : 0.0f;
        const float eo = (r.fid >= 0 && r.mode != TM_OCCLUDED) ? mtl[2 * __float_as_int(a.shade[3 * r.fid].w)].w : 0.0f;
        bad = er != eo;
    }
    if (!bad) return;
    const unsigned long long k = atomicAdd(&a.counters[24], 1ull);
    if (k >= kVerifyCap || !a.debug_waves) return;
    unsigned long long* o = a.debug_waves + 16 * k;
    o[0] = (unsigned long long)r.mode;
    o[1] = (unsigned long long)phase;
    o[2] = (unsigned long long)(long long)r.fid;
    o[3] = (unsigned long long)(long long)q.fid;
    o[4] = __float_as_uint(r.t);
    o[5] = __float_as_uint(q.t);
    o[6] = __float_as_uint(r.o.x);
    o[7] = __float_as_uint(r.o.y);
    o[8] = __float_as_uint(r.o.z);
    o[9] = __float_as_uint(r.d.x);
    o[10] = __float_as_uint(r.d.y);
    o[11] = __float_as_uint(r.d.z);
    o[12] = (unsigned long long)(long long)r.hpos;
    o[13] = (unsigned long long)(long long)q.hpos;
    o[14] = __float_as_uint(r.u);
    o[15] = (unsigned long long)(r.fin ? 1u : 0u) | ((unsigned long long)__float_as_uint(r.lim) << 32);   // culled path?, final entry-cull bound
}
#endif

// Pair mode's mid-pass exchange (round 6): 1 in every pair variant, 2 only with env
// importance sampling, 0 off (the side lanes' sums then reach their path lanes at the
// end of the pass only).
#ifndef TPT_PAIR_MID
#define TPT_PAIR_MID 2
#endif

// Shadow rays' first step in the pass (round 6): a fresh shadow ray (delta light or env
// sample) takes its root visit before the wave enters the traversal loop; when no
// child of the root passes, the ray is finished there, and the wave runs its shading
// pass again before traversing, so a side lane's next shadow ray (or its direct sum)
// follows at once instead of after the traversal round.  The same visit, the same
// counters: the frame is the same.  1 on, 0 off.
#ifndef TPT_SHADOW_FIRST
#define TPT_SHADOW_FIRST 0
#endif

// LIGHTS == false (no delta lights, packed 2-word records): the shadow-ray
// state (direct term, normal, light index, incoming direction -- r.d during an
// extension ray) is dead across traversals and drops out of the registers.
//
// PAIR (pair mode, delta-light scenes; DESIGN.md section 5 "Pair mode"): two
// lanes per pixel, 8x4 pixels per wave.  The even lane runs the pixel's path
// exactly as above; the odd lane is its side lane: when the path lane shades a
// hit while its side lane is idle, it hands that bounce's shadow rays
// (origin, material, level) to the side lane and goes straight on to the
// probe and the next extension ray.  The side lane traces the level's shadow
// rays in light order, sums the direct term exactly as the path lane would
// and hands it back; the path lane stores it in that level's record and waits
// for it, if need be, before the unwind.  Shadow rays consume no random
// numbers, so every pixel's XORWOW stream is consumed as in the reference, and
// each level's direct term is the same sum in the same order: the image is
// bit-identical.  A pixel's sample chain then pays one traversal per bounce
// instead of 1 + lights, which is what bounds tail-heavy frames (C3).
template <int MAXD, bool ORDERED, bool LIGHTS, bool MTL_LDS, typename StackT, bool ENVIS = false, bool INL = false,
          bool PAIR = false, bool DRAIN = false, bool QUAD = false, bool NOEMIT = false>
__global__ __launch_bounds__(256, ENVIS ? TPT_TRACE_WAVES_IS
                                        : (PAIR ? TPT_TRACE_WAVES_PAIR
                                                : (QUAD ? TPT_TRACE_WAVES_QUAD
                                                        : (DRAIN ? TPT_TRACE_WAVES_DRAIN : TPT_TRACE_WAVES))))
void k_trace(TraceArgs a) {
    static_assert(!PAIR || (ORDERED && LIGHTS), "pair mode: ordered variants with 5-word records");
    static_assert(!QUAD || (ORDERED && !LIGHTS && !PAIR && !ENVIS && !DRAIN), "four lanes per pixel: one-lane logic");
    extern __shared__ __attribute__((aligned(16))) char lds[];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    // grid y interleaves the frames of a batch: consecutive workgroups render the
    // same screen rows of successive frames, so the resident tiles keep the
    // screen locality of a single frame (node reuse in L1/L2)
    const int nfr = a.n_frames > 0 ? a.n_frames : 1;
    int bx = (int)blockIdx.x, by = (int)blockIdx.y;
    // XCD runs (scenes larger than an XCD's 4 MiB L2): blocks b and b + 8 share
    // an XCD.  Within each row of workgroups XCD k gets runs of xcd_run
    // adjacent tiles instead of every 8th tile, so its resident tiles see less
    // of the scene; the run-to-XCD assignment rotates by one every row so every
    // XCD gets every column over the launch (a permutation of the row's tiles;
    // the host checks that xcd_run divides gridDim.x / 8).  C5 +4 %; on box,
    // whose scene is L2-resident anyway, runs cost 2-7 % (the heavy middle
    // columns then load fewer XCDs), so it stays off there.  A launch of few rows
    // (a strong-scaled share: 6 rows of workgroups per set) does not complete the
    // rotation, and its heavy columns would load the same XCDs in every chunk of
    // the set's spp: the host rotates each chunk by one more (xcd_rot), so over 8
    // chunks every XCD takes every tile once.
    if (a.xcd_run > 0) {
        const int g = a.xcd_run, k = ((bx & 7) + by + a.xcd_rot) & 7, m = bx >> 3;
        bx = ((m / g) * 8 + k) * g + m % g;
    }
    const int frame = by % nfr;
    // Pixel pool (round 4; DESIGN.md section 5 "Round 4: N1"): workgroup b renders
    // tiles 2b and 2b + 1 of its row.  Its lanes start on the first; a lane whose
    // pixel has run all its samples stores it and takes the next unclaimed pixel
    // of the second (an LDS counter), so the lanes of cheap pixels (misses, walls)
    // keep working while their wave's heavy pixels finish.  Every pixel still runs
    // all its samples in order on one lane with its own XORWOW stream: the image
    // is bit-identical to one tile per workgroup.
    const bool pool = !PAIR && !DRAIN && TPT_TILE_POOL && a.tile_pool > 0;
    const int tx = pool ? 2 * bx : bx;
    // pair mode: lane 2q (path) and 2q + 1 (side) serve pixel q of the wave's 8x4 tile
    const bool side = PAIR && (lane & 1);
    // QUAD: lanes 4q..4q+3 all run pixel q of the wave's 4x4 tile (8x8 pixels per
    // workgroup) with the same state; lane 4q (lead) counts and stores it
    const bool lead = !QUAD || (lane & 3) == 0;
    const int pl = PAIR ? (lane >> 1) : (QUAD ? (lane >> 2) : lane);   // pixel slot in the wave
    int x = QUAD ? tx * 8 + (wave & 1) * 4 + (pl & 3) : tx * 16 + (wave & 1) * 8 + (pl & 7);
    const int ly = PAIR   ? (by / nfr) * 8 + (wave >> 1) * 4 + (pl >> 3)
                   : QUAD ? (by / nfr) * 8 + (wave >> 1) * 4 + (pl >> 2)
                          : (by / nfr) * 16 + (wave >> 1) * 8 + (pl >> 3);
    int y = band_row(ly, a.band_rows, a.band_count, a.band_index, a.band_list);
    const bool pixel = x < a.width && ly < a.band_height && y < a.height;
    // cost-balanced deals (tpt_params.band_cost): the wave's life in s_memrealtime
    // ticks, charged to the global band of its first row (lane 0's)
    const unsigned long long t_cost0 = a.band_cost ? wall_clock64() : 0ull;
    bool active = pixel && !side;   // owns the pixel's RNG stream and sums
    uint32_t c_trav = 0, c_inner = 0, c_wide = 0, c_leaf = 0, c_shade = 0, c_ovf = 0;
    uint32_t c_local = 0;   // rays resolved in the shading pass without a BVH traversal
    const size_t npix = (size_t)a.width * (size_t)a.height;
    size_t off = active ? (size_t)x + (size_t)y * (size_t)a.width : 0;
    // frame batch: each frame owns its own RNG and accumulator planes
    uint32_t* const g_rng = a.rng + (size_t)frame * 6 * npix;
    float* const g_acc = a.accum + (size_t)frame * 3 * npix;
    const int nint = a.n_faces - 1;
    // Material table in LDS when small (every shading, probe and unwind step
    // reads it; LDS latency instead of a dependent global load).  The copy is
    // the kernel's only barrier.
    TPT_LDS char* slds = (TPT_LDS char*)lds;
    TPT_LDS LdsF4* smtl = (TPT_LDS LdsF4*)(slds + a.lds_mtl_offset);
    if constexpr (MTL_LDS) {
        for (int i = tid; i < 2 * (a.n_materials + 1); i += 256) {
            const float4 m = a.mtl[i];
            smtl[i].x = m.x;
            smtl[i].y = m.y;
            smtl[i].z = m.z;
            smtl[i].w = m.w;
        }
    }
    // the top 4-wide nodes (breadth-first prefix of inner4): every ray starts
    // there, so their loads become LDS reads
    TPT_LDS LdsF4* snodes = (TPT_LDS LdsF4*)(slds + a.lds_nodes_offset);
    for (int i = tid; i < 8 * a.lds_nodes; i += 256) {
        const float4 m = a.inner4[i];
        snodes[i].x = m.x;
        snodes[i].y = m.y;
        snodes[i].z = m.z;
        snodes[i].w = m.w;
    }
    TPT_LDS int* pool_next = (TPT_LDS int*)(slds + a.lds_pool_offset);   // next unclaimed pixel of tile 2b + 1
    if (pool && tid == 0) *pool_next = (tx + 1) * 16 < a.width ? 0 : 256;   // (no second tile: an empty pool)
    if (MTL_LDS || a.lds_nodes > 0 || pool) __syncthreads();
    auto MT = [&](int i) -> float4 {
        if constexpr (MTL_LDS) {
            return make_float4(smtl[i].x, smtl[i].y, smtl[i].z, smtl[i].w);
        } else {
            return a.mtl[i];
        }
    };
    // (QUAD: one stack per quad in its four lanes' columns; the host keeps it all in LDS)
    LaneStack<StackT, QUAD> stk;
    stk.lds = (TPT_LDS StackT*)(slds + a.lds_stack_offset) +
              (QUAD ? (tid & ~3) : ((TPT_STACK_PAIRED && sizeof(StackT) == 2) ? 2 * tid : tid));
    stk.nlds = a.stack_lds_slots;
    PathRecords<MAXD, PAIR ? 128 : 256> rec;
    rec.lds = (TPT_LDS float*)(slds + a.lds_rec_offset) + (PAIR ? wave * 32 + pl : tid);
    rec.nlds = a.rec_lds_levels;
    rec.words = LIGHTS ? 5 : 2;

    uint32_t st[6];
    V3 total = v3(0.0f, 0.0f, 0.0f);
    if (active) {
#pragma unroll
        for (int i = 0; i < 6; ++i) st[i] = g_rng[i * npix + off];
        total = v3(g_acc[off], g_acc[npix + off], g_acc[2 * npix + off]);
    }
    int remaining = a.samples;
    int phase = PH_CAMERA;
    int depth = 0, li = 0;
    uint32_t mk = 0;   // material id | p-kind << 30 of the current bounce
    bool env_pending = false;   // A15: this bounce's env next-event sample is still to be drawn
    V3 env_k = v3(0.0f, 0.0f, 0.0f);
    // pair mode + A15: the env sample's uniforms and incident-side normal, drawn by
    // the path lane when it posts the bounce's shadow job (side lane: as received)
    float env_x1 = 0.0f, env_x2 = 0.0f;
    V3 env_nf = v3(0.0f, 0.0f, 0.0f);
    V3 rd = v3(0.0f, 0.0f, 0.0f), nd = rd, nrm = rd, direct = rd;
    Trav r;
    trav_begin(r, rd, v3(1.0f, 1.0f, 1.0f), TM_CLOSEST);
    int ts = active ? TS_DONE : ((PAIR && side && pixel) ? TS_IDLE : TS_DEAD);
#ifdef TPT_VERIFY_CULL
    bool vpend = false;   // a traversal of this lane awaits verification
#endif
    bool sl_pend = false;   // a traversal of this lane awaits the sliver pass
    // grazing() inputs: LIGHTS variants keep the geometric normal of the face the
    // current rays leave (shadow rays start in later passes); the others only the
    // verdict for the next extension ray
    Surf gsurf = no_surface();
    bool graze_next = false;
    // DRAIN variants (launches too small to fill the chip, where each wave's
    // chain latency is the frame time): a parked leaf's triangle is loaded when
    // the leaf is parked, in flight while the walk goes on (strong-scaled C2,
    // rank 0 of 8: -5 % time; C5 at full occupancy +5 %, so only these variants)
    float4 pq0 = make_float4(0.0f, 0.0f, 0.0f, 0.0f), pq1 = pq0, pq2 = pq0;
    const int refill = a.refill;
    // pair mode state.  Path lane: partner idle?, the level whose shadow rays the
    // partner holds (-1: none), this level's shadows delegated?, the unwind's seed
    // while waiting for the partner, a job to post at the next exchange.  Side
    // lane: the level it works on and the direct sum it hands back.
    bool delegated = false, post = false, ready = false;   // (partner idle <=> pend < 0)
    bool post_env = false;   // the posted job carries an env sample (A15)
    int pend = -1, jlevel = 0;
    // (the unwind's seed while the path lane waits for its side lane lives in
    // `direct`: the path's levels are all recorded by then)
    // a level's record: pm = the material the probe hit (kNoProbe: none), dl =
    // its direct term (delta lights + probe emission).  Pair mode keeps the
    // probe symbolic and the delta lights' sum apart (the side lane may still be
    // summing it); the unwind adds them in the same order, (1 * e) + direct.
    auto put_level = [&](uint32_t pm, V3 dl) {
        if constexpr (PAIR) {
            rec.template put_dst<true>(depth, mk, pm, dl);
            if (!delegated) {
                rec.put(depth, 2, direct.x);
                rec.put(depth, 3, direct.y);
                rec.put(depth, 4, direct.z);
            }
        } else {
            rec.put_dst(depth, mk, pm, dl);
        }
    };

#ifdef TPT_PROFILE_PHASES
    const unsigned long long t_wave0 = wall_clock64();
    unsigned long long p_done = 0, p_trav = 0, p_steps = 0, t_iter0 = 0, t_loop0 = 0, p_outer = 0;
    // lane states summed over traversal steps (DESIGN.md "N1"): traversing, a
    // finished ray waiting for the wave's next shading pass, no work (pixel done
    // or none, pair-mode idle); and the lanes each shading pass serves
    unsigned long long p_lt = 0, p_lw = 0, p_lx = 0, p_lp = 0;
    // shading-pass sections (profiling builds only): every boundary drains
    // the wave's outstanding memory operations, so a section is charged the
    // latency of its own loads; the pass's first active lane adds the time
    unsigned int p_sec[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    unsigned long long t_sec = 0;
    bool p_lead = false;
#endif
#ifdef TPT_PROFILE_PHASES
#define TPT_SEC_BEGIN()                                                       \
    {                                                                         \
        __builtin_amdgcn_s_waitcnt(0);                                        \
        t_sec = wall_clock64();                                               \
        p_lead = __builtin_amdgcn_readfirstlane(lane) == lane;                \
    }
#define TPT_SEC(k)                                                            \
    {                                                                         \
        __builtin_amdgcn_s_waitcnt(0);                                        \
        const unsigned long long t_ = wall_clock64();                         \
        if (p_lead) p_sec[k] += (unsigned int)(t_ - t_sec);                   \
        t_sec = t_;                                                           \
    }
#else
#define TPT_SEC_BEGIN()
#define TPT_SEC(k)
#endif
    for (;;) {
#ifdef TPT_PROFILE_PHASES
        {
            const unsigned long long now = wall_clock64();
            if (t_loop0) p_trav += now - t_loop0;   // the previous traversal loop
            t_iter0 = now;
        }
#endif
#ifndef TPT_NO_SLIVERS
        if (ORDERED && a.n_sliver_groups > 0) {   // (uniform) slivers after a culled traversal (Culling)
            if (ts == TS_DONE && sl_pend) {
                sl_pend = false;
                sliver_pass(r, a, c_leaf);
            }
        }
#endif
        if (TPT_GRAZE_HIT && ORDERED && !NOEMIT && ts == TS_DONE && phase == PH_PROBE && r.fin && r.fid >= 0 && r.mode == TM_EMIT &&
            a.graze && grazing(Surf{a.shade[3 * r.fid + 1].w, a.shade[3 * r.fid + 2].w}, r.d)) {
            // a grazing probe hit (Culling: "Grazing hits"): pass 1 again on the
            // uncull'd binary path, which tests every leaf whose box its line passes
            // (an extension ray's grazing hit is caught in its shading prelude)
            trav_begin(r, r.o, r.d, r.mode, a.boxes_finite != 0, a.emit_root, a.cull_eps, true);
            ts = TS_TRAV;
            sl_pend = false;
        }
        if (ORDERED && !NOEMIT && ts == TS_DONE && phase == PH_PROBE && r.mode == TM_EMIT && r.fid >= 0) {
            // direct probe, pass 2: the emitter hit stands unless something
            // beats it -- restart from the root keeping its t, position and fid
            r.mode = TM_OCCL;
            r.node = 0;
            r.sp = 0;
            r.pend = -1;
            ts = TS_TRAV;
            sl_pend = true;
        }
#ifdef TPT_VERIFY_CULL
        if (ts == TS_DONE && vpend) {
            vpend = false;
            // (an extension hit the shading prelude will trace again -- the grazing-hit
            // rule -- is verified after that traversal)
            if (!(TPT_GRAZE_HIT && phase == PH_EXT && r.fin && r.fid >= 0 && a.graze &&
                  grazing(Surf{a.shade[3 * r.fid + 1].w, a.shade[3 * r.fid + 2].w}, r.d)))
                verify_ray(a, r, phase, a.mtl);
        }
#endif
#ifdef TPT_PROFILE_PHASES
        if (__ballot(ts == TS_DONE) != 0ull) p_lp += (unsigned long long)__popcll(__ballot(ts == TS_DONE));
#endif
        // The shading pass, in two parts.  Pair mode exchanges the side lanes' finished
        // direct sums between them (round 6), so a path lane whose side lane completes
        // its level in this pass unwinds in this pass instead of waiting for the next.
        const bool in_pass = ts == TS_DONE;
        bool finish = false;   // the path ends this pass: unwind
        bool begun = false;    // the next ray is already set up (inline probe pass 1)
        bool redo = false;     // a grazing extension hit: traced again, uncull'd
        bool shadow = false;   // the next ray is a shadow ray
        bool tg = false;       // the next ray leaves its face within 1e-3 of its plane (grazing())
        V3 L = v3(0.0f, 0.0f, 0.0f), td = rd;
        if (in_pass) {
            TPT_SEC_BEGIN()
            // ---- consume the finished traversal (nothing yet for a fresh sample) ----
            bool lights_next = false, after = false;
            Hemi hb;              // this pass's hemisphere frame (new_direction), shared by the
            bool hb_ok = false;   // bounce's extension sample and its direct probe
            if (!LIGHTS) rd = r.d;   // the extension ray's direction (unused otherwise)
            Surf gpass = gsurf;   // the face this pass's new rays leave
            if (phase == PH_EXT) {
                if (r.fid < 0) {   // miss: env radiance seeds the unwind (:358-362)
                    if (a.env) L = env_lookup<ENVIS>(a.env, a.env_w, a.env_h, rd);
                    finish = true;
                } else {           // hit shading prelude (:364-381)
                    const float4* sh = a.shade + 3 * r.fid;
                    const float4 s0 = sh[0], s1 = sh[1], s2 = sh[2];
                    // the grazing-hit rule (Culling: "Grazing hits"): a culled walk's hit
                    // within 1e-3 of the face's plane is not shaded; the same ray is traced
                    // again on the uncull'd binary path (ray set-up below, not counted)
                    redo = TPT_GRAZE_HIT && ORDERED && r.fin && a.graze && grazing(Surf{s1.w, s2.w}, rd);
                    if (!redo) {
                        ++c_shade;
                        const float w = 1.0f - r.u - r.v;
                        nrm = normalize(((w * v3(s0.x, s0.y, s0.z)) + (r.u * v3(s1.x, s1.y, s1.z))) +
                                        (r.v * v3(s2.x, s2.y, s2.z)));
                        gpass = a.graze ? Surf{s1.w, s2.w} : no_surface();
                        if constexpr (LIGHTS) gsurf = gpass;
                        r.o = r.o + (r.t * rd);
                        const int mtl = __float_as_int(s0.w);
                        const float4 m1 = MT(2 * mtl + 1);
                        float af;
                        const float prob = new_direction(rd, nrm, m1.x, m1.y, st, nd, af, hb, hb_ok);
                        graze_next = grazing(gpass, nd);
                        rec.put(depth, 0, af);
                        mk = (uint32_t)mtl | (p_kind(prob) << 30);
                        direct = v3(0.0f, 0.0f, 0.0f);
                        li = 0;
                        delegated = false;
                        env_pending = ENVIS && !(m1.x > 0.0f) && !(m1.y > 0.0f);   // diffuse hit
                        lights_next = true;
                    }
                }
            } else if (LIGHTS && phase == PH_SHADOW) {
                if (r.fid < 0) {   // sampleDeltaLights :279-282 (light re-sampled: deterministic)
                    V3 ldir, lrad;
                    light_sample(a.lights, li, r.o, ldir, lrad);
                    const float4 m0 = MT(2 * (mk & 0x3fffffffu));
                    direct = direct + (v3(m0.x, m0.y, m0.z) * lrad);
                }
                ++li;
                lights_next = true;
            } else if (ENVIS && phase == PH_ENVSHADOW) {   // env next-event estimate (A15, opt-in)
                if (r.fid < 0) direct = direct + env_k;
                lights_next = true;
            } else if (!NOEMIT && phase == PH_PROBE) {   // :390-400
                V3 dl = LIGHTS ? direct : v3(0.0f, 0.0f, 0.0f);
                uint32_t pm = kNoProbe;
                if (r.fid >= 0 && r.mode != TM_OCCLUDED) {   // the closest hit (an unbeaten emitter, pass 2)
                    pm = (uint32_t)__float_as_int(a.shade[3 * r.fid].w);
                    const float e = MT(2 * pm).w;
                    if (!PAIR) dl = (v3(1.0f, 1.0f, 1.0f) * v3(e, e, e)) + dl;   // pair mode: at the unwind
                }
                put_level(pm, dl);
                after = true;
            } else if (PAIR && phase == PH_WAIT) {   // the side lane's direct sum has arrived
                L = direct;
                finish = true;
            }
            TPT_SEC(1)
            td = rd;
            tg = redo;
            if (PAIR && lights_next && !side && li == 0 && pend < 0 && (a.n_lights > 0 || (ENVIS && env_pending))) {
                // hand this bounce's shadow rays to the idle side lane (posted at the
                // exchange below: origin r.o, material mk, level depth)
                post = true;
                jlevel = depth;
                pend = depth;
                delegated = true;
                li = a.n_lights;
                if (ENVIS && env_pending) {
                    // A15: the env sample's two uniforms are this lane's to draw, after
                    // the extension direction and before the probe's (RNG order); the
                    // side lane evaluates the sample and traces its shadow ray
                    env_pending = false;
                    env_x1 = xorwow_uniform(st);
                    env_x2 = xorwow_uniform(st);
                    env_nf = (dot(rd, nrm) > 0.0f ? -1.0f : 1.0f) * nrm;   // getNewDirection's flip
                    post_env = true;
                }
            }
            if (PAIR && lights_next && side && li >= a.n_lights && !(ENVIS && env_pending)) {
                // the side lane's job is done: its direct sum goes back at the exchange
                ready = true;
                ts = TS_IDLE;
                lights_next = false;
            }
            if (lights_next) {
                const float4 m1 = MT(2 * (mk & 0x3fffffffu) + 1);
                if (LIGHTS && li < a.n_lights) {
                    V3 lrad;
                    light_sample(a.lights, li, r.o, td, lrad);
                    tg = grazing(gsurf, td);
                    phase = PH_SHADOW;
                    shadow = true;
                } else {
                    bool env_ray = false;
                    if (ENVIS && env_pending) {   // after the delta lights, before the probe
                        env_pending = false;
                        V3 nf = env_nf;
                        float x1 = env_x1, x2 = env_x2;
                        if (!(PAIR && side)) {
                            nf = (dot(rd, nrm) > 0.0f ? -1.0f : 1.0f) * nrm;   // getNewDirection's flip
                            x1 = xorwow_uniform(st);
                            x2 = xorwow_uniform(st);
                        }
                        if (env_is_sample(a, nf, x1, x2, td, env_k)) {
                            phase = PH_ENVSHADOW;
                            shadow = true;
                            env_ray = true;
                            tg = grazing(gsurf, td);
                        }
                    }
                    if (env_ray) {
                    } else if (PAIR && side) {   // the env sample cannot contribute: the job is done
                        ready = true;
                        ts = TS_IDLE;
                    } else if (!(m1.x >= 1.0f || m1.y > 0.0f)) {   // direct probe (:387-389)
                        float af2;
                        if (!TPT_SHARE_HEMI) hb_ok = false;   // (A/B builds: the frame recomputed)
                        new_direction(rd, nrm, m1.x, m1.y, st, td, af2, hb, hb_ok);
                        if ((TPT_PROBE_SHORTCUT && ORDERED && (NOEMIT || !a.any_emitter)) ||
                            (ORDERED && probe_misses_emitters(a, r.o, td))) {
                            // no triangle emits, or the probe's line passes no emitter's
                            // leaf box: the probe's emitter pass ends with no hit, exactly
                            // as a traversal would (the ray is still counted: the
                            // reference traces it)
                            ++c_trav;
                            ++c_local;
                            put_level(kNoProbe, direct);
                            after = true;
                        } else if (INL && TPT_PROBE_INLINE) {
                            tg = grazing(gpass, td);
                            // <= 4 emitters: pass 1 here; a miss resolves the probe in
                            // this pass, an emitter hit goes on to pass 2 (occlusion)
                            ++c_trav;
                            trav_begin(r, r.o, td, TM_EMIT, a.boxes_finite != 0, a.emit_root, a.cull_eps, tg);
                            begun = true;
                            phase = PH_PROBE;
                            if (r.mode == TM_EMIT && r.fin) {
                                ++c_wide;
                                emit_probe_inline<DRAIN>(r, a.inner4 + 8 * (size_t)a.emit_root, a.tri, nint, c_leaf,
                                                         a.cull_eps);
                                if (a.n_sliver_groups > 0) sliver_pass(r, a, c_leaf);
                                if (r.fid < 0) {
                                    ++c_local;
                                    put_level(kNoProbe, direct);
                                    after = true;
                                    begun = false;
                                } else {
                                    r.mode = TM_OCCL;
                                    r.node = 0;
                                }
                            }
                        } else {
                            tg = grazing(gpass, td);
                            phase = PH_PROBE;
                        }
                    } else {
                        put_level(kNoProbe, direct);
                        after = true;
                    }
                }
            }
            TPT_SEC(2)
            if (after) {
                const float e = MT(2 * (mk & 0x3fffffffu)).w;
                if (e > 0.0f) {   // an emitter ends the path (:408-412); the unwind starts from e
                    L = e * v3(1.0f, 1.0f, 1.0f);
                    finish = true;
                } else {
                    rd = nd;
                    td = rd;
                    tg = graze_next;
                    ++depth;
                    if (depth == a.max_depth) finish = true;
                    else phase = PH_EXT;
                }
            }
            TPT_SEC(3)
        }
        bool woke = false;   // pair mode: a path lane that waited for its side lane, released mid-pass
        if constexpr (PAIR && (TPT_PAIR_MID == 1 || (TPT_PAIR_MID == 2 && ENVIS))) {
            // ---- mid-pass exchange, side -> path: a level's direct sum, in light order ----
            // (a side lane becomes ready in the first part of its pass; a path lane that
            // finishes in this pass, or has waited since an earlier one, then unwinds in
            // the second part -- the same sums in the same order, one pass sooner)
            const int jready = __shfl_xor((int)ready, 1, 64);
            const float dx = __shfl_xor(direct.x, 1, 64), dy = __shfl_xor(direct.y, 1, 64),
                        dz = __shfl_xor(direct.z, 1, 64);
            const int rl = __shfl_xor(jlevel, 1, 64);
            if (!side && jready) {
                rec.put(rl, 2, dx);
                rec.put(rl, 3, dy);
                rec.put(rl, 4, dz);
                pend = -1;
                if (!in_pass && phase == PH_WAIT) {   // its unwind seed waits in `direct`
                    woke = true;
                    ts = TS_DONE;
                    L = direct;
                    finish = true;
                    td = rd;
                }
            }
            ready = false;
        }
        if (in_pass || woke) {
            if (PAIR && finish && pend >= 0) {
                // the side lane still sums a level's shadow rays: wait for it (exchange below)
                direct = L;
                phase = PH_WAIT;
                ts = TS_IDLE;
                finish = false;
            }
            bool unwound = false;
            if constexpr (DRAIN && !LIGHTS && MAXD == 8) {
                // DRAIN variants: every level's record and materials read before the
                // arithmetic, so the unwind pays one LDS latency chain instead of one
                // per level (the same operations in the same order as below)
                static_assert(!PAIR && !LIGHTS, "DRAIN unwind: one-lane 2-word records");
                if (finish && rec.nlds >= 8) {
                    unwound = true;
                    float af[8];
                    uint32_t w1[8];
#pragma unroll
                    for (int k = 0; k < 8; ++k) {
                        af[k] = rec.template lds_at<2>(k, 0);
                        w1[k] = k < depth ? __float_as_uint(rec.template lds_at<2>(k, 1)) : (kNoProbe << 15);
                    }
                    float4 mb[8];
                    float ee[8];
#pragma unroll
                    for (int k = 0; k < 8; ++k) {
                        mb[k] = MT(2 * (w1[k] & 0x7fffu));
                        const uint32_t pm = (w1[k] >> 15) & 0x7fffu;
                        ee[k] = MT(2 * (pm == kNoProbe ? 0u : pm)).w;
                    }
#pragma unroll
                    for (int k = 7; k >= 0; --k) {
                        if (k < depth) {
                            const V3 att = af[k] * v3(mb[k].x, mb[k].y, mb[k].z);   // :379
                            const uint32_t kind = w1[k] >> 30;
                            const float prob = kind == 0u ? af[k] : (kind == 1u ? -0.0f : 0.0f);
                            const float ivp = 1.0f / prob;                            // :427 "/ pStack"
                            const uint32_t pm = (w1[k] >> 15) & 0x7fffu;
                            const float e = pm == kNoProbe ? 0.0f : ee[k];
                            const V3 dst = pm == kNoProbe ? v3(0.0f, 0.0f, 0.0f)
                                                          : (v3(1.0f, 1.0f, 1.0f) * v3(e, e, e)) + v3(0.0f, 0.0f, 0.0f);
                            L = ivp * ((dst + L) * att);
                        }
                    }
                    total = total + L;
                    phase = PH_CAMERA;
                }
            }
            if (finish && !unwound) {   // unwind (:416-431): levels depth-1 .. 0
                for (int k = depth - 1; k >= 0; --k) {
                    const float af = rec.get(k, 0);
                    const uint32_t w1 = __float_as_uint(rec.get(k, 1));
                    const bool packed = rec.words == 2;
                    const float4 mb = MT(2 * (w1 & ((packed || PAIR) ? 0x7fffu : 0x3fffffffu)));
                    const V3 att = af * v3(mb.x, mb.y, mb.z);                   // :379
                    const uint32_t kind = w1 >> 30;
                    const float prob = kind == 0u ? af : (kind == 1u ? -0.0f : 0.0f);
                    const float ivp = 1.0f / prob;                              // :427 "/ pStack"
                    V3 dst;
                    if (packed) {
                        const uint32_t pm = (w1 >> 15) & 0x7fffu;
                        const float e = pm == kNoProbe ? 0.0f : MT(2 * pm).w;
                        dst = pm == kNoProbe ? v3(0.0f, 0.0f, 0.0f)
                                             : (v3(1.0f, 1.0f, 1.0f) * v3(e, e, e)) + v3(0.0f, 0.0f, 0.0f);
                    } else if (PAIR) {   // the delta lights' sum, then the probe's emission (1 * e) + direct
                        const uint32_t pm = (w1 >> 15) & 0x7fffu;
                        const V3 dd = v3(rec.get(k, 2), rec.get(k, 3), rec.get(k, 4));
                        const float e = pm == kNoProbe ? 0.0f : MT(2 * pm).w;
                        dst = pm == kNoProbe ? dd : (v3(1.0f, 1.0f, 1.0f) * v3(e, e, e)) + dd;
                    } else {
                        dst = v3(rec.get(k, 2), rec.get(k, 3), rec.get(k, 4));
                    }
                    L = ivp * ((dst + L) * att);
                }
                total = total + L;
                phase = PH_CAMERA;
            }
            TPT_SEC(4)
            V3 to = r.o;
            if (pool && phase == PH_CAMERA && remaining == 0 && active) {
                // this pixel is done: store it and draw the next pixel of the pool tile
#pragma unroll
                for (int i = 0; i < 6; ++i) g_rng[i * npix + off] = st[i];
                g_acc[off] = total.x;
                g_acc[npix + off] = total.y;
                g_acc[2 * npix + off] = total.z;
                active = false;
                for (;;) {
                    const int j = __atomic_fetch_add(pool_next, 1, __ATOMIC_RELAXED);
                    if (j >= 256) break;
                    const int wj = j >> 6, lj = j & 63;
                    const int px = (tx + 1) * 16 + (wj & 1) * 8 + (lj & 7);
                    const int ply = (by / nfr) * 16 + (wj >> 1) * 8 + (lj >> 3);
                    const int py = band_row(ply, a.band_rows, a.band_count, a.band_index, a.band_list);
                    if (px < a.width && ply < a.band_height && py < a.height) {
                        x = px;
                        y = py;
                        off = (size_t)x + (size_t)y * (size_t)a.width;
#pragma unroll
                        for (int i = 0; i < 6; ++i) st[i] = g_rng[i * npix + off];
                        total = v3(g_acc[off], g_acc[npix + off], g_acc[2 * npix + off]);
                        remaining = a.samples;
                        active = true;
                        break;
                    }
                }
            }
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
                    tg = false;   // the camera: no surface
                    depth = 0;
                    phase = PH_EXT;
                }
            }
            TPT_SEC(5)
            if (ts != TS_DEAD && ts != TS_IDLE) {
                if (!begun) {
                    if (!redo) ++c_trav;
                    trav_begin(r, to, td, shadow ? TM_ANY : ((ORDERED && phase == PH_PROBE) ? TM_EMIT : TM_CLOSEST),
                               a.boxes_finite != 0, a.emit_root, a.cull_eps, tg);
                }
                ts = TS_TRAV;
                sl_pend = true;
#ifdef TPT_VERIFY_CULL
                vpend = true;
#endif
            }
            TPT_SEC(6)
        }
        if constexpr (PAIR) {
            // ---- exchange between a pixel's path lane and its side lane (whole wave) ----
            // path -> side: a bounce's shadow rays (the path lane's r.o is that hit
            // point until its next hit: a posting pass only starts rays from it)
            const int jpost = __shfl_xor((int)post, 1, 64);
            const float jx = __shfl_xor(r.o.x, 1, 64), jy = __shfl_xor(r.o.y, 1, 64), jz = __shfl_xor(r.o.z, 1, 64);
            const int jmk = __shfl_xor((int)mk, 1, 64), jl = __shfl_xor(jlevel, 1, 64);
            const Surf jgs = Surf{__shfl_xor(gsurf.x, 1, 64), __shfl_xor(gsurf.y, 1, 64)};
            bool jenv = false;
            if constexpr (ENVIS) {   // A15: the env sample's uniforms and normal travel with the job
                jenv = __shfl_xor((int)post_env, 1, 64) != 0;
                const float e1 = __shfl_xor(env_x1, 1, 64), e2 = __shfl_xor(env_x2, 1, 64);
                const float n0 = __shfl_xor(env_nf.x, 1, 64), n1 = __shfl_xor(env_nf.y, 1, 64),
                            n2 = __shfl_xor(env_nf.z, 1, 64);
                if (side && jpost) {
                    env_pending = jenv;
                    env_x1 = e1;
                    env_x2 = e2;
                    env_nf = v3(n0, n1, n2);
                }
            }
            if (side && jpost) {
                mk = (uint32_t)jmk;
                jlevel = jl;
                gsurf = jgs;
                li = 0;
                direct = v3(0.0f, 0.0f, 0.0f);
                V3 ldir, lrad;
                const V3 jo = v3(jx, jy, jz);
                bool go = true;
                if (a.n_lights > 0) {
                    light_sample(a.lights, 0, jo, ldir, lrad);
                    phase = PH_SHADOW;
                } else if (ENVIS && env_pending) {   // env only: the sample, then its shadow ray
                    env_pending = false;
                    go = env_is_sample(a, env_nf, env_x1, env_x2, ldir, env_k);
                    phase = PH_ENVSHADOW;
                } else {
                    go = false;
                }
                if (go) {
                    ++c_trav;
                    trav_begin(r, jo, ldir, TM_ANY, a.boxes_finite != 0, a.emit_root, a.cull_eps, grazing(gsurf, ldir));
                    ts = TS_TRAV;
                    sl_pend = true;
#ifdef TPT_VERIFY_CULL
                    vpend = true;
#endif
                } else {   // nothing to trace: the direct sum (zero) goes back at once
                    r.o = jo;
                    ready = true;
                    ts = TS_IDLE;
                }
            }
            post = false;
            post_env = false;
            // side -> path: the level's direct sum, in light order
            const int jready = __shfl_xor((int)ready, 1, 64);
            const float dx = __shfl_xor(direct.x, 1, 64), dy = __shfl_xor(direct.y, 1, 64),
                        dz = __shfl_xor(direct.z, 1, 64);
            const int rl = __shfl_xor(jlevel, 1, 64);
            if (!side && jready) {
                rec.put(rl, 2, dx);
                rec.put(rl, 3, dy);
                rec.put(rl, 4, dz);
                pend = -1;
                if (phase == PH_WAIT) ts = TS_DONE;
            }
            ready = false;
            // a path lane with no samples left retires its side lane
            const int pdead = __shfl_xor((int)(ts == TS_DEAD), 1, 64);
            if (side && ts == TS_IDLE && pdead) ts = TS_DEAD;
        }
        if (__ballot(ts != TS_DEAD) == 0ull) break;
        if constexpr (TPT_SHADOW_FIRST && ORDERED && (LIGHTS || ENVIS) && !QUAD) {
            // a fresh shadow ray's root visit (the loop's first step for it, below)
            bool quick = false;
            if (ts == TS_TRAV && r.mode == TM_ANY && r.fin && r.node == 0 && r.sp == 0 && r.pend < 0 &&
                r.fid < 0 && r.t == kRealMax) {
                ++c_wide;
                const int next = inner_visit4(r, a.inner4, snodes, a.lds_nodes, stk, r.sp);
                r.node = next >= 0 ? next : (r.sp == 0 ? -1 : stk.get(--r.sp));
                if (r.node < 0) {   // no child passes: the ray is done, unoccluded
                    ts = TS_DONE;
                    quick = true;
                }
            }
            if (__ballot(quick) != 0ull) continue;   // shade those lanes before traversing
        }
#ifdef TPT_PROFILE_PHASES
        t_loop0 = wall_clock64();
        p_done += t_loop0 - t_iter0;
        ++p_outer;
#endif
        // ---- traversal: step while enough lanes of the wave are still traversing ----
        const int thr = refill;
        for (;;) {
#ifdef TPT_PROFILE_PHASES
            ++p_steps;
#endif
            const int cnt = __popcll(__ballot(lead && ts == TS_TRAV));   // (QUAD: pixels)
#ifdef TPT_PROFILE_PHASES
            p_lt += (unsigned long long)cnt;
            p_lw += (unsigned long long)__popcll(__ballot(ts == TS_DONE));
            p_lx += (unsigned long long)__popcll(__ballot(ts == TS_DEAD || ts == TS_IDLE));
#endif
            if (cnt == 0) break;
            if (cnt < thr && __ballot(lead && ts == TS_DONE) != 0ull) break;
            // Speculative leaf postponement: a lane that reaches a leaf parks it
            // (one slot) and keeps walking inner nodes; the wave runs the
            // triangle branch only when enough lanes hold a parked leaf, when
            // lanes are blocked (a second leaf, or nothing left but the parked
            // one), or when no lane has inner work.  Leaves are still tested in
            // the order the traversal reaches them; a stale r.t only weakens
            // the ordered culling, and the ordered winner (least t, then
            // largest leaf position) does not depend on test order.
            bool inner_ready = false, has = false, blocked = false;
            const bool at_inner = ts == TS_TRAV && r.node >= 0 && r.node < nint;
            if (ts == TS_TRAV) {
                if (at_inner) {
                    int next;
                    if (QUAD && r.fin) {   // 4-wide, split over the pixel's four lanes
                        ++c_wide;
                        bool stop;
                        next = inner_visit4_quad(r, a.inner4, a.tri, nint, a.cull_eps, stk, r.sp, stop, c_leaf);
                        if (stop) {
                            r.sp = 0;
                            next = -1;
                        }
                    } else if (ORDERED && r.fin) {   // 4-wide (r.fin includes a.boxes_finite)
                        ++c_wide;
                        next = inner_visit4(r, a.inner4, snodes, a.lds_nodes, stk, r.sp);
                    } else {                  // binary, the reference's exact slab test
                        ++c_inner;
                        int deferred;
                        bool push;
                        inner_visit<ORDERED>(r, a.inner, next, push, deferred);
                        stk.put(r.sp, deferred);
                        r.sp += push ? 1 : 0;
                    }
                    if (r.sp > a.stack_depth) {
                        ++c_ovf;
                        r.sp = 0;
                        next = -1;
                    }
                    r.node = next >= 0 ? next : (r.sp == 0 ? -1 : stk.get(--r.sp));
                }
                if (r.node >= nint && r.pend < 0) {
                    r.pend = r.node - nint;
                    r.node = r.sp == 0 ? -1 : stk.get(--r.sp);
                    if constexpr (DRAIN) {
                        const TriQ tq = tri_load(a.tri, r.pend);   // in flight while the walk goes on
                        pq0 = tq.q0;
                        pq1 = tq.q1;
                        pq2 = tq.q2;
                    }
                }
                has = r.pend >= 0;
                inner_ready = r.node >= 0 && r.node < nint;
                blocked = has && !inner_ready;
            }
            const unsigned long long hb = __ballot(has);
            if (hb != 0ull) {
                const bool go = __popcll(__ballot(blocked)) >= a.leaf_kb || __popcll(hb) >= TPT_LEAF_KP ||
                                __ballot(inner_ready) == 0ull;
                if (go && has) {
                    ++c_leaf;
                    const bool stop = DRAIN ? leaf_test_q<ORDERED>(r, pq0, pq1, pq2, r.pend, a.cull_eps)
                                            : leaf_test<ORDERED>(r, a.tri, r.pend, a.cull_eps);
                    if (stop) {
                        r.node = -1;
                        r.sp = 0;
                    }
                    r.pend = -1;
                }
            }
            if (ts == TS_TRAV && r.node < 0 && r.pend < 0) ts = TS_DONE;
        }
    }
    if (active && lead) {
#pragma unroll
        for (int i = 0; i < 6; ++i) g_rng[i * npix + off] = st[i];
        g_acc[off] = total.x;
        g_acc[npix + off] = total.y;
        g_acc[2 * npix + off] = total.z;
    }
    if (!lead) {   // QUAD: the pixel's work is counted once
        c_trav = c_inner = c_wide = c_leaf = c_shade = c_ovf = c_local = 0;
    }
    const unsigned long long s_wide = wave_sum(c_wide), s_local = wave_sum(c_local);
    const unsigned long long s_trav = wave_sum(c_trav), s_inner = wave_sum(c_inner), s_leaf = wave_sum(c_leaf),
                             s_shade = wave_sum(c_shade), s_ovf = wave_sum(c_ovf);
#ifdef TPT_PROFILE_PHASES
    unsigned long long m_trav = c_trav;   // heaviest lane's ray count
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        const unsigned long long o2 = __shfl_xor(m_trav, off, 64);
        m_trav = o2 > m_trav ? o2 : m_trav;
    }
#endif
#ifdef TPT_PROFILE_PHASES
    unsigned long long s_sec[7];
#pragma unroll
    for (int k = 0; k < 7; ++k) s_sec[k] = wave_sum(p_sec[k]);
    if (lane == 0) {
#pragma unroll
        for (int k = 0; k < 7; ++k) atomicAdd(&a.counters[16 + k], s_sec[k]);
    }
#endif
    if (lane == 0) {
        atomicAdd(&a.counters[0], s_trav);
        atomicAdd(&a.counters[1], s_inner);
        atomicAdd(&a.counters[2], s_leaf);
        atomicAdd(&a.counters[3], s_shade);
        if (s_ovf) atomicAdd(&a.counters[4], s_ovf);
        atomicAdd(&a.counters[5], s_wide);
        atomicAdd(&a.counters[9], s_local);
        if (a.band_cost && ly < a.band_height)
            atomicAdd(&a.band_cost[band_of(ly / a.band_rows, a.band_count, a.band_index, a.band_list)],
                      wall_clock64() - t_cost0);
#ifdef TPT_PROFILE_PHASES
        atomicAdd(&a.counters[6], p_done);
        atomicAdd(&a.counters[7], p_trav);
        atomicAdd(&a.counters[8], p_steps);
        atomicAdd(&a.counters[12], p_outer);
        atomicAdd(&a.counters[25], p_lt);
        atomicAdd(&a.counters[26], p_lw);
        atomicAdd(&a.counters[27], p_lx);
        atomicAdd(&a.counters[28], p_lp);
        const unsigned long long life = wall_clock64() - t_wave0;
        atomicMax(&a.counters[13], life);
        atomicAdd(&a.counters[14], life);
        atomicAdd(&a.counters[15], 1ull);
        if (a.debug_waves) {   // per-wave record: start, life, steps, shading passes, rays, wide, max lane rays, done-time
            const unsigned long long wid =
                ((unsigned long long)blockIdx.y * gridDim.x + blockIdx.x) * 4 + wave;
            unsigned long long* o = a.debug_waves + 8 * wid;
            o[0] = t_wave0;
            o[1] = life;
            o[2] = p_steps;
            o[3] = p_outer;
            o[4] = s_trav;
            o[5] = s_wide;
            o[6] = m_trav;
            o[7] = p_done;
        }
#endif
    }
}

// Spectrum::toUChar (material.h:74-81): truncating clamp to [0, 255]
__device__ __forceinline__ uint8_t to_uchar(float c) { return (uint8_t)fclamp(c * 255.0f, 255.0f, 0.0f); }

// copyToFB (path_tracer.cu:451-471) + the radiance readout (color / spp).
__global__ void k_resolve(ResolveArgs a) {
    const int x = blockIdx.x * blockDim.x + threadIdx.x;
    const int ly = blockIdx.y;
    if (x >= a.width || ly >= a.band_height) return;
    const int y = band_row(ly, a.band_rows, a.band_count, a.band_index, a.band_list);
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
        px[0] = to_uchar(b);
        px[1] = to_uchar(g);
        px[2] = to_uchar(r);
    }
}

// A ray batch through one traversal (tests, tpt_debug_trace_rays):
//  mode 0  closest hit in the reference's visit order (right-first DFS, no culling);
//  mode 1  closest hit through the production traversal (nearer-first, culled,
//          4-wide for finite rays), leaves tested as soon as they are reached;
//  mode 2  any hit (shadow rays, TM_ANY);
//  mode 3  direct probe in two passes (TM_EMIT, then TM_OCCL after an emitter
//          hit): hit = the unbeaten emitter's fid, -2 when something beats it
//          (the probe adds nothing), -1 when no emitter was hit.
// Modes 1-3 run the same visit / cull / leaf functions as k_trace.
constexpr int kRaysLdsSlots = 48;   // LDS stack slots per lane in k_trace_rays; deeper ones private

template <bool ORDERED>
__device__ __forceinline__ void trav_lane(Trav& r, const TraceArgs& a, LaneStack<int>& stk, uint32_t& c_ovf) {
    const int nint = a.n_faces - 1;
    while (r.node >= 0) {
        if (r.node < nint) {
            int next;
            if (ORDERED && r.fin) {
                next = inner_visit4(r, a.inner4, nullptr, 0, stk, r.sp);
            } else {
                int deferred;
                bool push;
                inner_visit<ORDERED>(r, a.inner, next, push, deferred);
                stk.put(r.sp, deferred);
                r.sp += push ? 1 : 0;
            }
            if (r.sp > a.stack_depth) {
                ++c_ovf;
                r.sp = 0;
                next = -1;
            }
            r.node = next >= 0 ? next : (r.sp == 0 ? -1 : stk.get(--r.sp));
        } else {
            const bool stop = leaf_test<ORDERED>(r, a.tri, r.node - nint, a.cull_eps);
            r.node = (stop || r.sp == 0) ? -1 : stk.get(--r.sp);
        }
    }
}

__global__ __launch_bounds__(256) void k_trace_rays(TraceArgs a, uint32_t n, const float* __restrict__ o,
                                                    const float* __restrict__ d, const int32_t* __restrict__ ofid,
                                                    int mode, int32_t* hit, float* t, float* uv) {
    extern __shared__ __attribute__((aligned(16))) char lds[];
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    uint32_t c_ovf = 0;
    if (i < n) {
        Trav r;
        const V3 ro = v3(o[3 * i], o[3 * i + 1], o[3 * i + 2]), rdir = v3(d[3 * i], d[3 * i + 1], d[3 * i + 2]);
        LaneStack<int> stk;
        stk.lds = (TPT_LDS int*)lds + threadIdx.x;
        stk.nlds = kRaysLdsSlots;
        int fid;
        if (mode == 0) {
            trav_begin(r, ro, rdir, TM_CLOSEST);   // binary nodes, the reference's ternary slab test
            trav_lane<false>(r, a, stk, c_ovf);
            fid = r.fid;
        } else {
            const int tm = mode == 1 ? TM_CLOSEST : (mode == 2 ? TM_ANY : TM_EMIT);
            // a ray leaving face ofid[i] (>= 0) gets the render's grazing test
            const Surf gs = (a.graze && ofid && ofid[i] >= 0)
                                ? Surf{a.shade[3 * ofid[i] + 1].w, a.shade[3 * ofid[i] + 2].w}
                                : no_surface();
            trav_begin(r, ro, rdir, tm, a.boxes_finite != 0, a.emit_root, a.cull_eps, grazing(gs, rdir));
            uint32_t c_leaf = 0;
            if (mode == 3 && probe_misses_emitters(a, ro, rdir)) r.node = -1;   // the render's probe pre-test
            trav_lane<true>(r, a, stk, c_ovf);
            if (a.n_sliver_groups > 0) sliver_pass(r, a, c_leaf);
            // the render's grazing-hit rule, under the render's own conditions: an
            // extension ray's closest hit (mode 1), a probe's pass-1 emitter hit (mode 3,
            // TM_EMIT only -- a probe that trav_begin turned into a closest-hit walk
            // because the scene has no emissive tree is not re-traced by k_trace either)
            if (r.fin && r.fid >= 0 && ((mode == 1 && r.mode == TM_CLOSEST) || (mode == 3 && r.mode == TM_EMIT)) &&
                a.graze && grazing(Surf{a.shade[3 * r.fid + 1].w, a.shade[3 * r.fid + 2].w}, r.d)) {
                // traced again on the uncull'd binary path
                trav_begin(r, ro, rdir, r.mode, a.boxes_finite != 0, a.emit_root, a.cull_eps, true);
                trav_lane<true>(r, a, stk, c_ovf);
            }
            if (mode == 3 && r.mode == TM_EMIT && r.fid >= 0) {   // pass 2: does anything beat the emitter hit?
                r.mode = TM_OCCL;
                r.node = 0;
                r.sp = 0;
                trav_lane<true>(r, a, stk, c_ovf);
                if (a.n_sliver_groups > 0) sliver_pass(r, a, c_leaf);
            }
            fid = (mode == 3 && r.mode == TM_OCCLUDED) ? -2 : r.fid;
            if (mode == 3 && fid >= 0) {   // a closest-hit probe (no emissive tree) may end on a non-emitter
                const int m = __float_as_int(a.shade[3 * fid].w);
                if (a.mtl[2 * m].w == 0.0f) fid = -2;
            }
        }
        hit[i] = fid;
        t[i] = r.t;
        uv[2 * i] = r.u;
        uv[2 * i + 1] = r.v;
    }
}

// The kernel's own hot-path device functions, one case per lane, for the
// known-answer tests against the reference's headers (tests only,
// tpt_debug_hot_kat).  op 0: box_hit (rayHitBBox) with 1/dir hoisted as
// trav_begin does, and the min/max form's verdict; op 1: tri_core on
// (v0, v1 - v0, v2 - v0) as the scene pack stores them; op 2: light_sample;
// op 3: to_uchar.  Layouts: see tpt.h.
__global__ __launch_bounds__(256) void k_hot_kat(int op, uint32_t n, const float* __restrict__ in,
                                                 float* __restrict__ out) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    if (op == 0) {
        const float* c = in + 12 * (size_t)i;
        const V3 o = v3(c[0], c[1], c[2]), d = v3(c[3], c[4], c[5]);
        const V3 inv = v3(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
        float t0, t1;
        const bool h = box_hit(o, inv, c[6], c[7], c[8], c[9], c[10], c[11], t0, t1);
        slab_minmax(o, inv, c[6], c[7], c[8], c[9], c[10], c[11], t0, t1);
        out[2 * (size_t)i] = h ? 1.0f : 0.0f;
        out[2 * (size_t)i + 1] = (fmaxf(t0, -kRealMax) <= fminf(t1, kRealMax)) ? 1.0f : 0.0f;
    } else if (op == 1) {
        const float* c = in + 15 * (size_t)i;
        const V3 v0 = v3(c[6], c[7], c[8]);
        const V3 e1 = v3(c[9], c[10], c[11]) - v0, e2 = v3(c[12], c[13], c[14]) - v0;
        float t, u, v;
        const bool h = tri_core(v3(c[0], c[1], c[2]), v3(c[3], c[4], c[5]), v0, e1, e2, t, u, v);
        float* q = out + 4 * (size_t)i;
        q[0] = h ? 1.0f : 0.0f;
        q[1] = t;
        q[2] = u;
        q[3] = v;
    } else if (op == 2) {
        const float* c = in + 16 * (size_t)i;
        DevLight L;
        L.type = (int)c[0];
        for (int k = 0; k < 3; ++k) {
            L.color[k] = c[1 + k];
            L.pos[k] = c[5 + k];
            L.dir[k] = c[8 + k];
        }
        L.intensity = c[4];
        L.cos_outer = c[11];
        L.inv_cos_cone_diff = c[12];
        V3 dir, rad;
        light_sample(&L, 0, v3(c[13], c[14], c[15]), dir, rad);
        float* q = out + 6 * (size_t)i;
        q[0] = dir.x;
        q[1] = dir.y;
        q[2] = dir.z;
        q[3] = rad.x;
        q[4] = rad.y;
        q[5] = rad.z;
    } else if (op == 3) {
        const float* c = in + 3 * (size_t)i;
        for (int k = 0; k < 3; ++k) out[3 * (size_t)i + k] = (float)to_uchar(c[k]);
    }
}

hipError_t launch_hot_kat(int op, uint32_t n, const float* in, float* out, hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_hot_kat, dim3((n + 255) / 256), dim3(256), 0, s, op, n, in, out);
    return hipGetLastError();
}

template <int MAXD, bool ORDERED, bool LIGHTS, bool MTL_LDS, typename StackT, bool ENVIS = false, bool INL = false,
          bool PAIR = false, bool DRAIN = false, bool QUAD = false, bool NOEMIT = false>
static void launch_one(const TraceArgs& a, dim3 grid, size_t lds, hipStream_t s) {
    hipLaunchKernelGGL((k_trace<MAXD, ORDERED, LIGHTS, MTL_LDS, StackT, ENVIS, INL, PAIR, DRAIN, QUAD, NOEMIT>), grid,
                       dim3(256), lds, s, a);
}
// four lanes per pixel (a.quad): one-lane logic without delta lights
template <bool MTL_LDS, typename StackT>
static void launch_quad(const TraceArgs& a, dim3 grid, size_t lds, hipStream_t s) {
    if (TPT_PROBE_INLINE && a.emit_inline) {
        if (a.max_depth <= 8) launch_one<8, true, false, MTL_LDS, StackT, false, true, false, false, true>(a, grid, lds, s);
        else launch_one<64, true, false, MTL_LDS, StackT, false, true, false, false, true>(a, grid, lds, s);
    } else {
        if (a.max_depth <= 8) launch_one<8, true, false, MTL_LDS, StackT, false, false, false, false, true>(a, grid, lds, s);
        else launch_one<64, true, false, MTL_LDS, StackT, false, false, false, false, true>(a, grid, lds, s);
    }
}

// INL: probe pass 1 in the shading pass (an emissive tree of one node); its own
// variant, so scenes with larger emitter sets keep the leaner kernel.  PAIR:
// pair mode (delta-light scenes only).  NOEMIT (pair variants): no triangle
// emits, so every direct probe ends in the shading pass (TPT_PROBE_SHORTCUT) and
// the probe's traversal phases are compiled out -- the pair kernel's registers
// for C3's and C3 + IS's ball.
#ifndef TPT_NOEMIT_PAIR
#define TPT_NOEMIT_PAIR 1
#endif
template <bool LIGHTS, bool MTL_LDS, typename StackT, bool PAIR = false, bool ENVIS = false, bool DRAIN = false>
static void launch_ordered_d(const TraceArgs& a, dim3 grid, size_t lds, hipStream_t s) {
    if constexpr (PAIR && TPT_NOEMIT_PAIR && TPT_PROBE_SHORTCUT) {
        if (!a.any_emitter) {
            if (a.max_depth <= 8)
                launch_one<8, true, LIGHTS, MTL_LDS, StackT, ENVIS, false, PAIR, DRAIN, false, true>(a, grid, lds, s);
            else
                launch_one<64, true, LIGHTS, MTL_LDS, StackT, ENVIS, false, PAIR, DRAIN, false, true>(a, grid, lds, s);
            return;
        }
    }
    if (TPT_PROBE_INLINE && a.emit_inline) {
        if (a.max_depth <= 8) launch_one<8, true, LIGHTS, MTL_LDS, StackT, ENVIS, true, PAIR, DRAIN>(a, grid, lds, s);
        else launch_one<64, true, LIGHTS, MTL_LDS, StackT, ENVIS, true, PAIR, DRAIN>(a, grid, lds, s);
    } else {
        if (a.max_depth <= 8) launch_one<8, true, LIGHTS, MTL_LDS, StackT, ENVIS, false, PAIR, DRAIN>(a, grid, lds, s);
        else launch_one<64, true, LIGHTS, MTL_LDS, StackT, ENVIS, false, PAIR, DRAIN>(a, grid, lds, s);
    }
}
// DRAIN variants (parked triangles prefetched) for launches that cannot fill the
// chip (a.drained), one-lane-per-pixel ordered kernels only
template <bool LIGHTS, bool MTL_LDS, typename StackT, bool PAIR = false, bool ENVIS = false>
static void launch_ordered(const TraceArgs& a, dim3 grid, size_t lds, hipStream_t s) {
    if constexpr (!PAIR && !ENVIS) {
        if (a.drained) {
            launch_ordered_d<LIGHTS, MTL_LDS, StackT, PAIR, ENVIS, true>(a, grid, lds, s);
            return;
        }
    }
    launch_ordered_d<LIGHTS, MTL_LDS, StackT, PAIR, ENVIS, false>(a, grid, lds, s);
}

// LDS per 256-lane workgroup: [material table][traversal stack][path records],
// within kLdsBudget (TPT_TRACE_WAVES workgroups per CU share the 160 KiB).
constexpr size_t kLdsBudget = (163840 / TPT_TRACE_WAVES) & ~(size_t)255;
constexpr size_t kLdsBudgetIS = (163840 / TPT_TRACE_WAVES_IS) & ~(size_t)255;
constexpr size_t kLdsBudgetPair = (163840 / TPT_TRACE_WAVES_PAIR) & ~(size_t)255;
constexpr size_t kLdsBudgetQuad = (163840 / TPT_TRACE_WAVES_QUAD) & ~(size_t)255;
#ifndef TPT_MTL_LDS_MAX
#define TPT_MTL_LDS_MAX 2048
#endif
constexpr size_t kLdsMtlMax = TPT_MTL_LDS_MAX;   // material tables up to 64 entries go to LDS
constexpr size_t kLdsNodesMax = TPT_LDS_NODES_MAX;

size_t trace_lds_bytes(TraceArgs& a, int words, size_t elem, bool mtl_lds, bool wide, int rec_cols = 256,
                       size_t lds_budget = kLdsBudget, bool quad = false) {
    // [material table][top 4-wide nodes][traversal stack][path records].
    // Priorities (measured on box): the whole stack (a
    // stack capped at 23 of its 40 slots cost 7 %), then path records up to
    // max_depth (records of long paths in private memory slow the heaviest
    // tiles), then as many top nodes as the remaining bytes hold.
    const size_t mtl_bytes = mtl_lds ? ((size_t)(a.n_materials + 1) * 2 * 16 + 127) / 128 * 128 : 0;
    a.mtl_in_lds = mtl_lds ? 1 : 0;
    a.lds_mtl_offset = 0;
    const size_t budget = lds_budget - mtl_bytes;
    const size_t slot = quad ? 64 * elem : 256 * elem;   // (quad: four slots per 256-lane row)
    const size_t level = (size_t)words * (size_t)rec_cols * sizeof(float);
    // The whole stack (capacity + 3 spare slots for the unconditional 4-wide
    // pushes) when the path records of max_depth levels fit beside it.  Else
    // the records first: the ordered walk rarely goes deep (C5: 99 % of visits
    // find <= 5 entries), so the stack keeps as many slots as the records leave,
    // at least 12, and deeper entries spill to private memory.  Measured on C5
    // (44 slots of 32-bit ids): 27 stack slots + 2 record levels 7.63 Grays/s,
    // 19 + 6: 7.97, 12 + 8: 8.20.
    size_t slots = (size_t)a.stack_depth + 3;
#ifndef TPT_RECORDS_FIRST
#define TPT_RECORDS_FIRST 1
#endif
    const size_t want = std::min<size_t>((size_t)a.max_depth, (budget - 12 * slot) / level);
    if (TPT_RECORDS_FIRST ? (slots * slot + want * level > budget) : (slots * slot + 2 * level > budget))
        slots = std::min(slots, std::max<size_t>(12, ((budget - want * level) / slot) & ~(size_t)1));   // even
    const size_t stack = quad ? ((slots + 3) / 4 * 4 * slot + 15) / 16 * 16
                              : ((slots + 1) / 2 * 2 * slot + 15) / 16 * 16;   // even slot count (paired u16 layout)
    size_t levels = (budget - stack) / level;
    if (levels > (size_t)a.max_depth) levels = (size_t)a.max_depth;
    size_t nodes = wide ? (budget - stack - levels * level) / 128 : 0;
    nodes = std::min(nodes, std::min<size_t>((size_t)a.n4, kLdsNodesMax / 128));
    a.lds_nodes = (int)nodes;
    a.lds_nodes_offset = (int)mtl_bytes;
    const size_t head = mtl_bytes + nodes * 128;
    a.stack_lds_slots = (int)slots;
    a.lds_stack_offset = (int)head;
    a.lds_rec_offset = (int)(head + stack);
    a.rec_lds_levels = (int)levels;
    return head + stack + levels * level;
}

// pixel pool (k_trace): two tiles per workgroup, the second drawn from by the
// lanes that finish their pixel first; its LDS counter follows the rest
static void use_tile_pool(TraceArgs& a, dim3& grid, size_t& lds) {
    a.tile_pool = 1;
    grid.x = (grid.x + 1) / 2;
    if (a.xcd_run > 0) {   // runs of workgroups now: half as many, each two tiles wide
        const int per = grid.x % 8 == 0 ? (int)grid.x / 8 : 0, want = std::max(2, a.xcd_run / 2);
        a.xcd_run = 0;
        for (int g = std::min(per, want); g >= 2 && a.xcd_run == 0; --g)
            if (per % g == 0) a.xcd_run = g;
    }
    a.lds_pool_offset = (int)((lds + 15) / 16 * 16);
    lds = (size_t)a.lds_pool_offset + 16;
}

// waves per SIMD the one-lane trace variants are built for (__launch_bounds__):
// with the device's CU count, the resident lanes the host's launch rules use
int trace_waves_per_simd() { return TPT_TRACE_WAVES; }

bool trace_quad_fits(const TraceArgs& a_in) {
    TraceArgs a = a_in;
    const bool small = (2 * (size_t)a.n_faces - 1) <= 65535;
    const bool mtl_lds = (size_t)(a.n_materials + 1) * 2 * sizeof(float4) <= kLdsMtlMax;
    trace_lds_bytes(a, 2, small ? 2 : 4, mtl_lds, true, 256, kLdsBudgetQuad, true);
    return rec_words(a.n_lights, a.n_materials) == 2 && a.stack_lds_slots >= a.stack_depth + 3;
}

hipError_t launch_trace(const TraceArgs& a_in, hipStream_t s) {
    TraceArgs a = a_in;
    a.tile_pool = 0;
    a.lds_pool_offset = 0;
    dim3 grid((a.width + 15) / 16, ((a.band_height + 15) / 16) * (a.n_frames > 0 ? a.n_frames : 1));
    // the XCD-run remap is a permutation of a row's tiles only if runs tile gridDim.x / 8
    if (a.xcd_run > 0 && (grid.x % 8 != 0 || (grid.x / 8) % (unsigned)a.xcd_run != 0)) a.xcd_run = 0;
    if (a.flags & TPT_FLAG_REF_ORDER) {
        // the reference's visit order (tests, diagnostics): one general variant
        const size_t lds = trace_lds_bytes(a, 5, sizeof(int), false, false);
        if (a.env_is) launch_one<64, false, true, false, int, true>(a, grid, lds, s);
        else launch_one<64, false, true, false, int>(a, grid, lds, s);
        return hipGetLastError();
    }
    const bool small = (2 * (size_t)a.n_faces - 1) <= 65535;
    const bool mtl_lds_ok = (size_t)(a.n_materials + 1) * 2 * sizeof(float4) <= kLdsMtlMax;
    if (a.env_is) {
        // opt-in env next-event estimation (A15): variants of their own (the
        // delta-light machinery: 5-word records), so the others stay lean; pair
        // mode hands each diffuse bounce's env shadow ray (and its delta lights'
        // rays) to the side lane
        const bool pair_is = a.pair && (a.n_materials + 1) < (int)kNoProbe;
        if (pair_is) grid.y = ((a.band_height + 7) / 8) * (a.n_frames > 0 ? a.n_frames : 1);
        const size_t lds = trace_lds_bytes(a, 5, small ? 2 : 4, mtl_lds_ok, true, pair_is ? 128 : 256, kLdsBudgetIS);
#define TPT_IS_LAUNCH(MTL, ST)                                                         \
    {                                                                                  \
        if (pair_is) launch_ordered<true, MTL, ST, true, true>(a, grid, lds, s);        \
        else launch_ordered<true, MTL, ST, false, true>(a, grid, lds, s);               \
    }
        if (mtl_lds_ok) {
            if (small) TPT_IS_LAUNCH(true, uint16_t) else TPT_IS_LAUNCH(true, int)
        } else {
            if (small) TPT_IS_LAUNCH(false, uint16_t) else TPT_IS_LAUNCH(false, int)
        }
#undef TPT_IS_LAUNCH
        return hipGetLastError();
    }
    const bool lights = rec_words(a.n_lights, a.n_materials) == 5;
    const bool mtl_lds = (size_t)(a.n_materials + 1) * 2 * sizeof(float4) <= kLdsMtlMax;
    if (a.quad) {
        // four lanes per pixel: 8x8-pixel workgroups; the quads' stacks must lie in
        // LDS whole (the host checked lights == 0)
        grid = dim3((a.width + 7) / 8, ((a.band_height + 7) / 8) * (a.n_frames > 0 ? a.n_frames : 1));
        a.xcd_run = 0;
        const size_t lds = trace_lds_bytes(a, 2, small ? 2 : 4, mtl_lds, true, 256, kLdsBudgetQuad, true);
        if (lights || a.stack_lds_slots < a.stack_depth + 3) return hipErrorInvalidValue;
        if (mtl_lds) {
            if (small) launch_quad<true, uint16_t>(a, grid, lds, s);
            else launch_quad<true, int>(a, grid, lds, s);
        } else {
            if (small) launch_quad<false, uint16_t>(a, grid, lds, s);
            else launch_quad<false, int>(a, grid, lds, s);
        }
        return hipGetLastError();
    }
    // pair mode: delta lights (shadow rays to hand off), packed probe ids
    const bool pair = a.pair && lights && a.n_lights > 0 && (a.n_materials + 1) < (int)kNoProbe;
    if (pair) {
        grid.y = ((a.band_height + 7) / 8) * (a.n_frames > 0 ? a.n_frames : 1);   // 16x8 pixels per workgroup
        const size_t lds = trace_lds_bytes(a, 5, small ? 2 : 4, mtl_lds, true, 128, kLdsBudgetPair);
        if (mtl_lds) {
            if (small) launch_ordered<true, true, uint16_t, true>(a, grid, lds, s);
            else launch_ordered<true, true, int, true>(a, grid, lds, s);
        } else {
            if (small) launch_ordered<true, false, uint16_t, true>(a, grid, lds, s);
            else launch_ordered<true, false, int, true>(a, grid, lds, s);
        }
        return hipGetLastError();
    }
    // pixel pool; its LDS counter comes out of the budget
    const bool use_pool = TPT_TILE_POOL && !a.drained;
    size_t lds = trace_lds_bytes(a, lights ? 5 : 2, small ? 2 : 4, mtl_lds, true, 256, kLdsBudget - (use_pool ? 16 : 0));
    if (use_pool) use_tile_pool(a, grid, lds);
    if (lights) {
        if (mtl_lds) {
            if (small) launch_ordered<true, true, uint16_t>(a, grid, lds, s);
            else launch_ordered<true, true, int>(a, grid, lds, s);
        } else {
            if (small) launch_ordered<true, false, uint16_t>(a, grid, lds, s);
            else launch_ordered<true, false, int>(a, grid, lds, s);
        }
    } else {
        if (mtl_lds) {
            if (small) launch_ordered<false, true, uint16_t>(a, grid, lds, s);
            else launch_ordered<false, true, int>(a, grid, lds, s);
        } else {
            if (small) launch_ordered<false, false, uint16_t>(a, grid, lds, s);
            else launch_ordered<false, false, int>(a, grid, lds, s);
        }
    }
    return hipGetLastError();
}

// Lone-wave step latency (tpt_debug_step_latency; DESIGN.md section 6, "The
// drained chain"): ONE 64-lane wave walks up to 64 rays with the production
// closest-hit traversal (4-wide ordered visits, leaves tested when reached, as
// k_trace_rays mode 1; the sliver pass after the timed walk), its 4-wide nodes read from global
// memory (nodes_lds 0, what k_trace does) or from a copy of the first
// nodes_lds nodes in LDS (the whole main tree: every visit an LDS read), the
// stack in LDS either way.  out[4 * lane]: this lane's visits + leaf tests,
// the wave's loop iterations, the wave's shader cycles (s_memtime) for the
// walk, the hit fid.
constexpr int kLatStackSlots = 64;
// LaneStack's [slot][lane] layout has a 256-lane row per slot (stack_slot_offset)
constexpr size_t kLatStackBytes = (size_t)kLatStackSlots * 256 * sizeof(int);
__global__ __launch_bounds__(64) void k_step_latency(TraceArgs a, uint32_t n, const float* __restrict__ o,
                                                     const float* __restrict__ d, int nodes_lds,
                                                     unsigned long long* __restrict__ out) {
    extern __shared__ __attribute__((aligned(16))) char lds[];
    TPT_LDS char* slds = (TPT_LDS char*)lds;
    const int lane = threadIdx.x;
    TPT_LDS LdsF4* snodes = (TPT_LDS LdsF4*)slds;
    for (int i = lane; i < 8 * nodes_lds; i += 64) {
        const float4 m = a.inner4[i];
        snodes[i].x = m.x;
        snodes[i].y = m.y;
        snodes[i].z = m.z;
        snodes[i].w = m.w;
    }
    __syncthreads();
    LaneStack<int> stk;
    stk.lds = (TPT_LDS int*)(slds + (size_t)nodes_lds * 128) + lane;
    stk.nlds = kLatStackSlots;
    const int nint = a.n_faces - 1;
    const bool active = (uint32_t)lane < n;
    Trav r;
    trav_begin(r, active ? v3(o[3 * lane], o[3 * lane + 1], o[3 * lane + 2]) : v3(0.0f, 0.0f, 0.0f),
               active ? v3(d[3 * lane], d[3 * lane + 1], d[3 * lane + 2]) : v3(1.0f, 1.0f, 1.0f), TM_CLOSEST,
               a.boxes_finite != 0, a.emit_root, a.cull_eps, false);
    if (!active) r.node = -1;
    unsigned long long steps = 0, iters = 0;
    __builtin_amdgcn_s_waitcnt(0);
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    while (__ballot(r.node >= 0) != 0ull) {
        ++iters;
        if (r.node >= 0) {
            ++steps;
            if (r.node < nint) {
                int next;
                if (r.fin) {
                    if (r.node < nodes_lds) {
                        const TPT_LDS LdsF4* nd = snodes + 8 * r.node;
                        next = inner_visit4_q(r, lds_f4(nd), lds_f4(nd + 1), lds_f4(nd + 2), lds_f4(nd + 3),
                                              lds_f4(nd + 4), lds_f4(nd + 5), lds_f4(nd + 6), stk, r.sp);
                    } else {
                        next = inner_visit4(r, a.inner4, nullptr, 0, stk, r.sp);
                    }
                } else {
                    int deferred;
                    bool push;
                    inner_visit<true>(r, a.inner, next, push, deferred);
                    stk.put(r.sp, deferred);
                    r.sp += push ? 1 : 0;
                }
                if (r.sp > a.stack_depth) {
                    r.sp = 0;
                    next = -1;
                }
                r.node = next >= 0 ? next : (r.sp == 0 ? -1 : stk.get(--r.sp));
            } else {
                const bool stop = leaf_test<true>(r, a.tri, r.node - nint, a.cull_eps);
                r.node = (stop || r.sp == 0) ? -1 : stk.get(--r.sp);
            }
        }
    }
    __builtin_amdgcn_s_waitcnt(0);
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    uint32_t c_leaf = 0;
    if (a.n_sliver_groups > 0 && r.fin) sliver_pass(r, a, c_leaf);   // (untimed) the render's hit
    out[4 * lane] = steps;
    out[4 * lane + 1] = iters;
    out[4 * lane + 2] = t1 - t0;
    out[4 * lane + 3] = (unsigned long long)(long long)r.fid;
}

// The same walk with FOUR lanes per ray (nodes_lds < 0; DESIGN.md section 6,
// "Four lanes per ray"): ONE wave, up to 16 rays, ray q on lanes 4q..4q+3 with
// its traversal state replicated, each 4-wide visit split over the quad
// (inner_visit4_quad).  out[4 * q]: ray q's node visits, the wave's iterations,
// the wave's shader cycles, the hit fid.
__global__ __launch_bounds__(64) void k_step_latency_quad(TraceArgs a, uint32_t n, const float* __restrict__ o,
                                                          const float* __restrict__ d,
                                                          unsigned long long* __restrict__ out) {
    extern __shared__ __attribute__((aligned(16))) char lds[];
    const int lane = threadIdx.x, q = lane >> 2, k = lane & 3;
    LaneStack<int, true> stk;
    stk.lds = (TPT_LDS int*)lds + 4 * q;   // the quad's four columns
    stk.nlds = kLatStackSlots;
    const int nint = a.n_faces - 1;
    const bool active = (uint32_t)q < n;
    Trav r;
    trav_begin(r, active ? v3(o[3 * q], o[3 * q + 1], o[3 * q + 2]) : v3(0.0f, 0.0f, 0.0f),
               active ? v3(d[3 * q], d[3 * q + 1], d[3 * q + 2]) : v3(1.0f, 1.0f, 1.0f), TM_CLOSEST,
               a.boxes_finite != 0, a.emit_root, a.cull_eps, false);
    if (!active || !r.fin) r.node = -1;   // finite rays only (chords, camera rays)
    unsigned long long steps = 0, iters = 0;
    uint32_t c_leaf = 0;
    __builtin_amdgcn_s_waitcnt(0);
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    while (__ballot(r.node >= 0) != 0ull) {
        ++iters;
        if (r.node >= 0) {
            ++steps;
            if (r.node >= nint) {   // a one-leaf tree
                leaf_test<true>(r, a.tri, r.node - nint, a.cull_eps);
                r.node = -1;
            } else {
                bool stop;
                int next = inner_visit4_quad(r, a.inner4, a.tri, nint, a.cull_eps, stk, r.sp, stop, c_leaf);
                if (stop || r.sp > a.stack_depth) {
                    r.sp = 0;
                    next = -1;
                }
                r.node = next >= 0 ? next : (r.sp == 0 ? -1 : stk.get(--r.sp));
            }
        }
    }
    __builtin_amdgcn_s_waitcnt(0);
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (a.n_sliver_groups > 0 && r.fin) sliver_pass(r, a, c_leaf);   // (untimed) the render's hit
    if (k == 0) {
        out[4 * q] = steps;
        out[4 * q + 1] = iters;
        out[4 * q + 2] = t1 - t0;
        out[4 * q + 3] = (unsigned long long)(long long)r.fid;
    }
}

hipError_t launch_step_latency_ptr(const void* a, uint32_t n, const float* o, const float* d, int nodes_lds,
                                   unsigned long long* out, hipStream_t s) {
    if (nodes_lds < 0) {   // four lanes per ray
        hipLaunchKernelGGL(k_step_latency_quad, dim3(1), dim3(64), kLatStackBytes, s,
                           *static_cast<const TraceArgs*>(a), n, o, d, out);
        return hipGetLastError();
    }
    const size_t lds = (size_t)nodes_lds * 128 + kLatStackBytes;
    hipLaunchKernelGGL(k_step_latency, dim3(1), dim3(64), lds, s, *static_cast<const TraceArgs*>(a), n, o, d,
                       nodes_lds, out);
    return hipGetLastError();
}

// The host calls the tolerance-mode build (namespace tpt_fast, the same TraceArgs
// layout) through this entry point.
hipError_t launch_trace_ptr(const void* a, hipStream_t s) { return launch_trace(*static_cast<const TraceArgs*>(a), s); }

hipError_t launch_resolve(const ResolveArgs& a, hipStream_t s) {
    dim3 grid((a.width + 255) / 256, a.band_height);
    hipLaunchKernelGGL(k_resolve, grid, dim3(256), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_trace_rays(const TraceArgs& a, uint32_t n, const float* o, const float* d, const int32_t* ofid,
                             int mode, int32_t* hit, float* t, float* uv, hipStream_t s) {
    if (n == 0) return hipSuccess;
    const size_t lds = (size_t)kRaysLdsSlots * 256 * sizeof(int);
    hipLaunchKernelGGL(k_trace_rays, dim3((n + 255) / 256), dim3(256), lds, s, a, n, o, d, ofid, mode, hit, t, uv);
    return hipGetLastError();
}

}  // namespace tpt
