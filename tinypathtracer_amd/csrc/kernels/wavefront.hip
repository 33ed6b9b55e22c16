// wavefront.hip -- the wavefront / ray-queue variant of the hot path
// (north_star "wavefront ballot/compaction ... across bounces"; SURVEY.md 2 and
// 7.6 "a wavefront/queue variant for high-divergence configs"; DESIGN.md
// section 5 "N1: the wavefront variant").  Opt-in: TPT_FLAG_WAVEFRONT.
//
// The reference's per-pixel loops (trace, src/path_tracer.cu:296-435) are cut
// at every traversal (traverseBVH, :61-107) into two kernels that alternate,
// one iteration per ray of every live path:
//   k_wf_logic  one lane per queued ray: consumes the ray's hit and runs the
//               path logic exactly as k_trace's shading pass does -- the hit
//               prelude (:364-381), getNewDirection (:187-225), the delta
//               lights (:265-286), the direct probe (:382-405), the unwind
//               (:416-433), the next sample's camera ray (:42-59) -- then
//               appends the path's next ray to the next queue (wave ballot +
//               one atomic per wave: compaction);
//   k_wf_trace  persistent: every wave keeps its lanes on rays, pulling the
//               next queued ray the moment a lane's ray is done (dynamic
//               fetch, Aila & Laine 2009), with k_trace's ordered 4-wide walk,
//               speculative leaf postponement and exactness guards (sliver
//               re-test, grazing rays and hits, the two-pass direct probe).
// A path's state lives in HBM between iterations: its path records by slot,
// and a 64-B record (RNG, sample counter, phase, ...; 128 B with delta lights)
// that travels with its ray through the queues (so the logic kernel issues the
// loads of a ray, its hit and its state at once); the trace kernel reads only
// the ray (32 B) and writes the hit (16 B).  A slot runs one pixel's samples in order on that
// pixel's own XORWOW stream (path_tracer.cu:39,320), then claims the next
// pixel (one atomic counter), so every pixel's random numbers are consumed in
// the reference's order and its sums are added in the same order as k_trace:
// the image is bit-identical to the megakernel's.
#include "trace_dev.hpp"

namespace tpt {

#ifndef TPT_WF_TRACE_WAVES
#define TPT_WF_TRACE_WAVES 6   // min waves per SIMD requested for k_wf_trace
#endif

// queue entry flags (float4 e1.w): mode | ext << 3 | graze << 4 | probe << 5
enum : uint32_t { WF_EXT = 8u, WF_GRAZE = 16u, WF_PROBE = 32u };
// hit code (q_hit .w): fid >= 0, -1 miss, -2 a probe whose emitter hit is beaten (TM_OCCLUDED)
constexpr int kWfOccluded = -2;
// Queues are split into kWfShards shards (one per XCD): a same-word atomic
// saturates at ~88 per microsecond (MI355X_MICROARCH.md "dequeue"), so one
// queue head and one tail per queue would bound an iteration of 2 M rays at
// ~0.5 ms.  Control words: queue sizes [kWfCount + q * kWfShards + k], fetch
// heads [kWfHead + q * kWfShards + k], the pixel-claim counter [kWfClaim].
// Each control word has a 4-KiB line of its own (kWfCtlStride words): atomics on
// words that share a cache line serialise as if they were one word (measured:
// 8 heads in one line, ~20 dequeues per microsecond in all).
constexpr int kWfCount = 0, kWfHead = 2 * kWfShards, kWfClaim = 4 * kWfShards;
__host__ __device__ constexpr size_t wf_ctl(int word) { return (size_t)word * kWfCtlStride; }

__device__ __forceinline__ uint32_t lane_prefix(unsigned long long mask) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
}

// claim id -> pixel, in k_trace's dispatch order (16x16 tiles, 8x8 per wave),
// so consecutive claims are neighbouring pixels (coherent camera rays)
__device__ __forceinline__ bool wf_pixel(const TraceArgs& a, int c, int& x, int& y, int& frame) {
    const int nfr = a.n_frames > 0 ? a.n_frames : 1;
    const int gx = (a.width + 15) >> 4;
    const int b = c >> 8, tid = c & 255;
    const int bx = b % gx, by = b / gx;
    frame = by % nfr;
    const int wave = tid >> 6, lane = tid & 63;
    x = bx * 16 + (wave & 1) * 8 + (lane & 7);
    const int ly = (by / nfr) * 16 + (wave >> 1) * 8 + (lane >> 3);
    y = band_row(ly, a.band_rows, a.band_count, a.band_index, a.band_list);
    return x < a.width && ly < a.band_height && y < a.height;
}

// ---------------------------------------------------------------------------
// k_wf_logic: one lane per ray of queue `cur` (init: one lane per slot, no ray).
// Path state words, beside each queue entry (LIGHTS: 32, else 16):
//   0-5 XORWOW {v0..v4, d}; 6 claim id (-1: none); 7 samples left;
//   8 phase | depth << 3 | li << 10 | graze_next << 15 | env_pending << 16;
//   9 mk (material | p-kind << 30); 10-12 nd (next extension direction);
//   13-15 totalRad;  LIGHTS: 16-18 rd (extension direction); 19-21 shading
//   normal; 22-24 direct; 25-26 gsurf (the face the shadow rays leave);
//   27-29 env_k (A15).
// ---------------------------------------------------------------------------
template <bool ORDERED, bool LIGHTS, bool ENVIS>
__global__ __launch_bounds__(256) void k_wf_logic(WfArgs w, int init) {
    constexpr int SW = LIGHTS ? 32 : 16;
    const TraceArgs& a = w.t;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int cur = w.it & 1, nxt = (w.it + 1) & 1;
    // the input: queue `cur`, the concatenation of its kWfShards shards (init: the slots)
    int pre[kWfShards + 1];
    pre[0] = 0;
#pragma unroll
    for (int k = 0; k < kWfShards; ++k)
        pre[k + 1] = pre[k] + (init ? 0 : (int)w.ctl[wf_ctl(kWfCount + cur * kWfShards + k)]);
    const int n = init ? w.n_slots : pre[kWfShards];
    const float4* __restrict__ qin = cur ? w.q_ray1 : w.q_ray0;
    float4* __restrict__ qout = nxt ? w.q_ray1 : w.q_ray0;
    // this block appends to shard blockIdx % kWfShards of the next queue (the grid is a
    // multiple of kWfShards, so a shard receives at most every kWfShards-th 256-chunk of
    // the input: shard_cap entries)
    const int oshard = (int)blockIdx.x & (kWfShards - 1);
    uint32_t* const ocount = w.ctl + wf_ctl(kWfCount + nxt * kWfShards + oshard);
    __shared__ uint32_t s_wcnt[4], s_base;
    const int rw = w.rec_words;
    const size_t npix = (size_t)a.width * (size_t)a.height;
    uint32_t c_trav = 0, c_shade = 0, c_local = 0;
    const float4* __restrict__ mt = a.mtl;
    for (int base = blockIdx.x * 256; base < n; base += gridDim.x * 256) {
        const int j = base + tid;
        const bool valid = j < n;
        int slot = init ? j : 0;
        size_t e = 0;   // the input entry's position (shard * shard_cap + offset)
        V3 ro = v3(0.0f, 0.0f, 0.0f), rdir = ro;
        float4 h = make_float4(0.0f, 0.0f, 0.0f, __int_as_float(-1));
        if (valid && !init) {
            int k = 0;
#pragma unroll
            for (int i = 1; i < kWfShards; ++i) k += j >= pre[i] ? 1 : 0;
            e = (size_t)k * (size_t)w.shard_cap + (size_t)(j - pre[k]);
            const float4 e0 = qin[2 * e], e1 = qin[2 * e + 1];
            slot = __float_as_int(e0.w);
            ro = v3(e0.x, e0.y, e0.z);
            rdir = v3(e1.x, e1.y, e1.z);
            h = w.q_hit[e];
        }
        // the path's state travels with its ray: entry e of the input queue's state array
        const uint32_t* sp = (cur ? w.st1 : w.st0) + e * SW;
        float* rec = w.rec + (size_t)slot * (size_t)a.max_depth * (size_t)rw;
        // ---- slot state ----
        uint32_t st[6] = {0, 0, 0, 0, 0, 0};
        int pix = -1, remaining = 0;
        uint32_t ctl = PH_CAMERA, mk = 0;
        V3 nd = v3(0.0f, 0.0f, 0.0f), total = nd, rd = nd, nrm = nd, direct = nd, env_k = nd;
        Surf gsurf = no_surface();
        if (valid && !init) {
            const uint4 s0 = ((const uint4*)sp)[0], s1 = ((const uint4*)sp)[1], s2 = ((const uint4*)sp)[2],
                        s3 = ((const uint4*)sp)[3];
            st[0] = s0.x; st[1] = s0.y; st[2] = s0.z; st[3] = s0.w; st[4] = s1.x; st[5] = s1.y;
            pix = (int)s1.z;
            remaining = (int)s1.w;
            ctl = s2.x;
            mk = s2.y;
            nd = v3(__uint_as_float(s2.z), __uint_as_float(s2.w), __uint_as_float(s3.x));
            total = v3(__uint_as_float(s3.y), __uint_as_float(s3.z), __uint_as_float(s3.w));
            if constexpr (LIGHTS) {
                const uint4 s4 = ((const uint4*)sp)[4], s5 = ((const uint4*)sp)[5], s6 = ((const uint4*)sp)[6],
                            s7 = ((const uint4*)sp)[7];
                rd = v3(__uint_as_float(s4.x), __uint_as_float(s4.y), __uint_as_float(s4.z));
                nrm = v3(__uint_as_float(s4.w), __uint_as_float(s5.x), __uint_as_float(s5.y));
                direct = v3(__uint_as_float(s5.z), __uint_as_float(s5.w), __uint_as_float(s6.x));
                gsurf = Surf{__uint_as_float(s6.y), __uint_as_float(s6.z)};
                env_k = v3(__uint_as_float(s6.w), __uint_as_float(s7.x), __uint_as_float(s7.y));
            }
        }
        int phase = (int)(ctl & 7u), depth = (int)((ctl >> 3) & 127u), li = (int)((ctl >> 10) & 31u);
        bool graze_next = (ctl >> 15) & 1u, env_pending = (ctl >> 16) & 1u;
        bool emit = false, shadow = false, tg = false;
        V3 to = ro, td = rd;
        // the level's record (k_trace put_level, non-pair): 2 words packed, or 5
        auto put_level = [&](uint32_t pm, V3 dl) {
            if (rw == 2) {
                rec[depth * 2 + 1] = __uint_as_float(mk | (pm << 15));
            } else {
                rec[depth * rw + 1] = __uint_as_float(mk);
                rec[depth * rw + 2] = dl.x;
                rec[depth * rw + 3] = dl.y;
                rec[depth * rw + 4] = dl.z;
            }
        };
        if (valid && !init) {
            // ---- consume the finished ray (k_trace's shading pass, path_tracer.cu:356-433) ----
            const int fid = __float_as_int(h.w);
            bool finish = false, lights_next = false, after = false;
            Hemi hb;
            bool hb_ok = false;
            V3 L = v3(0.0f, 0.0f, 0.0f);
            if (!LIGHTS) rd = rdir;   // the extension ray's direction
            Surf gpass = gsurf;
            if (phase == PH_EXT) {
                if (fid < 0) {   // miss: env radiance seeds the unwind (:358-362)
                    if (a.env) L = env_lookup<ENVIS>(a.env, a.env_w, a.env_h, rd);
                    finish = true;
                } else {   // hit shading prelude (:364-381); grazing hits were re-traced by k_wf_trace
                    const float4* sh = a.shade + 3 * fid;
                    const float4 s0 = sh[0], s1 = sh[1], s2 = sh[2];
                    ++c_shade;
                    const float u = h.y, v = h.z;
                    const float wb = 1.0f - u - v;
                    nrm = normalize(((wb * v3(s0.x, s0.y, s0.z)) + (u * v3(s1.x, s1.y, s1.z))) +
                                    (v * v3(s2.x, s2.y, s2.z)));
                    gpass = a.graze ? Surf{s1.w, s2.w} : no_surface();
                    if constexpr (LIGHTS) gsurf = gpass;
                    ro = ro + (h.x * rd);
                    const int mtl = __float_as_int(s0.w);
                    const float4 m1 = mt[2 * mtl + 1];
                    float af;
                    const float prob = new_direction(rd, nrm, m1.x, m1.y, st, nd, af, hb, hb_ok);
                    graze_next = grazing(gpass, nd);
                    rec[depth * rw] = af;
                    mk = (uint32_t)mtl | (p_kind(prob) << 30);
                    direct = v3(0.0f, 0.0f, 0.0f);
                    li = 0;
                    env_pending = ENVIS && !(m1.x > 0.0f) && !(m1.y > 0.0f);   // diffuse hit
                    lights_next = true;
                }
            } else if (LIGHTS && phase == PH_SHADOW) {
                if (fid < 0) {   // sampleDeltaLights :279-282
                    V3 ldir, lrad;
                    light_sample(a.lights, li, ro, ldir, lrad);
                    const float4 m0 = mt[2 * (mk & 0x3fffffffu)];
                    direct = direct + (v3(m0.x, m0.y, m0.z) * lrad);
                }
                ++li;
                lights_next = true;
            } else if (ENVIS && phase == PH_ENVSHADOW) {   // env next-event estimate (A15, opt-in)
                if (fid < 0) direct = direct + env_k;
                lights_next = true;
            } else if (phase == PH_PROBE) {   // :390-400
                V3 dl = LIGHTS ? direct : v3(0.0f, 0.0f, 0.0f);
                uint32_t pm = kNoProbe;
                if (fid >= 0) {   // the closest hit (an unbeaten emitter after pass 2)
                    pm = (uint32_t)__float_as_int(a.shade[3 * fid].w);
                    const float e = mt[2 * pm].w;
                    dl = (v3(1.0f, 1.0f, 1.0f) * v3(e, e, e)) + dl;
                }
                put_level(pm, dl);
                after = true;
            }
            td = rd;
            if (lights_next) {
                const float4 m1 = mt[2 * (mk & 0x3fffffffu) + 1];
                if (LIGHTS && li < a.n_lights) {
                    V3 lrad;
                    light_sample(a.lights, li, ro, td, lrad);
                    tg = grazing(gsurf, td);
                    phase = PH_SHADOW;
                    shadow = true;
                } else {
                    bool env_ray = false;
                    if (ENVIS && env_pending) {   // after the delta lights, before the probe
                        env_pending = false;
                        const V3 nf = (dot(rd, nrm) > 0.0f ? -1.0f : 1.0f) * nrm;   // getNewDirection's flip
                        const float x1 = xorwow_uniform(st);
                        const float x2 = xorwow_uniform(st);
                        if (env_is_sample(a, nf, x1, x2, td, env_k)) {
                            phase = PH_ENVSHADOW;
                            shadow = true;
                            env_ray = true;
                            tg = grazing(gsurf, td);
                        }
                    }
                    if (env_ray) {
                    } else if (!(m1.x >= 1.0f || m1.y > 0.0f)) {   // direct probe (:387-389)
                        float af2;
                        hb_ok = false;
                        new_direction(rd, nrm, m1.x, m1.y, st, td, af2, hb, hb_ok);
                        if ((TPT_PROBE_SHORTCUT && ORDERED && !a.any_emitter) ||
                            (ORDERED && probe_misses_emitters(a, ro, td))) {
                            // the probe's emitter pass ends with no hit, exactly as a
                            // traversal would (still counted: the reference traces it)
                            ++c_trav;
                            ++c_local;
                            put_level(kNoProbe, direct);
                            after = true;
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
            if (after) {
                const float e = mt[2 * (mk & 0x3fffffffu)].w;
                if (e > 0.0f) {   // an emitter ends the path (:408-412)
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
            if (finish) {   // unwind (:416-431): levels depth-1 .. 0
                for (int k = depth - 1; k >= 0; --k) {
                    const float af = rec[k * rw];
                    const uint32_t w1 = __float_as_uint(rec[k * rw + 1]);
                    const bool packed = rw == 2;
                    const float4 mb = mt[2 * (w1 & (packed ? 0x7fffu : 0x3fffffffu))];
                    const V3 att = af * v3(mb.x, mb.y, mb.z);   // :379
                    const uint32_t kind = w1 >> 30;
                    const float prob = kind == 0u ? af : (kind == 1u ? -0.0f : 0.0f);
                    const float ivp = 1.0f / prob;   // :427 "/ pStack"
                    V3 dst;
                    if (packed) {
                        const uint32_t pm = (w1 >> 15) & 0x7fffu;
                        const float e = pm == kNoProbe ? 0.0f : mt[2 * pm].w;
                        dst = pm == kNoProbe ? v3(0.0f, 0.0f, 0.0f)
                                             : (v3(1.0f, 1.0f, 1.0f) * v3(e, e, e)) + v3(0.0f, 0.0f, 0.0f);
                    } else {
                        dst = v3(rec[k * rw + 2], rec[k * rw + 3], rec[k * rw + 4]);
                    }
                    L = ivp * ((dst + L) * att);
                }
                total = total + L;
                phase = PH_CAMERA;
            }
            to = ro;
        }
        // ---- a finished pixel is stored, and the slot claims the next one ----
        bool need = valid && phase == PH_CAMERA && remaining == 0;
        if (need && pix >= 0) {
            int x, y, fr;
            wf_pixel(a, pix, x, y, fr);
            const size_t off = (size_t)x + (size_t)y * (size_t)a.width;
            uint32_t* g_rng = a.rng + (size_t)fr * 6 * npix;
            float* g_acc = a.accum + (size_t)fr * 3 * npix;
#pragma unroll
            for (int i = 0; i < 6; ++i) g_rng[i * npix + off] = st[i];
            g_acc[off] = total.x;
            g_acc[npix + off] = total.y;
            g_acc[2 * npix + off] = total.z;
        }
        bool alive = valid && !need;
        int px = 0, py = 0;
        if (init && valid && j < w.n_claims) {   // the first pixel of slot j is claim id j (no atomic)
            int fr;
            if (wf_pixel(a, j, px, py, fr)) {
                need = false;
                alive = true;
                pix = j;
                const size_t off = (size_t)px + (size_t)py * (size_t)a.width;
                const uint32_t* g_rng = a.rng + (size_t)fr * 6 * npix;
                const float* g_acc = a.accum + (size_t)fr * 3 * npix;
#pragma unroll
                for (int i = 0; i < 6; ++i) st[i] = g_rng[i * npix + off];
                total = v3(g_acc[off], g_acc[npix + off], g_acc[2 * npix + off]);
                remaining = a.samples;
                phase = PH_CAMERA;
            }
        }
        for (;;) {   // (wave-uniform) claims: one atomic per wave and round (ids from n_slots on)
            const unsigned long long m = __ballot(need);
            if (m == 0ull) break;
            const int first = __builtin_ctzll(m);
            int cb = 0;
            if (lane == first) cb = (int)atomicAdd(&w.ctl[wf_ctl(kWfClaim)], (uint32_t)__popcll(m));
            cb = __shfl(cb, first, 64);
            if (need) {
                const int c = cb + (int)lane_prefix(m);
                if (c >= w.n_claims) {
                    need = false;   // no pixel left: the slot retires
                } else {
                    int fr;
                    if (wf_pixel(a, c, px, py, fr)) {
                        need = false;
                        alive = true;
                        pix = c;
                        const size_t off = (size_t)px + (size_t)py * (size_t)a.width;
                        const uint32_t* g_rng = a.rng + (size_t)fr * 6 * npix;
                        const float* g_acc = a.accum + (size_t)fr * 3 * npix;
#pragma unroll
                        for (int i = 0; i < 6; ++i) st[i] = g_rng[i * npix + off];
                        total = v3(g_acc[off], g_acc[npix + off], g_acc[2 * npix + off]);
                        remaining = a.samples;
                        phase = PH_CAMERA;
                    }
                }
            }
        }
        if (alive && phase == PH_CAMERA) {
            if (remaining == 0) {
                alive = false;   // (a claimed pixel with no samples: samples == 0 is rejected by the host)
            } else {
                int fr;
                wf_pixel(a, pix, px, py, fr);
                --remaining;
                // sampleRays (path_tracer.cu:42-59)
                const float ju = xorwow_uniform(st);
                const float jv = xorwow_uniform(st);
                float lx = ju * 1.0f, lyf = jv * 1.0f;
                lx = lx + (float)px;
                lyf = lyf + (float)py;
                lx = lx * a.inv_w;
                lyf = lyf * a.inv_h;
                lx = lx * a.sensor_w;
                lyf = lyf * a.sensor_h;
                float r4[4];
                mat4_vec4(a.c2w, lx - a.half_sw, lyf - a.half_sh, 0.0f - 1.0f, 0.0f, r4);
                rd = normalize(v3(r4[0], r4[1], r4[2]));
                td = rd;
                to = v3(a.origin[0], a.origin[1], a.origin[2]);
                tg = false;
                depth = 0;
                phase = PH_EXT;
            }
        }
        emit = alive;
        // ---- the path's next ray, compacted into the next queue: one atomic per block ----
        const unsigned long long em = __ballot(emit);
        if (lane == 0) s_wcnt[wave] = (uint32_t)__popcll(em);
        __syncthreads();
        if (tid == 0) {
            const uint32_t tot = s_wcnt[0] + s_wcnt[1] + s_wcnt[2] + s_wcnt[3];
            s_base = tot ? atomicAdd(ocount, tot) : 0u;
        }
        __syncthreads();
        uint32_t wb = s_base;
        for (int i = 0; i < wave; ++i) wb += s_wcnt[i];
        __syncthreads();   // (s_wcnt / s_base are rewritten by the next stride)
        {
            if (emit) {
                ++c_trav;
                const size_t k = (size_t)oshard * (size_t)w.shard_cap + wb + lane_prefix(em);
                const int mode = shadow ? TM_ANY : ((ORDERED && phase == PH_PROBE) ? TM_EMIT : TM_CLOSEST);
                const uint32_t fl = (uint32_t)mode | (phase == PH_EXT ? WF_EXT : 0u) | (tg ? WF_GRAZE : 0u) |
                                    (phase == PH_PROBE ? WF_PROBE : 0u);
                qout[2 * (size_t)k] = make_float4(to.x, to.y, to.z, __int_as_float(slot));
                qout[2 * (size_t)k + 1] = make_float4(td.x, td.y, td.z, __uint_as_float(fl));
                const uint32_t c2 = (uint32_t)phase | ((uint32_t)depth << 3) | ((uint32_t)li << 10) |
                                    (graze_next ? 1u << 15 : 0u) | (env_pending ? 1u << 16 : 0u);
                uint4* so = (uint4*)((nxt ? w.st1 : w.st0) + k * SW);
                so[0] = make_uint4(st[0], st[1], st[2], st[3]);
                so[1] = make_uint4(st[4], st[5], (uint32_t)pix, (uint32_t)remaining);
                so[2] = make_uint4(c2, mk, __float_as_uint(nd.x), __float_as_uint(nd.y));
                so[3] = make_uint4(__float_as_uint(nd.z), __float_as_uint(total.x), __float_as_uint(total.y),
                                   __float_as_uint(total.z));
                if constexpr (LIGHTS) {
                    so[4] = make_uint4(__float_as_uint(rd.x), __float_as_uint(rd.y), __float_as_uint(rd.z),
                                       __float_as_uint(nrm.x));
                    so[5] = make_uint4(__float_as_uint(nrm.y), __float_as_uint(nrm.z), __float_as_uint(direct.x),
                                       __float_as_uint(direct.y));
                    so[6] = make_uint4(__float_as_uint(direct.z), __float_as_uint(gsurf.x), __float_as_uint(gsurf.y),
                                       __float_as_uint(env_k.x));
                    so[7] = make_uint4(__float_as_uint(env_k.y), __float_as_uint(env_k.z), 0u, 0u);
                }
            }
        }
    }
    const unsigned long long s_trav = wave_sum(c_trav), s_shade = wave_sum(c_shade), s_local = wave_sum(c_local);
    if (lane == 0 && (s_trav | s_shade | s_local)) {
        atomicAdd(&a.counters[0], s_trav);
        atomicAdd(&a.counters[3], s_shade);
        atomicAdd(&a.counters[9], s_local);
    }
}

// ---------------------------------------------------------------------------
// k_wf_trace: persistent; the waves pull rays from queue `cur` until every shard
// is exhausted.  Like k_trace, a wave steps its lanes' traversals while at least
// w.refill of them are traversing; then, in one pass, the lanes whose walk has
// ended run the culling guards' extra passes (sliver re-test, grazing re-trace,
// the probe's occlusion pass) or write their hit, and the idle lanes take the
// next queued rays.  A wave dequeues w.chunk entries per atomic from its XCD's
// shard (blockIdx % kWfShards), then from the others; it ends when the queue is
// exhausted and its lanes are done.
// ---------------------------------------------------------------------------
enum : int { WT_IDLE = 0, WT_TRAV = 1, WT_DONE = 2 };

template <bool ORDERED, typename StackT>
__global__ __launch_bounds__(256, TPT_WF_TRACE_WAVES) void k_wf_trace(WfArgs w) {
    extern __shared__ __attribute__((aligned(16))) char lds[];
    const TraceArgs& a = w.t;
    const int tid = threadIdx.x, lane = tid & 63;
    const int cur = w.it & 1, nxt = (w.it + 1) & 1;
    if (blockIdx.x == 0 && tid < 2 * kWfShards) {   // the next queue starts empty (its last reader was it - 1)
        const int k = tid & (kWfShards - 1);
        w.ctl[wf_ctl((tid < kWfShards ? kWfCount : kWfHead) + nxt * kWfShards + k)] = 0u;
    }
    int cnts[kWfShards];   // (uniform) shard sizes of queue `cur`
    int total = 0;
#pragma unroll
    for (int k = 0; k < kWfShards; ++k) {
        cnts[k] = (int)w.ctl[wf_ctl(kWfCount + cur * kWfShards + k)];
        total += cnts[k];
    }
    if (total == 0) return;
    uint32_t* heads = w.ctl + wf_ctl(kWfHead + cur * kWfShards);
    const float4* __restrict__ q = cur ? w.q_ray1 : w.q_ray0;
    const int nint = a.n_faces - 1;
    TPT_LDS char* slds = (TPT_LDS char*)lds;
    LaneStack<StackT> stk;
    stk.lds = (TPT_LDS StackT*)(slds + w.lds_stack_offset) + tid;
    stk.nlds = w.stack_lds_slots;
    uint32_t c_inner = 0, c_wide = 0, c_leaf = 0, c_ovf = 0;
    Trav r;
    trav_begin(r, v3(0.0f, 0.0f, 0.0f), v3(1.0f, 1.0f, 1.0f), TM_CLOSEST);
    r.node = -1;
    int ts = WT_IDLE;
    bool sl_pend = false;
    size_t qi = 0;
    uint32_t fl = 0;
    // (wave-uniform) the entries this wave has taken and not yet handed out, its shard
    int shard = (int)blockIdx.x & (kWfShards - 1), tried = 0;
    size_t chunk_next = 0, chunk_end = 0;
    bool exhausted = false;
    const int thr = w.refill;
    for (;;) {
        // ---- pass: finished walks, then refills ----
        if (ts == WT_DONE) {
            if (ORDERED && a.n_sliver_groups > 0 && sl_pend) {
                sl_pend = false;
                sliver_pass(r, a, c_leaf);
            }
            ts = WT_TRAV;
            if (TPT_GRAZE_HIT && ORDERED && (fl & WF_PROBE) && r.fin && r.fid >= 0 && r.mode == TM_EMIT && a.graze &&
                grazing(Surf{a.shade[3 * r.fid + 1].w, a.shade[3 * r.fid + 2].w}, r.d)) {
                // a grazing probe hit: pass 1 again on the uncull'd binary path
                trav_begin(r, r.o, r.d, r.mode, a.boxes_finite != 0, a.emit_root, a.cull_eps, true);
                sl_pend = false;
            } else if (ORDERED && (fl & WF_PROBE) && r.mode == TM_EMIT && r.fid >= 0) {
                // probe pass 2: does anything beat the emitter hit?
                r.mode = TM_OCCL;
                r.node = 0;
                r.sp = 0;
                r.pend = -1;
                sl_pend = true;
            } else if (TPT_GRAZE_HIT && ORDERED && (fl & WF_EXT) && r.fin && r.fid >= 0 && a.graze &&
                       grazing(Surf{a.shade[3 * r.fid + 1].w, a.shade[3 * r.fid + 2].w}, r.d)) {
                // a grazing extension hit: traced again on the uncull'd binary path
                trav_begin(r, r.o, r.d, TM_CLOSEST, a.boxes_finite != 0, a.emit_root, a.cull_eps, true);
                sl_pend = true;
            } else {
                w.q_hit[qi] = make_float4(r.t, r.u, r.v, __int_as_float(r.mode == TM_OCCLUDED ? kWfOccluded : r.fid));
                ts = WT_IDLE;
            }
        }
        const unsigned long long idle = __ballot(ts == WT_IDLE);
        if (idle != 0ull && !exhausted) {
            const int nidle = __popcll(idle), rank = (int)lane_prefix(idle);
            int got = 0;
            bool mine = false;
            while (got < nidle) {
                if (chunk_next >= chunk_end) {   // dequeue w.chunk entries: this shard, then the next ones
                    bool ok = false;
                    while (tried < kWfShards) {
                        int cnt = 0;
#pragma unroll
                        for (int k = 0; k < kWfShards; ++k) cnt = k == shard ? cnts[k] : cnt;
                        uint32_t* hd = heads + wf_ctl(shard);
                        // (a head read at or past its shard's size stays there: skip the atomic)
                        int b = cnt;
                        if (lane == 0 && (int)__hip_atomic_load(hd, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < cnt)
                            b = (int)atomicAdd(hd, (uint32_t)w.chunk);
                        b = __shfl(b, 0, 64);
                        if (b < cnt) {
                            chunk_next = (size_t)shard * (size_t)w.shard_cap + (size_t)b;
                            chunk_end = (size_t)shard * (size_t)w.shard_cap + (size_t)min(b + w.chunk, cnt);
                            ok = true;
                            break;
                        }
                        shard = (shard + 1) & (kWfShards - 1);
                        ++tried;
                    }
                    if (!ok) {
                        exhausted = true;
                        break;
                    }
                }
                const int take = min(nidle - got, (int)(chunk_end - chunk_next));
                if (ts == WT_IDLE && rank >= got && rank < got + take) {
                    qi = chunk_next + (size_t)(rank - got);
                    mine = true;
                }
                chunk_next += (size_t)take;
                got += take;
            }
            if (mine) {
                const float4 e0 = q[2 * qi], e1 = q[2 * qi + 1];
                fl = __float_as_uint(e1.w);
                trav_begin(r, v3(e0.x, e0.y, e0.z), v3(e1.x, e1.y, e1.z), (int)(fl & 7u), a.boxes_finite != 0,
                           a.emit_root, a.cull_eps, (fl & WF_GRAZE) != 0u);
                ts = WT_TRAV;
                sl_pend = true;
            }
        }
        if (__ballot(ts == WT_TRAV) == 0ull) break;   // nothing traversing, nothing left to take
        // ---- traversal: step while enough lanes are still traversing (k_trace's loop) ----
        for (;;) {
            const int cnt = __popcll(__ballot(ts == WT_TRAV));
            if (cnt == 0) break;
            if (cnt < thr && (__ballot(ts == WT_DONE) != 0ull || (!exhausted && __ballot(ts == WT_IDLE) != 0ull)))
                break;
            bool inner_ready = false, hl = false, blocked = false;
            const bool at_inner = ts == WT_TRAV && r.node >= 0 && r.node < nint;
            if (ts == WT_TRAV) {
                if (at_inner) {
                    int next;
                    if (ORDERED && r.fin) {
                        ++c_wide;
                        next = inner_visit4(r, a.inner4, nullptr, 0, stk, r.sp);
                    } else {
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
                }
                hl = r.pend >= 0;
                inner_ready = r.node >= 0 && r.node < nint;
                blocked = hl && !inner_ready;
            }
            const unsigned long long hb = __ballot(hl);
            if (hb != 0ull) {
                const bool go = __popcll(__ballot(blocked)) >= a.leaf_kb || __popcll(hb) >= TPT_LEAF_KP ||
                                __ballot(inner_ready) == 0ull;
                if (go && hl) {
                    ++c_leaf;
                    if (leaf_test<ORDERED>(r, a.tri, r.pend, a.cull_eps)) {
                        r.node = -1;
                        r.sp = 0;
                    }
                    r.pend = -1;
                }
            }
            if (ts == WT_TRAV && r.node < 0 && r.pend < 0) ts = WT_DONE;
        }
    }
    const unsigned long long s_inner = wave_sum(c_inner), s_wide = wave_sum(c_wide), s_leaf = wave_sum(c_leaf),
                             s_ovf = wave_sum(c_ovf);
    if (lane == 0 && (s_inner | s_wide | s_leaf | s_ovf)) {
        atomicAdd(&a.counters[1], s_inner);
        atomicAdd(&a.counters[2], s_leaf);
        if (s_ovf) atomicAdd(&a.counters[4], s_ovf);
        atomicAdd(&a.counters[5], s_wide);
    }
}

// ---------------------------------------------------------------------------
// host side: variant dispatch and the iteration loop
// ---------------------------------------------------------------------------
template <bool ORDERED, bool LIGHTS, bool ENVIS>
static void launch_logic(const WfArgs& w, int init, hipStream_t s) {
    hipLaunchKernelGGL((k_wf_logic<ORDERED, LIGHTS, ENVIS>), dim3(w.logic_blocks), dim3(256), 0, s, w, init);
}
static void wf_logic(const WfArgs& w, int init, hipStream_t s) {
    const bool lights = w.state_words == 32;
    if (!w.ordered) {
        if (w.t.env_is) launch_logic<false, true, true>(w, init, s);
        else launch_logic<false, true, false>(w, init, s);
    }
    else if (w.t.env_is) launch_logic<true, true, true>(w, init, s);
    else if (lights) launch_logic<true, true, false>(w, init, s);
    else launch_logic<true, false, false>(w, init, s);
}
static void wf_trace(const WfArgs& w, hipStream_t s) {
    const bool small = (2 * (size_t)w.t.n_faces - 1) <= 65535;
    const dim3 g(w.trace_blocks), b(256);
    if (!w.ordered) hipLaunchKernelGGL((k_wf_trace<false, int>), g, b, w.lds_bytes, s, w);
    else if (small) hipLaunchKernelGGL((k_wf_trace<true, uint16_t>), g, b, w.lds_bytes, s, w);
    else hipLaunchKernelGGL((k_wf_trace<true, int>), g, b, w.lds_bytes, s, w);
}

// LDS of k_wf_trace: the traversal stack only ([slot][lane]), within the share of
// a CU's 160 KiB one of TPT_WF_TRACE_WAVES workgroups gets; deeper slots private.
size_t wf_trace_lds(WfArgs& w) {
    const size_t elem = (w.ordered && (2 * (size_t)w.t.n_faces - 1) <= 65535) ? 2 : 4;
    const size_t budget = (163840 / TPT_WF_TRACE_WAVES) & ~(size_t)255;
    size_t slots = (size_t)w.t.stack_depth + 3;
    slots = std::min(slots, budget / (256 * elem));
    w.stack_lds_slots = (int)slots;
    w.lds_stack_offset = 0;
    w.lds_bytes = (int)(slots * 256 * elem);
    return (size_t)w.lds_bytes;
}

// persistent grid of k_wf_trace: as many workgroups as the CUs hold at once
static hipError_t wf_trace_grid(WfArgs& w) {
    int dev = 0, cus = 0, per = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e == hipSuccess) e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (e != hipSuccess) return e;
    const bool small = (2 * (size_t)w.t.n_faces - 1) <= 65535;
    if (!w.ordered)
        e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, k_wf_trace<false, int>, 256, w.lds_bytes);
    else if (small)
        e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, k_wf_trace<true, uint16_t>, 256, w.lds_bytes);
    else
        e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, k_wf_trace<true, int>, 256, w.lds_bytes);
    if (e != hipSuccess) return e;
    w.trace_blocks = std::max(1, cus) * std::max(1, per);
    return hipSuccess;
}

hipError_t launch_wavefront(WfArgs w, uint32_t* h_count, hipEvent_t ev[2], int32_t* iterations, hipStream_t s) {
    wf_trace_lds(w);
    hipError_t e0 = w.trace_blocks > 0 ? hipSuccess : wf_trace_grid(w);
    if (e0 != hipSuccess) return e0;
    hipError_t e = hipMemsetAsync(w.ctl, 0, kWfCtlWords * sizeof(uint32_t), s);
    if (e != hipSuccess) return e;
    // slot j starts on claim id j; later claims count from n_slots
    if ((e = hipMemsetD32Async((hipDeviceptr_t)(w.ctl + wf_ctl(kWfClaim)), (int)w.n_slots, 1, s)) != hipSuccess)
        return e;
    w.it = -1;   // init: every slot claims a pixel and queues its first camera ray into queue 0
    wf_logic(w, 1, s);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    // Iterations in batches; after each batch the next queue's size is copied
    // back, and the loop stops at the first empty queue (the batch enqueued
    // behind it then runs on empty queues: its kernels exit at once).
    const int kBatch = w.batch > 0 ? w.batch : 32;
    const long long kMaxIt = 1ll << 28;
    int it = 0, nb = 0;
    for (;;) {
        for (int k = 0; k < kBatch; ++k, ++it) {
            w.it = it;
            wf_trace(w, s);
            wf_logic(w, 0, s);
        }
        if ((e = hipGetLastError()) != hipSuccess) return e;
        // shard sizes of the queue the last logic launch wrote (queue it & 1)
        for (int k = 0; k < kWfShards; ++k)
            if ((e = hipMemcpyAsync(h_count + (nb & 1) * kWfShards + k, w.ctl + wf_ctl(kWfCount + (it & 1) * kWfShards + k),
                                    sizeof(uint32_t), hipMemcpyDeviceToHost, s)) != hipSuccess)
                return e;
        if ((e = hipEventRecord(ev[nb & 1], s)) != hipSuccess) return e;
        if (nb > 0) {   // the previous batch's count (the current one keeps the GPU busy meanwhile)
            if ((e = hipEventSynchronize(ev[(nb - 1) & 1])) != hipSuccess) return e;
            uint32_t left = 0;
            for (int k = 0; k < kWfShards; ++k) left += h_count[((nb - 1) & 1) * kWfShards + k];
            if (left == 0u) break;
        }
        ++nb;
        if (it > kMaxIt) return hipErrorLaunchTimeOut;
    }
    *iterations = it;
    return hipSuccess;
}

}  // namespace tpt
