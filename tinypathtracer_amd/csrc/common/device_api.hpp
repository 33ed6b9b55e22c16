// device_api.hpp -- launch entry points of the HIP kernels (host-callable).
//
// HBM layout of a built scene (see DESIGN.md "Data layout"):
//   inner[4*(F-1)] float4  internal node i: both child AABBs + child links
//       q0 = (L.min.xyz, L.max.x)  q1 = (L.max.yz, R.min.xy)
//       q2 = (R.min.z, R.max.xyz)  q3 = (bits(left), bits(right), 0, 0)
//     child ids use the reference numbering (bvh.cu:164-214): id >= F-1 is
//     the leaf at sorted position id-(F-1).  Bit 30 of every child link is
//     set when that child's subtree holds an emissive triangle; traversals
//     mask it off.
//   inner4[8*(F-1)] float4  4-wide nodes for the ordered traversal, numbered
//     breadth-first: child k box = floats 6k..6k+5 of q0..q5 (min.xyz,
//     max.xyz), q6 = child ids (-1: none; a 4-wide node id < F-1, or F-1 +
//     leaf position).  Default (wide_bvh.cpp, host): an SAH tree over the
//     LBVH's exact leaf boxes in [0, n4), then from emit_root a tree over the
//     emissive triangles alone.  Fallback
//     (non-finite boxes, or a tree deeper than the stack): the LBVH's
//     even-depth nodes, each holding its up to 4 grandchildren (a leaf child
//     stands for itself), bit 30 = emitter (ignored).
//   tri[3*F] float4    leaf slot j: (v0.xyz, bits(fid)), (e1.xyz, 0), (e2.xyz, 0) (tri_rec.hpp)
//   shade[3*F] float4  face fid: (n0.xyz, bits(mtl)), (n1.xyz, geometric unit normal .x, sign of .z in
//                      its lowest bit; NaN: none), (n2.xyz, geometric normal .y)
//   mtl[2*M] float4    (base.rgb, emission), (eta, metallic, 0, 0)
#pragma once

#include <hip/hip_runtime_api.h>
#include <stdint.h>

namespace tpt {

struct DevLight {
    int32_t type;
    float color[3];
    float intensity;
    float pos[3];
    float dir[3];
    float cos_outer;
    float inv_cos_cone_diff;
};

constexpr int kMaxLights = 16;
constexpr int kRngJumps = 16;            // base-4 digits: up to 4^16 = 2^32 pixels
constexpr int kJumpWords = 160 * 5;      // one 160x160 GF(2) matrix

struct TraceArgs {
    // scene
    const float4* inner;
    const float4* inner4;
    int32_t n4;                          // 4-wide nodes
    int32_t lds_nodes;                   // set by launch_trace: 4-wide nodes [0, lds_nodes) staged in LDS
    int32_t lds_nodes_offset;            // set by launch_trace: their byte offset in LDS
    const float4* tri;
    const float4* shade;
    const float4* mtl;
    int32_t n_faces;
    int32_t n_materials;
    int32_t n_lights;
    int32_t stack_depth;                 // LDS stack slots per lane
    const DevLight* lights;
    // env (nullable)
    const uint32_t* env;                 // RGBA8 packed, row 0 = bottom
    int32_t env_w, env_h;
    // env importance sampling (A15) over blocks of is_b x is_b texels (api.cpp build_env_is)
    int32_t is_b, is_bw, is_bh;          // block side; blocks per block row; block rows
    const float* is_cond;                //   block-row prefix sums [bh][bw]
    const float* is_row;                 //   block-row sums [bh]
    const float* is_marg;                //   marginal prefix over block rows [bh]
    float is_total;
    // guide tables of the two searches (exact lower_bound in few dependent loads):
    // is_guide_r[k] = lower_bound(is_marg, (k / kr) * is_total), k = 0..kr;
    // is_guide_c[by * (kc + 1) + k] = lower_bound(block row by of is_cond, (k / kc) * is_row[by])
    const int32_t* is_guide_r;
    const int32_t* is_guide_c;
    int32_t is_kr, is_kc;                // powers of two
    int32_t env_is;                      // TPT_FLAG_ENV_IS and a non-empty distribution
    // camera
    float c2w[16];
    float origin[3];                     // c2w * (0,0,0,1)
    float sensor_w, sensor_h;            // aspect*2tan(vfov/2), 2tan(vfov/2)
    float half_sw, half_sh;              // 0.5*sensor_w, 0.5*sensor_h
    float inv_w, inv_h;                  // 1/W, 1/H
    // frame
    int32_t width, height;
    int32_t band_rows, band_count, band_index, band_height;   // band_height: rows in this band
    const int32_t* band_list;            // nullable: local band k renders global band band_list[k] (explicit deal;
                                         //   only the last entry may be a short band); dispatched in list order
    unsigned long long* band_cost;       // nullable: per global band, the summed life of the waves that rendered
                                         //   it (s_memrealtime ticks, 100 MHz), for cost-balanced deals
    int32_t n_frames;                    // frames of the batch (grid z); frame f's state at f * planes * W*H
    int32_t max_depth;
    int32_t samples;                     // samples for this launch
    int32_t flags;
    int32_t refill;                      // leave the traversal loop below this many active lanes
    int32_t leaf_kb;                     // run the parked triangle tests once this many lanes are blocked
    int32_t boxes_finite;                // all node boxes finite: min/max slab test is exact
    int32_t any_emitter;                 // some triangle emits (else a direct probe adds nothing)
    int32_t emit_root;                   // inner4 id of the emissive-triangle tree (-1: none)
    int32_t emit_inline;                 // that tree is one node of leaves: probe pass 1 in the shading pass
    // Boxes enclosing every emissive triangle's leaf box (the emissive tree
    // root's child boxes, overlapping ones merged): (lo.xyz, 0), (hi.xyz, 0) per
    // box.  A direct probe whose line misses all of them by a margin can hit no
    // emitter and is resolved in the shading pass (trace.hip probe_misses_emitters)
    float4 emit_box[8];
    int32_t n_emit_box;                  // 0: no pre-test (no emissive tree, or non-finite boxes)
    const float4* sliver_groups;         // 2 per group: (lo.xyz, first), (hi.xyz, count) (trace.hip "Culling")
    const float4* sliver_list;           // 2 per sliver: (exact leaf box lo.xyz, position | emissive << 30), (hi.xyz, 0)
    int32_t n_sliver_groups;             // 0: no sliver triangles
    float cull_eps;                      // absolute position slack of the t-culls (trace.hip "Culling")
    int32_t graze;                       // 1: rays leaving a face within 1e-3 of its plane skip the culls (grazing())
    int32_t pair;                        // 1: pair mode (two lanes per pixel, shadow rays on the side lane)
    int32_t drained;                     // 1: the launch cannot fill the chip (latency-oriented DRAIN variants)
    int32_t quad;                        // 1: four lanes per pixel, each node visit split over them (k_trace QUAD)
    int32_t xcd_run;                     // > 0: workgroup tiles dealt to XCDs in runs of this many (k_trace)
    int32_t xcd_rot;                     // the runs' XCD rotation of this launch (its chunk of the set's spp)
    int32_t tile_pool;                   // 1: each workgroup renders two adjacent tiles, the second as a pixel
                                         //    pool its finished lanes draw from (k_trace; set by launch_trace)
    int32_t lds_pool_offset;             // set by launch_trace: byte offset of the pool counter in LDS
    int32_t lds_rec_offset;              // set by launch_trace: byte offset of the record region
    int32_t rec_lds_levels;              // set by launch_trace: path-record levels held in LDS
    int32_t stack_lds_slots;             // set by launch_trace: stack slots held in LDS (rest private)
    int32_t lds_stack_offset;            // set by launch_trace: byte offset of the stack region
    int32_t lds_mtl_offset;              // set by launch_trace: byte offset of the material table
    int32_t mtl_in_lds;                  // set by launch_trace: material table copied to LDS
    // per-pixel state (SoA over W*H pixels)
    uint32_t* rng;                       // 6 planes: v0..v4, d
    float* accum;                        // 3 planes: r, g, b (running totalRad)
    unsigned long long* counters;        // [0] trav [1] inner [2] leaf [3] shade [4] overflow [5] wide
    unsigned long long* debug_waves;     // phase-profiling builds: 8 words per wave (null: off)
};

// Path-record words per bounce (k_trace): 2 when the scene has no delta lights
// (atten; material | probe material | p-kind packed), else 5 (atten; material |
// p-kind; direct term x3).  The packed form needs material ids below 0x7fff.
__host__ __device__ inline int rec_words(int n_lights, int n_materials) {
    return (n_lights > 0 || n_materials >= 0x7ffe) ? 5 : 2;
}

struct ResolveArgs {
    const float* accum;
    float* radiance;                     // device, W*H*3 (nullable)
    uint8_t* bgra;                       // device, W*H*4 (nullable)
    int32_t width, height;
    int32_t band_rows, band_count, band_index, band_height;
    const int32_t* band_list;            // as TraceArgs
    int32_t spp;
};

// rng.hip
hipError_t launch_rng_init(const uint32_t* jumps, uint64_t seed, int32_t width, int32_t band_rows,
                           int32_t band_count, int32_t band_index, const int32_t* band_list, int32_t band_height,
                           int32_t height, uint32_t* rng, hipStream_t s);
hipError_t launch_rng_init_linear(const uint32_t* jumps, uint64_t seed, uint64_t first, uint32_t n,
                                  uint32_t* states_aos, hipStream_t s);

// build.hip
struct BuildBuffers {
    int32_t n_faces, n_vertices, n_objects, n_materials;
    const uint32_t* indices;
    const float* vertices;
    const float* normals;
    const int2* lut;
    const float* vert_trans;
    const float* normal_trans;
    const float4* mtl;
    float* wverts;
    float* wnorms;
    // temporaries
    unsigned long long* keys;
    unsigned long long* keys_sorted;
    uint32_t* fids;
    uint32_t* fids_sorted;
    float* leaf_box;                     // 6 per face (min.xyz, max.xyz) by fid
    int2* children;                      // F-1
    uint32_t* parent;                    // 2F-1
    float* node_box;                     // 6 per node (2F-1)
    uint32_t* flags;                     // F-1
    uint32_t* max_depth;                 // 3: deepest leaf, non-finite inner-box flag, 4-wide node count
    unsigned long long* bfs_keys;        // F-1: (level, id) keys of the 4-wide nodes
    unsigned long long* bfs_keys_sorted;
    uint32_t* bfs_ids;                   // F-1
    uint32_t* bfs_ids_sorted;
    uint32_t* bfs_newid;                 // F-1: binary id -> breadth-first 4-wide id
    uint32_t* emit;                      // 2F-1: subtree holds an emissive triangle
    void* sort_tmp;
    size_t sort_tmp_bytes;
    // outputs
    float4* inner;
    float4* inner4;
    float4* tri;
    float4* shade;
    void* nodes36;                       // reference layout (2F-1) * 36 B
    uint32_t out_max_depth;              // deepest leaf (root = 0), set by launch_build
    uint32_t out_boxes_finite;           // 1: every inner-node child box is finite
    uint32_t out_n4;                     // 4-wide nodes (breadth-first prefix of inner4)
};
// launch_build fails with hipErrorInvalidValue (out_max_depth >= kMaxLbvhDepth)
// when a leaf's parent chain does not reach the root within this many steps
constexpr uint32_t kMaxLbvhDepth = 4096;
hipError_t build_sort_tmp_bytes(int32_t n, size_t* bytes);
hipError_t launch_build(BuildBuffers& b, hipStream_t s);
// Culling exactness inputs (trace.hip "Culling"), per leaf position of the packed
// triangles: sliver[p] = 1 when sin of the angle at v0 between e1 and e2 is below
// 1e-3, and *coord_max (zeroed by the caller) = the bits of the largest
// |coordinate| of any vertex as a double (positive doubles order as integers).
hipError_t launch_sliver_scan(const float4* tri, int32_t n, uint8_t* sliver, unsigned long long* coord_max,
                              hipStream_t s);

// wavefront.hip: the wavefront / ray-queue variant (TPT_FLAG_WAVEFRONT).  The
// queues are split into kWfShards shards (one per XCD) of shard_cap entries.  Slots
// run pixels' sample chains; their state lives here between iterations, and the
// rays move through two ping-pong queues (2 float4 each: origin + slot, direction
// + flags) with one hit record (t, u, v, fid code) per queue position.
constexpr int kWfShards = 8;
constexpr int kWfCtlStride = 1024;                     // words between control words (4 KiB)
constexpr int kWfCtlWords = (4 * kWfShards + 1) * kWfCtlStride;
struct WfArgs {
    TraceArgs t;                         // scene, camera, frame, RNG/accumulator planes, counters
    int32_t n_slots;                     // concurrent paths (slots)
    int32_t state_words;                 // 16, or 32 with delta lights / env IS / reference order
    int32_t rec_words;                   // path-record words per bounce (2 or 5)
    int32_t ordered;                     // 0: the reference's visit order (TPT_FLAG_REF_ORDER)
    uint32_t* st0;                       // path state beside queue 0's entries: state_words per entry
    uint32_t* st1;                       // ... beside queue 1's
    float* rec;                          // n_slots * max_depth * rec_words
    float4* q_ray0;                      // 2 * kWfShards * shard_cap float4
    float4* q_ray1;                      // 2 * kWfShards * shard_cap float4
    float4* q_hit;                       // kWfShards * shard_cap float4
    uint32_t* ctl;                       // kWfCtlWords: shard sizes and fetch heads of both queues, claims
    int32_t shard_cap;                   // entries per shard: ceil(n_slots / 256 / kWfShards) * 256
    int32_t n_claims;                    // claim ids (k_trace dispatch order; those outside the band are skipped)
    int32_t refill;                      // k_wf_trace: a wave runs its pass (hits out, rays in) below this many
                                         //   traversing lanes
    int32_t chunk;                       // k_wf_trace: queue entries a wave takes per global atomic
    int32_t batch;                       // iterations enqueued between two checks of the queue size
    int32_t logic_blocks, trace_blocks;  // grid sizes (both kernels are grid-stride / persistent)
    int32_t it;                          // set per launch: iteration (queue it & 1 is consumed)
    int32_t stack_lds_slots, lds_stack_offset, lds_bytes;   // set by launch_wavefront
};
// Runs every iteration until the queues are empty (stream-ordered; the caller
// synchronises).  h_count: 2 * kWfShards words of pinned host memory; ev: 2 events.
hipError_t launch_wavefront(WfArgs w, uint32_t* h_count, hipEvent_t ev[2], int32_t* iterations, hipStream_t s);

// trace.hip
hipError_t launch_trace(const TraceArgs& a, hipStream_t s);
bool trace_quad_fits(const TraceArgs& a);   // lanes_per_pixel 4: one-lane records, the quads' stacks fit in LDS
int trace_waves_per_simd();                 // the one-lane variants' __launch_bounds__ waves per SIMD
hipError_t launch_trace_ptr(const void* a, hipStream_t s);   // a: const TraceArgs*
// lone-wave step latency probe (tpt_debug_step_latency), a: const TraceArgs*
hipError_t launch_step_latency_ptr(const void* a, uint32_t n, const float* o, const float* d, int nodes_lds,
                                   unsigned long long* out, hipStream_t s);
hipError_t launch_resolve(const ResolveArgs& a, hipStream_t s);
// KAT kernel over the trace kernel's device functions (tpt_debug_hot_kat)
hipError_t launch_hot_kat(int op, uint32_t n, const float* in, float* out, hipStream_t s);
hipError_t launch_trace_rays(const TraceArgs& a, uint32_t n, const float* o, const float* d, const int32_t* ofid,
                             int mode, int32_t* hit, float* t, float* uv, hipStream_t s);

}  // namespace tpt

// The tolerance-mode build of trace.hip (TPT_FLAG_FAST; Makefile trace_fast.hip.o):
// the same kernels in namespace tpt_fast, reached with a tpt::TraceArgs.
namespace tpt_fast {
hipError_t launch_trace_ptr(const void* a, hipStream_t s);
hipError_t launch_step_latency_ptr(const void* a, uint32_t n, const float* o, const float* d, int nodes_lds,
                                   unsigned long long* out, hipStream_t s);
}
