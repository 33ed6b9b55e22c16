/*
 * tpt.h -- C-ABI of the MI355X-native TinyPathTracer hot path (libtpt.so).
 *
 * Drop-in boundary for the reference's render job
 *   PathTracer::doTrace(DeviceScene&, Camera&, unsigned char* fb, int spp)
 *   (include/path_tracer.h:34, src/path_tracer.cu:491-554)
 * and for the device ABI of its `trace` kernel
 *   (src/path_tracer.cu:296-299).  Plain pointers and sizes only; no
 * exceptions cross this boundary (errors: tpt_status + tpt_last_error()).
 *
 * Handles own device memory; caller buffers are borrowed.  One tpt_scene per
 * HIP device; calls on different scenes may run concurrently from different
 * host threads, calls on one scene must be serialised by the caller.
 */
#ifndef TPT_H
#define TPT_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define TPT_VERSION_MAJOR 0
#define TPT_VERSION_MINOR 1

typedef enum {
    TPT_OK = 0,
    TPT_ERR_INVALID_ARG = 1,
    TPT_ERR_HIP = 2,
    TPT_ERR_OOM = 3,
    TPT_ERR_IO = 4,
    TPT_ERR_PARSE = 5,
    TPT_ERR_NO_DEVICE = 6
} tpt_status;

/* Material, 60 bytes: the reference's Material (include/material.h:86-120). */
typedef struct {
    float base_color[3];
    float emission_factor;
    float eta;
    float metallic;
    float subsurface, specular, roughness, specular_tint, anisotropic,
          sheen, sheen_tint, clearcoat, clearcoat_gloss;
} tpt_material;

/* DeltaLight flattened (include/delta_light.h:35-130); type 0 point,
 * 1 directional, 2 spot.  Intensities already in the reference's units
 * (point/spot lumens x 1/683, mesh.cu:276,290). */
typedef struct {
    int32_t type;
    float color[3];
    float intensity;
    float pos[3];
    float direction[3];
    float cos_outer;
    float inv_cos_cone_diff;
} tpt_light;

/* MtlInterval (include/mesh.cuh:74-78): object o owns faces [begin, next begin). */
typedef struct {
    int32_t begin;
    int32_t mtl;
} tpt_interval;

/* The content of DeviceScene (include/mesh.cuh:80-96).  Every array pointer
 * may be host memory or device memory (detected per pointer, as tpt_render
 * does for its outputs), so the reference's doTrace can pass its
 * thrust::device_vector buffers as they are -- the `trace` kernel's own
 * arguments (path_tracer.cu:297-299): raw_pointer_cast(d_scene.indices.data())
 * etc.  Vec3 arrays are 3 floats per vertex, Mat4 16 floats column-major,
 * Material is tpt_material byte for byte, MtlInterval is tpt_interval.
 * The scene keeps its own copy: the caller's buffers are only read during
 * tpt_scene_create. */
typedef struct {
    const uint32_t* indices;      uint32_t n_faces;      /* 3*n_faces global vertex ids */
    const float* vertices;        const float* normals;  uint32_t n_vertices; /* xyz, object space */
    const tpt_interval* lut;      uint32_t n_objects;
    const float* vert_trans;      const float* normal_trans; /* 16 floats/object, column-major */
    const tpt_material* materials; uint32_t n_materials;   /* empty -> Material() default */
    const tpt_light* lights;      uint32_t n_lights;
    uint32_t flags;               /* TPT_DESC_*; 0 for a zero-initialised desc */
} tpt_scene_desc;

/* desc->lights points at the reference's own DeltaLight array (delta_light.h:
 * 96-130: DeltaLightType, then the PointLight / DirectionalLight / SpotLight
 * union; 52 B, the offsets of tpt_light except that a directional light keeps
 * its direction where tpt_light has pos).  The library repacks it; the
 * union's unused bytes are never read. */
#define TPT_DESC_DELTALIGHT_LAYOUT 0x1

/* Camera (include/camera.h): c2w = m_transform->localToWorld(). */
typedef struct {
    float c2w[16];      /* column-major */
    float vfov;         /* radians */
    float aspect;       /* camera aspect ratio (the reference ignores W/H here) */
    float znear;
} tpt_camera;

typedef struct {
    int32_t width, height;        /* full frame */
    int32_t spp;                  /* samples per pixel (reference: 64 per frame) */
    int32_t max_depth;            /* DEPTH_TRACE (reference: 8), 1..64 */
    uint64_t seed;                /* curand_init seed (reference: time()) */
    /* Interleaved row bands for multi-GPU sharding: this call renders rows y
     * with (y / band_rows) % band_count == band_index.  band_count 1 = all.
     * band_list (below) replaces this deal with an explicit one. */
    int32_t band_rows, band_count, band_index;
    int32_t spp_per_launch;       /* 0 = auto; chunks the spp loop over launches */
    int32_t flags;                /* TPT_FLAG_* */
    int32_t refill;               /* 0 = auto: lanes (of 64) below which a wave stops to shade */
    /* Launch pipeline.  pipe_sets: 0 = auto (3 interleaved band sets
     * from 1024 spp, else 1), 1 = one stream, 2..4 = that many sets (from 256 spp);
     * pipe_chunks: spp chunks per set, 0 = auto (8).  Every schedule is bit-identical
     * to one launch.  The sets run on library-owned streams created at the device's
     * greatest stream priority: HIP gives each priority its own pool of hardware queues
     * (GPU_MAX_HW_QUEUES, 4 by default), and two sets whose streams share a queue run
     * one after the other (-25 % measured).  A host application that issues its own
     * greatest-priority work on the device while tpt_render runs shares those queues. */
    int32_t pipe_sets, pipe_chunks;
    /* Lanes per pixel: 0 = auto (pair mode with delta lights or env IS, else 4 on launches
     * of at most tpt_stats.resident_lanes pixels -- 327,680 on MI355X -- else 1), 1, or
     * 2 = pair mode (scenes with delta lights): a side lane per pixel traces each bounce's
     * shadow rays while the path lane goes on, so a sample's serial chain pays one traversal per bounce; 4 = four
     * lanes run each pixel's path together and split every 4-wide node visit (child k on
     * lane k, leaf children tested at once), a shorter serial chain at a quarter of the
     * pixels per wave (scenes without delta lights, no env IS, ordered traversal; DESIGN.md
     * section 6).  Bit-identical in every mode. */
    int32_t lanes_per_pixel;
    /* 0 = auto: a wave runs its parked triangle tests once this many lanes are blocked on
     * a parked leaf (speculative leaf postponement): 2 in pair mode,
     * else 4.  Bit-identical for any value. */
    int32_t leaf_batch;
    /* TPT_FLAG_WAVEFRONT only: concurrent paths (slots; 0 = every pixel of the call) and the
     * traversing lanes below which a trace wave runs its pass -- finished walks out, the next
     * queued rays in (0 = auto, 40).  Bit-identical for any values. */
    int32_t wf_slots, wf_refill;
    /* Explicit band deal (nullable; a zero-initialised params keeps the interleaved one): this
     * call renders global bands band_list[0 .. band_list_len), band b = rows [b * band_rows,
     * (b + 1) * band_rows) clipped to the frame; distinct ids, a short last band (height not a
     * multiple of band_rows) last; workgroups are dispatched in list order.  band_count and
     * band_index are then ignored.  Any deal is bit-identical to one GPU: the RNG subsequence
     * is the global pixel index (path_tracer.cu:39,320).  Host memory, read during the call. */
    int32_t band_list_len;
    const int32_t* band_list;
    /* Nullable, host memory, ceil(height / band_rows) floats: for each band this call renders,
     * band_cost[b] = the summed life in microseconds of the trace waves that rendered it (megakernel
     * only; 0 under TPT_FLAG_WAVEFRONT); other entries are left as they are.  A deal of the next
     * frame's bands balanced by these costs (tinypathtracer_amd.shard.cost_deal) evens out ranks
     * whose interleaved shares hold the heavy rows. */
    float* band_cost;
} tpt_params;

#define TPT_FLAG_NO_COUNTERS   0x1   /* skip visit counters (traversals still counted) */
#define TPT_FLAG_REF_ORDER     0x2   /* reference right-first traversal, no culling */
#define TPT_FLAG_ENV_IS        0x8   /* opt-in env next-event estimation with importance sampling (A15
                                        re-derived; the reference's trace never calls it, so the image
                                        differs from a reference render) */
#define TPT_FLAG_APPROX_CULL   0x10  /* the ordered traversal's culls without the exactness guards (no
                                        position slack, no sliver re-test, grazing rays culled too;
                                        DESIGN.md section 4): a few
                                        percent faster, and rays whose Moller-Trumbore t is rounding noise
                                        (sliver triangles, grazing edge hits) may then find another hit
                                        than the reference (5 of ~60 G rays over the BASELINE frames) */
#define TPT_FLAG_WAVEFRONT     0x20  /* the wavefront / ray-queue variant (DESIGN.md section 5 "N1"): a logic
                                        kernel and a persistent trace kernel alternate per ray of every
                                        live path, path state in device memory between them; bit-identical
                                        to the megakernel.  lanes_per_pixel, pipe_*, spp_per_launch are
                                        not used */
#define TPT_FLAG_FAST          0x40  /* tolerance mode: the trace kernel built with FMA
                                        contraction, FMA slab tests and the hardware's approximate reciprocal,
                                        sqrt, sin and cos, without the culling guards (implies
                                        TPT_FLAG_APPROX_CULL).  Not bit for bit.  Where the images meet SURVEY
                                        8(d)'s tolerance (mean |d| <= 1e-3, p99 <= 1e-2, >= 99.5 % of pixels
                                        within one 8-bit step): every BASELINE configuration at full
                                        resolution and 1-2 spp, and the full-spp bands of C2 (1024 spp), C3
                                        and C3 + env IS (4096) and C4 (8192).  Where they do not: C5's
                                        full-spp band (2048 spp) meets the mean only -- p99 0.0128 and 96.0 %
                                        within one step (measured with and without the culling guards alike:
                                        the tail is the rounding, not the culls).  Not with
                                        TPT_FLAG_WAVEFRONT */
#define TPT_FLAG_ACCUMULATE    0x4   /* progressive: continue the previous call's per-pixel streams and
                                        sums (same frame size, bands and seed); the output is the mean over
                                        all accumulated samples, bit-identical to one call with their total */

typedef struct {
    uint64_t traversals;          /* traverseBVH calls: primary+extension+probe+shadow */
    uint64_t internal_visits;     /* binary internal nodes popped (reference-order / non-finite rays) */
    uint64_t leaf_tests;          /* leaves popped (triangle tests) */
    uint64_t shade_hits;          /* extension-ray hits shaded */
    uint64_t pixels;              /* pixels rendered by this call */
    uint64_t samples;             /* pixels * spp */
    double rng_init_ms;           /* setupRandSeed equivalent */
    double trace_ms;              /* trace phase, first launch start to last launch end (HIP events) */
    double resolve_ms;            /* copyToFB equivalent */
    double total_ms;              /* whole tpt_render, host wall */
    int32_t trace_launches;
    int32_t pad;
    uint64_t wide_visits;         /* 4-wide internal nodes popped (ordered traversal) */
    uint64_t accumulated_spp;     /* samples per pixel in the output (> spp with TPT_FLAG_ACCUMULATE) */
    double trace_kernel_ms;       /* sum of the trace launches' own durations (HIP events per launch);
                                     > trace_ms when the launch pipeline overlaps them */
    uint64_t local_rays;          /* of `traversals`, the direct probes resolved in the shading pass without
                                     a BVH traversal (no emissive triangle, or a miss of the <= 4-emitter
                                     inline test); traversals - local_rays = BVH traversals run */
    double tree_wait_ms;          /* host wall time this call waited for a tpt_scene_build_async's host
                                     traversal-tree build, after enqueueing the RNG initialisation */
    uint64_t resident_lanes;      /* the device's resident trace lanes (hipDeviceProp_t CUs x 4 SIMDs x
                                     the one-lane variant's waves per SIMD x 64; MI355X 327,680): launches of
                                     at most this many pixels run four lanes per pixel (lanes_per_pixel 0),
                                     below twice it the latency-oriented (drained) variants */
    int32_t lanes_per_pixel;      /* the lane mode the trace launches ran: 1, 2 (pair) or 4 */
    int32_t drained;              /* 1: the drained-launch rule applied (refill, leaf batch, DRAIN variants) */
} tpt_stats;

typedef struct tpt_scene tpt_scene;
typedef struct tpt_env tpt_env;

/* Library identity and errors. */
const char* tpt_version(void);
const char* tpt_last_error(void);
int tpt_device_count(void);

/* Upload a scene to `device` (hipSetDevice index).  Replaces
 * Scene::copySceneToDevice (mesh.cu:309-397). */
tpt_status tpt_scene_create(const tpt_scene_desc* desc, int device, tpt_scene** out);
/* World transform + LBVH build on the device (path_tracer.cu:536-542,
 * bvh.cu:304-331) and the packed traversal layout. */
tpt_status tpt_scene_build(tpt_scene* scene);
/* tpt_scene_build whose host half -- the SAH traversal trees over the LBVH's
 * leaf boxes -- continues on a host thread after the call returns (the device
 * LBVH build and its read-back are done).  The next call that traces the scene
 * waits for it: tpt_render / tpt_render_frames after enqueueing the per-pixel
 * RNG initialisation (setupRandSeed, path_tracer.cu:513), so the two overlap;
 * tpt_debug_trace_rays first.  A failure of the host half is reported by that
 * call.  tpt_scene_build / _async and tpt_scene_destroy supersede a pending
 * one.  The scene is the same as tpt_scene_build's. */
tpt_status tpt_scene_build_async(tpt_scene* scene);
/* Host threads of the traversal-tree build inside tpt_scene_build (the SAH
 * 4-wide tree): < 0 = auto (the cores this process may
 * use: its affinity mask capped by the cgroup CPU quota), 0 or 1 = serial.
 * Every setting builds the same tree.  Processes sharing a host (one per GPU)
 * pass their share of the cores. */
tpt_status tpt_scene_set_build_threads(tpt_scene* scene, int32_t threads);
void tpt_scene_destroy(tpt_scene* scene);

/* Equirect environment, RGBA8, row 0 = bottom (FreeImage order), already in
 * RGB channel order (texture.cu:33-47 swizzle applied by the caller). */
tpt_status tpt_env_create(const uint8_t* rgba, int32_t width, int32_t height, int device, tpt_env** out);
void tpt_env_destroy(tpt_env* env);

/* Env map from an image file: EnvLight(file) (include/env_light.cuh:8-18,
 * src/texture.cu:64-171, include/picture.h:19-45).  Decodes JPEG (baseline and
 * progressive Huffman, libjpeg's default islow IDCT / fancy upsampling / YCbCr
 * tables) or binary PPM natively into the texel layout tpt_env_create takes
 * (RGBA8, row 0 = bottom).  Errors: TPT_ERR_IO (cannot open), TPT_ERR_PARSE
 * (unsupported or corrupt image, e.g. grayscale, which the reference's
 * Texture also rejects). */
tpt_status tpt_env_load(const char* path, int device, tpt_env** out);
/* The decoder alone: *rgba is allocated by the library (free with
 * tpt_image_free), width*height*4 bytes, row 0 = bottom. */
tpt_status tpt_image_load(const char* path, uint8_t** rgba, int32_t* width, int32_t* height);
void tpt_image_free(uint8_t* rgba);
/* One frame == doTrace: setupRandSeed, trace (spp), copyToFB.
 *   radiance_out: nullable, width*height*3 floats = color/spp, row 0 = bottom;
 *                 host or device pointer (detected).  Only band rows written.
 *   bgra_out:     nullable, width*height*4 bytes, row 0 = top, B,G,R written,
 *                 alpha untouched (copyToFB, path_tracer.cu:451-471).
 *   env:          nullable -> black on miss.
 * Device outputs are written on the library's own stream and are complete when
 * tpt_render returns; no other stream may have work pending that reads or
 * writes them when the call starts (the caller synchronises its stream first;
 * the Python host does this for torch tensors). */
tpt_status tpt_render(tpt_scene* scene, const tpt_env* env, const tpt_camera* camera,
                      const tpt_params* params, float* radiance_out, uint8_t* bgra_out,
                      tpt_stats* stats);

/* A batch of independent frames in one trace launch: frame f is a doTrace
 * with seed seeds[f] (the reference re-seeds every frame from time(),
 * path_tracer.cu:493-494,513); all frames share params (size, spp, bands,
 * flags) and params->seed is ignored.  Frame f is bit-identical to
 * tpt_render with seed seeds[f].  Used to keep every GPU of a node busy on
 * its share of several frames at once (bench.py weak scaling).
 *   radiance_outs / bgra_outs: nullable arrays of n_frames nullable pointers,
 *   each as in tpt_render.  stats: summed over the batch. */
tpt_status tpt_render_frames(tpt_scene* scene, const tpt_env* env, const tpt_camera* camera,
                             const tpt_params* params, int32_t n_frames, const uint64_t* seeds,
                             float* const* radiance_outs, uint8_t* const* bgra_outs, tpt_stats* stats);
/* Introspection for tests: copy back the built BVH in the reference node
 * layout (bvh.cuh:52-58, 36 B/node, 2F-1 nodes) and the sorted Morton keys. */
tpt_status tpt_scene_read_bvh(tpt_scene* scene, void* nodes36, int64_t* keys);
/* World-space vertices / normals after tpt_scene_build (n_vertices*3 each). */
tpt_status tpt_scene_read_world(tpt_scene* scene, float* wverts, float* wnorms);
/* Per-pixel RNG states after setupRandSeed for the first n pixels: 6 words
 * each {v0..v4, d}. */
tpt_status tpt_debug_rng_init(int device, uint64_t seed, uint64_t first_pixel, uint32_t n, uint32_t* states);
/* Trace n rays (origins/dirs xyz) against the built BVH: hit fid (-1 miss), t, u, v.
 * origin_fid: nullable; per ray the face it leaves (-1: none), for the render's
 * grazing test (a ray within 1e-3 of that face's plane takes the uncull'd path).
 * mode 0: closest hit in the reference's visit order (traverseBVH, path_tracer.cu:61-107);
 * 1: closest hit through the render's traversal (nearer-first, culled, 4-wide);
 * 2: any hit (shadow rays); 3: the render's two-pass direct probe -- hit = the
 * closest hit if it is an emitter, -2 if a non-emitter is closer, -1 if no emitter is hit. */
tpt_status tpt_debug_trace_rays(tpt_scene* scene, uint32_t n, const float* origins, const float* dirs,
                                const int32_t* origin_fid, int32_t mode, int32_t* hit, float* t, float* uv);
/* Known-answer evaluation of the trace kernel's own device functions, one case
 * per lane (tests pin them to the reference's headers):
 *   op 0 rayHitBBox   in 12/case (o3 d3 min3 max3)          out 2 (box_hit, min/max verdict)
 *   op 1 rayHitTriangle in 15 (o3 d3 v0_3 v1_3 v2_3)         out 4 (hit, dist, u, v)
 *   op 2 DeltaLight::sample in 16 (type color3 intensity pos3 dir3 cos_outer
 *        inv_cos_cone_diff p3)                              out 6 (dir3, radiance3)
 *   op 3 Spectrum::toUChar in 3                             out 3 (bytes as floats) */
tpt_status tpt_debug_hot_kat(int device, int32_t op, uint32_t n, const float* in, float* out);
/* Diagnostics: the per-step latency of ONE 64-lane wave walking n <= 64 closest-hit rays
 * with the render's traversal ("The drained chain"); mode 0 reads the
 * 4-wide nodes from global memory as the render does, 1 from a copy of the whole main tree
 * in LDS, 2 four lanes per ray (n <= 16: lane k of a ray's quad tests child k of each node,
 * its leaf children at once; node visits in out's first word); flags TPT_FLAG_FAST: the
 * tolerance-mode build.  out: 4 words per lane (64 lanes; per ray in mode 2): visits + leaf
 * tests of the lane, loop iterations of the wave, shader cycles of the wave's walk
 * (s_memtime), hit fid. */
tpt_status tpt_debug_step_latency(tpt_scene* scene, uint32_t n, const float* origins, const float* dirs,
                                  int32_t mode, int32_t flags, uint64_t* out);
/* Host-only: the SAH 4-wide traversal tree tpt_scene_build uploads, over n >= 2
 * leaf boxes (6 floats each, by LBVH sorted position) and emitter flags.  Writes
 * at most `cap` nodes of 32 floats (inner4 layout, device_api.hpp) and the
 * most stack entries its ordered walk can hold; returns the node count (> cap:
 * not written), or -1.  threads as in tpt_scene_set_build_threads. */
int32_t tpt_wide_tree_build(int32_t n, const float* leaf_box, const uint32_t* leaf_emit, float* nodes,
                            int32_t cap, int32_t* stack_need, int32_t threads);

/* ---- host-side glTF loader (mesh.cu:80-397 semantics) -------------------- */
typedef struct tpt_gltf tpt_gltf;
tpt_status tpt_gltf_load(const char* path, tpt_gltf** out);
/* Borrowed views valid until tpt_gltf_free. */
tpt_status tpt_gltf_desc(const tpt_gltf* g, tpt_scene_desc* desc, tpt_camera* camera);
/* 1 if a mesh had no material (reference reads out of bounds; we use Material()). */
int tpt_gltf_missing_material(const tpt_gltf* g);
void tpt_gltf_free(tpt_gltf* g);

#ifdef __cplusplus
}
#endif
#endif /* TPT_H */
