/*
 * tpt_oracle.h -- CPU restatement of the TinyPathTracer hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  This library is the parity checker: only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it.  The
 * product path (tinypathtracer_amd, libtpt.so) never links or calls it.
 *
 * Every function restates /root/reference behaviour with the same float
 * operation order (built with -ffp-contract=off), citing file:line.
 * Pinning: see oracle/README.md -- BVH topology hashes and mean radiances
 * from the host-compiled reference kernels, golden
 * fixtures in tests/golden/, and the L0 KAT harness oracle/_ref (built from
 * the reference's own header-only math).
 */
#ifndef TPT_ORACLE_H
#define TPT_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Material: 15 floats, the reference's layout (include/material.h:86-120). */
typedef struct {
    float base_color[3];
    float emission_factor;
    float eta;
    float metallic;
    float subsurface, specular, roughness, specular_tint, anisotropic,
          sheen, sheen_tint, clearcoat, clearcoat_gloss;
} orc_material;

/* Delta light, flattened union of include/delta_light.h:35-94. */
typedef struct {
    int32_t type;          /* 0 point, 1 directional, 2 spot (delta_light.h:7-12) */
    float color[3];
    float intensity;
    float pos[3];
    float direction[3];
    float cos_outer;
    float inv_cos_cone_diff;
} orc_light;

typedef struct {
    int32_t begin;   /* first face of the object (mesh.cuh:74-78) */
    int32_t mtl;
} orc_interval;

typedef struct {
    const uint32_t* indices;  uint32_t n_faces;      /* 3 per face, global vertex ids */
    const float* vertices;    const float* normals;  uint32_t n_vertices;  /* xyz */
    const orc_interval* lut;  uint32_t n_objects;
    const float* vert_trans;  const float* normal_trans; /* 16 floats, column-major */
    const orc_material* materials; uint32_t n_materials;
    const orc_light* lights;  uint32_t n_lights;
} orc_scene;

/* BVH node exactly as include/bvh.cuh:52-58 (36 bytes). */
typedef struct {
    uint32_t parent;
    int32_t a;   /* internal: leftChild;  leaf: fid */
    int32_t b;   /* internal: rightChild; leaf: placeHolder */
    float bmin[3];
    float bmax[3];
} orc_node;

typedef struct {
    const uint8_t* rgba;  /* w*h*4, row 0 = bottom (FreeImage order, picture.h:41-43) */
    int32_t w, h;
} orc_env;

typedef struct {
    float c2w[16];        /* column-major camera-to-world (camera.h, transform.h:16-33) */
    float vfov;           /* radians (mesh.cu:179) */
    float aspect;         /* from the glTF camera, not W/H (path_tracer.cu:503) */
} orc_camera;

typedef struct {
    int32_t width, height, spp, max_depth;
    uint64_t seed;
    /* interleaved row bands: rows y with (y / band_rows) % band_count == band_index */
    int32_t band_rows, band_count, band_index;
    int32_t trig_mode;    /* 0: libm float functions (as the survey harness);
                             1: parity trig, bit-identical to the HIP kernel */
    int32_t threads;      /* OpenMP threads, 0 = default */
    int32_t env_is;       /* 1: env next-event estimation with importance sampling (the
                             build's opt-in A15 re-derivation, TPT_FLAG_ENV_IS) */
} orc_params;

typedef struct {
    uint64_t traversals, internal_visits, leaf_tests, shade_hits, pixels;
    double init_ms, trace_ms;
} orc_counters;

/* Env importance sampling (the build's A15 re-derivation): n samples for
 * incident-side normal nf, stream (seed, 0); dirs/k_le are n*3 floats. */
int orc_env_is_samples(const uint8_t* rgba, int w, int h, const float nf[3], uint64_t seed, int n,
                       float* dirs, float* k_le);

/* cuRAND XORWOW restatement (curand_init / curand / curand_uniform). */
void orc_xorwow_init(uint64_t seed, uint64_t subsequence, uint32_t state[6]);
uint32_t orc_xorwow_next(uint32_t state[6]);
float orc_uniform(uint32_t state[6]);
/* 32 matrices A^(2^67 * 4^k), 160 rows x 5 words each (row = image of input bit). */
const uint32_t* orc_xorwow_jump_matrices(void);

/* path_tracer.cu:239-263 -- world-space vertices / normals. */
void orc_transform(const orc_scene* s, float* wverts, float* wnorms);
/* bvh.cu:304-331 -- LBVH over world vertices; nodes[2F-1], keys[F] (sorted). */
int orc_build_bvh(uint32_t n_faces, const float* wverts, const uint32_t* indices,
                  orc_node* nodes, int64_t* keys);
/* Morton helpers (bvh.cu:14-62) for KATs. */
int64_t orc_float_to_21int(float x);
int64_t orc_morton(float x, float y, float z);
/* 0 (default): shift >= 32 -> 0 (PTX); 1: shift count masked mod 32 (x86). */
void orc_set_x86_shift(int on);

/* Full frame: transform + BVH + setupRandSeed + trace + copyToFB
 * (path_tracer.cu:491-554).  radiance: W*H*3 floats (color/spp, row 0 = bottom),
 * bgra: W*H*4 (row 0 = top, copyToFB), either may be NULL. Rows outside the
 * band are left untouched.  Returns 0 on success. */
int orc_render(const orc_scene* s, const orc_env* env, const orc_camera* cam,
               const orc_params* p, float* radiance, uint8_t* bgra,
               orc_counters* counters);

/* Trace one ray against a built BVH (path_tracer.cu:61-107). */
int orc_trace_ray(const orc_node* nodes, uint32_t n_faces, const float* wverts,
                  const uint32_t* indices, const float o[3], const float d[3],
                  float* t_out, float uv_out[2]);

/* KAT entry points (tests/test_oracle_pinned.py vs tests/golden/ref_hot_kat.json):
 * rayHitBBox (geometry_queries.h:18-46); rayHitTriangle (:65-86), out = dist, u, v
 * (written only on a hit); DeltaLight::sample (delta_light.h:105-130);
 * CalcDistAttenuation (:25-33), rgb in place; Spectrum::toUChar (material.h:74-81);
 * Material() (material.h:88-103). */
int orc_kat_box_hit(const float o[3], const float d[3], const float bmin[3], const float bmax[3]);
int orc_kat_tri(const float o[3], const float d[3], const float v0[3], const float v1[3], const float v2[3],
                float out[3]);
void orc_kat_light(const orc_light* L, const float p[3], float dir[3], float rad[3]);
void orc_kat_dist_atten(float dist, float rgb[3]);
void orc_kat_to_uchar(const float rgb[3], uint8_t out[3]);
void orc_kat_default_material(orc_material* m);

float orc_parity_sinf(float x);
float orc_parity_cosf(float x);
/* trig_mode 1 sin/cos of phi in [0, 2pi] (identical to the HIP kernel) */
void orc_parity_sincos(float x, float* s, float* c);

#ifdef __cplusplus
}
#endif
#endif
