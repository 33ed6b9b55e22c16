// api.cpp -- the C-ABI (include/tpt.h) over the HIP kernels.
//
// Replaces the reference's per-frame orchestration PathTracer::doTrace
// (src/path_tracer.cu:491-554) and Scene::copySceneToDevice (src/mesh.cu:309-397).
// No exceptions cross the ABI: every entry point returns tpt_status and records
// a thread-local message for tpt_last_error().
#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <memory>
#include <new>
#include <string>
#include <system_error>
#include <thread>
#include <vector>

#include "../common/device_api.hpp"
#include "../common/ptrig.hpp"
#include "../common/rng.hpp"
#include "../common/tpt_math.hpp"
#include "../common/tri_rec.hpp"
#include "tpt.h"
#include "tpt_internal.hpp"

namespace {

thread_local std::string g_last_error;
constexpr float kInfF = __builtin_huge_valf();

tpt_status fail(tpt_status st, const std::string& msg) {
    g_last_error = msg;
    return st;
}

#define HIP_OR_FAIL(expr)                                                                             \
    do {                                                                                              \
        hipError_t e_ = (expr);                                                                       \
        if (e_ != hipSuccess)                                                                         \
            return fail(e_ == hipErrorOutOfMemory ? TPT_ERR_OOM : TPT_ERR_HIP,                         \
                        std::string(#expr) + ": " + hipGetErrorString(e_));                          \
    } while (0)

template <typename T>
struct DevBuf {
    T* p = nullptr;
    size_t n = 0;
    DevBuf() = default;
    DevBuf(const DevBuf&) = delete;
    DevBuf& operator=(const DevBuf&) = delete;
    ~DevBuf() { release(); }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        n = 0;
    }
    hipError_t alloc(size_t count) {
        if (count == n && p) return hipSuccess;
        release();
        if (count == 0) return hipSuccess;
        hipError_t e = hipMalloc((void**)&p, count * sizeof(T));
        if (e == hipSuccess) n = count;
        return e;
    }
    hipError_t upload(const T* src, size_t count, hipStream_t s) {
        hipError_t e = alloc(count);
        if (e != hipSuccess || count == 0) return e;
        return hipMemcpyAsync(p, src, count * sizeof(T), hipMemcpyHostToDevice, s);
    }
};

// Page-locked host memory (hipHostMalloc), grown on demand: the per-frame
// read-back of the leaf boxes runs at copy-engine speed instead of through a
// pageable bounce buffer.
template <class T>
struct HostPinned {
    T* p = nullptr;
    size_t n = 0;
    HostPinned() = default;
    HostPinned(const HostPinned&) = delete;
    HostPinned& operator=(const HostPinned&) = delete;
    ~HostPinned() {
        if (p) (void)hipHostFree(p);
    }
    hipError_t alloc(size_t count) {
        if (count <= n && p) return hipSuccess;
        if (p) (void)hipHostFree(p);
        p = nullptr;
        n = 0;
        hipError_t e = hipHostMalloc((void**)&p, std::max<size_t>(count, 1) * sizeof(T), hipHostMallocDefault);
        if (e == hipSuccess) n = count;
        return e;
    }
};

struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int dev) {
        (void)hipGetDevice(&prev);
        if (prev != dev) (void)hipSetDevice(dev);
    }
    ~DeviceGuard() {
        int cur = -1;
        (void)hipGetDevice(&cur);
        if (prev >= 0 && cur != prev) (void)hipSetDevice(prev);
    }
};

// *owner (optional): the device that owns a device-memory pointer (-1 for host
// or managed memory, which every device can address).
bool is_device_ptr(const void* p, int* owner = nullptr) {
    if (owner) *owner = -1;
    if (!p) return false;
    hipPointerAttribute_t attr;
    if (hipPointerGetAttributes(&attr, p) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    const bool dev = attr.type == hipMemoryTypeDevice || attr.type == hipMemoryTypeManaged;
    if (attr.type == hipMemoryTypeDevice && owner) *owner = attr.device;
    return dev;
}

// A desc array in device memory (the reference's DeviceScene buffers) read back
// to the host, or the host array itself.  Returns the host view (null on a
// failed copy, with *err set).
template <typename T>
const T* host_view(const T* p, size_t n, std::vector<T>& tmp, hipError_t* err) {
    if (!p || n == 0 || !is_device_ptr(p)) return p;
    tmp.resize(n);
    const hipError_t e = hipMemcpy(tmp.data(), p, n * sizeof(T), hipMemcpyDeviceToHost);
    if (e != hipSuccess) {
        *err = e;
        return nullptr;
    }
    return tmp.data();
}

std::vector<uint32_t>& host_jumps() {
    static std::vector<uint32_t> j;
    if (j.empty()) {
        j.resize((size_t)tpt::kRngJumps * tpt::kJumpWords);
        tpt::xorwow_jump_matrices(tpt::kRngJumps, j.data());
    }
    return j;
}

constexpr int kMaxPipe = 4;         // overlapped launch sets per frame (GPU_MAX_HW_QUEUES is 4)
constexpr int kPipeMinChunk = 128;  // spp per pipelined launch, at least
#ifndef TPT_XCD_ROT
#define TPT_XCD_ROT 1   // XCD runs rotate by one per chunk of a set (0: every chunk alike; A/B builds)
#endif

int band_height_of(int height, int band_rows, int band_count, int band_index) {
    int n = 0;
    for (int y = 0; y < height; ++y)
        if ((y / band_rows) % band_count == band_index) ++n;
    return n;
}

}  // namespace

struct tpt_env {
    int device = 0;
    int w = 0, h = 0;
    DevBuf<uint32_t> texels;
    // importance-sampling tables (A15, TPT_FLAG_ENV_IS) over blocks of B x B
    // texels: block-row prefix sums, block-row sums, marginal prefix over block
    // rows; total <= 0 disables
    DevBuf<float> is_cond, is_row, is_marg;
    float is_total = 0.0f;
    int32_t is_b = 1, is_bw = 0, is_bh = 0;   // block side, blocks per row, block rows
    DevBuf<int32_t> is_guide_r, is_guide_c;   // guide tables of the two CDF searches (trace.hip lower_bound_guided)
    int32_t is_kr = 1, is_kc = 1;
};

namespace {

// A15 re-derivation (env_light.cu:10-54 intends a 2-D piecewise-constant
// distribution; its weight uses theta for sin(theta), its normalisation races
// across blocks and its row orientation is the reverse of Vec2UV).  Here the
// distribution is piecewise constant over blocks of B x B texels (B = 1 for
// maps up to 2^17 texels; doubled until the block grid has at most 2^17 cells,
// so the tables stay L2-resident: 2048 x 1024 -> B = 4, 512 x 256 blocks,
// 0.5 MB): a block's weight is the sum over its texels of luma * sin(theta at
// the texel row's centre), rows iy = 0 (bottom) .. h-1 as the lookup reads them
// (v = 1 - acos(y)/pi), texel rows then columns, then sequential float prefix
// sums per block row and over block rows -- the oracle (env_is_build) builds
// the same tables with the same operations.  A sample picks a block by the two
// CDFs and a point uniformly inside it (trace.hip env_is_sample).
int env_is_block(int w, int h) {
    int b = 1;
    while ((long long)((w + b - 1) / b) * (long long)((h + b - 1) / b) > (1ll << 17)) b *= 2;
    return b;
}
void build_env_is(const uint8_t* rgba, int w, int h, int b, std::vector<float>& cond, std::vector<float>& row,
                  std::vector<float>& marg, float& total) {
    const int bw = (w + b - 1) / b, bh = (h + b - 1) / b;
    cond.resize((size_t)bw * bh);
    row.resize(bh);
    marg.resize(bh);
    std::vector<float> sw(h);
    for (int iy = 0; iy < h; ++iy) {
        const float theta = tpt::kPi * (1.0f - ((float)iy + 0.5f) / (float)h);
        float cw;
        tpt::fsincos_2pi(theta, sw[iy], cw);
    }
    float acc_rows = 0.0f;
    for (int by = 0; by < bh; ++by) {
        float acc = 0.0f;
        for (int bx = 0; bx < bw; ++bx) {
            float wb = 0.0f;
            for (int iy = by * b; iy < std::min(by * b + b, h); ++iy)
                for (int ix = bx * b; ix < std::min(bx * b + b, w); ++ix) {
                    const uint8_t* px = rgba + 4 * ((size_t)iy * w + ix);
                    const float luma = (0.2126f * (float)px[0] + 0.7152f * (float)px[1]) + 0.0722f * (float)px[2];
                    wb = wb + luma * sw[iy];
                }
            acc = acc + wb;
            cond[(size_t)by * bw + bx] = acc;
        }
        row[by] = acc;
        acc_rows = acc_rows + acc;
        marg[by] = acc_rows;
    }
    total = acc_rows;
}

// Guide table of a nondecreasing prefix array a[0, n) with last entry `total`:
// g[k] = lower_bound(a, fl((k / K) * total)) for k = 0..K (trace.hip
// lower_bound_guided).  The thresholds are computed in float exactly as the
// kernel's t = x * total is, so the guided search returns the plain search's index.
void build_guide(const float* a, int n, float total, int K, int32_t* g) {
    const float inv = 1.0f / (float)K;   // exact: K is a power of two
    int i = 0;
    for (int k = 0; k <= K; ++k) {
        const float thr = ((float)k * inv) * total;
        while (i < n - 1 && a[i] < thr) ++i;
        g[k] = i;
    }
}

int pow2_at_least(int n) {
    int k = 1;
    while (k < n && k < (1 << 20)) k <<= 1;
    return k;
}

}  // namespace

namespace {
// TPT_BUILD_TIMING=1: per-phase wall times of tpt_scene_build on stderr
struct PhaseClock {
    bool on;
    std::chrono::steady_clock::time_point t;
    explicit PhaseClock(bool on_) : on(on_), t(std::chrono::steady_clock::now()) {}
    void mark(const char* what) {
        if (!on) return;
        const auto now = std::chrono::steady_clock::now();
        std::fprintf(stderr, "tpt_scene_build %-10s %8.3f ms\n", what,
                     std::chrono::duration<double, std::milli>(now - t).count());
        t = now;
    }
};

// The host half of a scene build: the SAH traversal trees over the LBVH's leaf
// boxes (wide_bvh.cpp).  Pure host work -- no HIP call, no access to the scene
// but its read-back staging -- so tpt_scene_build_async runs it on a thread of
// its own while the caller goes on (tpt_render enqueues the RNG
// initialisation, then waits for it: finish_pending).  One per scene, kept
// between builds with its work arrays and output buffers (no per-frame
// allocation to fault in).
struct HostTrees {
    size_t n = 0;
    const float* lbox = nullptr;      // 6 per leaf position (not owned: the scene's staging)
    const uint32_t* lemit = nullptr;  // per leaf position
    tpt::WideParams prm;
    int32_t lbvh_n4 = 0;      // the LBVH even-depth view's node count (inner4 when no SAH tree)
    bool timing = false;
    // results
    tpt::HostFloats w4, e4;
    int n4 = -1, need = 0, ne4 = -1, eneed = 0;
    tpt_status st = TPT_OK;
    std::string msg;
    tpt::WideWorkspace ws;
    std::thread th;
    ~HostTrees() { join(); }
    void join() {
        if (th.joinable()) th.join();
    }
    void reset_results() {
        n4 = -1;
        need = 0;
        ne4 = -1;
        eneed = 0;
        st = TPT_OK;
        msg.clear();
        prm.ws = &ws;
    }
    bool main_ok() const { return n4 > 0 && (size_t)n4 <= n - 1 && need <= 150; }
    int32_t base() const { return main_ok() ? n4 : lbvh_n4; }   // the emitter tree's first id
    bool emit_ok() const { return ne4 > 0 && (size_t)(base() + ne4) <= n - 1 && eneed <= 150; }
};

void build_host_trees(HostTrees& j) {
    PhaseClock clk(j.timing);
    const size_t n = j.n;
    const int leaf_base = (int)n - 1;
#ifdef TPT_WIDE_TREE_LBVH
    const bool sah = false;   // A/B builds: keep the LBVH's even-depth view
#else
    const bool sah = true;
#endif
    try {
        if (sah) {
            // SAH 4-wide traversal tree over the LBVH's exact leaf boxes (wide_bvh.cpp)
            std::vector<int> all(n);
            for (size_t p = 0; p < n; ++p) all[p] = (int)p;
            j.n4 = tpt::build_wide_sah(all, j.lbox, j.lemit, leaf_base, 0, j.w4, &j.need, j.prm);
        }
        clk.mark("sah");
        // The direct probe's first pass (closest emissive hit, trace.hip
        // TM_EMIT) walks a tree over the emissive triangles alone, appended
        // after the main tree's nodes: same exact leaf boxes and positions, so
        // the same hit as the emitter-filtered walk of the whole tree.
        std::vector<int> em;
        for (size_t p = 0; p < n; ++p)
            if (j.lemit[p]) em.push_back((int)p);
        if (!em.empty())
            j.ne4 = tpt::build_wide_sah(em, j.lbox, j.lemit, leaf_base, j.base(), j.e4, &j.eneed, j.prm);
        clk.mark("emit_tree");
    } catch (const std::bad_alloc&) {
        j.st = TPT_ERR_OOM;
        j.msg = "traversal tree build: host allocation failed";
    } catch (const std::exception& ex) {
        j.st = TPT_ERR_HIP;
        j.msg = std::string("traversal tree build: ") + ex.what();
    }
}

}  // namespace

struct tpt_scene {
    int device = 0;
    hipStream_t stream = nullptr;
    hipEvent_t ev[4] = {nullptr, nullptr, nullptr, nullptr};
    int32_t n_faces = 0, n_vertices = 0, n_objects = 0, n_materials = 0, n_lights = 0;
    bool built = false;
    int32_t stack_depth = 0;
    int32_t boxes_finite = 0;
    int32_t any_emitter = 1;                // some triangle's material has emissionFactor != 0
    int32_t n4 = 0;
    int32_t wide_tree = 0;                  // 1: inner4 holds the SAH 4-wide tree (wide_bvh.cpp)
    int32_t emit_root = -1;                 // inner4 id of the emissive-triangle tree's root (-1: none)
    int32_t emit_inline = 0;                // that tree is one node of leaves (<= 4 emitters)
    float emit_box[24] = {};                // boxes around the emitters' leaf boxes (TraceArgs emit_box)
    int32_t n_emit_box = 0;
    int32_t slivers = 0;                    // sliver triangles (trace.hip "Culling"), re-tested after traversal
    int32_t n_sliver_groups = 0;
    DevBuf<float4> sliver_groups, sliver_list;
    float cull_eps = 0.0f;                  // absolute position slack of the t-culls
    uint32_t tree_depth = 0;
    int32_t build_threads = -1;             // SAH tree build threads (tpt_scene_set_build_threads)
    DevBuf<uint8_t> sliver_flags;           // k_sliver_scan outputs
    DevBuf<unsigned long long> coord_max;
    HostPinned<float> h_lbox;               // read-back staging of a build (leaf boxes, emitter flags,
    HostPinned<uint32_t> h_lemit;           // sliver flags + coord_max); declared before `trees`, which
    HostPinned<uint8_t> h_sliver;           // reads them and is destroyed (joined) first
    std::unique_ptr<HostTrees> trees;       // the host half of the builds
    bool pending = false;                   // tpt_scene_build_async's host half runs / is not uploaded yet
    uint32_t pending_need = 0;              // its stack bound before the trees
    // inputs
    DevBuf<uint32_t> indices;
    DevBuf<float> vertices, normals, vert_trans, normal_trans;
    DevBuf<int2> lut;
    DevBuf<float4> mtl;
    DevBuf<tpt::DevLight> lights;
    DevBuf<uint32_t> jumps;
    // world + BVH
    DevBuf<float> wverts, wnorms, leaf_box, node_box;
    DevBuf<unsigned long long> keys, keys_sorted, bfs_keys, bfs_keys_sorted;
    DevBuf<uint32_t> fids, fids_sorted, parent, flags, max_depth, bfs_ids, bfs_ids_sorted, bfs_newid, emit;
    DevBuf<int2> children;
    DevBuf<uint8_t> sort_tmp, nodes36;
    DevBuf<float4> inner, inner4, tri, shade;
    // frame state
    DevBuf<uint32_t> rng;
    DevBuf<float> accum, radiance_tmp;
    DevBuf<uint8_t> bgra_tmp;
    DevBuf<unsigned long long> counters, debug;
    size_t frame_pixels = 0;
    // progressive accumulation (TPT_FLAG_ACCUMULATE): the frame the rng/accum state belongs to
    bool acc_valid = false;
    int acc_w = 0, acc_h = 0, acc_rows = 0, acc_count = 0, acc_index = 0;
    std::vector<int32_t> acc_list;          // the explicit deal it was rendered with (empty: interleaved)
    uint64_t acc_spp = 0;
    // explicit band deals (tpt_params.band_list): the call's list, then each band
    // set's share of it (host copy kept until the call's copies have run)
    DevBuf<int32_t> band_lists;
    std::vector<int32_t> band_lists_h;
    DevBuf<unsigned long long> band_cost;   // per global band: summed wave life (tpt_params.band_cost)
    std::vector<unsigned long long> band_cost_h;
    // the chip, from hipDeviceProp_t: compute units, and the lanes the one-lane
    // trace variant keeps resident (CUs x 4 SIMDs x its waves per SIMD x 64)
    int32_t n_cu = 0;
    uint64_t resident_lanes = 0;
    std::vector<uint64_t> acc_seeds;        // one per frame of the batch
    // overlapped launch pipeline: extra streams (set k >= 1 of a frame's rows)
    // and a pool of per-launch timing events
    std::vector<hipStream_t> pipe;
    std::vector<hipEvent_t> lev;
    hipEvent_t pipe_ev[2 * kMaxPipe] = {};
    // wavefront variant (TPT_FLAG_WAVEFRONT, wavefront.hip): slot state, path
    // records, the two ray queues, the hit records, the control words
    DevBuf<uint32_t> wf_state, wf_ctl;
    DevBuf<float> wf_rec;
    DevBuf<float4> wf_q0, wf_q1, wf_hit;
    HostPinned<uint32_t> wf_count;
    hipEvent_t wf_ev[2] = {nullptr, nullptr};

    ~tpt_scene() {
        DeviceGuard g(device);
        for (auto& e : ev)
            if (e) (void)hipEventDestroy(e);
        for (auto& e : lev)
            if (e) (void)hipEventDestroy(e);
        for (auto& e : pipe_ev)
            if (e) (void)hipEventDestroy(e);
        for (auto& e : wf_ev)
            if (e) (void)hipEventDestroy(e);
        for (auto& q : pipe)
            if (q) (void)hipStreamDestroy(q);
        if (stream) (void)hipStreamDestroy(stream);
    }

    // streams for the n band sets and the fork/join events.  Every set needs a
    // hardware queue of its own: two streams on one queue run their launches
    // one after another (a process has GPU_MAX_HW_QUEUES = 4; measured on the
    // box, one or two idle streams created earlier in the process -- a
    // communicator's -- made two sets share a queue: -25 %).  The runtime
    // keeps a queue pool per stream priority, so the sets' streams are created
    // at the greatest priority, where nothing else in the process competes.
    hipError_t ensure_pipe(int n) {
        hipError_t e = hipSuccess;
        int lo = 0, hi = 0;
        e = hipDeviceGetStreamPriorityRange(&lo, &hi);
        while (e == hipSuccess && (int)pipe.size() < n) {
            hipStream_t q = nullptr;
            e = hipStreamCreateWithPriority(&q, hipStreamNonBlocking, hi);
            if (e == hipSuccess) pipe.push_back(q);
        }
        for (int i = 0; e == hipSuccess && i < 2 * kMaxPipe; ++i)
            if (!pipe_ev[i]) e = hipEventCreateWithFlags(&pipe_ev[i], hipEventDisableTiming);
        return e;
    }
    hipError_t ensure_launch_events(size_t n) {
        hipError_t e = hipSuccess;
        while (e == hipSuccess && lev.size() < n) {
            hipEvent_t x = nullptr;
            e = hipEventCreate(&x);
            if (e == hipSuccess) lev.push_back(x);
        }
        return e;
    }
};

extern "C" {

const char* tpt_version(void) { return "tpt-mi355x 0.1 (gfx950)"; }

const char* tpt_last_error(void) { return g_last_error.c_str(); }

int tpt_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) {
        (void)hipGetLastError();
        return 0;
    }
    return n;
}

tpt_status tpt_scene_create(const tpt_scene_desc* d_in, int device, tpt_scene** out) {
    if (!d_in || !out) return fail(TPT_ERR_INVALID_ARG, "null argument");
    *out = nullptr;
    if (d_in->n_faces == 0 || !d_in->indices || !d_in->vertices || !d_in->normals || d_in->n_vertices == 0)
        return fail(TPT_ERR_INVALID_ARG, "scene needs faces, vertices and normals");
    if (d_in->n_objects == 0 || !d_in->lut || !d_in->vert_trans || !d_in->normal_trans)
        return fail(TPT_ERR_INVALID_ARG, "scene needs at least one object (LUT + transforms)");
    if (d_in->n_lights > (uint32_t)tpt::kMaxLights) return fail(TPT_ERR_INVALID_ARG, "too many delta lights (max 16)");
    if (d_in->n_lights > 0 && !d_in->lights) return fail(TPT_ERR_INVALID_ARG, "null light array");
    if (d_in->n_faces > (1u << 30)) return fail(TPT_ERR_INVALID_ARG, "too many faces");
    if (d_in->flags & ~(uint32_t)TPT_DESC_DELTALIGHT_LAYOUT) return fail(TPT_ERR_INVALID_ARG, "unknown desc flags");
    int ndev = tpt_device_count();
    if (ndev <= 0) return fail(TPT_ERR_NO_DEVICE, "no HIP device available");
    if (device < 0 || device >= ndev) return fail(TPT_ERR_INVALID_ARG, "bad device index");

    DeviceGuard g(device);
    // Arrays may live in device memory (DeviceScene's thrust buffers, the
    // `trace` kernel's arguments): the small ones and the indices (validated
    // here) are read back; vertices and normals are copied device to device.
    tpt_scene_desc dh = *d_in;
    const tpt_scene_desc* d = &dh;
    std::vector<uint32_t> t_idx;
    std::vector<tpt_interval> t_lut;
    std::vector<float> t_vt, t_nt;
    std::vector<tpt_material> t_mtl;
    std::vector<tpt_light> t_lights;
    hipError_t herr = hipSuccess;
    dh.indices = host_view(d_in->indices, 3 * (size_t)d_in->n_faces, t_idx, &herr);
    dh.lut = host_view(d_in->lut, d_in->n_objects, t_lut, &herr);
    dh.vert_trans = host_view(d_in->vert_trans, 16 * (size_t)d_in->n_objects, t_vt, &herr);
    dh.normal_trans = host_view(d_in->normal_trans, 16 * (size_t)d_in->n_objects, t_nt, &herr);
    dh.materials = host_view(d_in->materials, d_in->n_materials, t_mtl, &herr);
    dh.lights = host_view(d_in->lights, d_in->n_lights, t_lights, &herr);
    if (herr != hipSuccess) return fail(TPT_ERR_HIP, std::string("scene desc readback: ") + hipGetErrorString(herr));
    // Device vertices / normals are copied device to device on this scene's
    // stream, so they must live on `device` itself (another GPU's buffers would
    // need peer access): a buffer of another device is rejected.
    int v_owner = -1, n_owner = -1;
    const bool verts_dev = is_device_ptr(d_in->vertices, &v_owner), norms_dev = is_device_ptr(d_in->normals, &n_owner);
    if ((v_owner >= 0 && v_owner != device) || (n_owner >= 0 && n_owner != device))
        return fail(TPT_ERR_INVALID_ARG, "device vertex/normal buffers must live on the scene's device");

    for (uint64_t i = 0; i < 3ull * d->n_faces; ++i)
        if (d->indices[i] >= d->n_vertices) return fail(TPT_ERR_INVALID_ARG, "vertex index out of range");
    if (d->lut[0].begin != 0) return fail(TPT_ERR_INVALID_ARG, "first object must begin at face 0");

    tpt_scene* s = new (std::nothrow) tpt_scene();
    if (!s) return fail(TPT_ERR_OOM, "host allocation failed");
    s->device = device;
    auto cleanup = [&](tpt_status st) {
        delete s;
        return st;
    };
    hipError_t e = hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking);
    for (int i = 0; e == hipSuccess && i < 4; ++i) e = hipEventCreate(&s->ev[i]);
    if (e != hipSuccess) return cleanup(fail(TPT_ERR_HIP, std::string("stream/event: ") + hipGetErrorString(e)));
    {
        // the launch rules that key on the chip's resident lanes (tpt_render_frames:
        // four lanes per pixel, drained launches) take them from the device
        hipDeviceProp_t prop{};
        e = hipGetDeviceProperties(&prop, device);
        if (e != hipSuccess) return cleanup(fail(TPT_ERR_HIP, std::string("device properties: ") + hipGetErrorString(e)));
        s->n_cu = prop.multiProcessorCount;
        s->resident_lanes = (uint64_t)std::max(s->n_cu, 1) * 4u * (uint64_t)tpt::trace_waves_per_simd() * 64u;
    }

    s->n_faces = (int32_t)d->n_faces;
    s->n_vertices = (int32_t)d->n_vertices;
    s->n_objects = (int32_t)d->n_objects;
    s->n_materials = (int32_t)d->n_materials;
    s->n_lights = (int32_t)d->n_lights;

    std::vector<int2> lut(d->n_objects);
    for (uint32_t i = 0; i < d->n_objects; ++i) lut[i] = make_int2(d->lut[i].begin, d->lut[i].mtl);
    // materials + one Material() slot for meshes without a material (App. A.9)
    std::vector<float4> mtl(2 * ((size_t)d->n_materials + 1));
    for (uint32_t i = 0; i <= d->n_materials; ++i) {
        tpt_material m = (i < d->n_materials && d->materials) ? d->materials[i] : tpt::default_material();
        mtl[2 * i] = make_float4(m.base_color[0], m.base_color[1], m.base_color[2], m.emission_factor);
        mtl[2 * i + 1] = make_float4(m.eta, m.metallic, 0.0f, 0.0f);
    }
    const bool union_layout = (d->flags & TPT_DESC_DELTALIGHT_LAYOUT) != 0;
    std::vector<tpt::DevLight> lights(d->n_lights);
    for (uint32_t i = 0; i < d->n_lights; ++i) {
        const tpt_light& L = d->lights[i];
        if (L.type < 0 || L.type > 2) return cleanup(fail(TPT_ERR_INVALID_ARG, "unknown delta light type"));
        tpt::DevLight& o = lights[i];
        o.type = L.type;
        std::memcpy(o.color, L.color, sizeof o.color);
        o.intensity = L.intensity;
        if (union_layout) {
            // DeltaLight (delta_light.h:96-130): the union's members share their
            // first bytes -- color, intensity, then PointLight::pos /
            // DirectionalLight::direction / SpotLight::pos; only a spot light has
            // the direction and cone fields behind them.  Bytes a light type does
            // not own are not read.
            std::memset(o.pos, 0, sizeof o.pos);
            std::memset(o.dir, 0, sizeof o.dir);
            o.cos_outer = 0.0f;
            o.inv_cos_cone_diff = 0.0f;
            if (L.type == 1) {
                std::memcpy(o.dir, L.pos, sizeof o.dir);
            } else {
                std::memcpy(o.pos, L.pos, sizeof o.pos);
                if (L.type == 2) {
                    std::memcpy(o.dir, L.direction, sizeof o.dir);
                    o.cos_outer = L.cos_outer;
                    o.inv_cos_cone_diff = L.inv_cos_cone_diff;
                }
            }
        } else {
            std::memcpy(o.pos, L.pos, sizeof o.pos);
            std::memcpy(o.dir, L.direction, sizeof o.dir);
            o.cos_outer = L.cos_outer;
            o.inv_cos_cone_diff = L.inv_cos_cone_diff;
        }
    }
    const auto& jumps = host_jumps();
    hipStream_t st = s->stream;
    auto copy_in = [&](DevBuf<float>& dst, const float* src, size_t count, bool dev) {
        if (!dev) return dst.upload(src, count, st);
        hipError_t e2 = dst.alloc(count);
        if (e2 == hipSuccess) e2 = hipMemcpyAsync(dst.p, src, count * sizeof(float), hipMemcpyDeviceToDevice, st);
        return e2;
    };
    e = s->indices.upload(d->indices, 3 * (size_t)d->n_faces, st);
    if (e == hipSuccess) e = copy_in(s->vertices, d_in->vertices, 3 * (size_t)d->n_vertices, verts_dev);
    if (e == hipSuccess) e = copy_in(s->normals, d_in->normals, 3 * (size_t)d->n_vertices, norms_dev);
    if (e == hipSuccess) e = s->lut.upload(lut.data(), lut.size(), st);
    if (e == hipSuccess) e = s->vert_trans.upload(d->vert_trans, 16 * (size_t)d->n_objects, st);
    if (e == hipSuccess) e = s->normal_trans.upload(d->normal_trans, 16 * (size_t)d->n_objects, st);
    if (e == hipSuccess) e = s->mtl.upload(mtl.data(), mtl.size(), st);
    if (e == hipSuccess && !lights.empty()) e = s->lights.upload(lights.data(), lights.size(), st);
    if (e == hipSuccess) e = s->jumps.upload(jumps.data(), jumps.size(), st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    if (e != hipSuccess)
        return cleanup(fail(e == hipErrorOutOfMemory ? TPT_ERR_OOM : TPT_ERR_HIP,
                            std::string("scene upload: ") + hipGetErrorString(e)));
    *out = s;
    return TPT_OK;
}

tpt_status tpt_scene_set_build_threads(tpt_scene* s, int32_t threads) {
    if (!s) return fail(TPT_ERR_INVALID_ARG, "null scene");
    s->build_threads = threads;
    return TPT_OK;
}

namespace {

// The direct-probe pre-test's boxes (trace.hip probe_misses_emitters): the
// child boxes of the emissive tree's root node (4-wide layout, wide_bvh.cpp;
// they enclose every emissive triangle's leaf box), with a pair merged into
// its union while the union's surface area is at most the pair's summed areas
// (heavily overlapping boxes, e.g. the two triangles of one quad light, cost
// a test each for nothing).  Writes lo.xyz, hi.xyz per box and returns the box
// count (0: a non-finite box, no pre-test).
float box_area(const float* b) {
    const float x = b[3] - b[0], y = b[4] - b[1], z = b[5] - b[2];
    return 2.0f * (x * y + y * z + z * x);
}
int emitter_boxes(const float* root, float* out) {
    float bx[4][6];
    int n = 0;
    int32_t links[4];
    std::memcpy(links, root + 24, sizeof links);
    for (int k = 0; k < 4; ++k) {
        if (links[k] < 0) continue;
        for (int i = 0; i < 6; ++i) {
            if (!std::isfinite(root[6 * k + i])) return 0;
            bx[n][i] = root[6 * k + i];
        }
        ++n;
    }
    for (bool merged = true; merged && n > 1;) {
        merged = false;
        for (int a = 0; a < n && !merged; ++a)
            for (int b = a + 1; b < n && !merged; ++b) {
                float u[6];
                for (int i = 0; i < 3; ++i) {
                    u[i] = std::min(bx[a][i], bx[b][i]);
                    u[3 + i] = std::max(bx[a][3 + i], bx[b][3 + i]);
                }
                if (box_area(u) <= box_area(bx[a]) + box_area(bx[b])) {
                    std::memcpy(bx[a], u, sizeof u);
                    std::memcpy(bx[b], bx[n - 1], sizeof u);
                    --n;
                    merged = true;
                }
            }
    }
    for (int k = 0; k < n; ++k) std::memcpy(out + 6 * k, bx[k], sizeof bx[k]);
    return n;
}

// Uploads a finished HostTrees job and completes the scene (the stack bound).
tpt_status upload_host_trees(tpt_scene* s, HostTrees& j, uint32_t* wide_need) {
    if (j.st != TPT_OK) return fail(j.st, j.msg);
    if (j.main_ok()) {
        HIP_OR_FAIL(hipMemcpyAsync(s->inner4.p, j.w4.data(), j.w4.size() * sizeof(float), hipMemcpyHostToDevice,
                                   s->stream));
        s->n4 = j.n4;
        *wide_need = (uint32_t)j.need;
        s->wide_tree = 1;
    }
    if (j.emit_ok()) {
        HIP_OR_FAIL(hipMemcpyAsync(s->inner4.p + 8 * (size_t)s->n4, j.e4.data(), j.e4.size() * sizeof(float),
                                   hipMemcpyHostToDevice, s->stream));
        s->emit_root = s->n4;
        s->emit_inline = j.ne4 == 1 ? 1 : 0;
        s->n_emit_box = emitter_boxes(j.e4.data(), s->emit_box);
        *wide_need = std::max(*wide_need, (uint32_t)j.eneed);
    }
    HIP_OR_FAIL(hipStreamSynchronize(s->stream));   // (the host buffers are freed after this)
    return TPT_OK;
}

// Stack capacity: the binary DFS that pushes one sibling per level holds at
// most depth + 1 entries; the 4-wide ordered walk holds at most the tree's
// stack need (wide_bvh.cpp), 3 * ceil(depth / 2) for the LBVH's even-depth view.
tpt_status finish_stack(tpt_scene* s, uint32_t wide_need) {
    s->stack_depth = (int32_t)std::max<uint32_t>(std::max<uint32_t>(s->tree_depth + 2, wide_need), 2);
    if (s->stack_depth > 160) return fail(TPT_ERR_INVALID_ARG, "BVH deeper than the LDS stack supports");
    s->built = true;
    return TPT_OK;
}

}  // namespace

// Joins an asynchronous build's host half and uploads its trees (a no-op
// without one).  Every entry point that reads the traversal trees calls it.
static tpt_status finish_pending(tpt_scene* s, double* wait_ms = nullptr) {
    if (!s->pending) return TPT_OK;
    const auto t0 = std::chrono::steady_clock::now();
    HostTrees& j = *s->trees;
    j.join();
    s->pending = false;
    if (wait_ms) *wait_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    DeviceGuard g(s->device);
    uint32_t wide_need = s->pending_need;
    tpt_status st = upload_host_trees(s, j, &wide_need);
    if (st == TPT_OK) st = finish_stack(s, wide_need);
    if (st != TPT_OK) s->built = false;
    return st;
}

static tpt_status scene_build(tpt_scene* s, bool async) {
    if (!s) return fail(TPT_ERR_INVALID_ARG, "null scene");
    if (s->trees) s->trees->join();   // a previous asynchronous build still running: its trees are superseded
    s->pending = false;
    s->built = false;
    DeviceGuard g(s->device);
    const size_t n = (size_t)s->n_faces, nn = 2 * n - 1, nv = (size_t)s->n_vertices;
    size_t sort_bytes = 0;
    HIP_OR_FAIL(tpt::build_sort_tmp_bytes((int32_t)n, &sort_bytes));
    HIP_OR_FAIL(s->wverts.alloc(3 * nv));
    HIP_OR_FAIL(s->wnorms.alloc(3 * nv));
    HIP_OR_FAIL(hipMemsetAsync(s->wverts.p, 0, 3 * nv * sizeof(float), s->stream));
    HIP_OR_FAIL(hipMemsetAsync(s->wnorms.p, 0, 3 * nv * sizeof(float), s->stream));
    HIP_OR_FAIL(s->keys.alloc(n));
    HIP_OR_FAIL(s->keys_sorted.alloc(n));
    HIP_OR_FAIL(s->fids.alloc(n));
    HIP_OR_FAIL(s->fids_sorted.alloc(n));
    HIP_OR_FAIL(s->leaf_box.alloc(6 * n));
    HIP_OR_FAIL(s->children.alloc(std::max<size_t>(n - 1, 1)));
    HIP_OR_FAIL(s->parent.alloc(nn));
    HIP_OR_FAIL(s->node_box.alloc(6 * nn));
    HIP_OR_FAIL(s->flags.alloc(nn));
    HIP_OR_FAIL(s->max_depth.alloc(3));
    HIP_OR_FAIL(s->bfs_keys.alloc(std::max<size_t>(n - 1, 1)));
    HIP_OR_FAIL(s->bfs_keys_sorted.alloc(std::max<size_t>(n - 1, 1)));
    HIP_OR_FAIL(s->bfs_ids.alloc(std::max<size_t>(n - 1, 1)));
    HIP_OR_FAIL(s->bfs_ids_sorted.alloc(std::max<size_t>(n - 1, 1)));
    HIP_OR_FAIL(s->bfs_newid.alloc(std::max<size_t>(n - 1, 1)));
    HIP_OR_FAIL(s->emit.alloc(nn));
    HIP_OR_FAIL(s->sort_tmp.alloc(std::max<size_t>(sort_bytes, 16)));
    HIP_OR_FAIL(s->inner.alloc(4 * std::max<size_t>(n - 1, 1)));
    HIP_OR_FAIL(s->inner4.alloc(8 * std::max<size_t>(n - 1, 1)));
    HIP_OR_FAIL(s->tri.alloc(tpt::tri_float4s(n)));
    HIP_OR_FAIL(s->shade.alloc(3 * n));
    HIP_OR_FAIL(s->nodes36.alloc(36 * nn));
    HIP_OR_FAIL(hipMemsetAsync(s->parent.p, 0, nn * sizeof(uint32_t), s->stream));
    PhaseClock clk(std::getenv("TPT_BUILD_TIMING") != nullptr);

    tpt::BuildBuffers b{};
    b.n_faces = s->n_faces;
    b.n_vertices = s->n_vertices;
    b.n_objects = s->n_objects;
    b.n_materials = s->n_materials;
    b.indices = s->indices.p;
    b.vertices = s->vertices.p;
    b.normals = s->normals.p;
    b.lut = s->lut.p;
    b.vert_trans = s->vert_trans.p;
    b.normal_trans = s->normal_trans.p;
    b.mtl = s->mtl.p;
    b.wverts = s->wverts.p;
    b.wnorms = s->wnorms.p;
    b.keys = s->keys.p;
    b.keys_sorted = s->keys_sorted.p;
    b.fids = s->fids.p;
    b.fids_sorted = s->fids_sorted.p;
    b.leaf_box = s->leaf_box.p;
    b.children = s->children.p;
    b.parent = s->parent.p;
    b.node_box = s->node_box.p;
    b.flags = s->flags.p;
    b.max_depth = s->max_depth.p;
    b.sort_tmp = s->sort_tmp.p;
    b.sort_tmp_bytes = sort_bytes;
    b.inner = s->inner.p;
    b.inner4 = s->inner4.p;
    b.bfs_keys = s->bfs_keys.p;
    b.bfs_keys_sorted = s->bfs_keys_sorted.p;
    b.bfs_ids = s->bfs_ids.p;
    b.bfs_ids_sorted = s->bfs_ids_sorted.p;
    b.bfs_newid = s->bfs_newid.p;
    b.emit = s->emit.p;
    b.tri = s->tri.p;
    b.shade = s->shade.p;
    b.nodes36 = s->nodes36.p;
    {
        const hipError_t be = tpt::launch_build(b, s->stream);
        if (be != hipSuccess && b.out_max_depth >= tpt::kMaxLbvhDepth)
            return fail(TPT_ERR_INVALID_ARG,
                        "LBVH topology invalid: duplicate Morton keys made a node's parent chain miss the root "
                        "(computeNodeRange, bvh.cu:150-217, has no tie-break; the reference would not terminate)");
        HIP_OR_FAIL(be);
    }
    s->tree_depth = b.out_max_depth;
    s->boxes_finite = (int32_t)b.out_boxes_finite;
    s->n4 = (int32_t)b.out_n4;
    {   // the root's emitter flag: does any triangle emit (a probe can only add emission)
        uint32_t root_emit = 1;
        HIP_OR_FAIL(hipMemcpyAsync(&root_emit, s->emit.p, sizeof root_emit, hipMemcpyDeviceToHost, s->stream));
        HIP_OR_FAIL(hipStreamSynchronize(s->stream));
        s->any_emitter = root_emit != 0 ? 1 : 0;
    }
    clk.mark("lbvh");
    const uint32_t td = b.out_max_depth;
    uint32_t wide_need = 3 * ((td + 1) / 2) + 1;
    s->wide_tree = 0;
    s->emit_root = -1;
    s->emit_inline = 0;
    s->n_emit_box = 0;
    s->slivers = 0;
    s->n_sliver_groups = 0;
    s->cull_eps = 0.0f;
    if (n > 1 && s->boxes_finite) {
        // Culling exactness (trace.hip "Culling"): sliver triangles -- sin of the
        // angle at v0 between the edges rayHitTriangle uses below 1e-3 -- give
        // an arbitrary t, so they are listed (in up to 4 groups with union
        // boxes) and re-tested after every culled traversal; the culls'
        // absolute position slack is 4 ulps of the largest world coordinate (a
        // hit point, the next ray's origin, is rounded to its ulp; an edge hit
        // accepted by barycentric rounding lies a few ulps outside its triangle).
        // Both come from k_sliver_scan; the leaf boxes and emitter flags (for
        // the host trees) come back with them into pinned staging.
        HIP_OR_FAIL(s->sliver_flags.alloc(n));
        HIP_OR_FAIL(s->coord_max.alloc(1));
        HIP_OR_FAIL(hipMemsetAsync(s->coord_max.p, 0, sizeof(unsigned long long), s->stream));
        HIP_OR_FAIL(tpt::launch_sliver_scan(s->tri.p, (int32_t)n, s->sliver_flags.p, s->coord_max.p, s->stream));
        HIP_OR_FAIL(s->h_lbox.alloc(6 * n));
        HIP_OR_FAIL(s->h_lemit.alloc(n));
        HIP_OR_FAIL(s->h_sliver.alloc(n + 8));
        float* const lbox = s->h_lbox.p;
        uint32_t* const lemit = s->h_lemit.p;
        uint8_t* const lsliver = s->h_sliver.p;
        HIP_OR_FAIL(hipMemcpyAsync(lbox, s->node_box.p + 6 * (n - 1), 6 * n * sizeof(float), hipMemcpyDeviceToHost,
                                   s->stream));
        HIP_OR_FAIL(hipMemcpyAsync(lemit, s->emit.p + (n - 1), n * sizeof(uint32_t), hipMemcpyDeviceToHost, s->stream));
        HIP_OR_FAIL(hipMemcpyAsync(lsliver, s->sliver_flags.p, n, hipMemcpyDeviceToHost, s->stream));
        HIP_OR_FAIL(hipMemcpyAsync(lsliver + n, s->coord_max.p, sizeof(unsigned long long), hipMemcpyDeviceToHost,
                                   s->stream));
        HIP_OR_FAIL(hipStreamSynchronize(s->stream));
        clk.mark("readback");
        std::vector<int> sl;
        for (size_t p = 0; p < n; ++p)
            if (lsliver[p]) sl.push_back((int)p);
        unsigned long long mbits = 0;
        std::memcpy(&mbits, lsliver + n, sizeof mbits);
        double max_coord = 0.0;
        std::memcpy(&max_coord, &mbits, sizeof max_coord);
        s->slivers = (int32_t)sl.size();
        s->cull_eps = 0.0f;
        if (std::isfinite(max_coord) && max_coord > 0.0) {
            int ex = 0;
            (void)std::frexp(max_coord, &ex);                     // max_coord < 2^ex
            s->cull_eps = (float)std::ldexp(4.0, ex - 24);        // 4 ulps of a float below 2^ex
        }
        s->n_sliver_groups = 0;
        if (!sl.empty()) {
            // groups 1..: split the list at the median of the longest centroid axis
            // while a group holds more than 8 slivers and there are < 8 groups;
            // group 0 is the union of all (tested first by every ray)
            std::vector<std::pair<int, int>> grp{{0, (int)sl.size()}};
            auto cen = [&](int p, int k) { return lbox[6 * p + k] + lbox[6 * p + 3 + k]; };
            for (bool split = true; split && grp.size() < 8;) {
                split = false;
                size_t big = 0;
                for (size_t g = 1; g < grp.size(); ++g)
                    if (grp[g].second - grp[g].first > grp[big].second - grp[big].first) big = g;
                const int b0 = grp[big].first, b1 = grp[big].second;
                if (b1 - b0 <= 8) break;
                float lo[3] = {kInfF, kInfF, kInfF}, hi[3] = {-kInfF, -kInfF, -kInfF};
                for (int i = b0; i < b1; ++i)
                    for (int k = 0; k < 3; ++k) {
                        lo[k] = std::min(lo[k], cen(sl[i], k));
                        hi[k] = std::max(hi[k], cen(sl[i], k));
                    }
                int ax = 0;
                for (int k = 1; k < 3; ++k)
                    if (hi[k] - lo[k] > hi[ax] - lo[ax]) ax = k;
                const int mid = (b0 + b1) / 2;
                std::nth_element(sl.begin() + b0, sl.begin() + mid, sl.begin() + b1,
                                 [&](int x, int y) { return cen(x, ax) < cen(y, ax); });
                grp[big] = {b0, mid};
                grp.push_back({mid, b1});
                split = true;
            }
            grp.insert(grp.begin(), {0, (int)sl.size()});   // group 0: the union
            std::vector<float4> gb(2 * grp.size());
            std::vector<float4> lst(2 * sl.size());   // exact leaf box, position | emissive << 30
            for (size_t i = 0; i < sl.size(); ++i) {
                const int32_t e = sl[i] | (lemit[sl[i]] ? (1 << 30) : 0);
                float fe;
                std::memcpy(&fe, &e, 4);
                const float* b = &lbox[6 * sl[i]];
                lst[2 * i] = make_float4(b[0], b[1], b[2], fe);
                lst[2 * i + 1] = make_float4(b[3], b[4], b[5], 0.0f);
            }
            for (size_t g = 0; g < grp.size(); ++g) {
                float lo[3] = {kInfF, kInfF, kInfF}, hi[3] = {-kInfF, -kInfF, -kInfF};
                for (int i = grp[g].first; i < grp[g].second; ++i)
                    for (int k = 0; k < 3; ++k) {
                        lo[k] = std::min(lo[k], lbox[6 * sl[i] + k]);
                        hi[k] = std::max(hi[k], lbox[6 * sl[i] + 3 + k]);
                    }
                int32_t first = grp[g].first, count = grp[g].second - grp[g].first;
                float ff, fc;
                std::memcpy(&ff, &first, 4);
                std::memcpy(&fc, &count, 4);
                gb[2 * g] = make_float4(lo[0], lo[1], lo[2], ff);
                gb[2 * g + 1] = make_float4(hi[0], hi[1], hi[2], fc);
            }
            HIP_OR_FAIL(s->sliver_groups.upload(gb.data(), gb.size(), s->stream));
            HIP_OR_FAIL(s->sliver_list.upload(lst.data(), lst.size(), s->stream));
            HIP_OR_FAIL(hipStreamSynchronize(s->stream));   // (gb and lst are freed below)
            s->n_sliver_groups = (int32_t)grp.size();
        }
        clk.mark("slivers");
        if (!s->trees) {
            try {
                s->trees = std::make_unique<HostTrees>();
            } catch (const std::bad_alloc&) {
                return fail(TPT_ERR_OOM, "traversal tree build: host allocation failed");
            }
        }
        HostTrees& j = *s->trees;
        j.reset_results();
        j.n = n;
        j.lbox = lbox;     // the scene's pinned staging: the next build joins this job first
        j.lemit = lemit;
        j.prm.threads = s->build_threads;
#ifdef TPT_WIDE_SWEEP
        j.prm.sweep_max = TPT_WIDE_SWEEP;   // A/B builds: exact-sweep threshold
#endif
        j.lbvh_n4 = s->n4;
        j.timing = clk.on;
        if (async) {
            s->pending_need = wide_need;
            HostTrees* jp = &j;
            try {
                j.th = std::thread([jp] { build_host_trees(*jp); });
                s->pending = true;
                s->built = true;   // (finish_pending completes it)
                return TPT_OK;
            } catch (const std::exception&) {   // no thread (system_error, bad_alloc): build it here
            }
        }
        build_host_trees(j);
        const tpt_status st = upload_host_trees(s, j, &wide_need);
        if (st != TPT_OK) return st;
        clk.mark("upload");
    }
    return finish_stack(s, wide_need);
}

tpt_status tpt_scene_build(tpt_scene* s) { return scene_build(s, false); }

tpt_status tpt_scene_build_async(tpt_scene* s) { return scene_build(s, true); }

void tpt_scene_destroy(tpt_scene* s) { delete s; }

tpt_status tpt_env_create(const uint8_t* rgba, int32_t w, int32_t h, int device, tpt_env** out) {
    if (!rgba || !out || w <= 0 || h <= 0) return fail(TPT_ERR_INVALID_ARG, "bad env arguments");
    *out = nullptr;
    int ndev = tpt_device_count();
    if (ndev <= 0) return fail(TPT_ERR_NO_DEVICE, "no HIP device available");
    if (device < 0 || device >= ndev) return fail(TPT_ERR_INVALID_ARG, "bad device index");
    DeviceGuard g(device);
    tpt_env* env = new (std::nothrow) tpt_env();
    if (!env) return fail(TPT_ERR_OOM, "host allocation failed");
    env->device = device;
    env->w = w;
    env->h = h;
    hipError_t e = env->texels.alloc((size_t)w * (size_t)h);
    if (e == hipSuccess) e = hipMemcpy(env->texels.p, rgba, (size_t)w * h * 4, hipMemcpyHostToDevice);
    std::vector<float> icond, irow, imarg;
    env->is_b = env_is_block(w, h);
    env->is_bw = (w + env->is_b - 1) / env->is_b;
    env->is_bh = (h + env->is_b - 1) / env->is_b;
    const int bw = env->is_bw, bh = env->is_bh;
    build_env_is(rgba, w, h, env->is_b, icond, irow, imarg, env->is_total);
    if (e == hipSuccess) e = env->is_cond.upload(icond.data(), icond.size(), nullptr);
    if (e == hipSuccess) e = env->is_row.upload(irow.data(), irow.size(), nullptr);
    if (e == hipSuccess) e = env->is_marg.upload(imarg.data(), imarg.size(), nullptr);
    {   // guide tables: block rows at the block-row count, columns at a quarter of a block row
        env->is_kr = pow2_at_least(bh);
        env->is_kc = pow2_at_least(std::max(1, bw / 4));
        std::vector<int32_t> gr((size_t)env->is_kr + 1), gc((size_t)bh * (env->is_kc + 1));
        build_guide(imarg.data(), bh, env->is_total, env->is_kr, gr.data());
        for (int by = 0; by < bh; ++by)
            build_guide(icond.data() + (size_t)by * bw, bw, irow[by], env->is_kc,
                        gc.data() + (size_t)by * (env->is_kc + 1));
        if (e == hipSuccess) e = env->is_guide_r.upload(gr.data(), gr.size(), nullptr);
        if (e == hipSuccess) e = env->is_guide_c.upload(gc.data(), gc.size(), nullptr);
    }
    if (e == hipSuccess) e = hipDeviceSynchronize();
    if (e != hipSuccess) {
        delete env;
        return fail(TPT_ERR_HIP, std::string("env upload: ") + hipGetErrorString(e));
    }
    *out = env;
    return TPT_OK;
}

void tpt_env_destroy(tpt_env* env) {
    if (!env) return;
    DeviceGuard g(env->device);
    delete env;
}

tpt_status tpt_image_load(const char* path, uint8_t** rgba, int32_t* width, int32_t* height) {
    if (!path || !rgba || !width || !height) return fail(TPT_ERR_INVALID_ARG, "null argument");
    *rgba = nullptr;
    std::vector<uint8_t> px;
    int w = 0, h = 0;
    try {
        tpt::load_image(path, px, w, h);
    } catch (const tpt::io_error& e) {
        return fail(TPT_ERR_IO, e.what());
    } catch (const std::exception& e) {
        return fail(TPT_ERR_PARSE, e.what());
    }
    uint8_t* buf = static_cast<uint8_t*>(std::malloc(px.size()));
    if (!buf) return fail(TPT_ERR_OOM, "host allocation failed");
    std::memcpy(buf, px.data(), px.size());
    *rgba = buf;
    *width = w;
    *height = h;
    return TPT_OK;
}

void tpt_image_free(uint8_t* rgba) { std::free(rgba); }

tpt_status tpt_env_load(const char* path, int device, tpt_env** out) {
    if (!path || !out) return fail(TPT_ERR_INVALID_ARG, "null argument");
    *out = nullptr;
    uint8_t* px = nullptr;
    int32_t w = 0, h = 0;
    const tpt_status st = tpt_image_load(path, &px, &w, &h);
    if (st != TPT_OK) return st;
    const tpt_status st2 = tpt_env_create(px, w, h, device, out);
    tpt_image_free(px);
    return st2;
}

static tpt_status fill_trace_args(tpt_scene* s, const tpt_env* env, const tpt_camera* cam, tpt::TraceArgs& a) {
    a.inner = s->inner.p;
    a.inner4 = s->inner4.p;
    a.n4 = s->n4;
    a.tri = s->tri.p;
    a.shade = s->shade.p;
    a.mtl = s->mtl.p;
    a.n_faces = s->n_faces;
    a.n_materials = s->n_materials;
    a.n_lights = s->n_lights;
    a.lights = s->lights.p;
    a.stack_depth = s->stack_depth;
    a.boxes_finite = s->boxes_finite;
    a.any_emitter = s->any_emitter;
    a.emit_root = s->emit_root;
    a.n_emit_box = s->any_emitter ? s->n_emit_box : 0;
    for (int k = 0; k < a.n_emit_box; ++k) {
        const float* b = s->emit_box + 6 * k;
        a.emit_box[2 * k] = make_float4(b[0], b[1], b[2], 0.0f);
        a.emit_box[2 * k + 1] = make_float4(b[3], b[4], b[5], 0.0f);
    }
#ifdef TPT_NO_PROBE_PRETEST
    a.n_emit_box = 0;   // A/B builds: no probe pre-test
#endif
    a.sliver_groups = s->sliver_groups.p;
    a.sliver_list = s->sliver_list.p;
    a.n_sliver_groups = s->n_sliver_groups;
    a.cull_eps = s->cull_eps;
    a.graze = 1;
#ifdef TPT_NO_EMIT_INLINE
    a.emit_inline = 0;   // A/B builds: probe pass 1 as a traversal always
#else
    a.emit_inline = s->emit_inline;
#endif
    a.env = env ? env->texels.p : nullptr;
    a.env_w = env ? env->w : 0;
    a.env_h = env ? env->h : 0;
    a.is_b = env ? env->is_b : 1;
    a.is_bw = env ? env->is_bw : 0;
    a.is_bh = env ? env->is_bh : 0;
    a.is_cond = env ? env->is_cond.p : nullptr;
    a.is_row = env ? env->is_row.p : nullptr;
    a.is_marg = env ? env->is_marg.p : nullptr;
    a.is_total = env ? env->is_total : 0.0f;
    a.is_guide_r = env ? env->is_guide_r.p : nullptr;
    a.is_guide_c = env ? env->is_guide_c.p : nullptr;
    a.is_kr = env ? env->is_kr : 1;
    a.is_kc = env ? env->is_kc : 1;
    if (cam) {
        std::memcpy(a.c2w, cam->c2w, sizeof a.c2w);
        float r[4];
        tpt::mat4_vec4(cam->c2w, 0.0f, 0.0f, 0.0f, 1.0f, r);   // sampleRays :57
        a.origin[0] = r[0];
        a.origin[1] = r[1];
        a.origin[2] = r[2];
        const float tan_half = tpt::ptan(cam->vfov * 0.5f);    // :50-52
        a.sensor_h = 2.0f * tan_half;
        a.sensor_w = cam->aspect * a.sensor_h;
        a.half_sw = 0.5f * a.sensor_w;
        a.half_sh = 0.5f * a.sensor_h;
    }
    return TPT_OK;
}

tpt_status tpt_render(tpt_scene* s, const tpt_env* env, const tpt_camera* cam, const tpt_params* p,
                      float* radiance_out, uint8_t* bgra_out, tpt_stats* stats) {
    if (!p) return fail(TPT_ERR_INVALID_ARG, "null argument");
    const uint64_t seed = p->seed;
    return tpt_render_frames(s, env, cam, p, 1, &seed, &radiance_out, &bgra_out, stats);
}

// The wavefront / ray-queue variant (TPT_FLAG_WAVEFRONT; wavefront.hip, DESIGN.md
// section 5 "N1"): every pixel's samples on one slot, in order, so the frame is
// bit-identical to k_trace's.  Slots default to every pixel of the call (the
// whole frame in flight: the fewest iterations); the buffers stay with the
// scene between calls.  The trace phase runs on the scene's stream after the
// RNG initialisation (event ev[1]).
static tpt_status render_wavefront(tpt_scene* s, const tpt::TraceArgs& a, const tpt_params* p, int n_frames, int bh,
                                   double& trace_ms, double& kernel_ms, int& launches) {
    hipStream_t st = s->stream;
    const bool ordered = !(p->flags & TPT_FLAG_REF_ORDER);
    // the megakernel's record layout: 5 words with delta lights, env IS or the reference order
    const bool lights = !ordered || a.env_is || tpt::rec_words(s->n_lights, s->n_materials) == 5;
    tpt::WfArgs w{};
    w.t = a;
    w.t.samples = p->spp;
    w.ordered = ordered ? 1 : 0;
    w.state_words = lights ? 32 : 16;
    w.rec_words = lights ? 5 : 2;
    const size_t gx = (size_t)(p->width + 15) / 16, gy = (size_t)((bh + 15) / 16) * (size_t)n_frames;
    const size_t claims = gx * gy * 256;
    if (bh <= 0) return TPT_OK;
    if (claims > (size_t)INT32_MAX / 2) return fail(TPT_ERR_INVALID_ARG, "wavefront: frame batch too large");
    if (p->wf_slots < 0 || p->wf_refill < 0 || p->wf_refill > 64)
        return fail(TPT_ERR_INVALID_ARG, "wavefront: wf_slots >= 0, wf_refill 0..64");
    size_t slots = p->wf_slots > 0 ? (size_t)p->wf_slots : claims;
    slots = std::min(slots, claims);
    slots = (slots + 255) / 256 * 256;
    w.n_claims = (int32_t)claims;
    w.n_slots = (int32_t)slots;
    HIP_OR_FAIL(s->wf_rec.alloc(slots * (size_t)p->max_depth * (size_t)w.rec_words));
    // queue shards: a logic block appends to shard blockIdx % kWfShards, and the grid
    // (a multiple of kWfShards) deals 256-entry chunks round-robin, so a shard
    // receives at most every kWfShards-th chunk of a queue of <= slots entries
    const size_t cap = ((slots / 256) + tpt::kWfShards - 1) / tpt::kWfShards * 256;
    const size_t qn = cap * tpt::kWfShards;
    HIP_OR_FAIL(s->wf_q0.alloc(2 * qn));
    HIP_OR_FAIL(s->wf_q1.alloc(2 * qn));
    HIP_OR_FAIL(s->wf_hit.alloc(qn));
    HIP_OR_FAIL(s->wf_state.alloc(2 * qn * (size_t)w.state_words));
    HIP_OR_FAIL(s->wf_ctl.alloc(tpt::kWfCtlWords));
    HIP_OR_FAIL(s->wf_count.alloc(2 * tpt::kWfShards));
    w.shard_cap = (int32_t)cap;
    for (auto& e : s->wf_ev)
        if (!e) HIP_OR_FAIL(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    w.st0 = s->wf_state.p;
    w.st1 = s->wf_state.p + qn * (size_t)w.state_words;
    w.rec = s->wf_rec.p;
    w.q_ray0 = s->wf_q0.p;
    w.q_ray1 = s->wf_q1.p;
    w.q_hit = s->wf_hit.p;
    w.ctl = s->wf_ctl.p;
    w.refill = p->wf_refill > 0 ? p->wf_refill : 40;
    w.chunk = 128;
    w.batch = 32;
    w.logic_blocks = (int32_t)((std::min<size_t>((slots + 255) / 256, 2048) + tpt::kWfShards - 1) / tpt::kWfShards *
                               tpt::kWfShards);
    w.trace_blocks = 0;   // launch_wavefront: the CUs' occupancy
    int32_t iters = 0;
    HIP_OR_FAIL(tpt::launch_wavefront(w, s->wf_count.p, s->wf_ev, &iters, st));
    HIP_OR_FAIL(hipEventRecord(s->ev[2], st));
    HIP_OR_FAIL(hipEventSynchronize(s->ev[2]));
    float ms = 0.0f;
    HIP_OR_FAIL(hipEventElapsedTime(&ms, s->ev[1], s->ev[2]));
    trace_ms = ms;
    kernel_ms = ms;
    launches = 1 + 2 * iters;
    return TPT_OK;
}

tpt_status tpt_render_frames(tpt_scene* s, const tpt_env* env, const tpt_camera* cam, const tpt_params* p,
                             int32_t n_frames, const uint64_t* seeds, float* const* radiance_outs,
                             uint8_t* const* bgra_outs, tpt_stats* stats) {
    auto t_start = std::chrono::steady_clock::now();
    if (!s || !cam || !p || !seeds) return fail(TPT_ERR_INVALID_ARG, "null argument");
    if (n_frames < 1 || n_frames > 65535) return fail(TPT_ERR_INVALID_ARG, "bad frame count");
    if (!s->built) return fail(TPT_ERR_INVALID_ARG, "scene not built (call tpt_scene_build)");
    if (p->width <= 0 || p->height <= 0 || p->spp <= 0 || p->max_depth < 1 || p->max_depth > 64)
        return fail(TPT_ERR_INVALID_ARG, "bad frame parameters");
    if ((int64_t)p->width * p->height > (int64_t)1 << 30) return fail(TPT_ERR_INVALID_ARG, "frame too large");
    const int band_rows = p->band_rows > 0 ? p->band_rows : 16;
    // an explicit deal (band_list) replaces the interleaved one (band_count, band_index)
    const bool listed = p->band_list != nullptr;
    const int band_count = listed ? 1 : (p->band_count > 0 ? p->band_count : 1);
    const int band_index = listed ? 0 : p->band_index;
    if (!listed && (p->band_index < 0 || p->band_index >= band_count))
        return fail(TPT_ERR_INVALID_ARG, "bad band index");
    if (env && env->device != s->device) return fail(TPT_ERR_INVALID_ARG, "env lives on another device");
    const int W = p->width, H = p->height;
    const int n_bands = (H + band_rows - 1) / band_rows;
    std::vector<int32_t> list;
    if (listed) {
        if (p->band_list_len < 0 || p->band_list_len > n_bands)
            return fail(TPT_ERR_INVALID_ARG, "band_list_len: 0 .. ceil(height / band_rows)");
        list.assign(p->band_list, p->band_list + p->band_list_len);
        std::vector<uint8_t> seen((size_t)n_bands, 0);
        const bool partial = H % band_rows != 0;   // the last band is short: it must come last (kernels
        for (size_t i = 0; i < list.size(); ++i) {  // map local row ly to list[ly / band_rows])
            if (list[i] < 0 || list[i] >= n_bands || seen[(size_t)list[i]]++ ||
                (partial && list[i] == n_bands - 1 && i + 1 != list.size()))
                return fail(TPT_ERR_INVALID_ARG, "band_list: distinct band ids below ceil(height / band_rows), "
                                                 "a short last band last");
        }
    }
    auto rows_of = [&](const std::vector<int32_t>& l) {
        int n = 0;
        for (int32_t b : l) n += std::min(band_rows, H - b * band_rows);
        return n;
    };
    DeviceGuard g(s->device);
    hipStream_t st = s->stream;
    const size_t npix = (size_t)W * (size_t)H;
    const size_t nf = (size_t)n_frames;
    const int bh = listed ? rows_of(list) : band_height_of(H, band_rows, band_count, band_index);
    const std::vector<uint64_t> fseeds(seeds, seeds + nf);

    const bool resume = (p->flags & TPT_FLAG_ACCUMULATE) && s->acc_valid && s->acc_w == W && s->acc_h == H &&
                        s->acc_rows == band_rows && s->acc_count == band_count && s->acc_index == band_index &&
                        s->acc_list == list && s->acc_seeds == fseeds && s->rng.n == 6 * npix * nf &&
                        s->accum.n == 3 * npix * nf;
    s->acc_valid = false;   // re-armed once this call has completed
    // per-frame state planes, frame f at offset f * (6|3) * npix
    HIP_OR_FAIL(s->rng.alloc(6 * npix * nf));
    HIP_OR_FAIL(s->accum.alloc(3 * npix * nf));
    HIP_OR_FAIL(s->counters.alloc(32));
    if (!resume) HIP_OR_FAIL(hipMemsetAsync(s->accum.p, 0, 3 * npix * nf * sizeof(float), st));   // thrust::fill (:534)
    HIP_OR_FAIL(hipMemsetAsync(s->counters.p, 0, 32 * sizeof(unsigned long long), st));
    // the explicit deal's list on the device: the whole list first, the band sets'
    // shares after it (written once the launch plan is known)
    const int32_t* d_list = nullptr;
    if (listed && !list.empty()) {
        s->band_lists_h.assign(2 * list.size(), 0);
        std::copy(list.begin(), list.end(), s->band_lists_h.begin());
        HIP_OR_FAIL(s->band_lists.alloc(std::max(s->band_lists.n, 2 * list.size())));
        HIP_OR_FAIL(hipMemcpyAsync(s->band_lists.p, s->band_lists_h.data(), list.size() * sizeof(int32_t),
                                   hipMemcpyHostToDevice, st));
        d_list = s->band_lists.p;
    }
    if (p->band_cost) {
        HIP_OR_FAIL(s->band_cost.alloc(std::max<size_t>(s->band_cost.n, (size_t)n_bands)));
        HIP_OR_FAIL(hipMemsetAsync(s->band_cost.p, 0, (size_t)n_bands * sizeof(unsigned long long), st));
    }

    // setupRandSeed (:513), one seed per frame; a progressive call continues the persisted streams
    HIP_OR_FAIL(hipEventRecord(s->ev[0], st));
    if (bh > 0 && !resume)
        for (size_t f = 0; f < nf; ++f)
            HIP_OR_FAIL(tpt::launch_rng_init(s->jumps.p, fseeds[f], W, band_rows, band_count, band_index, d_list, bh,
                                             H, s->rng.p + f * 6 * npix, st));
    HIP_OR_FAIL(hipEventRecord(s->ev[1], st));
    // an asynchronous scene build's host half ran while the above was enqueued
    double tree_wait_ms = 0.0;
    {
        const tpt_status bs = finish_pending(s, &tree_wait_ms);
        if (bs != TPT_OK) return bs;
    }
    const uint64_t total_spp = (resume ? s->acc_spp : 0) + (uint64_t)p->spp;
    if (total_spp > (uint64_t)INT32_MAX) return fail(TPT_ERR_INVALID_ARG, "accumulated spp overflow");

    tpt::TraceArgs a{};
    fill_trace_args(s, env, cam, a);
    a.inv_w = 1.0f / (float)W;
    a.inv_h = 1.0f / (float)H;
    a.width = W;
    a.height = H;
    a.band_rows = band_rows;
    a.band_count = band_count;
    a.band_index = band_index;
    a.band_list = d_list;
    a.band_cost = p->band_cost ? s->band_cost.p : nullptr;
    a.band_height = bh;
    a.n_frames = n_frames;
    a.max_depth = p->max_depth;
    a.flags = p->flags;
    // culls without the exactness guards (trace.hip "Culling"); the tolerance mode too:
    // its C5 band measures the same with the guards kept
    if (p->flags & (TPT_FLAG_APPROX_CULL | TPT_FLAG_FAST)) {
        a.cull_eps = 0.0f;
        a.n_sliver_groups = 0;
        a.graze = 0;
    }
    // A15 env next-event estimation: opt-in, needs an env with a non-empty distribution
    a.env_is = ((p->flags & TPT_FLAG_ENV_IS) && env && env->is_total > 0.0f) ? 1 : 0;

    if (p->lanes_per_pixel < 0 || p->lanes_per_pixel > 4 || p->lanes_per_pixel == 3)
        return fail(TPT_ERR_INVALID_ARG, "lanes_per_pixel: 0, 1, 2 or 4");
    // auto: pair mode wherever there are shadow rays to hand off (C3 1080p 4096 spp:
    // 4.91 -> 6.65 Grays/s); the kernel falls back to one lane per pixel otherwise
    // (A15 env IS: the env shadow ray of every diffuse bounce is the side lane's job too)
    a.pair = (p->lanes_per_pixel == 2 || (p->lanes_per_pixel == 0 && (s->n_lights > 0 || a.env_is))) ? 1 : 0;
    // Refill: a wave leaves its traversal loop to shade once fewer than this many
    // lanes still traverse.  A shading pass costs ~5 node steps, so passes are
    // batched; in pair mode half the lanes (the side lanes) are mostly idle and
    // the threshold scales down with them (C3 1080p 4096 spp: 24 -> 5.88,
    // 8 -> 6.44, 2..12 within 6.2-6.6 Grays/s; C2 single-lane: 16-24 best).
    const bool pair_kernel = a.pair && (s->n_lights > 0 || a.env_is) && (s->n_materials + 1) < 0x7fff &&
                             !(p->flags & TPT_FLAG_REF_ORDER);
    // Four lanes per pixel ("Four lanes per ray"): every lane
    // of a quad runs the pixel's path, each 4-wide visit split over them -- the
    // one-lane kernel logic, so no delta lights, env IS or reference order, and the
    // quads' stacks in LDS.  Auto on launches with no more pixels than the chip's
    // resident lanes (s->resident_lanes, from the device: MI355X 256 CUs x 4 SIMDs x
    // 5 waves x 64 = 327,680), which are their heaviest tiles' serial chains:
    // strong-scaled C2 at N = 8 (259 K pixels per GPU, slowest rank) 314 -> 250 ms;
    // at N = 4 (518 K) four lanes lose (463 vs 328 ms: four times the waves), so
    // the chip is the bound.
    const double launch_pix = (double)W * (double)std::max(bh, 1) * (double)nf;
    const double resident = (double)s->resident_lanes;
    // (the wavefront variant has no lane modes: tpt.h, lanes_per_pixel is not used there)
    const bool wavefront = (p->flags & TPT_FLAG_WAVEFRONT) != 0;
    const bool quad_ok = !wavefront && p->lanes_per_pixel != 2 && s->n_lights == 0 && !a.env_is &&
                         !(p->flags & TPT_FLAG_REF_ORDER) && tpt::trace_quad_fits(a);
    if (p->lanes_per_pixel == 4 && !quad_ok && !wavefront)
        return fail(TPT_ERR_INVALID_ARG,
                    "lanes_per_pixel 4: scenes without delta lights, no env IS, ordered traversal, stacks in LDS");
    a.quad = (p->lanes_per_pixel == 4 || (p->lanes_per_pixel == 0 && launch_pix <= resident && quad_ok)) ? 1 : 0;
    // the trace grid's y extent is (band row blocks) x frames: 8-row workgroups in
    // pair mode, 16 otherwise (launch_trace)
    if (!wavefront) {
        const int wg_rows = (pair_kernel || a.quad) ? 8 : 16;
        if ((size_t)((bh + wg_rows - 1) / wg_rows) * nf > 65535)
            return fail(TPT_ERR_INVALID_ARG, "frame batch too large for one launch");
    }
    // A launch with fewer pixels than about twice the chip's resident lanes
    // (s->resident_lanes; strong-scaled frames, small images) is bound by its
    // heaviest waves' chains, not by throughput: batch the shading passes harder
    // (C2 rank 0 of 8: refill 24 318 ms, 4: 276 ms; rank 0 of 4: flat).
    const bool drained = launch_pix < 2.0 * resident;
    // Shallow trees (few triangles) make a traversal short against a shading
    // pass, so passes are batched harder there: tir (6 triangles) refill 16
    // 84.6 Grays/s vs 24 72.6-78.9; box (1,932) 16 = 24; C5 (131 K) 16 -3 %.
    const int full = s->n_faces <= 4096 ? 16 : 24;
    // Pair mode (round 3, after the 4-wave pair variants and the fp32-bounded env
    // lookup; C3 1080p 4096 spp, Mrays/s): refill 8 7,711, 6 7,720, 4 7,790-7,942,
    // 3 7,911-7,934, 2 7,860-7,983 -> 3; with env IS (the side lane's env sample
    // and shadow ray per diffuse bounce): 8 5,562-5,630, 4 5,745-5,803, 2
    // 5,934-5,970, 1 6,070-6,153 -> 1 (the wave shades only once no lane traverses).
    // Round 5, after the emitter-free pair variants (C3, 2 reps): 4 8,071 / 8,129,
    // 3 8,185 / 8,156, 2 8,223 / 8,260, 1 8,676 / 8,710 -> 1 without env IS too.
    a.refill = p->refill > 0 ? std::min(p->refill, 64) : (pair_kernel ? 1 : (drained ? 4 : full));
    a.drained = drained ? 1 : 0;   // latency-oriented kernel variants (trace.hip DRAIN)
    // Parked-leaf batch (speculative leaf postponement): a wave runs its triangle
    // tests once this many lanes are blocked on a parked leaf.  Pair mode has
    // half the path lanes and its heavy waves few traversing lanes, so it
    // batches less (C3 4096 spp: 4 -> 6.84, 2 -> 7.45, 8 -> 5.86 Grays/s;
    // C2, C4 and C5 within 2 % either way).
    // Drained launches likewise (strong-scaled C2, rank 0 of 8: 4 -> 259 ms, 2 -> 252 ms, 8 -> 277 ms).
    // Re-swept at the end of round 3 with the new pair refill (C3: 1 -> 7,988-8,092,
    // 2 -> 7,826-7,886, 3 -> 7,414-7,457 Mrays/s; C3 + IS: 1 -> 6,191-6,212,
    // 2 -> 6,111-6,133): 1 in pair mode.
    a.leaf_kb = p->leaf_batch > 0 ? std::min(p->leaf_batch, 64) : (pair_kernel ? 1 : (drained ? 2 : 4));
    // XCD runs (trace.hip k_trace prologue) for scenes that do not fit one XCD's
    // 4 MiB L2 (≈ 200 B of nodes, triangles and shading data per face): the
    // largest run length <= 10 that divides a row's tiles per XCD (C5 3840 px:
    // 10 +4.1 %, 30 +3.7 %, 5 +2.1 %, 3 +1.9 %).
    a.xcd_run = 0;
    a.xcd_rot = 0;
#ifndef TPT_XCD_RUNS_OFF   // (A/B builds: round-robin workgroups on every scene)
    if (s->n_faces > 16384) {
        const int gx = (W + 15) / 16, per = gx / 8;
        if (gx % 8 == 0)
            for (int g = std::min(per, 10); g >= 2 && a.xcd_run == 0; --g)
                if (per % g == 0) a.xcd_run = g;
    }
#endif
    a.rng = s->rng.p;
    a.accum = s->accum.p;
    a.counters = s->counters.p;
    // Launch schedule.  A launch ends in a tail where CUs drain: a wave's life
    // is its heaviest pixel's serial chain (samples run in order on one lane),
    // and the waves dispatched last (the top rows of the box) live ~40x longer
    // than the miss tiles -- measured on box at 256 spp, 25 % of the launch's
    // wave slots idle.  Default (spp >= 1024): the rows split into P = 3 interleaved band sets,
    // each on its own stream, and the spp into chunks, set k's chunk boundaries
    // offset by k/P of a chunk: while one set's launch drains, another set's
    // launch is mid-flight and takes the freed slots.  A pixel's samples still
    // run in order (its set's launches are stream-ordered, RNG and sums persist
    // between chunks), so the result is bit-identical to one launch.
    // params pipe_sets (1: one stream) and pipe_chunks (chunks per set) override;
    // an explicit spp_per_launch keeps the single-stream chunked loop.
    double trace_ms = 0.0, kernel_ms = 0.0;
    int launches = 0;
    const char* dbg_path = nullptr;
    size_t dbg_words = 0;
    if ((p->flags & TPT_FLAG_WAVEFRONT) && (p->flags & (TPT_FLAG_FAST | TPT_FLAG_APPROX_CULL)))
        return fail(TPT_ERR_INVALID_ARG, "TPT_FLAG_WAVEFRONT runs the exact traversal only");
    if (p->flags & TPT_FLAG_WAVEFRONT) {   // the wavefront / ray-queue variant (wavefront.hip)
        const tpt_status ws = render_wavefront(s, a, p, n_frames, bh, trace_ms, kernel_ms, launches);
        if (ws != TPT_OK) return ws;
    } else {
    int chunk = p->spp_per_launch;
    int nset = 1;
    if (chunk <= 0) {
        // one stream: chunk only past ~4096 spp of 1080p pixels so one launch stays below ~5 s
        const double band_pix = (double)W * (double)std::max(bh, 1) * (double)nf;
        chunk = (int)std::max(1.0, std::floor(4096.0 * 2073600.0 / band_pix));
        const bool forced = p->pipe_sets > 0;
        nset = forced ? p->pipe_sets : 3;
        // (pair mode: 16 -- C3 4096 spp, 256-spp chunks: 8,180 vs 8,016-8,032 Mrays/s with 8,
        // 7,743 with 4; C3 + IS 6,322 vs 6,206-6,267)
        const int per_set = p->pipe_chunks > 0 ? p->pipe_chunks : (pair_kernel ? 16 : 8);
        nset = std::max(1, std::min(nset, kMaxPipe));
        // worth it only with several chunks of real work and rows for every set
        if (bh < nset * band_rows) nset = 1;
        // chunks of at least 128 spp, and by default only from 1024 spp on
        // (measured on box 1080p, 3 sets: 1024 spp +6.7 %; 256 spp -2 %, 32-spp
        // chunks -4 %: concurrently running launches at different rows cost
        // locality, and every launch its prologue)
        // (both pipe_sets and pipe_chunks given: exactly that schedule, any chunk
        // size -- tests run the pipeline at full resolution and a few spp)
        const bool exact = forced && p->pipe_chunks > 0;
        const int min_chunk = exact ? 1 : kPipeMinChunk;
        if (nset > 1) chunk = std::min(chunk, std::max(min_chunk, (p->spp + per_set - 1) / per_set));
        if (!exact && p->spp < (forced ? 2 : 8) * kPipeMinChunk) nset = 1;
    }
    chunk = std::min(chunk, p->spp);
    struct Launch {
        int set, samples;
    };
    std::vector<Launch> plan;
    for (int k = 0; k < nset; ++k) {
        int done = 0;
        const int first = chunk - (k * chunk) / nset;   // set k starts k/nset of a chunk early
        for (int c = first; done < p->spp && bh > 0; c = chunk) {
            const int n = std::min(c, p->spp - done);
            plan.push_back({k, n});
            done += n;
        }
    }
    a.debug_waves = nullptr;
#if defined(TPT_PROFILE_PHASES) || defined(TPT_VERIFY_CULL)
    // per-wave dump (phase-profiling builds) / traversal mismatch log (cull-verification builds)
    dbg_path = std::getenv("TPT_DEBUG_WAVES");
#endif
    // one record per wave of the largest grid: 8x8-pixel workgroups (four lanes per
    // pixel; pair mode 16x8, one lane 16x16), 4 waves each, 8 words per wave
    const size_t dbg_launch =
        8ull * 4 * (size_t)((W + 7) / 8) * (size_t)((std::max(bh, 1) + 7) / 8) * nf;
    dbg_words = dbg_launch * std::max<size_t>(plan.size(), 1);   // one region per launch
    if (dbg_path) {
        HIP_OR_FAIL(s->debug.alloc(dbg_words));
        HIP_OR_FAIL(hipMemsetAsync(s->debug.p, 0, dbg_words * sizeof(unsigned long long), st));
    }
    HIP_OR_FAIL(s->ensure_launch_events(2 * plan.size()));
    // set k renders bands band_index + k * band_count of the band_count * nset
    // interleave; of an explicit deal, list entries k, k + nset, ... (a short last
    // band, last in the list, stays last in its set)
    int set_bh[kMaxPipe] = {bh};
    size_t set_off[kMaxPipe] = {0};
    for (int k = 0; k < nset; ++k) {
        if (nset == 1) break;
        if (listed) {
            std::vector<int32_t> sub;
            for (size_t i = (size_t)k; i < list.size(); i += (size_t)nset) sub.push_back(list[i]);
            set_bh[k] = rows_of(sub);
            set_off[k] = list.size();   // after the whole list, then the shares of sets 0 .. k-1
            for (int j = 0; j < k; ++j) set_off[k] += (list.size() + nset - 1 - j) / nset;
            std::copy(sub.begin(), sub.end(), s->band_lists_h.begin() + set_off[k]);
        } else {
            set_bh[k] = band_height_of(H, band_rows, band_count * nset, band_index + k * band_count);
        }
    }
    if (listed && nset > 1 && !list.empty())
        HIP_OR_FAIL(hipMemcpyAsync(s->band_lists.p + list.size(), s->band_lists_h.data() + list.size(),
                                   list.size() * sizeof(int32_t), hipMemcpyHostToDevice, st));   // (before the fork)
    hipStream_t qs[kMaxPipe] = {st};
    if (nset > 1) {
        HIP_OR_FAIL(s->ensure_pipe(nset));
        HIP_OR_FAIL(hipEventRecord(s->pipe_ev[0], st));   // fork: RNG init, the sums' reset, the sets' band lists are done
        for (int k = 0; k < nset; ++k) {
            qs[k] = s->pipe[k];
            HIP_OR_FAIL(hipStreamWaitEvent(qs[k], s->pipe_ev[0], 0));
        }
    }
    // issue the sets' launches interleaved in time order (chunk starts), so no
    // stream's queue runs ahead of the others on the host side
    std::vector<size_t> order(plan.size());
    {
        std::vector<double> t0(plan.size());
        double at[kMaxPipe] = {};
        for (size_t j = 0; j < plan.size(); ++j) {
            t0[j] = at[plan[j].set];
            at[plan[j].set] += plan[j].samples;
        }
        for (size_t j = 0; j < order.size(); ++j) order[j] = j;
        std::stable_sort(order.begin(), order.end(), [&](size_t x, size_t y) { return t0[x] < t0[y]; });
    }
    // An error while the sets' launches are being queued must not leave set
    // streams writing the rng/accumulator planes behind the caller's back (the
    // next call's reset runs on the main stream): join every set before failing.
#define SET_OR_FAIL(expr)                                                                                      \
    do {                                                                                                       \
        hipError_t e_ = (expr);                                                                                \
        if (e_ != hipSuccess) {                                                                                \
            for (int k_ = 0; nset > 1 && k_ < nset; ++k_) (void)hipStreamSynchronize(qs[k_]);                  \
            (void)hipStreamSynchronize(st);                                                                    \
            return fail(e_ == hipErrorOutOfMemory ? TPT_ERR_OOM : TPT_ERR_HIP,                                 \
                        std::string(#expr) + ": " + hipGetErrorString(e_));                                    \
        }                                                                                                      \
    } while (0)
    int set_chunks[kMaxPipe] = {};   // launches issued per set so far (XCD run rotation)
    for (size_t oi = 0; oi < order.size(); ++oi) {
        const size_t j = order[oi];
        const int k = plan[j].set;
        if (set_bh[k] <= 0) continue;
        tpt::TraceArgs ak = a;
        ak.samples = plan[j].samples;
        // XCD runs: chunk c of a set rotates the runs' XCDs by c (trace.hip prologue), so a
        // set whose few rows leave the per-launch rotation incomplete still spreads its heavy
        // columns over every XCD across its chunks
        ak.xcd_rot = TPT_XCD_ROT ? (set_chunks[k]++ & 7) : 0;
        if (nset > 1) {
            ak.band_count = band_count * nset;
            ak.band_index = band_index + k * band_count;
            ak.band_height = set_bh[k];
            if (listed) ak.band_list = s->band_lists.p + set_off[k];
        }
#ifdef TPT_VERIFY_CULL
        if (dbg_path) ak.debug_waves = s->debug.p;   // one log, counters[24] indexes it
#else
        if (dbg_path) ak.debug_waves = s->debug.p + oi * dbg_launch;
#endif
        SET_OR_FAIL(hipEventRecord(s->lev[2 * j], qs[k]));
        SET_OR_FAIL((p->flags & TPT_FLAG_FAST) ? tpt_fast::launch_trace_ptr(&ak, qs[k]) : tpt::launch_trace(ak, qs[k]));
        SET_OR_FAIL(hipEventRecord(s->lev[2 * j + 1], qs[k]));
    }
    for (int k = 0; nset > 1 && k < nset; ++k) {   // join
        SET_OR_FAIL(hipEventRecord(s->pipe_ev[1 + k], qs[k]));
        SET_OR_FAIL(hipStreamWaitEvent(st, s->pipe_ev[1 + k], 0));
    }
    SET_OR_FAIL(hipEventRecord(s->ev[2], st));   // end of the trace phase
    SET_OR_FAIL(hipEventSynchronize(s->ev[2]));
#undef SET_OR_FAIL
    {
        float ms = 0.0f;
        HIP_OR_FAIL(hipEventElapsedTime(&ms, s->ev[1], s->ev[2]));
        trace_ms = ms;   // wall time of the trace phase (overlapping launches counted once)
        for (size_t j = 0; j < plan.size(); ++j) {
            if (set_bh[plan[j].set] <= 0) continue;
            HIP_OR_FAIL(hipEventElapsedTime(&ms, s->lev[2 * j], s->lev[2 * j + 1]));
            kernel_ms += ms;
            ++launches;
        }
    }
    }   // launch plan (k_trace)

    // copyToFB (:553) + radiance readout, per frame
    HIP_OR_FAIL(hipEventRecord(s->ev[2], st));
    for (size_t f = 0; f < nf; ++f) {
        float* radiance_out = radiance_outs ? radiance_outs[f] : nullptr;
        uint8_t* bgra_out = bgra_outs ? bgra_outs[f] : nullptr;
        const bool rad_dev = is_device_ptr(radiance_out);
        const bool bgra_dev = is_device_ptr(bgra_out);
        tpt::ResolveArgs r{};
        r.accum = s->accum.p + f * 3 * npix;
        r.width = W;
        r.height = H;
        r.band_rows = band_rows;
        r.band_count = band_count;
        r.band_index = band_index;
        r.band_list = d_list;
        r.band_height = bh;
        r.spp = (int)total_spp;
        if (radiance_out) {
            if (rad_dev) {
                r.radiance = radiance_out;
            } else {
                HIP_OR_FAIL(s->radiance_tmp.alloc(3 * npix));
                HIP_OR_FAIL(hipMemcpyAsync(s->radiance_tmp.p, radiance_out, 3 * npix * sizeof(float),
                                           hipMemcpyHostToDevice, st));
                r.radiance = s->radiance_tmp.p;
            }
        }
        if (bgra_out) {
            if (bgra_dev) {
                r.bgra = bgra_out;
            } else {
                HIP_OR_FAIL(s->bgra_tmp.alloc(4 * npix));
                HIP_OR_FAIL(hipMemcpyAsync(s->bgra_tmp.p, bgra_out, 4 * npix, hipMemcpyHostToDevice, st));
                r.bgra = s->bgra_tmp.p;
            }
        }
        if (bh > 0 && (r.radiance || r.bgra)) HIP_OR_FAIL(tpt::launch_resolve(r, st));
        // host outputs share one staging buffer: copy back before the next frame reuses it
        if (radiance_out && !rad_dev)
            HIP_OR_FAIL(hipMemcpyAsync(radiance_out, s->radiance_tmp.p, 3 * npix * sizeof(float),
                                       hipMemcpyDeviceToHost, st));
        if (bgra_out && !bgra_dev)
            HIP_OR_FAIL(hipMemcpyAsync(bgra_out, s->bgra_tmp.p, 4 * npix, hipMemcpyDeviceToHost, st));
    }
    HIP_OR_FAIL(hipEventRecord(s->ev[3], st));
    unsigned long long cnt[32] = {0};
    HIP_OR_FAIL(hipMemcpyAsync(cnt, s->counters.p, sizeof cnt, hipMemcpyDeviceToHost, st));
    HIP_OR_FAIL(hipStreamSynchronize(st));
    if (cnt[4] != 0) return fail(TPT_ERR_HIP, "traversal stack overflow (BVH deeper than sized)");
    if (p->band_cost) {   // per band this call rendered: its waves' summed life, in microseconds
        s->band_cost_h.resize((size_t)n_bands);
        HIP_OR_FAIL(hipMemcpy(s->band_cost_h.data(), s->band_cost.p, (size_t)n_bands * sizeof(unsigned long long),
                              hipMemcpyDeviceToHost));
        for (int b = 0; b < n_bands; ++b) {
            const bool mine = listed ? std::find(list.begin(), list.end(), b) != list.end()
                                     : b % band_count == band_index;
            if (mine) p->band_cost[b] = (float)((double)s->band_cost_h[(size_t)b] / 100.0);   // 100-MHz ticks
        }
    }
    if (dbg_path) {
#ifdef TPT_VERIFY_CULL
        const size_t dump_words = std::min<size_t>(dbg_words, 16 * std::min<unsigned long long>(cnt[24], 4096));
#else
        const size_t dump_words = dbg_words;
#endif
        std::vector<unsigned long long> h(dump_words);
        if (dump_words)
            HIP_OR_FAIL(hipMemcpy(h.data(), s->debug.p, dump_words * sizeof(unsigned long long), hipMemcpyDeviceToHost));
        if (FILE* f = std::fopen(dbg_path, "wb")) {
            std::fwrite(h.data(), sizeof(unsigned long long), h.size(), f);
            std::fclose(f);
        }
    }
#if defined(TPT_PROFILE_PHASES) || defined(TPT_VERIFY_CULL)
    if (std::getenv("TPT_DEBUG_COUNTERS")) {   // raw kernel counters (TPT_PROFILE_PHASES builds: 6..15 phases, 16..22 shading-pass sections)
        std::fprintf(stderr, "tpt counters:");
        for (int i = 0; i < 32; ++i) std::fprintf(stderr, " %llu", cnt[i]);
        std::fprintf(stderr, "\n");
    }
#endif
    if (stats) {
        std::memset(stats, 0, sizeof *stats);
        stats->traversals = cnt[0];
        stats->internal_visits = cnt[1];
        stats->wide_visits = cnt[5];
        stats->local_rays = cnt[9];
        stats->accumulated_spp = total_spp;
        stats->leaf_tests = cnt[2];
        stats->shade_hits = cnt[3];
        stats->pixels = (uint64_t)W * (uint64_t)bh * (uint64_t)nf;
        stats->samples = stats->pixels * (uint64_t)p->spp;
        float ms = 0.0f;
        (void)hipEventElapsedTime(&ms, s->ev[0], s->ev[1]);
        stats->rng_init_ms = ms;
        stats->trace_ms = trace_ms;
        stats->trace_kernel_ms = kernel_ms;
        stats->tree_wait_ms = tree_wait_ms;
        (void)hipEventElapsedTime(&ms, s->ev[2], s->ev[3]);
        stats->resolve_ms = ms;
        stats->trace_launches = launches;
        stats->resident_lanes = s->resident_lanes;
        stats->lanes_per_pixel = a.quad ? 4 : (pair_kernel ? 2 : 1);
        stats->drained = a.drained;
        stats->total_ms =
            std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_start).count();
    }
    // the persisted streams and sums now belong to this batch: a following
    // TPT_FLAG_ACCUMULATE call with the same frames continues them
    s->acc_valid = true;
    s->acc_w = W;
    s->acc_h = H;
    s->acc_rows = band_rows;
    s->acc_count = band_count;
    s->acc_index = band_index;
    s->acc_list = list;
    s->acc_seeds = fseeds;
    s->acc_spp = total_spp;
    return TPT_OK;
}

tpt_status tpt_scene_read_bvh(tpt_scene* s, void* nodes36, int64_t* keys) {
    if (!s || !s->built) return fail(TPT_ERR_INVALID_ARG, "scene not built");
    DeviceGuard g(s->device);
    const size_t n = (size_t)s->n_faces;
    if (nodes36) HIP_OR_FAIL(hipMemcpy(nodes36, s->nodes36.p, 36 * (2 * n - 1), hipMemcpyDeviceToHost));
    if (keys) HIP_OR_FAIL(hipMemcpy(keys, s->keys_sorted.p, 8 * n, hipMemcpyDeviceToHost));
    return TPT_OK;
}

tpt_status tpt_scene_read_world(tpt_scene* s, float* wv, float* wn) {
    if (!s || !s->built) return fail(TPT_ERR_INVALID_ARG, "scene not built");
    DeviceGuard g(s->device);
    const size_t nv = (size_t)s->n_vertices;
    if (wv) HIP_OR_FAIL(hipMemcpy(wv, s->wverts.p, 12 * nv, hipMemcpyDeviceToHost));
    if (wn) HIP_OR_FAIL(hipMemcpy(wn, s->wnorms.p, 12 * nv, hipMemcpyDeviceToHost));
    return TPT_OK;
}

tpt_status tpt_debug_rng_init(int device, uint64_t seed, uint64_t first, uint32_t n, uint32_t* states) {
    if (!states && n) return fail(TPT_ERR_INVALID_ARG, "null output");
    int ndev = tpt_device_count();
    if (ndev <= 0) return fail(TPT_ERR_NO_DEVICE, "no HIP device available");
    if (device < 0 || device >= ndev) return fail(TPT_ERR_INVALID_ARG, "bad device index");
    DeviceGuard g(device);
    DevBuf<uint32_t> jumps, out;
    const auto& hj = host_jumps();
    HIP_OR_FAIL(jumps.upload(hj.data(), hj.size(), nullptr));
    HIP_OR_FAIL(out.alloc(6 * (size_t)std::max(n, 1u)));
    HIP_OR_FAIL(tpt::launch_rng_init_linear(jumps.p, seed, first, n, out.p, nullptr));
    HIP_OR_FAIL(hipDeviceSynchronize());
    if (n) HIP_OR_FAIL(hipMemcpy(states, out.p, 24 * (size_t)n, hipMemcpyDeviceToHost));
    return TPT_OK;
}

tpt_status tpt_debug_trace_rays(tpt_scene* s, uint32_t n, const float* o, const float* d, const int32_t* origin_fid,
                                int32_t mode, int32_t* hit, float* t, float* uv) {
    if (!s || !s->built) return fail(TPT_ERR_INVALID_ARG, "scene not built");
    if (mode < 0 || mode > 3) return fail(TPT_ERR_INVALID_ARG, "unknown trace mode");
    {
        const tpt_status bs = finish_pending(s);
        if (bs != TPT_OK) return bs;
    }
    if (n && (!o || !d || !hit || !t || !uv)) return fail(TPT_ERR_INVALID_ARG, "null argument");
    DeviceGuard g(s->device);
    DevBuf<float> dorg, ddir, dt, duv;
    DevBuf<int32_t> dhit, dofid;
    HIP_OR_FAIL(dorg.upload(o, 3 * (size_t)n, s->stream));
    if (origin_fid) {
        for (uint32_t i = 0; i < n; ++i)
            if (origin_fid[i] >= s->n_faces) return fail(TPT_ERR_INVALID_ARG, "origin face out of range");
        HIP_OR_FAIL(dofid.upload(origin_fid, n, s->stream));
    }
    HIP_OR_FAIL(ddir.upload(d, 3 * (size_t)n, s->stream));
    HIP_OR_FAIL(dhit.alloc(n));
    HIP_OR_FAIL(dt.alloc(n));
    HIP_OR_FAIL(duv.alloc(2 * (size_t)n));
    tpt::TraceArgs a{};
    fill_trace_args(s, nullptr, nullptr, a);
    HIP_OR_FAIL(tpt::launch_trace_rays(a, n, dorg.p, ddir.p, origin_fid ? dofid.p : nullptr, mode, dhit.p, dt.p, duv.p,
                                       s->stream));
    HIP_OR_FAIL(hipStreamSynchronize(s->stream));
    if (n) {
        HIP_OR_FAIL(hipMemcpy(hit, dhit.p, 4 * (size_t)n, hipMemcpyDeviceToHost));
        HIP_OR_FAIL(hipMemcpy(t, dt.p, 4 * (size_t)n, hipMemcpyDeviceToHost));
        HIP_OR_FAIL(hipMemcpy(uv, duv.p, 8 * (size_t)n, hipMemcpyDeviceToHost));
    }
    return TPT_OK;
}

tpt_status tpt_debug_step_latency(tpt_scene* s, uint32_t n, const float* o, const float* d, int32_t mode,
                                  int32_t flags, uint64_t* out) {
    if (!s || !s->built) return fail(TPT_ERR_INVALID_ARG, "scene not built");
    if (n > 64 || (n && (!o || !d || !out))) return fail(TPT_ERR_INVALID_ARG, "1..64 rays and outputs");
    if (mode < 0 || mode > 2)
        return fail(TPT_ERR_INVALID_ARG, "mode: 0 nodes in global memory, 1 in LDS, 2 four lanes per ray");
    if (mode == 2 && n > 16) return fail(TPT_ERR_INVALID_ARG, "four lanes per ray: at most 16 rays");
    {
        const tpt_status bs = finish_pending(s);
        if (bs != TPT_OK) return bs;
    }
    const int nodes_lds = mode == 1 ? s->n4 : (mode == 2 ? -1 : 0);
    if ((size_t)std::max(nodes_lds, 0) * 128 + 64 * 256 * sizeof(int) > 160 * 1024)
        return fail(TPT_ERR_INVALID_ARG, "the 4-wide tree does not fit in LDS");
    DeviceGuard g(s->device);
    DevBuf<float> dorg, ddir;
    DevBuf<unsigned long long> dout;
    HIP_OR_FAIL(dorg.upload(o, 3 * (size_t)std::max(n, 1u), s->stream));
    HIP_OR_FAIL(ddir.upload(d, 3 * (size_t)std::max(n, 1u), s->stream));
    HIP_OR_FAIL(dout.alloc(4 * 64));
    tpt::TraceArgs a{};
    fill_trace_args(s, nullptr, nullptr, a);
    if (mode == 2 && a.stack_depth + 3 > 64) return fail(TPT_ERR_INVALID_ARG, "four lanes per ray: stack too deep");
    if (flags & TPT_FLAG_FAST) {   // the tolerance-mode build, without the culling guards
        a.cull_eps = 0.0f;
        a.n_sliver_groups = 0;
        a.graze = 0;
        HIP_OR_FAIL(tpt_fast::launch_step_latency_ptr(&a, n, dorg.p, ddir.p, nodes_lds, dout.p, s->stream));
    } else {
        HIP_OR_FAIL(tpt::launch_step_latency_ptr(&a, n, dorg.p, ddir.p, nodes_lds, dout.p, s->stream));
    }
    HIP_OR_FAIL(hipStreamSynchronize(s->stream));
    HIP_OR_FAIL(hipMemcpy(out, dout.p, 4 * 64 * sizeof(unsigned long long), hipMemcpyDeviceToHost));
    return TPT_OK;
}

tpt_status tpt_debug_hot_kat(int device, int32_t op, uint32_t n, const float* in, float* out) {
    static const int kIn[4] = {12, 15, 16, 3}, kOut[4] = {2, 4, 6, 3};
    if (op < 0 || op > 3) return fail(TPT_ERR_INVALID_ARG, "unknown KAT op");
    if (n && (!in || !out)) return fail(TPT_ERR_INVALID_ARG, "null argument");
    int ndev = tpt_device_count();
    if (ndev <= 0) return fail(TPT_ERR_NO_DEVICE, "no HIP device available");
    if (device < 0 || device >= ndev) return fail(TPT_ERR_INVALID_ARG, "bad device index");
    DeviceGuard g(device);
    DevBuf<float> din, dout;
    HIP_OR_FAIL(din.upload(in, (size_t)kIn[op] * n, nullptr));
    HIP_OR_FAIL(dout.alloc((size_t)kOut[op] * std::max(n, 1u)));
    HIP_OR_FAIL(tpt::launch_hot_kat(op, n, din.p, dout.p, nullptr));
    HIP_OR_FAIL(hipDeviceSynchronize());
    if (n) HIP_OR_FAIL(hipMemcpy(out, dout.p, sizeof(float) * kOut[op] * (size_t)n, hipMemcpyDeviceToHost));
    return TPT_OK;
}

tpt_status tpt_gltf_load(const char* path, tpt_gltf** out) {
    if (!path || !out) return fail(TPT_ERR_INVALID_ARG, "null argument");
    *out = nullptr;
    tpt_gltf* g = new (std::nothrow) tpt_gltf();
    if (!g) return fail(TPT_ERR_OOM, "host allocation failed");
    try {
        tpt::load_gltf(path, g->hs);
    } catch (const tpt::io_error& e) {
        delete g;
        return fail(TPT_ERR_IO, e.what());
    } catch (const std::exception& e) {
        delete g;
        return fail(TPT_ERR_PARSE, e.what());
    }
    *out = g;
    return TPT_OK;
}

tpt_status tpt_gltf_desc(const tpt_gltf* g, tpt_scene_desc* d, tpt_camera* cam) {
    if (!g || !d) return fail(TPT_ERR_INVALID_ARG, "null argument");
    const tpt::HostScene& h = g->hs;
    d->indices = h.indices.data();
    d->n_faces = (uint32_t)(h.indices.size() / 3);
    d->vertices = h.vertices.data();
    d->normals = h.normals.data();
    d->n_vertices = (uint32_t)(h.vertices.size() / 3);
    d->lut = h.lut.data();
    d->n_objects = (uint32_t)h.lut.size();
    d->vert_trans = h.vert_trans.data();
    d->normal_trans = h.normal_trans.data();
    d->materials = h.materials.empty() ? nullptr : h.materials.data();
    d->n_materials = (uint32_t)h.materials.size();
    d->lights = h.lights.empty() ? nullptr : h.lights.data();
    d->n_lights = (uint32_t)h.lights.size();
    d->flags = 0;
    if (cam) *cam = h.camera;
    return TPT_OK;
}

int tpt_gltf_missing_material(const tpt_gltf* g) { return g && g->hs.missing_material ? 1 : 0; }

void tpt_gltf_free(tpt_gltf* g) { delete g; }

}  // extern "C"
