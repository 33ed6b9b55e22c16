// tpt.hpp -- C++ host API over the C-ABI (tpt.h), mirroring the reference's
// PathTracer / Scene / BVH / Camera classes:
//   include/path_tracer.h:16-35   PathTracer(), PathTracer(envFile), render(meshFile)
//   include/mesh.cuh:98-115       Scene(file, "gltf"), copySceneToDevice(), m_camera
//   include/bvh.cuh:60-68         BVH(size), construct(...), m_nodes, m_keys
//   include/camera.h:9-65         getVFov / getAspRatio / getNearPlane
// Errors throw std::runtime_error, as the reference's CUDA_CHECK and loader do
// (include/intellisense_cuda.h:14-20, src/mesh.cu:76,94,303).  Header-only:
// link against libtpt.so.
#pragma once

#include <cstdint>
#include <cstring>
#include <ctime>
#include <functional>
#include <memory>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "tpt.h"

namespace tpt {

inline void check(tpt_status st) {
    if (st != TPT_OK) throw std::runtime_error(std::string("tpt: ") + tpt_last_error());
}

struct Camera {
    tpt_camera c{};
    float getVFov() const { return c.vfov; }
    float getAspRatio() const { return c.aspect; }
    float getNearPlane() const { return c.znear; }
};

// BVHNode (include/bvh.cuh:52-58): 36 bytes
struct BVHNode {
    uint32_t parent;
    int32_t a, b;       // internal: left/right child; leaf: fid, placeHolder
    float bmin[3], bmax[3];
};
static_assert(sizeof(BVHNode) == 36, "BVHNode layout");

class DeviceScene;

class Scene {
public:
    Scene(const std::string& filename, const std::string& type) {
        if (type != "gltf") throw std::runtime_error("Unsupported file format. Only support .gltf file.");
        tpt_gltf* g = nullptr;
        check(tpt_gltf_load(filename.c_str(), &g));
        gltf_.reset(g);
        check(tpt_gltf_desc(gltf_.get(), &desc_, &m_camera.c));
    }
    DeviceScene copySceneToDevice(int device = 0) const;
    const tpt_scene_desc& desc() const { return desc_; }
    bool missingMaterial() const { return tpt_gltf_missing_material(gltf_.get()) != 0; }

    Camera m_camera;

private:
    struct Free {
        void operator()(tpt_gltf* g) const { tpt_gltf_free(g); }
    };
    std::unique_ptr<tpt_gltf, Free> gltf_;
    tpt_scene_desc desc_{};
};

class DeviceScene {
public:
    DeviceScene(const tpt_scene_desc& d, int device) : n_faces_(d.n_faces), n_vertices_(d.n_vertices) {
        tpt_scene* s = nullptr;
        check(tpt_scene_create(&d, device, &s));
        scene_.reset(s);
    }
    // World transform + LBVH on the device (path_tracer.cu:536-542)
    DeviceScene& build() {
        check(tpt_scene_build(scene_.get()));
        built_ = true;
        return *this;
    }
    bool built() const { return built_; }
    tpt_scene* handle() const { return scene_.get(); }
    uint32_t nFaces() const { return n_faces_; }
    uint32_t nVertices() const { return n_vertices_; }

private:
    struct Free {
        void operator()(tpt_scene* s) const { tpt_scene_destroy(s); }
    };
    std::unique_ptr<tpt_scene, Free> scene_;
    uint32_t n_faces_, n_vertices_;
    bool built_ = false;
};

inline DeviceScene Scene::copySceneToDevice(int device) const { return DeviceScene(desc_, device); }

struct BVH {
    BVH() = default;
    explicit BVH(size_t size) : m_nodes(size ? 2 * size - 1 : 0), m_keys(size) {}
    // Builds on the device and reads back the reference node array.
    void construct(DeviceScene& scene) {
        if (!scene.built()) scene.build();
        m_nodes.resize(2 * (size_t)scene.nFaces() - 1);
        m_keys.resize(scene.nFaces());
        check(tpt_scene_read_bvh(scene.handle(), m_nodes.data(), m_keys.data()));
    }
    std::vector<BVHNode> m_nodes;
    std::vector<int64_t> m_keys;
};

class EnvLight {
public:
    EnvLight() = default;
    // rgba: width*height*4, row 0 = top (image order); stored bottom-up like
    // FreeImage (picture.h:41-43).
    EnvLight(const uint8_t* rgba_top_down, int width, int height, int device = 0) {
        std::vector<uint8_t> flipped((size_t)width * height * 4);
        for (int y = 0; y < height; ++y)
            std::memcpy(&flipped[(size_t)y * width * 4], rgba_top_down + (size_t)(height - 1 - y) * width * 4,
                        (size_t)width * 4);
        tpt_env* e = nullptr;
        check(tpt_env_create(flipped.data(), width, height, device, &e));
        env_.reset(e, Free());
    }
    // EnvLight(file) (env_light.cuh:8-18): JPEG or binary PPM decoded natively
    // as FreeImage would (tpt_env_load); throws std::runtime_error like Picture.
    explicit EnvLight(const std::string& file, int device = 0) {
        tpt_env* e = nullptr;
        check(tpt_env_load(file.c_str(), device, &e));
        env_.reset(e, Free());
    }
    const tpt_env* handle() const { return env_.get(); }

private:
    struct Free {
        void operator()(tpt_env* e) const { tpt_env_destroy(e); }
    };
    std::shared_ptr<tpt_env> env_;
    friend class PathTracer;
};

struct Frame {
    int width = 0, height = 0;
    std::vector<uint8_t> bgra;     // row 0 = top (copyToFB layout), B,G,R,A
    std::vector<float> radiance;   // row 0 = bottom, color / spp
    tpt_stats stats{};
};

class PathTracer {
public:
    PathTracer() : PathTracer(1920, 1080) {}   // VkEngine default extent (vkEngine.h:24)
    PathTracer(int width, int height, int device = 0) : m_width(width), m_height(height), device_(device) {}
    explicit PathTracer(const EnvLight& env, int width = 1920, int height = 1080, int device = 0)
        : m_width(width), m_height(height), device_(device), envLight(env) {}

    // doTrace (path_tracer.cu:491-554): one frame into a caller framebuffer
    // (host or device pointer, W*H*4 BGRA).  seed 0 -> time(), as the reference.
    // accumulate: progressive rendering (TPT_FLAG_ACCUMULATE) -- continue the
    // previous call's samples for the same frame instead of starting afresh
    // (the reference re-renders fresh samples every frame, vkEngine.cu:244).
    tpt_stats doTrace(DeviceScene& scene, const Camera& camera, uint8_t* framebuffer, int nSamplesPerPixel,
                      uint64_t seed = 0, int max_depth = 8, float* radiance = nullptr,
                      int band_count = 1, int band_index = 0, bool accumulate = false) {
        if (!scene.built()) scene.build();
        tpt_params p{};
        p.width = m_width;
        p.height = m_height;
        p.spp = nSamplesPerPixel;
        p.max_depth = max_depth;
        p.seed = seed ? seed : (accumulate && last_seed_ ? last_seed_ : (uint64_t)std::time(nullptr));
        last_seed_ = p.seed;
        p.band_rows = 16;
        p.band_count = band_count;
        p.band_index = band_index;
        p.flags = accumulate ? TPT_FLAG_ACCUMULATE : 0;
        tpt_stats st{};
        check(tpt_render(scene.handle(), envLight.handle(), &camera.c, &p, radiance, framebuffer, &st));
        return st;
    }

    // A batch of independent frames (seeds[f]) in one trace launch
    // (tpt_render_frames); frame f equals doTrace with seed seeds[f].
    tpt_stats doTraceFrames(DeviceScene& scene, const Camera& camera, const std::vector<uint64_t>& seeds,
                            const std::vector<uint8_t*>& framebuffers, int nSamplesPerPixel, int max_depth = 8,
                            const std::vector<float*>& radiances = {}, int band_count = 1, int band_index = 0) {
        if (!scene.built()) scene.build();
        const size_t n = seeds.size();
        if ((!framebuffers.empty() && framebuffers.size() != n) || (!radiances.empty() && radiances.size() != n))
            throw std::runtime_error("doTraceFrames: need one output buffer per frame");
        tpt_params p{};
        p.width = m_width;
        p.height = m_height;
        p.spp = nSamplesPerPixel;
        p.max_depth = max_depth;
        p.band_rows = 16;
        p.band_count = band_count;
        p.band_index = band_index;
        tpt_stats st{};
        check(tpt_render_frames(scene.handle(), envLight.handle(), &camera.c, &p, (int32_t)n, seeds.data(),
                                radiances.empty() ? nullptr : radiances.data(),
                                framebuffers.empty() ? nullptr : framebuffers.data(), &st));
        return st;
    }

    // render(meshFile) (path_tracer.cu:556-579), headless: the reference loops
    // frames in a window; this renders `frames` frames and returns the last --
    // with progressive = true each frame adds its samples to the previous ones.
    Frame render(const std::string& meshFile, int nSamplesPerPixel = 64, uint64_t seed = 0, int max_depth = 8,
                 int frames = 1, bool progressive = false) {
        Scene scene(meshFile, "gltf");
        DeviceScene d = scene.copySceneToDevice(device_);
        d.build();
        Frame f;
        f.width = m_width;
        f.height = m_height;
        f.bgra.assign((size_t)m_width * m_height * 4, 255);
        f.radiance.assign((size_t)m_width * m_height * 3, 0.0f);
        for (int i = 0; i < frames; ++i)
            f.stats = doTrace(d, scene.m_camera, f.bgra.data(), nSamplesPerPixel, seed, max_depth, f.radiance.data(),
                              1, 0, progressive && i > 0);
        return f;
    }

    int m_width, m_height;

private:
    int device_;
    uint64_t last_seed_ = 0;
    EnvLight envLight;
};

}  // namespace tpt
