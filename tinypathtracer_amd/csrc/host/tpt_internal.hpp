// tpt_internal.hpp -- library internals shared by the host API and kernels.
#pragma once

#include <array>
#include <cstdint>
#include <memory>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "tpt.h"

namespace tpt {

struct io_error : std::runtime_error {
    using std::runtime_error::runtime_error;
};
struct parse_error : std::runtime_error {
    using std::runtime_error::runtime_error;
};

// Material() defaults (include/material.h:88-103)
inline tpt_material default_material() {
    tpt_material m{};
    m.base_color[0] = 0.82f; m.base_color[1] = 0.67f; m.base_color[2] = 0.16f;
    m.emission_factor = 0.0f; m.eta = 0.0f; m.metallic = 0.0f; m.subsurface = 0.0f;
    m.specular = 0.5f; m.roughness = 0.5f; m.specular_tint = 0.0f; m.anisotropic = 0.0f;
    m.sheen = 0.0f; m.sheen_tint = 0.0f; m.clearcoat = 0.0f; m.clearcoat_gloss = 1.0f;
    return m;
}

// Host scene produced by the glTF loader (the content of Scene + DeviceScene).
struct HostScene {
    std::vector<uint32_t> indices;
    std::vector<float> vertices, normals;
    std::vector<tpt_interval> lut;
    std::vector<float> vert_trans, normal_trans;
    std::vector<tpt_material> materials;
    std::vector<tpt_light> lights;
    tpt_camera camera{};
    bool missing_material = false;
};

void load_gltf(const std::string& path, HostScene& hs);

// Env-map image (JPEG / binary PPM) decoded as FreeImage + Texture would hand it
// to the GPU: RGBA8, row 0 = bottom, RGB order, alpha 255 (image.cpp).
void load_image(const std::string& path, std::vector<uint8_t>& rgba, int& w, int& h);

// SAH 4-wide traversal tree over (a subset of) the LBVH's exact leaf boxes
// (wide_bvh.cpp): 32 floats per node in the inner4 layout; returns the node count.
// A host vector whose resize leaves new elements uninitialised (the writer
// fills every one), so a 6-MB tree buffer is not zero-filled first.
template <class T>
struct NoInitAlloc : std::allocator<T> {
    template <class U>
    struct rebind {
        using other = NoInitAlloc<U>;
    };
    NoInitAlloc() noexcept = default;
    template <class U>
    NoInitAlloc(const NoInitAlloc<U>&) noexcept {}
    template <class U>
    void construct(U* p) noexcept {
        ::new ((void*)p) U;
    }
    template <class U, class... A>
    void construct(U* p, A&&... a) {
        ::new ((void*)p) U(std::forward<A>(a)...);
    }
};
using HostFloats = std::vector<float, NoInitAlloc<float>>;

// The build's work arrays (≈ 30 MB for 131 K leaves), kept between the builds
// of a scene: a fresh allocation is first touched page by page every frame.
struct WideWorkspace {
    struct Impl;
    std::unique_ptr<Impl> impl;
    WideWorkspace();
    ~WideWorkspace();
    WideWorkspace(const WideWorkspace&) = delete;
    WideWorkspace& operator=(const WideWorkspace&) = delete;
};

struct WideParams {
    int sweep_max = 32;    // SAH ranges up to this size use an exact sweep, larger ones 32 bins
    int threads = -1;      // build threads: < 0 the usable cores (affinity, cgroup quota); 0, 1 serial
    WideWorkspace* ws = nullptr;   // reused work arrays (nullptr: the build's own); one build at a time
};
int usable_cores();
int build_wide_sah(const std::vector<int>& pos, const float* leaf_box, const uint32_t* leaf_emit, int leaf_base,
                   int id_base, HostFloats& out, int* stack_need, const WideParams& prm);

}  // namespace tpt

struct tpt_gltf {
    tpt::HostScene hs;
};
