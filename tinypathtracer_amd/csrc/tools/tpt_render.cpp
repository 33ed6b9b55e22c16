// tpt_render -- headless replacement for the reference's main.cu + Vulkan
// display loop (src/main.cu:6-14, src/vkEngine.cu:180-302): renders one glTF
// scene through the C++ host API (tpt.hpp) and writes the framebuffer as PPM
// (8-bit, copyToFB's truncating tone map) and the radiance as PFM (fp32).
//
//   tpt_render scene.gltf [--width W] [--height H] [--spp N] [--depth D]
//              [--seed S] [--env equirect.jpg|.ppm|--sky] [--out prefix] [--device i]
//              [--frames F [--progressive]]
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iostream>
#include <string>
#include <vector>

#include "tpt.hpp"

namespace {

// Deterministic procedural sky (stand-in for the missing kloppenheim_07 env,
// SURVEY 8(d) C3); same formula as tinypathtracer_amd.procedural_sky.
std::vector<uint8_t> procedural_sky(int w, int h) {
    std::vector<uint8_t> img((size_t)w * h * 4);
    for (int y = 0; y < h; ++y) {
        const double theta = (y + 0.5) / h * M_PI;
        const double elev = std::cos(theta);
        const double sky = elev > 0 ? elev : 0.0, ground = elev < 0 ? -elev : 0.0;
        for (int x = 0; x < w; ++x) {
            const double phi = (x + 0.5) / w * 2.0 * M_PI;
            const double sun = std::exp(-((theta - 0.9) * (theta - 0.9) + (std::cos(phi) - 1.0) * (std::cos(phi) - 1.0)) * 40.0);
            const double c[3] = {0.45 + 0.25 * sky - 0.25 * ground + 0.5 * sun,
                                 0.55 + 0.25 * sky - 0.30 * ground + 0.45 * sun,
                                 0.75 + 0.20 * sky - 0.45 * ground + 0.30 * sun};
            for (int k = 0; k < 3; ++k) {
                double v = c[k] * 255.0;
                v = v < 0 ? 0 : (v > 255 ? 255 : v);
                img[((size_t)y * w + x) * 4 + k] = (uint8_t)v;
            }
            img[((size_t)y * w + x) * 4 + 3] = 255;
        }
    }
    return img;
}

}  // namespace

int main(int argc, char** argv) {
    if (argc < 2) {
        std::fprintf(stderr, "usage: %s scene.gltf [--width W] [--height H] [--spp N] [--depth D] [--seed S] "
                             "[--env file.jpg|file.ppm | --sky] [--out prefix] [--device i] [--frames F [--progressive]]\n", argv[0]);
        return 2;
    }
    std::string scene_file = argv[1], env_file, out = "out";
    int W = 1920, H = 1080, spp = 64, depth = 8, device = 0, frames = 1;
    bool progressive = false;
    uint64_t seed = 0;
    bool sky = false;
    for (int i = 2; i < argc; ++i) {
        std::string a = argv[i];
        auto next = [&]() -> std::string {
            if (i + 1 >= argc) throw std::runtime_error("missing value for " + a);
            return argv[++i];
        };
        if (a == "--width") W = std::stoi(next());
        else if (a == "--height") H = std::stoi(next());
        else if (a == "--spp") spp = std::stoi(next());
        else if (a == "--depth") depth = std::stoi(next());
        else if (a == "--seed") seed = std::stoull(next());
        else if (a == "--env") env_file = next();
        else if (a == "--sky") sky = true;
        else if (a == "--out") out = next();
        else if (a == "--device") device = std::stoi(next());
        else if (a == "--frames") frames = std::stoi(next());
        else if (a == "--progressive") progressive = true;
        else { std::fprintf(stderr, "unknown option %s\n", a.c_str()); return 2; }
    }
    try {
        tpt::EnvLight env;
        if (!env_file.empty()) {
            env = tpt::EnvLight(env_file, device);   // JPEG / PPM, decoded natively (tpt_env_load)
        } else if (sky) {
            auto img = procedural_sky(2048, 1024);
            env = tpt::EnvLight(img.data(), 2048, 1024, device);
        }
        tpt::PathTracer pt(env, W, H, device);
        tpt::Frame f = pt.render(scene_file, spp, seed, depth, frames, progressive);
        std::ofstream ppm(out + ".ppm", std::ios::binary);
        ppm << "P6\n" << W << " " << H << "\n255\n";
        for (size_t i = 0; i < (size_t)W * H; ++i) {   // BGRA -> RGB, rows already top-down
            const char px[3] = {(char)f.bgra[4 * i + 2], (char)f.bgra[4 * i + 1], (char)f.bgra[4 * i]};
            ppm.write(px, 3);
        }
        std::ofstream pfm(out + ".pfm", std::ios::binary);   // PFM rows are bottom-up, like the radiance
        pfm << "PF\n" << W << " " << H << "\n-1.0\n";
        pfm.write((const char*)f.radiance.data(), (std::streamsize)(f.radiance.size() * sizeof(float)));
        const tpt_stats& s = f.stats;
        std::printf("{\"scene\": \"%s\", \"width\": %d, \"height\": %d, \"spp\": %llu, \"rays\": %llu, "
                    "\"trace_ms\": %.3f, \"mrays_per_s\": %.1f, \"out\": \"%s.ppm\"}\n",
                    scene_file.c_str(), W, H, (unsigned long long)s.accumulated_spp, (unsigned long long)s.traversals,
                    s.trace_ms,
                    s.trace_ms > 0 ? s.traversals / (s.trace_ms * 1e3) : 0.0, out.c_str());
    } catch (const std::exception& e) {
        std::cerr << e.what() << std::endl;   // render() prints and returns (path_tracer.cu:575-578)
        return 1;
    }
    return 0;
}
