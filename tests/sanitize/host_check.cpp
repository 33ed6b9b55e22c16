// host_check.cpp -- CPU-only driver of the host parsers and the wide-tree
// builder for the sanitizer build (tests/sanitize/Makefile, SURVEY.md section 5
// "CPU restatement under ASan/UBSan").  Never built for or run on the GPU box.
//
//   host_check gltf FILE...   load_gltf (host/gltf.cpp, json_lite.hpp)
//   host_check image FILE...  load_image (host/image.cpp: JPEG / PPM)
//   host_check wide N SEED    build_wide_sah (host/wide_bvh.cpp) on N random leaf boxes
//
// Prints one line per input: "ok", or "error: <message>" for a parse error
// (the library's exception, which tpt_gltf_load / tpt_env_load turn into a
// status).  Any memory error or undefined behaviour aborts with the
// sanitizer's report instead.
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <exception>
#include <random>
#include <string>
#include <vector>

#include "tpt_internal.hpp"

static int check_wide(int n, unsigned seed, int threads) {
    std::mt19937 rng(seed);
    std::uniform_real_distribution<float> u(-10.0f, 10.0f), e(0.0f, 2.0f);
    std::vector<float> box(6 * (size_t)n);
    std::vector<uint32_t> emit((size_t)n);
    for (int i = 0; i < n; ++i) {
        float c[3];
        for (int k = 0; k < 3; ++k) c[k] = (rng() % 7 == 0) ? 0.0f : u(rng);   // duplicated centroids
        for (int k = 0; k < 3; ++k) {
            const float h = (rng() % 5 == 0) ? 0.0f : e(rng);                // flat and point boxes
            box[6 * i + k] = c[k] - h;
            box[6 * i + 3 + k] = c[k] + h;
        }
        emit[i] = rng() % 11 == 0;
    }
    std::vector<int> pos((size_t)n);
    for (int i = 0; i < n; ++i) pos[i] = i;
    tpt::HostFloats out;
    int need = 0;
    tpt::WideParams prm;
    prm.threads = threads;
    const int nodes = tpt::build_wide_sah(pos, box.data(), emit.data(), n - 1, 0, out, &need, prm);
    if (nodes <= 0 || out.size() < 32 * (size_t)nodes || need <= 0) {
        std::printf("error: wide tree n=%d nodes=%d need=%d\n", n, nodes, need);
        return 1;
    }
    if (threads != 1) {   // the threaded build must equal the serial one byte for byte
        tpt::HostFloats ser;
        int sneed = 0;
        prm.threads = 1;
        const int snodes = tpt::build_wide_sah(pos, box.data(), emit.data(), n - 1, 0, ser, &sneed, prm);
        if (snodes != nodes || sneed != need || ser.size() != out.size() ||
            std::memcmp(ser.data(), out.data(), out.size() * sizeof(float)) != 0) {
            std::printf("error: wide tree n=%d threads=%d differs from the serial build\n", n, threads);
            return 1;
        }
    }
    {   // a reused workspace (the scene's, frame after frame) builds the same tree,
        // also after a build of another size in it
        tpt::WideWorkspace ws;
        tpt::WideParams wp;
        wp.threads = threads;
        wp.ws = &ws;
        std::vector<int> half(pos.begin(), pos.begin() + (n + 1) / 2);
        for (int rep = 0; rep < 3; ++rep) {
            tpt::HostFloats o2;
            int n2 = 0;
            const std::vector<int>& pp = rep == 1 ? half : pos;
            const int k = tpt::build_wide_sah(pp, box.data(), emit.data(), n - 1, 0, o2, &n2, wp);
            if (rep != 1 && (k != nodes || n2 != need || o2.size() != out.size() ||
                             std::memcmp(o2.data(), out.data(), out.size() * sizeof(float)) != 0)) {
                std::printf("error: wide tree n=%d: a reused workspace builds another tree\n", n);
                return 1;
            }
        }
    }
    std::printf("ok wide n=%d nodes=%d stack=%d\n", n, nodes, need);
    return 0;
}

int main(int argc, char** argv) {
    if (argc < 3) {
        std::fprintf(stderr, "usage: host_check gltf|image FILE... | wide N SEED [THREADS]\n");
        return 2;
    }
    const std::string mode = argv[1];
    if (mode == "wide")
        return check_wide(std::atoi(argv[2]), argc > 3 ? (unsigned)std::atoi(argv[3]) : 1u, argc > 4 ? std::atoi(argv[4]) : -1);
    for (int i = 2; i < argc; ++i) {
        try {
            if (mode == "gltf") {
                tpt::HostScene hs;
                tpt::load_gltf(argv[i], hs);
                std::printf("ok %zu faces\n", hs.indices.size() / 3);
            } else if (mode == "image") {
                std::vector<uint8_t> rgba;
                int w = 0, h = 0;
                tpt::load_image(argv[i], rgba, w, h);
                if (rgba.size() != 4 * (size_t)w * (size_t)h) {
                    std::printf("error: size mismatch\n");
                    return 1;
                }
                std::printf("ok %dx%d\n", w, h);
            } else {
                return 2;
            }
        } catch (const std::exception& ex) {
            std::printf("error: %s\n", ex.what());
        }
    }
    return 0;
}
