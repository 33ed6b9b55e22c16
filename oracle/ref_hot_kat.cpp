// ref_hot_kat.cpp -- TEST INFRASTRUCTURE ONLY.
//
// Drives the reference's own header-only hot-path functions, compiled by
// hipcc (host only) from where the files lie under /root/reference/include
// (oracle/Makefile target _ref/ref_hot_kat):
//   include/geometry_queries.h:18-86  rayHitBBox, rayHitTriangle
//   include/delta_light.h:25-130      CalcDistAttenuation, DeltaLight::sample
//   include/material.h:74-103         Spectrum::toUChar, Material()
// Only <cfloat> and <hip/hip_runtime.h> (which supplies uchar3; bvh.cuh pulls
// rocThrust's <thrust/device_vector.h>) go ahead of them -- no stand-ins.
//
// Protocol (stdin -> stdout, one request per line, floats as hex bit patterns):
//   B o3 d3 min3 max3          -> "B hit"                       rayHitBBox
//   X o3 d3 v0_3 v1_3 v2_3     -> "X hit dist u v"              rayHitTriangle
//                                 (dist/u/v keep their 7fc00001 sentinels on a miss)
//   L type color3 intensity pos3 dir3 cosOuter invCosDiff p3
//                              -> "L rad3 dir3 dist"            DeltaLight::sample
//   A dist r g b               -> "A r g b"                     CalcDistAttenuation
//   U r g b                    -> "U x y z" (decimal bytes)     Spectrum::toUChar
//   M                          -> "M" + 15 floats               Material() defaults
//   S                          -> "S" + decimal byte sizes and offsets of the
//                                 structs the C-ABI takes as they are (tpt.h):
//                                 sizeof(DeltaLight), then the offsets within
//                                 DeltaLight of type, pl.color, pl.intensity,
//                                 pl.pos, dl.color, dl.intensity, dl.direction,
//                                 sl.color, sl.intensity, sl.pos, sl.direction,
//                                 sl.cosOuterAngle, sl.invCosConeDifference;
//                                 sizeof(Material), offsets of baseColor,
//                                 emissionFactor, eta, metallic, clearcoatGloss;
//                                 sizeof(Vec3), sizeof(Spectrum)
#include <cfloat>
#include <hip/hip_runtime.h>

#include "geometry_queries.h"
#include "delta_light.h"
#include "material.h"

#include <cstdint>
#include <cstdio>
#include <cstring>
#include <iostream>
#include <new>
#include <sstream>
#include <string>

static float hf(const std::string& s) {
    uint32_t u = (uint32_t)std::stoul(s, nullptr, 16);
    float f;
    std::memcpy(&f, &u, 4);
    return f;
}
static void pf(float f) {
    uint32_t u;
    std::memcpy(&u, &f, 4);
    std::printf(" %08x", u);
}
static float sentinel() { return hf("7fc00001"); }

int main() {
    std::string line;
    while (std::getline(std::cin, line)) {
        std::istringstream in(line);
        std::string op;
        in >> op;
        std::string tok[32];
        int n = 0;
        while (n < 32 && in >> tok[n]) ++n;
        auto v3 = [&](int i) { return Vec3(hf(tok[i]), hf(tok[i + 1]), hf(tok[i + 2])); };
        if (op == "B" && n == 12) {
            Ray r(v3(0), v3(3));
            BBox b(v3(6), v3(9));
            std::printf("B %d\n", rayHitBBox(r, b) ? 1 : 0);
        } else if (op == "X" && n == 15) {
            Ray r(v3(0), v3(3));
            Real dist = sentinel();
            Vec2 uv(sentinel(), sentinel());
            const bool h = rayHitTriangle(r, v3(6), v3(9), v3(12), dist, uv);
            std::printf("X %d", h ? 1 : 0);
            pf(dist); pf(uv.x); pf(uv.y);
            std::printf("\n");
        } else if (op == "L" && n == 16) {
            DeltaLight dl;
            const int type = std::stoi(tok[0]);
            if (type == 0) {
                dl.type = POINT_LIGHT;
                new (&dl.light.pl) PointLight();
                dl.light.pl.color = Spectrum(hf(tok[1]), hf(tok[2]), hf(tok[3]));
                dl.light.pl.intensity = hf(tok[4]);
                dl.light.pl.pos = v3(5);
            } else if (type == 1) {
                dl.type = DIRECTIONAL_LIGHT;
                new (&dl.light.dl) DirectionalLight();
                dl.light.dl.color = Spectrum(hf(tok[1]), hf(tok[2]), hf(tok[3]));
                dl.light.dl.intensity = hf(tok[4]);
                dl.light.dl.direction = v3(8);
            } else {
                dl.type = SPOT_LIGHT;
                new (&dl.light.sl) SpotLight();
                dl.light.sl.color = Spectrum(hf(tok[1]), hf(tok[2]), hf(tok[3]));
                dl.light.sl.intensity = hf(tok[4]);
                dl.light.sl.pos = v3(5);
                dl.light.sl.direction = v3(8);
                dl.light.sl.cosOuterAngle = hf(tok[11]);
                dl.light.sl.invCosConeDifference = hf(tok[12]);
            }
            Incoming inc = dl.sample(v3(13));
            std::printf("L");
            pf(inc.radiance.r); pf(inc.radiance.g); pf(inc.radiance.b);
            pf(inc.direction.x); pf(inc.direction.y); pf(inc.direction.z);
            pf(inc.distance);
            std::printf("\n");
        } else if (op == "A" && n == 4) {
            Incoming inc;
            inc.distance = hf(tok[0]);
            inc.radiance = Spectrum(hf(tok[1]), hf(tok[2]), hf(tok[3]));
            CalcDistAttenuation(inc);
            std::printf("A");
            pf(inc.radiance.r); pf(inc.radiance.g); pf(inc.radiance.b);
            std::printf("\n");
        } else if (op == "U" && n == 3) {
            Spectrum s(hf(tok[0]), hf(tok[1]), hf(tok[2]));
            uchar3 c = s.toUChar();
            std::printf("U %d %d %d\n", (int)c.x, (int)c.y, (int)c.z);
        } else if (op == "M" && n == 0) {
            Material m;
            std::printf("M");
            pf(m.baseColor.r); pf(m.baseColor.g); pf(m.baseColor.b);
            pf(m.emissionFactor); pf(m.eta); pf(m.metallic); pf(m.subsurface); pf(m.specular);
            pf(m.roughness); pf(m.specularTint); pf(m.anisotropic); pf(m.sheen); pf(m.sheenTint);
            pf(m.clearcoat); pf(m.clearcoatGloss);
            std::printf("\n");
        } else if (op == "S" && n == 0) {
            DeltaLight d;
            Material m;
            const char* b = (const char*)&d;
            auto off = [&](const void* p) { return (long)((const char*)p - b); };
            const char* mb = (const char*)&m;
            auto moff = [&](const void* p) { return (long)((const char*)p - mb); };
            std::printf("S %zu %ld %ld %ld %ld %ld %ld %ld %ld %ld %ld %ld %ld %ld", sizeof(DeltaLight), off(&d.type),
                        off(&d.light.pl.color), off(&d.light.pl.intensity), off(&d.light.pl.pos),
                        off(&d.light.dl.color), off(&d.light.dl.intensity), off(&d.light.dl.direction),
                        off(&d.light.sl.color), off(&d.light.sl.intensity), off(&d.light.sl.pos),
                        off(&d.light.sl.direction), off(&d.light.sl.cosOuterAngle),
                        off(&d.light.sl.invCosConeDifference));
            std::printf(" %zu %ld %ld %ld %ld %ld %zu %zu\n", sizeof(Material), moff(&m.baseColor),
                        moff(&m.emissionFactor), moff(&m.eta), moff(&m.metallic), moff(&m.clearcoatGloss),
                        sizeof(Vec3), sizeof(Spectrum));
        } else {
            std::printf("E\n");
        }
        std::fflush(stdout);
    }
    return 0;
}
