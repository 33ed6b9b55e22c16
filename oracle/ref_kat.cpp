// ref_kat.cpp -- TEST INFRASTRUCTURE ONLY.
//
// Drives the reference's own header-only L0 math (include/math/vec.h, mat.h,
// quat.h, transform.h, camera.h), compiled by g++ from where the files lie
// under /root/reference/include (see oracle/Makefile target _ref/ref_kat).
// Only standard-library headers are supplied ahead of them; no stand-ins.
//
// Protocol (stdin -> stdout, one request per line, floats as hex bit patterns):
//   T lx ly lz qx qy qz qw sx sy sz   -> L2W: 16 words, N2W: 16 words
//                                        (Transform::localToWorld, mesh.cu:370-378 lambda)
//   R x                               -> frsqrt(x)          (vec.h:44-57)
//   N x y z                           -> normalize(Vec3)    (vec.h:155)
//   V m0..m15 x y z w                 -> Mat4 * Vec4        (mat.h:37-51)
#include <cfloat>
#include <cmath>
#include <math.h>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <iostream>
#include <memory>
#include <sstream>
#include <string>

#include "math/vec.h"
#include "math/mat.h"
#include "math/quat.h"
#include "transform.h"
#include "camera.h"

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
static void pm(const Mat4& m) {
    for (int c = 0; c < 4; ++c)
        for (int r = 0; r < 4; ++r) pf(m[c][r]);
}

int main() {
    std::string line;
    while (std::getline(std::cin, line)) {
        std::istringstream in(line);
        std::string op;
        in >> op;
        std::string tok[32];
        int n = 0;
        while (n < 32 && in >> tok[n]) ++n;
        if (op == "T" && n == 10) {
            Vec3 loc(hf(tok[0]), hf(tok[1]), hf(tok[2]));
            Quat q(hf(tok[3]), hf(tok[4]), hf(tok[5]), hf(tok[6]));
            Vec3 s(hf(tok[7]), hf(tok[8]), hf(tok[9]));
            Transform t(loc, q, s);
            Mat4 l2w = t.localToWorld();
            Mat4 m{Vec4{l2w[0][0], l2w[0][1], l2w[0][2], 0.0f}, Vec4{l2w[1][0], l2w[1][1], l2w[1][2], 0.0f},
                   Vec4{l2w[2][0], l2w[2][1], l2w[2][2], 0.0f}, Vec4{0.0f, 0.0f, 0.0f, 1.0f}};
            Mat4 n2w = m.transpose().inverse();
            std::printf("T");
            pm(l2w);
            pm(n2w);
            std::printf("\n");
        } else if (op == "R" && n == 1) {
            std::printf("R");
            pf(frsqrt(hf(tok[0])));
            std::printf("\n");
        } else if (op == "N" && n == 3) {
            Vec3 v = normalize(Vec3(hf(tok[0]), hf(tok[1]), hf(tok[2])));
            std::printf("N");
            pf(v.x); pf(v.y); pf(v.z);
            std::printf("\n");
        } else if (op == "V" && n == 20) {
            Mat4 m;
            for (int c = 0; c < 4; ++c)
                for (int r = 0; r < 4; ++r) m[c][r] = hf(tok[4 * c + r]);
            Vec4 v(hf(tok[16]), hf(tok[17]), hf(tok[18]), hf(tok[19]));
            Vec4 o = m * v;
            std::printf("V");
            pf(o.x); pf(o.y); pf(o.z); pf(o.w);
            std::printf("\n");
        } else {
            std::printf("E\n");
        }
        std::fflush(stdout);
    }
    return 0;
}
