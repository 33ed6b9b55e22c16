// build.hip -- world transform + LBVH construction on the device.
//
// Same tree as the reference's BVH::construct (src/bvh.cu:304-331):
//   k_transform    path_tracer.cu:239-263 (per face, benign duplicate writes)
//   k_morton       initNodes bvh.cu:128-148 (triangle AABB, centroid, 63-bit Morton)
//   radix sort     thrust::sort_by_key bvh.cu:326 -> rocPRIM LSD radix sort (stable)
//   k_karras       computeNodeRange bvh.cu:150-217 (Karras 2012 range + split)
//   k_depth/level  computeBBox bvh.cu:219-302: exact min/max unions bottom-up,
//                  one launch per tree level (kernel boundaries order the levels,
//                  so no cross-XCD hand-off inside a launch is needed)
//   k_pack_*       the traversal layout of device_api.hpp
#include <hip/hip_runtime.h>

#include <rocprim/device/device_radix_sort.hpp>

#include <vector>

#include "../common/device_api.hpp"
#include "../common/tri_rec.hpp"
#include "../common/tpt_math.hpp"

namespace tpt {

// findIdxOfTrans / mtlLinearSearch (path_tracer.cu:125-135, 227-237)
__device__ __forceinline__ int find_object(int fid, const int2* __restrict__ lut, int n) {
    int i = n - 1;
    for (; i >= 0; --i)
        if (fid >= lut[i].x) return i;
    return i;
}

__global__ void k_transform(BuildBuffers b) {
    const int f = blockIdx.x * blockDim.x + threadIdx.x;
    if (f >= b.n_faces) return;
    const int obj = find_object(f, b.lut, b.n_objects);
    const float* vt = b.vert_trans + 16 * obj;
    const float* nt = b.normal_trans + 16 * obj;
    float r[4];
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        const uint32_t vid = b.indices[3 * f + c];
        mat4_vec4(vt, b.vertices[3 * vid], b.vertices[3 * vid + 1], b.vertices[3 * vid + 2], 1.0f, r);
        b.wverts[3 * vid] = r[0];
        b.wverts[3 * vid + 1] = r[1];
        b.wverts[3 * vid + 2] = r[2];
    }
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        const uint32_t vid = b.indices[3 * f + c];
        mat4_vec4(nt, b.normals[3 * vid], b.normals[3 * vid + 1], b.normals[3 * vid + 2], 0.0f, r);
        const V3 n = normalize(v3(r[0], r[1], r[2]));
        b.wnorms[3 * vid] = n.x;
        b.wnorms[3 * vid + 1] = n.y;
        b.wnorms[3 * vid + 2] = n.z;
    }
}

// floatTo21Int (bvh.cu:23-46).  Right shifts of >= 32 give 0 (PTX semantics,
// the hardware shifter would otherwise use the count mod 32);
// the signed overflow at :42 is computed with unsigned wrap.
__device__ __forceinline__ uint64_t float_to_21int(float x) {
    const int32_t ix = __float_as_int(x);
    int32_t exponent = ((ix >> 23) & 0xff) - 127;
    const int32_t mantissa = (ix & 0x00ffffff) | 0x00800000;
    const uint32_t signbit = ((uint32_t)ix & 0x80000000u) >> 30;
    const int32_t sign = -1 * ((int32_t)signbit - 1);
    uint32_t value;
    if (exponent >= 8) value = 0x7fffffffu;
    else if (exponent >= 0) value = (uint32_t)mantissa << exponent;
    else value = (-exponent >= 32) ? 0u : (uint32_t)(mantissa >> (-exponent));
    value = value * (uint32_t)sign + 0x7fffffffu;
    return (uint64_t)((value & 0xfffff800u) >> 11);
}

__device__ __forceinline__ uint64_t expand_bits(uint64_t u) {   // bvh.cu:14-21
    u = (u | u << 32) & 0x1f00000000ffffull;
    u = (u | u << 16) & 0x1f0000ff0000ffull;
    u = (u | u << 8) & 0x100f00f00f00f00full;
    u = (u | u << 4) & 0x10c30c30c30c30c3ull;
    u = (u | u << 2) & 0x1249249249249249ull;
    return u;
}

__global__ void k_morton(BuildBuffers b) {
    const int f = blockIdx.x * blockDim.x + threadIdx.x;
    if (f >= b.n_faces) return;
    const float* w = b.wverts;
    const uint32_t i0 = b.indices[3 * f], i1 = b.indices[3 * f + 1], i2 = b.indices[3 * f + 2];
    const V3 p0 = v3(w[3 * i0], w[3 * i0 + 1], w[3 * i0 + 2]);
    const V3 p1 = v3(w[3 * i1], w[3 * i1 + 1], w[3 * i1 + 2]);
    const V3 p2 = v3(w[3 * i2], w[3 * i2 + 1], w[3 * i2 + 2]);
    const V3 mn = vmin(vmin(p0, p1), p2), mx = vmax(vmax(p0, p1), p2);   // BBox(v0,v1,v2)
    const V3 c = 0.5f * (mn + mx);                                       // BBox::center
    b.keys[f] = expand_bits(float_to_21int(c.x)) | (expand_bits(float_to_21int(c.y)) << 1) |
                (expand_bits(float_to_21int(c.z)) << 2);
    b.fids[f] = (uint32_t)f;
    float* lb = b.leaf_box + 6 * f;
    lb[0] = mn.x; lb[1] = mn.y; lb[2] = mn.z;
    lb[3] = mx.x; lb[4] = mx.y; lb[5] = mx.z;
}

__device__ __forceinline__ int clz64(uint64_t v) { return v == 0 ? 64 : __clzll((long long)v); }

__global__ void k_karras(BuildBuffers b) {
    const int n = b.n_faces;
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n - 1) return;
    const unsigned long long* keys = b.keys_sorted;
    // getTheOtherEnd (bvh.cu:64-99)
    const uint64_t self = keys[i];
    const uint64_t left = i == 0 ? ~0ull : keys[i - 1];
    const int lc = clz64(left ^ self), rc = clz64(keys[i + 1] ^ self);
    const int dir = lc > rc ? -1 : 1;
    const int minr = lc < rc ? lc : rc;
    int lmax = 2;
    int e = i + dir * lmax;
    while (e >= 0 && e < n && clz64(self ^ keys[e]) > minr) {
        lmax <<= 1;
        e = i + dir * lmax;
    }
    int range = 0;
    for (int step = lmax >> 1; step > 0; step >>= 1) {
        e = i + (range + step) * dir;
        if (e < 0 || e >= n) continue;
        if (clz64(self ^ keys[e]) > minr) range += step;
    }
    const int oe = i + range * dir;
    // findSplitPosition (bvh.cu:101-120)
    const int lo = dir == -1 ? oe : i, hi = dir == -1 ? i : oe;
    const int delta = clz64(keys[lo] ^ keys[hi]);
    int split = 0;
    for (int t = lmax >> 1; t > 0; t >>= 1) {
        const int pos = i + dir * (split + t);
        if (pos < lo || pos > hi) continue;
        if (clz64(self ^ keys[pos]) > delta) split += t;
    }
    const int sp = i + split * dir;
    // child links in the reference numbering (bvh.cu:164-214)
    int lchild, rchild;
    if (dir == 1) {
        rchild = (hi == sp + 1) ? sp + n : sp + 1;
        lchild = (lo == sp) ? sp + n - 1 : sp;
    } else {
        lchild = (lo == sp - 1) ? sp + n - 2 : sp - 1;
        rchild = (hi == sp) ? sp + n - 1 : sp;
    }
    b.children[i] = make_int2(lchild, rchild);
    b.parent[lchild] = (uint32_t)i;
    b.parent[rchild] = (uint32_t)i;
}

// Leaf boxes at their sorted positions; internal depth (root = 0) by walking up.
__global__ void k_depth(BuildBuffers b, uint32_t* depth) {
    const int n = b.n_faces, nn = 2 * n - 1;
    const int id = blockIdx.x * blockDim.x + threadIdx.x;
    if (id >= nn) return;
    if (id >= n - 1) {
        const uint32_t fid = b.fids_sorted[id - (n - 1)];
        const float* src = b.leaf_box + 6 * fid;
        float* dst = b.node_box + 6 * id;
#pragma unroll
        for (int k = 0; k < 6; ++k) dst[k] = src[k];
        // emitter flag of the leaf: its material's emissionFactor != 0 (the
        // direct probe only needs the closest emissive hit, see trace.hip)
        int mtl = b.lut[find_object((int)fid, b.lut, b.n_objects)].y;
        if (mtl < 0 || mtl >= b.n_materials) mtl = b.n_materials;   // Material() slot
        b.emit[id] = b.mtl[2 * mtl].w != 0.0f ? 1u : 0u;
    }
    uint32_t d = 0;
    int cur = id;
    while (cur != 0 && d < kMaxLbvhDepth) {
        cur = (int)b.parent[cur];
        ++d;
    }
    depth[id] = d;
    atomicMax(b.max_depth, d);
}

// One level of computeBBox: box = left.box; box.enclose(right.box)
__global__ void k_union_level(BuildBuffers b, const uint32_t* __restrict__ depth, uint32_t level) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= b.n_faces - 1 || depth[i] != level) return;
    const int2 c = b.children[i];
    const float* l = b.node_box + 6 * c.x;
    const float* r = b.node_box + 6 * c.y;
    float* o = b.node_box + 6 * i;
    o[0] = fmn(l[0], r[0]); o[1] = fmn(l[1], r[1]); o[2] = fmn(l[2], r[2]);
    o[3] = fmx(l[3], r[3]); o[4] = fmx(l[4], r[4]); o[5] = fmx(l[5], r[5]);
    b.emit[i] = b.emit[c.x] | b.emit[c.y];   // subtree holds an emissive triangle
}

// Child links carry the child's emitter flag in bit 30 (ids < 2^30).
__device__ __forceinline__ int link(const BuildBuffers& b, int id) {
    return id < 0 ? id : (id | (int)(b.emit[id] << 30));
}

__global__ void k_pack_inner(BuildBuffers b) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= b.n_faces - 1) return;
    const int2 c = b.children[i];
    const float* l = b.node_box + 6 * c.x;
    const float* r = b.node_box + 6 * c.y;
    float4* q = b.inner + 4 * i;
    q[0] = make_float4(l[0], l[1], l[2], l[3]);
    q[1] = make_float4(l[4], l[5], r[0], r[1]);
    q[2] = make_float4(r[2], r[3], r[4], r[5]);
    q[3] = make_float4(__int_as_float(link(b, c.x)), __int_as_float(link(b, c.y)), 0.0f, 0.0f);
    bool fin = true;
#pragma unroll
    for (int k = 0; k < 6; ++k) fin = fin && isfinite(l[k]) && isfinite(r[k]);
    if (!fin) atomicOr(b.max_depth + 1, 1u);
}

// 4-wide nodes are the even-depth internal nodes: the children of a kept
// node's internal children are themselves kept (depth + 2), so depth parity
// decides.  They are numbered breadth-first -- key (level, id), odd-depth nodes
// sorted past the end -- so the top levels are a prefix the trace kernel can
// stage in LDS.
__global__ void k_bfs_keys(BuildBuffers b, const uint32_t* __restrict__ depth) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= b.n_faces - 1) return;
    const uint32_t d = depth[i];
    b.bfs_keys[i] = (d & 1u) ? ~0ull : (((unsigned long long)(d >> 1) << 32) | (unsigned)i);
    b.bfs_ids[i] = (uint32_t)i;
    if (!(d & 1u)) atomicAdd(b.max_depth + 2, 1u);
}

__global__ void k_bfs_newid(BuildBuffers b, uint32_t n4) {
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j < n4) b.bfs_newid[b.bfs_ids_sorted[j]] = j;
}

__global__ void k_pack_inner4(BuildBuffers b, const uint32_t* __restrict__ depth) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const int nint = b.n_faces - 1;
    if (i >= nint || (depth[i] & 1u)) return;
    const int2 c = b.children[i];
    int ids[4] = {-1, -1, -1, -1};
    int n = 0;
    const int cs[2] = {c.x, c.y};
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        if (cs[h] >= nint) {
            ids[n++] = cs[h];
        } else {
            const int2 g = b.children[cs[h]];
            ids[n++] = g.x;
            ids[n++] = g.y;
        }
    }
    float f[24];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const float* bx = b.node_box + 6 * (ids[k] < 0 ? 0 : ids[k]);
#pragma unroll
        for (int j = 0; j < 6; ++j) f[6 * k + j] = ids[k] < 0 ? 0.0f : bx[j];
    }
    float4* q = b.inner4 + 8 * (size_t)b.bfs_newid[i];
#pragma unroll
    for (int k = 0; k < 6; ++k) q[k] = make_float4(f[4 * k], f[4 * k + 1], f[4 * k + 2], f[4 * k + 3]);
    int out[4];
#pragma unroll
    for (int k = 0; k < 4; ++k)   // internal grandchildren -> breadth-first id; leaves keep nint + position
        out[k] = (ids[k] >= 0 && ids[k] < nint) ? ((int)b.bfs_newid[ids[k]] | (int)(b.emit[ids[k]] << 30))
                                                : link(b, ids[k]);
    q[6] = make_float4(__int_as_float(out[0]), __int_as_float(out[1]), __int_as_float(out[2]),
                       __int_as_float(out[3]));
    q[7] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
}

__global__ void k_pack_leaf(BuildBuffers b) {
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    const int n = b.n_faces;
    if (j >= n) return;
    const uint32_t fid = b.fids_sorted[j];
    const float* w = b.wverts;
    const uint32_t i0 = b.indices[3 * fid], i1 = b.indices[3 * fid + 1], i2 = b.indices[3 * fid + 2];
    const V3 p0 = v3(w[3 * i0], w[3 * i0 + 1], w[3 * i0 + 2]);
    const V3 p1 = v3(w[3 * i1], w[3 * i1 + 1], w[3 * i1 + 2]);
    const V3 p2 = v3(w[3 * i2], w[3 * i2 + 1], w[3 * i2 + 2]);
    const V3 e1 = p1 - p0, e2 = p2 - p0;   // rayHitTriangle :66-67, hoisted (same rounding)
    tri_store(b.tri, j, p0.x, p0.y, p0.z, (int)fid, e1.x, e1.y, e1.z, e2.x, e2.y, e2.z);
}

__global__ void k_pack_shade(BuildBuffers b) {
    const int f = blockIdx.x * blockDim.x + threadIdx.x;
    if (f >= b.n_faces) return;
    const float* w = b.wnorms;
    const uint32_t i0 = b.indices[3 * f], i1 = b.indices[3 * f + 1], i2 = b.indices[3 * f + 2];
    int mtl = b.lut[find_object(f, b.lut, b.n_objects)].y;
    if (mtl < 0 || mtl >= b.n_materials) mtl = b.n_materials;   // -> Material() slot (App. A.9)
    float4* s = b.shade + 3 * f;
    // the face's geometric unit normal n for the trace kernel's grazing test of rays
    // leaving this face (trace.hip grazing(), "Culling"): n.x in s[1].w, n.y in
    // s[2].w, the sign of n.z in n.x's lowest mantissa bit (1: negative); n.z is
    // recomputed from the unit length.  A non-finite n.x marks "no normal"
    // (degenerate or non-finite face: never grazing).
    const float* v = b.wverts;
    const float ax = v[3 * i1] - v[3 * i0], ay = v[3 * i1 + 1] - v[3 * i0 + 1], az = v[3 * i1 + 2] - v[3 * i0 + 2];
    const float bx = v[3 * i2] - v[3 * i0], by = v[3 * i2 + 1] - v[3 * i0 + 1], bz = v[3 * i2 + 2] - v[3 * i0 + 2];
    const float gx = ay * bz - az * by, gy = az * bx - ax * bz, gz = ax * by - ay * bx;
    const float len = sqrtf(gx * gx + gy * gy + gz * gz);
    float nxs = __builtin_nanf(""), nys = 0.0f;
    if (len > 0.0f && __builtin_isfinite(len)) {
        const uint32_t xb = (__float_as_uint(gx / len) & ~1u) | (gz < 0.0f ? 1u : 0u);
        nxs = __uint_as_float(xb);
        nys = gy / len;
    }
    s[0] = make_float4(w[3 * i0], w[3 * i0 + 1], w[3 * i0 + 2], __int_as_float(mtl));
    s[1] = make_float4(w[3 * i1], w[3 * i1 + 1], w[3 * i1 + 2], nxs);
    s[2] = make_float4(w[3 * i2], w[3 * i2 + 1], w[3 * i2 + 2], nys);
}

// Reference node layout (bvh.cuh:52-58) for introspection / parity tests.
__global__ void k_pack_nodes36(BuildBuffers b) {
    const int n = b.n_faces, nn = 2 * n - 1;
    const int id = blockIdx.x * blockDim.x + threadIdx.x;
    if (id >= nn) return;
    uint32_t* o = (uint32_t*)((char*)b.nodes36 + 36 * (size_t)id);
    o[0] = id == 0 ? 0u : b.parent[id];
    if (id < n - 1) {
        o[1] = (uint32_t)b.children[id].x;
        o[2] = (uint32_t)b.children[id].y;
    } else {
        o[1] = b.fids_sorted[id - (n - 1)];
        o[2] = 0u;
    }
    const float* bx = b.node_box + 6 * id;
#pragma unroll
    for (int k = 0; k < 6; ++k) o[3 + k] = __float_as_uint(bx[k]);
}

// The host's sliver criterion and cull-slack scale, in double as it computed
// them: a sliver's |e1 x e2| < 1e-3 |e1| |e2| (a zero-length edge makes the
// determinant exactly 0 or NaN: never accepted, so not a sliver); the largest
// |v0|, |v0 + e1|, |v0 + e2| coordinate, reduced per block, then one 64-bit
// atomic max per block.
__global__ __launch_bounds__(256) void k_sliver_scan(const float4* __restrict__ tri, int n, uint8_t* __restrict__ sliver,
                                                     unsigned long long* coord_max) {
    __shared__ double smax[256];
    const int p = blockIdx.x * 256 + threadIdx.x;
    double m = 0.0;
    if (p < n) {
        const TriQ tq = tri_load(tri, p);
        const float4 q0 = tq.q0, q1 = tq.q1, q2 = tq.q2;
        const double a0 = q1.x, a1 = q1.y, a2 = q1.z, b0 = q2.x, b1 = q2.y, b2 = q2.z;
        const double c0 = a1 * b2 - a2 * b1, c1 = a2 * b0 - a0 * b2, c2 = a0 * b1 - a1 * b0;
        const double la = sqrt(a0 * a0 + a1 * a1 + a2 * a2);
        const double lb = sqrt(b0 * b0 + b1 * b1 + b2 * b2);
        const double lc = sqrt(c0 * c0 + c1 * c1 + c2 * c2);
        sliver[p] = (la > 0.0 && lb > 0.0 && !(lc >= 1e-3 * la * lb)) ? 1 : 0;   // NaN-safe
        const double v[3] = {q0.x, q0.y, q0.z}, a[3] = {a0, a1, a2}, b[3] = {b0, b1, b2};
#pragma unroll
        for (int k = 0; k < 3; ++k) m = fmax(m, fmax(fabs(v[k]), fmax(fabs(v[k] + a[k]), fabs(v[k] + b[k]))));
    }
    smax[threadIdx.x] = m;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w) smax[threadIdx.x] = fmax(smax[threadIdx.x], smax[threadIdx.x + w]);
        __syncthreads();
    }
    if (threadIdx.x == 0) atomicMax(coord_max, (unsigned long long)__double_as_longlong(smax[0]));
}

hipError_t launch_sliver_scan(const float4* tri, int32_t n, uint8_t* sliver, unsigned long long* coord_max,
                              hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_sliver_scan, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, tri, n, sliver, coord_max);
    return hipGetLastError();
}

hipError_t build_sort_tmp_bytes(int32_t n, size_t* bytes) {
    // the Morton sort (63 bits) and the breadth-first numbering sort (64 bits) share the buffer
    size_t a = 0, b = 0;
    hipError_t e = rocprim::radix_sort_pairs((void*)nullptr, a, (unsigned long long*)nullptr,
                                             (unsigned long long*)nullptr, (uint32_t*)nullptr, (uint32_t*)nullptr,
                                             (size_t)n, 0, 63);
    if (e != hipSuccess) return e;
    e = rocprim::radix_sort_pairs((void*)nullptr, b, (unsigned long long*)nullptr, (unsigned long long*)nullptr,
                                  (uint32_t*)nullptr, (uint32_t*)nullptr, (size_t)n, 0, 64);
    *bytes = a > b ? a : b;
    return e;
}

#define TPT_TRY(x)                         \
    do {                                   \
        hipError_t e_ = (x);               \
        if (e_ != hipSuccess) return e_;   \
    } while (0)

hipError_t launch_build(BuildBuffers& b, hipStream_t s) {
    const int n = b.n_faces;
    const int nn = 2 * n - 1;
    const dim3 blk(256);
    auto grid = [](int m) { return dim3((unsigned)((m + 255) / 256)); };
    hipLaunchKernelGGL(k_transform, grid(n), blk, 0, s, b);
    TPT_TRY(hipGetLastError());
    hipLaunchKernelGGL(k_morton, grid(n), blk, 0, s, b);
    TPT_TRY(hipGetLastError());
    size_t tmp = b.sort_tmp_bytes;
    TPT_TRY(rocprim::radix_sort_pairs(b.sort_tmp, tmp, b.keys, b.keys_sorted, b.fids, b.fids_sorted, (size_t)n, 0,
                                      63, s));
    if (n > 1) {
        hipLaunchKernelGGL(k_karras, grid(n - 1), blk, 0, s, b);
        TPT_TRY(hipGetLastError());
    }
    uint32_t* depth = b.flags;   // reused: 2F-1 words
    TPT_TRY(hipMemsetAsync(b.max_depth, 0, 3 * sizeof(uint32_t), s));
    b.out_n4 = 0;
    hipLaunchKernelGGL(k_depth, grid(nn), blk, 0, s, b, depth);
    TPT_TRY(hipGetLastError());
    uint32_t maxd = 0;
    TPT_TRY(hipMemcpyAsync(&maxd, b.max_depth, sizeof(uint32_t), hipMemcpyDeviceToHost, s));
    TPT_TRY(hipStreamSynchronize(s));
    b.out_max_depth = maxd;
    // k_depth stops a parent walk at kMaxLbvhDepth steps: only a parent chain that
    // never reaches the root gets there -- runs of duplicate Morton keys, which
    // computeNodeRange (bvh.cu:150-217) splits without an index tie-break, can
    // produce a node claimed by two parents and a cycle (the reference's own
    // undefined behaviour: its computeBBox and traversal would not terminate).
    // Refuse such a topology before any kernel walks it.
    if (maxd >= kMaxLbvhDepth) return hipErrorInvalidValue;
    // internal nodes live at depth <= maxd - 1; deepest first
    for (int level = (int)maxd - 1; level >= 0 && n > 1; --level) {
        hipLaunchKernelGGL(k_union_level, grid(n - 1), blk, 0, s, b, depth, (uint32_t)level);
        TPT_TRY(hipGetLastError());
    }
    if (n > 1) {
        hipLaunchKernelGGL(k_pack_inner, grid(n - 1), blk, 0, s, b);
        TPT_TRY(hipGetLastError());
        hipLaunchKernelGGL(k_bfs_keys, grid(n - 1), blk, 0, s, b, depth);
        TPT_TRY(hipGetLastError());
        size_t tmp2 = b.sort_tmp_bytes;
        TPT_TRY(rocprim::radix_sort_pairs(b.sort_tmp, tmp2, b.bfs_keys, b.bfs_keys_sorted, b.bfs_ids,
                                          b.bfs_ids_sorted, (size_t)(n - 1), 0, 64, s));
        uint32_t n4 = 0;
        TPT_TRY(hipMemcpyAsync(&n4, b.max_depth + 2, sizeof(uint32_t), hipMemcpyDeviceToHost, s));
        TPT_TRY(hipStreamSynchronize(s));
        b.out_n4 = n4;
        hipLaunchKernelGGL(k_bfs_newid, grid((int)n4), blk, 0, s, b, n4);
        TPT_TRY(hipGetLastError());
        hipLaunchKernelGGL(k_pack_inner4, grid(n - 1), blk, 0, s, b, depth);
        TPT_TRY(hipGetLastError());
    }
    hipLaunchKernelGGL(k_pack_leaf, grid(n), blk, 0, s, b);
    TPT_TRY(hipGetLastError());
    hipLaunchKernelGGL(k_pack_shade, grid(n), blk, 0, s, b);
    TPT_TRY(hipGetLastError());
    hipLaunchKernelGGL(k_pack_nodes36, grid(nn), blk, 0, s, b);
    TPT_TRY(hipGetLastError());
    uint32_t nonfinite = 0;
    TPT_TRY(hipMemcpyAsync(&nonfinite, b.max_depth + 1, sizeof(uint32_t), hipMemcpyDeviceToHost, s));
    TPT_TRY(hipStreamSynchronize(s));
    b.out_boxes_finite = nonfinite ? 0u : 1u;
    return hipSuccess;
}

}  // namespace tpt
