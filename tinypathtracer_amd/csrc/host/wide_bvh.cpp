// wide_bvh.cpp -- the 4-wide traversal tree of the ordered traversal, built on
// the host with the surface-area heuristic over the LBVH's exact leaf boxes.
//
// Why a second tree is exact.  For a finite ray and finite boxes, the
// reference (traverseBVH, path_tracer.cu:61-107) reaches a leaf iff the leaf's
// own box passes rayHitBBox (geometry_queries.h:18-46): every ancestor box is
// the exact min/max union of boxes that contain it and the slab arithmetic is
// monotonic in the bounds, so an ancestor passes whenever the leaf does.  The
// closest hit is then "least t > Delta, ties to the leaf met first", and the
// right-first DFS meets leaves in decreasing sorted position.  None of this
// depends on the tree's inner nodes: any hierarchy whose leaves carry the
// reference's leaf boxes (bvh.cu:128-148, the LBVH build's node_box) and
// positions finds the same hit under the kernel's ordered tie rule (equal t ->
// larger position).  Its inner boxes only steer the walk and cull, so they may
// be any supersets; here they are exact unions.
//
// The LBVH's Morton split ignores triangle sizes (large wall triangles straddle
// many splits) and its even-depth 4-wide view leaves many nodes with 2-3
// children.  This tree splits by binned SAH and collapses to 4 children per
// node by opening the largest-area internal child first.
#include <algorithm>
#include <array>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <exception>
#include <memory>
#include <system_error>
#include <thread>
#include <vector>

#include <sched.h>

#include "tpt_internal.hpp"

namespace tpt {

namespace {

struct Box {
    float lo[3], hi[3];
    void empty() {
        for (int k = 0; k < 3; ++k) {
            lo[k] = __builtin_inff();
            hi[k] = -__builtin_inff();
        }
    }
    void grow(const Box& b) {
        for (int k = 0; k < 3; ++k) {
            lo[k] = std::min(lo[k], b.lo[k]);
            hi[k] = std::max(hi[k], b.hi[k]);
        }
    }
    double area() const {
        const double dx = (double)hi[0] - lo[0], dy = (double)hi[1] - lo[1], dz = (double)hi[2] - lo[2];
        if (!(dx >= 0.0) || !(dy >= 0.0) || !(dz >= 0.0)) return 0.0;
        return 2.0 * (dx * dy + dy * dz + dz * dx);
    }
};

struct BNode {          // binary SAH node
    Box box;
    int left, right;   // child BNode ids; a leaf has left = -1
    int pos;           // leaf: the LBVH sorted position of its triangle (-1: inner)
    uint32_t emit;
};

// A build array left uninitialised: the build writes every element it reads,
// so each page is first touched by the thread that builds its subtree instead
// of in one serial zero-fill (≈ 3 ms for 131 K leaves).
template <class T>
struct Uninit {
    std::unique_ptr<T[]> p;
    size_t n = 0;
    void reset(size_t m) {
        p.reset(new T[m]);
        n = m;
    }
    T& operator[](size_t i) { return p[i]; }
    const T& operator[](size_t i) const { return p[i]; }
    size_t size() const { return n; }
};

struct Builder {
    const float* lbox;    // 6 per position
    int sweep_max = 32;   // ranges up to this size split by an exact sweep, larger ones binned
    Uninit<BNode> nodes;
    std::vector<int> idx;
    std::vector<float> cen;   // 3 per position

    Box leaf_box(int p) const {
        Box b;
        for (int k = 0; k < 3; ++k) {
            b.lo[k] = lbox[6 * p + k];
            b.hi[k] = lbox[6 * p + 3 + k];
        }
        return b;
    }

    // Stable insertion sort of v[0, m) by centroid coordinate `axis`: the same
    // order as std::stable_sort, without its buffer (m <= sweep_max is small).
    void sort_axis(int* v, int m, int axis) const {
        for (int i = 1; i < m; ++i) {
            const int x = v[i];
            const float kx = cen[3 * x + axis];
            int j = i;
            for (; j > 0 && kx < cen[3 * v[j - 1] + axis]; --j) v[j] = v[j - 1];
            v[j] = x;
        }
    }

    // Splits idx[b, e) in place; returns the split point (b < m < e).
    int split(int b, int e) {
        const int m = e - b;
        double best = __builtin_inf();
        int best_axis = -1, best_m = -1;
        if (m <= sweep_max) {
            // exact sweep over sorted centroids on each axis (each axis sorts the
            // previous axis's order, ties keep it; the range itself is then sorted
            // from its own order by the chosen axis)
            constexpr int kLocal = 64;
            int tmp_l[kLocal];
            double ra_l[kLocal];
            std::vector<int> tmp_v;
            std::vector<double> ra_v;
            if (m > kLocal) {
                tmp_v.resize(m);
                ra_v.resize(m);
            }
            int* tmp = m > kLocal ? tmp_v.data() : tmp_l;
            double* right_area = m > kLocal ? ra_v.data() : ra_l;
            std::copy(idx.begin() + b, idx.begin() + e, tmp);
            for (int axis = 0; axis < 3; ++axis) {
                sort_axis(tmp, m, axis);
                Box acc;
                acc.empty();
                for (int i = m - 1; i > 0; --i) {
                    acc.grow(leaf_box(tmp[i]));
                    right_area[i] = acc.area();
                }
                acc.empty();
                for (int i = 1; i < m; ++i) {
                    acc.grow(leaf_box(tmp[i - 1]));
                    const double c = acc.area() * i + right_area[i] * (m - i);
                    if (c < best) {
                        best = c;
                        best_axis = axis;
                        best_m = i;
                    }
                }
            }
            if (best_axis < 0) {   // no finite cost (NaN boxes): halve by position
                std::sort(idx.begin() + b, idx.begin() + e);
                return b + m / 2;
            }
            sort_axis(idx.data() + b, m, best_axis);
            return b + best_m;
        }
        Box cb;
        cb.empty();
        for (int i = b; i < e; ++i)
            for (int k = 0; k < 3; ++k) {
                cb.lo[k] = std::min(cb.lo[k], cen[3 * idx[i] + k]);
                cb.hi[k] = std::max(cb.hi[k], cen[3 * idx[i] + k]);
            }
        constexpr int kBins = 32;
        // one pass bins every axis (each leaf's box and centroid read once)
        Box bb[3][kBins];
        int bn[3][kBins] = {};
        float scl[3];
        bool live[3];
        for (int axis = 0; axis < 3; ++axis) {
            const float ext = cb.hi[axis] - cb.lo[axis];
            live[axis] = ext > 0.0f;
            scl[axis] = kBins / ext;
            for (auto& x : bb[axis]) x.empty();
        }
        for (int i = b; i < e; ++i) {
            const int p = idx[i];
            const Box lb = leaf_box(p);
            for (int axis = 0; axis < 3; ++axis) {
                if (!live[axis]) continue;
                int k = (int)((cen[3 * p + axis] - cb.lo[axis]) * scl[axis]);
                k = std::min(std::max(k, 0), kBins - 1);
                ++bn[axis][k];
                bb[axis][k].grow(lb);
            }
        }
        for (int axis = 0; axis < 3; ++axis) {
            if (!live[axis]) continue;
            double ra[kBins];
            int rn[kBins];
            Box acc;
            acc.empty();
            int cnt = 0;
            for (int k = kBins - 1; k > 0; --k) {
                acc.grow(bb[axis][k]);
                cnt += bn[axis][k];
                ra[k] = acc.area();
                rn[k] = cnt;
            }
            acc.empty();
            cnt = 0;
            for (int k = 1; k < kBins; ++k) {
                acc.grow(bb[axis][k - 1]);
                cnt += bn[axis][k - 1];
                if (cnt == 0 || rn[k] == 0) continue;
                const double c = acc.area() * cnt + ra[k] * rn[k];
                if (c < best) {
                    best = c;
                    best_axis = axis;
                    best_m = k;
                }
            }
        }
        if (best_axis < 0) {   // all centroids coincide: halve by position
            std::sort(idx.begin() + b, idx.begin() + e);
            return b + m / 2;
        }
        const float sc = kBins / (cb.hi[best_axis] - cb.lo[best_axis]);
        // stable partition: bins < best_m first, both sides in their order
        auto left_of = [&](int p) {
            int k = (int)((cen[3 * p + best_axis] - cb.lo[best_axis]) * sc);
            k = std::min(std::max(k, 0), kBins - 1);
            return k < best_m;
        };
        thread_local std::vector<int> right;
        right.clear();
        int s = b;
        for (int i = b; i < e; ++i) {
            const int p = idx[i];
            if (left_of(p)) idx[s++] = p;
            else right.push_back(p);
        }
        std::copy(right.begin(), right.end(), idx.begin() + s);
        if (s == b || s == e) s = b + m / 2;
        return s;
    }

    // Builds idx[b, e) as the subtree rooted at nodes[id].  Every leaf holds one
    // triangle, so a subtree of m leaves has 2m - 1 nodes and its pre-order ids
    // are known before it is built: the left child is id + 1, the right child
    // id + 2 * (left leaves).  Large left subtrees therefore build on their own
    // thread straight into the shared array (disjoint idx ranges and node ids),
    // and the tree is identical to a serial build's.
    void build(int b, int e, int id, const uint32_t* emit, int spawn) {
        BNode& nd = nodes[id];
        if (e - b == 1) {
            nd.pos = idx[b];
            nd.box = leaf_box(idx[b]);
            nd.emit = emit[idx[b]] ? 1u : 0u;
            nd.left = nd.right = -1;
            collapse_cost(id);
            return;
        }
        const int s = split(b, e);
        const int l = id + 1, r = id + 2 * (s - b);
        bool serial = true;
        if (spawn > 0 && s - b >= kParMin && e - s >= kParMin) {
            // The left subtree on its own thread.  Exceptions (bad_alloc in the
            // subtree) are carried back and rethrown after the join; a thread
            // that cannot be started (std::system_error under a pid or ulimit
            // cap) leaves the subtree to this thread -- the same tree either way.
            std::exception_ptr err;
            std::thread t;
            try {
                t = std::thread([&, b, s, l] {
                    try {
                        build(b, s, l, emit, spawn - 1);
                    } catch (...) {
                        err = std::current_exception();
                    }
                });
                serial = false;
            } catch (const std::system_error&) {
            }
            if (!serial) {
                try {
                    build(s, e, r, emit, spawn - 1);
                } catch (...) {
                    t.join();
                    throw;
                }
                t.join();
                if (err) std::rethrow_exception(err);
            }
        }
        if (serial) {   // (a lopsided split keeps its threads for the larger side)
            build(b, s, l, emit, spawn);
            build(s, e, r, emit, spawn);
        }
        nd.left = l;
        nd.right = r;
        nd.pos = -1;
        nd.box = nodes[l].box;
        nd.box.grow(nodes[r].box);
        nd.emit = nodes[l].emit | nodes[r].emit;
        collapse_cost(id);
    }
    static constexpr int kParMin = 4096;   // smallest subtree worth a thread

    // The collapse's dynamic program at node x (see build_wide_sah), run as soon
    // as both children are built, so it shares the build's threads.
    Uninit<std::array<double, 5>> D;
    Uninit<std::array<int8_t, 5>> pick;   // k >= 2: left share of the split (0: keep whole)
    void collapse_cost(int x) {
        const BNode& c = nodes[x];
        if (c.left < 0) {
            for (int k = 1; k <= 4; ++k) D[x][k] = 0.0;
            return;
        }
        auto forest = [&](int k, int8_t& a_best) {
            double best = __builtin_inf();
            for (int a = 1; a < k; ++a) {
                const double v = D[c.left][a] + D[c.right][k - a];
                if (v < best) {
                    best = v;
                    a_best = (int8_t)a;
                }
            }
            return best;
        };
        int8_t a4 = 1;
        const double whole = c.box.area() + forest(4, a4);
        pick[x][1] = a4;   // the split of a node kept whole (its own 4-wide node)
        D[x][1] = whole;
        for (int k = 2; k <= 4; ++k) {
            int8_t a = 1;
            const double f = forest(k, a);
            if (f < whole) {
                D[x][k] = f;
                pick[x][k] = a;
            } else {
                D[x][k] = whole;
                pick[x][k] = 0;
            }
        }
    }
};

}  // namespace

// Host cores this process may use: its CPU affinity mask, capped by a cgroup v2
// CPU quota (/sys/fs/cgroup/cpu.max).  std::thread::hardware_concurrency()
// reports every CPU of the host (256 on the GPU box, whose quota is 16).
int usable_cores() {
    int n = 0;
    cpu_set_t set;
    CPU_ZERO(&set);
    if (sched_getaffinity(0, sizeof set, &set) == 0) n = CPU_COUNT(&set);
    if (n <= 0) n = (int)std::max(1u, std::thread::hardware_concurrency());
    if (FILE* f = std::fopen("/sys/fs/cgroup/cpu.max", "r")) {
        char q[32] = {0};
        long long per = 0;
        if (std::fscanf(f, "%31s %lld", q, &per) == 2 && std::strcmp(q, "max") != 0 && per > 0) {
            const long long quota = std::atoll(q);
            if (quota > 0) n = std::min<long long>(n, std::max<long long>(1, quota / per));
        }
        std::fclose(f);
    }
    return std::max(1, n);
}

// Leaves: the LBVH sorted positions `pos` (all of them, or a subset such as the
// emissive triangles); leaf_box[6 * p] / leaf_emit[p] by position p.  Writes 32
// floats per 4-wide node in the inner4 layout of device_api.hpp (breadth-first,
// root first; child links: id_base + a node's index, or leaf_base + position
// for a leaf, with the emitter flag in bit 30; -1 none) and returns the node
// count; *stack_need = the most stack entries the ordered 4-wide walk can hold
// right after a visit (trace.hip inner_visit4; see below).
int build_wide_sah(const std::vector<int>& pos, const float* leaf_box, const uint32_t* leaf_emit, int leaf_base,
                   int id_base, std::vector<float>& out, int* stack_need, const WideParams& prm) {
    const int n = (int)pos.size();
    out.clear();
    *stack_need = 0;
    if (n == 0) return 0;
    Builder B;
    B.lbox = leaf_box;
    B.sweep_max = prm.sweep_max;
    B.idx = pos;
    int pmax = 0;
    for (int p : pos) pmax = std::max(pmax, p);
    B.cen.resize(3 * (size_t)(pmax + 1));
    for (int p : pos)
        for (int k = 0; k < 3; ++k) B.cen[3 * p + k] = 0.5f * (leaf_box[6 * p + k] + leaf_box[6 * p + 3 + k]);
    B.nodes.reset(2 * (size_t)n - 1);
    B.D.reset(B.nodes.size());
    B.pick.reset(B.nodes.size());
    // threads: up to 2^spawn concurrent subtrees, at most prm.threads (< 0: the
    // cores this process may use; 0 or 1: a serial build -- the same tree)
    const int hw = prm.threads < 0 ? usable_cores() : prm.threads;
    int spawn = 0;
    while (spawn < 5 && (2 << spawn) <= hw) ++spawn;
    const int root = 0;
    B.build(0, n, root, leaf_emit, spawn);
    const auto& N = B.nodes;
    if (N[root].left < 0) {   // a single leaf: one node holding it
        out.assign(32, 0.0f);
        for (int j = 0; j < 3; ++j) {
            out[j] = N[root].box.lo[j];
            out[3 + j] = N[root].box.hi[j];
        }
        const int32_t links[4] = {(leaf_base + N[root].pos) | (int32_t)(N[root].emit << 30), -1, -1, -1};
        std::memcpy(out.data() + 24, links, sizeof links);
        *stack_need = 0;
        return 1;
    }

    // Collapse to 4-wide nodes by dynamic programming over the binary tree
    // (the SAH cost of Ylitie et al. 2017's wide-BVH collapse, 1 triangle per
    // leaf): D[x][k] is the least cost of representing subtree x as a forest
    // of at most k subtrees.  Every leaf is some node's child exactly once, so
    // its triangle-test cost (area-weighted) is the same in every collapse and
    // drops out; a subtree kept whole costs its area (the probability that its
    // 4-wide node is visited) plus the best 4-way forest of its children.
    // Greedy opening of the largest child leaves the bottom levels with 2-leaf
    // nodes; the DP pulls leaves up into their grandparents.  (Builder::collapse_cost
    // runs it during the build.)
    const size_t nb = N.size();
    const auto& pick = B.pick;
    // Stack bound: a visit of node X finds at most A(X) entries on the stack --
    // the deferred siblings of X and of its ancestors, A(X) = sum over the
    // proper ancestors a of (children(a) - 1) -- and leaves at most A(X) +
    // children(X) - 1.
    struct Wide {
        int kids[4];
        int nk;
        int above;   // A(X)
    };
    std::vector<Wide> wide;
    std::vector<int> wide_of(nb, -1);
    std::vector<int> queue{root};   // breadth-first over binary nodes that become 4-wide nodes
    std::vector<int> qabove{0};
    int need = 0;
    for (size_t qi = 0; qi < queue.size(); ++qi) {
        const int b = queue[qi];
        Wide w{};
        w.nk = 0;
        w.above = qabove[qi];
        // expand (x, k): x's children as a forest of at most k roots
        struct Item {
            int x, k;
        };
        Item st[8];
        int sp = 0;
        st[sp++] = {N[b].right, 4 - pick[b][1]};
        st[sp++] = {N[b].left, pick[b][1]};
        while (sp > 0) {
            const Item it = st[--sp];
            const BNode& c = N[it.x];
            const int a = (c.left >= 0 && it.k >= 2) ? pick[it.x][it.k] : 0;
            if (a == 0) {
                w.kids[w.nk++] = it.x;
            } else {
                st[sp++] = {c.right, it.k - a};
                st[sp++] = {c.left, a};
            }
        }
        wide_of[b] = (int)wide.size();
        wide.push_back(w);
        need = std::max(need, w.above + w.nk - 1);
        for (int k = 0; k < w.nk; ++k)
            if (N[w.kids[k]].left >= 0) {
                queue.push_back(w.kids[k]);
                qabove.push_back(w.above + w.nk - 1);
            }
    }
    out.assign(32 * wide.size(), 0.0f);
    for (size_t i = 0; i < wide.size(); ++i) {
        float* q = out.data() + 32 * i;
        int32_t links[4] = {-1, -1, -1, -1};
        for (int k = 0; k < wide[i].nk; ++k) {
            const BNode& c = N[wide[i].kids[k]];
            for (int j = 0; j < 3; ++j) {
                q[6 * k + j] = c.box.lo[j];
                q[6 * k + 3 + j] = c.box.hi[j];
            }
            const int32_t id = c.left >= 0 ? id_base + wide_of[wide[i].kids[k]] : leaf_base + c.pos;
            links[k] = id | (int32_t)(c.emit << 30);
        }
        std::memcpy(q + 24, links, sizeof links);
    }
    *stack_need = need;
    return (int)wide.size();
}

}  // namespace tpt

extern "C" int32_t tpt_wide_tree_build(int32_t n, const float* leaf_box, const uint32_t* leaf_emit, float* nodes,
                                       int32_t cap, int32_t* stack_need, int32_t threads) {
    if (n < 2 || !leaf_box || !leaf_emit || cap < 0) return -1;
    std::vector<float> out;
    int lv = 0;
    int n4 = -1;
    try {
        std::vector<int> pos(n);
        for (int p = 0; p < n; ++p) pos[p] = p;
        tpt::WideParams prm;
        prm.threads = threads;
        n4 = tpt::build_wide_sah(pos, leaf_box, leaf_emit, n - 1, 0, out, &lv, prm);
    } catch (const std::exception&) {
        return -1;
    }
    if (stack_need) *stack_need = lv;
    if (n4 <= cap && nodes) std::memcpy(nodes, out.data(), out.size() * sizeof(float));
    return n4;
}
