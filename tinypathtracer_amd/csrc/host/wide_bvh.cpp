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
#include <atomic>
#include <condition_variable>
#include <deque>
#include <functional>
#include <mutex>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <exception>
#include <memory>
#include <system_error>
#include <thread>
#include <vector>

#include <emmintrin.h>
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

// One leaf as the build moves it: its exact box and LBVH position in 32 bytes,
// so the binning and partition passes stream contiguous records instead of
// gathering boxes and centroids through an index array.  Each half loads as
// one SSE vector; lane 3 (the position's bits, or 0) never enters arithmetic.
struct alignas(16) Rec {
    float lo[3];
    int32_t pos;
    float hi[3];
    float pad;
};

// SSE helpers.  The min/max operand order reproduces Box::grow exactly:
// _mm_min_ps(b, a) = b < a ? b : a = std::min(a, b) (NaN in b is ignored, the
// accumulator kept on ties), likewise _mm_max_ps(b, a) = std::max(a, b).
inline __m128 lane3_zero(__m128 v) { return _mm_and_ps(v, _mm_castsi128_ps(_mm_setr_epi32(-1, -1, -1, 0))); }
inline __m128 rec_lo(const Rec& q) { return _mm_load_ps(q.lo); }
inline __m128 rec_hi(const Rec& q) { return _mm_load_ps(q.hi); }
// 0.5f * (lo + hi) per axis, the centroid the binning and sweeps sort by
inline __m128 rec_cen(const Rec& q) {
    return _mm_mul_ps(_mm_set1_ps(0.5f), _mm_add_ps(lane3_zero(rec_lo(q)), lane3_zero(rec_hi(q))));
}

struct VBox {
    __m128 lo, hi;
    void empty() {
        lo = _mm_set1_ps(__builtin_inff());
        hi = _mm_set1_ps(-__builtin_inff());
    }
    void grow(__m128 blo, __m128 bhi) {
        lo = _mm_min_ps(blo, lo);
        hi = _mm_max_ps(bhi, hi);
    }
    void grow(const VBox& b) { grow(b.lo, b.hi); }
    void grow(const Rec& q) { grow(rec_lo(q), rec_hi(q)); }
    Box box() const {
        alignas(16) float l[4], h[4];
        _mm_store_ps(l, lo);
        _mm_store_ps(h, hi);
        Box b;
        for (int k = 0; k < 3; ++k) {
            b.lo[k] = l[k];
            b.hi[k] = h[k];
        }
        return b;
    }
    // Box::area on the vectors: the same double subtractions and products
    double area() const {
        const __m128d l01 = _mm_cvtps_pd(lo), h01 = _mm_cvtps_pd(hi);
        const __m128d l2 = _mm_cvtps_pd(_mm_movehl_ps(lo, lo)), h2 = _mm_cvtps_pd(_mm_movehl_ps(hi, hi));
        const __m128d d01 = _mm_sub_pd(h01, l01), d2 = _mm_sub_pd(h2, l2);
        const double dx = _mm_cvtsd_f64(d01), dy = _mm_cvtsd_f64(_mm_unpackhi_pd(d01, d01)), dz = _mm_cvtsd_f64(d2);
        if (!(dx >= 0.0) || !(dy >= 0.0) || !(dz >= 0.0)) return 0.0;
        return 2.0 * (dx * dy + dy * dz + dz * dx);
    }
};

// A build array left uninitialised: the build writes every element it reads,
// so each page is first touched by the thread that builds its subtree instead
// of in one serial zero-fill (≈ 3 ms for 131 K leaves).
template <class T>
struct Uninit {
    std::unique_ptr<T[]> p;
    size_t n = 0, cap = 0;
    void reset(size_t m) {   // m elements; the storage is reused when it holds them
        if (m > cap) {
            p.reset();
            cap = 0;
            p.reset(new T[m]);
            cap = m;
        }
        n = m;
    }
    void swap(Uninit& o) {
        p.swap(o.p);
        std::swap(n, o.n);
        std::swap(cap, o.cap);
    }
    T& operator[](size_t i) { return p[i]; }
    const T& operator[](size_t i) const { return p[i]; }
    size_t size() const { return n; }
};

// The build's worker threads: a FIFO of tasks run by threads - 1 workers and
// by whichever thread waits on a task group (it runs queued tasks while there
// are any, so nested waits cannot deadlock, and sleeps otherwise).  Threads are started once per
// build: on the GPU box starting one costs ≈ 35 µs, 15 at once ≈ 0.6 ms.  A
// thread that cannot be started (std::system_error under a pid or ulimit cap)
// just leaves its share to the others.  A task that throws (std::bad_alloc from
// a split's scratch vectors or a submit) never escapes its thread: the first
// exception is kept, every counter still moves, and wait_all() / chunks()
// rethrow it once no task can still reference the waiting frame.
class Pool {
public:
    explicit Pool(int threads) {
        for (int i = 1; i < threads; ++i) {
            try {
                th_.emplace_back([this] { work(); });
            } catch (const std::system_error&) {
                break;
            }
        }
    }
    ~Pool() {
        {
            std::lock_guard<std::mutex> g(mu_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto& t : th_) t.join();
    }
    int threads() const { return 1 + (int)th_.size(); }
    // Queues f.  Throws (std::bad_alloc) only before anything is counted.
    void submit(std::function<void()> f) {
        {
            std::lock_guard<std::mutex> g(mu_);
            q_.push_back(std::move(f));
            pending_.fetch_add(1, std::memory_order_relaxed);   // (under the lock: before any pop)
        }
        cv_.notify_one();
        done_cv_.notify_all();   // a waiter may run it
    }
    // Runs queued tasks until every submitted task (and what they submit) is
    // done, then rethrows the first exception a task threw.
    void wait_all() {
        help_until(pending_);
        rethrow();
    }
    // Runs queued tasks until `left` reaches 0 (never throws).
    void help_until(const std::atomic<int>& left) {
        while (left.load(std::memory_order_acquire) > 0) {
            if (run_one()) continue;
            std::unique_lock<std::mutex> g(mu_);
            done_cv_.wait(g, [&] { return left.load(std::memory_order_acquire) == 0 || !q_.empty(); });
        }
    }
    // f(c) for c in [0, nc), chunk 0 on this thread; returns when all are done
    // (rethrowing the first exception of any chunk once none is running).
    template <class F>
    void chunks(int nc, F&& f) {
        std::atomic<int> left{nc - 1};
        int queued = 0;
        try {
            for (int c = 1; c < nc; ++c, ++queued)
                submit([this, &f, &left, c] {
                    try {
                        f(c);
                    } catch (...) {
                        keep(std::current_exception());
                    }
                    left.fetch_sub(1, std::memory_order_acq_rel);
                });
            f(0);
        } catch (...) {
            keep(std::current_exception());
        }
        left.fetch_sub((nc - 1) - queued, std::memory_order_acq_rel);   // chunks never queued
        help_until(left);
        rethrow();
    }
    // Records an exception thrown on this thread by work that shares the pool
    // (the caller then waits with wait_all(), which rethrows it).
    void keep(std::exception_ptr e) {
        std::lock_guard<std::mutex> g(err_mu_);
        if (!err_) err_ = e;
    }

private:
    void rethrow() {
        std::exception_ptr e;
        {
            std::lock_guard<std::mutex> g(err_mu_);
            std::swap(e, err_);
        }
        if (e) std::rethrow_exception(e);
    }
    void run(std::function<void()>& f) {
        try {
            f();
        } catch (...) {
            keep(std::current_exception());
        }
    }
    bool run_one() {
        std::function<void()> f;
        {
            std::lock_guard<std::mutex> g(mu_);
            if (q_.empty()) return false;
            f = std::move(q_.front());
            q_.pop_front();
        }
        run(f);
        finished();
        return true;
    }
    // After a task: its counters have moved; wake the waiters (the empty
    // critical section orders this against a waiter's predicate check).
    void finished() {
        pending_.fetch_sub(1, std::memory_order_acq_rel);
        { std::lock_guard<std::mutex> g(mu_); }
        done_cv_.notify_all();
    }
    void work() {
        for (;;) {
            std::function<void()> f;
            {
                std::unique_lock<std::mutex> g(mu_);
                cv_.wait(g, [this] { return stop_ || !q_.empty(); });
                if (q_.empty()) return;   // stop_ with nothing queued
                f = std::move(q_.front());
                q_.pop_front();
            }
            run(f);
            finished();
        }
    }
    std::vector<std::thread> th_;
    std::mutex mu_;
    std::condition_variable cv_;        // workers: a task is queued (or stop)
    std::condition_variable done_cv_;   // waiters: a task finished or was queued
    std::deque<std::function<void()>> q_;
    std::atomic<int> pending_{0};
    bool stop_ = false;
    std::mutex err_mu_;
    std::exception_ptr err_;
};

#ifndef TPT_WIDE_BINS
#define TPT_WIDE_BINS 32   // (A/B builds: other bin counts)
#endif
constexpr int kBins = TPT_WIDE_BINS;
constexpr int kMaxThreads = 64;   // build threads at most (build_wide_sah)

struct alignas(16) Bins {   // the binned-SAH histogram of a range, all three axes
    VBox bb[3][kBins];
    int bn[3][kBins];
    void clear() {
        for (int a = 0; a < 3; ++a)
            for (int k = 0; k < kBins; ++k) {
                bb[a][k].empty();
                bn[a][k] = 0;
            }
    }
    void merge(const Bins& o) {   // exact: box unions and counts do not depend on order
        for (int a = 0; a < 3; ++a)
            for (int k = 0; k < kBins; ++k) {
                bb[a][k].grow(o.bb[a][k]);
                bn[a][k] += o.bn[a][k];
            }
    }
};

// Bin of each axis for centroid c: (int)((c - lo) * scale) clamped to [0, kBins)
// (a NaN or out-of-range product truncates to INT_MIN and lands in bin 0).
inline void bin_of(__m128 c, __m128 lo, __m128 scale, int k[4]) {
    _mm_storeu_si128(reinterpret_cast<__m128i*>(k), _mm_cvttps_epi32(_mm_mul_ps(_mm_sub_ps(c, lo), scale)));
    for (int j = 0; j < 3; ++j) k[j] = std::min(std::max(k[j], 0), kBins - 1);
}

struct Builder {
    int sweep_max = 32;   // ranges up to this size split by an exact sweep, larger ones binned
    Uninit<BNode> nodes;
    // The leaves, each subtree's range contiguous, in one of two buffers: a
    // split reads its range from one and writes both sides to the other.
    Uninit<Rec> buf[2];
    Pool* pool = nullptr;
    static constexpr int kParChunk = 8192;   // least records per thread of a parallel pass
    static constexpr int kTask = 2048;       // ranges at least this big are split as tasks of their own
    std::mutex upper_mu;
    std::vector<int> upper;                  // ids of the nodes split as tasks (finished after the tasks)

    static void cen_bounds(const Rec* r, int m, VBox& cb) {
        for (int i = 0; i < m; ++i) {
            const __m128 c = rec_cen(r[i]);
            cb.grow(c, c);
        }
    }

    // Stable insertion sort of (key, id) pairs by key: std::stable_sort's order.
    static void sort_pairs(float* kk, int* id, int m) {
        for (int i = 1; i < m; ++i) {
            const float kx = kk[i];
            const int x = id[i];
            int j = i;
            for (; j > 0 && kx < kk[j - 1]; --j) {
                kk[j] = kk[j - 1];
                id[j] = id[j - 1];
            }
            kk[j] = kx;
            id[j] = x;
        }
    }

    // Exact sweep over sorted centroids on each axis (each axis sorts the
    // previous axis's order, ties keep it; the range is then written to the
    // other buffer sorted, from its own order, by the chosen axis).  Returns
    // the split point; *w = the buffer now holding the range.
    int split_sweep(int b, int e, int* w) {
        const int m = e - b;
        const Rec* r = &buf[*w][b];
        double best = __builtin_inf();
        int best_axis = -1, best_m = -1;
        constexpr int kLocal = 64;
        alignas(16) float c_l[3][kLocal];
        float kk_l[kLocal];
        int ord_l[kLocal];
        double ra_l[kLocal];
        std::vector<float> c_v, kk_v;
        std::vector<int> ord_v;
        std::vector<double> ra_v;
        if (m > kLocal) {
            c_v.resize(3 * (size_t)m);
            kk_v.resize(m);
            ord_v.resize(m);
            ra_v.resize(m);
        }
        float* cx[3] = {m > kLocal ? c_v.data() : c_l[0], m > kLocal ? c_v.data() + m : c_l[1],
                        m > kLocal ? c_v.data() + 2 * m : c_l[2]};
        float* kk = m > kLocal ? kk_v.data() : kk_l;
        int* ord = m > kLocal ? ord_v.data() : ord_l;
        double* right_area = m > kLocal ? ra_v.data() : ra_l;
        for (int i = 0; i < m; ++i) {
            alignas(16) float c4[4];
            _mm_store_ps(c4, rec_cen(r[i]));
            for (int k = 0; k < 3; ++k) cx[k][i] = c4[k];
            ord[i] = i;
        }
        for (int axis = 0; axis < 3; ++axis) {
            for (int i = 0; i < m; ++i) kk[i] = cx[axis][ord[i]];
            sort_pairs(kk, ord, m);
            VBox acc;
            acc.empty();
            for (int i = m - 1; i > 0; --i) {
                acc.grow(r[ord[i]]);
                right_area[i] = acc.area();
            }
            acc.empty();
            for (int i = 1; i < m; ++i) {
                acc.grow(r[ord[i - 1]]);
                const double c = acc.area() * i + right_area[i] * (m - i);
                if (c < best) {
                    best = c;
                    best_axis = axis;
                    best_m = i;
                }
            }
        }
        if (best_axis < 0) {   // no finite cost (NaN boxes): halve by position
            halve_by_position(b, e, *w);
            return b + m / 2;
        }
        for (int i = 0; i < m; ++i) {
            kk[i] = cx[best_axis][i];
            ord[i] = i;
        }
        sort_pairs(kk, ord, m);
        Rec* dst = &buf[*w ^ 1][b];
        for (int i = 0; i < m; ++i) dst[i] = r[ord[i]];
        *w ^= 1;
        return b + best_m;
    }

    void halve_by_position(int b, int e, int w) {
        Rec* r = &buf[w][b];
        std::sort(r, r + (e - b), [](const Rec& x, const Rec& y) { return x.pos < y.pos; });
    }

    // Binned SAH split of buf[*w][b, e), centroid bounds cb, over nc threads:
    // one pass bins every axis per chunk, one scatters both sides (stable: the
    // left side is bins < best_m, each in its order) to the other buffer and
    // takes the two sides' centroid bounds cl / cr.  Returns the split point.
    int split_binned(int b, int e, const VBox& cb, int nc, int* w, VBox& cl, VBox& cr) {
        const int m = e - b;
        const Rec* src = &buf[*w][0];
        double best = __builtin_inf();
        int best_axis = -1, best_m = -1;
        alignas(16) float cl4[4], ch4[4], sc4[4] = {0.0f, 0.0f, 0.0f, 0.0f};
        _mm_store_ps(cl4, cb.lo);
        _mm_store_ps(ch4, cb.hi);
        bool live[3];
        for (int axis = 0; axis < 3; ++axis) {
            const float ext = ch4[axis] - cl4[axis];
            live[axis] = ext > 0.0f;
            sc4[axis] = kBins / ext;
        }
        const __m128 clo = cb.lo, scale = _mm_load_ps(sc4);
        auto chunk_lo = [&](int c) { return b + (int)((int64_t)m * c / nc); };
        // nc == 1 (every range below 2 chunks): one histogram on the stack, no
        // allocation, copy or merge -- a split of 33..16 K leaves is mostly this
        Bins one;
        std::vector<Bins> many;   // nc > 1: [0] the merged histogram, [c + 1] chunk c's
        if (nc > 1) many.resize(nc + 1);
        auto hist = [&](int c) -> Bins& { return nc > 1 ? many[c + 1] : one; };
        pool->chunks(nc, [&](int c) {
            Bins& h = hist(c);
            h.clear();
            const int i1 = chunk_lo(c + 1);
            for (int i = chunk_lo(c); i < i1; ++i) {
                const Rec& q = src[i];
                const __m128 lo = rec_lo(q), hi = rec_hi(q);
                alignas(16) int k[4];
                bin_of(_mm_mul_ps(_mm_set1_ps(0.5f), _mm_add_ps(lane3_zero(lo), lane3_zero(hi))), clo, scale, k);
                for (int axis = 0; axis < 3; ++axis) {
                    ++h.bn[axis][k[axis]];
                    h.bb[axis][k[axis]].grow(lo, hi);
                }
            }
        });
        Bins& h = nc > 1 ? many[0] : one;
        if (nc > 1) {
            h = many[1];
            for (int c = 1; c < nc; ++c) h.merge(many[c + 1]);
        }
        for (int axis = 0; axis < 3; ++axis) {
            if (!live[axis]) continue;
            double ra[kBins];
            int rn[kBins];
            VBox acc;
            acc.empty();
            int cnt = 0;
            for (int k = kBins - 1; k > 0; --k) {
                acc.grow(h.bb[axis][k]);
                cnt += h.bn[axis][k];
                ra[k] = acc.area();
                rn[k] = cnt;
            }
            acc.empty();
            cnt = 0;
            for (int k = 1; k < kBins; ++k) {
                acc.grow(h.bb[axis][k - 1]);
                cnt += h.bn[axis][k - 1];
                if (cnt == 0 || rn[k] == 0) continue;
                const double c = acc.area() * cnt + ra[k] * rn[k];
                if (c < best) {
                    best = c;
                    best_axis = axis;
                    best_m = k;
                }
            }
        }
        cl.empty();
        cr.empty();
        if (best_axis < 0) {   // all centroids coincide: halve by position
            halve_by_position(b, e, *w);
            cen_bounds(src + b, m / 2, cl);
            cen_bounds(src + b + m / 2, m - m / 2, cr);
            return b + m / 2;
        }
        const int ax = best_axis;
        // each chunk's left count from its own histogram
        int nl[kMaxThreads + 1];   // (nc <= the pool's threads <= kMaxThreads)
        nl[0] = 0;
        for (int c = 0; c < nc; ++c) {
            int k = 0;
            const Bins& hc = hist(c);
            for (int j = 0; j < best_m; ++j) k += hc.bn[ax][j];
            nl[c + 1] = nl[c] + k;
        }
        const int s = b + nl[nc];
        Rec* dst = &buf[*w ^ 1][0];
        VBox bl[kMaxThreads], br[kMaxThreads];
        pool->chunks(nc, [&](int c) {
            const int i0 = chunk_lo(c), i1 = chunk_lo(c + 1);
            int ol = b + nl[c], orr = s + (i0 - b - nl[c]);
            VBox xl, xr;
            xl.empty();
            xr.empty();
            for (int i = i0; i < i1; ++i) {
                const Rec& q = src[i];
                const __m128 cen = _mm_mul_ps(_mm_set1_ps(0.5f), _mm_add_ps(lane3_zero(rec_lo(q)), lane3_zero(rec_hi(q))));
                alignas(16) int k[4];
                bin_of(cen, clo, scale, k);
                if (k[ax] < best_m) {
                    dst[ol++] = q;
                    xl.grow(cen, cen);
                } else {
                    dst[orr++] = q;
                    xr.grow(cen, cen);
                }
            }
            bl[c] = xl;
            br[c] = xr;
        });
        for (int c = 0; c < nc; ++c) {
            cl.grow(bl[c]);
            cr.grow(br[c]);
        }
        *w ^= 1;
        return s;   // (b < s < e: both sides of best_m hold records)
    }

    // Splits buf[w][b, e) (centroid bounds cb when it is binned) into
    // nodes[id]'s two children.  Returns the split point; *w = the buffer
    // now holding the range.
    int split(int b, int e, const VBox& cb, int* w, VBox& cl, VBox& cr) {
        if (e - b <= sweep_max) return split_sweep(b, e, w);
        const int nc = std::max(1, std::min(pool->threads(), (e - b) / kParChunk));
        return split_binned(b, e, cb, nc, w, cl, cr);
    }

    void make_leaf(int id, const Rec& q, const uint32_t* emit) {
        BNode& nd = nodes[id];
        nd.pos = q.pos;
        for (int k = 0; k < 3; ++k) {
            nd.box.lo[k] = q.lo[k];
            nd.box.hi[k] = q.hi[k];
        }
        nd.emit = emit[q.pos] ? 1u : 0u;
        nd.left = nd.right = -1;
        collapse_cost(id);
    }

    void finish(int id, int l, int r) {   // an inner node once both children are complete
        BNode& nd = nodes[id];
        nd.left = l;
        nd.right = r;
        nd.pos = -1;
        nd.box = nodes[l].box;
        nd.box.grow(nodes[r].box);
        nd.emit = nodes[l].emit | nodes[r].emit;
        collapse_cost(id);
    }

    // Builds buf[w][b, e) as the subtree rooted at nodes[id] on this thread.
    // Every leaf holds one triangle, so a subtree of m leaves has 2m - 1 nodes
    // and its pre-order ids are known before it is built: the left child is
    // id + 1, the right child id + 2 * (left leaves).
    void build_serial(int b, int e, int id, const uint32_t* emit, const VBox& cb, int w) {
        if (e - b == 1) {
            make_leaf(id, buf[w][b], emit);
            return;
        }
        VBox cl, cr;
        const int s = split(b, e, cb, &w, cl, cr);
        const int l = id + 1, r = id + 2 * (s - b);
        build_serial(b, s, l, emit, cl, w);
        build_serial(s, e, r, emit, cr, w);
        finish(id, l, r);
    }

    // A range of at least kTask leaves: split here, children of kTask or more
    // leaves go back to the pool as tasks, smaller ones build on this thread.
    // The node itself is finished after every task has run (build_wide_sah,
    // in decreasing id order: children before parents).  Ids, ranges and
    // buffers are fixed by the split alone, so the tree is identical to a
    // serial build's whatever thread runs what.
    void build_task(int b, int e, int id, const uint32_t* emit, VBox cb, int w) {
        VBox cl, cr;
        const int s = split(b, e, cb, &w, cl, cr);
        const int l = id + 1, r = id + 2 * (s - b);
        nodes[id].left = l;
        nodes[id].right = r;
        {
            std::lock_guard<std::mutex> g(upper_mu);
            upper.push_back(id);
        }
        auto child = [&](int cb_, int ce, int cid, const VBox& ccb) {
            if (ce - cb_ >= kTask)
                pool->submit([this, cb_, ce, cid, emit, ccb, w] { build_task(cb_, ce, cid, emit, ccb, w); });
            else
                build_serial(cb_, ce, cid, emit, ccb, w);
        };
        child(s, e, r, cr);   // (queued first: FIFO hands it to another thread)
        child(b, s, l, cl);
    }

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

struct WideWorkspace::Impl {
    Uninit<BNode> nodes;
    Uninit<Rec> buf[2];
    Uninit<std::array<double, 5>> D;
    Uninit<std::array<int8_t, 5>> pick;
    Uninit<int> wide_of;
};
WideWorkspace::WideWorkspace() : impl(new Impl) {}
WideWorkspace::~WideWorkspace() = default;

namespace {
// Lends a workspace's arrays to a build and takes them back (also when the
// build throws: the storage is kept for the next one).
struct Lend {
    WideWorkspace::Impl* w;
    Builder& b;
    Uninit<int>& wide_of;
    Lend(WideWorkspace* ws, Builder& b_, Uninit<int>& wo) : w(ws ? ws->impl.get() : nullptr), b(b_), wide_of(wo) {
        swap_all();
    }
    ~Lend() { swap_all(); }
    void swap_all() {
        if (!w) return;
        b.nodes.swap(w->nodes);
        b.buf[0].swap(w->buf[0]);
        b.buf[1].swap(w->buf[1]);
        b.D.swap(w->D);
        b.pick.swap(w->pick);
        wide_of.swap(w->wide_of);
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
                   int id_base, HostFloats& out, int* stack_need, const WideParams& prm) {
    const int n = (int)pos.size();
    out.clear();
    *stack_need = 0;
    if (n == 0) return 0;
    const bool timing = std::getenv("TPT_BUILD_TIMING") != nullptr;
    auto t_last = std::chrono::steady_clock::now();
    auto mark = [&](const char* what) {
        if (!timing) return;
        const auto t = std::chrono::steady_clock::now();
        std::fprintf(stderr, "  wide tree (%d leaves) %-8s %8.3f ms\n", n, what,
                     std::chrono::duration<double, std::milli>(t - t_last).count());
        t_last = t;
    };
    // threads: at most prm.threads (< 0: the cores this process may use; 0 or
    // 1: a serial build -- the same tree), and about one per 4 K leaves
    const int hw = std::max(1, std::min(prm.threads < 0 ? usable_cores() : prm.threads, kMaxThreads));
    Pool pool(std::min(hw, n / 4096 + 1));
    Builder B;
    Uninit<int> wide_of;   // binary node -> 4-wide node id (set for every node that becomes one)
    Lend lend(prm.ws, B, wide_of);
    B.pool = &pool;
    B.sweep_max = prm.sweep_max;
    B.buf[0].reset(n);
    B.buf[1].reset(n);
    // the leaf records and the root's centroid bounds, in chunks (merged exactly)
    const int nc = std::max(1, std::min(pool.threads(), n / Builder::kParChunk));
    std::vector<VBox> cbs(nc);
    pool.chunks(nc, [&](int c) {
        const int i0 = (int)((int64_t)n * c / nc), i1 = (int)((int64_t)n * (c + 1) / nc);
        for (int i = i0; i < i1; ++i) {
            const int p = pos[i];
            Rec& q = B.buf[0][i];
            for (int k = 0; k < 3; ++k) {
                q.lo[k] = leaf_box[6 * p + k];
                q.hi[k] = leaf_box[6 * p + 3 + k];
            }
            q.pos = p;
            q.pad = 0.0f;
        }
        cbs[c].empty();
        Builder::cen_bounds(&B.buf[0][i0], i1 - i0, cbs[c]);
    });
    VBox cb;
    cb.empty();
    for (const VBox& x : cbs) cb.grow(x);
    B.nodes.reset(2 * (size_t)n - 1);
    B.D.reset(B.nodes.size());
    B.pick.reset(B.nodes.size());
    const int root = 0;
    mark("setup");
    if (n >= Builder::kTask) {
        try {
            B.build_task(0, n, root, leaf_emit, cb, 0);
        } catch (...) {   // tasks it queued may still run: they reference B
            pool.keep(std::current_exception());
        }
        pool.wait_all();   // (rethrows once no task is left)
        std::sort(B.upper.begin(), B.upper.end(), std::greater<int>());
        for (int id : B.upper) B.finish(id, B.nodes[id].left, B.nodes[id].right);
    } else {
        B.build_serial(0, n, root, leaf_emit, cb, 0);
    }
    mark("binary");
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
    const auto& pick = B.pick;
    // Stack bound: a visit of node X finds at most A(X) entries on the stack --
    // the deferred siblings of X and of its ancestors, A(X) = sum over the
    // proper ancestors a of (children(a) - 1) -- and leaves at most A(X) +
    // children(X) - 1.
    struct Wide {
        int kids[4];
        int nk;
        int above;   // A(X)
        int b;       // the binary node it stands for
    };
    auto expand = [&](int b, int above) {   // (x, k): x's children as a forest of at most k roots
        Wide w;
        w.nk = 0;
        w.above = above;
        w.b = b;
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
        return w;
    };
    // Node ids are breadth-first.  The top levels are expanded level by level
    // here until a level holds enough nodes to share out; below that level
    // each of its nodes' subtrees is walked depth-first (children in order) on
    // whichever thread takes it.  A depth-first walk meets a level's nodes in
    // their left-to-right order, so the breadth-first id of a node at level L
    // is: the nodes above L, then level L's nodes of the subtrees before its
    // own, then its rank in its own subtree's level-L list.
    std::vector<Wide> top;
    std::vector<int> front{root}, front_above{0};
    const int kCut = 64;
    while (!front.empty() && (int)front.size() < kCut) {
        std::vector<int> nx, nx_above;
        for (size_t i = 0; i < front.size(); ++i) {
            const Wide w = expand(front[i], front_above[i]);
            top.push_back(w);
            for (int k = 0; k < w.nk; ++k)
                if (N[w.kids[k]].left >= 0) {
                    nx.push_back(w.kids[k]);
                    nx_above.push_back(w.above + w.nk - 1);
                }
        }
        front.swap(nx);
        front_above.swap(nx_above);
    }
    const int nt = (int)front.size();
    std::vector<std::vector<std::vector<Wide>>> lists(nt);   // [subtree][depth below the cut]
    std::vector<int> task_need(nt, 0);
    const int nth = std::max(1, std::min(pool.threads(), nt));
    auto for_tasks = [&](auto&& f) {   // subtrees handed out one at a time
        std::atomic<int> next{0};
        pool.chunks(nth, [&](int) {
            for (int t; (t = next.fetch_add(1, std::memory_order_relaxed)) < nt;) f(t);
        });
    };
    for_tasks([&](int t) {
        struct Item {
            int b, above, depth;
        };
        std::vector<Item> st{{front[t], front_above[t], 0}};
        auto& L = lists[t];
        int nd = 0;
        while (!st.empty()) {
            const Item it = st.back();
            st.pop_back();
            const Wide w = expand(it.b, it.above);
            if ((int)L.size() <= it.depth) L.resize(it.depth + 1);
            L[it.depth].push_back(w);
            nd = std::max(nd, w.above + w.nk - 1);
            for (int k = w.nk - 1; k >= 0; --k)
                if (N[w.kids[k]].left >= 0) st.push_back({w.kids[k], w.above + w.nk - 1, it.depth + 1});
        }
        task_need[t] = nd;
    });
    int need = 0;
    for (const Wide& w : top) need = std::max(need, w.above + w.nk - 1);
    for (int t = 0; t < nt; ++t) need = std::max(need, task_need[t]);
    size_t depth = 0;
    for (const auto& L : lists) depth = std::max(depth, L.size());
    std::vector<std::vector<int>> first(nt, std::vector<int>(depth, 0));   // id of lists[t][d][0]
    int total = (int)top.size();
    for (size_t d = 0; d < depth; ++d)
        for (int t = 0; t < nt; ++t) {
            first[t][d] = total;
            if (d < lists[t].size()) total += (int)lists[t][d].size();
        }
    wide_of.reset(N.size());
    for (size_t i = 0; i < top.size(); ++i) wide_of[top[i].b] = (int)i;
    out.resize(32 * (size_t)total);
    auto emit_node = [&](const Wide& w, int id) {   // all 32 floats: unused slots zero boxes, link -1; pad 0
        float* q = out.data() + 32 * (size_t)id;
        int32_t links[4] = {-1, -1, -1, -1};
        for (int k = 0; k < 4; ++k) {
            if (k >= w.nk) {
                for (int j = 0; j < 6; ++j) q[6 * k + j] = 0.0f;
                continue;
            }
            const BNode& c = N[w.kids[k]];
            for (int j = 0; j < 3; ++j) {
                q[6 * k + j] = c.box.lo[j];
                q[6 * k + 3 + j] = c.box.hi[j];
            }
            const int32_t cid = c.left >= 0 ? id_base + wide_of[w.kids[k]] : leaf_base + c.pos;
            links[k] = cid | (int32_t)(c.emit << 30);
        }
        std::memcpy(q + 24, links, sizeof links);
        for (int j = 28; j < 32; ++j) q[j] = 0.0f;
    };
    for_tasks([&](int t) {   // a subtree's ids, then its nodes (their children lie in the same subtree)
        const auto& L = lists[t];
        for (size_t d = 0; d < L.size(); ++d)
            for (size_t j = 0; j < L[d].size(); ++j) wide_of[L[d][j].b] = first[t][d] + (int)j;
        for (size_t d = 0; d < L.size(); ++d)
            for (size_t j = 0; j < L[d].size(); ++j) emit_node(L[d][j], first[t][d] + (int)j);
    });
    for (size_t i = 0; i < top.size(); ++i) emit_node(top[i], (int)i);
    mark("collapse");
    *stack_need = need;
    return total;
}

}  // namespace tpt

extern "C" int32_t tpt_wide_tree_build(int32_t n, const float* leaf_box, const uint32_t* leaf_emit, float* nodes,
                                       int32_t cap, int32_t* stack_need, int32_t threads) {
    if (n < 2 || !leaf_box || !leaf_emit || cap < 0) return -1;
    tpt::HostFloats out;
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
