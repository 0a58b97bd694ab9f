// libmeshsearch C ABI (include/meshsearch.h): handle management, host<->HBM staging, validation and
// error mapping around the HIP kernels.  Mirrors the entry points of the reference's extensions:
//   spatialsearch  (mesh/src/spatialsearchmodule.cpp)   aabbtree_compute / _nearest / _nearest_alongnormal
//                                                         / _intersections_indices
//   aabb_normals   (mesh/src/aabb_normals.cpp)          aabbtree_n_compute / _n_nearest / _n_selfintersects
//   visibility     (mesh/src/py_visibility.cpp)         visibility_compute
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <chrono>
#include <map>
#include <atomic>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <set>
#include <string>
#include <thread>
#include <vector>

#include "internal.h"

namespace msh {

static thread_local std::string g_err;
static thread_local int g_device = -1;
// devices of the trees built next on this thread (msh_set_devices / msh_set_device_list); empty: one device
static thread_local std::vector<int> g_devices;

void set_error(const char* fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_err = buf;
}

static void release_idle_device(int dev);  // idle pooled workspaces / staging slabs of a device (below)

// Device allocations of the library (tree buffers, build temporaries, scratch) go through one process-wide cache: a
// freed block is kept for the next request of a similar size on its device instead of being unmapped, so a caller
// that builds a tree per call (Mesh.closest_faces_and_points; C4's batched build + query: ~11 GB of buffers per
// call) does not pay hipMalloc / hipFree of gigabytes every time.  A free waits for the device as hipFree does (a
// block still read by queued launches is never handed out again), the cache holds at most MESH_AMD_DEVICE_CACHE_MB
// (default 16384; 0 turns it off) and msh_device_pool_trim empties it.
class DevCache {
  public:
    hipError_t alloc(void** p, size_t bytes) {
        int dev = 0;
        hipError_t e = hipGetDevice(&dev);
        if (e != hipSuccess) return e;
        const size_t want = grain(bytes);
        if (cap() > 0) {
            std::lock_guard<std::mutex> g(mu_);
            auto& fl = free_[dev];
            auto it = fl.lower_bound(want);
            if (it != fl.end() && it->first <= want + want / 4) {
                *p = it->second;
                cached_ -= it->first;
                fl.erase(it);
                return hipSuccess;
            }
        }
        e = hipMalloc(p, want);
        if (e == hipErrorOutOfMemory) {
            // everything the library holds idle on this device goes first: the idle query workspace and staging
            // slabs (their blocks come back into this cache), then the cached blocks themselves.  No lock of
            // this cache is held here, so the pools' lock -> cache lock order is kept.
            (void)hipGetLastError();
            release_idle_device(dev);
            trim_device(dev);
            e = hipMalloc(p, want);
        }
        if (e != hipSuccess) return e;
        std::lock_guard<std::mutex> g(mu_);
        blocks_[*p] = Blk{want, dev};
        return hipSuccess;
    }
    hipError_t free(void* p) {
        if (!p) return hipSuccess;
        Blk b;
        {
            std::lock_guard<std::mutex> g(mu_);
            auto it = blocks_.find(p);
            if (it == blocks_.end()) return hipFree(p);  // not ours
            b = it->second;
            if (cap() == 0) {
                blocks_.erase(it);
                return hipFree(p);
            }
        }
        int cur = -1;
        (void)hipGetDevice(&cur);
        if (cur != b.dev) (void)hipSetDevice(b.dev);
        const hipError_t e = hipDeviceSynchronize();  // the wait hipFree would make
        if (cur != b.dev && cur >= 0) (void)hipSetDevice(cur);
        std::vector<std::pair<void*, int>> drop;
        {
            std::lock_guard<std::mutex> g(mu_);
            free_[b.dev].emplace(b.bytes, p);
            cached_ += b.bytes;
            while (cached_ > cap()) {  // over the cap: unmap the largest cached blocks
                std::multimap<size_t, void*>* big = nullptr;
                int bd = 0;
                for (auto& kv : free_)
                    if (!kv.second.empty() && (!big || std::prev(kv.second.end())->first > std::prev(big->end())->first)) {
                        big = &kv.second;
                        bd = kv.first;
                    }
                if (!big) break;
                auto last = std::prev(big->end());
                cached_ -= last->first;
                blocks_.erase(last->second);
                drop.emplace_back(last->second, bd);
                big->erase(last);
            }
        }
        for (auto& d : drop) unmap(d.first, d.second);
        return e;
    }
    size_t trim() {
        std::vector<std::pair<void*, int>> drop;
        size_t n = 0;
        {
            std::lock_guard<std::mutex> g(mu_);
            for (auto& kv : free_) {
                for (auto& x : kv.second) {
                    n += x.first;
                    blocks_.erase(x.second);
                    drop.emplace_back(x.second, kv.first);
                }
                kv.second.clear();
            }
            cached_ = 0;
        }
        for (auto& d : drop) unmap(d.first, d.second);
        return n;
    }
    size_t cached() {
        std::lock_guard<std::mutex> g(mu_);
        return cached_;
    }

  private:
    struct Blk {
        size_t bytes = 0;
        int dev = 0;
    };
    static size_t grain(size_t n) {
        if (n == 0) n = 16;
        const size_t g = n >= ((size_t)1 << 20) ? ((size_t)2 << 20) : 4096;
        return (n + g - 1) / g * g;
    }
    static size_t cap() {
        static const size_t c = [] {
            const char* e = getenv("MESH_AMD_DEVICE_CACHE_MB");
            const long long mb = e ? atoll(e) : 16384;
            return mb > 0 ? (size_t)mb << 20 : (size_t)0;
        }();
        return c;
    }
    static void unmap(void* p, int dev) {
        int cur = -1;
        (void)hipGetDevice(&cur);
        if (cur != dev) (void)hipSetDevice(dev);
        (void)hipFree(p);
        if (cur != dev && cur >= 0) (void)hipSetDevice(cur);
    }
    void trim_device(int dev) {
        std::vector<std::pair<void*, int>> drop;
        {
            std::lock_guard<std::mutex> g(mu_);
            for (auto& x : free_[dev]) {
                cached_ -= x.first;
                blocks_.erase(x.second);
                drop.emplace_back(x.second, dev);
            }
            free_[dev].clear();
        }
        for (auto& d : drop) unmap(d.first, d.second);
    }
    std::mutex mu_;
    std::map<void*, Blk> blocks_;                     // every block this cache allocated (handed out or cached)
    std::map<int, std::multimap<size_t, void*>> free_;  // cached blocks per device, by size
    size_t cached_ = 0;
};
static DevCache& dev_cache() {
    static DevCache* c = new DevCache;  // never destroyed: the runtime may be gone at static destruction
    return *c;
}
hipError_t dmalloc_raw(void** p, size_t bytes) { return dev_cache().alloc(p, bytes); }
hipError_t dfree(void* p) { return dev_cache().free(p); }
size_t dcache_trim() { return dev_cache().trim(); }
size_t dcache_bytes() { return dev_cache().cached(); }

int DevBuf::reserve(size_t need) {
    if (need <= bytes && ptr) return MSH_OK;
    if (ptr) {
        hipError_t e = dfree(ptr);
        ptr = nullptr;
        bytes = 0;
        MSH_HIP(e);
    }
    if (need == 0) need = 16;
    MSH_HIP(dmalloc(&ptr, need));
    bytes = need;
    return MSH_OK;
}

void DevBuf::release() {
    if (ptr) (void)dfree(ptr);
    ptr = nullptr;
    bytes = 0;
}

void Workspace::release() {
    DevBuf* all[] = {&keys, &vals, &keys_alt, &vals_alt, &hist, &scan, &q, &n, &out_a, &out_b, &out_c, &out_d,
                     &flags, &counters, &spill, &stats, &ranges, &qs, &ns, &inv, &res, &res_w, &resume, &p2cand};
    for (DevBuf* b : all) b->release();
}

size_t Workspace::bytes() const {
    const DevBuf* all[] = {&keys, &vals, &keys_alt, &vals_alt, &hist, &scan, &q, &n, &out_a, &out_b, &out_c, &out_d,
                           &flags, &counters, &spill, &stats, &ranges, &qs, &ns, &inv, &res, &res_w, &resume, &p2cand};
    size_t t = 0;
    for (const DevBuf* b : all) t += b->bytes;
    return t;
}

// Query workspaces handed from a freed triangle tree to the next one built on the device.  A caller that builds a
// tree per query batch — the reference's Mesh.closest_faces_and_points (mesh.py:454-455) — otherwise allocated and
// freed the whole query workspace per call (~8 GB of device buffers at 100M queries).  free_tree gives the
// workspace back only after the tree's work has finished; one idle workspace is kept per device, others are freed.
class WsPool {
  public:
    void give(int dev, Workspace& ws) {
        std::lock_guard<std::mutex> g(mu_);
        idle_[dev] = std::move(ws);  // keep the newest (move-assignment frees the one it replaces)
    }
    void take(int dev, Workspace& ws) {
        std::lock_guard<std::mutex> g(mu_);
        auto it = idle_.find(dev);
        if (it == idle_.end()) return;
        ws = std::move(it->second);
        idle_.erase(it);
    }
    // frees every idle workspace; returns the bytes released
    size_t trim() {
        std::lock_guard<std::mutex> g(mu_);
        size_t n = 0;
        int cur = 0;
        const bool have = hipGetDevice(&cur) == hipSuccess;
        for (auto& kv : idle_) {
            n += kv.second.bytes();
            (void)hipSetDevice(kv.first);
            kv.second.release();
        }
        if (have) (void)hipSetDevice(cur);
        idle_.clear();
        return n;
    }
    size_t bytes() {
        std::lock_guard<std::mutex> g(mu_);
        size_t n = 0;
        for (auto& kv : idle_) n += kv.second.bytes();
        return n;
    }
    // the idle workspace of one device (the caller is on that device)
    void trim_device(int dev) {
        Workspace ws;
        take(dev, ws);
        ws.release();
    }

  private:
    std::mutex mu_;
    std::map<int, Workspace> idle_;
};
static WsPool& ws_pool() {
    static WsPool* p = new WsPool;  // never destroyed: the runtime may be gone at static destruction
    return *p;
}

// ---- kernel timing ----
struct Pending {
    std::string name;
    hipEvent_t a, b;
};
static std::mutex g_tmu;
static bool g_timing = false;
static std::vector<Pending> g_pending;
static std::map<std::string, std::pair<double, int64_t>> g_times;

TimedLaunch::TimedLaunch(const char* n, hipStream_t st) : name(n), s(st) {
    std::lock_guard<std::mutex> g(g_tmu);
    if (!g_timing) return;
    if (hipEventCreate(&a) != hipSuccess || hipEventCreate(&b) != hipSuccess) {
        a = b = nullptr;
        return;
    }
    (void)hipEventRecord(a, s);
}

TimedLaunch::~TimedLaunch() {
    if (!a) return;
    (void)hipEventRecord(b, s);
    std::lock_guard<std::mutex> g(g_tmu);
    g_pending.push_back(Pending{name, a, b});
}

// host-side intervals under the same names (msh_timing_get): the host pipeline's copies and waits
static void host_time(const char* name, std::chrono::steady_clock::time_point t0) {
    const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    std::lock_guard<std::mutex> g(g_tmu);
    if (!g_timing) return;
    auto& t = g_times[name];
    t.first += ms;
    t.second += 1;
}

static void resolve_pending() {
    std::vector<Pending> p;
    {
        std::lock_guard<std::mutex> g(g_tmu);
        p.swap(g_pending);
    }
    for (auto& e : p) {
        float ms = 0.f;
        if (hipEventSynchronize(e.b) == hipSuccess && hipEventElapsedTime(&ms, e.a, e.b) == hipSuccess) {
            std::lock_guard<std::mutex> g(g_tmu);
            auto& t = g_times[e.name];
            t.first += ms;
            t.second += 1;
        }
        (void)hipEventDestroy(e.a);
        (void)hipEventDestroy(e.b);
    }
}

static int use_device(int dev) {
    MSH_HIP(hipSetDevice(dev));
    return MSH_OK;
}

static int current_device(int* dev) {
    if (g_device >= 0) {
        *dev = g_device;
        return MSH_OK;
    }
    int d = 0;
    MSH_HIP(hipGetDevice(&d));
    *dev = d;
    return MSH_OK;
}

static int check_faces(const uint32_t* f, size_t T, size_t P, const char* what) {
    for (size_t i = 0; i < 3 * T; ++i) {
        if (f[i] >= P) {
            set_error("%s: face %zu references vertex %u but only %zu vertices were given", what, i / 3, f[i], P);
            return MSH_EINVAL;
        }
    }
    return MSH_OK;
}

// queries, rays and permutation slots are 32-bit indices on the device
static int check_count(size_t S, const char* fn) {
    if (S > (size_t)0xFFFFFFFFull) {
        set_error("%s: %zu queries exceed the 32-bit index range of one call (split the batch)", fn, S);
        return MSH_EINVAL;
    }
    return MSH_OK;
}

template <class T>
static int upload(DevBuf& buf, const T* host, size_t n, hipStream_t s) {
    MSH_TRY(buf.reserve(n * sizeof(T)));
    if (n) MSH_HIP(hipMemcpyAsync(buf.ptr, host, n * sizeof(T), hipMemcpyHostToDevice, s));
    return MSH_OK;
}

// End of an asynchronous batched build: wait for its last kernel, free its temporaries, read its GPU time.  A kernel
// failure of the build surfaces here (MSH_EDEVICE), at the first call that needs the tree.
static int finish_pending(msh_tree* t) {
    if (!t->pending) return MSH_OK;
    (void)hipSetDevice(t->device);
    const hipError_t e = hipEventSynchronize(t->pend_done);
    float ms = 0.f;
    if (e == hipSuccess && hipEventElapsedTime(&ms, t->pend_e0, t->pend_done) == hipSuccess) t->build_ms += ms;
    for (void* p : t->pend_free)
        if (p) (void)dfree(p);
    t->pend_free.clear();
    t->pend_ws.release();
    (void)hipEventDestroy(t->pend_e0);
    (void)hipEventDestroy(t->pend_done);
    t->pend_e0 = t->pend_done = nullptr;
    t->pending = false;
    if (e != hipSuccess) {
        set_error("batched LBVH build failed: %s", hipGetErrorString(e));
        return MSH_EDEVICE;
    }
    return MSH_OK;
}

static void free_tree(msh_tree* t) {
    if (!t) return;
    if (t->pending) {
        const std::string keep = g_err;
        (void)finish_pending(t);
        g_err = keep;
    }
    for (msh_tree* r : t->replicas) free_tree(r);
    t->replicas.clear();
    (void)hipSetDevice(t->device);
    if (t->stream) (void)hipStreamSynchronize(t->stream);
    if (t->ws_done) (void)hipEventSynchronize(t->ws_done);
    // triangle trees (single, batched, normals metric) took one when they were built, if one was idle
    if (t->kind != kPoints) ws_pool().give(t->device, t->ws);
    t->ws.release();
    if (t->d_v) (void)dfree(t->d_v);
    if (t->d_nodes) (void)dfree(t->d_nodes);
    if (t->d_orgs) (void)dfree(t->d_orgs);
    if (t->d_boxes) (void)dfree(t->d_boxes);
    if (t->d_leaves) (void)dfree(t->d_leaves);
    if (t->d_vorder) (void)dfree(t->d_vorder);
    if (t->d_vorder_shard) (void)dfree(t->d_vorder_shard);
    if (t->d_cut) (void)dfree(t->d_cut);
    if (t->d_face_leaf) (void)dfree(t->d_face_leaf);
    for (int b = 0; b < 3; ++b) {
        if (b < 2 && t->h_stage[b]) (void)hipHostFree(t->h_stage[b]);
        if (t->d_stage[b]) (void)dfree(t->d_stage[b]);
        if (t->e_up[b]) (void)hipEventDestroy(t->e_up[b]);
        if (t->e_run[b]) (void)hipEventDestroy(t->e_run[b]);
        if (t->e_down[b]) (void)hipEventDestroy(t->e_down[b]);
    }
    if (t->s_up) (void)hipStreamDestroy(t->s_up);
    if (t->s_down) (void)hipStreamDestroy(t->s_down);
    if (t->ws_done) (void)hipEventDestroy(t->ws_done);
    if (t->stream) (void)hipStreamDestroy(t->stream);
    delete t;
}

static int new_tree(int kind, msh_tree** out) {
    int dev = 0;
    MSH_TRY(current_device(&dev));
    MSH_TRY(use_device(dev));
    msh_tree* t = new msh_tree();
    t->device = dev;
    t->kind = kind;
    // A blocking stream: it orders with the legacy default stream, so a caller that queues its inputs there (torch's
    // default stream is handle 0, which the *_device entry points read as "the handle's own stream") and then
    // passes NULL sees its writes before the handle's kernels read them, and its later default-stream work after
    // them.  (A non-blocking stream here let the C3 query order read rows torch's generator was still writing.)
    hipError_t e = hipStreamCreateWithFlags(&t->stream, hipStreamDefault);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&t->ws_done, hipEventDisableTiming);
    if (e != hipSuccess) {
        set_error("hipStreamCreate / hipEventCreate failed on device %d: %s", dev, hipGetErrorString(e));
        free_tree(t);
        return MSH_EDEVICE;
    }
    *out = t;
    return MSH_OK;
}

// Stream ordering of the handle's workspace: every launch sequence that uses `ws` first waits for the
// previous one (whatever stream it ran on) and then marks its own end, so a *_device call on a
// caller's stream followed by any other call on the same handle cannot overwrite scratch still in use.
struct WsOrder {
    msh_tree* t;
    hipStream_t s;
    WsOrder(msh_tree* tree, hipStream_t st) : t(tree), s(st) {
        if (t->ws_done) (void)hipStreamWaitEvent(s, t->ws_done, 0);
    }
    ~WsOrder() {
        if (t->ws_done) (void)hipEventRecord(t->ws_done, s);
    }
};

// Entry cut of a single triangle tree (nearest.hip cut_start / k_cut_build): a G^3 grid over the scene box
// widened by 1/4 on every side (each axis at least 1/20 of the largest, so flat meshes get cells of a sane
// shape), MSH_CUT_PER_LEAF cells per leaf up to 2^MSH_CUT_MAX_LOG2 cells (below; round 3 with leader phases:
// G = 64 / 126 / 160: 1718 / 1742-1765 / 1782 M q/s against 1789-1800 at G = 200); the cell centres are answered
// by the tree itself, then every cell's start entries are cut from the root.  Trees under kCutMinLeaves
// leaves start at the root (their top levels are few).  Built lazily (ensure_entry_cut): the automatic grid once the
// handle's closest-point and alongnormal calls have brought enough rows (ensure_entry_cut), so visibility and
// normals-metric trees and a few small calls never pay its memory or build time; msh_tree_set_entry_cut chooses the
// grid (built by the next closest-point or alongnormal call) or turns it off.
constexpr size_t kCutMinLeaves = 4096;
enum { kCutPending = 0, kCutBuilt = 1, kCutOff = 2, kCutFailed = 3 };

static bool cut_applies(const msh_tree* t) {
    return t->kind == kTriangles && t->B == 1 && !t->d_boxes && t->T >= kCutMinLeaves && t->d_nodes && t->cut_req != 0;
}

static void free_entry_cut(msh_tree* t) {
    if (t->d_cut) {
        (void)hipSetDevice(t->device);
        if (t->ws_done) (void)hipEventSynchronize(t->ws_done);  // no launch may still read the cut
        (void)dfree(t->d_cut);
    }
    t->d_cut = nullptr;
    t->cut_G = 0;
    t->cut_ms = 0.0;
}

// The automatic grid comes in two sizes (round 6).  A coarse grid, 8 cells per leaf (at most 2^23 cells; C3: G = 200,
// 256 MB), is built by the call that brings the handle's rows to 1/16 of its cells (C3: 500k rows); it costs a
// one-shot caller ~10 ms.  The fine grid, 64 cells per leaf (at most 2^26; C3: G = 400, 2.05 GB), replaces it once the
// handle has answered kFineRowsPerCell rows per fine cell (C3: ~1G rows): its ~46-ms build pays back after that many
// queries (C3 100M-query batches: ~3 ms faster each than with the coarse grid).  msh_tree_set_entry_cut(t, -1) asks
// for the fine grid at the next call (a caller that keeps the tree for many batches, as bench.py does).
// Round-5 figures (68-B cells of 8 entries and a separate hint), C3 in M q/s: 8 per leaf, 2^23 cells: G = 200, 46.9
// node visits per query, 2156-2213; 16, 2^25: G = 252, 45.2 visits, 2238; 32, 2^25: G = 318, 43.6 visits, 2247-2290
// (profiles/r05_ab_noleaders_cut.jsonl); in another session 32: 2261-2286, 64, 2^26: G = 400, 42.2 visits,
// 2293-2321, 128, 2^27: G = 505, 41.0 visits, 2297-2333 (profiles/r05_ab_cut_size.jsonl).  Round 6's 32-B records of
// 7 entries at G = 400: 42.5 visits, 2322-2363 against 2301-2351 for the 68-B cells in one session
// (profiles/r06_c3_cut_levels_ab.jsonl).
#ifndef MSH_CUT_PER_LEAF
#define MSH_CUT_PER_LEAF 64
#endif
#ifndef MSH_CUT_MAX_LOG2
#define MSH_CUT_MAX_LOG2 26
#endif
#ifndef MSH_CUT_FROM_HALF
#define MSH_CUT_FROM_HALF 1
#endif
constexpr bool kCutFromHalf = MSH_CUT_FROM_HALF;
#ifndef MSH_CUT_STAGED
#define MSH_CUT_STAGED 1
#endif
constexpr bool kCutStaged = MSH_CUT_STAGED;
constexpr size_t kCutCoarsePerLeaf = 8;
constexpr int kCutCoarseMaxLog2 = 23;
constexpr size_t kFineRowsPerCell = 16;
static size_t auto_cut_cells(const msh_tree* t, bool fine) {
    return fine ? std::min<size_t>((size_t)MSH_CUT_PER_LEAF * t->T, (size_t)1 << MSH_CUT_MAX_LOG2)
                : std::min<size_t>(kCutCoarsePerLeaf * t->T, (size_t)1 << kCutCoarseMaxLog2);
}
// record bytes per cell: 32 (4-B entries) for trees of <= 2^20 leaves, else 64
static size_t cut_rec_bytes(const msh_tree* t) { return t->T <= kEnt4MaxLeaves ? 32 : 64; }

// cells per axis of the grid to build: the caller's G, else the automatic coarse grid or the fine one at twice its
// resolution (8 x its cells: the fine grid's cells nest in the coarse one's, whose records then start them)
static int cut_grid(const msh_tree* t, bool fine) {
    if (t->cut_req > 0) return t->cut_req;
    const int Gc = std::max(16, (int)std::lround(std::cbrt((double)auto_cut_cells(t, false))));
    if (!fine) return Gc;
    return kCutFromHalf ? 2 * Gc : std::max(16, (int)std::lround(std::cbrt((double)auto_cut_cells(t, true))));
}

// The grid's cell centres are answered exactly by the tree (walks from the installed coarse grid when the fine one is
// built, else from the root), then every cell is cut (nearest.hip k_cut_level): from the enclosing coarse cell's start
// list when the coarse grid is installed and this grid is twice its resolution, else from the root.  C3 (round 6):
// coarse grid 11 ms; fine grid from it 46 ms (centre walks 26, cut 18), 67 ms from the root
// (profiles/r06_c3_cut_staged_ab.jsonl).  Round 6 also tried a pyramid -- the
// coarsest grid answered exactly, each finer level cut from the coarser one's records with hints taken from the 8
// coarse cells around it -- which built C3's grid in 41 ms instead of ~70 but started queries from worse hints:
// 49.4 node visits per query against 42.5, 2.02-2.06 G q/s against 2.32-2.36 (profiles/r06_c3_cut_levels_ab.jsonl).
static int build_entry_cut(msh_tree* t, bool fine) {
    const int G = cut_grid(t, fine);
    double half[3], H = 0.0, lo[3], w[3];
    for (int k = 0; k < 3; ++k) {
        half[k] = 0.5 * ((double)t->scene_hi[k] - (double)t->scene_lo[k]);
        H = std::max(H, half[k]);
    }
    if (!(H > 0.0) || !std::isfinite(H)) {
        set_error("entry cut: degenerate scene box");
        return MSH_EINVAL;
    }
    for (int k = 0; k < 3; ++k) {
        const double m = 0.5 * ((double)t->scene_hi[k] + (double)t->scene_lo[k]);
        const double e = 1.25 * std::max(half[k], 0.05 * H);
        lo[k] = m - e;
        w[k] = 2.0 * e / G;
    }
    const size_t n = (size_t)G * G * G;
    if (n > 0xFFFFFFFFull) {
        set_error("entry cut: %d^3 cells exceed one query call", G);
        return MSH_ENOMEM;
    }
    const bool e4 = t->T <= kEnt4MaxLeaves;
    const size_t rb = cut_rec_bytes(t);
    hipStream_t s = t->stream;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    MSH_HIP(hipEventCreate(&e0));
    hipError_t e = hipEventCreate(&e1);
    if (e != hipSuccess) {
        (void)hipEventDestroy(e0);
        MSH_HIP(e);
    }
    (void)hipEventRecord(e0, s);
    uint32_t* cut = nullptr;
    int st = MSH_OK;
    {
        DevBuf dq, df, dp, dinv, dhint;
        do {
            if ((st = dq.reserve(n * 3 * sizeof(double))) != MSH_OK) break;
            if ((st = df.reserve(n * sizeof(uint32_t))) != MSH_OK) break;
            if ((st = dp.reserve(n * 3 * sizeof(double))) != MSH_OK) break;
            if ((st = dhint.reserve(n * sizeof(int))) != MSH_OK) break;
            if ((st = dinv.reserve(t->T * sizeof(uint32_t))) != MSH_OK) break;
            if ((st = cut_centres(G, lo, w, dq.as<double>(), s)) != MSH_OK) break;
            // (capping the centres' walks at 64 / 128 node steps, their best face so far an upper bound of d(c): the
            // walks 32 -> 27 / 29.5 ms on C3, the queries from the grid 42.46 -> 43.45 / 42.61 node visits,
            // profiles/r06_c3_cut_build_probe.jsonl; not kept)
            if ((st = msh_tree_nearest_device(t, dq.as<double>(), n, df.as<uint32_t>(), nullptr, dp.as<double>(), s)) !=
                MSH_OK)
                break;
            if ((st = cut_hints(t, df.as<uint32_t>(), n, dinv.as<uint32_t>(), dhint.as<int>(), s)) != MSH_OK) break;
            dq.release();  // the centres' rows are not needed by the cut itself
            e = dmalloc(&cut, n * rb);
            if (e != hipSuccess) {
                set_error("hipMalloc entry cut (%zu cells): %s", n, hipGetErrorString(e));
                st = MSH_ENOMEM;
                break;
            }
            // the installed grid, when it is this one at half resolution over the same box (the automatic coarse grid
            // under the fine one), gives every cell its start list (k_cut_level)
            const uint32_t* half = nullptr;
            if (kCutFromHalf && t->d_cut && 2 * t->cut_G == G && t->cut_wide == (e4 ? 0 : 1) &&
                t->cut_lo[0] == lo[0] && t->cut_lo[1] == lo[1] && t->cut_lo[2] == lo[2])
                half = t->d_cut;
            if ((st = cut_level(t, G, lo, w, dp.as<double>(), dhint.as<int>(), cut, e4, s, half)) != MSH_OK) break;
            (void)hipEventRecord(e1, s);
            if ((e = hipStreamSynchronize(s)) != hipSuccess) {
                set_error("entry cut build: %s", hipGetErrorString(e));
                st = MSH_EDEVICE;
            }
        } while (0);
        (void)hipStreamSynchronize(s);  // the temporaries are freed (DevBuf destructors) as this scope ends
    }
    if (st == MSH_OK) {
        float ms = 0.f;
        (void)hipEventElapsedTime(&ms, e0, e1);
        t->cut_ms = ms;
        t->d_cut = cut;
        t->cut_wide = e4 ? 0 : 1;
        t->cut_G = G;
        for (int k = 0; k < 3; ++k) {
            t->cut_lo[k] = lo[k];
            t->cut_iw[k] = 1.0 / w[k];
        }
    } else if (cut) {
        (void)dfree(cut);
    }
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    return st;
}

// Closest-point call of S rows: settle the handle's cut first.  The automatic policy (above auto_cut_cells): the
// coarse grid once the handle has answered one row per kCutAutoCellsPerRow of its cells (C3: 500k rows; a few small
// calls on a large mesh walk from the root instead of paying for it), the fine grid once it has answered
// kFineRowsPerCell rows per fine cell; after msh_tree_set_entry_cut, the grid asked for at the next call.  The cut is
// an optimisation, so a failure (device memory, most likely) is not the query's: the partial buffers are freed, the
// error is cleared and queries start at the root (or from the coarse grid, if the fine one failed).
constexpr size_t kCutAutoCellsPerRow = 16;
static void ensure_entry_cut(msh_tree* t, size_t S) {
    if (t->cut_state == kCutOff || t->cut_state == kCutFailed) return;
    if (!cut_applies(t)) {
        if (t->cut_state == kCutPending) t->cut_state = kCutOff;
        return;
    }
    const bool automatic = !t->cut_force && t->cut_req < 0;
    bool fine = t->cut_req < 0;  // an automatic request: the fine grid (explicit -1, or the volume reached)
    if (automatic) {
        t->cut_rows += S;
        const size_t coarse_rows = auto_cut_cells(t, false) / kCutAutoCellsPerRow;
        const size_t fine_rows = auto_cut_cells(t, true) * kFineRowsPerCell;
        if (t->cut_state == kCutBuilt) {  // a coarse grid: upgrade once the volume pays for the fine one
            if (t->cut_fine || t->cut_rows < fine_rows) return;
        } else if (t->cut_rows < coarse_rows) {
            return;
        }
        fine = t->cut_rows >= fine_rows;
    } else if (t->cut_state == kCutBuilt) {
        return;
    }
    const std::string keep = g_err;
    // a fine grid asked for with no grid installed (msh_tree_set_entry_cut(t, -1) before the first call) is built in
    // two stages: the coarse grid first (its own centre walks from the root), then the fine one, whose centre walks and
    // start lists begin from it (build_entry_cut); the coarse grid is then freed like an upgrade's
    double staged_ms = 0.0;
    if (kCutStaged && fine && !t->d_cut && t->cut_req < 0) {
        t->cut_state = kCutOff;
        if (build_entry_cut(t, false) == MSH_OK) {
            staged_ms = t->cut_ms;
        } else {
            (void)hipGetLastError();  // the fine grid is then built from the root
            t->d_cut = nullptr;
        }
    }
    // while a grid is built its cell-centre queries start from the coarse grid, when one is installed (an upgrade),
    // else from the root; the state is off meanwhile, so the build's own queries do not build again
    uint32_t* old = t->d_cut;
    const int old_G = t->cut_G, old_wide = t->cut_wide;
    const double old_ms = t->cut_ms;
    double old_lo[3], old_iw[3];
    for (int k = 0; k < 3; ++k) {
        old_lo[k] = t->cut_lo[k];
        old_iw[k] = t->cut_iw[k];
    }
    t->cut_state = kCutOff;
    const int st = build_entry_cut(t, fine);
    if (st == MSH_OK) {
        t->cut_ms += staged_ms;
        if (old) {
            if (t->ws_done) (void)hipEventSynchronize(t->ws_done);
            (void)dfree(old);
        }
        t->cut_state = kCutBuilt;
        t->cut_fine = fine;
    } else {
        (void)hipGetLastError();  // clear a sticky launch / allocation error of the failed build
        if (old) {  // a failed upgrade keeps the coarse grid
            t->d_cut = old;
            t->cut_G = old_G;
            t->cut_wide = old_wide;
            t->cut_ms = old_ms;
            for (int k = 0; k < 3; ++k) {
                t->cut_lo[k] = old_lo[k];
                t->cut_iw[k] = old_iw[k];
            }
            t->cut_state = kCutBuilt;
            t->cut_fine = true;  // no second try
        } else {
            // an automatic grid is tried again after another threshold of rows (memory may have been freed by then),
            // at most twice; a grid the caller asked for fails at once (msh_tree_set_entry_cut re-arms it)
            t->cut_state = automatic && ++t->cut_fails <= 2 ? kCutPending : kCutFailed;
            t->cut_rows = 0;
        }
    }
    g_err = keep;
}

// Triangle tree over v (P rows) and f (T rows, indices into v).
// Subtrees of the LBVH over at most 2^kResplitLog2 leaves are rebuilt top down along the surface (refine.hip;
// C3: 2^12 and 2^17 measured slower, profiles/r03_c3_resplit_ab.jsonl)
constexpr int kResplitLog2 = 16;

static int build_triangles(msh_tree* t, const double* v, size_t Pall, const uint32_t* f, size_t T) {
    hipStream_t s = t->stream;
    hipEvent_t e0, e1;
    MSH_HIP(hipEventCreate(&e0));
    MSH_HIP(hipEventCreate(&e1));
    MSH_HIP(dmalloc(&t->d_v, std::max<size_t>(Pall, 1) * 3 * sizeof(double)));
    MSH_HIP(hipMemcpyAsync(t->d_v, v, Pall * 3 * sizeof(double), hipMemcpyHostToDevice, s));
    DevBuf dF, dLo, dHi, dOrder;
    int st = MSH_OK;
    do {
        if ((st = upload(dF, f, 3 * T, s)) != MSH_OK) break;
        if ((st = dLo.reserve(3 * T * sizeof(double))) != MSH_OK) break;
        if ((st = dHi.reserve(3 * T * sizeof(double))) != MSH_OK) break;
        if ((st = dOrder.reserve(T * sizeof(uint32_t))) != MSH_OK) break;
        if (T > 1) {
            hipError_t e = dmalloc(&t->d_nodes, (T - 1) * sizeof(BNode));
            if (e != hipSuccess) { set_error("hipMalloc nodes: %s", hipGetErrorString(e)); st = MSH_ENOMEM; break; }
        }
        hipError_t e = dmalloc(&t->d_leaves, T * sizeof(TriRec));
        if (e != hipSuccess) { set_error("hipMalloc leaves: %s", hipGetErrorString(e)); st = MSH_ENOMEM; break; }
        (void)hipEventRecord(e0, s);
        if ((st = tri_bounds(t->d_v, dF.as<uint32_t>(), T, dLo.as<double>(), dHi.as<double>(), s)) != MSH_OK) break;
        if ((st = build_lbvh(t, dLo.as<double>(), dHi.as<double>(), T, dOrder.as<uint32_t>())) != MSH_OK) break;
        if ((st = resplit_tree(t, t->d_v, dF.as<uint32_t>(), T, dOrder.as<uint32_t>(), kResplitLog2)) != MSH_OK) break;
        if ((st = pack_tri_leaves(t->d_v, dF.as<uint32_t>(), dOrder.as<uint32_t>(), T, 0u,
                                  static_cast<TriRec*>(t->d_leaves), s)) != MSH_OK)
            break;
        if ((st = build_obb(t, true)) != MSH_OK) break;
        (void)hipEventRecord(e1, s);
        e = hipStreamSynchronize(s);
        if (e != hipSuccess) { set_error("LBVH build failed: %s", hipGetErrorString(e)); st = MSH_EDEVICE; break; }
        float ms = 0.f;
        (void)hipEventElapsedTime(&ms, e0, e1);
        t->build_ms = ms;
    } while (0);
    (void)hipStreamSynchronize(s);
    dF.release(); dLo.release(); dHi.release(); dOrder.release();
    t->ws.release();  // build scratch (sort buffers, parents, ranges) is not needed by queries
    // a freed tree's query workspace, if one is idle (free_tree gives it back)
    if (st == MSH_OK) ws_pool().take(t->device, t->ws);
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    return st;
}

static const size_t kSortMin = 4096;  // below this the query Morton sort costs more than it saves
#ifndef MSH_ALONG_LAZY
#define MSH_ALONG_LAZY 1
#endif
static constexpr bool kAlongLazy = MSH_ALONG_LAZY;  // alongnormal rays read at perm[slot] instead of gathered

// Query order for S point rows (device): below kSortMin the caller's arrays are used as they are;
// otherwise Morton codes + radix sort give the permutation (ws.vals).  With allow_lazy (closest-point
// launches, and alongnormal rays with their normals: kAlongLazy) the traversal reads row perm[i] itself (and the
// closest-point one writes the inverse permutation, ws.inv); otherwise (the normals-metric queries) the rows and
// normals are gathered once into slot order (ws.qs / ws.ns) with the inverse permutation (gathering the
// closest-point rows too measured 3 % slower on C3; the C5 rays 0.5 ms slower, profiles/r06_c5_along_lazy_ab.jsonl).
// Queries are ordered by the Hilbert index of their cell of a 256^3 grid (the top 24 bits of their 30-bit Morton
// code, mapped through sort.hip's Hilbert state table; 3 radix passes): C3's 100M queries put ~6 in a cell, and the
// traversal runs the same node counts as with the full code.  The order within a cell is the caller's (stable sort).
constexpr int kQuerySortLo = 6;
static int sort_queries(msh_tree* t, const double* d_q, const double* d_n, size_t S, hipStream_t s,
                        QueryOrder* ord, bool allow_lazy = false) {
    *ord = QueryOrder{d_q, d_n, nullptr, nullptr};
    if (S < kSortMin) return MSH_OK;
    Workspace& ws = t->ws;
    MSH_TRY(ws.inv.reserve(S * sizeof(uint32_t)));
    float lo[3], hi[3];
    query_box(t, lo, hi);
    MSH_TRY(query_sort(lo, hi, d_q, S, kQuerySortLo, ws, s));
    if (allow_lazy) {
        *ord = QueryOrder{d_q, d_n, ws.vals.as<uint32_t>(), ws.inv.as<uint32_t>(), false};
        return MSH_OK;
    }
    MSH_TRY(ws.qs.reserve(3 * S * sizeof(double)));
    if (d_n) MSH_TRY(ws.ns.reserve(3 * S * sizeof(double)));
    MSH_TRY(gather_rows(d_q, d_n, ws.vals.as<uint32_t>(), S, ws.qs.as<double>(), d_n ? ws.ns.as<double>() : nullptr,
                        ws.inv.as<uint32_t>(), s));
    *ord = QueryOrder{ws.qs.as<double>(), d_n ? ws.ns.as<double>() : nullptr, ws.vals.as<uint32_t>(),
                      ws.inv.as<uint32_t>()};
    return MSH_OK;
}

// Batched trees: Morton order inside each mesh, meshes in order (two stable passes), then the gather.
static int sort_batch_queries(msh_tree* t, const double* d_q, size_t n, size_t S, hipStream_t s, QueryOrder* ord,
                              size_t mesh0 = 0) {
    *ord = QueryOrder{d_q, nullptr, nullptr, nullptr};
    if (n < kSortMin) return MSH_OK;
    Workspace& ws = t->ws;
    MSH_TRY(ws.keys.reserve(n * sizeof(uint32_t)));
    MSH_TRY(ws.vals.reserve(n * sizeof(uint32_t)));
    MSH_TRY(ws.keys_alt.reserve(n * sizeof(uint32_t)));
    MSH_TRY(ws.vals_alt.reserve(n * sizeof(uint32_t)));
    MSH_TRY(ws.qs.reserve(3 * n * sizeof(double)));
    MSH_TRY(ws.inv.reserve(n * sizeof(uint32_t)));
    uint32_t* keys = ws.keys.as<uint32_t>();
    uint32_t* vals = ws.vals.as<uint32_t>();
    MSH_TRY(query_morton_batch(t, d_q, n, S, keys, vals, s, mesh0));
    MSH_TRY(radix_sort_pairs(keys, vals, ws.keys_alt.as<uint32_t>(), ws.vals_alt.as<uint32_t>(), n, 30, ws, s));
    const size_t meshes = n / S;  // of this launch
    if (meshes > 1) {
        MSH_TRY(mesh_keys(vals, n, S, keys, s));
        int bits = 0;
        while (bits < 32 && ((size_t)1 << bits) < meshes) ++bits;
        MSH_TRY(radix_sort_pairs(keys, vals, ws.keys_alt.as<uint32_t>(), ws.vals_alt.as<uint32_t>(), n, bits, ws, s));
    }
    MSH_TRY(gather_rows(d_q, nullptr, vals, n, ws.qs.as<double>(), nullptr, ws.inv.as<uint32_t>(), s));
    *ord = QueryOrder{ws.qs.as<double>(), nullptr, vals, ws.inv.as<uint32_t>()};
    return MSH_OK;
}

static int check_tree(const msh_tree* t, int want_kind, const char* fn) {
    if (!t) {
        set_error("%s: null tree handle", fn);
        return MSH_EINVAL;
    }
    if (want_kind == kPoints ? t->kind != kPoints : t->kind == kPoints) {
        set_error("%s: wrong handle kind %d", fn, t->kind);
        return MSH_EINVAL;
    }
    // any batched handle (also B == 1: its bounds are relative to the per-mesh origins)
    if (t->B != 1 || t->d_boxes) {
        set_error("%s: batched tree handle (use the msh_batch_* entry points)", fn);
        return MSH_EINVAL;
    }
    return use_device(t->device);
}

static int check_batch(const msh_tree* t, const char* fn) {
    if (!t) {
        set_error("%s: null tree handle", fn);
        return MSH_EINVAL;
    }
    if (!t->d_boxes) {
        set_error("%s: not a batched tree handle (build it with msh_batch_build)", fn);
        return MSH_EINVAL;
    }
    return use_device(t->device);
}

static hipStream_t pick(msh_tree* t, void* stream) { return stream ? static_cast<hipStream_t>(stream) : t->stream; }

// ---- host staging: pinned double-buffered chunks, copies overlapped with the kernels ----
static int host_threads() {
    const char* e = getenv("MESH_AMD_COPY_THREADS");
    int n = e ? atoi(e) : 0;
    if (n <= 0) {
        const char* o = getenv("OMP_NUM_THREADS");
        n = o ? atoi(o) : 8;
    }
    return std::max(1, std::min(n, 32));
}

// Persistent host copy workers (created on first use, one pool per process): run(tasks) splits a list of
// memcpys into ~2 MB pieces and executes them on all workers plus the caller, so the pageable <-> pinned
// staging copies of one pipeline step (inputs of chunk k and outputs of chunk k - 2) move together at the
// host's memory bandwidth instead of one after the other, without creating threads per copy.
struct CopyTask {
    void* dst;
    const void* src;
    size_t bytes;
};
class CopyPool {
  public:
    explicit CopyPool(int n) {
        for (int i = 0; i < n; ++i) th_.emplace_back([this] { loop(); });
    }
    ~CopyPool() {
        {
            std::lock_guard<std::mutex> g(mu_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto& t : th_) t.join();
    }
    void run(const std::vector<CopyTask>& tasks) {
        constexpr size_t kPiece = (size_t)2 << 20;
        std::vector<CopyTask> pieces;
        for (const CopyTask& t : tasks)
            for (size_t o = 0; o < t.bytes; o += kPiece)
                pieces.push_back({static_cast<char*>(t.dst) + o, static_cast<const char*>(t.src) + o,
                                  std::min(kPiece, t.bytes - o)});
        if (pieces.empty()) return;
        std::lock_guard<std::mutex> job(job_mu_);  // one job at a time
        {
            std::lock_guard<std::mutex> g(mu_);
            pieces_ = &pieces;
            next_.store(0);
            ++gen_;
        }
        cv_.notify_all();
        work(&pieces);
        // every worker that took this job has left it before `pieces` goes away
        std::unique_lock<std::mutex> g(mu_);
        done_cv_.wait(g, [&] { return busy_ == 0; });
        pieces_ = nullptr;
    }

  private:
    void work(std::vector<CopyTask>* p) {
        for (;;) {
            const size_t i = next_.fetch_add(1);
            if (i >= p->size()) return;
            std::memcpy((*p)[i].dst, (*p)[i].src, (*p)[i].bytes);
        }
    }
    void loop() {
        size_t seen = 0;
        for (;;) {
            std::vector<CopyTask>* p = nullptr;
            {
                std::unique_lock<std::mutex> g(mu_);
                cv_.wait(g, [&] { return stop_ || gen_ != seen; });
                if (stop_) return;
                seen = gen_;
                p = pieces_;
                if (p) ++busy_;
            }
            if (!p) continue;
            work(p);
            std::lock_guard<std::mutex> g(mu_);
            if (--busy_ == 0) done_cv_.notify_all();
        }
    }
    std::vector<std::thread> th_;
    std::mutex mu_, job_mu_;
    std::condition_variable cv_, done_cv_;
    std::vector<CopyTask>* pieces_ = nullptr;
    std::atomic<size_t> next_{0};
    int busy_ = 0;
    size_t gen_ = 0;
    bool stop_ = false;
};
static CopyPool& copy_pool() {
    static CopyPool pool(host_threads() - 1);
    return pool;
}

// One pipelined host call: rows [0, S) in chunks; inputs (ni arrays of in_w doubles per row) are staged
// through pinned buffers and uploaded on a copy stream, `run(chunk, n, dev_in, dev_out)` enqueues the
// kernels on the handle's stream, and outputs (no arrays of out_b bytes per row) come back on a second
// copy stream while the next chunk computes.
struct HostArr {
    const void* in;   // input (caller memory) or nullptr
    void* out;        // output (caller memory) or nullptr
    size_t row_bytes;
};

static void release_stage(msh_tree* t, bool host, bool dev) {
    for (int b = 0; b < 3; ++b) {
        if (host && b < 2 && t->h_stage[b]) (void)hipHostFree(t->h_stage[b]);
        if (dev && t->d_stage[b]) (void)dfree(t->d_stage[b]);
        if (host && b < 2) t->h_stage[b] = nullptr;
        if (dev) t->d_stage[b] = nullptr;
    }
    if (host) t->hstage_bytes = 0;
    if (dev) t->stage_bytes = 0;
}
static void release_stage(msh_tree* t) { release_stage(t, true, true); }

// Staging slabs shared by the handles of a device: a pipelined call leases one set (two pinned host slabs and two
// device slabs) into its handle and hands it back when it returns, so a caller that builds a tree per call (the
// reference's Mesh.closest_faces_and_points, mesh.py:454-455) pays the page-locking of ~1.5 GB of host slabs
// once per process instead of once per tree.  At most kStageKeep idle sets are kept per device.
struct StageSet {
    void* h[2] = {nullptr, nullptr};
    void* d[3] = {nullptr, nullptr, nullptr};
    size_t hbytes = 0, dbytes = 0;
};
class StagePool {
  public:
    StageSet take(int dev) {
        std::lock_guard<std::mutex> g(mu_);
        std::vector<StageSet>& v = idle_[dev];
        if (v.empty()) return StageSet{};
        StageSet s = v.back();
        v.pop_back();
        return s;
    }
    void give(int dev, const StageSet& s) {
        constexpr size_t kStageKeep = 2;
        std::lock_guard<std::mutex> g(mu_);
        std::vector<StageSet>& v = idle_[dev];
        if (v.size() < kStageKeep) {
            v.push_back(s);
            return;
        }
        for (int b = 0; b < 3; ++b) {  // an extra set (concurrent calls): freed
            if (b < 2 && s.h[b]) (void)hipHostFree(s.h[b]);
            if (s.d[b]) (void)dfree(s.d[b]);
        }
    }

    size_t device_bytes() {
        std::lock_guard<std::mutex> g(mu_);
        size_t n = 0;
        for (auto& kv : idle_)
            for (const StageSet& s : kv.second) n += 3 * s.dbytes;
        return n;
    }
    void trim() {
        std::lock_guard<std::mutex> g(mu_);
        for (auto& kv : idle_) {
            for (const StageSet& s : kv.second)
                for (int b = 0; b < 3; ++b) {
                    if (b < 2 && s.h[b]) (void)hipHostFree(s.h[b]);
                    if (s.d[b]) (void)dfree(s.d[b]);
                }
            kv.second.clear();
        }
    }
    // the idle sets' device slabs of one device (the caller is on that device); their pinned host slabs stay
    void trim_device(int dev) {
        std::vector<void*> drop;
        {
            std::lock_guard<std::mutex> g(mu_);
            for (StageSet& s : idle_[dev]) {
                for (int b = 0; b < 3; ++b) {
                    if (s.d[b]) drop.push_back(s.d[b]);
                    s.d[b] = nullptr;
                }
                s.dbytes = 0;
            }
        }
        for (void* p : drop) (void)dfree(p);
    }

  private:
    std::mutex mu_;
    std::map<int, std::vector<StageSet>> idle_;
};
static StagePool& stage_pool() {
    static StagePool* p = new StagePool;  // never destroyed: the runtime may be gone at static destruction
    return *p;
}

static void release_idle_device(int dev) {
    ws_pool().trim_device(dev);
    stage_pool().trim_device(dev);
}
// the handle holds the leased set for one call (stage_setup grows it in place)
struct StageLease {
    msh_tree* t;
    explicit StageLease(msh_tree* tree) : t(tree) {
        const StageSet s = stage_pool().take(t->device);
        for (int b = 0; b < 3; ++b) {
            if (b < 2) t->h_stage[b] = s.h[b];
            t->d_stage[b] = s.d[b];
        }
        t->hstage_bytes = s.hbytes;
        t->stage_bytes = s.dbytes;
    }
    ~StageLease() {
        StageSet s;
        for (int b = 0; b < 3; ++b) {
            if (b < 2) {
                s.h[b] = t->h_stage[b];
                t->h_stage[b] = nullptr;
            }
            s.d[b] = t->d_stage[b];
            t->d_stage[b] = nullptr;
        }
        s.hbytes = t->hstage_bytes;
        s.dbytes = t->stage_bytes;
        t->hstage_bytes = t->stage_bytes = 0;
        stage_pool().give(t->device, s);
    }
};

// copy streams, events, and two host slabs of >= host_bytes and two device slabs of >= dev_bytes (grow-only)
static int stage_setup(msh_tree* t, size_t host_bytes, size_t dev_bytes) {
    if (!t->s_up) MSH_HIP(hipStreamCreateWithFlags(&t->s_up, hipStreamNonBlocking));
    if (!t->s_down) MSH_HIP(hipStreamCreateWithFlags(&t->s_down, hipStreamNonBlocking));
    for (int b = 0; b < 3; ++b) {
        if (!t->e_up[b]) MSH_HIP(hipEventCreateWithFlags(&t->e_up[b], hipEventDisableTiming));
        if (!t->e_run[b]) MSH_HIP(hipEventCreateWithFlags(&t->e_run[b], hipEventDisableTiming));
        if (!t->e_down[b]) MSH_HIP(hipEventCreateWithFlags(&t->e_down[b], hipEventDisableTiming));
    }
    if (t->hstage_bytes < host_bytes) {
        release_stage(t, true, false);
        for (int b = 0; b < 2; ++b) MSH_HIP(hipHostMalloc(&t->h_stage[b], host_bytes, hipHostMallocDefault));
        t->hstage_bytes = host_bytes;
    }
    if (t->stage_bytes < dev_bytes) {
        release_stage(t, false, true);
        for (int b = 0; b < 3; ++b) MSH_HIP(dmalloc(&t->d_stage[b], dev_bytes));
        t->stage_bytes = dev_bytes;
    }
    return MSH_OK;
}

// MESH_AMD_HOST_REGISTER=1: page-lock the caller's arrays in place instead of staging.  Off by default:
// registering C3's 5.6 GB of rows per call cost more than the staging copies (C3 numpy path 395 vs 280 ms).
static bool host_register_enabled() {
    const char* e = getenv("MESH_AMD_HOST_REGISTER");
    return e && atoi(e) != 0;
}

// Chunk plan of a pipelined call: the rows of each chunk, the last entry repeated.  Larger chunks keep the sorted
// traversal coherent and cut per-chunk launch tails; a small first chunk lets the first download start early.
// The host link moves both directions at ~57 GB/s combined (scripts/pcie_probe.py), and a C3 call moves 2.4 GB
// up and 3.2 GB down per 100M queries, so a call is bound by its copies once they overlap the kernels.
// Measured on C3 (100M queries, results in pinned pool arrays, three device slabs; profiles/r04_c3np_plan_ab.json):
// 32M chunks 98 ms, 24M 94-96, 16M 120, 6M + 30M 96, 4M + 12M + 28M 94-96, 8M + 16M + 32M 92-94, 12M + 28M 91,
// 8M + 24M 89-91, 8M + 20M 86-89.  Staged outputs (caller arrays outside the pool): 16M chunks (4M 155 ms, 8M 137,
// 16M 134, 32M 150).  Test hook: MESH_AMD_HOST_CHUNK = rows (uniform chunks, so small calls run several chunks; it
// also overrides the plans of callers whose rows are meshes or cameras).
static size_t host_chunk_env() {
    const char* e = getenv("MESH_AMD_HOST_CHUNK");
    const long long c = e ? atoll(e) : 0;
    return c > 0 ? (size_t)c : 0;
}
static std::vector<size_t> host_plan(bool direct_out) {
    if (const size_t c = host_chunk_env()) return {c};
    if (direct_out) return {(size_t)8 << 20, (size_t)20 << 20};
    return {(size_t)16 << 20};
}

// Page-locked result pool (msh_host_alloc / msh_host_free, meshsearch.h).  Blocks are hipHostMalloc'd in 2-MB
// granules and kept after release for the next call of similar size, up to a cap; the host-buffer entry points
// download results straight into output arrays that lie inside a live block (pinned_range).
class PinnedPool {
  public:
    int alloc(size_t bytes, void** out) {
        constexpr size_t kGran = (size_t)2 << 20;
        const size_t want = (std::max<size_t>(bytes, 1) + kGran - 1) / kGran * kGran;
        std::lock_guard<std::mutex> g(mu_);
        auto it = free_.lower_bound(want);  // best fit, at most 5/4 of the request
        if (it != free_.end() && it->first <= want + want / 4) {
            *out = it->second;
            live_.insert(it->second);
            free_.erase(it);
            return MSH_OK;
        }
        const size_t cap = cap_bytes();
        // make room: release free blocks, largest first, until the new block fits under the cap
        while (total_ + want > cap && !free_.empty()) release_locked(std::prev(free_.end()));
        if (total_ + want > cap) {
            set_error("msh_host_alloc: pinned pool cap %zu MB reached", cap >> 20);
            return MSH_ENOMEM;
        }
        void* p = nullptr;
        if (hipHostMalloc(&p, want, hipHostMallocDefault) != hipSuccess) {
            (void)hipGetLastError();
            while (!free_.empty()) release_locked(std::prev(free_.end()));
            if (hipHostMalloc(&p, want, hipHostMallocDefault) != hipSuccess) {
                (void)hipGetLastError();
                set_error("msh_host_alloc: hipHostMalloc of %zu bytes failed", want);
                return MSH_ENOMEM;
            }
        }
        blocks_[p] = want;
        live_.insert(p);
        total_ += want;
        *out = p;
        return MSH_OK;
    }
    void release(void* p) {
        std::lock_guard<std::mutex> g(mu_);
        auto b = blocks_.find(p);
        if (b == blocks_.end() || !live_.erase(p)) return;
        free_.emplace(b->second, p);
    }
    int trim() {
        std::lock_guard<std::mutex> g(mu_);
        while (!free_.empty()) release_locked(std::prev(free_.end()));
        return MSH_OK;
    }
    size_t bytes() {
        std::lock_guard<std::mutex> g(mu_);
        return total_;
    }
    // [p, p + n) lies inside one live block
    bool contains(const void* p, size_t n) {
        std::lock_guard<std::mutex> g(mu_);
        auto it = blocks_.upper_bound(const_cast<void*>(p));
        if (it == blocks_.begin()) return false;
        --it;
        const char* b = static_cast<const char*>(it->first);
        const char* c = static_cast<const char*>(p);
        return live_.count(it->first) && c >= b && c + n <= b + it->second;
    }

  private:
    static size_t cap_bytes() {
        const char* e = getenv("MESH_AMD_PINNED_POOL_MB");
        const long long mb = e ? atoll(e) : 16384;
        return mb > 0 ? (size_t)mb << 20 : 0;
    }
    void release_locked(std::multimap<size_t, void*>::iterator it) {
        void* p = it->second;
        (void)hipHostFree(p);
        total_ -= it->first;
        blocks_.erase(p);
        free_.erase(it);
    }
    std::mutex mu_;
    std::map<void*, size_t> blocks_;       // every block: base -> bytes
    std::set<void*> live_;                 // blocks handed out
    std::multimap<size_t, void*> free_;    // released blocks by size
    size_t total_ = 0;
};
static PinnedPool& pinned_pool() {
    static PinnedPool* p = new PinnedPool;  // never destroyed: live arrays may outlive static destructors
    return *p;
}

// pipelined() over caller arrays that are page-locked in place: per chunk an H2D copy of the input rows into a
// device slab (copy stream `up`), the kernels (handle stream), a D2H copy of the output rows straight into
// the caller's arrays (stream `down`); two device slabs alternate, so chunk k uploads while k - 1 computes and
// k - 2 downloads.
template <class Run>
static int pipelined_registered(msh_tree* t, size_t S, const std::vector<HostArr>& arrs, size_t chunk, Run run) {
    size_t row = 0;
    for (const HostArr& a : arrs) row += a.row_bytes;
    MSH_TRY(stage_setup(t, 0, chunk * row));
    hipStream_t sc = t->stream, up = t->s_up, down = t->s_down;
    int st = MSH_OK;
    hipError_t e = hipSuccess;
    const size_t nch = (S + chunk - 1) / chunk;
    for (size_t k = 0; k < nch && st == MSH_OK && e == hipSuccess; ++k) {
        const int b = (int)(k & 1);
        const size_t r0 = k * chunk, n = std::min(chunk, S - r0);
        char* dev = static_cast<char*>(t->d_stage[b]);
        // the slab's previous chunk (k - 2) must have been downloaded before it is overwritten
        if (k >= 2 && (e = hipStreamWaitEvent(up, t->e_down[b], 0)) != hipSuccess) break;
        size_t off = 0;
        for (const HostArr& a : arrs) {
            if (a.in && (e = hipMemcpyAsync(dev + off * chunk, static_cast<const char*>(a.in) + r0 * a.row_bytes,
                                            n * a.row_bytes, hipMemcpyHostToDevice, up)) != hipSuccess)
                break;
            off += a.row_bytes;
        }
        if (e != hipSuccess || (e = hipEventRecord(t->e_up[b], up)) != hipSuccess ||
            (e = hipStreamWaitEvent(sc, t->e_up[b], 0)) != hipSuccess)
            break;
        std::vector<char*> slabs;
        off = 0;
        for (const HostArr& a : arrs) {
            slabs.push_back(dev + off * chunk);
            off += a.row_bytes;
        }
        if ((st = run(r0, n, slabs)) != MSH_OK) break;
        if ((e = hipEventRecord(t->e_run[b], sc)) != hipSuccess || (e = hipStreamWaitEvent(down, t->e_run[b], 0)) != hipSuccess)
            break;
        off = 0;
        for (const HostArr& a : arrs) {
            if (a.out && (e = hipMemcpyAsync(static_cast<char*>(a.out) + r0 * a.row_bytes, dev + off * chunk,
                                             n * a.row_bytes, hipMemcpyDeviceToHost, down)) != hipSuccess)
                break;
            off += a.row_bytes;
        }
        if (e == hipSuccess) e = hipEventRecord(t->e_down[b], down);
    }
    const hipError_t e1 = hipStreamSynchronize(up), e2 = hipStreamSynchronize(sc), e3 = hipStreamSynchronize(down);
    if (e == hipSuccess) e = e1 != hipSuccess ? e1 : (e2 != hipSuccess ? e2 : e3);
    if (st == MSH_OK && e != hipSuccess) {
        set_error("host call (registered): %s", hipGetErrorString(e));
        st = e == hipErrorOutOfMemory ? MSH_ENOMEM : MSH_EDEVICE;
    }
    return st;
}

// plan_rows (optional): the chunk plan in rows (the last entry repeated) instead of host_plan's, for callers whose
// rows are whole meshes (batched trees) or cameras (visibility)
template <class Run>
static int pipelined(msh_tree* t, size_t S, const std::vector<HostArr>& arrs, Run run,
                     const std::vector<size_t>* plan_rows = nullptr) {
    size_t row = 0, in_end = 0;  // in_end: the inputs' share of a slab row (they come first)
    for (const HostArr& a : arrs) {
        row += a.row_bytes;
        if (a.in) in_end = row;
    }
    // outputs inside the pinned result pool (msh_host_alloc) are downloaded straight into place: no staging
    // copy, and the host only waits for a slab's previous upload before refilling it
    bool direct_out = true;
    for (const HostArr& a : arrs)
        if (a.out && !pinned_pool().contains(a.out, S * a.row_bytes)) direct_out = false;
    hipStream_t sc = t->stream;
    int st = MSH_OK;
    if (S * row <= ((size_t)16 << 20)) {  // small call: one pageable round trip through device scratch
        DevBuf tmp;
        MSH_TRY(tmp.reserve(S * row));
        std::vector<char*> slabs;
        size_t off = 0;
        hipError_t e = hipSuccess;
        for (const HostArr& a : arrs) {
            char* d = static_cast<char*>(tmp.ptr) + off * S;
            slabs.push_back(d);
            if (a.in && e == hipSuccess) e = hipMemcpyAsync(d, a.in, S * a.row_bytes, hipMemcpyHostToDevice, sc);
            off += a.row_bytes;
        }
        if (e == hipSuccess) st = run(0, S, slabs);
        off = 0;
        for (const HostArr& a : arrs) {
            if (a.out && e == hipSuccess && st == MSH_OK)
                e = hipMemcpyAsync(a.out, static_cast<char*>(tmp.ptr) + off * S, S * a.row_bytes, hipMemcpyDeviceToHost, sc);
            off += a.row_bytes;
        }
        const hipError_t e2 = hipStreamSynchronize(sc);
        if (e == hipSuccess) e = e2;
        tmp.release();
        if (st == MSH_OK && e != hipSuccess) {
            set_error("host call: %s", hipGetErrorString(e));
            st = MSH_EDEVICE;
        }
        return st;
    }
    // chunks (host_plan): first rows c0s[k], rows cns[k]; slabs are sized for the largest
    std::vector<size_t> c0s, cns;
    {
        const std::vector<size_t> plan =
            plan_rows && !plan_rows->empty() && !host_chunk_env() ? *plan_rows : host_plan(direct_out);
        for (size_t r = 0, j = 0; r < S; ++j) {
            const size_t n = std::min(std::max<size_t>(1, plan[std::min(j, plan.size() - 1)]), S - r);
            c0s.push_back(r);
            cns.push_back(n);
            r += n;
        }
    }
    const size_t chunk = *std::max_element(cns.begin(), cns.end());
    const size_t nch = cns.size();
    StageLease lease(t);  // every stream is synchronised before pipelined returns, so the slabs are idle then
    // Optionally (host_register_enabled) page-lock the caller's arrays in place (hipHostRegister): the copy
    // engines then move the rows straight between the caller's memory and HBM, with no pageable <-> pinned
    // staging copies on the host.  Any registration failure falls back to staging.
    if (host_register_enabled()) {
        std::vector<std::pair<void*, size_t>> reg;
        bool ok = true;
        for (const HostArr& a : arrs) {
            void* p = a.in ? const_cast<void*>(a.in) : a.out;
            if (!p) continue;
            if (hipHostRegister(p, S * a.row_bytes, hipHostRegisterDefault) != hipSuccess) {
                (void)hipGetLastError();
                ok = false;
                break;
            }
            reg.emplace_back(p, S * a.row_bytes);
        }
        if (ok) st = pipelined_registered(t, S, arrs, chunk, run);
        for (auto& r : reg) (void)hipHostUnregister(r.first);
        if (ok) return st;
    }
    MSH_TRY(stage_setup(t, chunk * (direct_out ? in_end : row), chunk * row));
    hipStream_t up = t->s_up, down = t->s_down;
    hipEvent_t* e_up = t->e_up;
    hipEvent_t* e_run = t->e_run;
    hipEvent_t* e_down = t->e_down;
    void* const* host = t->h_stage;
    void* const* dev = t->d_stage;
    auto fail = [&](hipError_t e, const char* what) {
        set_error("%s: %s", what, hipGetErrorString(e));
        st = e == hipErrorOutOfMemory ? MSH_ENOMEM : MSH_EDEVICE;
    };
    // Step k (host slab b = k & 1, device slab db = k % 3; a slab holds one chunk's input rows and, after them,
    // its output rows; events are per device slab):
    //   wait for chunk k - 2's upload (direct_out) or download (staged outputs, copied out of host slab b here),
    //   then copy chunk k's inputs into host slab b, on all copy workers at once, while the GPU works on earlier
    //   chunks; then enqueue chunk k's upload (copy stream; into device slab db once chunk k - 3's download has
    //   left it), kernels (handle stream) and download (second copy stream).  Three device slabs let chunk k's
    //   upload run while chunk k - 2 is still downloading (with two, each upload waited for the download of the
    //   chunk before: C3 numpy API 112 ms per 100M queries).
    auto outs_of = [&](size_t kk, std::vector<CopyTask>& tasks) {
        const int b = (int)(kk & 1);
        const size_t r0 = c0s[kk], n = cns[kk];
        size_t off = 0;
        for (const HostArr& a : arrs) {
            if (a.out)
                tasks.push_back({static_cast<char*>(a.out) + r0 * a.row_bytes, static_cast<char*>(host[b]) + off * chunk,
                                 n * a.row_bytes});
            off += a.row_bytes;
        }
    };
    do {
        hipError_t e = hipSuccess;
        for (size_t k = 0; k < nch + 2 && st == MSH_OK; ++k) {
            const int b = (int)(k & 1), db = (int)(k % 3), pb = (int)((k + 1) % 3);  // pb: chunk k - 2's slab
            std::vector<CopyTask> tasks;
            if (k >= 2) {
                const auto tw = std::chrono::steady_clock::now();
                if (direct_out) {
                    if ((e = hipEventSynchronize(e_up[pb])) != hipSuccess) { fail(e, "upload"); break; }
                } else {
                    if ((e = hipEventSynchronize(e_down[pb])) != hipSuccess) { fail(e, "kernels / download"); break; }
                    outs_of(k - 2, tasks);
                }
                host_time("host_wait", tw);
            }
            const bool have = k < nch;
            const size_t r0 = have ? c0s[k] : S, n = have ? cns[k] : 0;
            if (have) {
                size_t off = 0;
                for (const HostArr& a : arrs) {
                    if (a.in)
                        tasks.push_back({static_cast<char*>(host[b]) + off * chunk,
                                         static_cast<const char*>(a.in) + r0 * a.row_bytes, n * a.row_bytes});
                    off += a.row_bytes;
                }
            }
            const auto tc = std::chrono::steady_clock::now();
            copy_pool().run(tasks);
            host_time("host_copy", tc);
            if (!have) continue;
            // the device slab's previous chunk (k - 3) must have been downloaded before it is overwritten (staged
            // outputs: the host waited for chunk k - 2's download above, which the in-order download stream implies)
            if (direct_out && k >= 3 && (e = hipStreamWaitEvent(up, e_down[db], 0)) != hipSuccess) { fail(e, "upload"); break; }
            size_t off = 0;
            for (const HostArr& a : arrs) {
                if (a.in && (e = hipMemcpyAsync(static_cast<char*>(dev[db]) + off * chunk,
                                                static_cast<char*>(host[b]) + off * chunk, n * a.row_bytes,
                                                hipMemcpyHostToDevice, up)) != hipSuccess)
                    break;
                off += a.row_bytes;
            }
            if (e == hipSuccess) e = hipEventRecord(e_up[db], up);
            if (e == hipSuccess) e = hipStreamWaitEvent(sc, e_up[db], 0);
            if (e != hipSuccess) { fail(e, "upload"); break; }
            std::vector<char*> slabs;
            off = 0;
            for (const HostArr& a : arrs) {
                slabs.push_back(static_cast<char*>(dev[db]) + off * chunk);
                off += a.row_bytes;
            }
            if ((st = run(r0, n, slabs)) != MSH_OK) break;
            if ((e = hipEventRecord(e_run[db], sc)) != hipSuccess || (e = hipStreamWaitEvent(down, e_run[db], 0)) != hipSuccess) {
                fail(e, "launch");
                break;
            }
            off = 0;
            for (const HostArr& a : arrs) {
                if (a.out) {
                    char* dst = direct_out ? static_cast<char*>(a.out) + r0 * a.row_bytes
                                           : static_cast<char*>(host[b]) + off * chunk;
                    if ((e = hipMemcpyAsync(dst, static_cast<char*>(dev[db]) + off * chunk, n * a.row_bytes,
                                            hipMemcpyDeviceToHost, down)) != hipSuccess)
                        break;
                }
                off += a.row_bytes;
            }
            if (e == hipSuccess) e = hipEventRecord(e_down[db], down);
            if (e != hipSuccess) { fail(e, "download"); break; }
        }
    } while (0);
    // every chunk's kernels and copies end here: in direct_out mode no earlier wait saw their status (the loop
    // only waits for uploads), so an asynchronous kernel or copy failure surfaces through these syncs
    const hipError_t e1 = hipStreamSynchronize(up), e2 = hipStreamSynchronize(down), e3 = hipStreamSynchronize(sc);
    const hipError_t ef = e1 != hipSuccess ? e1 : (e2 != hipSuccess ? e2 : e3);
    if (st == MSH_OK && ef != hipSuccess) fail(ef, "host call (kernels / download)");
    return st;
}


// ---- one handle on several devices (msh_set_devices) ----
// Contiguous shards of n rows over G parts, the first n % G one row larger (mesh_amd/distributed.py shard_range).
static void shard_rows(size_t n, size_t G, size_t g, size_t* r0, size_t* cnt) {
    const size_t base = n / G, rem = n % G;
    *r0 = g * base + std::min(g, rem);
    *cnt = base + (g < rem ? 1 : 0);
}

// Host-buffer calls below this many bytes of rows stay on the handle's own device (a fan-out costs a thread per
// replica and a chunk pipeline per device).
constexpr size_t kFanMinBytes = (size_t)32 << 20;

// Rows [0, S) of a host-buffer call over the handle and its replicas: replica g - 1 answers shard g (shard 0 stays
// here), each from its own host thread through the entry point's own pipelined path, so every device's host link
// and copy engines carry their share.  The shards are disjoint row ranges of the caller's arrays, so the answer is
// the one-device answer bit for bit.  call(h, r0, n) runs rows [r0, r0 + n) on handle h.
template <class Call>
static int fan_out(msh_tree* t, size_t S, size_t row_bytes, Call call) {
    const size_t G = 1 + t->replicas.size();
    if (G == 1 || S * row_bytes < kFanMinBytes || S < G) return call(t, (size_t)0, S);
    std::vector<int> st(G, MSH_OK);
    std::vector<std::string> err(G);
    std::vector<std::thread> th;
    th.reserve(G - 1);
    for (size_t g = 1; g < G; ++g)
        th.emplace_back([&, g] {
            size_t r0, n;
            shard_rows(S, G, g, &r0, &n);
            if (n) st[g] = call(t->replicas[g - 1], r0, n);
            if (st[g] != MSH_OK) err[g] = g_err;
        });
    size_t r0, n;
    shard_rows(S, G, 0, &r0, &n);
    st[0] = call(t, r0, n);
    if (st[0] != MSH_OK) err[0] = g_err;
    for (auto& x : th) x.join();
    (void)use_device(t->device);  // the caller's thread stays on the handle's device
    for (size_t g = 0; g < G; ++g)
        if (st[g] != MSH_OK) {
            g_err = err[g];
            return st[g];
        }
    return MSH_OK;
}

}  // namespace msh

using namespace msh;

static int replicate_tree(msh_tree* t);

extern "C" {

const char* msh_last_error(void) { return g_err.c_str(); }

int msh_version(void) { return 2; }

#ifndef MSH_SRC_HASH
#define MSH_SRC_HASH "unknown"
#endif
const char* msh_build_id(void) { return MSH_SRC_HASH; }

int msh_device_count(int* n) {
    int c = 0;
    hipError_t e = hipGetDeviceCount(&c);
    if (e != hipSuccess) {
        *n = 0;
        set_error("hipGetDeviceCount: %s", hipGetErrorString(e));
        return MSH_EDEVICE;
    }
    *n = c;
    return MSH_OK;
}

// the calling thread's device, without touching its device list (msh_set_device_list selects its first entry here)
static int select_device(int device) {
    int c = 0;
    MSH_TRY(msh_device_count(&c));
    if (device < 0 || device >= c) {
        set_error("device %d out of range (%d devices)", device, c);
        return MSH_EINVAL;
    }
    g_device = device;
    return use_device(device);
}

// One device: the device list of msh_set_devices / msh_set_device_list is dropped too, so later trees are built
// on `device` alone and never replicated onto devices the caller no longer asked for.
int msh_set_device(int device) {
    MSH_TRY(select_device(device));
    g_devices.clear();
    return MSH_OK;
}

int msh_set_device_list(const int* devices, int G) {
    if (G < 0 || (G > 0 && !devices) || G > 64) { set_error("msh_set_device_list: bad device list (G = %d)", G); return MSH_EINVAL; }
    int c = 0;
    MSH_TRY(msh_device_count(&c));
    for (int g = 0; g < G; ++g)
        if (devices[g] < 0 || devices[g] >= c) {
            set_error("msh_set_device_list: device %d out of range (%d devices)", devices[g], c);
            return MSH_EINVAL;
        }
    if (G <= 1) {
        g_devices.clear();
        return G == 1 ? select_device(devices[0]) : MSH_OK;
    }
    MSH_TRY(select_device(devices[0]));
    g_devices.assign(devices, devices + G);
    return MSH_OK;
}

int msh_set_devices(int G) {
    int c = 0, d = 0;
    MSH_TRY(msh_device_count(&c));
    MSH_TRY(current_device(&d));
    if (G < 1 || d + G > c) {
        set_error("msh_set_devices: %d devices from device %d (%d visible)", G, d, c);
        return MSH_EINVAL;
    }
    std::vector<int> list(G);
    for (int g = 0; g < G; ++g) list[g] = d + g;
    return msh_set_device_list(list.data(), G);
}

int msh_tree_devices(const msh_tree* t, int* devices, int cap, int* G) {
    if (!t || !G) { set_error("msh_tree_devices: null argument"); return MSH_EINVAL; }
    *G = 1 + (int)t->replicas.size();
    if (devices && cap > 0) devices[0] = t->device;
    for (int g = 1; g < *G && g < cap; ++g)
        if (devices) devices[g] = t->replicas[g - 1]->device;
    return MSH_OK;
}

int msh_device_plan(uint64_t S, int G, uint64_t* begins) {
    if (G < 1 || !begins) { set_error("msh_device_plan: bad argument"); return MSH_EINVAL; }
    for (int g = 0; g < G; ++g) {
        size_t r0, n;
        shard_rows((size_t)S, (size_t)G, (size_t)g, &r0, &n);
        begins[g] = r0;
    }
    begins[G] = S;
    return MSH_OK;
}

int msh_tree_build_ex(const double* v, size_t P, const uint32_t* f, size_t T, const double* ev, size_t EP,
                      const uint32_t* ef, size_t ET, msh_tree** out) {
    if (!out) { set_error("null output handle"); return MSH_EINVAL; }
    *out = nullptr;
    if (T + ET == 0) { set_error("cannot build a tree over an empty mesh (0 faces)"); return MSH_EINVAL; }
    if (P > 0xFFFFFFFFull || T + ET > 0x7FFFFFFFull) { set_error("mesh too large"); return MSH_EINVAL; }
    MSH_TRY(check_faces(f, T, P, "faces"));
    if (ET) MSH_TRY(check_faces(ef, ET, EP, "extra faces"));
    msh_tree* t = nullptr;
    MSH_TRY(new_tree(kTriangles, &t));
    t->P = P;
    t->T = T + ET;
    t->T_main = T;
    int st;
    if (ET == 0) {
        st = build_triangles(t, v, P, f, T);
    } else {
        std::vector<double> vall(3 * (P + EP));
        std::memcpy(vall.data(), v, 3 * P * sizeof(double));
        std::memcpy(vall.data() + 3 * P, ev, 3 * EP * sizeof(double));
        std::vector<uint32_t> fall(3 * (T + ET));
        std::memcpy(fall.data(), f, 3 * T * sizeof(uint32_t));
        for (size_t i = 0; i < 3 * ET; ++i) fall[3 * T + i] = ef[i] + (uint32_t)P;
        st = build_triangles(t, vall.data(), P + EP, fall.data(), T + ET);
    }
    if (st == MSH_OK) st = replicate_tree(t);
    if (st != MSH_OK) {
        std::string keep = g_err;
        free_tree(t);
        g_err = keep;
        return st;
    }
    *out = t;
    return MSH_OK;
}

int msh_tree_build(const double* v, size_t P, const uint32_t* f, size_t T, msh_tree** out) {
    return msh_tree_build_ex(v, P, f, T, nullptr, 0, nullptr, 0, out);
}

int msh_ntree_build(const double* v, size_t P, const uint32_t* f, size_t T, double eps, msh_tree** out) {
    MSH_TRY(msh_tree_build_ex(v, P, f, T, nullptr, 0, nullptr, 0, out));
    for (msh_tree* h : {*out}) {
        h->kind = kNormals;  // the normals metric starts at the root: no entry cut is ever built
        h->eps = eps;
        for (msh_tree* r : h->replicas) {
            r->kind = kNormals;
            r->eps = eps;
        }
    }
    return MSH_OK;
}

int msh_points_build(const double* v, size_t P, msh_tree** out) {
    if (!out) { set_error("null output handle"); return MSH_EINVAL; }
    *out = nullptr;
    if (P == 0) { set_error("cannot build a point tree over 0 vertices"); return MSH_EINVAL; }
    if (P > 0x7FFFFFFFull) { set_error("too many points"); return MSH_EINVAL; }
    msh_tree* t = nullptr;
    MSH_TRY(new_tree(kPoints, &t));
    t->P = P;
    t->T = P;
    t->T_main = P;
    hipStream_t s = t->stream;
    int st = MSH_OK;
    DevBuf dLo, dHi, dOrder;
    do {
        hipError_t e = dmalloc(&t->d_v, P * 3 * sizeof(double));
        if (e != hipSuccess) { set_error("hipMalloc: %s", hipGetErrorString(e)); st = MSH_ENOMEM; break; }
        e = hipMemcpyAsync(t->d_v, v, P * 3 * sizeof(double), hipMemcpyHostToDevice, s);
        if (e != hipSuccess) { set_error("H2D: %s", hipGetErrorString(e)); st = MSH_EDEVICE; break; }
        if ((st = dLo.reserve(3 * P * sizeof(double))) != MSH_OK) break;
        if ((st = dHi.reserve(3 * P * sizeof(double))) != MSH_OK) break;
        if ((st = dOrder.reserve(P * sizeof(uint32_t))) != MSH_OK) break;
        if (P > 1) {
            e = dmalloc(&t->d_nodes, (P - 1) * sizeof(BNode));
            if (e != hipSuccess) { set_error("hipMalloc nodes: %s", hipGetErrorString(e)); st = MSH_ENOMEM; break; }
        }
        e = dmalloc(&t->d_leaves, P * sizeof(PtRec));
        if (e != hipSuccess) { set_error("hipMalloc leaves: %s", hipGetErrorString(e)); st = MSH_ENOMEM; break; }
        if ((st = point_bounds(t->d_v, P, dLo.as<double>(), dHi.as<double>(), s)) != MSH_OK) break;
        if ((st = build_lbvh(t, dLo.as<double>(), dHi.as<double>(), P, dOrder.as<uint32_t>())) != MSH_OK) break;
        if ((st = pack_point_leaves(t->d_v, dOrder.as<uint32_t>(), P, static_cast<PtRec*>(t->d_leaves), s)) != MSH_OK)
            break;
        if ((st = build_obb(t, false)) != MSH_OK) break;
        e = hipStreamSynchronize(s);
        if (e != hipSuccess) { set_error("point LBVH build failed: %s", hipGetErrorString(e)); st = MSH_EDEVICE; break; }
    } while (0);
    (void)hipStreamSynchronize(s);
    dLo.release(); dHi.release(); dOrder.release();
    t->ws.release();
    if (st == MSH_OK) st = replicate_tree(t);
    if (st != MSH_OK) {
        std::string keep = g_err;
        free_tree(t);
        g_err = keep;
        return st;
    }
    *out = t;
    return MSH_OK;
}

void msh_tree_free(msh_tree* tree) { free_tree(tree); }

int msh_tree_query_order(msh_tree* t, const double* d_q, size_t S, uint32_t* d_perm, void* stream) {
    MSH_TRY(check_tree(t, kTriangles, "msh_tree_query_order"));
    MSH_TRY(check_count(S, "msh_tree_query_order"));
    if (S == 0) return MSH_OK;
    if (!d_q || !d_perm) { set_error("msh_tree_query_order: null argument"); return MSH_EINVAL; }
    hipStream_t s = pick(t, stream);
    WsOrder order(t, s);
    Workspace& ws = t->ws;
    float lo[3], hi[3];
    query_box(t, lo, hi);
    MSH_TRY(query_sort(lo, hi, d_q, S, kQuerySortLo, ws, s));
    MSH_HIP(hipMemcpyAsync(d_perm, ws.vals.ptr, S * sizeof(uint32_t), hipMemcpyDeviceToDevice, s));
    return MSH_OK;
}

int msh_tree_set_entry_cut(msh_tree* t, int G) {
    if (!t) { set_error("msh_tree_set_entry_cut: null tree handle"); return MSH_EINVAL; }
    if (G > 4096) { set_error("msh_tree_set_entry_cut: G = %d cells per axis (at most 4096)", G); return MSH_EINVAL; }
    const int want = G < 0 ? -1 : G;
    for (msh_tree* r : t->replicas) MSH_TRY(msh_tree_set_entry_cut(r, G));
    // the same grid again: a pending grid is built by the next call whatever its size (an automatic request on a
    // handle holding the coarse automatic grid asks for the fine one, below)
    if (want == t->cut_req && t->cut_state != kCutFailed && !(want < 0 && t->cut_state == kCutBuilt && !t->cut_fine)) {
        t->cut_force = true;
        return MSH_OK;
    }
    free_entry_cut(t);
    t->cut_req = want;
    t->cut_state = kCutPending;
    t->cut_force = true;
    return MSH_OK;
}

int msh_tree_entry_cut_info(const msh_tree* t, int* state, int* G, uint64_t* bytes, double* build_ms) {
    if (!t) { set_error("msh_tree_entry_cut_info: null tree handle"); return MSH_EINVAL; }
    const uint64_t n = t->d_cut ? (uint64_t)t->cut_G * t->cut_G * t->cut_G : 0;
    auto shown = [](const msh_tree* h) { return h->cut_state == kCutPending && !cut_applies(h) ? kCutOff : h->cut_state; };
    if (state) {
        // the handle's state, or the worst of its replicas' (failed, then still pending) when one differs
        *state = shown(t);
        for (const msh_tree* r : t->replicas) {
            const int rs = shown(r);
            if (rs == kCutFailed || (rs == kCutPending && *state != kCutFailed)) *state = rs;
        }
    }
    if (G) *G = t->d_cut ? t->cut_G : 0;
    if (bytes) *bytes = n * (t->cut_wide ? 64 : 32);
    if (build_ms) *build_ms = t->cut_ms;
    return MSH_OK;
}

int msh_tree_get_info(const msh_tree* t, msh_tree_info* info) {
    if (!t || !info) { set_error("null argument"); return MSH_EINVAL; }
    MSH_TRY(finish_pending(const_cast<msh_tree*>(t)));  // an asynchronous batched build: its GPU time
    info->device = t->device;
    info->kind = t->kind;
    info->n_points = t->P;
    info->n_faces = t->T;
    info->n_main_faces = t->T_main;
    info->n_nodes = t->T > 0 ? t->B * (t->T - 1) : 0;
    info->n_meshes = t->B;
    const size_t leaf = t->kind == kPoints ? sizeof(PtRec) : sizeof(TriRec);
    info->bytes = info->n_nodes * sizeof(BNode) + t->B * t->T * leaf;
    info->eps = t->eps;
    for (int k = 0; k < 3; ++k) {
        info->scene_lo[k] = t->scene_lo[k];
        info->scene_hi[k] = t->scene_hi[k];
    }
    info->build_ms = t->build_ms;
    info->node_bytes = (uint32_t)sizeof(BNode);
    info->leaf_bytes = (uint32_t)leaf;
    info->max_depth = t->max_depth;
    return MSH_OK;
}

// ---------------------------------------------------------------------------------------------
// one sorted closest-point launch over d_q (validated; the entry cut already settled by the caller)
static int nearest_run(msh_tree* t, const double* d_q, size_t S, const SlotOut& o, hipStream_t s) {
    WsOrder order(t, s);
    QueryOrder ord;
    MSH_TRY(sort_queries(t, d_q, nullptr, S, s, &ord, true));
    return launch_nearest(t, ord, S, o, s);
}

int msh_tree_nearest_device(msh_tree* t, const double* d_q, size_t S, uint32_t* d_face, uint32_t* d_part, double* d_pt,
                            void* stream) {
    MSH_TRY(check_tree(t, kTriangles, "msh_tree_nearest_device"));
    MSH_TRY(check_count(S, "msh_tree_nearest_device"));
    if (S == 0) return MSH_OK;
    if (!d_q || !d_face || !d_pt) { set_error("msh_tree_nearest_device: null argument"); return MSH_EINVAL; }
    ensure_entry_cut(t, S);
    return nearest_run(t, d_q, S, SlotOut{d_face, d_part, d_pt, nullptr, nullptr}, pick(t, stream));
}

int msh_tree_points_from_faces_device(msh_tree* t, const double* d_q, size_t S, const uint32_t* d_face, uint32_t* d_part,
                                      double* d_pt, void* stream) {
    MSH_TRY(check_tree(t, kTriangles, "msh_tree_points_from_faces_device"));
    MSH_TRY(check_count(S, "msh_tree_points_from_faces_device"));
    if (S == 0) return MSH_OK;
    if (!d_q || !d_face || !d_pt) { set_error("msh_tree_points_from_faces_device: null argument"); return MSH_EINVAL; }
    hipStream_t s = pick(t, stream);
    if (!t->d_face_leaf) {
        uint32_t* inv = nullptr;
        MSH_HIP(dmalloc(&inv, t->T * sizeof(uint32_t)));
        const int st = face_leaf_map(t, inv, s);
        if (st != MSH_OK) {
            (void)hipStreamSynchronize(s);
            (void)dfree(inv);
            return st;
        }
        MSH_HIP(hipStreamSynchronize(s));  // the map is complete before any stream reads it
        t->d_face_leaf = inv;
    }
    // no workspace is used (tree leaves and the map only), so no WsOrder: a rebuild of other ranks' points on a side
    // stream overlaps the next batch's traversal
    return points_from_faces(t, t->d_face_leaf, d_q, S, d_face, d_part, d_pt, s);
}

int msh_tree_nearest_bary_device(msh_tree* t, const double* d_q, size_t S, uint32_t* d_face, double* d_pt, double* d_w,
                                 void* stream) {
    MSH_TRY(check_tree(t, kTriangles, "msh_tree_nearest_bary_device"));
    MSH_TRY(check_count(S, "msh_tree_nearest_bary_device"));
    if (S == 0) return MSH_OK;
    if (!d_q || !d_face || !d_pt || !d_w) { set_error("msh_tree_nearest_bary_device: null argument"); return MSH_EINVAL; }
    ensure_entry_cut(t, S);
    return nearest_run(t, d_q, S, SlotOut{d_face, nullptr, d_pt, nullptr, d_w}, pick(t, stream));
}

// the whole call's rows settle the entry cut once, before its chunks run
// (S_call: the rows of the whole call, over every replica -- each replica's automatic cut counts them all, so a
// G-device handle builds its cuts at the call a one-device handle would)
static int nearest_host(msh_tree* t, const double* q, size_t S, uint32_t* face, uint32_t* part, double* pt,
                        size_t S_call) {
    MSH_TRY(use_device(t->device));
    ensure_entry_cut(t, S_call);
    // rows: q (24 B in) | face (4 B out) | part (4 B out) | point (24 B out)
    const std::vector<HostArr> arrs = {{q, nullptr, 24}, {nullptr, face, 4}, {nullptr, part, 4}, {nullptr, pt, 24}};
    return pipelined(t, S, arrs, [&](size_t, size_t n, const std::vector<char*>& d) {
        return nearest_run(t, reinterpret_cast<const double*>(d[0]), n,
                           SlotOut{reinterpret_cast<uint32_t*>(d[1]), part ? reinterpret_cast<uint32_t*>(d[2]) : nullptr,
                                   reinterpret_cast<double*>(d[3]), nullptr, nullptr},
                           t->stream);
    });
}

int msh_tree_nearest(msh_tree* t, const double* q, size_t S, uint32_t* face, uint32_t* part, double* pt) {
    MSH_TRY(check_tree(t, kTriangles, "msh_tree_nearest"));
    MSH_TRY(check_count(S, "msh_tree_nearest"));
    if (S == 0) return MSH_OK;
    if (!q || !face || !pt) { set_error("msh_tree_nearest: null argument"); return MSH_EINVAL; }
    return fan_out(t, S, 56, [&](msh_tree* h, size_t r0, size_t n) {
        return nearest_host(h, q + 3 * r0, n, face + r0, part ? part + r0 : nullptr, pt + 3 * r0, S);
    });
}

int msh_tree_nearest_bary(msh_tree* t, const double* q, size_t S, uint32_t* face, double* pt, double* w) {
    MSH_TRY(check_tree(t, kTriangles, "msh_tree_nearest_bary"));
    MSH_TRY(check_count(S, "msh_tree_nearest_bary"));
    if (S == 0) return MSH_OK;
    if (!q || !face || !pt || !w) { set_error("msh_tree_nearest_bary: null argument"); return MSH_EINVAL; }
    return fan_out(t, S, 76, [&](msh_tree* h, size_t r0, size_t S_h) {
        MSH_TRY(use_device(h->device));
        ensure_entry_cut(h, S);
        const std::vector<HostArr> arrs = {{q + 3 * r0, nullptr, 24}, {nullptr, face + r0, 4}, {nullptr, pt + 3 * r0, 24},
                                           {nullptr, w + 3 * r0, 24}};
        return pipelined(h, S_h, arrs, [&](size_t, size_t n, const std::vector<char*>& d) {
            return nearest_run(h, reinterpret_cast<const double*>(d[0]), n,
                               SlotOut{reinterpret_cast<uint32_t*>(d[1]), nullptr, reinterpret_cast<double*>(d[2]),
                                       nullptr, reinterpret_cast<double*>(d[3])},
                               h->stream);
        });
    });
}

int msh_tree_nearest_stats(msh_tree* t, const double* d_q, size_t S, uint64_t* nodes, uint64_t* leaves) {
    MSH_TRY(check_tree(t, kTriangles, "msh_tree_nearest_stats"));
    MSH_TRY(check_count(S, "msh_tree_nearest_stats"));
    *nodes = 0;
    *leaves = 0;
    if (S == 0) return MSH_OK;
    ensure_entry_cut(t, S);
    hipStream_t s = t->stream;
    unsigned long long h[48] = {0};
    {
        WsOrder order(t, s);
        QueryOrder ord;
        MSH_TRY(sort_queries(t, d_q, nullptr, S, s, &ord, true));
        MSH_TRY(t->ws.stats.reserve(sizeof(h)));
        MSH_HIP(hipMemsetAsync(t->ws.stats.ptr, 0, sizeof(h), s));
        MSH_TRY(launch_nearest_stats(t, ord, S, t->ws.stats.as<unsigned long long>(), s));
        MSH_HIP(hipMemcpyAsync(h, t->ws.stats.ptr, sizeof(h), hipMemcpyDeviceToHost, s));
    }
    MSH_HIP(hipStreamSynchronize(s));
    *nodes = h[0];
    *leaves = h[1];
    if (getenv("MESH_AMD_STATS_DUMP")) {  // development: wave-iteration utilisation of pass 1
        fprintf(stderr, "[msh stats] S=%zu nodes=%llu leaves=%llu trav_it=%llu trav_lanes=%llu leaf_it=%llu "
                        "leaf_lanes=%llu pass2_items=%llu\n", S, h[0], h[1], h[2], h[3], h[4], h[5], h[6]);
        // per phase: tiles, sum of per-tile max node steps, sum of lane steps, sum of min(tile max, 128 / 256 /
        // 512), lanes over 128 / 256 / 512 steps
        const char* nm[3] = {"super", "lead", "follow"};
        for (int p = 0; p < 3; ++p) {
            const unsigned long long* x = h + 8 + 9 * p;
            fprintf(stderr, "[msh tiles] %s tiles=%llu sum_max=%llu sum_steps=%llu cap128=%llu cap256=%llu "
                            "cap512=%llu over128=%llu over256=%llu over512=%llu\n", nm[p], x[0], x[1], x[2], x[3],
                    x[4], x[5], x[6], x[7], x[8]);
        }
        fprintf(stderr, "[msh pass2] waves=%llu items=%llu visits_sum=%llu visits_max_item=%llu\n", h[6], h[46], h[44],
                h[45]);
        fprintf(stderr, "[msh leaves] improving_phase_tests=%llu hinted=%llu hint_leaf_won=%llu\n", h[36], h[37], h[38]);
    }
    return MSH_OK;
}

// the rays' walks start from the tree's entry cut (built by the automatic policy on these rows too: rays_cut)
static int along_run(msh_tree* t, const double* d_p, const double* d_n, size_t S, double* d_dist, uint32_t* d_face,
                     double* d_pt, hipStream_t s) {
    WsOrder order(t, s);
    QueryOrder ord;
    MSH_TRY(sort_queries(t, d_p, d_n, S, s, &ord, kAlongLazy));
    return launch_alongnormal(t, ord, S, SlotOut{d_face, nullptr, d_pt, nullptr, d_dist}, s);
}

int msh_tree_nearest_alongnormal_device(msh_tree* t, const double* d_p, const double* d_n, size_t S, double* d_dist,
                                        uint32_t* d_face, double* d_pt, void* stream) {
    MSH_TRY(check_tree(t, kTriangles, "msh_tree_nearest_alongnormal_device"));
    MSH_TRY(check_count(S, "msh_tree_nearest_alongnormal_device"));
    if (S == 0) return MSH_OK;
    ensure_entry_cut(t, S);
    return along_run(t, d_p, d_n, S, d_dist, d_face, d_pt, pick(t, stream));
}

static int read_stats(msh_tree* t, hipStream_t s, uint64_t* nodes, uint64_t* leaves) {
    unsigned long long h[2] = {0, 0};
    MSH_HIP(hipMemcpyAsync(h, t->ws.stats.ptr, sizeof(h), hipMemcpyDeviceToHost, s));
    MSH_HIP(hipStreamSynchronize(s));
    *nodes = h[0];
    *leaves = h[1];
    return MSH_OK;
}

int msh_tree_nearest_alongnormal_stats(msh_tree* t, const double* d_p, const double* d_n, size_t S, uint64_t* nodes,
                                       uint64_t* leaves) {
    MSH_TRY(check_tree(t, kTriangles, "msh_tree_nearest_alongnormal_stats"));
    MSH_TRY(check_count(S, "msh_tree_nearest_alongnormal_stats"));
    if (!nodes || !leaves) { set_error("msh_tree_nearest_alongnormal_stats: null argument"); return MSH_EINVAL; }
    *nodes = *leaves = 0;
    if (S == 0) return MSH_OK;
    ensure_entry_cut(t, S);
    hipStream_t s = t->stream;
    {
        WsOrder order(t, s);
        QueryOrder ord;
        MSH_TRY(sort_queries(t, d_p, d_n, S, s, &ord, kAlongLazy));
        MSH_TRY(t->ws.stats.reserve(8 * sizeof(unsigned long long)));
        MSH_HIP(hipMemsetAsync(t->ws.stats.ptr, 0, 8 * sizeof(unsigned long long), s));
        MSH_TRY(launch_alongnormal_stats(t, ord, S, t->ws.stats.as<unsigned long long>(), s));
    }
    return read_stats(t, s, nodes, leaves);
}

int msh_visibility_stats(msh_tree* t, const double* d_cams, size_t C, double min_dist, uint64_t* nodes,
                         uint64_t* leaves) {
    MSH_TRY(check_tree(t, kTriangles, "msh_visibility_stats"));
    if (!nodes || !leaves || (C && !d_cams)) { set_error("msh_visibility_stats: null argument"); return MSH_EINVAL; }
    *nodes = *leaves = 0;
    if (C == 0 || t->P == 0) return MSH_OK;
    hipStream_t s = t->stream;
    {
        WsOrder order(t, s);
        MSH_TRY(t->ws.stats.reserve(8 * sizeof(unsigned long long)));
        MSH_HIP(hipMemsetAsync(t->ws.stats.ptr, 0, 8 * sizeof(unsigned long long), s));
        MSH_TRY(launch_visibility_stats(t, d_cams, C, min_dist, t->ws.stats.as<unsigned long long>(), s));
    }
    return read_stats(t, s, nodes, leaves);
}

int msh_tree_nearest_alongnormal(msh_tree* t, const double* p, const double* n, size_t S, double* dist, uint32_t* face,
                                 double* pt) {
    MSH_TRY(check_tree(t, kTriangles, "msh_tree_nearest_alongnormal"));
    MSH_TRY(check_count(S, "msh_tree_nearest_alongnormal"));
    if (S == 0) return MSH_OK;
    if (!p || !n || !dist || !face || !pt) { set_error("msh_tree_nearest_alongnormal: null argument"); return MSH_EINVAL; }
    return fan_out(t, S, 84, [&](msh_tree* h, size_t r0, size_t S_h) {
        MSH_TRY(use_device(h->device));
        ensure_entry_cut(h, S);  // the whole call's rows, once (as nearest_host)
        const std::vector<HostArr> arrs = {{p + 3 * r0, nullptr, 24}, {n + 3 * r0, nullptr, 24}, {nullptr, dist + r0, 8},
                                           {nullptr, face + r0, 4}, {nullptr, pt + 3 * r0, 24}};
        return pipelined(h, S_h, arrs, [&](size_t, size_t c, const std::vector<char*>& d) {
            return along_run(h, reinterpret_cast<const double*>(d[0]), reinterpret_cast<const double*>(d[1]), c,
                             reinterpret_cast<double*>(d[2]), reinterpret_cast<uint32_t*>(d[3]),
                             reinterpret_cast<double*>(d[4]), h->stream);
        });
    });
}

static void host_tris(const double* v, const uint32_t* f, size_t T, std::vector<TriRec>& out) {
    out.resize(T);
    for (size_t t = 0; t < T; ++t) {
        for (int c = 0; c < 3; ++c)
            for (int k = 0; k < 3; ++k) out[t].v[3 * c + k] = v[3 * (size_t)f[3 * t + c] + k];
        out[t].face = (uint32_t)t;
        out[t].pad = 0;
    }
}

int msh_tree_intersections(msh_tree* t, const double* qv, size_t Pq, const uint32_t* qf, size_t Tq, uint32_t* out,
                           size_t* K) {
    MSH_TRY(check_tree(t, kTriangles, "msh_tree_intersections"));
    *K = 0;
    if (Tq == 0) return MSH_OK;
    MSH_TRY(check_count(Tq, "msh_tree_intersections"));
    MSH_TRY(check_faces(qf, Tq, Pq, "query faces"));
    hipStream_t s = t->stream;
    std::vector<TriRec> ht;
    host_tris(qv, qf, Tq, ht);
    DevBuf dq, df;
    int st = MSH_OK;
    std::vector<uint32_t> flags(Tq);
    do {
        WsOrder order(t, s);
        if ((st = upload(dq, ht.data(), Tq, s)) != MSH_OK) break;
        if ((st = df.reserve(Tq * sizeof(uint32_t))) != MSH_OK) break;
        if ((st = launch_tri_intersect(t, dq.as<TriRec>(), Tq, 0, df.as<uint32_t>(), s)) != MSH_OK) break;
        hipError_t e;
        if ((e = hipMemcpyAsync(flags.data(), df.ptr, Tq * sizeof(uint32_t), hipMemcpyDeviceToHost, s)) != hipSuccess ||
            (e = hipStreamSynchronize(s)) != hipSuccess) {
            set_error("intersections: %s", hipGetErrorString(e));
            st = MSH_EDEVICE;
        }
    } while (0);
    (void)hipStreamSynchronize(s);
    dq.release();
    df.release();
    if (st != MSH_OK) return st;
    size_t k = 0;
    for (size_t i = 0; i < Tq; ++i)
        if (flags[i]) out[k++] = (uint32_t)i;
    *K = k;
    return MSH_OK;
}

int msh_ntree_nearest(msh_tree* t, const double* q, const double* n, size_t S, uint32_t* face, double* pt) {
    MSH_TRY(check_tree(t, kNormals, "msh_ntree_nearest"));
    MSH_TRY(check_count(S, "msh_ntree_nearest"));
    if (S == 0) return MSH_OK;
    if (!q || !n || !face || !pt) { set_error("msh_ntree_nearest: null argument"); return MSH_EINVAL; }
    return fan_out(t, S, 76, [&](msh_tree* h, size_t r0, size_t S_h) {
        MSH_TRY(use_device(h->device));
        // rows: q (24 B in) | n (24 B in) | face (4 B out) | point (24 B out); chunked like msh_tree_nearest
        const std::vector<HostArr> arrs = {{q + 3 * r0, nullptr, 24}, {n + 3 * r0, nullptr, 24}, {nullptr, face + r0, 4},
                                           {nullptr, pt + 3 * r0, 24}};
        return pipelined(h, S_h, arrs, [&](size_t, size_t c, const std::vector<char*>& d) {
            hipStream_t s = h->stream;
            WsOrder order(h, s);
            QueryOrder ord;
            MSH_TRY(sort_queries(h, reinterpret_cast<const double*>(d[0]), reinterpret_cast<const double*>(d[1]), c, s, &ord));
            return launch_nnearest(h, ord, c, SlotOut{reinterpret_cast<uint32_t*>(d[2]), nullptr,
                                                      reinterpret_cast<double*>(d[3]), nullptr, nullptr}, s);
        });
    });
}

int msh_ntree_selfintersects(msh_tree* t, int64_t* count) {
    MSH_TRY(check_tree(t, kNormals, "msh_ntree_selfintersects"));
    *count = 0;
    hipStream_t s = t->stream;
    DevBuf df;
    std::vector<uint32_t> flags(t->T);
    int st = MSH_OK;
    do {
        WsOrder order(t, s);
        if ((st = df.reserve(t->T * sizeof(uint32_t))) != MSH_OK) break;
        if ((st = launch_tri_intersect(t, static_cast<const TriRec*>(t->d_leaves), t->T, 1, df.as<uint32_t>(), s)) !=
            MSH_OK)
            break;
        hipError_t e;
        if ((e = hipMemcpyAsync(flags.data(), df.ptr, t->T * sizeof(uint32_t), hipMemcpyDeviceToHost, s)) != hipSuccess ||
            (e = hipStreamSynchronize(s)) != hipSuccess) {
            set_error("selfintersects: %s", hipGetErrorString(e));
            st = MSH_EDEVICE;
        }
    } while (0);
    (void)hipStreamSynchronize(s);
    df.release();
    if (st != MSH_OK) return st;
    int64_t c = 0;
    for (uint32_t x : flags) c += x ? 1 : 0;
    *count = c;
    return MSH_OK;
}

int msh_visibility_device(msh_tree* t, const double* d_cams, size_t C, const double* d_normals, const double* d_sensors,
                          double min_dist, size_t v_begin, size_t v_count, uint32_t* d_vis, double* d_ndc, void* stream) {
    MSH_TRY(check_tree(t, kTriangles, "msh_visibility_device"));
    if (v_begin > t->P || v_count > t->P - v_begin) {
        set_error("msh_visibility_device: vertex range [%zu, %zu) outside the %zu main-mesh vertices", v_begin,
                  v_begin + v_count, t->P);
        return MSH_EINVAL;
    }
    if (C * v_count == 0) return MSH_OK;
    hipStream_t s = pick(t, stream);
    WsOrder order(t, s);
    return launch_visibility(t, d_cams, C, d_normals, d_sensors, min_dist, v_begin, v_count, d_vis, d_ndc, s);
}

// Host arrays: the cameras, normals and sensors are uploaded once; the (C, P) outputs come back through the pinned
// pipeline a few cameras at a time (api.cpp pipelined(): rows = cameras), so the downloads of earlier cameras (C5:
// 30 MB per camera, 1.92 GB in all) overlap the rays of later ones, and land straight in page-locked pool arrays
// when the caller's arrays are carved from it.
static int visibility_host(msh_tree* t, const double* cams, size_t C, const double* normals, const double* sensors,
                           double min_dist, uint32_t* vis, double* ndc) {
    MSH_TRY(use_device(t->device));
    const size_t P = t->P;
    hipStream_t s = t->stream;
    DevBuf dc, dn, ds;
    int st = MSH_OK;
    do {
        if ((st = upload(dc, cams, 3 * C, s)) != MSH_OK) break;
        if (normals && (st = upload(dn, normals, 3 * P, s)) != MSH_OK) break;
        if (sensors && (st = upload(ds, sensors, 9 * C, s)) != MSH_OK) break;
        const std::vector<HostArr> arrs = {{nullptr, vis, P * sizeof(uint32_t)}, {nullptr, ndc, P * sizeof(double)}};
        const std::vector<size_t> plan = {std::max<size_t>(1, ((size_t)16 << 20) / P)};  // ~16M rays a chunk
        st = pipelined(t, C, arrs, [&](size_t c0, size_t nc, const std::vector<char*>& d) {
            return msh_visibility_device(t, dc.as<double>() + 3 * c0, nc, normals ? dn.as<double>() : nullptr,
                                         sensors ? ds.as<double>() + 9 * c0 : nullptr, min_dist, 0, P,
                                         reinterpret_cast<uint32_t*>(d[0]), reinterpret_cast<double*>(d[1]), s);
        }, &plan);
    } while (0);
    (void)hipStreamSynchronize(s);
    return st;
}

// Host arrays: the cameras, normals and sensors are uploaded once; the (C, P) outputs come back through the pinned
// pipeline a few cameras at a time (api.cpp pipelined(): rows = cameras), so the downloads of earlier cameras (C5:
// 30 MB per camera, 1.92 GB in all) overlap the rays of later ones, and land straight in page-locked pool arrays
// when the caller's arrays are carved from it.  With replicas (msh_set_devices) each device casts a camera range.
int msh_visibility(msh_tree* t, const double* cams, size_t C, const double* normals, const double* sensors,
                   double min_dist, uint32_t* vis, double* ndc) {
    MSH_TRY(check_tree(t, kTriangles, "msh_visibility"));
    const size_t P = t->P;
    if (C * P == 0) return MSH_OK;
    if (!cams || !vis || !ndc) { set_error("msh_visibility: null argument"); return MSH_EINVAL; }
    return fan_out(t, C, 12 * P, [&](msh_tree* h, size_t c0, size_t nc) {
        return visibility_host(h, cams + 3 * c0, nc, normals, sensors ? sensors + 9 * c0 : nullptr, min_dist,
                               vis + c0 * P, ndc + c0 * P);
    });
}

int msh_points_nearest(msh_tree* t, const double* q, size_t S, uint32_t* idx, double* dist) {
    MSH_TRY(check_tree(t, kPoints, "msh_points_nearest"));
    MSH_TRY(check_count(S, "msh_points_nearest"));
    if (S == 0) return MSH_OK;
    if (!q || !idx || !dist) { set_error("msh_points_nearest: null argument"); return MSH_EINVAL; }
    return fan_out(t, S, 36, [&](msh_tree* h, size_t r0, size_t S_h) {
        MSH_TRY(use_device(h->device));
        // rows: q (24 B in) | index (4 B out) | distance (8 B out); chunked like msh_tree_nearest
        const std::vector<HostArr> arrs = {{q + 3 * r0, nullptr, 24}, {nullptr, idx + r0, 4}, {nullptr, dist + r0, 8}};
        return pipelined(h, S_h, arrs, [&](size_t, size_t c, const std::vector<char*>& d) {
            hipStream_t s = h->stream;
            WsOrder order(h, s);
            QueryOrder ord;
            MSH_TRY(sort_queries(h, reinterpret_cast<const double*>(d[0]), nullptr, c, s, &ord));
            return launch_points_nearest(h, ord, c, SlotOut{reinterpret_cast<uint32_t*>(d[1]), nullptr, nullptr,
                                                            reinterpret_cast<double*>(d[2]), nullptr}, s);
        });
    });
}

// ---- mesh geometry ----
int msh_vertex_normals_device(const double* d_v, size_t P, const uint32_t* d_f, size_t T, double* d_vn, void* stream) {
    if (P && (!d_v || !d_vn)) { set_error("msh_vertex_normals_device: null argument"); return MSH_EINVAL; }
    if (T && !d_f) { set_error("msh_vertex_normals_device: null faces"); return MSH_EINVAL; }
    if (P > 0xFFFFFFFFull) { set_error("msh_vertex_normals_device: too many vertices"); return MSH_EINVAL; }
    int dev = 0;
    MSH_TRY(current_device(&dev));
    MSH_TRY(use_device(dev));
    hipStream_t s = static_cast<hipStream_t>(stream);
    Workspace ws;
    int st = ws.flags.reserve(sizeof(uint32_t));
    uint32_t h_err = 0;
    if (st == MSH_OK && hipMemsetAsync(ws.flags.ptr, 0, sizeof(uint32_t), s) != hipSuccess) st = MSH_EDEVICE;
    if (st == MSH_OK) st = vertex_normals(d_v, P, d_f, T, d_vn, ws, s, ws.flags.as<uint32_t>());
    if (st == MSH_OK && hipMemcpyAsync(&h_err, ws.flags.ptr, sizeof(uint32_t), hipMemcpyDeviceToHost, s) != hipSuccess)
        st = MSH_EDEVICE;
    hipError_t e = hipStreamSynchronize(s);  // the scratch below is released on return
    ws.release();
    if (st == MSH_OK && e != hipSuccess) {
        set_error("vertex normals: %s", hipGetErrorString(e));
        st = MSH_EDEVICE;
    }
    if (st == MSH_OK && h_err) {
        set_error("msh_vertex_normals_device: face index out of range (>= %zu vertices)", P);
        st = MSH_EINVAL;
    }
    return st;
}

int msh_vertex_normals(const double* v, size_t P, const uint32_t* f, size_t T, double* vn) {
    if (P && (!v || !vn)) { set_error("msh_vertex_normals: null argument"); return MSH_EINVAL; }
    MSH_TRY(check_faces(f, T, P, "msh_vertex_normals"));
    if (P == 0) return MSH_OK;
    int dev = 0;
    MSH_TRY(current_device(&dev));
    MSH_TRY(use_device(dev));
    hipStream_t s = nullptr;
    MSH_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    DevBuf dv, df, dn;
    int st = MSH_OK;
    do {
        if ((st = upload(dv, v, 3 * P, s)) != MSH_OK) break;
        if ((st = upload(df, f, 3 * T, s)) != MSH_OK) break;
        if ((st = dn.reserve(3 * P * sizeof(double))) != MSH_OK) break;
        if ((st = msh_vertex_normals_device(dv.as<double>(), P, df.as<uint32_t>(), T, dn.as<double>(), s)) != MSH_OK)
            break;
        hipError_t e;
        if ((e = hipMemcpyAsync(vn, dn.ptr, 3 * P * sizeof(double), hipMemcpyDeviceToHost, s)) != hipSuccess ||
            (e = hipStreamSynchronize(s)) != hipSuccess) {
            set_error("vertex normals: %s", hipGetErrorString(e));
            st = MSH_EDEVICE;
        }
    } while (0);
    (void)hipStreamSynchronize(s);
    dv.release(); df.release(); dn.release();
    (void)hipStreamDestroy(s);
    return st;
}

// ---- blob (RCCL replication) ----
struct BlobHeader {
    uint64_t magic;
    int32_t kind, max_depth;
    uint64_t P, T, T_main, v_rows;
    double eps;
    float scene_lo[3], scene_hi[3];
    uint64_t off_v, off_nodes, off_leaves, total;
    double origin[3];
    uint32_t node_bytes, leaf_bytes;
};
static const uint64_t kBlobMagic = 0x4d53484c42564835ull;  // "MSHLBVH5" (interleaved node frame, bf16 scales)

static size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

static void blob_layout_sizes(int kind, uint64_t P, uint64_t T, BlobHeader& h) {
    std::memset(&h, 0, sizeof(h));
    h.magic = kBlobMagic;
    h.kind = kind;
    h.P = P;
    h.T = T;
    // visibility trees keep the extra-mesh vertices after the main rows; only the main rows are needed
    h.v_rows = P;
    h.node_bytes = (uint32_t)sizeof(BNode);
    h.leaf_bytes = (uint32_t)(kind == kPoints ? sizeof(PtRec) : sizeof(TriRec));
    h.off_v = align256(sizeof(BlobHeader));
    h.off_nodes = align256(h.off_v + h.v_rows * 3 * sizeof(double));
    h.off_leaves = align256(h.off_nodes + (T > 1 ? (T - 1) * sizeof(BNode) : 0));
    h.total = align256(h.off_leaves + T * h.leaf_bytes);
}

static void blob_layout(const msh_tree* t, BlobHeader& h) {
    blob_layout_sizes(t->kind, t->P, t->T, h);
    h.max_depth = t->max_depth;
    h.T_main = t->T_main;
    h.eps = t->eps;
    for (int k = 0; k < 3; ++k) {
        h.scene_lo[k] = t->scene_lo[k];
        h.scene_hi[k] = t->scene_hi[k];
        h.origin[k] = t->origin[k];
    }
}

static int blob_check(const BlobHeader& h, size_t bytes) {
    BlobHeader want;
    if (h.magic != kBlobMagic) {
        set_error("not a meshsearch tree blob (magic %llx)", (unsigned long long)h.magic);
        return MSH_EINVAL;
    }
    if (h.kind < 0 || h.kind > 2 || h.T == 0 || h.T > 0x7FFFFFFFull || h.P > 0xFFFFFFFFull) {
        set_error("corrupt tree blob header (kind %d, P %llu, T %llu)", h.kind, (unsigned long long)h.P,
                  (unsigned long long)h.T);
        return MSH_EINVAL;
    }
    blob_layout_sizes(h.kind, h.P, h.T, want);
    if (h.node_bytes != want.node_bytes || h.leaf_bytes != want.leaf_bytes || h.off_v != want.off_v ||
        h.off_nodes != want.off_nodes || h.off_leaves != want.off_leaves || h.total != want.total) {
        set_error("tree blob layout mismatch (built by a different library version?)");
        return MSH_EINVAL;
    }
    if (h.total > bytes) {
        set_error("tree blob truncated: header says %llu bytes, %zu given", (unsigned long long)h.total, bytes);
        return MSH_EINVAL;
    }
    return MSH_OK;
}

static void blob_info_of(const BlobHeader& h, msh_blob_info* out) {
    out->kind = h.kind;
    out->max_depth = h.max_depth;
    out->n_points = h.P;
    out->n_faces = h.T;
    out->n_main_faces = h.T_main;
    out->off_vertices = h.off_v;
    out->off_nodes = h.off_nodes;
    out->off_leaves = h.off_leaves;
    out->total = h.total;
    out->node_bytes = h.node_bytes;
    out->leaf_bytes = h.leaf_bytes;
    for (int k = 0; k < 3; ++k) out->origin[k] = h.origin[k];
}

int msh_blob_header_write(int kind, uint64_t P, uint64_t T, uint64_t T_main, void* dst, size_t cap, msh_blob_info* info) {
    if (!dst || kind < 0 || kind > 2 || T == 0) { set_error("msh_blob_header_write: bad argument"); return MSH_EINVAL; }
    BlobHeader h;
    blob_layout_sizes(kind, P, T, h);
    h.T_main = T_main;
    if (cap < sizeof(h)) { set_error("msh_blob_header_write: %zu bytes < header", cap); return MSH_EINVAL; }
    std::memcpy(dst, &h, sizeof(h));
    if (info) blob_info_of(h, info);
    return MSH_OK;
}

int msh_blob_header_parse(const void* src, size_t bytes, msh_blob_info* info) {
    if (!src || !info) { set_error("msh_blob_header_parse: null argument"); return MSH_EINVAL; }
    BlobHeader h;
    if (bytes < sizeof(h)) { set_error("tree blob shorter than its header (%zu bytes)", bytes); return MSH_EINVAL; }
    std::memcpy(&h, src, sizeof(h));
    MSH_TRY(blob_check(h, bytes));
    blob_info_of(h, info);
    return MSH_OK;
}

int msh_tree_blob_size(const msh_tree* t, size_t* bytes) {
    if (!t || !bytes) { set_error("null argument"); return MSH_EINVAL; }
    if (t->B != 1 || t->d_boxes) { set_error("msh_tree_blob_size: batched trees are not serialisable"); return MSH_EINVAL; }
    BlobHeader h;
    blob_layout(t, h);
    *bytes = h.total;
    return MSH_OK;
}

int msh_tree_blob_pack(const msh_tree* t, void* d_dst, void* stream) {
    if (!t || !d_dst) { set_error("null argument"); return MSH_EINVAL; }
    if (t->B != 1 || t->d_boxes) { set_error("msh_tree_blob_pack: batched trees are not serialisable"); return MSH_EINVAL; }
    MSH_TRY(use_device(t->device));
    hipStream_t s = stream ? static_cast<hipStream_t>(stream) : t->stream;
    BlobHeader h;
    blob_layout(t, h);
    char* dst = static_cast<char*>(d_dst);
    MSH_HIP(hipMemcpyAsync(dst, &h, sizeof(h), hipMemcpyHostToDevice, s));
    if (h.v_rows) MSH_HIP(hipMemcpyAsync(dst + h.off_v, t->d_v, h.v_rows * 3 * sizeof(double), hipMemcpyDeviceToDevice, s));
    if (t->T > 1)
        MSH_HIP(hipMemcpyAsync(dst + h.off_nodes, t->d_nodes, (t->T - 1) * sizeof(BNode), hipMemcpyDeviceToDevice, s));
    MSH_HIP(hipMemcpyAsync(dst + h.off_leaves, t->d_leaves, t->T * h.leaf_bytes, hipMemcpyDeviceToDevice, s));
    MSH_HIP(hipStreamSynchronize(s));
    return MSH_OK;
}

int msh_tree_blob_unpack(const void* d_src, size_t bytes, int device, void* stream, msh_tree** out) {
    if (!d_src || !out) { set_error("null argument"); return MSH_EINVAL; }
    *out = nullptr;
    MSH_TRY(use_device(device));
    BlobHeader h;
    if (bytes < sizeof(h)) { set_error("tree blob shorter than its header (%zu bytes)", bytes); return MSH_EINVAL; }
    hipStream_t us = static_cast<hipStream_t>(stream);
    MSH_HIP(hipMemcpyAsync(&h, d_src, sizeof(h), hipMemcpyDeviceToHost, us));
    MSH_HIP(hipStreamSynchronize(us));
    MSH_TRY(blob_check(h, bytes));
    const int prev = g_device;
    g_device = device;
    msh_tree* t = nullptr;
    int st = new_tree(h.kind, &t);
    g_device = prev;
    MSH_TRY(st);
    t->max_depth = h.max_depth;
    t->P = h.P;
    t->T = h.T;
    t->T_main = h.T_main;
    t->eps = h.eps;
    for (int k = 0; k < 3; ++k) {
        t->scene_lo[k] = h.scene_lo[k];
        t->scene_hi[k] = h.scene_hi[k];
        t->origin[k] = h.origin[k];
    }
    {
        // from the fp32-rounded scene box: widened by far more than its rounding (2^-24 relative)
        const double box[6] = {h.scene_lo[0], h.scene_lo[1], h.scene_lo[2], h.scene_hi[0], h.scene_hi[1], h.scene_hi[2]};
        t->half_diag = half_diagonal(box, t->origin) * (1.0 + 1e-6);
    }
    const char* src = static_cast<const char*>(d_src);
    const size_t leaf = h.leaf_bytes;
    hipStream_t s = us ? us : t->stream;
    do {
        hipError_t e = dmalloc(&t->d_v, std::max<uint64_t>(h.v_rows, 1) * 3 * sizeof(double));
        if (e == hipSuccess && h.v_rows)
            e = hipMemcpyAsync(t->d_v, src + h.off_v, h.v_rows * 3 * sizeof(double), hipMemcpyDeviceToDevice, s);
        if (e == hipSuccess && h.T > 1) e = dmalloc(&t->d_nodes, (h.T - 1) * sizeof(BNode));
        if (e == hipSuccess && h.T > 1)
            e = hipMemcpyAsync(t->d_nodes, src + h.off_nodes, (h.T - 1) * sizeof(BNode), hipMemcpyDeviceToDevice, s);
        if (e == hipSuccess) e = dmalloc(&t->d_leaves, h.T * leaf);
        if (e == hipSuccess) e = hipMemcpyAsync(t->d_leaves, src + h.off_leaves, h.T * leaf, hipMemcpyDeviceToDevice, s);
        if (e == hipSuccess) e = hipStreamSynchronize(s);
        if (e != hipSuccess) {
            set_error("blob unpack: %s", hipGetErrorString(e));
            st = MSH_EDEVICE;
            break;
        }
        if ((st = upload_origin(t, t->stream)) != MSH_OK) break;
        if (hipStreamSynchronize(t->stream) != hipSuccess) {
            set_error("blob unpack: origin upload failed");
            st = MSH_EDEVICE;
            break;
        }
        // the entry cut is derived from the tree: not shipped, built by the first closest-point query here
        t->ws.release();
    } while (0);
    if (st != MSH_OK) {
        std::string keep = g_err;
        free_tree(t);
        g_err = keep;
        return st;
    }
    *out = t;
    return MSH_OK;
}

// ---- timing ----
int msh_timing_enable(int on) {
    std::lock_guard<std::mutex> g(g_tmu);
    g_timing = on != 0;
    return MSH_OK;
}

int msh_timing_get(const char* name, double* ms, int64_t* count) {
    resolve_pending();
    std::lock_guard<std::mutex> g(g_tmu);
    auto it = g_times.find(name ? name : "");
    *ms = it == g_times.end() ? 0.0 : it->second.first;
    *count = it == g_times.end() ? 0 : it->second.second;
    return MSH_OK;
}

int msh_host_alloc(size_t bytes, void** out) {
    if (!out) { set_error("msh_host_alloc: null argument"); return MSH_EINVAL; }
    *out = nullptr;
    return pinned_pool().alloc(bytes, out);
}

void msh_host_free(void* p) {
    if (p) pinned_pool().release(p);
}

int msh_host_pool_trim(void) {
    stage_pool().trim();
    return pinned_pool().trim();
}

size_t msh_host_pool_bytes(void) { return pinned_pool().bytes(); }

int msh_device_pool_trim(void) {
    ws_pool().trim();
    stage_pool().trim();
    dcache_trim();  // last: the workspaces and slabs above were returned to it
    return MSH_OK;
}

int msh_device_pool_bytes(uint64_t* workspace, uint64_t* staging, uint64_t* cached) {
    if (workspace) *workspace = ws_pool().bytes();
    if (staging) *staging = stage_pool().device_bytes();
    if (cached) *cached = dcache_bytes();
    return MSH_OK;
}

int msh_timing_reset(void) {
    resolve_pending();
    std::lock_guard<std::mutex> g(g_tmu);
    g_times.clear();
    return MSH_OK;
}

// ---- batched trees (C4: B meshes sharing one topology) ----
int msh_batch_build(const double* v, size_t B, size_t P, const uint32_t* f, size_t T, msh_tree** out) {
    if (!out) { set_error("msh_batch_build: null output"); return MSH_EINVAL; }
    *out = nullptr;
    if (!v || !f || B == 0 || P == 0 || T < 2) {
        set_error("msh_batch_build: need B >= 1 meshes of P >= 1 vertices and T >= 2 faces (got B=%zu P=%zu T=%zu)",
                  B, P, T);
        return MSH_EINVAL;
    }
    if (B * T > (size_t)0x7FFFFFFF) {
        set_error("msh_batch_build: %zu x %zu faces exceed the 31-bit leaf index range", B, T);
        return MSH_EINVAL;
    }
    MSH_TRY(check_faces(f, T, P, "msh_batch_build"));
    msh_tree* t = nullptr;
    MSH_TRY(new_tree(kTriangles, &t));
    t->B = B;
    t->P = P;
    t->T = T;
    t->T_main = T;
    hipStream_t s = t->stream;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    DevBuf dF, dLo, dHi, dOrder;
    int st = MSH_OK;
    do {
        hipError_t e = hipEventCreate(&e0);
        if (e == hipSuccess) e = hipEventCreate(&e1);
        if (e == hipSuccess) e = dmalloc(&t->d_v, B * P * 3 * sizeof(double));
        if (e == hipSuccess) e = dmalloc(&t->d_nodes, B * (T - 1) * sizeof(BNode));
        if (e == hipSuccess) e = dmalloc(&t->d_leaves, B * T * sizeof(TriRec));
        if (e != hipSuccess) { set_error("msh_batch_build: %s", hipGetErrorString(e)); st = MSH_ENOMEM; break; }
        // the vertices (C4: 496 MB) through the pinned staging pipeline, a chunk of meshes at a time (one pageable
        // hipMemcpy of them ran well below the host link's rate)
        // chunks of ~32 MB, so the host's copies into the pinned slabs overlap the uploads
        const std::vector<HostArr> va = {{v, nullptr, P * 3 * sizeof(double)}};
        const std::vector<size_t> vplan = {std::max<size_t>(1, ((size_t)32 << 20) / (P * 3 * sizeof(double)))};
        st = pipelined(t, B, va, [&](size_t m0, size_t nm, const std::vector<char*>& d) {
            MSH_HIP(hipMemcpyAsync(t->d_v + m0 * P * 3, d[0], nm * P * 3 * sizeof(double), hipMemcpyDeviceToDevice, s));
            return MSH_OK;
        }, &vplan);
        if (st != MSH_OK) break;
        if ((st = upload(dF, f, 3 * T, s)) != MSH_OK) break;
        if ((st = dLo.reserve(3 * B * T * sizeof(double))) != MSH_OK) break;
        if ((st = dHi.reserve(3 * B * T * sizeof(double))) != MSH_OK) break;
        if ((st = dOrder.reserve(B * T * sizeof(uint32_t))) != MSH_OK) break;
        (void)hipEventRecord(e0, s);
        if ((st = tri_bounds_batch(t->d_v, P, dF.as<uint32_t>(), B, T, dLo.as<double>(), dHi.as<double>(), s)) != MSH_OK)
            break;
        if ((st = build_lbvh_batch(t, dLo.as<double>(), dHi.as<double>(), T, dOrder.as<uint32_t>())) != MSH_OK) break;
        if ((st = pack_tri_leaves_batch(t->d_v, P, dF.as<uint32_t>(), dOrder.as<uint32_t>(), B, T,
                                        static_cast<TriRec*>(t->d_leaves), s)) != MSH_OK)
            break;
        if ((st = build_obb(t, true, true)) != MSH_OK) break;
        (void)hipEventRecord(e1, s);
        if (t->ws_done) (void)hipEventRecord(t->ws_done, s);  // *_device calls on other streams wait for the build
    } while (0);
    if (st == MSH_OK) {
        // The tail of the build (leaf packing, oriented boxes) is still running on the handle's stream: return now, so
        // the caller's next call overlaps it (C4 through numpy: the queries' uploads run on the copy stream while the
        // boxes are built; the query kernels follow the build on the handle's stream).  Its temporaries and workspace
        // are freed by finish_pending once it has passed.
        t->pending = true;
        t->pend_e0 = e0;
        t->pend_done = e1;
        e0 = e1 = nullptr;
        for (DevBuf* b : {&dF, &dLo, &dHi, &dOrder}) {
            t->pend_free.push_back(b->ptr);
            b->ptr = nullptr;
            b->bytes = 0;
        }
        t->pend_ws = std::move(t->ws);
        ws_pool().take(t->device, t->ws);  // a freed tree's query workspace, if one is idle
    } else {
        (void)hipStreamSynchronize(s);
        dF.release(); dLo.release(); dHi.release(); dOrder.release();
        t->ws.release();
    }
    if (e0) (void)hipEventDestroy(e0);
    if (e1) (void)hipEventDestroy(e1);
    if (st != MSH_OK) {
        std::string keep = g_err;
        free_tree(t);
        g_err = keep;
        return st;
    }
    *out = t;
    return MSH_OK;
}

// meshes [mesh0, mesh0 + nmesh) of a batched tree; d_q and the outputs hold those meshes' rows only
static int batch_query_range(msh_tree* t, const double* d_q, size_t S, size_t mesh0, size_t nmesh, const SlotOut& o,
                             hipStream_t s) {
    const size_t n = nmesh * S;
    if (n == 0) return MSH_OK;
    WsOrder order(t, s);
    QueryOrder ord;
    MSH_TRY(sort_batch_queries(t, d_q, n, S, s, &ord, mesh0));
    return launch_nearest_batch(t, ord, n, S, o, s, mesh0);
}

static int batch_query(msh_tree* t, const double* d_q, size_t S, const SlotOut& o, void* stream, const char* fn) {
    MSH_TRY(check_batch(t, fn));
    const size_t n = t->B * S;
    if (n == 0) return MSH_OK;
    MSH_TRY(check_count(n, fn));
    // a build still running is waited for on the device (ws_done); its temporaries go once it has passed
    if (t->pending) {
        const hipError_t q = hipEventQuery(t->pend_done);
        // done, or failed: finish_pending reports a failed build's error instead of answering from it
        if (q != hipErrorNotReady) {
            (void)hipGetLastError();
            MSH_TRY(finish_pending(t));
        }
    }
    return batch_query_range(t, d_q, S, 0, t->B, o, pick(t, stream));
}

int msh_batch_nearest_device(msh_tree* t, const double* d_q, size_t S, uint32_t* d_face, uint32_t* d_part, double* d_pt,
                             void* stream) {
    return batch_query(t, d_q, S, SlotOut{d_face, d_part, d_pt, nullptr, nullptr}, stream, "msh_batch_nearest_device");
}

int msh_batch_nearest_bary_device(msh_tree* t, const double* d_q, size_t S, uint32_t* d_face, double* d_pt, double* d_w,
                                  void* stream) {
    if (!d_w) { set_error("msh_batch_nearest_bary_device: null weights"); return MSH_EINVAL; }
    return batch_query(t, d_q, S, SlotOut{d_face, nullptr, d_pt, nullptr, d_w}, stream, "msh_batch_nearest_bary_device");
}

// Host arrays of a batched tree, pipelined over meshes (api.cpp pipelined(): a chunk is a range of whole meshes, so
// its queries sort and run as the meshes' own launch): uploads, kernels and downloads of consecutive chunks overlap,
// and results go straight into page-locked pool arrays (msh_host_alloc) when the caller's arrays are carved from it.
// C4 (4096 meshes x 10k queries): one pageable upload of 983 MB and downloads of 1.3 GB had made the call 4x slower
// than its host-link bound.
static int batch_host(msh_tree* t, const double* q, size_t S, uint32_t* face, uint32_t* part, double* pt, double* w,
                      const char* fn) {
    MSH_TRY(check_batch(t, fn));
    const size_t n = t->B * S;
    if (n == 0) return MSH_OK;
    MSH_TRY(check_count(n, fn));
    if (!q || !face || !pt) { set_error("%s: null argument", fn); return MSH_EINVAL; }
    if (w) part = nullptr;
    // rows = meshes: q (24 S B in) | face (4 S out) | [part (4 S out)] | point (24 S out) | [weights (24 S out)]
    std::vector<HostArr> arrs = {{q, nullptr, 24 * S}, {nullptr, face, 4 * S}};
    const int ipart = part ? (int)arrs.size() : -1;
    if (part) arrs.push_back({nullptr, part, 4 * S});
    const int ipt = (int)arrs.size();
    arrs.push_back({nullptr, pt, 24 * S});
    const int iw = w ? (int)arrs.size() : -1;
    if (w) arrs.push_back({nullptr, w, 24 * S});
    // chunks of ~2M then ~6M queries (whole meshes)
    const std::vector<size_t> plan = {std::max<size_t>(1, ((size_t)2 << 20) / S), std::max<size_t>(1, ((size_t)6 << 20) / S)};
    // the uploads of the first chunks overlap the tail of an asynchronous build; its kernels follow it on t->stream
    const int st = pipelined(t, t->B, arrs, [&](size_t m0, size_t nm, const std::vector<char*>& d) {
        const SlotOut o{reinterpret_cast<uint32_t*>(d[1]), ipart >= 0 ? reinterpret_cast<uint32_t*>(d[ipart]) : nullptr,
                        reinterpret_cast<double*>(d[ipt]), nullptr, iw >= 0 ? reinterpret_cast<double*>(d[iw]) : nullptr};
        return batch_query_range(t, reinterpret_cast<const double*>(d[0]), S, m0, nm, o, t->stream);
    }, &plan);
    const int sb = finish_pending(t);
    return st != MSH_OK ? st : sb;
}

int msh_batch_nearest(msh_tree* t, const double* q, size_t S, uint32_t* face, uint32_t* part, double* pt) {
    return batch_host(t, q, S, face, part, pt, nullptr, "msh_batch_nearest");
}

int msh_batch_nearest_bary(msh_tree* t, const double* q, size_t S, uint32_t* face, double* pt, double* w) {
    if (!w) { set_error("msh_batch_nearest_bary: null weights"); return MSH_EINVAL; }
    return batch_host(t, q, S, face, nullptr, pt, w, "msh_batch_nearest_bary");
}

}  // extern "C"

// Copies of a freshly built tree on the other devices of the calling thread's device list (msh_set_devices): the
// tree is packed into one device blob (msh_tree_blob_pack), copied peer to peer to each device and unpacked there
// (msh_tree_blob_unpack) — the in-process form of bench.py's RCCL broadcast.  A replica on the handle's own device
// (a repeated entry of the list) unpacks from the blob in place.
static int replicate_tree(msh_tree* t) {
    // the list replicates trees built on its first device only (msh_set_device drops it; this is the backstop)
    if (g_devices.size() <= 1 || t->device != g_devices[0]) return MSH_OK;
    size_t bytes = 0;
    MSH_TRY(msh_tree_blob_size(t, &bytes));
    MSH_TRY(use_device(t->device));
    void* blob = nullptr;
    MSH_HIP(dmalloc(&blob, bytes));
    int st = msh_tree_blob_pack(t, blob, nullptr);
    const std::vector<int> devs = g_devices;
    for (size_t g = 1; g < devs.size() && st == MSH_OK; ++g) {
        const int d = devs[g];
        void* src = blob;
        void* copy = nullptr;
        if (d != t->device) {
            (void)hipSetDevice(d);
            hipError_t e = dmalloc(&copy, bytes);
            if (e == hipSuccess) e = hipMemcpyPeer(copy, d, blob, t->device, bytes);
            if (e != hipSuccess) {
                set_error("replicating the tree to device %d: %s", d, hipGetErrorString(e));
                st = e == hipErrorOutOfMemory ? MSH_ENOMEM : MSH_EDEVICE;
                if (copy) (void)dfree(copy);
                break;
            }
            src = copy;
        }
        msh_tree* r = nullptr;
        st = msh_tree_blob_unpack(src, bytes, d, nullptr, &r);
        if (copy) {
            (void)hipSetDevice(d);
            (void)dfree(copy);
        }
        if (st == MSH_OK) {
            r->cut_req = t->cut_req;
            r->cut_force = t->cut_force;
            r->build_ms = t->build_ms;
            t->replicas.push_back(r);
        }
    }
    (void)use_device(t->device);
    (void)dfree(blob);
    return st;
}
