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
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "internal.h"

namespace msh {

static thread_local std::string g_err;
static thread_local int g_device = -1;

void set_error(const char* fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_err = buf;
}

int DevBuf::reserve(size_t need) {
    if (need <= bytes && ptr) return MSH_OK;
    if (ptr) {
        hipError_t e = hipFree(ptr);
        ptr = nullptr;
        bytes = 0;
        MSH_HIP(e);
    }
    if (need == 0) need = 16;
    MSH_HIP(hipMalloc(&ptr, need));
    bytes = need;
    return MSH_OK;
}

void DevBuf::release() {
    if (ptr) (void)hipFree(ptr);
    ptr = nullptr;
    bytes = 0;
}

void Workspace::release() {
    DevBuf* all[] = {&keys, &vals, &keys_alt, &vals_alt, &hist, &scan, &q, &out_a, &out_b, &out_c,
                     &flags, &counters, &spill, &stats, &ranges};
    for (DevBuf* b : all) b->release();
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

template <class T>
static int upload(DevBuf& buf, const T* host, size_t n, hipStream_t s) {
    MSH_TRY(buf.reserve(n * sizeof(T)));
    if (n) MSH_HIP(hipMemcpyAsync(buf.ptr, host, n * sizeof(T), hipMemcpyHostToDevice, s));
    return MSH_OK;
}

static void free_tree(msh_tree* t) {
    if (!t) return;
    (void)hipSetDevice(t->device);
    if (t->stream) (void)hipStreamSynchronize(t->stream);
    t->ws.release();
    if (t->d_v) (void)hipFree(t->d_v);
    if (t->d_nodes) (void)hipFree(t->d_nodes);
    if (t->d_orgs) (void)hipFree(t->d_orgs);
    if (t->d_boxes) (void)hipFree(t->d_boxes);
    if (t->d_leaves) (void)hipFree(t->d_leaves);
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
    hipError_t e = hipStreamCreateWithFlags(&t->stream, hipStreamNonBlocking);
    if (e != hipSuccess) {
        set_error("hipStreamCreate failed on device %d: %s", dev, hipGetErrorString(e));
        delete t;
        return MSH_EDEVICE;
    }
    *out = t;
    return MSH_OK;
}

// Triangle tree over v (P rows) and f (T rows, indices into v).
static int build_triangles(msh_tree* t, const double* v, size_t Pall, const uint32_t* f, size_t T) {
    hipStream_t s = t->stream;
    hipEvent_t e0, e1;
    MSH_HIP(hipEventCreate(&e0));
    MSH_HIP(hipEventCreate(&e1));
    MSH_HIP(hipMalloc(&t->d_v, std::max<size_t>(Pall, 1) * 3 * sizeof(double)));
    MSH_HIP(hipMemcpyAsync(t->d_v, v, Pall * 3 * sizeof(double), hipMemcpyHostToDevice, s));
    DevBuf dF, dLo, dHi, dOrder;
    int st = MSH_OK;
    do {
        if ((st = upload(dF, f, 3 * T, s)) != MSH_OK) break;
        if ((st = dLo.reserve(3 * T * sizeof(double))) != MSH_OK) break;
        if ((st = dHi.reserve(3 * T * sizeof(double))) != MSH_OK) break;
        if ((st = dOrder.reserve(T * sizeof(uint32_t))) != MSH_OK) break;
        if (T > 1) {
            hipError_t e = hipMalloc(&t->d_nodes, (T - 1) * sizeof(BNode));
            if (e != hipSuccess) { set_error("hipMalloc nodes: %s", hipGetErrorString(e)); st = MSH_ENOMEM; break; }
        }
        hipError_t e = hipMalloc(&t->d_leaves, T * sizeof(TriRec));
        if (e != hipSuccess) { set_error("hipMalloc leaves: %s", hipGetErrorString(e)); st = MSH_ENOMEM; break; }
        (void)hipEventRecord(e0, s);
        if ((st = tri_bounds(t->d_v, dF.as<uint32_t>(), T, dLo.as<double>(), dHi.as<double>(), s)) != MSH_OK) break;
        if ((st = build_lbvh(t, dLo.as<double>(), dHi.as<double>(), T, dOrder.as<uint32_t>())) != MSH_OK) break;
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
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    return st;
}

static const size_t kSortMin = 4096;  // below this the query Morton sort costs more than it saves

// Morton-sort S points (device) into ws.vals; returns the permutation (or nullptr for small S).
static int sort_queries(msh_tree* t, const double* d_q, size_t S, hipStream_t s, const uint32_t** perm) {
    *perm = nullptr;
    if (S < kSortMin) return MSH_OK;
    Workspace& ws = t->ws;
    MSH_TRY(ws.keys.reserve(S * sizeof(uint32_t)));
    MSH_TRY(ws.vals.reserve(S * sizeof(uint32_t)));
    MSH_TRY(ws.keys_alt.reserve(S * sizeof(uint32_t)));
    MSH_TRY(ws.vals_alt.reserve(S * sizeof(uint32_t)));
    MSH_TRY(query_morton(t, d_q, S, ws.keys.as<uint32_t>(), ws.vals.as<uint32_t>(), s));
    MSH_TRY(radix_sort_pairs(ws.keys.as<uint32_t>(), ws.vals.as<uint32_t>(), ws.keys_alt.as<uint32_t>(),
                             ws.vals_alt.as<uint32_t>(), S, 30, ws, s));
    *perm = ws.vals.as<uint32_t>();
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
    if (t->B != 1) {
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

}  // namespace msh

using namespace msh;

extern "C" {

const char* msh_last_error(void) { return g_err.c_str(); }

int msh_version(void) { return 1; }

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

int msh_set_device(int device) {
    int c = 0;
    MSH_TRY(msh_device_count(&c));
    if (device < 0 || device >= c) {
        set_error("device %d out of range (%d devices)", device, c);
        return MSH_EINVAL;
    }
    g_device = device;
    return use_device(device);
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
    (*out)->kind = kNormals;
    (*out)->eps = eps;
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
        hipError_t e = hipMalloc(&t->d_v, P * 3 * sizeof(double));
        if (e != hipSuccess) { set_error("hipMalloc: %s", hipGetErrorString(e)); st = MSH_ENOMEM; break; }
        e = hipMemcpyAsync(t->d_v, v, P * 3 * sizeof(double), hipMemcpyHostToDevice, s);
        if (e != hipSuccess) { set_error("H2D: %s", hipGetErrorString(e)); st = MSH_EDEVICE; break; }
        if ((st = dLo.reserve(3 * P * sizeof(double))) != MSH_OK) break;
        if ((st = dHi.reserve(3 * P * sizeof(double))) != MSH_OK) break;
        if ((st = dOrder.reserve(P * sizeof(uint32_t))) != MSH_OK) break;
        if (P > 1) {
            e = hipMalloc(&t->d_nodes, (P - 1) * sizeof(BNode));
            if (e != hipSuccess) { set_error("hipMalloc nodes: %s", hipGetErrorString(e)); st = MSH_ENOMEM; break; }
        }
        e = hipMalloc(&t->d_leaves, P * sizeof(PtRec));
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

int msh_tree_get_info(const msh_tree* t, msh_tree_info* info) {
    if (!t || !info) { set_error("null argument"); return MSH_EINVAL; }
    info->device = t->device;
    info->kind = t->kind;
    info->n_points = t->P;
    info->n_faces = t->T;
    info->n_main_faces = t->T_main;
    info->n_nodes = t->T > 0 ? t->B * (t->T - 1) : 0;
    info->n_meshes = t->B;
    const size_t leaf = t->kind == kPoints ? sizeof(PtRec) : sizeof(TriRec);
    const size_t vrows = t->kind == kPoints ? t->P : t->P;  // main vertices (extra mesh rows follow)
    (void)vrows;
    info->bytes = info->n_nodes * sizeof(BNode) + t->B * t->T * leaf;
    info->eps = t->eps;
    for (int k = 0; k < 3; ++k) {
        info->scene_lo[k] = t->scene_lo[k];
        info->scene_hi[k] = t->scene_hi[k];
    }
    info->build_ms = t->build_ms;
    return MSH_OK;
}

// ---------------------------------------------------------------------------------------------
int msh_tree_nearest_device(msh_tree* t, const double* d_q, size_t S, uint32_t* d_face, uint32_t* d_part, double* d_pt,
                            void* stream) {
    MSH_TRY(check_tree(t, kTriangles, "msh_tree_nearest_device"));
    if (S == 0) return MSH_OK;
    hipStream_t s = stream ? static_cast<hipStream_t>(stream) : t->stream;
    const uint32_t* perm = nullptr;
    MSH_TRY(sort_queries(t, d_q, S, s, &perm));
    return launch_nearest(t, d_q, perm, S, d_face, d_part, d_pt, s);
}

int msh_tree_nearest(msh_tree* t, const double* q, size_t S, uint32_t* face, uint32_t* part, double* pt) {
    MSH_TRY(check_tree(t, kTriangles, "msh_tree_nearest"));
    if (S == 0) return MSH_OK;
    hipStream_t s = t->stream;
    Workspace& ws = t->ws;
    MSH_TRY(upload(ws.q, q, 3 * S, s));
    MSH_TRY(ws.out_a.reserve(S * sizeof(uint32_t)));
    MSH_TRY(ws.out_b.reserve(S * sizeof(uint32_t)));
    MSH_TRY(ws.out_c.reserve(3 * S * sizeof(double)));
    MSH_TRY(msh_tree_nearest_device(t, ws.q.as<double>(), S, ws.out_a.as<uint32_t>(),
                                    part ? ws.out_b.as<uint32_t>() : nullptr, ws.out_c.as<double>(), s));
    MSH_HIP(hipMemcpyAsync(face, ws.out_a.ptr, S * sizeof(uint32_t), hipMemcpyDeviceToHost, s));
    if (part) MSH_HIP(hipMemcpyAsync(part, ws.out_b.ptr, S * sizeof(uint32_t), hipMemcpyDeviceToHost, s));
    MSH_HIP(hipMemcpyAsync(pt, ws.out_c.ptr, 3 * S * sizeof(double), hipMemcpyDeviceToHost, s));
    MSH_HIP(hipStreamSynchronize(s));
    return MSH_OK;
}

int msh_tree_nearest_stats(msh_tree* t, const double* d_q, size_t S, uint64_t* nodes, uint64_t* leaves) {
    MSH_TRY(check_tree(t, kTriangles, "msh_tree_nearest_stats"));
    *nodes = 0;
    *leaves = 0;
    if (S == 0) return MSH_OK;
    hipStream_t s = t->stream;
    const uint32_t* perm = nullptr;
    MSH_TRY(sort_queries(t, d_q, S, s, &perm));
    MSH_TRY(t->ws.stats.reserve(8 * sizeof(unsigned long long)));
    MSH_HIP(hipMemsetAsync(t->ws.stats.ptr, 0, 8 * sizeof(unsigned long long), s));
    MSH_TRY(launch_nearest_stats(t, d_q, perm, S, t->ws.stats.as<unsigned long long>(), s));
    unsigned long long h[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    MSH_HIP(hipMemcpyAsync(h, t->ws.stats.ptr, sizeof(h), hipMemcpyDeviceToHost, s));
    MSH_HIP(hipStreamSynchronize(s));
    *nodes = h[0];
    *leaves = h[1];
    if (getenv("MESH_AMD_STATS_DUMP"))  // development: wave-iteration utilisation of pass 1
        fprintf(stderr, "[msh stats] S=%zu nodes=%llu leaves=%llu trav_it=%llu trav_lanes=%llu leaf_it=%llu "
                        "leaf_lanes=%llu exact=%llu\n", S, h[0], h[1], h[2], h[3], h[4], h[5], h[6]);
    return MSH_OK;
}

int msh_tree_nearest_alongnormal(msh_tree* t, const double* p, const double* n, size_t S, double* dist, uint32_t* face,
                                 double* pt) {
    MSH_TRY(check_tree(t, kTriangles, "msh_tree_nearest_alongnormal"));
    if (S == 0) return MSH_OK;
    hipStream_t s = t->stream;
    Workspace& ws = t->ws;
    DevBuf dn, dd;
    int st = MSH_OK;
    do {
        if ((st = upload(ws.q, p, 3 * S, s)) != MSH_OK) break;
        if ((st = upload(dn, n, 3 * S, s)) != MSH_OK) break;
        if ((st = dd.reserve(S * sizeof(double))) != MSH_OK) break;
        if ((st = ws.out_a.reserve(S * sizeof(uint32_t))) != MSH_OK) break;
        if ((st = ws.out_c.reserve(3 * S * sizeof(double))) != MSH_OK) break;
        const uint32_t* perm = nullptr;
        if ((st = sort_queries(t, ws.q.as<double>(), S, s, &perm)) != MSH_OK) break;
        if ((st = launch_alongnormal(t, ws.q.as<double>(), dn.as<double>(), perm, S, dd.as<double>(),
                                     ws.out_a.as<uint32_t>(), ws.out_c.as<double>(), s)) != MSH_OK)
            break;
        hipError_t e;
        if ((e = hipMemcpyAsync(dist, dd.ptr, S * sizeof(double), hipMemcpyDeviceToHost, s)) != hipSuccess ||
            (e = hipMemcpyAsync(face, ws.out_a.ptr, S * sizeof(uint32_t), hipMemcpyDeviceToHost, s)) != hipSuccess ||
            (e = hipMemcpyAsync(pt, ws.out_c.ptr, 3 * S * sizeof(double), hipMemcpyDeviceToHost, s)) != hipSuccess ||
            (e = hipStreamSynchronize(s)) != hipSuccess) {
            set_error("alongnormal: %s", hipGetErrorString(e));
            st = MSH_EDEVICE;
        }
    } while (0);
    (void)hipStreamSynchronize(s);
    dn.release();
    dd.release();
    return st;
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
    MSH_TRY(check_faces(qf, Tq, Pq, "query faces"));
    hipStream_t s = t->stream;
    std::vector<TriRec> ht;
    host_tris(qv, qf, Tq, ht);
    DevBuf dq, df;
    int st = MSH_OK;
    std::vector<uint32_t> flags(Tq);
    do {
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
    if (S == 0) return MSH_OK;
    hipStream_t s = t->stream;
    Workspace& ws = t->ws;
    DevBuf dn;
    int st = MSH_OK;
    do {
        if ((st = upload(ws.q, q, 3 * S, s)) != MSH_OK) break;
        if ((st = upload(dn, n, 3 * S, s)) != MSH_OK) break;
        if ((st = ws.out_a.reserve(S * sizeof(uint32_t))) != MSH_OK) break;
        if ((st = ws.out_c.reserve(3 * S * sizeof(double))) != MSH_OK) break;
        const uint32_t* perm = nullptr;
        if ((st = sort_queries(t, ws.q.as<double>(), S, s, &perm)) != MSH_OK) break;
        if ((st = launch_nnearest(t, ws.q.as<double>(), dn.as<double>(), perm, S, ws.out_a.as<uint32_t>(),
                                  ws.out_c.as<double>(), s)) != MSH_OK)
            break;
        hipError_t e;
        if ((e = hipMemcpyAsync(face, ws.out_a.ptr, S * sizeof(uint32_t), hipMemcpyDeviceToHost, s)) != hipSuccess ||
            (e = hipMemcpyAsync(pt, ws.out_c.ptr, 3 * S * sizeof(double), hipMemcpyDeviceToHost, s)) != hipSuccess ||
            (e = hipStreamSynchronize(s)) != hipSuccess) {
            set_error("normals nearest: %s", hipGetErrorString(e));
            st = MSH_EDEVICE;
        }
    } while (0);
    (void)hipStreamSynchronize(s);
    dn.release();
    return st;
}

int msh_ntree_selfintersects(msh_tree* t, int64_t* count) {
    MSH_TRY(check_tree(t, kNormals, "msh_ntree_selfintersects"));
    *count = 0;
    hipStream_t s = t->stream;
    DevBuf df;
    std::vector<uint32_t> flags(t->T);
    int st = MSH_OK;
    do {
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

int msh_visibility(msh_tree* t, const double* cams, size_t C, const double* normals, const double* sensors,
                   double min_dist, uint32_t* vis, double* ndc) {
    MSH_TRY(check_tree(t, kTriangles, "msh_visibility"));
    const size_t n = C * t->P;
    if (n == 0) return MSH_OK;
    hipStream_t s = t->stream;
    DevBuf dc, dn, ds, dv, dd;
    int st = MSH_OK;
    do {
        if ((st = upload(dc, cams, 3 * C, s)) != MSH_OK) break;
        if (normals && (st = upload(dn, normals, 3 * t->P, s)) != MSH_OK) break;
        if (sensors && (st = upload(ds, sensors, 9 * C, s)) != MSH_OK) break;
        if ((st = dv.reserve(n * sizeof(uint32_t))) != MSH_OK) break;
        if ((st = dd.reserve(n * sizeof(double))) != MSH_OK) break;
        if ((st = launch_visibility(t, dc.as<double>(), C, normals ? dn.as<double>() : nullptr,
                                    sensors ? ds.as<double>() : nullptr, min_dist, dv.as<uint32_t>(), dd.as<double>(),
                                    s)) != MSH_OK)
            break;
        hipError_t e;
        if ((e = hipMemcpyAsync(vis, dv.ptr, n * sizeof(uint32_t), hipMemcpyDeviceToHost, s)) != hipSuccess ||
            (e = hipMemcpyAsync(ndc, dd.ptr, n * sizeof(double), hipMemcpyDeviceToHost, s)) != hipSuccess ||
            (e = hipStreamSynchronize(s)) != hipSuccess) {
            set_error("visibility: %s", hipGetErrorString(e));
            st = MSH_EDEVICE;
        }
    } while (0);
    (void)hipStreamSynchronize(s);
    dc.release(); dn.release(); ds.release(); dv.release(); dd.release();
    return st;
}

int msh_points_nearest(msh_tree* t, const double* q, size_t S, uint32_t* idx, double* dist) {
    MSH_TRY(check_tree(t, kPoints, "msh_points_nearest"));
    if (S == 0) return MSH_OK;
    hipStream_t s = t->stream;
    Workspace& ws = t->ws;
    MSH_TRY(upload(ws.q, q, 3 * S, s));
    MSH_TRY(ws.out_a.reserve(S * sizeof(uint32_t)));
    MSH_TRY(ws.out_c.reserve(S * sizeof(double)));
    const uint32_t* perm = nullptr;
    MSH_TRY(sort_queries(t, ws.q.as<double>(), S, s, &perm));
    MSH_TRY(launch_points_nearest(t, ws.q.as<double>(), perm, S, ws.out_a.as<uint32_t>(), ws.out_c.as<double>(), s));
    MSH_HIP(hipMemcpyAsync(idx, ws.out_a.ptr, S * sizeof(uint32_t), hipMemcpyDeviceToHost, s));
    MSH_HIP(hipMemcpyAsync(dist, ws.out_c.ptr, S * sizeof(double), hipMemcpyDeviceToHost, s));
    MSH_HIP(hipStreamSynchronize(s));
    return MSH_OK;
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
};
static const uint64_t kBlobMagic = 0x4d53484c42564832ull;  // "MSHLBVH2"

static size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

static void blob_layout(const msh_tree* t, BlobHeader& h) {
    std::memset(&h, 0, sizeof(h));
    h.magic = kBlobMagic;
    h.kind = t->kind;
    h.max_depth = t->max_depth;
    h.P = t->P;
    h.T = t->T;
    h.T_main = t->T_main;
    // visibility trees keep the extra-mesh vertices after the main rows; only the main rows are needed
    h.v_rows = t->P;
    h.eps = t->eps;
    for (int k = 0; k < 3; ++k) {
        h.scene_lo[k] = t->scene_lo[k];
        h.scene_hi[k] = t->scene_hi[k];
        h.origin[k] = t->origin[k];
    }
    const size_t leaf = t->kind == kPoints ? sizeof(PtRec) : sizeof(TriRec);
    h.off_v = align256(sizeof(BlobHeader));
    h.off_nodes = align256(h.off_v + h.v_rows * 3 * sizeof(double));
    h.off_leaves = align256(h.off_nodes + (t->T > 1 ? (t->T - 1) * sizeof(BNode) : 0));
    h.total = align256(h.off_leaves + t->T * leaf);
}

int msh_tree_blob_size(const msh_tree* t, size_t* bytes) {
    if (!t || !bytes) { set_error("null argument"); return MSH_EINVAL; }
    if (t->B != 1) { set_error("msh_tree_blob_size: batched trees are not serialisable"); return MSH_EINVAL; }
    BlobHeader h;
    blob_layout(t, h);
    *bytes = h.total;
    return MSH_OK;
}

int msh_tree_blob_pack(const msh_tree* t, void* d_dst, void* stream) {
    if (!t || !d_dst) { set_error("null argument"); return MSH_EINVAL; }
    if (t->B != 1) { set_error("msh_tree_blob_pack: batched trees are not serialisable"); return MSH_EINVAL; }
    MSH_TRY(use_device(t->device));
    hipStream_t s = stream ? static_cast<hipStream_t>(stream) : t->stream;
    BlobHeader h;
    blob_layout(t, h);
    char* dst = static_cast<char*>(d_dst);
    MSH_HIP(hipMemcpyAsync(dst, &h, sizeof(h), hipMemcpyHostToDevice, s));
    if (h.v_rows) MSH_HIP(hipMemcpyAsync(dst + h.off_v, t->d_v, h.v_rows * 3 * sizeof(double), hipMemcpyDeviceToDevice, s));
    if (t->T > 1)
        MSH_HIP(hipMemcpyAsync(dst + h.off_nodes, t->d_nodes, (t->T - 1) * sizeof(BNode), hipMemcpyDeviceToDevice, s));
    const size_t leaf = t->kind == kPoints ? sizeof(PtRec) : sizeof(TriRec);
    MSH_HIP(hipMemcpyAsync(dst + h.off_leaves, t->d_leaves, t->T * leaf, hipMemcpyDeviceToDevice, s));
    MSH_HIP(hipStreamSynchronize(s));
    return MSH_OK;
}

int msh_tree_blob_unpack(const void* d_src, size_t bytes, int device, void* stream, msh_tree** out) {
    if (!d_src || !out) { set_error("null argument"); return MSH_EINVAL; }
    *out = nullptr;
    MSH_TRY(use_device(device));
    BlobHeader h;
    hipStream_t us = static_cast<hipStream_t>(stream);
    MSH_HIP(hipMemcpyAsync(&h, d_src, sizeof(h), hipMemcpyDeviceToHost, us));
    MSH_HIP(hipStreamSynchronize(us));
    if (h.magic != kBlobMagic || h.total > bytes) {
        set_error("not a meshsearch tree blob (magic %llx, %zu bytes)", (unsigned long long)h.magic, bytes);
        return MSH_EINVAL;
    }
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
    const char* src = static_cast<const char*>(d_src);
    const size_t leaf = h.kind == kPoints ? sizeof(PtRec) : sizeof(TriRec);
    hipStream_t s = us ? us : t->stream;
    do {
        hipError_t e = hipMalloc(&t->d_v, std::max<uint64_t>(h.v_rows, 1) * 3 * sizeof(double));
        if (e == hipSuccess && h.v_rows)
            e = hipMemcpyAsync(t->d_v, src + h.off_v, h.v_rows * 3 * sizeof(double), hipMemcpyDeviceToDevice, s);
        if (e == hipSuccess && h.T > 1) e = hipMalloc(&t->d_nodes, (h.T - 1) * sizeof(BNode));
        if (e == hipSuccess && h.T > 1)
            e = hipMemcpyAsync(t->d_nodes, src + h.off_nodes, (h.T - 1) * sizeof(BNode), hipMemcpyDeviceToDevice, s);
        if (e == hipSuccess) e = hipMalloc(&t->d_leaves, h.T * leaf);
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
        }
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
        if (e == hipSuccess) e = hipMalloc(&t->d_v, B * P * 3 * sizeof(double));
        if (e == hipSuccess) e = hipMalloc(&t->d_nodes, B * (T - 1) * sizeof(BNode));
        if (e == hipSuccess) e = hipMalloc(&t->d_leaves, B * T * sizeof(TriRec));
        if (e != hipSuccess) { set_error("msh_batch_build: %s", hipGetErrorString(e)); st = MSH_ENOMEM; break; }
        e = hipMemcpyAsync(t->d_v, v, B * P * 3 * sizeof(double), hipMemcpyHostToDevice, s);
        if (e != hipSuccess) { set_error("msh_batch_build: %s", hipGetErrorString(e)); st = MSH_EDEVICE; break; }
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
        if ((st = build_obb(t, true)) != MSH_OK) break;
        (void)hipEventRecord(e1, s);
        e = hipStreamSynchronize(s);
        if (e != hipSuccess) { set_error("batched LBVH build failed: %s", hipGetErrorString(e)); st = MSH_EDEVICE; break; }
        float ms = 0.f;
        (void)hipEventElapsedTime(&ms, e0, e1);
        t->build_ms = ms;
    } while (0);
    (void)hipStreamSynchronize(s);
    dF.release(); dLo.release(); dHi.release(); dOrder.release();
    t->ws.release();
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

int msh_batch_nearest_device(msh_tree* t, const double* d_q, size_t S, uint32_t* d_face, uint32_t* d_part, double* d_pt,
                             void* stream) {
    MSH_TRY(check_batch(t, "msh_batch_nearest_device"));
    const size_t n = t->B * S;
    if (n == 0) return MSH_OK;
    if (n > (size_t)0xFFFFFFFFu) { set_error("msh_batch_nearest: %zu queries exceed 2^32", n); return MSH_EINVAL; }
    hipStream_t s = stream ? static_cast<hipStream_t>(stream) : t->stream;
    Workspace& ws = t->ws;
    const uint32_t* perm = nullptr;
    if (n >= kSortMin) {  // Morton order inside each mesh, meshes in order (two stable passes)
        MSH_TRY(ws.keys.reserve(n * sizeof(uint32_t)));
        MSH_TRY(ws.vals.reserve(n * sizeof(uint32_t)));
        MSH_TRY(ws.keys_alt.reserve(n * sizeof(uint32_t)));
        MSH_TRY(ws.vals_alt.reserve(n * sizeof(uint32_t)));
        uint32_t* keys = ws.keys.as<uint32_t>();
        uint32_t* vals = ws.vals.as<uint32_t>();
        MSH_TRY(query_morton_batch(t, d_q, n, S, keys, vals, s));
        MSH_TRY(radix_sort_pairs(keys, vals, ws.keys_alt.as<uint32_t>(), ws.vals_alt.as<uint32_t>(), n, 30, ws, s));
        if (t->B > 1) {
            MSH_TRY(mesh_keys(vals, n, S, keys, s));
            int bits = 0;
            while (bits < 32 && ((size_t)1 << bits) < t->B) ++bits;
            MSH_TRY(radix_sort_pairs(keys, vals, ws.keys_alt.as<uint32_t>(), ws.vals_alt.as<uint32_t>(), n, bits, ws, s));
        }
        perm = vals;
    }
    return launch_nearest_batch(t, d_q, perm, n, S, d_face, d_part, d_pt, s);
}

int msh_batch_nearest(msh_tree* t, const double* q, size_t S, uint32_t* face, uint32_t* part, double* pt) {
    MSH_TRY(check_batch(t, "msh_batch_nearest"));
    const size_t n = t->B * S;
    if (n == 0) return MSH_OK;
    if (!q || !face || !pt) { set_error("msh_batch_nearest: null argument"); return MSH_EINVAL; }
    hipStream_t s = t->stream;
    Workspace& ws = t->ws;
    MSH_TRY(upload(ws.q, q, 3 * n, s));
    MSH_TRY(ws.out_a.reserve(n * sizeof(uint32_t)));
    MSH_TRY(ws.out_b.reserve(n * sizeof(uint32_t)));
    MSH_TRY(ws.out_c.reserve(3 * n * sizeof(double)));
    MSH_TRY(msh_batch_nearest_device(t, ws.q.as<double>(), S, ws.out_a.as<uint32_t>(),
                                     part ? ws.out_b.as<uint32_t>() : nullptr, ws.out_c.as<double>(), s));
    MSH_HIP(hipMemcpyAsync(face, ws.out_a.ptr, n * sizeof(uint32_t), hipMemcpyDeviceToHost, s));
    if (part) MSH_HIP(hipMemcpyAsync(part, ws.out_b.ptr, n * sizeof(uint32_t), hipMemcpyDeviceToHost, s));
    MSH_HIP(hipMemcpyAsync(pt, ws.out_c.ptr, 3 * n * sizeof(double), hipMemcpyDeviceToHost, s));
    MSH_HIP(hipStreamSynchronize(s));
    return MSH_OK;
}

}  // extern "C"
