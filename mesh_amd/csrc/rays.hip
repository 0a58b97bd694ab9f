// K4 — nearest_alongnormal: nearest hit of the rays (p, n) and (p, -n)
//      (replaces spatialsearchmodule.cpp:222-323: two CGAL all_intersections lists per point, serial)
// K5 — visibility any-hit over (camera x vertex) rays
//      (replaces visibility.cpp:75-115 VisibilityTask: tree.do_intersect(Ray) per camera and vertex)
//
// Ray semantics (shared with the oracle restatement): a CGAL Ray_3(p, v) is stored as two points
// (p, p + v) and its predicates use (p + v) - p as direction; the ray is closed (t >= 0) and so are
// the triangles.  A ray hits a triangle iff its supporting line passes the three edges with consistent
// orientation (edge determinants flip sign exactly for the shared edge of two triangles, so a ray
// through a shared edge is never lost) and the plane crossing parameter is >= 0; a ray lying in the
// triangle's plane enters it at the clipped parameter.
//
// Execution shape: one lane per ray, persistent near-first traversal over the same 64-B nodes as K2;
// box tests are slab tests on the fp32 (outward-padded) boxes evaluated in fp64 with a relative margin.
#include <algorithm>

#include "internal.h"

namespace msh {

__device__ inline double det3(const D3& a, const D3& b, const D3& c) { return vdot(vcross(a, b), c); }

__device__ inline bool coplanar_ray_tri(const D3& p, const D3& d, const D3& a, const D3& b, const D3& c, double& tout) {
    const D3 n = vcross(vsub(b, a), vsub(c, a));
    if (n.x == 0.0 && n.y == 0.0 && n.z == 0.0) return false;
    double tlo = 0.0, thi = INFINITY;
    const D3 v[3] = {a, b, c};
#pragma unroll
    for (int e = 0; e < 3; ++e) {
        const D3& s = v[e];
        const D3& t = v[(e + 1) % 3];
        const D3 et = vsub(t, s);
        const double f0 = vdot(n, vcross(et, vsub(p, s)));
        const double f1 = vdot(n, vcross(et, d));
        if (f1 == 0.0) {
            if (f0 < 0.0) return false;
        } else {
            const double tt = -f0 / f1;
            if (f1 > 0.0) tlo = fmax(tlo, tt);
            else thi = fmin(thi, tt);
        }
    }
    if (tlo > thi) return false;
    tout = tlo;
    return true;
}

__device__ inline bool ray_tri(const D3& p, const D3& d, const D3& a, const D3& b, const D3& c, double& tout) {
    const D3 u = vsub(a, p), v = vsub(b, p), w = vsub(c, p);
    const double s0 = det3(u, v, d), s1 = det3(v, w, d), s2 = det3(w, u, d);
    const bool pos = s0 >= 0.0 && s1 >= 0.0 && s2 >= 0.0;
    const bool neg = s0 <= 0.0 && s1 <= 0.0 && s2 <= 0.0;
    if (!pos && !neg) return false;
    const D3 n = vcross(vsub(b, a), vsub(c, a));
    const double num = vdot(n, u);
    const double den = vdot(n, d);
    if (den == 0.0 || (s0 == 0.0 && s1 == 0.0 && s2 == 0.0)) {
        if (num != 0.0) return false;
        return coplanar_ray_tri(p, d, a, b, c, tout);
    }
    const double t = num / den;
    if (t < 0.0) return false;
    tout = t;
    return true;
}

__device__ inline D3 ray_dir(const D3& p, const D3& v) { return vsub(vadd(p, v), p); }

// Slab test of the line p + t d, t in [tlo, thi], against an fp32 box; tnear = entry parameter.
__device__ inline bool slab(const D3& p, const D3& d, float lx, float ly, float lz, float hx, float hy, float hz, double tlo,
                            double thi, double& tnear) {
    const double po[3] = {p.x, p.y, p.z}, dd[3] = {d.x, d.y, d.z};
    const double lo[3] = {(double)lx, (double)ly, (double)lz}, hi[3] = {(double)hx, (double)hy, (double)hz};
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        if (dd[k] == 0.0) {
            if (po[k] < lo[k] || po[k] > hi[k]) return false;
        } else {
            const double inv = 1.0 / dd[k];
            double t1 = (lo[k] - po[k]) * inv, t2 = (hi[k] - po[k]) * inv;
            if (t1 > t2) { const double x = t1; t1 = t2; t2 = x; }
            tlo = fmax(tlo, t1);
            thi = fmin(thi, t2);
        }
    }
    tnear = tlo;
    return tlo <= thi + 1e-12 * (fabs(tlo) + fabs(thi)) + 1e-300;
}

// ---- generic traversal: the policy decides box hits (and ordering key) and leaf tests ----
template <class Pol>
__device__ inline void traverse_rays(const BNode* __restrict__ nodes, size_t T, Pol& pol, uint2* __restrict__ lds,
                                     uint2* __restrict__ spill) {
    if (T == 1) {
        pol.test(0);
        return;
    }
    int node = 0, sp = 0;
    for (size_t guard = 0; guard < T; ++guard) {
        const NodeV nd = load_node(nodes, node);
        double k0, k1;
        float l0[3], u0[3], l1[3], u1[3];
        node_aabb(nd, 0, l0, u0);
        node_aabb(nd, 1, l1, u1);
        bool h0 = pol.box(l0[0], l0[1], l0[2], u0[0], u0[1], u0[2], k0);
        bool h1 = pol.box(l1[0], l1[1], l1[2], u1[0], u1[1], u1[2], k1);
        const int c0 = nd.child(0), c1 = nd.child(1);
        if (h0 && c0 < 0) {
            pol.test(~c0);
            h0 = false;
            if (pol.done()) return;
        }
        if (h1 && c1 < 0) {
            pol.test(~c1);
            h1 = false;
            if (pol.done()) return;
        }
        h0 = h0 && pol.keep(k0);
        h1 = h1 && pol.keep(k1);
        if (h0 && h1) {
            int nearc = c0, farc = c1;
            double kf = k1;
            if (k1 < k0) { nearc = c1; farc = c0; kf = k0; }
            const uint2 e = make_uint2((unsigned)farc, __float_as_uint(__double2float_rd(kf)));
            if (sp < kStack) lds[sp * kBlock] = e;
            else spill[sp - kStack] = e;
            ++sp;
            node = nearc;
            continue;
        }
        if (h0) { node = c0; continue; }
        if (h1) { node = c1; continue; }
        bool found = false;
        while (sp > 0) {
            --sp;
            const uint2 e = sp < kStack ? lds[sp * kBlock] : spill[sp - kStack];
            if (pol.keep((double)__uint_as_float(e.y))) {
                node = (int)e.x;
                found = true;
                break;
            }
        }
        if (!found) break;
    }
}

// nearest hit along +-n; key = squared point-box distance (a lower bound of any hit's distance^2)
struct AlongPol {
    const TriRec* __restrict__ tris;
    D3 p, dp, dm;
    D3 pr;  // p relative to the tree origin (node bounds are origin-relative)
    double best;  // distance
    uint32_t best_face;
    D3 best_pt;
    __device__ double lim2() const { return best == INFINITY ? INFINITY : best * best * kSlack; }
    __device__ bool box(float lx, float ly, float lz, float hx, float hy, float hz, double& key) const {
        key = box_d2(pr, lx, ly, lz, hx, hy, hz);
        if (key > lim2()) return false;
        double tn;
        return slab(pr, dp, lx, ly, lz, hx, hy, hz, -INFINITY, INFINITY, tn);
    }
    __device__ bool keep(double key) const { return key <= lim2(); }
    __device__ bool done() const { return false; }
    __device__ void test(int leaf) {
        D3 a, b, c;
        uint32_t face;
        load_tri(tris, leaf, a, b, c, face);
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            const D3& d = k == 0 ? dp : dm;
            double t;
            if (!ray_tri(p, d, a, b, c, t)) continue;
            const D3 hit = vadd(p, vscale(t, d));
            const double dist = sqrt(sqdist(hit, p));
            if (dist < best || (dist == best && face < best_face)) {
                best = dist;
                best_face = face;
                best_pt = hit;
            }
        }
    }
};

// any hit of the closed ray src + t d, t >= 0; key = entry parameter
struct AnyPol {
    const TriRec* __restrict__ tris;
    D3 src, d;
    D3 sr;  // src relative to the tree origin
    bool hit;
    __device__ bool box(float lx, float ly, float lz, float hx, float hy, float hz, double& key) const {
        return slab(sr, d, lx, ly, lz, hx, hy, hz, 0.0, INFINITY, key);
    }
    __device__ bool keep(double) const { return !hit; }
    __device__ bool done() const { return hit; }
    __device__ void test(int leaf) {
        D3 a, b, c;
        uint32_t face;
        load_tri(tris, leaf, a, b, c, face);
        double t;
        if (ray_tri(src, d, a, b, c, t)) hit = true;
    }
};

struct RayArgs {
    const BNode* nodes;
    const TriRec* tris;
    size_t T;
    // alongnormal
    const double* p;
    const double* n;
    const uint32_t* perm;
    size_t S;
    double* out_dist;
    uint32_t* out_face;
    double* out_pt;
    // visibility
    const double* v;
    size_t P;
    const double* cams;
    const double* normals;
    const double* sensors;
    double min_dist;
    uint32_t* vis;
    double* ndc;
    // common
    unsigned* counters;
    unsigned ntiles;
    uint2* spill;
    int spill_depth;
    double org[3];  // tree origin
};

__device__ inline unsigned dequeue_tile_r(unsigned* counters, unsigned ntiles, unsigned group) {
    for (unsigned k = 0; k < 8; ++k) {
        const unsigned g = (group + k) & 7u;
        const unsigned lo = (unsigned)(((unsigned long long)ntiles * g) >> 3);
        const unsigned hi = (unsigned)(((unsigned long long)ntiles * (g + 1)) >> 3);
        if (lo >= hi) continue;
        if (__hip_atomic_load(&counters[g * 32], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= hi - lo) continue;
        const unsigned t = atomicAdd(&counters[g * 32], 1u);
        if (lo + t < hi) return lo + t;
    }
    return ntiles;
}

template <int MODE>  // 0 alongnormal, 1 visibility
__global__ __launch_bounds__(kBlock) void k_rays(RayArgs a) {
    __shared__ uint2 stk[kStack * kBlock];
    const int tid = threadIdx.x, lane = tid & 63;
    uint2* lds = stk + tid;
    uint2* spill = a.spill ? a.spill + ((size_t)blockIdx.x * kBlock + tid) * (size_t)a.spill_depth : nullptr;
    const unsigned group = blockIdx.x & 7u;
    const size_t total = MODE == 0 ? a.S : a.S;  // S = number of rays
    for (;;) {
        unsigned tile = 0;
        if (lane == 0) tile = dequeue_tile_r(a.counters, a.ntiles, group);
        tile = __shfl(tile, 0);
        if (tile >= a.ntiles) break;
        const size_t i = (size_t)tile * 64 + lane;
        if (i >= total) continue;
        if (MODE == 0) {
            const size_t qi = a.perm ? (size_t)a.perm[i] : i;
            const D3 p = D3{a.p[3 * qi], a.p[3 * qi + 1], a.p[3 * qi + 2]};
            const D3 n = D3{a.n[3 * qi], a.n[3 * qi + 1], a.n[3 * qi + 2]};
            AlongPol pol{a.tris, p, ray_dir(p, n), ray_dir(p, D3{-n.x, -n.y, -n.z}),
                         D3{p.x - a.org[0], p.y - a.org[1], p.z - a.org[2]}, INFINITY, 0xFFFFFFFFu,
                         D3{NAN, NAN, NAN}};
            traverse_rays<AlongPol>(a.nodes, a.T, pol, lds, spill);
            a.out_dist[qi] = pol.best == INFINITY ? 1e100 : pol.best;
            a.out_face[qi] = pol.best_face;
            a.out_pt[3 * qi] = pol.best_pt.x;
            a.out_pt[3 * qi + 1] = pol.best_pt.y;
            a.out_pt[3 * qi + 2] = pol.best_pt.z;
        } else {
            const size_t ic = i / a.P, iv = i - ic * a.P;
            const D3 cam = D3{a.cams[3 * ic], a.cams[3 * ic + 1], a.cams[3 * ic + 2]};
            const D3 vv = D3{a.v[3 * iv], a.v[3 * iv + 1], a.v[3 * iv + 2]};
            D3 dir = vsub(cam, vv);
            const double len = sqrt(vdot(dir, dir));
            dir = D3{dir.x / len, dir.y / len, dir.z / len};
            const D3 src = vadd(vv, vscale(a.min_dist, dir));
            AnyPol pol{a.tris, src, ray_dir(src, dir), D3{src.x - a.org[0], src.y - a.org[1], src.z - a.org[2]}, false};
            traverse_rays<AnyPol>(a.nodes, a.T, pol, lds, spill);
            const uint32_t reach = pol.hit ? 0u : 1u;
            a.ndc[i] = a.normals ? vdot(D3{a.normals[3 * iv], a.normals[3 * iv + 1], a.normals[3 * iv + 2]}, dir) : 0.0;
            uint32_t out = reach;
            if (a.sensors) {
                const double* s = a.sensors + 9 * ic;
                const D3 xoff = D3{s[0], s[1], s[2]}, yoff = D3{s[3], s[4], s[5]}, zoff = D3{-s[6], -s[7], -s[8]};
                const double planeoff = vdot(zoff, vadd(cam, zoff));
                if (reach) {
                    const double t = -(vdot(zoff, vv) - planeoff) / vdot(zoff, dir);
                    const D3 pi = vsub(vadd(vv, vscale(t, dir)), vadd(cam, zoff));
                    out = (fabs(vdot(pi, xoff)) < vdot(xoff, xoff) && fabs(vdot(pi, yoff)) < vdot(yoff, yoff)) ? 1u : 0u;
                } else {
                    out = 0u;
                }
            }
            a.vis[i] = out;
        }
    }
}

static int device_cus_r(int dev) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
    return n;
}

template <int MODE>
static int launch_rays(msh_tree* tree, RayArgs a, size_t nrays, hipStream_t s, const char* timer) {
    if (nrays == 0) return MSH_OK;
    if (nrays > (size_t)0xFFFFFFFFull * 64) {
        set_error("too many rays (%zu)", nrays);
        return MSH_EINVAL;
    }
    a.S = nrays;
    for (int k = 0; k < 3; ++k) a.org[k] = tree->origin[k];
    a.ntiles = (unsigned)((nrays + 63) / 64);
    const unsigned nblk = std::min<unsigned>((a.ntiles + 3) / 4, (unsigned)device_cus_r(tree->device) * 5u);
    MSH_TRY(tree->ws.counters.reserve(8 * 32 * sizeof(unsigned)));
    a.counters = tree->ws.counters.as<unsigned>();
    MSH_HIP(hipMemsetAsync(a.counters, 0, 8 * 32 * sizeof(unsigned), s));
    a.spill = nullptr;
    a.spill_depth = 0;
    if (tree->max_depth + 1 > kStack) {
        a.spill_depth = tree->max_depth + 1 - kStack + 1;
        MSH_TRY(tree->ws.spill.reserve((size_t)nblk * kBlock * (size_t)a.spill_depth * sizeof(uint2)));
        a.spill = tree->ws.spill.as<uint2>();
    }
    TimedLaunch tl(timer, s);
    k_rays<MODE><<<nblk, kBlock, 0, s>>>(a);
    MSH_HIP(hipGetLastError());
    return MSH_OK;
}

int launch_alongnormal(const msh_tree* tree, const double* d_p, const double* d_n, const uint32_t* d_perm, size_t S,
                       double* d_dist, uint32_t* d_face, double* d_pt, hipStream_t s) {
    RayArgs a{};
    a.nodes = tree->d_nodes; a.tris = static_cast<const TriRec*>(tree->d_leaves); a.T = tree->T;
    a.p = d_p; a.n = d_n; a.perm = d_perm;
    a.out_dist = d_dist; a.out_face = d_face; a.out_pt = d_pt;
    return launch_rays<0>(const_cast<msh_tree*>(tree), a, S, s, "alongnormal");
}

int launch_visibility(const msh_tree* tree, const double* d_cams, size_t C, const double* d_normals,
                      const double* d_sensors, double min_dist, uint32_t* d_vis, double* d_ndc, hipStream_t s) {
    RayArgs a{};
    a.nodes = tree->d_nodes; a.tris = static_cast<const TriRec*>(tree->d_leaves); a.T = tree->T;
    a.v = tree->d_v; a.P = tree->P; a.cams = d_cams; a.normals = d_normals; a.sensors = d_sensors;
    a.min_dist = min_dist; a.vis = d_vis; a.ndc = d_ndc;
    if (tree->P == 0) return MSH_OK;
    return launch_rays<1>(const_cast<msh_tree*>(tree), a, C * tree->P, s, "visibility");
}

}  // namespace msh
