// K6 — triangle/triangle any-hit against the LBVH.
//   * aabbtree_intersections_indices (spatialsearchmodule.cpp:326-417; CGAL do_intersect(Triangle_3)):
//     one lane per query-mesh triangle, flag = 1 iff it touches any mesh triangle (closed test).
//   * aabbtree_n_selfintersects (aabb_normals.cpp:192-207, AABB_n_tree.h:107-116): one lane per mesh
//     triangle, pairs sharing an exactly equal vertex coordinate are skipped.
// The overlap test is the orientation-predicate test of Guigue & Devillers (2003) evaluated in fp64,
// with a 2-D edge/containment test for the coplanar case.  Boxes: closed fp64 separating-axis test of
// the triangle against each child's outward-rounded oriented box, on the node frame's three axes.
#include <algorithm>

#include "internal.h"

namespace msh {

__device__ inline bool seg_seg_2d(double ax, double ay, double bx, double by, double cx, double cy, double dx, double dy) {
    auto o2 = [](double px, double py, double qx, double qy, double rx, double ry) {
        return (qx - px) * (ry - py) - (qy - py) * (rx - px);
    };
    const double o1 = o2(ax, ay, bx, by, cx, cy), o2v = o2(ax, ay, bx, by, dx, dy);
    const double o3 = o2(cx, cy, dx, dy, ax, ay), o4 = o2(cx, cy, dx, dy, bx, by);
    if (((o1 > 0 && o2v < 0) || (o1 < 0 && o2v > 0)) && ((o3 > 0 && o4 < 0) || (o3 < 0 && o4 > 0))) return true;
    auto onseg = [](double px, double py, double qx, double qy, double rx, double ry) {
        return fmin(px, qx) <= rx && rx <= fmax(px, qx) && fmin(py, qy) <= ry && ry <= fmax(py, qy);
    };
    if (o1 == 0 && onseg(ax, ay, bx, by, cx, cy)) return true;
    if (o2v == 0 && onseg(ax, ay, bx, by, dx, dy)) return true;
    if (o3 == 0 && onseg(cx, cy, dx, dy, ax, ay)) return true;
    if (o4 == 0 && onseg(cx, cy, dx, dy, bx, by)) return true;
    return false;
}

__device__ inline bool pt_in_tri_2d(double px, double py, const double* t) {
    auto o2 = [](double ax, double ay, double bx, double by, double cx, double cy) {
        return (bx - ax) * (cy - ay) - (by - ay) * (cx - ax);
    };
    const double d0 = o2(t[0], t[1], t[2], t[3], px, py);
    const double d1 = o2(t[2], t[3], t[4], t[5], px, py);
    const double d2 = o2(t[4], t[5], t[0], t[1], px, py);
    return (d0 >= 0 && d1 >= 0 && d2 >= 0) || (d0 <= 0 && d1 <= 0 && d2 <= 0);
}

__device__ bool coplanar_tri_tri(const D3& p1, const D3& q1, const D3& r1, const D3& p2, const D3& q2, const D3& r2,
                                 const D3& n) {
    const double ax = fabs(n.x), ay = fabs(n.y), az = fabs(n.z);
    const int drop = (ax > az && ax >= ay) ? 0 : ((ay > az && ay > ax) ? 1 : 2);
    auto pr = [drop](const D3& p, double* o) {
        if (drop == 0) { o[0] = p.y; o[1] = p.z; }
        else if (drop == 1) { o[0] = p.x; o[1] = p.z; }
        else { o[0] = p.x; o[1] = p.y; }
    };
    double t1[6], t2[6];
    pr(p1, t1); pr(q1, t1 + 2); pr(r1, t1 + 4);
    pr(p2, t2); pr(q2, t2 + 2); pr(r2, t2 + 4);
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j)
            if (seg_seg_2d(t1[2 * i], t1[2 * i + 1], t1[(2 * i + 2) % 6], t1[(2 * i + 3) % 6], t2[2 * j], t2[2 * j + 1],
                           t2[(2 * j + 2) % 6], t2[(2 * j + 3) % 6]))
                return true;
    if (pt_in_tri_2d(t1[0], t1[1], t2)) return true;
    if (pt_in_tri_2d(t2[0], t2[1], t1)) return true;
    return false;
}

__device__ inline bool check_min_max(const D3& p1, const D3& q1, const D3& r1, const D3& p2, const D3& q2, const D3& r2) {
    D3 n = vcross(vsub(p2, q1), vsub(p1, q1));
    if (vdot(vsub(q2, q1), n) > 0.0) return false;
    n = vcross(vsub(p2, p1), vsub(r1, p1));
    if (vdot(vsub(r2, p1), n) > 0.0) return false;
    return true;
}

__device__ bool tri_tri_3d(const D3& p1, const D3& q1, const D3& r1, const D3& p2, const D3& q2, const D3& r2, double dp2,
                           double dq2, double dr2, const D3& n1) {
    if (dp2 > 0.0) {
        if (dq2 > 0.0) return check_min_max(p1, r1, q1, r2, p2, q2);
        if (dr2 > 0.0) return check_min_max(p1, r1, q1, q2, r2, p2);
        return check_min_max(p1, q1, r1, p2, q2, r2);
    }
    if (dp2 < 0.0) {
        if (dq2 < 0.0) return check_min_max(p1, q1, r1, r2, p2, q2);
        if (dr2 < 0.0) return check_min_max(p1, q1, r1, q2, r2, p2);
        return check_min_max(p1, r1, q1, p2, q2, r2);
    }
    if (dq2 < 0.0) {
        if (dr2 >= 0.0) return check_min_max(p1, r1, q1, q2, r2, p2);
        return check_min_max(p1, q1, r1, p2, q2, r2);
    }
    if (dq2 > 0.0) {
        if (dr2 > 0.0) return check_min_max(p1, r1, q1, p2, q2, r2);
        return check_min_max(p1, q1, r1, q2, r2, p2);
    }
    if (dr2 > 0.0) return check_min_max(p1, q1, r1, r2, p2, q2);
    if (dr2 < 0.0) return check_min_max(p1, r1, q1, r2, p2, q2);
    return coplanar_tri_tri(p1, q1, r1, p2, q2, r2, n1);
}

__device__ bool tri_tri_overlap(const D3& p1, const D3& q1, const D3& r1, const D3& p2, const D3& q2, const D3& r2) {
    const D3 n2 = vcross(vsub(p2, r2), vsub(q2, r2));
    const double dp1 = vdot(vsub(p1, r2), n2), dq1 = vdot(vsub(q1, r2), n2), dr1 = vdot(vsub(r1, r2), n2);
    if (dp1 * dq1 > 0.0 && dp1 * dr1 > 0.0) return false;
    const D3 n1 = vcross(vsub(q1, p1), vsub(r1, p1));
    const double dp2 = vdot(vsub(p2, r1), n1), dq2 = vdot(vsub(q2, r1), n1), dr2 = vdot(vsub(r2, r1), n1);
    if (dp2 * dq2 > 0.0 && dp2 * dr2 > 0.0) return false;
    if (dp1 > 0.0) {
        if (dq1 > 0.0) return tri_tri_3d(r1, p1, q1, p2, r2, q2, dp2, dr2, dq2, n1);
        if (dr1 > 0.0) return tri_tri_3d(q1, r1, p1, p2, r2, q2, dp2, dr2, dq2, n1);
        return tri_tri_3d(p1, q1, r1, p2, q2, r2, dp2, dq2, dr2, n1);
    }
    if (dp1 < 0.0) {
        if (dq1 < 0.0) return tri_tri_3d(r1, p1, q1, p2, q2, r2, dp2, dq2, dr2, n1);
        if (dr1 < 0.0) return tri_tri_3d(q1, r1, p1, p2, q2, r2, dp2, dq2, dr2, n1);
        return tri_tri_3d(p1, q1, r1, p2, r2, q2, dp2, dr2, dq2, n1);
    }
    if (dq1 < 0.0) {
        if (dr1 >= 0.0) return tri_tri_3d(q1, r1, p1, p2, r2, q2, dp2, dr2, dq2, n1);
        return tri_tri_3d(p1, q1, r1, p2, q2, r2, dp2, dq2, dr2, n1);
    }
    if (dq1 > 0.0) {
        if (dr1 > 0.0) return tri_tri_3d(p1, q1, r1, p2, r2, q2, dp2, dr2, dq2, n1);
        return tri_tri_3d(q1, r1, p1, p2, q2, r2, dp2, dq2, dr2, n1);
    }
    if (dr1 > 0.0) return tri_tri_3d(r1, p1, q1, p2, q2, r2, dp2, dq2, dr2, n1);
    if (dr1 < 0.0) return tri_tri_3d(r1, p1, q1, p2, r2, q2, dp2, dr2, dq2, n1);
    return coplanar_tri_tri(p1, q1, r1, p2, q2, r2, n1);
}

// Interval of the query triangle (vertices relative to the tree origin) along each frame axis, widened
// by a 2^-40 relative margin for the fp64 projections.
struct TriProj {
    double lo[3], hi[3];
};
__device__ inline TriProj tri_proj(const FrameD& f, const D3& a, const D3& b, const D3& c) {
    TriProj r;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const double pa = vdot(f.a[k], a), pb = vdot(f.a[k], b), pc = vdot(f.a[k], c);
        const double lo = fmin(fmin(pa, pb), pc), hi = fmax(fmax(pa, pb), pc);
        const double m = 9.094947017729282e-13 * (fabs(lo) + fabs(hi)) + 1e-300;
        r.lo[k] = lo - m;
        r.hi[k] = hi + m;
    }
    return r;
}
// separating-axis test on the node frame's three axes: false only if the triangle and the child's oriented
// box are disjoint along one of them
__device__ inline bool obb_overlap(const TriProj& p, const float* ext) {
    return p.lo[0] <= (double)ext[3] && (double)ext[0] <= p.hi[0] && p.lo[1] <= (double)ext[4] &&
           (double)ext[1] <= p.hi[1] && p.lo[2] <= (double)ext[5] && (double)ext[2] <= p.hi[2];
}

struct TriArgs {
    const BNode* nodes;
    const TriRec* tris;
    size_t T;
    const TriRec* q;
    size_t Tq;
    int self_mode;
    uint32_t* flags;
    uint2* spill;
    int spill_depth;
    double org[3];  // tree origin
};

__global__ __launch_bounds__(kBlock) void k_tritri(TriArgs a) {
    __shared__ uint2 stk[kStack * kBlock];
    const int tid = threadIdx.x;
    uint2* lds = stk + tid;
    for (size_t i = (size_t)blockIdx.x * kBlock + tid; i < a.Tq; i += (size_t)gridDim.x * kBlock) {
        uint2* spill = a.spill ? a.spill + (size_t)blockIdx.x * kBlock * (size_t)a.spill_depth + tid : nullptr;
        D3 qa, qb, qc;
        uint32_t qface;
        load_tri(a.q, (int)i, qa, qb, qc, qface);
        // query vertices relative to the tree origin (node bounds are origin-relative and padded >= 1 fp32
        // ulp, far above the fp64 rounding of this subtraction)
        const D3 org = D3{a.org[0], a.org[1], a.org[2]};
        const D3 ra = vsub(qa, org), rb = vsub(qb, org), rc = vsub(qc, org);
        bool hit = false;
        auto leaf_test = [&](int leaf) {
            D3 a0, a1, a2;
            uint32_t f;
            load_tri(a.tris, leaf, a0, a1, a2, f);
            if (a.self_mode) {
                if (veq(qa, a0) || veq(qa, a1) || veq(qa, a2) || veq(qb, a0) || veq(qb, a1) || veq(qb, a2) ||
                    veq(qc, a0) || veq(qc, a1) || veq(qc, a2))
                    return;
            }
            if (tri_tri_overlap(qa, qb, qc, a0, a1, a2)) hit = true;
        };
        if (a.T == 1) {
            leaf_test(0);
        } else {
            int node = 0, sp = 0;
            for (size_t guard = 0; guard < a.T; ++guard) {
                const NodeV nd = load_node(a.nodes, node);
                float e0[6], e1[6];
                nd.extents(e0, e1);
                const TriProj tp = tri_proj(frame_d(nd), ra, rb, rc);
                bool h0 = obb_overlap(tp, e0);
                bool h1 = obb_overlap(tp, e1);
                const int c0 = nd.child(0), c1 = nd.child(1);
                if (h0 && c0 < 0) { leaf_test(~c0); h0 = false; if (hit) break; }
                if (h1 && c1 < 0) { leaf_test(~c1); h1 = false; if (hit) break; }
                if (h0 && h1) {
                    const uint2 e = make_uint2((unsigned)c1, 0u);
                    stack_put(lds, spill, sp, e);
                    ++sp;
                    node = c0;
                    continue;
                }
                if (h0) { node = c0; continue; }
                if (h1) { node = c1; continue; }
                if (sp == 0) break;
                --sp;
                node = (int)stack_get(lds, spill, sp).x;
            }
        }
        a.flags[i] = hit ? 1u : 0u;
    }
}

int launch_tri_intersect(const msh_tree* tree, const TriRec* d_qtris, size_t Tq, int self_mode, uint32_t* d_flags,
                         hipStream_t s) {
    if (Tq == 0) return MSH_OK;
    TriArgs a{};
    a.nodes = tree->d_nodes;
    a.tris = static_cast<const TriRec*>(tree->d_leaves);
    a.T = tree->T;
    a.q = d_qtris;
    a.Tq = Tq;
    a.self_mode = self_mode;
    for (int k = 0; k < 3; ++k) a.org[k] = tree->origin[k];
    a.flags = d_flags;
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, tree->device) != hipSuccess || n <= 0) n = 256;
    const unsigned nblk = (unsigned)std::min<size_t>((Tq + kBlock - 1) / kBlock, (size_t)n * 5);
    msh_tree* t = const_cast<msh_tree*>(tree);
    if (tree->max_depth + 1 > kStack) {
        a.spill_depth = tree->max_depth + 1 - kStack + 1;
        MSH_TRY(t->ws.spill.reserve((size_t)nblk * kBlock * (size_t)a.spill_depth * sizeof(uint2)));
        a.spill = t->ws.spill.as<uint2>();
    }
    TimedLaunch tl("tritri", s);
    k_tritri<<<nblk, kBlock, 0, s>>>(a);
    MSH_HIP(hipGetLastError());
    return MSH_OK;
}

}  // namespace msh
