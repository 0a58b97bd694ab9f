// Shared device-side definitions for the MI355X (gfx950) point-to-mesh search engine.
//
// Data layout in HBM:
//   BNode  — one LBVH internal node, 64 B: the fp32 AABBs of BOTH children (outward-rounded, so
//            every fp64 primitive lies inside) + both child references.  A traversal step is one
//            coalesced 64-B read (4 x 16-B loads) that tests two children.
//   TriRec — one leaf triangle, 80 B: the 9 fp64 vertex coordinates (exact copies of the input) +
//            the original face index.  Leaves are stored in Morton order, so a subtree's
//            triangles are contiguous.
//   PtRec  — one leaf point (ClosestPointTree), 32 B: fp64 xyz + original vertex index.
// Child reference: c >= 0 internal node index, c < 0 leaf index ~c.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#pragma clang fp contract(off)

namespace msh {

constexpr int kBlock = 256;          // 4 waves of 64 lanes
constexpr int kStack = 16;           // per-lane LDS stack entries (ring; overflow => restart)
constexpr double kSlack = 1.0 + 9.094947017729282e-13;  // 1 + 2^-40: fp64 rounding margin for culls

struct alignas(16) BNode {
    float4 a;  // lo0.x lo0.y lo0.z hi0.x
    float4 b;  // hi0.y hi0.z lo1.x lo1.y
    float4 c;  // lo1.z hi1.x hi1.y hi1.z
    int4 d;    // child0, child1, unused, unused
};
static_assert(sizeof(BNode) == 64, "BNode must be 64 B");

struct alignas(16) TriRec {
    double v[9];
    uint32_t face;
    uint32_t pad;
};
static_assert(sizeof(TriRec) == 80, "TriRec must be 80 B");

struct alignas(16) PtRec {
    double x, y, z;
    uint32_t idx;
    uint32_t pad;
};
static_assert(sizeof(PtRec) == 32, "PtRec must be 32 B");

struct D3 {
    double x, y, z;
};

__host__ __device__ inline D3 d3(double x, double y, double z) { return D3{x, y, z}; }
// CGAL Construct_vector_3(a, b) == b - a
__host__ __device__ inline D3 vsub(const D3& b, const D3& a) { return D3{b.x - a.x, b.y - a.y, b.z - a.z}; }
__host__ __device__ inline D3 vadd(const D3& a, const D3& b) { return D3{a.x + b.x, a.y + b.y, a.z + b.z}; }
__host__ __device__ inline D3 vscale(double s, const D3& a) { return D3{s * a.x, s * a.y, s * a.z}; }
__host__ __device__ inline double vdot(const D3& a, const D3& b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
__host__ __device__ inline D3 vcross(const D3& v, const D3& w) {
    return D3{v.y * w.z - v.z * w.y, v.z * w.x - v.x * w.z, v.x * w.y - v.y * w.x};
}
__host__ __device__ inline double sqdist(const D3& p, const D3& q) {
    const double dx = p.x - q.x, dy = p.y - q.y, dz = p.z - q.z;
    return dx * dx + dy * dy + dz * dz;
}
__host__ __device__ inline bool veq(const D3& a, const D3& b) { return a.x == b.x && a.y == b.y && a.z == b.z; }

// Squared distance from q to an fp32 box, evaluated in fp64 (the box corners convert exactly).
__device__ inline double box_d2(const D3& q, float lx, float ly, float lz, float hx, float hy, float hz) {
    const double dx = fmax(fmax((double)lx - q.x, q.x - (double)hx), 0.0);
    const double dy = fmax(fmax((double)ly - q.y, q.y - (double)hy), 0.0);
    const double dz = fmax(fmax((double)lz - q.z, q.z - (double)hz), 0.0);
    return dx * dx + dy * dy + dz * dz;
}

struct Box6 {
    float lx, ly, lz, hx, hy, hz;
};

__device__ inline void node_boxes(const BNode& n, Box6& b0, Box6& b1) {
    b0 = Box6{n.a.x, n.a.y, n.a.z, n.a.w, n.b.x, n.b.y};
    b1 = Box6{n.b.z, n.b.w, n.c.x, n.c.y, n.c.z, n.c.w};
}

__device__ inline BNode load_node(const BNode* __restrict__ nodes, int i) {
    const float4* p = reinterpret_cast<const float4*>(nodes + i);
    BNode n;
    n.a = p[0];
    n.b = p[1];
    n.c = p[2];
    n.d = reinterpret_cast<const int4*>(p)[3];
    return n;
}

__device__ inline void load_tri(const TriRec* __restrict__ tris, int i, D3& a, D3& b, D3& c, uint32_t& face) {
    const double2* p = reinterpret_cast<const double2*>(tris + i);
    const double2 x0 = p[0], x1 = p[1], x2 = p[2], x3 = p[3], x4 = p[4];
    a = D3{x0.x, x0.y, x1.x};
    b = D3{x1.y, x2.x, x2.y};
    c = D3{x3.x, x3.y, x4.x};
    face = (uint32_t)__double_as_longlong(x4.y);
}

// --- CGAL constructions (Simple_cartesian<double>), evaluated without FMA contraction ---
// plane_from_pointsC3(p, q, r)
__device__ inline void plane_of(const D3& p, const D3& q, const D3& r, double& a, double& b, double& c, double& d) {
    const double rpx = p.x - r.x, rpy = p.y - r.y, rpz = p.z - r.z;
    const double rqx = q.x - r.x, rqy = q.y - r.y, rqz = q.z - r.z;
    a = rpy * rqz - rqy * rpz;
    b = rpz * rqx - rqz * rpx;
    c = rpx * rqy - rqx * rpy;
    d = -a * r.x - b * r.y - c * r.z;
}

// Construct_projected_point_3(Line_3(p1, p2), q)
__device__ inline D3 project_line(const D3& p1, const D3& p2, const D3& q) {
    const double ldx = p2.x - p1.x, ldy = p2.y - p1.y, ldz = p2.z - p1.z;
    const double dpx = q.x - p1.x, dpy = q.y - p1.y, dpz = q.z - p1.z;
    const double lambda = (ldx * dpx + ldy * dpy + ldz * dpz) / (ldx * ldx + ldy * ldy + ldz * ldz);
    return D3{p1.x + lambda * ldx, p1.y + lambda * ldy, p1.z + lambda * ldz};
}

// edge test of the reference's is_inside_triangle_3_aux (nearest_point_triangle_3.h:22-60)
__device__ inline bool edge_test(const D3& w, const D3& p1, const D3& p2, const D3& q, D3& result, bool& outside) {
    const D3 e = vsub(p2, p1), pq = vsub(q, p1);
    const D3 v = vcross(e, pq);
    if (vdot(v, w) < 0.0) {
        if (vdot(pq, e) >= 0.0 && vdot(vsub(q, p2), vsub(p1, p2)) >= 0.0) {
            result = project_line(p1, p2, q);
            return true;
        }
        outside = true;
    }
    return false;
}

__device__ inline D3 seg_closest(const D3& a, const D3& b, const D3& p) {
    const D3 ab = vsub(b, a);
    const double den = vdot(ab, ab);
    if (!(den > 0.0)) return a;
    const double t = vdot(vsub(p, a), ab) / den;
    if (t <= 0.0) return a;
    if (t >= 1.0) return b;
    return D3{a.x + t * ab.x, a.y + t * ab.y, a.z + t * ab.z};
}

// Closest point of triangle (t0, t1, t2) to o with CGAL's construction; part code as
// iev::nearest_primitive (0 interior, 1/2/3 edges, 4/5/6 vertices).  Returns squared distance.
// Degenerate triangle (zero plane normal): nearest point over the three closed edges.
__device__ inline double closest_on_triangle(const D3& o, const D3& t0, const D3& t1, const D3& t2, D3& out, int& part) {
    double a, b, c, d;
    plane_of(t0, t1, t2, a, b, c, d);
    const double den = a * a + b * b + c * c;
    if (den == 0.0) {
        const D3 c0 = seg_closest(t0, t1, o), c1 = seg_closest(t1, t2, o), c2 = seg_closest(t2, t0, o);
        const double d0 = sqdist(o, c0), d1 = sqdist(o, c1), d2 = sqdist(o, c2);
        double best = d0;
        out = c0;
        part = 1;
        if (d1 < best) { best = d1; out = c1; part = 2; }
        if (d2 < best) { best = d2; out = c2; part = 3; }
        if (veq(out, t0)) part = 4; else if (veq(out, t1)) part = 5; else if (veq(out, t2)) part = 6;
        return best;
    }
    const double num = a * o.x + b * o.y + c * o.z + d;
    const double lambda = num / den;
    const D3 p = D3{o.x - lambda * a, o.y - lambda * b, o.z - lambda * c};
    const D3 w = vcross(vsub(t1, t0), vsub(t2, t1));
    bool outside = false;
    D3 r;
    if (edge_test(w, t0, t1, p, r, outside)) { out = r; part = 1; }
    else if (edge_test(w, t1, t2, p, r, outside)) { out = r; part = 2; }
    else if (edge_test(w, t2, t0, p, r, outside)) { out = r; part = 3; }
    else if (outside) {
        const double d0 = sqdist(p, t0), d1 = sqdist(p, t1), d2 = sqdist(p, t2);
        if (d1 >= d0 && d2 >= d0) { out = t0; part = 4; }
        else if (d2 >= d1) { out = t1; part = 5; }
        else { out = t2; part = 6; }
    } else {
        out = p;
        part = 0;
    }
    return sqdist(o, out);
}

// XCD-aware bijective block remap (cdna_hip_programming.md §5 "XCD swizzle must be bijective"):
// blocks b and b+8 share an XCD, so give each XCD a contiguous range of logical tiles — adjacent
// Morton-sorted query tiles then share that XCD's L2.
__device__ inline unsigned xcd_remap(unsigned bid, unsigned nwg) {
    const unsigned xcd = bid & 7u, q = nwg >> 3, r = nwg & 7u;
    const unsigned base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
    return base + (bid >> 3);
}

}  // namespace msh
