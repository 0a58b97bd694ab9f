// Shared device-side definitions for the MI355X (gfx950) point-to-mesh search engine.
//
// Data layout in HBM:
//   BNode  — one LBVH internal node, 64 B: a node frame (unit normal n and tangent t of the node's
//            triangles, area-weighted; b = n x t is recomputed), both child references, and for BOTH
//            children the extents of the child's vertices along (n, t, b) — an oriented box that is thin
//            along the surface normal — quantised to 8 bits per bound against a per-node fp32 base and a
//            power-of-two scale per axis.  All bounds are relative to the tree's fp64 `origin`
//            (scene-box centre) and rounded outward (the decoded fp32 value base + u * 2^e is <= every
//            lower and >= every upper projection), so every fp64 primitive lies inside every ancestor's
//            boxes.  A traversal step is one 64-B read (4 x 16-B loads) that bounds two children.
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
#ifndef MSH_KSTACK
#define MSH_KSTACK 16
#endif
constexpr int kStack = MSH_KSTACK;         // per-lane LDS stack entries; deeper entries spill to global memory
constexpr double kSlack = 1.0 + 9.094947017729282e-13;  // 1 + 2^-40: fp64 rounding margin for culls

// float index within a node:  0-5 frame (n0 t0 n1 t1 n2 t2: the (n_k, t_k) pairs are 8-B aligned, so
//   the node test reads them as packed-fp32 operands) | 6 child0 | 7 child1 | 8-10 base (n, t, b) |
//   bytes 44-55: u[side][6] quantised extents (lo n t b, hi n t b) of child 0 then child 1 |
//   float 14: S0 << 16 | S2, float 15: S1 << 16 — the three axis scales as bf16 bit patterns S (the scale is
//   the fp32 whose top half is S: axis 1's scale is float 15 itself, axes 0 and 2 take one and / shift).
//   A bf16 scale rounds range / 254 up by at most 2^-8 relative, where a power of two wasted up to 2x of
//   the 8-bit code range (host model: 3.5 -> 1.5 % extra node visits over exact extents).
struct alignas(16) BNode {
    float f[16];
};
static_assert(sizeof(BNode) == 64, "BNode must be 64 B");
constexpr int kBase = 8;      // float index of base[3]
constexpr int kQuant = 44;    // byte offset of u[2][6]

// decoded bound: base + u * scale, one rounding (u * scale is exact: 8-bit code, 8-bit bf16 mantissa); the
// build encodes with this expression
__host__ __device__ inline float dequant(uint32_t u, float scale, float base) { return fmaf((float)u, scale, base); }

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

// third frame axis b = n x t in fp32 — the build and every query evaluate this same expression
__host__ __device__ inline void frame_b(const float* n, const float* t, float* b) {
    b[0] = n[1] * t[2] - n[2] * t[1];
    b[1] = n[2] * t[0] - n[0] * t[2];
    b[2] = n[0] * t[1] - n[1] * t[0];
}

// ---- node loads ----
// bit casts usable on the host (the bound property test) and the device
__host__ __device__ inline float u2f(uint32_t u) {
    union { uint32_t u; float f; } c;
    c.u = u;
    return c.f;
}
__host__ __device__ inline uint32_t f2u(float f) {
    union { float f; uint32_t u; } c;
    c.f = f;
    return c.u;
}
// fp32 rounding of x towards +inf
__host__ __device__ inline float f32_up(double x) {
    const float f = (float)x;
    return (double)f < x ? nextafterf(f, INFINITY) : f;
}

// node writers shared by the build and the host property test: frame pairs (n_k, t_k) and scale words
__host__ __device__ inline void encode_frame(float* f, const float* n, const float* t) {
    f[0] = n[0]; f[1] = t[0]; f[2] = n[1]; f[3] = t[1]; f[4] = n[2]; f[5] = t[2];
}
// smallest bf16-representable fp32 scale >= range / 254 (>= 2^-126; 2^127 for a non-finite range), so the
// codes 0..255 span the axis with a code to spare for the outward rounding
__host__ __device__ inline float bf16_scale_up(double range) {
    if (!(range < 1e38)) return u2f(0x7F000000u);
    double x = range / 254.0;
    if (!(x > 1.1754943508222875e-38)) x = 1.1754943508222875e-38;
    uint32_t u = f2u(f32_up(x));
    if (u & 0xFFFFu) u = (u & 0xFFFF0000u) + 0x10000u;
    return u2f(u);
}
__host__ __device__ inline void encode_scales(float* f, const float* sc) {
    f[14] = u2f((f2u(sc[0]) & 0xFFFF0000u) | (f2u(sc[2]) >> 16));
    f[15] = u2f(f2u(sc[1]) & 0xFFFF0000u);
}

struct NodeV {
    float4 q[4];
    __host__ __device__ float at(int i) const { return reinterpret_cast<const float*>(q)[i]; }
    __host__ __device__ uint32_t word(int i) const { return f2u(at(i)); }
    __host__ __device__ int child(int s) const { return (int)word(6 + s); }
    // frame axes n, t and b = n x t
    __host__ __device__ void frame(float* n, float* t, float* b) const {
        n[0] = at(0); n[1] = at(2); n[2] = at(4);
        t[0] = at(1); t[1] = at(3); t[2] = at(5);
        frame_b(n, t, b);
    }
    // scale of axis k (encode_scales)
    __host__ __device__ float scale(int k) const {
        return k == 0 ? u2f(word(14) & 0xFFFF0000u) : (k == 1 ? at(15) : u2f(word(14) << 16));
    }
    // decoded oriented extents of both children: e0/e1 = lo n t b, hi n t b
    __host__ __device__ void extents(float* e0, float* e1) const {
        const uint32_t w0 = word(11), w1 = word(12), w2 = word(13);
        const float sc[3] = {scale(0), scale(1), scale(2)};
        const float bs[3] = {at(kBase), at(kBase + 1), at(kBase + 2)};
        const uint32_t u[12] = {w0 & 0xffu, (w0 >> 8) & 0xffu, (w0 >> 16) & 0xffu, w0 >> 24,
                                w1 & 0xffu, (w1 >> 8) & 0xffu, (w1 >> 16) & 0xffu, w1 >> 24,
                                w2 & 0xffu, (w2 >> 8) & 0xffu, (w2 >> 16) & 0xffu, w2 >> 24};
#pragma unroll
        for (int k = 0; k < 6; ++k) {
            e0[k] = dequant(u[k], sc[k % 3], bs[k % 3]);
            e1[k] = dequant(u[6 + k], sc[k % 3], bs[k % 3]);
        }
    }
};
__device__ inline NodeV load_node(const BNode* __restrict__ nodes, int i) {
    const float4* p = reinterpret_cast<const float4*>(nodes + i);
    NodeV n;
#pragma unroll
    for (int k = 0; k < 4; ++k) n.q[k] = p[k];
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

// Squared distance from q to an fp64-rounded fp32 box, evaluated in fp64 (box corners convert exactly).
__device__ inline double box_d2(const D3& q, float lx, float ly, float lz, float hx, float hy, float hz) {
    const double dx = fmax(fmax((double)lx - q.x, q.x - (double)hx), 0.0);
    const double dy = fmax(fmax((double)ly - q.y, q.y - (double)hy), 0.0);
    const double dz = fmax(fmax((double)lz - q.z, q.z - (double)hz), 0.0);
    return dx * dx + dy * dy + dz * dz;
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
    // is_inside_triangle_3_aux (nearest_point_triangle_3.h:22-60) for the edges (t0, t1), (t1, t2), (t2, t0)
    // in that order: the first edge whose side test is negative and whose two projections are >= 0 gives
    // the answer (projection onto its line); else any negative side test means a vertex, else p.  All three
    // tests are evaluated without branches (lanes of a leaf phase test different triangles, and a divergent
    // block per edge would run once per edge for the wave), with CGAL's operand order:
    // (q - p2) . (p1 - p2) is -((q - p2) . e) exactly (negation commutes with rounding), so the second
    // projection test of edge k is pq[k + 1] . e[k] <= 0.
    const D3 e0 = vsub(t1, t0), e1 = vsub(t2, t1), e2 = vsub(t0, t2);
    const D3 q0 = vsub(p, t0), q1 = vsub(p, t1), q2 = vsub(p, t2);
    const bool n0 = vdot(vcross(e0, q0), w) < 0.0, n1 = vdot(vcross(e1, q1), w) < 0.0,
               n2 = vdot(vcross(e2, q2), w) < 0.0;
    const bool k0 = n0 && vdot(q0, e0) >= 0.0 && vdot(q1, e0) <= 0.0;
    const bool k1 = n1 && vdot(q1, e1) >= 0.0 && vdot(q2, e1) <= 0.0;
    const bool k2 = n2 && vdot(q2, e2) >= 0.0 && vdot(q0, e2) <= 0.0;
    if (k0 || k1 || k2) {
        const D3& p1 = k0 ? t0 : (k1 ? t1 : t2);
        const D3& p2 = k0 ? t1 : (k1 ? t2 : t0);
        out = project_line(p1, p2, p);
        part = k0 ? 1 : (k1 ? 2 : 3);
    } else if (n0 || n1 || n2) {
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

// ---- conservative fp32 culling (never rejects what the exact fp64 test would accept) ----
// The query relative to the tree origin, rounded to fp32; e = largest per-axis rounding error (rounded
// up); pe = the margin of the slab gaps in node_child_bounds: the fp32 projection error onto a unit
// axis, pe0 = 2^-21 |q|_1 + 2e, plus 2^-21 |q|_1 + tm for the roundings of the fused gap expressions,
// tm = 2^-21 * 1.25 * M (tree_margin), all rounded up.
// Two-lane fp32 vectors: gfx950 issues their arithmetic as packed v_pk_fma/mul/add_f32.
typedef float F2 __attribute__((ext_vector_type(2)));
__host__ __device__ inline F2 f2(float a, float b) {
    F2 r;
    r.x = a;
    r.y = b;
    return r;
}
__host__ __device__ inline F2 f2(float a) { return f2(a, a); }
__host__ __device__ inline F2 pfma(F2 a, F2 b, F2 c) { return __builtin_elementwise_fma(a, b, c); }
// xy = (x, y), zp = (z, pe): pairs, so the node test broadcasts any one of them from its register pair
struct QF {
    F2 xy, zp;
    float e;
};
__host__ __device__ inline double tree_margin(double half_diagonal) { return 5.9604644775390625e-7 * half_diagonal; }
__host__ __device__ inline QF make_qf(const D3& q, const double* origin, double tm) {
    const double rx = q.x - origin[0], ry = q.y - origin[1], rz = q.z - origin[2];
    const float x = (float)rx, y = (float)ry, z = (float)rz;
    const double e = fmax(fmax(fabs(rx - (double)x), fabs(ry - (double)y)), fabs(rz - (double)z));
    const double l1 = fabs((double)x) + fabs((double)y) + fabs((double)z);
    QF r;
    r.xy = f2(x, y);
    r.zp = f2(z, f32_up(9.5367431640625e-7 * l1 + 2.0 * e + tm));  // pe: 2^-20 |q|_1 + 2e + tm
    r.e = f32_up(e);
    return r;
}

// Both children's lower bounds of the squared distance from the query to their oriented boxes
// {x : lo_k <= a_k . x <= hi_k}, axes a = (n, t, b = n x t) in fp32, lo/hi = base + u s (s the axis scale;
// u s is exact in fp32).
// Per axis: p = fl(a . q) (fma dot product, error <= pe0 = 2^-21 |q|_1 + 2e with the query rounding);
// the gaps are formed as fma(u_lo, s, base - (p + pe)) and fma(-u_hi, s, (p - pe) - base), i.e. the
// decoded bound and the margin folded into one rounding each.  pe (make_qf) adds 2^-21 (1.25 M + |q|_1)
// to pe0, M = the tree's largest half-diagonal, which covers the roundings of p +- pe and base - (..)
// (<= 2^-23 (|base| + |bound| + |p| + pe), and |base|, |bound| <= 1.02 M) and the one of the decoded
// bound itself, so each computed gap g satisfies g <= (1 + 2^-24) * (true slab gap).  The sum of
// squares (two fmas) is scaled by 1 - 2^-18, which covers those roundings and the division by
// lambda_max(A A^T) <= 1 + 1e-6 of the nearly orthonormal fp32 axes.
// Written with two-lane fp32 vectors so gfx950 issues packed v_pk_fma/mul/add_f32 (two fp32 operations per
// lane per instruction); every lane computes exactly the scalar expression it replaces:
//   b = n x t: frame_b's products, as (n1 t2, t1 n2), (n2 t0, t2 n0), (n0 t1, t0 n1), then one subtraction;
//   p_n = fma(n0, qx, fma(n1, qy, n2 qz)), p_t, p_b likewise;
//   per axis r = (p + pe - base, (p - pe) - base) = (-(base - (p + pe)), hi side);
//   per child and axis fma(-u_lo, s, r.x) = -fma(u_lo, s, base - (p + pe)) exactly (round-to-nearest
//   is symmetric), so the slab gap is max3(-t.x, t.y, 0) with t = fma((-u_lo, -u_hi), s, r).
__host__ __device__ inline void node_child_bounds(const NodeV& nd, const QF& q, float& d0, float& d1) {
    const F2 P0 = f2(nd.q[0].x, nd.q[0].y), P1 = f2(nd.q[0].z, nd.q[0].w), P2 = f2(nd.q[1].x, nd.q[1].y);
    const F2 m0 = P1 * P2.yx, m1 = P2 * P0.yx, m2 = P0 * P1.yx;
    const float b0 = m0.x - m0.y, b1 = m1.x - m1.y, b2 = m2.x - m2.y;
    // the projections stay scalar: packed, the compiler keeps splatted query pairs live across the loop and
    // pass 1 spills twice as many registers (C3: -7 %)
    const F2 pnt = f2(fmaf(P0.x, q.xy.x, fmaf(P1.x, q.xy.y, P2.x * q.zp.x)),
                      fmaf(P0.y, q.xy.x, fmaf(P1.y, q.xy.y, P2.y * q.zp.x)));
    const float pb = fmaf(b0, q.xy.x, fmaf(b1, q.xy.y, b2 * q.zp.x));
    const F2 pe = f2(q.zp.y, -q.zp.y);
    const F2 r[3] = {(f2(pnt.x) + pe) - f2(nd.q[2].x), (f2(pnt.y) + pe) - f2(nd.q[2].y), (f2(pb) + pe) - f2(nd.q[2].z)};
    const uint32_t w0 = nd.word(11), w1 = nd.word(12), w2 = nd.word(13), we = nd.word(14);
    const float sc[3] = {u2f(we & 0xFFFF0000u), nd.q[3].w, u2f(we << 16)};
    // codes u[6 c + k] (lo) and u[6 c + 3 + k] (hi) of child c, axis k
    const uint32_t u[12] = {w0 & 0xffu, (w0 >> 8) & 0xffu, (w0 >> 16) & 0xffu, w0 >> 24,
                            w1 & 0xffu, (w1 >> 8) & 0xffu, (w1 >> 16) & 0xffu, w1 >> 24,
                            w2 & 0xffu, (w2 >> 8) & 0xffu, (w2 >> 16) & 0xffu, w2 >> 24};
    F2 g[3];  // (child 0, child 1) gap per axis
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const F2 t0 = pfma(-f2((float)u[k], (float)u[3 + k]), f2(sc[k]), r[k]);
        const F2 t1 = pfma(-f2((float)u[6 + k], (float)u[9 + k]), f2(sc[k]), r[k]);
        g[k] = f2(fmaxf(fmaxf(-t0.x, t0.y), 0.f), fmaxf(fmaxf(-t1.x, t1.y), 0.f));
    }
    const float c18 = 0.999996185302734375f;  // 1 - 2^-18
    const F2 d = pfma(g[0], g[0], pfma(g[1], g[1], g[2] * g[2])) * f2(c18);
    d0 = d.x;
    d1 = d.y;
}

// A node's 64 B loaded into LDS ahead of its step (global_load_lds: no registers hold it while the lane appends
// leaves or runs leaf rounds).  The wave's slot array holds 4 x 64 float4 (piece k of lane l at k * 64 + l); wsl =
// its LDS byte address (wave-uniform: M0), nb = this lane's first piece.
__device__ inline void node_prefetch(const BNode* __restrict__ nodes, int i, uint32_t wsl) {
    const float4* g = reinterpret_cast<const float4*>(nodes + i);
    // One address register for the four pieces (immediate offsets 0, 16, 32, 48) and M0 stepped by scalar adds of
    // 1024 - 16: the immediate offset moves the LDS destination too (tools/glds_offset_probe.hip: a lane's 16 B
    // land at M0 + offset + 16 lane).  The builtin form (__builtin_amdgcn_global_load_lds per piece, no offsets)
    // computed three more 64-bit addresses and reloaded three spilled M0 values per step: C3 0.6-0.7 % slower
    // (profiles/r04_c3_prefetch_asm_lead_ab.jsonl).  The compiler does not see these loads; node_from_lds waits
    // for them explicitly, and its own vmcnt waits stay conservative (the loads only add younger operations).
    uint32_t keep;
    asm volatile(
        "s_mov_b32 %0, m0\n\t"
        "s_mov_b32 m0, %2\n\t"
        "s_nop 0\n\t"
        "global_load_lds_dwordx4 %1, off\n\t"
        "s_add_u32 m0, m0, 0x3f0\n\t"
        "s_nop 0\n\t"
        "global_load_lds_dwordx4 %1, off offset:16\n\t"
        "s_add_u32 m0, m0, 0x3f0\n\t"
        "s_nop 0\n\t"
        "global_load_lds_dwordx4 %1, off offset:32\n\t"
        "s_add_u32 m0, m0, 0x3f0\n\t"
        "s_nop 0\n\t"
        "global_load_lds_dwordx4 %1, off offset:48\n\t"
        "s_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(g), "s"(wsl)
        : "memory", "scc");
}
__device__ inline NodeV node_from_lds(const float4* nb) {
    // the compiler does not order LDS reads after an LDS DMA: wait for it (vmcnt counts the DMA in issue order)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    NodeV n;
#pragma unroll
    for (int k = 0; k < 4; ++k) n.q[k] = nb[k * 64];
    return n;
}

// fp64 oriented-box tools for the ray and triangle kernels (fp32 frame and extents widen exactly to fp64).
// Projections of a point relative to the tree origin onto the node frame.
struct FrameD {
    D3 a[3];
};
__device__ inline FrameD frame_d(const NodeV& nd) {
    float n[3], t[3], b[3];
    nd.frame(n, t, b);
    FrameD f;
    f.a[0] = D3{n[0], n[1], n[2]};
    f.a[1] = D3{t[0], t[1], t[2]};
    f.a[2] = D3{b[0], b[1], b[2]};
    return f;
}

// v_rcp_f32 on the device (1 ulp); the host property test uses the correctly rounded quotient
__host__ __device__ inline float rcp_f32(float x) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_rcpf(x);
#else
    return 1.0f / x;
#endif
}
// ---- conservative fp32 node test of a ray (never rejects a box the ray meets at a real hit) ----
// The ray o + t d (o relative to the tree origin) is modelled in fp32 as o_f + s u_f, u = d / |d| (s = t |d|).
// Every hit x lies in the scene ball |x| <= M (M = the tree's half-diagonal), so only |s| <= s_max =
// |o| + M matters.  Per node axis a_k (fp32 frame, |a_k| <= 1 + 1e-6): po = fl(a_k . o_f) and
// pd = fl(a_k . u_f) by fma chains.  With u = 2^-24 the model's slab coordinate po + s pd differs from the
// real a_k . x(s) by <= 4.01u |o| (rounding of o and of the dot) + s_max 4.01u (the same for u).  A slab
// side is formed as fma(code, s, base - (po +- mg)), the decoded bound and the margin in one rounding:
// against the decoded fp32 bound the build verified (|bound|, |base| <= 1.02M) that adds <= u(3|o| + 3.06M
// + 3mg).  All of it is below mg = 2^-20 (|o| + M) + 2^-100, so a
// real hit at s* satisfies side_lo <= s* pd <= side_hi, i.e. s* lies in [side_lo, side_hi] / pd.  The
// computed endpoints side * rcp(pd) are within 3u relative of those quotients (v_rcp_f32: 1 ulp), so the
// interval test is widened by 2^-20 (|s_near| + |s_far|).  pd == 0 (or flushed) gives +-inf endpoints, or
// NaN where a side is exactly 0; fminf / fmaxf drop a NaN operand, which only loosens the test, and a model
// line exactly on a widened side cannot carry a real hit (mg has slack well above every rounding).  A ray
// the fp32 model cannot represent (|o| + M beyond 2^100) takes every box (`wide`).
struct RayF {
    float o[3], u[3];
    float mg, slo, shi;  // margin, parameter range [slo, shi] in units of |d|
    bool wide;
};
__host__ __device__ inline RayF make_rayf(const D3& o, const D3& d, double M, bool line) {
    RayF r;
    const double on = sqrt(vdot(o, o)), dn = sqrt(vdot(d, d));
    const double smax = (on + M) * (1.0 + 9.5367431640625e-7);
    r.wide = !(on + M < 1.2676506002282294e30) || !(dn > 0.0 && dn < INFINITY);  // 2^100; NaN -> wide
    const double inv = r.wide ? 0.0 : 1.0 / dn;
    r.o[0] = (float)o.x; r.o[1] = (float)o.y; r.o[2] = (float)o.z;
    r.u[0] = (float)(d.x * inv); r.u[1] = (float)(d.y * inv); r.u[2] = (float)(d.z * inv);
    r.mg = f32_up(9.5367431640625e-7 * (on + M) + 7.888609052210118e-31);
    r.shi = f32_up(smax);
    r.slo = line ? -r.shi : 0.f;
    return r;
}

// Both children of a node: the ray's parameter interval [n_c, f_c] inside child c's oriented box, clipped to
// [slo, shi] (before the 2^-20 widening of the tests below; `wide` rays: the whole range).
__host__ __device__ inline void ray_child_range(const NodeV& nd, const RayF& r, float& n0, float& f0, float& n1,
                                                float& f1) {
    n0 = n1 = r.slo;
    f0 = f1 = r.shi;
    if (r.wide) return;
#if defined(MUTATE_RAY_MARGIN)  // tests/csrc/bound_check.cpp's sensitivity check: must find violations
    const float mg = 0.f;
#else
    const float mg = r.mg;
#endif
    // frame pairs (n_k, t_k) and b = n x t exactly as frame_b / node_child_bounds form them
    const F2 P0 = f2(nd.q[0].x, nd.q[0].y), P1 = f2(nd.q[0].z, nd.q[0].w), P2 = f2(nd.q[1].x, nd.q[1].y);
    const F2 m0 = P1 * P2.yx, m1 = P2 * P0.yx, m2 = P0 * P1.yx;
    const float bx = m0.x - m0.y, by = m1.x - m1.y, bz = m2.x - m2.y;
    // (n, t) projections of origin and direction as packed fma chains, b's scalar
    const F2 po_nt = pfma(P0, f2(r.o[0]), pfma(P1, f2(r.o[1]), P2 * f2(r.o[2])));
    const F2 pd_nt = pfma(P0, f2(r.u[0]), pfma(P1, f2(r.u[1]), P2 * f2(r.u[2])));
    const float po[3] = {po_nt.x, po_nt.y, fmaf(bx, r.o[0], fmaf(by, r.o[1], bz * r.o[2]))};
    const float pd[3] = {pd_nt.x, pd_nt.y, fmaf(bx, r.u[0], fmaf(by, r.u[1], bz * r.u[2]))};
    const uint32_t w0 = nd.word(11), w1 = nd.word(12), w2 = nd.word(13), we = nd.word(14);
    const float sc[3] = {u2f(we & 0xFFFF0000u), nd.q[3].w, u2f(we << 16)};
    const uint32_t u[12] = {w0 & 0xffu, (w0 >> 8) & 0xffu, (w0 >> 16) & 0xffu, w0 >> 24,
                            w1 & 0xffu, (w1 >> 8) & 0xffu, (w1 >> 16) & 0xffu, w1 >> 24,
                            w2 & 0xffu, (w2 >> 8) & 0xffu, (w2 >> 16) & 0xffu, w2 >> 24};
    const F2 pm = f2(mg, -mg);
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const F2 inv = f2(rcp_f32(pd[k]));
        // (base - (po + mg), base - (po - mg)); each slab side is one fma of the code, the scale and that
        const F2 g = f2(nd.at(kBase + k)) - (f2(po[k]) + pm);
        const F2 t0 = pfma(f2((float)u[k], (float)u[3 + k]), f2(sc[k]), g) * inv;
        const F2 t1 = pfma(f2((float)u[6 + k], (float)u[9 + k]), f2(sc[k]), g) * inv;
        n0 = fmaxf(n0, fminf(t0.x, t0.y));
        f0 = fminf(f0, fmaxf(t0.x, t0.y));
        n1 = fmaxf(n1, fminf(t1.x, t1.y));
        f1 = fminf(f1, fmaxf(t1.x, t1.y));
    }
}

// Does the ray meet each child (the interval test widened by 2^-20 (|n| + |f|)), and at which entry parameter
// (the near-first key of the visibility traversal).
__host__ __device__ inline void ray_child_slabs(const NodeV& nd, const RayF& r, bool& h0, bool& h1, float& s0, float& s1) {
    float n0, f0, n1, f1;
    ray_child_range(nd, r, n0, f0, n1, f1);
    const float w = 9.5367431640625e-7f;  // 2^-20
    h0 = n0 <= f0 + w * (fabsf(n0) + fabsf(f0));
    h1 = n1 <= f1 + w * (fabsf(n1) + fabsf(f1));
    s0 = n0;
    s1 = n1;
}

// Lines (nearest_alongnormal): as ray_child_slabs, and for each child a lower bound of the squared distance from
// the line's point p (parameter 0) to any real hit inside the child.  u = d / |d| is a unit direction, so the
// parameter s of a hit x = p + s u is its signed distance from p; a real hit's s* lies in the widened interval
// [n - e, f + e], e = 2^-20 (|n| + |f|) (the derivation above: the endpoints are within 3u relative of the exact
// quotients, and e is 16x that), so |x - p| >= max(n - e, -(f + e), 0).  That bound, shrunk by 2^-20 and its square
// by 2^-19 against the fp32 roundings of forming it, is the key: it is never larger than the exact distance of a
// hit in the child (tests/csrc/bound_check.cpp checks it on the same rays as the slab test), and it is at least
// the distance from p to the child's box, which the line's hits lie in.
__host__ __device__ inline void ray_child_line_dist2(const NodeV& nd, const RayF& r, bool& h0, bool& h1, float& k0,
                                                     float& k1) {
    float n0, f0, n1, f1;
    ray_child_range(nd, r, n0, f0, n1, f1);
    const float w = 9.5367431640625e-7f;  // 2^-20
    const float e0 = w * (fabsf(n0) + fabsf(f0)), e1 = w * (fabsf(n1) + fabsf(f1));
    h0 = n0 <= f0 + e0;
    h1 = n1 <= f1 + e1;
#if defined(MUTATE_LINE_DIST)  // tests/csrc/bound_check.cpp's sensitivity check: the far end instead of the near one
    const float g0 = fmaxf(fmaxf(f0, -n0), 0.f), g1 = fmaxf(fmaxf(f1, -n1), 0.f);
#else
    const float g0 = fmaxf(fmaxf(n0 - e0, -(f0 + e0)), 0.f) * (1.f - w);
    const float g1 = fmaxf(fmaxf(n1 - e1, -(f1 + e1)), 0.f) * (1.f - w);
#endif
    k0 = g0 * g0 * (1.f - 2.f * w);
    k1 = g1 * g1 * (1.f - 2.f * w);
}

// Per-lane traversal stack: entry sp lives in LDS (lds[sp * kBlock], lane-interleaved) for
// sp < kStack and in the block's global spill area beyond.  The spill side uses the nontemporal
// builtins so the compiler cannot fold the two cases into one generic (flat) access through a
// pointer select: flat accesses to LDS go through the vector memory pipe and make every stack
// push/pop wait for the outstanding node loads.
// (D: the LDS depth; the ray kernels' alongnormal instantiation keeps a shallower one, rays.hip kAlongStack)
template <int D = kStack>
__device__ inline void stack_put(uint2* __restrict__ lds, uint2* __restrict__ spill, int sp, uint2 e) {
    if (sp < D) {
        lds[sp * kBlock] = e;
    } else {
        unsigned long long* p = reinterpret_cast<unsigned long long*>(spill + (size_t)(sp - D) * kBlock);
        __builtin_nontemporal_store(((unsigned long long)e.y << 32) | e.x, p);
    }
}
template <int D = kStack>
__device__ inline uint2 stack_get(const uint2* __restrict__ lds, const uint2* __restrict__ spill, int sp) {
    if (sp < D) return lds[sp * kBlock];
    const unsigned long long* p = reinterpret_cast<const unsigned long long*>(spill + (size_t)(sp - D) * kBlock);
    const unsigned long long v = __builtin_nontemporal_load(p);
    return make_uint2((unsigned)v, (unsigned)(v >> 32));
}
// 4-B entries (compact stacks, trees of <= 2^20 leaves): the same placement; the spill side takes a 64-bit slot
// like the 8-B stack's (a 32-bit access let the compiler merge both sides into one flat access)
__device__ inline void stack_put(uint32_t* __restrict__ lds, uint2* __restrict__ spill, int sp, uint32_t e) {
    if (sp < kStack) {
        lds[sp * kBlock] = e;
    } else {
        __builtin_nontemporal_store((unsigned long long)e,
                                    reinterpret_cast<unsigned long long*>(spill + (size_t)(sp - kStack) * kBlock));
    }
}
__device__ inline uint32_t stack_get(const uint32_t* __restrict__ lds, const uint2* __restrict__ spill, int sp) {
    if (sp < kStack) return lds[sp * kBlock];
    return (uint32_t)__builtin_nontemporal_load(
        reinterpret_cast<const unsigned long long*>(spill + (size_t)(sp - kStack) * kBlock));
}

// 30-bit Morton code of a query point in the box [l, h] (fp32 cell coordinates, 1024 cells per axis, clamped)
__device__ inline uint32_t query_morton30(double x, double y, double z, float lx, float ly, float lz, float hx, float hy,
                                          float hz) {
    const float ex = hx - lx, ey = hy - ly, ez = hz - lz;
    float nx = ex > 0.f ? ((float)x - lx) / ex : 0.5f;
    float ny = ey > 0.f ? ((float)y - ly) / ey : 0.5f;
    float nz = ez > 0.f ? ((float)z - lz) / ez : 0.5f;
    nx = fminf(fmaxf(nx * 1024.f, 0.f), 1023.f);
    ny = fminf(fmaxf(ny * 1024.f, 0.f), 1023.f);
    nz = fminf(fmaxf(nz * 1024.f, 0.f), 1023.f);
    auto ex10 = [](uint32_t v) {
        v = (v * 0x00010001u) & 0xFF0000FFu;
        v = (v * 0x00000101u) & 0x0F00F00Fu;
        v = (v * 0x00000011u) & 0xC30C30C3u;
        v = (v * 0x00000005u) & 0x49249249u;
        return v;
    };
    return (ex10((uint32_t)nx) << 2) | (ex10((uint32_t)ny) << 1) | ex10((uint32_t)nz);
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
