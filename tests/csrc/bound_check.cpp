// Host property test of the traversal's child-box bound (mesh_amd/csrc/common.h node_child_bounds +
// make_qf): for nodes whose decoded oriented boxes contain their points (the build's contract, checked on
// the GPU by scripts/check_tree.py), the fp32 bound must never exceed the squared distance from the fp64
// query to any of those points.  Random frames, point clouds and queries at every scale, adversarial
// placements (queries on / just off the points, far away, at a large offset from the origin), codes
// chosen as tight as the contract allows.  Prints "violations=N" (and the worst cases) and exits 1 when
// N > 0.  -DMUTATE_TREE_TERM / -DMUTATE_QUERY_MARGIN drop a margin term: those builds must fail (the
// test's sensitivity check, tests/test_abi.py).  The same nodes check the ray kernels' fp32 slab test
// (common.h make_rayf / ray_child_slabs): a ray or line through a point of a child must take that child;
// -DMUTATE_RAY_MARGIN drops its margin and must fail.
//   hipcc -O2 -std=c++17 -ffp-contract=off -x hip bound_check.cpp -I<csrc> -o bound_check && ./bound_check 200000
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>

#include "common.h"

using namespace msh;

namespace {

// tightest valid 8-bit code for a bound v against base / scale: dequant(lo code) <= v <= dequant(hi code)
uint32_t code_lo(double v, float base, float sc) {
    double c = std::floor((v - (double)base) / (double)sc);
    uint32_t u = (uint32_t)std::fmin(std::fmax(c, 0.0), 255.0);
    while (u > 0u && (double)dequant(u, sc, base) > v) --u;
    while (u < 255u && (double)dequant(u + 1, sc, base) <= v) ++u;
    return u;
}
uint32_t code_hi(double v, float base, float sc) {
    double c = std::ceil((v - (double)base) / (double)sc);
    uint32_t u = (uint32_t)std::fmin(std::fmax(c, 0.0), 255.0);
    while (u < 255u && (double)dequant(u, sc, base) < v) ++u;
    while (u > 0u && (double)dequant(u - 1, sc, base) >= v) --u;
    return u;
}

}  // namespace

int main(int argc, char** argv) {
    const long trials = argc > 1 ? std::atol(argv[1]) : 100000;
    std::mt19937_64 rng(12345);
    std::uniform_real_distribution<double> U(-1.0, 1.0);
    auto unit = [&]() {
        for (;;) {
            double x = U(rng), y = U(rng), z = U(rng);
            double l = std::sqrt(x * x + y * y + z * z);
            if (l > 0.1 && l <= 1.0) return D3{x / l, y / l, z / l};
        }
    };
    long viol = 0, checks = 0, tight = 0, skipped = 0, skipped_anchor = 0, ray_checks = 0, ray_viol = 0, ray_skipped = 0;
    long line_checks = 0, line_viol = 0, line_tight = 0;
    double worst = 0.0;
    for (long tr = 0; tr < trials; ++tr) {
        // scene scale, node size relative to it, offset of the tree origin
        const double S = std::pow(10.0, (int)(rng() % 7) - 3);            // 1e-3 .. 1e3
        const double node = S * std::pow(10.0, -(double)(rng() % 7));     // node size S .. 1e-6 S
        const double off = (rng() % 3 == 0) ? 0.0 : S * std::pow(10.0, (double)(rng() % 6));
        const double origin[3] = {off * U(rng), off * U(rng), off * U(rng)};
        // node centre relative to the origin.  Every 4th trial centres the node on the origin with child 0
        // below and child 1 above t = 0, and later moves a child-1 point onto its box's lower t bound: a
        // query just below that point is then close to it while |q| << the node's range, so the rounding
        // of base - (p + pe) is not covered by the query's own terms (the case of the tree term tm)
        const bool at_origin = tr % 4 == 0;
        const D3 c = at_origin ? D3{0, 0, 0} : D3{S * U(rng), S * U(rng), S * U(rng)};
        // frame as the build makes it: unit n, t = e - (e.n) n normalised, b = n x t in fp32
        const D3 n = unit();
        const D3 e = std::fabs(n.x) < 0.9 ? D3{1, 0, 0} : D3{0, 1, 0};
        D3 t = vsub(e, vscale(vdot(e, n), n));
        const double tl = std::sqrt(vdot(t, t));
        t = D3{t.x / tl, t.y / tl, t.z / tl};
        float nf[3] = {(float)n.x, (float)n.y, (float)n.z}, tf[3] = {(float)t.x, (float)t.y, (float)t.z}, bf[3];
        frame_b(nf, tf, bf);
        const double A[3][3] = {{nf[0], nf[1], nf[2]}, {tf[0], tf[1], tf[2]}, {bf[0], bf[1], bf[2]}};
        // two children: 6 points each, flattened along n like surface patches (absolute fp64 coordinates)
        D3 pts[2][6];
        double mn[2][3], mx[2][3];
        double half_diag = 0.0;
        for (int ch = 0; ch < 2; ++ch) {
            for (int k = 0; k < 3; ++k) { mn[ch][k] = INFINITY; mx[ch][k] = -INFINITY; }
            for (int i = 0; i < 6; ++i) {
                double a = node * U(rng);
                const double b = node * U(rng), h = node * 1e-3 * U(rng);
                if (at_origin) a = ch == 0 ? -std::fabs(a) : std::fabs(a);
                const D3 r = D3{c.x + a * t.x + b * (n.y * t.z - n.z * t.y) + h * n.x,
                                c.y + a * t.y + b * (n.z * t.x - n.x * t.z) + h * n.y,
                                c.z + a * t.z + b * (n.x * t.y - n.y * t.x) + h * n.z};
                pts[ch][i] = D3{origin[0] + r.x, origin[1] + r.y, origin[2] + r.z};
                if (at_origin && ch == 1 && i == 0) {
                    const double tiny = node * 1e-6;
                    pts[ch][i] = D3{origin[0] + tiny * U(rng), origin[1] + tiny * U(rng), origin[2] + tiny * U(rng)};
                }
                const double rx = pts[ch][i].x - origin[0], ry = pts[ch][i].y - origin[1], rz = pts[ch][i].z - origin[2];
                half_diag = std::fmax(half_diag, std::sqrt(rx * rx + ry * ry + rz * rz));
                for (int k = 0; k < 3; ++k) {
                    const double pr = A[k][0] * rx + A[k][1] * ry + A[k][2] * rz;
                    mn[ch][k] = std::fmin(mn[ch][k], pr);
                    mx[ch][k] = std::fmax(mx[ch][k], pr);
                }
            }
        }
        // the build first rounds each bound outward to fp32 (build.hip out_lo / out_hi)
        for (int ch = 0; ch < 2; ++ch)
            for (int k = 0; k < 3; ++k) {
                float lo = (float)mn[ch][k], hi = (float)mx[ch][k];
                if ((double)lo > mn[ch][k]) lo = nextafterf(lo, -INFINITY);
                if ((double)hi < mx[ch][k]) hi = nextafterf(hi, INFINITY);
                mn[ch][k] = lo;
                mx[ch][k] = hi;
            }
        // node encoding: fp32 base below both children, bf16 scale (build.hip encode_node), tightest codes
        BNode bn;
        std::memset(&bn, 0, sizeof(bn));
        float* f = bn.f;
        encode_frame(f, nf, tf);
        f[6] = u2f(~0u);
        f[7] = u2f(~1u);
        uint32_t u[12];
        float scs[3];
        for (int k = 0; k < 3; ++k) {
            float base = (float)std::fmin(mn[0][k], mn[1][k]);
            if ((double)base > std::fmin(mn[0][k], mn[1][k])) base = nextafterf(base, -INFINITY);
            const double range = std::fmax(mx[0][k], mx[1][k]) - (double)base;
            const float sc = bf16_scale_up(range);
            f[kBase + k] = base;
            scs[k] = sc;
            for (int ch = 0; ch < 2; ++ch) {
                u[6 * ch + k] = code_lo(mn[ch][k], base, sc);
                u[6 * ch + 3 + k] = code_hi(mx[ch][k], base, sc);
            }
        }
        for (int j = 0; j < 3; ++j) f[11 + j] = u2f(u[4 * j] | (u[4 * j + 1] << 8) | (u[4 * j + 2] << 16) | (u[4 * j + 3] << 24));
        encode_scales(f, scs);
        NodeV nd;
        std::memcpy(&nd, &bn, sizeof(bn));
        // the decoded boxes must contain the points (what the build guarantees); skip codes that cannot
        float e0[6], e1[6];
        nd.extents(e0, e1);
        bool ok = true;
        for (int k = 0; k < 3; ++k)
            ok = ok && (double)e0[k] <= mn[0][k] && (double)e0[3 + k] >= mx[0][k] && (double)e1[k] <= mn[1][k] &&
                 (double)e1[3 + k] >= mx[1][k];
        if (!ok) {
            ++skipped;
            continue;
        }
        const double tm = tree_margin(half_diag);
        D3 anchor = pts[1][0];
        const D3 td = D3{tf[0], tf[1], tf[2]};
        if (at_origin) {
            // slide child 1's point 0 along t until its t projection is just above the decoded bound
            const D3 r = D3{anchor.x - origin[0], anchor.y - origin[1], anchor.z - origin[2]};
            const double shift = ((double)e1[1] - (A[1][0] * r.x + A[1][1] * r.y + A[1][2] * r.z)) * (1.0 - 1e-12) / vdot(td, td);
            const D3 moved = D3{origin[0] + (r.x + shift * td.x), origin[1] + (r.y + shift * td.y),
                                origin[2] + (r.z + shift * td.z)};
            // containment of the stored (rounded) point, projected as the build projects vertices
            const D3 r2 = D3{moved.x - origin[0], moved.y - origin[1], moved.z - origin[2]};
            bool in = true;
            for (int k = 0; k < 3; ++k) {
                const double pr = A[k][0] * r2.x + A[k][1] * r2.y + A[k][2] * r2.z;
                in = in && pr >= (double)e1[k] && pr <= (double)e1[3 + k];
            }
            if (in) {
                anchor = moved;
                pts[1][0] = anchor;
            } else {
                ++skipped_anchor;
            }
        }
        // rays (ray_child_slabs + make_rayf): every ray or line through a point of a child must take that child.
        // Directions at random, along a frame axis (parallel to two slab pairs) or grazing the n = const faces;
        // the ray starts at the point or up to 1e3 scene sizes before it (behind it too for lines).
        {
            double M = half_diag;
            const D3 an = D3{anchor.x - origin[0], anchor.y - origin[1], anchor.z - origin[2]};
            M = std::fmax(M, std::sqrt(vdot(an, an))) * (1.0 + 1e-9);
            for (int ri = 0; ri < 8; ++ri) {
                const int ch = at_origin && ri % 2 == 0 ? 1 : (int)(rng() % 2);
                const D3 x = at_origin && ri % 2 == 0 ? anchor : pts[ch][rng() % 6];
                const int dk = (int)(rng() % 4);
                D3 d = unit();
                if (dk == 1) {
                    const int ax = (int)(rng() % 3);
                    d = D3{A[ax][0], A[ax][1], A[ax][2]};
                } else if (dk == 2) {
                    const double g = std::pow(10.0, -(double)(3 + rng() % 8)) * U(rng);
                    d = D3{A[1][0] + g * A[0][0], A[1][1] + g * A[0][1], A[1][2] + g * A[0][2]};
                } else if (dk == 3) {
                    d = vscale(std::pow(10.0, (double)((int)(rng() % 13) - 6)), d);  // any length
                }
                const bool line = rng() % 2 == 0;
                const int sk = (int)(rng() % 4);
                double s = sk == 0 ? 0.0 : (sk == 1 ? node * std::pow(10.0, -(double)(rng() % 8))
                                                    : S * std::pow(10.0, (double)(rng() % 4)));
                s /= std::sqrt(vdot(d, d));
                if (line && rng() % 2 == 0) s = -s;
                const D3 o = D3{x.x - s * d.x, x.y - s * d.y, x.z - s * d.z};
                // the rounded origin moves the ray off x by ~1 ulp of |o|: keep the rays that still pass a point
                // of the decoded box (x' = o + s d in long double)
                {
                    const long double xr[3] = {(long double)o.x + (long double)s * d.x - origin[0],
                                               (long double)o.y + (long double)s * d.y - origin[1],
                                               (long double)o.z + (long double)s * d.z - origin[2]};
                    const float* e = ch == 0 ? e0 : e1;
                    bool in = true;
                    for (int k = 0; k < 3; ++k) {
                        const long double pr = A[k][0] * xr[0] + A[k][1] * xr[1] + A[k][2] * xr[2];
                        in = in && pr >= (long double)e[k] && pr <= (long double)e[3 + k];
                    }
                    if (!in) {
                        ++ray_skipped;
                        continue;
                    }
                }
                const RayF rf = make_rayf(D3{o.x - origin[0], o.y - origin[1], o.z - origin[2]}, d, M, line);
                bool h[2];
                float s0, s1;
                ray_child_slabs(nd, rf, h[0], h[1], s0, s1);
                ++ray_checks;
                if (line) {
                    // nearest_alongnormal's node test (ray_child_line_dist2): the child is taken and its key is at
                    // most the squared distance from the line's point o to the point x' of the child it passes
                    bool hl[2];
                    float kl[2];
                    ray_child_line_dist2(nd, rf, hl[0], hl[1], kl[0], kl[1]);
                    const long double dist = fabsl((long double)s) *
                        sqrtl((long double)d.x * d.x + (long double)d.y * d.y + (long double)d.z * d.z);
                    ++line_checks;
                    if (hl[ch] && (long double)kl[ch] > 0.5L * dist * dist) ++line_tight;
                    if (!hl[ch] || (long double)kl[ch] > dist * dist) {
                        ++viol;
                        ++line_viol;
                        if (line_viol <= 5)
                            std::fprintf(stderr, "line violation: dk=%d sk=%d hit=%d key=%.9g dist2=%.17Lg s=%g\n", dk, sk,
                                         (int)hl[ch], kl[ch], dist * dist, s);
                    }
                }
                if (!h[ch]) {
                    ++viol;
                    ++ray_viol;
                    if (ray_viol <= 5)
                        std::fprintf(stderr, "ray violation: dk=%d sk=%d line=%d S=%g node=%g off=%g s=%g\n", dk, sk,
                                     (int)line, S, node, off, s);
                }
            }
        }
        // queries: on a point, just off it (1e-12 .. 1e-3 node), inside the box, far away
        for (int qi = 0; qi < 8; ++qi) {
            const int ch = (int)(rng() % 2), pi = (int)(rng() % 6);
            const D3 p = pts[ch][pi];
            D3 q;
            const int kind = at_origin ? 4 + qi % 2 : qi % 4;
            if (kind >= 4) {  // just below the anchor along t: 0 .. 1e-6 of the node size
                const double eta = kind == 4 ? 0.0 : node * std::pow(10.0, -(double)(6 + rng() % 6));
                q = D3{anchor.x - eta * td.x, anchor.y - eta * td.y, anchor.z - eta * td.z};
            } else if (kind == 0) q = p;
            else if (kind == 1) {
                const double d = node * std::pow(10.0, -(double)(3 + rng() % 10));
                const D3 dir = unit();
                q = D3{p.x + d * dir.x, p.y + d * dir.y, p.z + d * dir.z};
            } else if (kind == 2) {
                q = D3{origin[0] + c.x + node * U(rng), origin[1] + c.y + node * U(rng), origin[2] + c.z + node * U(rng)};
            } else {
                const double d = node * std::pow(10.0, (double)(rng() % 4));
                const D3 dir = unit();
                q = D3{p.x + d * dir.x, p.y + d * dir.y, p.z + d * dir.z};
            }
#if defined(MUTATE_TREE_TERM)  // the test's own check: without the tree term it must find violations
            QF qf = make_qf(q, origin, 0.0);
#else
            QF qf = make_qf(q, origin, tm);
#endif
#if defined(MUTATE_QUERY_MARGIN)  // ... and without any margin
            qf.zp.y = 0.f;
#endif
            float d2[2];
            node_child_bounds(nd, qf, d2[0], d2[1]);
            for (int c2 = 0; c2 < 2; ++c2) {
                long double best = INFINITY;
                for (int i = 0; i < 6; ++i) {
                    const long double dx = (long double)q.x - pts[c2][i].x, dy = (long double)q.y - pts[c2][i].y,
                                      dz = (long double)q.z - pts[c2][i].z;
                    best = std::fmin(best, dx * dx + dy * dy + dz * dz);
                }
                ++checks;
                if (best > 0 && (long double)d2[c2] > 0.5L * best) ++tight;
                if ((long double)d2[c2] > best) {
                    ++viol;
                    const double rel = best > 0 ? (double)(((long double)d2[c2] - best) / best) : INFINITY;
                    worst = std::fmax(worst, rel);
                    if (viol <= 5)
                        std::fprintf(stderr, "violation: kind=%d S=%g node=%g off=%g bound=%.9g exact=%.17Lg\n", kind, S,
                                     node, off, d2[c2], best);
                }
            }
        }
    }
    std::printf("line_checks=%ld line_tight=%ld line_violations=%ld\n", line_checks, line_tight, line_viol);
    std::printf("trials=%ld skipped=%ld anchors_skipped=%ld checks=%ld tight=%ld ray_checks=%ld ray_skipped=%ld ray_violations=%ld "
                "violations=%ld worst_rel=%g\n", trials, skipped, skipped_anchor, checks, tight, ray_checks, ray_skipped, ray_viol,
                viol, worst);
    return viol == 0 && skipped == 0 ? 0 : 1;
}
