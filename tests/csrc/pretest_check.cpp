// Host-side property check of the conservative fp32 culling bounds in mesh_amd/csrc/common.h
// (tri_d2_lo, tri_d2_bounds): on random and adversarial triangles the fp32 lower bound must never
// exceed, and the upper bound never undercut, the exact squared distance (closest_on_triangle in
// common.h is device-only, so the exact value here is re-derived in long double).  Built with hipcc
// as host code; prints "violations=<n> checked=<m> rejected=<r> upper=<u>".
// Kinds: random, sliver, near a vertex, near an edge, on the face, large offset, and above the
// face/edge (6) and face/vertex (7) region boundaries, where a misclassified region matters most.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>

#include "../../mesh_amd/csrc/common.h"

// exact-ish point/triangle squared distance in long double (Ericson, well-conditioned for the check)
static long double seg_d2(long double p[3], long double a[3], long double b[3]) {
    long double ab[3], ap[3];
    for (int k = 0; k < 3; ++k) { ab[k] = b[k] - a[k]; ap[k] = p[k] - a[k]; }
    long double den = ab[0] * ab[0] + ab[1] * ab[1] + ab[2] * ab[2];
    long double t = den > 0 ? (ap[0] * ab[0] + ap[1] * ab[1] + ap[2] * ab[2]) / den : 0;
    if (t < 0) t = 0;
    if (t > 1) t = 1;
    long double d = 0;
    for (int k = 0; k < 3; ++k) { long double x = a[k] + t * ab[k] - p[k]; d += x * x; }
    return d;
}
static long double tri_d2(long double p[3], long double a[3], long double b[3], long double c[3]) {
    long double ab[3], ac[3], n[3];
    for (int k = 0; k < 3; ++k) { ab[k] = b[k] - a[k]; ac[k] = c[k] - a[k]; }
    n[0] = ab[1] * ac[2] - ab[2] * ac[1]; n[1] = ab[2] * ac[0] - ab[0] * ac[2]; n[2] = ab[0] * ac[1] - ab[1] * ac[0];
    long double nn = n[0] * n[0] + n[1] * n[1] + n[2] * n[2];
    long double best = std::min(seg_d2(p, a, b), std::min(seg_d2(p, b, c), seg_d2(p, c, a)));
    if (nn > 0) {
        long double ap[3] = {p[0] - a[0], p[1] - a[1], p[2] - a[2]};
        long double s = (ap[0] * n[0] + ap[1] * n[1] + ap[2] * n[2]) / nn;
        long double pr[3] = {p[0] - s * n[0], p[1] - s * n[1], p[2] - s * n[2]};
        // barycentric inside test
        long double v0[3] = {ab[0], ab[1], ab[2]}, v1[3] = {ac[0], ac[1], ac[2]}, v2[3] = {pr[0] - a[0], pr[1] - a[1], pr[2] - a[2]};
        long double d00 = v0[0] * v0[0] + v0[1] * v0[1] + v0[2] * v0[2], d01 = v0[0] * v1[0] + v0[1] * v1[1] + v0[2] * v1[2];
        long double d11 = v1[0] * v1[0] + v1[1] * v1[1] + v1[2] * v1[2], d20 = v2[0] * v0[0] + v2[1] * v0[1] + v2[2] * v0[2];
        long double d21 = v2[0] * v1[0] + v2[1] * v1[1] + v2[2] * v1[2];
        long double den = d00 * d11 - d01 * d01;
        long double v = (d11 * d20 - d01 * d21) / den, w = (d00 * d21 - d01 * d20) / den;
        if (v >= 0 && w >= 0 && v + w <= 1) best = std::min(best, s * s * nn);
    }
    return best;
}

int main(int argc, char** argv) {
    long n = argc > 1 ? atol(argv[1]) : 2000000;
    std::mt19937_64 rng(12345);
    std::normal_distribution<double> N(0.0, 1.0);
    std::uniform_real_distribution<double> U(0.0, 1.0);
    long viol = 0, rej = 0, pruned = 0;
    for (long it = 0; it < n; ++it) {
        const int kind = it % 8;
        double scale = std::pow(10.0, -3 + 6 * U(rng));  // triangle size
        double off = std::pow(10.0, -4 + 8 * U(rng));    // query distance
        double q[3], t[9];
        for (int k = 0; k < 3; ++k) q[k] = N(rng) * off;
        for (int k = 0; k < 9; ++k) t[k] = N(rng) * scale;
        if (kind == 1) for (int k = 0; k < 3; ++k) t[6 + k] = t[k] + (t[3 + k] - t[k]) * U(rng) + N(rng) * scale * 1e-6;  // sliver
        if (kind == 2) for (int k = 0; k < 3; ++k) q[k] = t[k] + N(rng) * scale * 1e-3;  // near a vertex
        if (kind == 3) for (int k = 0; k < 3; ++k) q[k] = 0.5 * (t[k] + t[3 + k]) + N(rng) * scale * 0.1;  // near an edge
        if (kind == 4) { double s = U(rng), r = U(rng) * (1 - s); for (int k = 0; k < 3; ++k) q[k] = t[k] + s * (t[3+k]-t[k]) + r * (t[6+k]-t[k]); }  // on face
        if (kind == 5) for (int k = 0; k < 9; ++k) t[k] += 1e6;  // large offset
        if (kind == 6 || kind == 7) {
            // above a point of the face/edge boundary (kind 6: on edge ab; kind 7: at vertex a) along the
            // normal, with a lateral jitter around the region boundary: the misclassification case
            double ab[3], ac[3], n[3];
            for (int k = 0; k < 3; ++k) { ab[k] = t[3 + k] - t[k]; ac[k] = t[6 + k] - t[k]; }
            n[0] = ab[1] * ac[2] - ab[2] * ac[1]; n[1] = ab[2] * ac[0] - ab[0] * ac[2]; n[2] = ab[0] * ac[1] - ab[1] * ac[0];
            const double nl = std::sqrt(n[0] * n[0] + n[1] * n[1] + n[2] * n[2]);
            const double s = kind == 6 ? U(rng) : 0.0;
            const double h = off * (U(rng) < 0.5 ? 1 : -1);
            for (int k = 0; k < 3; ++k)
                q[k] = t[k] + s * ab[k] + h * n[k] / nl + N(rng) * scale * std::pow(10.0, -7 + 6 * U(rng));
        }
        float f[9];
        for (int c = 0; c < 3; ++c)
            for (int k = 0; k < 3; ++k) f[3 * c + k] = (float)(t[3 * c + k] - q[k]);
        float lo, hi;
        msh::tri_d2_bounds(f[0], f[1], f[2], f[3], f[4], f[5], f[6], f[7], f[8], lo, hi);
        const float lo1 = msh::tri_d2_lo(f[0], f[1], f[2], f[3], f[4], f[5], f[6], f[7], f[8]);
        long double P[3] = {q[0], q[1], q[2]}, A[3] = {t[0], t[1], t[2]}, B[3] = {t[3], t[4], t[5]}, C[3] = {t[6], t[7], t[8]};
        const long double ex = tri_d2(P, A, B, C);
        if (lo > 0) ++rej;
        if ((long double)lo > ex * (1 + 1e-12L) + 1e-300L) {
            if (viol < 5) fprintf(stderr, "violation kind=%d lo=%.9g exact=%.17Lg\n", kind, lo, ex);
            ++viol;
        }
        if ((long double)hi < ex * (1 - 1e-12L)) {  // the upper bound may not undercut either
            if (viol < 5) fprintf(stderr, "violation kind=%d hi=%.9g exact=%.17Lg\n", kind, hi, ex);
            ++viol;
        }
        if (hi < INFINITY) ++pruned;
        if ((long double)lo1 > ex * (1 + 1e-12L) + 1e-300L) {  // the exact policies' pretest
            if (viol < 5) fprintf(stderr, "violation kind=%d tri_d2_lo=%.9g exact=%.17Lg\n", kind, lo1, ex);
            ++viol;
        }
    }
    printf("violations=%ld checked=%ld rejected=%ld upper=%ld\n", viol, n, rej, pruned);
    return viol != 0;
}
