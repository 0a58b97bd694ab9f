// K10 — vertex normals on the GPU (replaces Mesh.estimate_vertex_normals, mesh.py:208-216:
// TriNormalsScaled = CrossProduct(v[f1] - v[f0], v[f2] - v[f0]) (geometry/tri_normals.py:23-24), summed
// per vertex by the sparse face->vertex incidence product in ascending face order, then divided by the
// row norm, 0 -> 1).  These normals feed visibility_compute (mesh.py:300) and the normals-tree queries.
//
//   k_face_normals    one lane per face: scaled normal (fp64, the reference's cross-product terms)
//   radix sort        (vertex id, corner index) pairs, stable: every vertex's faces in ascending order
//   k_vertex_ranges   [first, end) of every vertex's run in the sorted corner list
//   k_vertex_sum      one lane per vertex: ordered sum of its faces' normals, norm ((x^2 + y^2) + z^2,
//                     numpy's reduction order over a row of 3), division
#include <algorithm>

#include "internal.h"

namespace msh {

// Face indices are checked here (device callers hand over unchecked faces): a face with an index >= P
// raises *err and contributes a zero normal instead of reading past v.
__global__ __launch_bounds__(kBlock) void k_face_normals(const double* __restrict__ v, size_t P,
                                                         const uint32_t* __restrict__ f, size_t T,
                                                         double* __restrict__ fn, uint32_t* __restrict__ err) {
    const size_t t = (size_t)blockIdx.x * kBlock + threadIdx.x;
    if (t >= T) return;
    const size_t i0 = f[3 * t], i1 = f[3 * t + 1], i2 = f[3 * t + 2];
    if (i0 >= P || i1 >= P || i2 >= P) {
        *err = 1u;
        fn[3 * t] = fn[3 * t + 1] = fn[3 * t + 2] = 0.0;
        return;
    }
    const D3 a = D3{v[3 * i0], v[3 * i0 + 1], v[3 * i0 + 2]};
    const D3 b = D3{v[3 * i1], v[3 * i1 + 1], v[3 * i1 + 2]};
    const D3 c = D3{v[3 * i2], v[3 * i2 + 1], v[3 * i2 + 2]};
    const D3 n = vcross(vsub(b, a), vsub(c, a));
    fn[3 * t] = n.x;
    fn[3 * t + 1] = n.y;
    fn[3 * t + 2] = n.z;
}

// keys = vertex of corner e (f flattened; an index >= P becomes P, which sorts last), vals = e
__global__ __launch_bounds__(kBlock) void k_corner_keys(const uint32_t* __restrict__ f, size_t n, size_t P,
                                                        uint32_t* __restrict__ keys, uint32_t* __restrict__ vals) {
    const size_t e = (size_t)blockIdx.x * kBlock + threadIdx.x;
    if (e >= n) return;
    keys[e] = f[e] < P ? f[e] : (uint32_t)P;
    vals[e] = (uint32_t)e;
}

// sorted corner keys == P (out-of-range faces, flagged by k_face_normals) sort last and are skipped
__global__ __launch_bounds__(kBlock) void k_vertex_ranges(const uint32_t* __restrict__ keys, size_t n, size_t P,
                                                          uint32_t* __restrict__ first, uint32_t* __restrict__ end) {
    const size_t p = (size_t)blockIdx.x * kBlock + threadIdx.x;
    if (p >= n) return;
    const uint32_t k = keys[p];
    if (k >= P) return;
    if (p == 0 || keys[p - 1] != k) first[k] = (uint32_t)p;
    if (p + 1 == n || keys[p + 1] != k) end[k] = (uint32_t)(p + 1);
}

__global__ __launch_bounds__(kBlock) void k_vertex_sum(const double* __restrict__ fn, const uint32_t* __restrict__ corners,
                                                       const uint32_t* __restrict__ first, const uint32_t* __restrict__ end,
                                                       size_t P, double* __restrict__ vn) {
    const size_t i = (size_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= P) return;
    double x = 0.0, y = 0.0, z = 0.0;
    for (uint32_t p = first[i]; p < end[i]; ++p) {
        const size_t t = corners[p] / 3u;
        x += fn[3 * t];
        y += fn[3 * t + 1];
        z += fn[3 * t + 2];
    }
    double nrm = sqrt(x * x + y * y + z * z);  // np.sum(x ** 2, axis=1) on (P,3): left to right
    if (nrm == 0.0) nrm = 1.0;
    vn[3 * i] = x / nrm;
    vn[3 * i + 1] = y / nrm;
    vn[3 * i + 2] = z / nrm;
}

static unsigned nblk(size_t n) { return (unsigned)((n + kBlock - 1) / kBlock); }

int vertex_normals(const double* d_v, size_t P, const uint32_t* d_f, size_t T, double* d_vn, Workspace& ws,
                   hipStream_t s, uint32_t* d_err) {
    if (P == 0) return MSH_OK;
    const size_t n = 3 * T;
    if (n > 0xFFFFFFFFull) {
        set_error("vertex normals: %zu face corners exceed the 32-bit index range", n);
        return MSH_EINVAL;
    }
    TimedLaunch tl("vertex_normals", s);
    MSH_TRY(ws.out_d.reserve(std::max<size_t>(n, 1) * sizeof(double)));  // face normals (T,3)
    MSH_TRY(ws.keys.reserve(std::max<size_t>(n, 1) * sizeof(uint32_t)));
    MSH_TRY(ws.vals.reserve(std::max<size_t>(n, 1) * sizeof(uint32_t)));
    MSH_TRY(ws.keys_alt.reserve(std::max<size_t>(n, 1) * sizeof(uint32_t)));
    MSH_TRY(ws.vals_alt.reserve(std::max<size_t>(n, 1) * sizeof(uint32_t)));
    MSH_TRY(ws.ranges.reserve(2 * P * sizeof(uint32_t)));
    double* fn = ws.out_d.as<double>();
    uint32_t* first = ws.ranges.as<uint32_t>();
    uint32_t* end = first + P;
    MSH_HIP(hipMemsetAsync(first, 0, 2 * P * sizeof(uint32_t), s));
    if (T) {
        k_face_normals<<<nblk(T), kBlock, 0, s>>>(d_v, P, d_f, T, fn, d_err);
        MSH_HIP(hipGetLastError());
        k_corner_keys<<<nblk(n), kBlock, 0, s>>>(d_f, n, P, ws.keys.as<uint32_t>(), ws.vals.as<uint32_t>());
        MSH_HIP(hipGetLastError());
        int bits = 1;  // keys are <= P (P marks an out-of-range index)
        while (bits < 32 && ((size_t)1 << bits) <= P) ++bits;
        MSH_TRY(radix_sort_pairs(ws.keys.as<uint32_t>(), ws.vals.as<uint32_t>(), ws.keys_alt.as<uint32_t>(),
                                 ws.vals_alt.as<uint32_t>(), n, bits, ws, s));
        k_vertex_ranges<<<nblk(n), kBlock, 0, s>>>(ws.keys.as<uint32_t>(), n, P, first, end);
        MSH_HIP(hipGetLastError());
    }
    k_vertex_sum<<<nblk(P), kBlock, 0, s>>>(fn, ws.vals.as<uint32_t>(), first, end, P, d_vn);
    MSH_HIP(hipGetLastError());
    return MSH_OK;
}

}  // namespace msh
