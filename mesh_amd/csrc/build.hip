// K1 — GPU LBVH build (replaces CGAL AABB_tree::rebuild's median-split build,
// spatialsearchmodule.cpp:122, and accelerate_distance_queries' KD hint, :123).
//
//   1. k_tri_bounds / k_point_bounds   fp64 bounds of every primitive
//   2. k_reduce_box                    scene box (fp64); origin = its centre (fp32 bounds are relative
//                                      to it, so meshes far from (0,0,0) keep full fp32 precision)
//   3. k_morton                        30-bit Morton code of each primitive's box centre
//   4. radix_sort_pairs (sort.hip)     stable LDS radix sort (key, primitive id): equal codes keep id order
//   5. k_karras                        Karras (HPG 2012) internal-node emission; codes made unique by
//                                      augmenting them with the sorted position; also records each
//                                      node's contiguous leaf range and split
//   6. (in k_karras)                   a bound of the leaf depth from the prefix lengths (sizes the stack spill)
//   7. (after leaf packing) k_obb_lane / k_obb_wave   one lane (<= 32 leaves) or one wave per node over
//                                      its Morton leaf range: area-weighted
//                                      normal -> node frame (n, t, b = n x t), then both children's vertex
//                                      extents along the frame (oriented boxes, thin along the surface),
//                                      quantised to 8 bits against a per-node base and bf16 scale
// All bounds are rounded outward (fp32 round-down lo / round-up hi plus one ulp, then the quantised code
// rounds down / up, checked against the decoder), so every fp64 primitive lies inside the bounds of
// every ancestor.  Round 1 also stored an fp32 AABB per child (128-B nodes, filled by a bottom-up refit);
// the oriented boxes alone traverse faster.
#include <algorithm>
#include <memory>

#include <vector>

#include "internal.h"

namespace msh {

// largest distance from `origin` to a corner of box (lo[3], hi[3]); a non-finite box gives +inf (the
// query margin then disables culling rather than under-bounding it)
double half_diagonal(const double* box, const double* origin) {
    double s = 0.0;
    for (int k = 0; k < 3; ++k) {
        const double d = std::max(fabs(box[k] - origin[k]), fabs(box[3 + k] - origin[k]));
        s += d * d;
    }
    const double r = sqrt(s) * (1.0 + 1e-12);
    return r == r ? r : INFINITY;
}

// Batched kernels: B meshes of P vertices / T primitives each, stored back to back (primitive
// g = b*T + t of mesh b = g / T); the single-mesh build is B = 1.
__global__ __launch_bounds__(kBlock) void k_tri_bounds(const double* __restrict__ v, size_t P, const uint32_t* __restrict__ f,
                                                       size_t n, size_t T, double* __restrict__ lo, double* __restrict__ hi) {
    const size_t g = (size_t)blockIdx.x * kBlock + threadIdx.x;
    if (g >= n) return;
    const size_t b = g / T, t = g - b * T;
    const double* vb = v + 3 * P * b;
    const uint32_t i0 = f[3 * t], i1 = f[3 * t + 1], i2 = f[3 * t + 2];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const double a = vb[3 * (size_t)i0 + k], bb = vb[3 * (size_t)i1 + k], c = vb[3 * (size_t)i2 + k];
        lo[3 * g + k] = fmin(fmin(a, bb), c);
        hi[3 * g + k] = fmax(fmax(a, bb), c);
    }
}

__global__ __launch_bounds__(kBlock) void k_point_bounds(const double* __restrict__ v, size_t P, double* __restrict__ lo,
                                                         double* __restrict__ hi) {
    const size_t t = (size_t)blockIdx.x * kBlock + threadIdx.x;
    if (t >= 3 * P) return;
    lo[t] = v[t];
    hi[t] = v[t];
}

// out[6*b .. 6*b+5] = (min lo xyz, max hi xyz) over the block's range
__global__ __launch_bounds__(kBlock) void k_reduce_box(const double* __restrict__ lo, const double* __restrict__ hi,
                                                       size_t n, double* __restrict__ out) {
    __shared__ double sh[6][kBlock];
    const int tid = threadIdx.x;
    double r[6] = {INFINITY, INFINITY, INFINITY, -INFINITY, -INFINITY, -INFINITY};
    for (size_t i = (size_t)blockIdx.x * kBlock + tid; i < n; i += (size_t)gridDim.x * kBlock) {
        r[0] = fmin(r[0], lo[3 * i]); r[1] = fmin(r[1], lo[3 * i + 1]); r[2] = fmin(r[2], lo[3 * i + 2]);
        r[3] = fmax(r[3], hi[3 * i]); r[4] = fmax(r[4], hi[3 * i + 1]); r[5] = fmax(r[5], hi[3 * i + 2]);
    }
    for (int k = 0; k < 6; ++k) sh[k][tid] = r[k];
    __syncthreads();
    for (int s = kBlock / 2; s > 0; s >>= 1) {
        if (tid < s) {
            for (int k = 0; k < 3; ++k) sh[k][tid] = fmin(sh[k][tid], sh[k][tid + s]);
            for (int k = 3; k < 6; ++k) sh[k][tid] = fmax(sh[k][tid], sh[k][tid + s]);
        }
        __syncthreads();
    }
    if (tid < 6) out[6 * blockIdx.x + tid] = sh[tid][0];
}

// one block per mesh: box of mesh b over its T primitives -> boxes[6b..6b+5], origin (box centre)
// -> orgs[3b..3b+2]
__global__ __launch_bounds__(kBlock) void k_mesh_boxes(const double* __restrict__ lo, const double* __restrict__ hi,
                                                       size_t T, double* __restrict__ boxes, double* __restrict__ orgs) {
    __shared__ double sh[6][kBlock];
    const int tid = threadIdx.x;
    const size_t base = (size_t)blockIdx.x * T;
    double r[6] = {INFINITY, INFINITY, INFINITY, -INFINITY, -INFINITY, -INFINITY};
    for (size_t i = base + tid; i < base + T; i += kBlock) {
        r[0] = fmin(r[0], lo[3 * i]); r[1] = fmin(r[1], lo[3 * i + 1]); r[2] = fmin(r[2], lo[3 * i + 2]);
        r[3] = fmax(r[3], hi[3 * i]); r[4] = fmax(r[4], hi[3 * i + 1]); r[5] = fmax(r[5], hi[3 * i + 2]);
    }
    for (int k = 0; k < 6; ++k) sh[k][tid] = r[k];
    __syncthreads();
    for (int s = kBlock / 2; s > 0; s >>= 1) {
        if (tid < s) {
            for (int k = 0; k < 3; ++k) sh[k][tid] = fmin(sh[k][tid], sh[k][tid + s]);
            for (int k = 3; k < 6; ++k) sh[k][tid] = fmax(sh[k][tid], sh[k][tid + s]);
        }
        __syncthreads();
    }
    if (tid < 6) boxes[6 * blockIdx.x + tid] = sh[tid][0];
    if (tid < 3) {
        const double c = 0.5 * (sh[tid][0] + sh[3 + tid][0]);
        orgs[3 * blockIdx.x + tid] = (c == c && fabs(c) < INFINITY) ? c : 0.0;
    }
}

__device__ inline uint32_t expand_bits10(uint32_t v) {
    v = (v * 0x00010001u) & 0xFF0000FFu;
    v = (v * 0x00000101u) & 0x0F00F00Fu;
    v = (v * 0x00000011u) & 0xC30C30C3u;
    v = (v * 0x00000005u) & 0x49249249u;
    return v;
}

__device__ inline uint32_t morton30(double x, double y, double z, const double* box) {
    const double ex = box[3] - box[0], ey = box[4] - box[1], ez = box[5] - box[2];
    double nx = ex > 0 ? (x - box[0]) / ex : 0.5, ny = ey > 0 ? (y - box[1]) / ey : 0.5, nz = ez > 0 ? (z - box[2]) / ez : 0.5;
    nx = fmin(fmax(nx * 1024.0, 0.0), 1023.0);
    ny = fmin(fmax(ny * 1024.0, 0.0), 1023.0);
    nz = fmin(fmax(nz * 1024.0, 0.0), 1023.0);
    return (expand_bits10((uint32_t)nx) << 2) | (expand_bits10((uint32_t)ny) << 1) | expand_bits10((uint32_t)nz);
}

__device__ inline uint32_t prim_morton(const double* __restrict__ lo, const double* __restrict__ hi, size_t i,
                                       const double* box) {
    const double cx = 0.5 * (lo[3 * i] + hi[3 * i]);
    const double cy = 0.5 * (lo[3 * i + 1] + hi[3 * i + 1]);
    const double cz = 0.5 * (lo[3 * i + 2] + hi[3 * i + 2]);
    return morton30(cx, cy, cz, box);
}

// key = Morton code of the primitive's box centre in its mesh's box (boxes + 6 * (i / T))
__global__ __launch_bounds__(kBlock) void k_morton(const double* __restrict__ lo, const double* __restrict__ hi, size_t n,
                                                   size_t T, const double* __restrict__ boxes, uint32_t* __restrict__ keys,
                                                   uint32_t* __restrict__ vals) {
    const size_t i = (size_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    keys[i] = prim_morton(lo, hi, i, boxes + 6 * (i / T));
    vals[i] = (uint32_t)i;
}

// batched build, between the two sort phases: key = mesh of the primitive
__global__ __launch_bounds__(kBlock) void k_mesh_key(const uint32_t* __restrict__ vals, size_t n, size_t T,
                                                     uint32_t* __restrict__ keys) {
    const size_t j = (size_t)blockIdx.x * kBlock + threadIdx.x;
    if (j < n) keys[j] = (uint32_t)(vals[j] / T);
}

// batched build, after the sort: Morton codes in sorted order (for node emission)
__global__ __launch_bounds__(kBlock) void k_sorted_morton(const double* __restrict__ lo, const double* __restrict__ hi,
                                                          const uint32_t* __restrict__ vals, size_t n, size_t T,
                                                          const double* __restrict__ boxes, uint32_t* __restrict__ keys) {
    const size_t j = (size_t)blockIdx.x * kBlock + threadIdx.x;
    if (j >= n) return;
    const size_t i = vals[j];
    keys[j] = prim_morton(lo, hi, i, boxes + 6 * (i / T));
}

// delta(i, j): common-prefix length of the augmented keys (code, position)
__device__ inline int lbvh_delta(const uint32_t* __restrict__ k, int n, int i, int j) {
    if (j < 0 || j >= n) return -1;
    const uint32_t a = k[i], b = k[j];
    if (a != b) return __clz(a ^ b);
    return 32 + __clz((uint32_t)i ^ (uint32_t)j);
}

// Mesh b owns internal nodes [b(n-1), (b+1)(n-1)) and leaves [bn, (b+1)n); child references are
// global (internal >= 0, leaf = ~global leaf).  parent[c]: (parent << 1) | side for internal c in
// [0, B(n-1)) and global leaf l at B(n-1) + l.  ranges[g] = (first leaf, last leaf, split gamma, 0),
// global leaf positions: the left child covers [first, gamma].
// node gi of k_karras; returns its depth bound delta(node) - delta(root) + 1
__device__ inline unsigned karras_node(const uint32_t* __restrict__ all_keys, int B, int n, long long gi,
                                       BNode* __restrict__ nodes, uint32_t* __restrict__ parent,
                                       int4* __restrict__ ranges) {
    const int mb = (int)(gi / (n - 1)), i = (int)(gi - (long long)mb * (n - 1));
    const uint32_t* keys = all_keys + (size_t)mb * n;
    const int nb = mb * (n - 1), lb = mb * n;  // node / leaf base of this mesh
    const int d = (lbvh_delta(keys, n, i, i + 1) - lbvh_delta(keys, n, i, i - 1)) >= 0 ? 1 : -1;
    const int dmin = lbvh_delta(keys, n, i, i - d);
    int lmax = 2;
    while (lbvh_delta(keys, n, i, i + lmax * d) > dmin) lmax <<= 1;
    int l = 0;
    for (int t = lmax >> 1; t >= 1; t >>= 1)
        if (lbvh_delta(keys, n, i, i + (l + t) * d) > dmin) l += t;
    const int j = i + l * d;
    const int dnode = lbvh_delta(keys, n, i, j);
    int s = 0, t = l;
    do {
        t = (t + 1) >> 1;
        if (lbvh_delta(keys, n, i, i + (s + t) * d) > dnode) s += t;
    } while (t > 1);
    const int gamma = i + s * d + (d < 0 ? -1 : 0);
    const int lo = min(i, j), hi = max(i, j);
    const int left = (lo == gamma) ? ~(lb + gamma) : nb + gamma;
    const int right = (hi == gamma + 1) ? ~(lb + gamma + 1) : nb + gamma + 1;
    const int g = nb + i;
    float* f = nodes[g].f;
    *reinterpret_cast<float2*>(f + 6) = make_float2(__int_as_float(left), __int_as_float(right));
    ranges[g] = make_int4(lb + lo, lb + hi, lb + gamma, 0);
    const size_t leaf0 = (size_t)B * (n - 1);
    parent[left >= 0 ? (size_t)left : leaf0 + ~left] = ((uint32_t)g << 1) | 0u;
    parent[right >= 0 ? (size_t)right : leaf0 + ~right] = ((uint32_t)g << 1) | 1u;
    return (unsigned)(dnode - lbvh_delta(keys, n, 0, n - 1) + 1);
}

// depth_bound: every step down a Karras tree lengthens the common key prefix (delta) by at least one bit,
// so a leaf below node x lies at most delta(x) - delta(root) + 1 internal nodes deep; the maximum of
// that over the nodes bounds the tree depth (it sizes the traversal stacks' spill areas) without walking
// every leaf to its root (C4: 7.3 ms of dependent parent loads for 41M leaves).
__global__ __launch_bounds__(kBlock) void k_karras(const uint32_t* __restrict__ all_keys, int B, int n,
                                                   BNode* __restrict__ nodes, uint32_t* __restrict__ parent,
                                                   int4* __restrict__ ranges, unsigned* __restrict__ depth_bound) {
    const long long gi = (long long)blockIdx.x * kBlock + threadIdx.x;
    unsigned dep = 0;
    if (gi < (long long)B * (n - 1)) dep = karras_node(all_keys, B, n, gi, nodes, parent, ranges);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) dep = max(dep, (unsigned)__shfl_xor((int)dep, o, 64));
    if ((threadIdx.x & 63) == 0 && dep > 0) atomicMax(depth_bound, dep);
}


__device__ inline float down1(float x) { return nextafterf(x, -INFINITY); }
__device__ inline float up1(float x) { return nextafterf(x, INFINITY); }
__device__ inline float out_lo(double x) { return down1(__double2float_rd(x)); }
__device__ inline float out_hi(double x) { return up1(__double2float_ru(x)); }

// depth of every leaf (root's children = 1); out = max
// ---- oriented boxes: one wave per internal node ----
__device__ inline double wsum(double x) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) x += __shfl_xor(x, o, 64);
    return x;
}
__device__ inline double wmin(double x) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) x = fmin(x, __shfl_xor(x, o, 64));
    return x;
}
__device__ inline double wmax(double x) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) x = fmax(x, __shfl_xor(x, o, 64));
    return x;
}

template <bool TRI>
__device__ inline int leaf_points(const void* leaves, int i, D3* p) {
    if (TRI) {
        uint32_t face;
        load_tri(static_cast<const TriRec*>(leaves), i, p[0], p[1], p[2], face);
        return 3;
    }
    const PtRec& r = static_cast<const PtRec*>(leaves)[i];
    p[0] = D3{r.x, r.y, r.z};
    return 1;
}

// Node frame from the area-weighted normal sum (sx, sy, sz): n, t = e - (e.n) n normalised (e the x or y
// axis), b = n x t in fp32; A = the fp32 axes widened to fp64 (what the vertices are projected on).
struct ObbFrame {
    float n[3], t[3], b[3];
    double A[3][3];
};
// sa = the sum of the area vectors' lengths: a node whose normals cancel (|s| <= 1e-6 sa: a closed surface,
// e.g. the root of a sphere) has no meaningful normal, and its rounding-noise direction would give its
// children arbitrarily tilted boxes; it takes the axis frame (n = x) instead.
__device__ inline ObbFrame obb_frame(double sx, double sy, double sz, double sa) {
    const double len = sqrt(sx * sx + sy * sy + sz * sz);
    const D3 n = (len > 1e-6 * sa && len < INFINITY) ? D3{sx / len, sy / len, sz / len} : D3{1.0, 0.0, 0.0};
    const D3 e = fabs(n.x) < 0.9 ? D3{1.0, 0.0, 0.0} : D3{0.0, 1.0, 0.0};
    D3 t = vsub(e, vscale(vdot(e, n), n));
    const double tl = sqrt(vdot(t, t));
    t = D3{t.x / tl, t.y / tl, t.z / tl};
    ObbFrame f;
    f.n[0] = (float)n.x; f.n[1] = (float)n.y; f.n[2] = (float)n.z;
    f.t[0] = (float)t.x; f.t[1] = (float)t.y; f.t[2] = (float)t.z;
    frame_b(f.n, f.t, f.b);
    for (int k = 0; k < 3; ++k) {
        f.A[0][k] = f.n[k];
        f.A[1][k] = f.t[k];
        f.A[2][k] = f.b[k];
    }
    return f;
}

// area vector (p1 - p0) x (p2 - p0) of leaf i (points: none)
template <bool TRI>
__device__ inline D3 leaf_area(const void* leaves, int i) {
    if (!TRI) return D3{0.0, 0.0, 0.0};
    D3 p[3];
    leaf_points<TRI>(leaves, i, p);
    return vcross(vsub(p[1], p[0]), vsub(p[2], p[0]));
}

// min / max projections onto the frame of leaf i's points (relative to the origin o)
template <bool TRI>
__device__ inline void leaf_extent(const void* leaves, int i, const ObbFrame& f, const double* o, double* mn, double* mx) {
    D3 p[3];
    const int np = leaf_points<TRI>(leaves, i, p);
    for (int c = 0; c < np; ++c) {
        const double rx = p[c].x - o[0], ry = p[c].y - o[1], rz = p[c].z - o[2];
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            const double pr = f.A[k][0] * rx + f.A[k][1] * ry + f.A[k][2] * rz;
            mn[k] = fmin(mn[k], pr);
            mx[k] = fmax(mx[k], pr);
        }
    }
}

// Write node: frame, and both children's fp32 extents ext[side][lo n t b, hi n t b] quantised against
// base = min lower bound with a bf16 scale per axis (bf16_scale_up: >= range / 254); lower codes round down
// and upper codes up, checked with the decoder's own expression, so the decoded box contains the fp32 one.
__device__ inline void encode_node(BNode* node, const ObbFrame& fr, const float (*ext)[6]) {
    float* f = node->f;
    float base[3], scs[3];
    uint32_t u[12];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        base[k] = fminf(ext[0][k], ext[1][k]);
        const double top = fmax((double)ext[0][3 + k], (double)ext[1][3 + k]);
        const float sc = bf16_scale_up(top - (double)base[k]);
        scs[k] = sc;
#pragma unroll
        for (int side = 0; side < 2; ++side) {
            const float lo = ext[side][k], hi = ext[side][3 + k];
            const double ql = floor(((double)lo - (double)base[k]) / (double)sc);
            const double qh = ceil(((double)hi - (double)base[k]) / (double)sc);
            uint32_t ul = (uint32_t)fmin(fmax(ql, 0.0), 255.0), uh = (uint32_t)fmin(fmax(qh, 0.0), 255.0);
            while (ul > 0u && dequant(ul, sc, base[k]) > lo) --ul;
            while (uh < 255u && dequant(uh, sc, base[k]) < hi) ++uh;
            u[6 * side + k] = ul;
            u[6 * side + 3 + k] = uh;
        }
    }
    uint32_t w[3];
#pragma unroll
    for (int j = 0; j < 3; ++j) w[j] = u[4 * j] | (u[4 * j + 1] << 8) | (u[4 * j + 2] << 16) | (u[4 * j + 3] << 24);
    float h[16];
    encode_frame(h, fr.n, fr.t);
    encode_scales(h, scs);
    *reinterpret_cast<float4*>(f) = make_float4(h[0], h[1], h[2], h[3]);
    *reinterpret_cast<float2*>(f + 4) = make_float2(h[4], h[5]);
    *reinterpret_cast<float4*>(f + 8) = make_float4(base[0], base[1], base[2], __uint_as_float(w[0]));
    *reinterpret_cast<float4*>(f + 12) = make_float4(__uint_as_float(w[1]), __uint_as_float(w[2]), h[14], h[15]);
}

// ---- area prefix sums: a node's frame needs the area-weighted normal sum over its Morton leaf range,
// which is P[last + 1] - P[first] for the exclusive prefix P of the leaves' (area vector, |area|) in
// leaf order — one O(T) scan instead of a pass over every node's range (O(T log T) leaf reads).  The scan
// is two-level with a fixed association (deterministic); the differences lose ~1e-16 |P| to
// cancellation, far below what the fp32 frame keeps.
constexpr int kScanPer = 8;                      // leaves per thread
constexpr int kScanBlock = kBlock * kScanPer;    // leaves per block
__device__ inline double4 d4add(const double4& a, const double4& b) {
    return make_double4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
}
// exclusive block scan of one double4 per thread (fixed order: wave inclusive shuffles, then wave totals)
__device__ inline double4 block_exscan(double4 v, double4* sh, double4& total) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    double4 inc = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const double4 u = make_double4(__shfl_up(inc.x, o, 64), __shfl_up(inc.y, o, 64), __shfl_up(inc.z, o, 64),
                                       __shfl_up(inc.w, o, 64));
        if (lane >= o) inc = d4add(inc, u);
    }
    if (lane == 63) sh[w] = inc;
    __syncthreads();
    double4 off = make_double4(0, 0, 0, 0);
    for (int k = 0; k < w; ++k) off = d4add(off, sh[k]);
    total = d4add(d4add(d4add(sh[0], sh[1]), sh[2]), sh[3]);
    __syncthreads();
    return d4add(off, make_double4(inc.x - v.x, inc.y - v.y, inc.z - v.z, inc.w - v.w));
}
template <bool TRI>
__device__ inline double4 leaf_area4(const void* leaves, int i) {
    const D3 a = leaf_area<TRI>(leaves, i);
    return make_double4(a.x, a.y, a.z, sqrt(vdot(a, a)));
}
// block-local inclusive prefixes P[i + 1] of the block's leaves, and the block total
template <bool TRI>
__global__ __launch_bounds__(kBlock) void k_area_scan(const void* __restrict__ leaves, int n, double4* __restrict__ P,
                                                      double4* __restrict__ btot) {
    __shared__ double4 sh[4];
    const int base = blockIdx.x * kScanBlock + threadIdx.x * kScanPer;
    double4 loc[kScanPer];
    double4 run = make_double4(0, 0, 0, 0);
#pragma unroll
    for (int k = 0; k < kScanPer; ++k) {
        const int i = base + k;
        if (i < n) run = d4add(run, leaf_area4<TRI>(leaves, i));
        loc[k] = run;
    }
    double4 total;
    const double4 off = block_exscan(run, sh, total);
#pragma unroll
    for (int k = 0; k < kScanPer; ++k)
        if (base + k < n) P[base + k + 1] = d4add(off, loc[k]);
    if (threadIdx.x == 0) btot[blockIdx.x] = total;
}
// exclusive scan of the block totals in place (one block, each thread a contiguous run)
__global__ __launch_bounds__(kBlock) void k_area_scan_tops(double4* __restrict__ btot, int nb) {
    __shared__ double4 sh[4];
    const int per = (nb + kBlock - 1) / kBlock, b0 = threadIdx.x * per, b1 = min(nb, b0 + per);
    double4 run = make_double4(0, 0, 0, 0);
    for (int b = b0; b < b1; ++b) run = d4add(run, btot[b]);
    double4 total;
    double4 off = block_exscan(run, sh, total);
    for (int b = b0; b < b1; ++b) {
        const double4 t = btot[b];
        btot[b] = off;
        off = d4add(off, t);
    }
}
__global__ __launch_bounds__(kBlock) void k_area_scan_add(double4* __restrict__ P, int n, const double4* __restrict__ btot) {
    const int i = blockIdx.x * kBlock + threadIdx.x;
    if (i == 0) P[0] = make_double4(0, 0, 0, 0);
    if (i >= n) return;
    P[i + 1] = d4add(btot[i / kScanBlock], P[i + 1]);
}
// the frame of the leaf range [first, last]
__device__ inline ObbFrame range_frame(const double4* __restrict__ P, int first, int last) {
    const double4 a = P[last + 1], b = P[first];
    return obb_frame(a.x - b.x, a.y - b.y, a.z - b.z, a.w - b.w);
}

constexpr int kObbLane = 32;    // nodes over at most this many leaves: one lane each; up to kObbBig: one wave each
constexpr int kObbBig = 4096;  // larger nodes (the top levels): kObbChunk-leaf chunks, one block per chunk
constexpr int kObbChunk = 1024;

// Oriented boxes of nodes over at most kObbLane leaves, one lane per node (most nodes: the lower levels)
template <bool TRI>
__global__ __launch_bounds__(kBlock) void k_obb_lane(const void* __restrict__ leaves, const int4* __restrict__ ranges,
                                                     int nn, int npm, BNode* __restrict__ nodes,
                                                     const double* __restrict__ orgs, const double4* __restrict__ P) {
    const int node = blockIdx.x * kBlock + threadIdx.x;
    if (node >= nn) return;
    const int4 r = ranges[node];
    if (r.y - r.x + 1 > kObbLane) return;
    const int mb = node / npm;  // mesh of the node (npm internal nodes per mesh)
    const double o[3] = {orgs[3 * mb], orgs[3 * mb + 1], orgs[3 * mb + 2]};
    const ObbFrame fr = range_frame(P, r.x, r.y);
    float ext[2][6];
    for (int side = 0; side < 2; ++side) {
        double mn[3] = {INFINITY, INFINITY, INFINITY}, mx[3] = {-INFINITY, -INFINITY, -INFINITY};
        const int b = side == 0 ? r.x : r.z + 1, e = side == 0 ? r.z : r.y;
        for (int i = b; i <= e; ++i) leaf_extent<TRI>(leaves, i, fr, o, mn, mx);
        for (int k = 0; k < 3; ++k) {
            ext[side][k] = out_lo(mn[k]);
            ext[side][3 + k] = out_hi(mx[k]);
        }
    }
    encode_node(nodes + node, fr, ext);
}

// Oriented boxes of nodes over more than kObbLane leaves, one wave per node over its Morton leaf range
template <bool TRI>
__global__ __launch_bounds__(kBlock) void k_obb_wave(const void* __restrict__ leaves, const int4* __restrict__ ranges,
                                                     int nn, int npm, BNode* __restrict__ nodes,
                                                     const double* __restrict__ orgs, int maxr,
                                                     const double4* __restrict__ P) {
    const int lane = threadIdx.x & 63;
    const int waves = gridDim.x * (kBlock / 64);
    for (int node = (blockIdx.x * kBlock + threadIdx.x) >> 6; node < nn; node += waves) {
        const int4 r = ranges[node];
        if (r.y - r.x + 1 <= kObbLane || r.y - r.x + 1 > maxr) continue;
        const int mb = node / npm;
        const double o[3] = {orgs[3 * mb], orgs[3 * mb + 1], orgs[3 * mb + 2]};
        const ObbFrame fr = range_frame(P, r.x, r.y);
        float ext[2][6];
#pragma unroll
        for (int side = 0; side < 2; ++side) {
            double mn[3] = {INFINITY, INFINITY, INFINITY}, mx[3] = {-INFINITY, -INFINITY, -INFINITY};
            const int b = side == 0 ? r.x : r.z + 1, e = side == 0 ? r.z : r.y;
            for (int i = b + lane; i <= e; i += 64) leaf_extent<TRI>(leaves, i, fr, o, mn, mx);
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                ext[side][k] = out_lo(wmin(mn[k]));
                ext[side][3 + k] = out_hi(wmax(mx[k]));
            }
        }
        if (lane == 0) encode_node(nodes + node, fr, ext);
    }
}

// ---- nodes over more than kObbBig leaves: one wave per node would leave the root's wave walking T leaves
// alone (C5, 5M faces: 85 ms).  Their ranges are cut into kObbChunk-leaf chunks, one block per chunk; the
// partial area sums are added in chunk order (deterministic) into the frame, the partial extents are
// min / max-reduced, and the node is encoded as k_obb_wave would.
__global__ __launch_bounds__(kBlock) void k_big_count(const int4* __restrict__ ranges, int nn, unsigned* __restrict__ count) {
    const int node = blockIdx.x * kBlock + threadIdx.x;
    bool big = false;
    if (node < nn) {
        const int4 r = ranges[node];
        big = r.y - r.x + 1 > kObbBig;
    }
    const unsigned long long m = __ballot(big);
    if ((threadIdx.x & 63) == 0 && m) atomicAdd(count, (unsigned)__popcll(m));
}
__global__ __launch_bounds__(kBlock) void k_big_nodes(const int4* __restrict__ ranges, int nn, int* __restrict__ list,
                                                      int4* __restrict__ lr, unsigned* __restrict__ count) {
    const int node = blockIdx.x * kBlock + threadIdx.x;
    if (node >= nn) return;
    const int4 r = ranges[node];
    if (r.y - r.x + 1 <= kObbBig) return;
    const unsigned k = atomicAdd(count, 1u);
    list[k] = node;
    lr[k] = r;
}

// block reduction in a fixed order (waves, then the 4 wave results in order)
__device__ inline double block_sum(double x, double* sh) {
    x = wsum(x);
    __syncthreads();
    if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = x;
    __syncthreads();
    return ((sh[0] + sh[1]) + sh[2]) + sh[3];
}
__device__ inline double block_min(double x, double* sh) {
    x = wmin(x);
    __syncthreads();
    if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = x;
    __syncthreads();
    return fmin(fmin(sh[0], sh[1]), fmin(sh[2], sh[3]));
}
__device__ inline double block_max(double x, double* sh) {
    x = wmax(x);
    __syncthreads();
    if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = x;
    __syncthreads();
    return fmax(fmax(sh[0], sh[1]), fmax(sh[2], sh[3]));
}

// one thread per big node: its frame
__global__ __launch_bounds__(kBlock) void k_big_frame(int nbig, const int4* __restrict__ lr, const double4* __restrict__ P,
                                                      ObbFrame* __restrict__ frames) {
    const int b = blockIdx.x * kBlock + threadIdx.x;
    if (b >= nbig) return;
    frames[b] = range_frame(P, lr[b].x, lr[b].y);
}

// partial extents of a chunk on its node's frame, per side of the node's split: ext[item][side][lo k, hi k]
template <bool TRI>
__global__ __launch_bounds__(kBlock) void k_big_extent(const void* __restrict__ leaves, const int* __restrict__ list,
                                                       const int4* __restrict__ lr, const int2* __restrict__ items,
                                                       const ObbFrame* __restrict__ frames, int npm,
                                                       const double* __restrict__ orgs, double* __restrict__ ext) {
    __shared__ double sh[4];
    const int2 it = items[blockIdx.x];
    const int4 r = lr[it.x];
    const ObbFrame fr = frames[it.x];
    const int mb = list[it.x] / npm;
    const double o[3] = {orgs[3 * mb], orgs[3 * mb + 1], orgs[3 * mb + 2]};
    const int b = r.x + it.y * kObbChunk, e = min(r.y, b + kObbChunk - 1);
    double mn[2][3], mx[2][3];
#pragma unroll
    for (int side = 0; side < 2; ++side)
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            mn[side][k] = INFINITY;
            mx[side][k] = -INFINITY;
        }
    for (int i = b + (int)threadIdx.x; i <= e; i += kBlock) {
        if (i <= r.z) leaf_extent<TRI>(leaves, i, fr, o, mn[0], mx[0]);
        else leaf_extent<TRI>(leaves, i, fr, o, mn[1], mx[1]);
    }
    double* out = ext + 12 * (size_t)blockIdx.x;
#pragma unroll
    for (int side = 0; side < 2; ++side)
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            const double lo = block_min(mn[side][k], sh);
            const double hi = block_max(mx[side][k], sh);
            if (threadIdx.x == 0) {
                out[6 * side + k] = lo;
                out[6 * side + 3 + k] = hi;
            }
        }
}

// one thread per big node: reduce its chunks' extents and encode the node
__global__ __launch_bounds__(kBlock) void k_big_encode(int nbig, const int* __restrict__ list, const int* __restrict__ off,
                                                       const ObbFrame* __restrict__ frames, const double* __restrict__ ext,
                                                       BNode* __restrict__ nodes) {
    const int b = blockIdx.x * kBlock + threadIdx.x;
    if (b >= nbig) return;
    double m[12];
#pragma unroll
    for (int j = 0; j < 12; ++j) m[j] = (j % 6) < 3 ? INFINITY : -INFINITY;
    for (int k = off[b]; k < off[b + 1]; ++k)
#pragma unroll
        for (int j = 0; j < 12; ++j) m[j] = (j % 6) < 3 ? fmin(m[j], ext[12 * (size_t)k + j]) : fmax(m[j], ext[12 * (size_t)k + j]);
    float e[2][6];
#pragma unroll
    for (int side = 0; side < 2; ++side)
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            e[side][k] = out_lo(m[6 * side + k]);
            e[side][3 + k] = out_hi(m[6 * side + 3 + k]);
        }
    encode_node(nodes + list[b], frames[b], e);
}

// leaf k holds primitive order[k] = b*T + t of mesh b; its face id is the mesh-local t (+ face_base)
__global__ __launch_bounds__(kBlock) void k_pack_tris(const double* __restrict__ v, size_t P, const uint32_t* __restrict__ f,
                                                      const uint32_t* __restrict__ order, size_t n, size_t T,
                                                      uint32_t face_base, TriRec* __restrict__ out) {
    const size_t k = (size_t)blockIdx.x * kBlock + threadIdx.x;
    if (k >= n) return;
    const size_t g = order[k], b = g / T, t = g - b * T;
    const double* vb = v + 3 * P * b;
    TriRec r;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        const size_t vi = f[3 * t + c];
        r.v[3 * c] = vb[3 * vi];
        r.v[3 * c + 1] = vb[3 * vi + 1];
        r.v[3 * c + 2] = vb[3 * vi + 2];
    }
    r.face = (uint32_t)t + face_base;
    r.pad = 0;
    out[k] = r;
}

__global__ __launch_bounds__(kBlock) void k_pack_points(const double* __restrict__ v, const uint32_t* __restrict__ order,
                                                        size_t P, PtRec* __restrict__ out) {
    const size_t k = (size_t)blockIdx.x * kBlock + threadIdx.x;
    if (k >= P) return;
    const uint32_t i = order[k];
    PtRec r;
    r.x = v[3 * (size_t)i];
    r.y = v[3 * (size_t)i + 1];
    r.z = v[3 * (size_t)i + 2];
    r.idx = i;
    r.pad = 0;
    out[k] = r;
}

static unsigned nblocks(size_t n) { return (unsigned)((n + kBlock - 1) / kBlock); }

int tri_bounds(const double* d_v, const uint32_t* d_f, size_t T, double* d_lo, double* d_hi, hipStream_t s) {
    k_tri_bounds<<<nblocks(T), kBlock, 0, s>>>(d_v, 0, d_f, T, T, d_lo, d_hi);
    MSH_HIP(hipGetLastError());
    return MSH_OK;
}

int point_bounds(const double* d_v, size_t P, double* d_lo, double* d_hi, hipStream_t s) {
    k_point_bounds<<<nblocks(3 * P), kBlock, 0, s>>>(d_v, P, d_lo, d_hi);
    MSH_HIP(hipGetLastError());
    return MSH_OK;
}

int pack_tri_leaves(const double* d_v, const uint32_t* d_f, const uint32_t* d_order, size_t T, uint32_t face_base,
                    TriRec* d_out, hipStream_t s) {
    k_pack_tris<<<nblocks(T), kBlock, 0, s>>>(d_v, 0, d_f, d_order, T, T, face_base, d_out);
    MSH_HIP(hipGetLastError());
    return MSH_OK;
}

int pack_point_leaves(const double* d_v, const uint32_t* d_order, size_t P, PtRec* d_out, hipStream_t s) {
    k_pack_points<<<nblocks(P), kBlock, 0, s>>>(d_v, d_order, P, d_out);
    MSH_HIP(hipGetLastError());
    return MSH_OK;
}

// nodes over more than kObbBig leaves (k_big_*): list them, cut their ranges into chunks (host-side item
// map, a few thousand entries), then partial sums / frames / partial extents / encode
static int build_obb_big(msh_tree* tree, bool triangles, const int4* ranges, int nn, int npm, hipStream_t s,
                         int& maxr, const double4* P) {
    // meshes of up to 4 kObbBig faces: their largest nodes are short work for one wave, and the list /
    // item set-up (a few allocations and host round trips) would cost more (C2: 1.7 -> 2.5 ms)
    if (tree->T <= 4 * (size_t)kObbBig) return MSH_OK;
    struct Tmp {
        void* p = nullptr;
        ~Tmp() { if (p) (void)dfree(p); }
    } t_list, t_lr, t_cnt, t_items, t_off, t_frames, t_ext;
    const unsigned nblk = (unsigned)(((size_t)nn + kBlock - 1) / kBlock);
    MSH_HIP(dmalloc(&t_cnt.p, sizeof(unsigned)));
    MSH_HIP(hipMemsetAsync(t_cnt.p, 0, sizeof(unsigned), s));
    k_big_count<<<nblk, kBlock, 0, s>>>(ranges, nn, static_cast<unsigned*>(t_cnt.p));
    MSH_HIP(hipGetLastError());
    unsigned nbig = 0;
    MSH_HIP(hipMemcpyAsync(&nbig, t_cnt.p, sizeof(unsigned), hipMemcpyDeviceToHost, s));
    MSH_HIP(hipStreamSynchronize(s));
    if (nbig == 0) return MSH_OK;
    MSH_HIP(dmalloc(&t_list.p, (size_t)nbig * sizeof(int)));
    MSH_HIP(dmalloc(&t_lr.p, (size_t)nbig * sizeof(int4)));
    MSH_HIP(hipMemsetAsync(t_cnt.p, 0, sizeof(unsigned), s));
    k_big_nodes<<<nblk, kBlock, 0, s>>>(ranges, nn, static_cast<int*>(t_list.p), static_cast<int4*>(t_lr.p),
                                        static_cast<unsigned*>(t_cnt.p));
    MSH_HIP(hipGetLastError());
    std::vector<int> list(nbig);
    std::vector<int4> lr(nbig);
    MSH_HIP(hipMemcpyAsync(list.data(), t_list.p, nbig * sizeof(int), hipMemcpyDeviceToHost, s));
    MSH_HIP(hipMemcpyAsync(lr.data(), t_lr.p, nbig * sizeof(int4), hipMemcpyDeviceToHost, s));
    MSH_HIP(hipStreamSynchronize(s));
    // node order (the atomic list order is arbitrary), chunk items per node
    std::vector<int> idx(nbig);
    for (unsigned b = 0; b < nbig; ++b) idx[b] = (int)b;
    std::sort(idx.begin(), idx.end(), [&](int x, int y) { return list[x] < list[y]; });
    std::vector<int> slist(nbig), off(nbig + 1, 0);
    std::vector<int4> slr(nbig);
    std::vector<int2> items;
    for (unsigned j = 0; j < nbig; ++j) {
        slist[j] = list[idx[j]];
        slr[j] = lr[idx[j]];
        const int n = slr[j].y - slr[j].x + 1;
        const int nch = (n + kObbChunk - 1) / kObbChunk;
        for (int c = 0; c < nch; ++c) items.push_back(make_int2((int)j, c));
        off[j + 1] = (int)items.size();
    }
    const size_t ni = items.size();
    // a degenerate (caterpillar-like) tree has O(T^2 / kObbChunk) items: leave its big nodes to k_obb_wave
    if (ni > ((size_t)1 << 22)) return MSH_OK;
    MSH_HIP(dmalloc(&t_items.p, ni * sizeof(int2)));
    MSH_HIP(dmalloc(&t_off.p, (nbig + 1) * sizeof(int)));
    MSH_HIP(dmalloc(&t_frames.p, nbig * sizeof(ObbFrame)));
    MSH_HIP(dmalloc(&t_ext.p, ni * 12 * sizeof(double)));
    MSH_HIP(hipMemcpyAsync(t_list.p, slist.data(), nbig * sizeof(int), hipMemcpyHostToDevice, s));
    MSH_HIP(hipMemcpyAsync(t_lr.p, slr.data(), nbig * sizeof(int4), hipMemcpyHostToDevice, s));
    MSH_HIP(hipMemcpyAsync(t_items.p, items.data(), ni * sizeof(int2), hipMemcpyHostToDevice, s));
    MSH_HIP(hipMemcpyAsync(t_off.p, off.data(), (nbig + 1) * sizeof(int), hipMemcpyHostToDevice, s));
    const int* d_list = static_cast<const int*>(t_list.p);
    const int4* d_lr = static_cast<const int4*>(t_lr.p);
    const int2* d_items = static_cast<const int2*>(t_items.p);
    const int* d_off = static_cast<const int*>(t_off.p);
    ObbFrame* d_frames = static_cast<ObbFrame*>(t_frames.p);
    double* d_ext = static_cast<double*>(t_ext.p);
    const unsigned nb = (nbig + kBlock - 1) / kBlock;
    k_big_frame<<<nb, kBlock, 0, s>>>((int)nbig, d_lr, P, d_frames);
    if (triangles) {
        k_big_extent<true><<<(unsigned)ni, kBlock, 0, s>>>(tree->d_leaves, d_list, d_lr, d_items, d_frames, npm,
                                                          tree->d_orgs, d_ext);
    } else {
        k_big_extent<false><<<(unsigned)ni, kBlock, 0, s>>>(tree->d_leaves, d_list, d_lr, d_items, d_frames, npm,
                                                           tree->d_orgs, d_ext);
    }
    k_big_encode<<<nb, kBlock, 0, s>>>((int)nbig, d_list, d_off, d_frames, d_ext, tree->d_nodes);
    MSH_HIP(hipGetLastError());
    MSH_HIP(hipStreamSynchronize(s));  // the temporaries are freed on return
    maxr = kObbBig;
    return MSH_OK;
}

int build_obb(msh_tree* tree, bool triangles, bool defer) {
    if (tree->T < 2) return MSH_OK;
    const int nn = (int)(tree->B * (tree->T - 1));
    const int nl = (int)(tree->B * tree->T);
    const unsigned blocks = (unsigned)std::min<size_t>(((size_t)nn + 3) / 4, 65536);
    hipStream_t s = tree->stream;
    const int4* ranges = tree->ws.ranges.as<int4>();
    const int npm = (int)(tree->T - 1);  // internal nodes per mesh
    const unsigned lane_blocks = (unsigned)(((size_t)nn + kBlock - 1) / kBlock);
    // area prefix sums over all leaves (batched trees: the meshes' leaf ranges are disjoint)
    struct Tmp {
        void* p = nullptr;
        ~Tmp() { if (p) (void)dfree(p); }
    } t_P, t_tot;
    const int nsb = (nl + kScanBlock - 1) / kScanBlock;
    MSH_HIP(dmalloc(&t_P.p, ((size_t)nl + 1) * sizeof(double4)));
    MSH_HIP(dmalloc(&t_tot.p, (size_t)nsb * sizeof(double4)));
    double4* P = static_cast<double4*>(t_P.p);
    double4* tot = static_cast<double4*>(t_tot.p);
    if (triangles) k_area_scan<true><<<(unsigned)nsb, kBlock, 0, s>>>(tree->d_leaves, nl, P, tot);
    else k_area_scan<false><<<(unsigned)nsb, kBlock, 0, s>>>(tree->d_leaves, nl, P, tot);
    k_area_scan_tops<<<1, kBlock, 0, s>>>(tot, nsb);
    k_area_scan_add<<<(unsigned)(((size_t)nl + kBlock - 1) / kBlock), kBlock, 0, s>>>(P, nl, tot);
    MSH_HIP(hipGetLastError());
    int maxr = 0x7fffffff;
    if (triangles) {
        k_obb_lane<true><<<lane_blocks, kBlock, 0, s>>>(tree->d_leaves, ranges, nn, npm, tree->d_nodes, tree->d_orgs, P);
    } else {
        k_obb_lane<false><<<lane_blocks, kBlock, 0, s>>>(tree->d_leaves, ranges, nn, npm, tree->d_nodes, tree->d_orgs, P);
    }
    MSH_HIP(hipGetLastError());
    MSH_TRY(build_obb_big(tree, triangles, ranges, nn, npm, s, maxr, P));
    if (triangles) {
        k_obb_wave<true><<<blocks, kBlock, 0, s>>>(tree->d_leaves, ranges, nn, npm, tree->d_nodes, tree->d_orgs, maxr, P);
    } else {
        k_obb_wave<false><<<blocks, kBlock, 0, s>>>(tree->d_leaves, ranges, nn, npm, tree->d_nodes, tree->d_orgs, maxr, P);
    }
    MSH_HIP(hipGetLastError());
    if (defer) {  // freed by finish_pending once the build's last kernel has passed
        tree->pend_free.push_back(t_P.p);
        tree->pend_free.push_back(t_tot.p);
        t_P.p = t_tot.p = nullptr;
        return MSH_OK;
    }
    MSH_HIP(hipStreamSynchronize(s));  // P is freed on return
    return MSH_OK;
}

// device copy of the single-mesh origin (kernels read per-mesh origins from tree->d_orgs)
int upload_origin(msh_tree* tree, hipStream_t s) {
    if (!tree->d_orgs) MSH_HIP(dmalloc(&tree->d_orgs, 3 * sizeof(double)));
    MSH_HIP(hipMemcpyAsync(tree->d_orgs, tree->origin, 3 * sizeof(double), hipMemcpyHostToDevice, s));
    return MSH_OK;
}

int build_lbvh(msh_tree* tree, const double* d_lo, const double* d_hi, size_t T, uint32_t* d_order) {
    hipStream_t s = tree->stream;
    Workspace& ws = tree->ws;
    if (T > (size_t)0x7FFFFFFF) {
        set_error("LBVH build: %zu primitives exceed the 31-bit node index range", T);
        return MSH_EINVAL;
    }
    // scene box
    const unsigned rb = (unsigned)std::min<size_t>(1024, std::max<size_t>(1, (T + kBlock - 1) / kBlock));
    MSH_TRY(ws.flags.reserve(std::max<size_t>((size_t)(rb + 1) * 6 * sizeof(double), T * sizeof(uint32_t) + 64)));
    double* part = ws.flags.as<double>();
    k_reduce_box<<<rb, kBlock, 0, s>>>(d_lo, d_hi, T, part);
    MSH_HIP(hipGetLastError());
    DevBuf box;  // released at the end of the build (after its final stream sync)
    struct Rel { DevBuf& b; ~Rel() { b.release(); } } rel{box};
    MSH_TRY(box.reserve(6 * sizeof(double)));
    double* d_box = box.as<double>();
    double box_h[6];
    {
        // at most 1024 partial boxes: fetch and combine them on the host (the build syncs anyway
        // to learn the scene box used by query Morton codes)
        std::unique_ptr<double[]> hp(new double[6 * rb]);
        MSH_HIP(hipMemcpyAsync(hp.get(), part, 6 * rb * sizeof(double), hipMemcpyDeviceToHost, s));
        MSH_HIP(hipStreamSynchronize(s));
        for (int k = 0; k < 3; ++k) { box_h[k] = INFINITY; box_h[3 + k] = -INFINITY; }
        for (unsigned b = 0; b < rb; ++b)
            for (int k = 0; k < 3; ++k) {
                box_h[k] = std::min(box_h[k], hp[6 * b + k]);
                box_h[3 + k] = std::max(box_h[3 + k], hp[6 * b + 3 + k]);
            }
        MSH_HIP(hipMemcpyAsync(d_box, box_h, sizeof(box_h), hipMemcpyHostToDevice, s));
    }
    for (int k = 0; k < 3; ++k) {
        tree->scene_lo[k] = (float)box_h[k];
        tree->scene_hi[k] = (float)box_h[3 + k];
        const double c = 0.5 * (box_h[k] + box_h[3 + k]);
        tree->origin[k] = (c == c && fabs(c) < INFINITY) ? c : 0.0;
    }
    tree->half_diag = half_diagonal(box_h, tree->origin);
    MSH_TRY(upload_origin(tree, s));
    // Morton codes + sort
    MSH_TRY(ws.keys.reserve(T * sizeof(uint32_t)));
    MSH_TRY(ws.keys_alt.reserve(T * sizeof(uint32_t)));
    MSH_TRY(ws.vals_alt.reserve(T * sizeof(uint32_t)));
    uint32_t* keys = ws.keys.as<uint32_t>();
    k_morton<<<nblocks(T), kBlock, 0, s>>>(d_lo, d_hi, T, T, d_box, keys, d_order);
    MSH_HIP(hipGetLastError());
    MSH_TRY(radix_sort_pairs(keys, d_order, ws.keys_alt.as<uint32_t>(), ws.vals_alt.as<uint32_t>(), T, 30, ws, s));
    tree->max_depth = 0;
    if (T < 2) {
        MSH_HIP(hipStreamSynchronize(s));
        return MSH_OK;
    }
    // Karras emission
    MSH_TRY(ws.vals.reserve((2 * T - 1) * sizeof(uint32_t)));
    MSH_TRY(ws.ranges.reserve((T - 1) * sizeof(int4)));
    uint32_t* parent = ws.vals.as<uint32_t>();
    // node bounds come from k_obb (build_obb), after the leaves are packed
    uint32_t* flags = ws.flags.as<uint32_t>();
    unsigned* d_depth = flags + T;
    MSH_HIP(hipMemsetAsync(d_depth, 0, sizeof(unsigned), s));
    k_karras<<<nblocks(T - 1), kBlock, 0, s>>>(keys, 1, (int)T, tree->d_nodes, parent, ws.ranges.as<int4>(), d_depth);
    MSH_HIP(hipGetLastError());
    unsigned depth = 0;
    MSH_HIP(hipMemcpyAsync(&depth, d_depth, sizeof(unsigned), hipMemcpyDeviceToHost, s));
    MSH_HIP(hipStreamSynchronize(s));
    tree->max_depth = (int)depth;
    return MSH_OK;
}


// ---- batched build (C4: many meshes sharing one topology) ----
int tri_bounds_batch(const double* d_v, size_t P, const uint32_t* d_f, size_t B, size_t T, double* d_lo, double* d_hi,
                     hipStream_t s) {
    k_tri_bounds<<<nblocks(B * T), kBlock, 0, s>>>(d_v, P, d_f, B * T, T, d_lo, d_hi);
    MSH_HIP(hipGetLastError());
    return MSH_OK;
}

int pack_tri_leaves_batch(const double* d_v, size_t P, const uint32_t* d_f, const uint32_t* d_order, size_t B, size_t T,
                          TriRec* d_out, hipStream_t s) {
    k_pack_tris<<<nblocks(B * T), kBlock, 0, s>>>(d_v, P, d_f, d_order, B * T, T, 0u, d_out);
    MSH_HIP(hipGetLastError());
    return MSH_OK;
}

static int bits_for(size_t n) {  // bits needed for values in [0, n)
    int b = 0;
    while (b < 32 && ((size_t)1 << b) < n) ++b;
    return b;
}

int build_lbvh_batch(msh_tree* tree, const double* d_lo, const double* d_hi, size_t T, uint32_t* d_order) {
    hipStream_t s = tree->stream;
    Workspace& ws = tree->ws;
    const size_t B = tree->B, n = B * T;
    if (n > (size_t)0x7FFFFFFF || B * (T - 1) > (size_t)0x7FFFFFFF) {
        set_error("batched LBVH build: %zu primitives exceed the 31-bit node index range", n);
        return MSH_EINVAL;
    }
    MSH_HIP(dmalloc(&tree->d_boxes, 6 * B * sizeof(double)));
    MSH_HIP(dmalloc(&tree->d_orgs, 3 * B * sizeof(double)));
    k_mesh_boxes<<<(unsigned)B, kBlock, 0, s>>>(d_lo, d_hi, T, tree->d_boxes, tree->d_orgs);
    MSH_HIP(hipGetLastError());
    // Morton codes in each mesh's own box; sort by code, then (stable) by mesh: order = (mesh, code, id)
    MSH_TRY(ws.keys.reserve(n * sizeof(uint32_t)));
    MSH_TRY(ws.keys_alt.reserve(n * sizeof(uint32_t)));
    MSH_TRY(ws.vals_alt.reserve(n * sizeof(uint32_t)));
    uint32_t* keys = ws.keys.as<uint32_t>();
    k_morton<<<nblocks(n), kBlock, 0, s>>>(d_lo, d_hi, n, T, tree->d_boxes, keys, d_order);
    MSH_HIP(hipGetLastError());
    MSH_TRY(radix_sort_pairs(keys, d_order, ws.keys_alt.as<uint32_t>(), ws.vals_alt.as<uint32_t>(), n, 30, ws, s));
    if (B > 1) {
        k_mesh_key<<<nblocks(n), kBlock, 0, s>>>(d_order, n, T, keys);
        MSH_HIP(hipGetLastError());
        MSH_TRY(radix_sort_pairs(keys, d_order, ws.keys_alt.as<uint32_t>(), ws.vals_alt.as<uint32_t>(), n,
                                 bits_for(B), ws, s));
        k_sorted_morton<<<nblocks(n), kBlock, 0, s>>>(d_lo, d_hi, d_order, n, T, tree->d_boxes, keys);
        MSH_HIP(hipGetLastError());
    }
    const size_t nn = B * (T - 1);
    MSH_TRY(ws.vals.reserve((nn + n) * sizeof(uint32_t)));
    MSH_TRY(ws.ranges.reserve(nn * sizeof(int4)));
    uint32_t* parent = ws.vals.as<uint32_t>();
    MSH_TRY(ws.flags.reserve(nn * sizeof(uint32_t) + 64));
    uint32_t* flags = ws.flags.as<uint32_t>();
    unsigned* d_depth = flags + nn;
    MSH_HIP(hipMemsetAsync(d_depth, 0, sizeof(unsigned), s));
    k_karras<<<nblocks(nn), kBlock, 0, s>>>(keys, (int)B, (int)T, tree->d_nodes, parent, ws.ranges.as<int4>(), d_depth);
    MSH_HIP(hipGetLastError());
    unsigned depth = 0;
    MSH_HIP(hipMemcpyAsync(&depth, d_depth, sizeof(unsigned), hipMemcpyDeviceToHost, s));
    // overall scene box (informational: msh_tree_get_info)
    std::unique_ptr<double[]> hb(new double[6 * B]);
    MSH_HIP(hipMemcpyAsync(hb.get(), tree->d_boxes, 6 * B * sizeof(double), hipMemcpyDeviceToHost, s));
    MSH_HIP(hipStreamSynchronize(s));
    for (int k = 0; k < 3; ++k) {
        double lo = INFINITY, hi = -INFINITY;
        for (size_t b = 0; b < B; ++b) {
            lo = std::min(lo, hb[6 * b + k]);
            hi = std::max(hi, hb[6 * b + 3 + k]);
        }
        tree->scene_lo[k] = (float)lo;
        tree->scene_hi[k] = (float)hi;
    }
    tree->half_diag = 0.0;
    for (size_t b = 0; b < B; ++b) {
        const double c[3] = {0.5 * (hb[6 * b] + hb[6 * b + 3]), 0.5 * (hb[6 * b + 1] + hb[6 * b + 4]),
                             0.5 * (hb[6 * b + 2] + hb[6 * b + 5])};
        tree->half_diag = std::max(tree->half_diag, half_diagonal(&hb[6 * b], c));
    }
    tree->max_depth = (int)depth;
    return MSH_OK;
}

// query i of mesh i / S: 30-bit Morton code in that mesh's box
__global__ __launch_bounds__(kBlock) void k_query_morton_batch(const double* __restrict__ q, size_t n, size_t S,
                                                               const double* __restrict__ boxes,
                                                               uint32_t* __restrict__ keys, uint32_t* __restrict__ vals) {
    const size_t i = (size_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    keys[i] = morton30(q[3 * i], q[3 * i + 1], q[3 * i + 2], boxes + 6 * (i / S));
    vals[i] = (uint32_t)i;
}

int mesh_keys(const uint32_t* vals, size_t n, size_t per, uint32_t* keys, hipStream_t s) {
    k_mesh_key<<<nblocks(n), kBlock, 0, s>>>(vals, n, per, keys);
    MSH_HIP(hipGetLastError());
    return MSH_OK;
}

int query_morton_batch(const msh_tree* tree, const double* d_q, size_t n, size_t S, uint32_t* keys, uint32_t* vals,
                       hipStream_t s, size_t mesh0) {
    k_query_morton_batch<<<nblocks(n), kBlock, 0, s>>>(d_q, n, S, tree->d_boxes + 6 * mesh0, keys, vals);
    MSH_HIP(hipGetLastError());
    return MSH_OK;
}

}  // namespace msh
