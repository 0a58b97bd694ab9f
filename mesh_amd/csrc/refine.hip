// K1' — top-down re-split of the LBVH's subtrees (tree quality for the closest-point traversal).
//
// The Karras LBVH (build.hip) splits every node at the highest differing Morton bit: an axis-aligned plane
// through the middle of a power-of-two cell, the axes in fixed x, y, z rotation.  On a surface that cuts
// patches into slivers wherever the surface is oblique to the cycling planes, and a closest-point query
// visits every node whose oriented box comes within its distance — ~3 per level.  Here every subtree of at
// most K leaves is rebuilt top down, level by level over all subtrees at once: a node's primitives are split
// at the spatial middle of the longer centroid spread along the two tangent axes (t, b) of the node's own
// frame (the area-weighted normal of its triangles, t from the x or y axis, as k_obb's frames); x, y and z
// only when neither tangent axis separates them.  Splitting along the surface, and along the axes of the
// frame the children's boxes are taken in, keeps patches compact in the plane the oriented boxes are thin
// across (C3: 77.2 node visits for the plain LBVH, 64.4 with the longest of the five spreads, 62.5 tangent
// axes first).  Host model (tools/bvh_model.cpp, C3 followers with leader hints): 68.0 -> 56.7 node visits.
// CGAL's own tree (spatialsearchmodule.cpp:122, AABB_tree::rebuild) is also a top-down split, at the median
// of the longest axis of the primitives' box.
//
// Per level (every active subtree segment [s, e) of the leaf order at once; positions p of the order):
//   k_rb_scan_*     prefix sums of the area vectors in the current order (deterministic two-level scan):
//                   a segment's area-weighted normal is P[e] - P[s]
//   k_rb_frame      per segment: the frame (t, b), min / max slots reset
//   k_rb_minmax     per position: projections of its centroid on x, y, z, t, b -> segment min / max
//                   (ordered-int atomics; a wave whose lanes share a segment reduces first)
//   k_rb_choose     per segment: the tangent axis of larger spread (else x, y or z) and its middle (else: by count)
//   k_rb_flags      per position: left of the split?  -> exclusive scan (sort.hip)
//   k_rb_scatter    stable partition into the other order buffer; per segment the node record: id, range,
//                   leaf children, the link from its parent, and the two child segments of the next level
// Node ids: every internal node of a binary tree over an ordered leaf sequence owns one gap between adjacent
// leaves, its split gamma (the last leaf of its left child), so gamma -> id is a bijection onto [0, T - 2]:
// the root takes id 0 and the node whose gap is 0 takes the root's gap; every other node id = gamma.  All
// nodes are renumbered this way into a fresh node array (the LBVH nodes above the cut keep their structure
// and move to their new ids; k_rb_bignodes); ranges (first, last, gamma) and child references keep the
// conventions build_obb and the traversal rely on, and the result is deterministic (scans in fixed order,
// min / max atomics are order-free).
#include <algorithm>

#include "internal.h"

namespace msh {

constexpr uint32_t kInact = 0xFFFFFFFFu;    // position not in an active segment
constexpr uint32_t kRootPar = 0xFFFFFFFFu;  // segment parent of the tree root (id 0)
constexpr int kRbAxes = 5;  // split directions: x, y, z, t, b
constexpr int kSpatialLevels = 40;          // deeper levels split by count (bounds the depth)

struct RbSeg {
    float t[3], b[3];
    float mid;
    int axis;  // 0..kRbAxes-1 (x, y, z, t, b, ...), -1: split by count
    uint32_t mm[2 * kRbAxes];
};

__device__ inline uint32_t ford(float x) {
    const uint32_t u = __float_as_uint(x);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ inline float unord(uint32_t u) { return __uint_as_float((u & 0x80000000u) ? (u & 0x7fffffffu) : ~u); }
// node id of split gap gamma (groot: the root's gap)
__device__ inline uint32_t gap_id(uint32_t gamma, uint32_t groot) {
    return gamma == groot ? 0u : (gamma == 0u ? groot : gamma);
}
__device__ inline double4 add4(const double4& a, const double4& b) {
    return make_double4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
}

// centroid relative to the tree origin (fp32) and area vector (b - a) x (c - a) with its length
__global__ __launch_bounds__(kBlock) void k_rb_prims(const double* __restrict__ v, const uint32_t* __restrict__ f,
                                                     size_t T, double ox, double oy, double oz,
                                                     float4* __restrict__ cen, double4* __restrict__ area) {
    const size_t t = (size_t)blockIdx.x * kBlock + threadIdx.x;
    if (t >= T) return;
    const size_t i0 = f[3 * t], i1 = f[3 * t + 1], i2 = f[3 * t + 2];
    const D3 a = D3{v[3 * i0], v[3 * i0 + 1], v[3 * i0 + 2]};
    const D3 b = D3{v[3 * i1], v[3 * i1 + 1], v[3 * i1 + 2]};
    const D3 c = D3{v[3 * i2], v[3 * i2 + 1], v[3 * i2 + 2]};
    cen[t] = make_float4((float)((a.x + b.x + c.x) / 3.0 - ox), (float)((a.y + b.y + c.y) / 3.0 - oy),
                         (float)((a.z + b.z + c.z) / 3.0 - oz), 0.f);
    const D3 n = vcross(vsub(b, a), vsub(c, a));
    area[t] = make_double4(n.x, n.y, n.z, sqrt(vdot(n, n)));
}

// Segments of the first level: every position walks down the LBVH from the root to the first node over at
// most K leaves (its subtree is rebuilt: segment start = the node's first leaf; its parent link = the new id
// of the last larger node and the side taken) or to a leaf child of a larger node (inactive).
__global__ __launch_bounds__(kBlock) void k_rb_cut(const BNode* __restrict__ nodes, const int4* __restrict__ ranges,
                                                   size_t T, uint32_t K, uint32_t* __restrict__ sb,
                                                   uint32_t* __restrict__ tabE, uint32_t* __restrict__ tabPar) {
    const size_t p = (size_t)blockIdx.x * kBlock + threadIdx.x;
    if (p >= T) return;
    const uint32_t groot = (uint32_t)ranges[0].z;  // used only when the root is larger than K (kept)
    int g = 0;
    uint32_t par = kRootPar;
    for (;;) {
        const int4 r = ranges[g];
        if ((uint32_t)(r.y - r.x + 1) <= K) {
            sb[p] = (uint32_t)r.x;
            if (p == (size_t)r.x) {
                tabE[p] = (uint32_t)r.y + 1u;
                tabPar[p] = par;
            }
            return;
        }
        const int side = (int)p <= r.z ? 0 : 1;
        const int c = __float_as_int(nodes[g].f[6 + side]);
        if (c < 0) {
            sb[p] = kInact;
            return;
        }
        par = (gap_id((uint32_t)r.z, groot) << 1) | (uint32_t)side;
        g = c;
    }
}

// LBVH nodes over more than K leaves keep their split and move to id gap_id(gamma): children that are leaves
// or larger nodes are written here, rebuilt children link themselves (k_rb_scatter); groot <- the root's gap
__global__ __launch_bounds__(kBlock) void k_rb_bignodes(const BNode* __restrict__ nodes, const int4* __restrict__ ranges,
                                                        size_t nn, uint32_t K, BNode* __restrict__ out,
                                                        int4* __restrict__ out_ranges, unsigned* __restrict__ groot_out) {
    const size_t g = (size_t)blockIdx.x * kBlock + threadIdx.x;
    if (g >= nn) return;
    const int4 r = ranges[g];
    if ((uint32_t)(r.y - r.x + 1) <= K) return;
    const uint32_t groot = (uint32_t)ranges[0].z;
    if (g == 0) *groot_out = groot;
    const uint32_t id = gap_id((uint32_t)r.z, groot);
    out_ranges[id] = r;
#pragma unroll
    for (int side = 0; side < 2; ++side) {
        const int c = __float_as_int(nodes[g].f[6 + side]);
        if (c < 0) {
            out[id].f[6 + side] = __int_as_float(c);
        } else {
            const int4 rc = ranges[c];
            if ((uint32_t)(rc.y - rc.x + 1) > K) out[id].f[6 + side] = __int_as_float((int)gap_id((uint32_t)rc.z, groot));
        }
    }
}

// ---- exclusive prefix sums of the area vectors of active positions in the current order: P[0] = 0,
// P[p + 1] = sum over q <= p (two-level, fixed association)
constexpr int kRbPer = 8;
constexpr int kRbTile = kBlock * kRbPer;
__device__ inline double4 rb_block_exscan(double4 v, double4* sh, double4& total) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    double4 inc = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const double4 u = make_double4(__shfl_up(inc.x, o, 64), __shfl_up(inc.y, o, 64), __shfl_up(inc.z, o, 64),
                                       __shfl_up(inc.w, o, 64));
        if (lane >= o) inc = add4(inc, u);
    }
    if (lane == 63) sh[w] = inc;
    __syncthreads();
    double4 off = make_double4(0, 0, 0, 0);
    for (int k = 0; k < w; ++k) off = add4(off, sh[k]);
    total = add4(add4(add4(sh[0], sh[1]), sh[2]), sh[3]);
    __syncthreads();
    return add4(off, make_double4(inc.x - v.x, inc.y - v.y, inc.z - v.z, inc.w - v.w));
}
__global__ __launch_bounds__(kBlock) void k_rb_scan_blocks(const uint32_t* __restrict__ idx, const uint32_t* __restrict__ sb,
                                                           const double4* __restrict__ area, size_t n,
                                                           double4* __restrict__ P, double4* __restrict__ btot) {
    __shared__ double4 sh[4];
    const size_t base = (size_t)blockIdx.x * kRbTile + (size_t)threadIdx.x * kRbPer;
    double4 loc[kRbPer];
    double4 run = make_double4(0, 0, 0, 0);
#pragma unroll
    for (int k = 0; k < kRbPer; ++k) {
        const size_t i = base + k;
        if (i < n && sb[i] != kInact) run = add4(run, area[idx[i]]);
        loc[k] = run;
    }
    double4 total;
    const double4 off = rb_block_exscan(run, sh, total);
#pragma unroll
    for (int k = 0; k < kRbPer; ++k)
        if (base + k < n) P[base + k + 1] = add4(off, loc[k]);
    if (threadIdx.x == 0) btot[blockIdx.x] = total;
}
__global__ __launch_bounds__(kBlock) void k_rb_scan_tops(double4* __restrict__ btot, int nb) {
    __shared__ double4 sh[4];
    const int per = (nb + kBlock - 1) / kBlock, b0 = threadIdx.x * per, b1 = min(nb, b0 + per);
    double4 run = make_double4(0, 0, 0, 0);
    for (int b = b0; b < b1; ++b) run = add4(run, btot[b]);
    double4 total;
    double4 off = rb_block_exscan(run, sh, total);
    for (int b = b0; b < b1; ++b) {
        const double4 t = btot[b];
        btot[b] = off;
        off = add4(off, t);
    }
}
__global__ __launch_bounds__(kBlock) void k_rb_scan_add(double4* __restrict__ P, size_t n, const double4* __restrict__ btot) {
    const size_t i = (size_t)blockIdx.x * kBlock + threadIdx.x;
    if (i == 0) P[0] = make_double4(0, 0, 0, 0);
    if (i >= n) return;
    P[i + 1] = add4(btot[i / kRbTile], P[i + 1]);
}

// the segment's frame (as k_obb's obb_frame: n from the area sum unless it cancels, t = e - (e.n) n with e the
// x or y axis, b = n x t) and reset min / max slots
__global__ __launch_bounds__(kBlock) void k_rb_frame(const uint32_t* __restrict__ sb, const uint32_t* __restrict__ tabE,
                                                     const double4* __restrict__ P, size_t T, RbSeg* __restrict__ seg) {
    const size_t s = (size_t)blockIdx.x * kBlock + threadIdx.x;
    if (s >= T || sb[s] != (uint32_t)s) return;
    const uint32_t e = tabE[s];
    const double4 a = P[e], b0 = P[s];
    const double sx = a.x - b0.x, sy = a.y - b0.y, sz = a.z - b0.z, sa = a.w - b0.w;
    const double len = sqrt(sx * sx + sy * sy + sz * sz);
    const D3 n = (len > 1e-6 * sa && len < INFINITY) ? D3{sx / len, sy / len, sz / len} : D3{1.0, 0.0, 0.0};
    const D3 ex = fabs(n.x) < 0.9 ? D3{1.0, 0.0, 0.0} : D3{0.0, 1.0, 0.0};
    D3 t = vsub(ex, vscale(vdot(ex, n), n));
    const double tl = sqrt(vdot(t, t));
    t = D3{t.x / tl, t.y / tl, t.z / tl};
    const D3 bb = vcross(n, t);
    RbSeg& g = seg[s];
    g.t[0] = (float)t.x; g.t[1] = (float)t.y; g.t[2] = (float)t.z;
    g.b[0] = (float)bb.x; g.b[1] = (float)bb.y; g.b[2] = (float)bb.z;
#pragma unroll
    for (int k = 0; k < kRbAxes; ++k) {
        g.mm[k] = 0xFFFFFFFFu;
        g.mm[kRbAxes + k] = 0u;
    }
}

// projection of centroid c on direction k (0..4: x, y, z, t, b) of segment g
__device__ inline float rb_key(const float4& c, const RbSeg& g, int k) {
    if (k == 0) return c.x;
    if (k == 1) return c.y;
    if (k == 2) return c.z;
    const float* a = k == 3 ? g.t : g.b;
    return fmaf(a[0], c.x, fmaf(a[1], c.y, a[2] * c.z));
}

__global__ __launch_bounds__(kBlock) void k_rb_minmax(const uint32_t* __restrict__ idx, const uint32_t* __restrict__ sb,
                                                      const float4* __restrict__ cen, size_t T, RbSeg* __restrict__ seg) {
    const size_t p = (size_t)blockIdx.x * kBlock + threadIdx.x;
    const bool act = p < T && sb[p] != kInact;
    const uint32_t s = act ? sb[p] : kInact;
    uint32_t v[2 * kRbAxes];
    if (act) {
        const float4 c = cen[idx[p]];
        const RbSeg& g = seg[s];
#pragma unroll
        for (int k = 0; k < kRbAxes; ++k) {
            const uint32_t o = ford(rb_key(c, g, k));
            v[k] = o;
            v[kRbAxes + k] = o;
        }
    } else {
#pragma unroll
        for (int k = 0; k < kRbAxes; ++k) {
            v[k] = 0xFFFFFFFFu;
            v[kRbAxes + k] = 0u;
        }
    }
    // a wave whose active lanes all belong to one segment reduces first (the top levels: one atomic per wave)
    const unsigned long long am = __ballot(act);
    if (am == 0ull) return;
    const int first = __ffsll((long long)am) - 1;
    const uint32_t s0 = (uint32_t)__shfl((int)s, first);
    if (__all(!act || s == s0)) {
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
#pragma unroll
            for (int k = 0; k < kRbAxes; ++k) {
                v[k] = min(v[k], (uint32_t)__shfl_xor((int)v[k], o));
                v[kRbAxes + k] = max(v[kRbAxes + k], (uint32_t)__shfl_xor((int)v[kRbAxes + k], o));
            }
        }
        if ((threadIdx.x & 63) == (unsigned)first) {
#pragma unroll
            for (int k = 0; k < kRbAxes; ++k) {
                atomicMin(&seg[s0].mm[k], v[k]);
                atomicMax(&seg[s0].mm[kRbAxes + k], v[kRbAxes + k]);
            }
        }
    } else if (act) {
#pragma unroll
        for (int k = 0; k < kRbAxes; ++k) {
            atomicMin(&seg[s].mm[k], v[k]);
            atomicMax(&seg[s].mm[kRbAxes + k], v[kRbAxes + k]);
        }
    }
}

__global__ __launch_bounds__(kBlock) void k_rb_choose(const uint32_t* __restrict__ sb, size_t T, int level,
                                                      RbSeg* __restrict__ seg) {
    const size_t s = (size_t)blockIdx.x * kBlock + threadIdx.x;
    if (s >= T || sb[s] != (uint32_t)s) return;
    RbSeg& g = seg[s];
    int axis = -1;
    float best = 0.f, mid = 0.f;
    if (level < kSpatialLevels) {
#pragma unroll
        for (int k = 0; k < kRbAxes; ++k) {
            const float lo = unord(g.mm[k]), hi = unord(g.mm[kRbAxes + k]);
            // the node frame's tangent axes take precedence: splitting along t or b keeps the children's boxes in
            // that frame compact, x, y and z are the fallback (C3: 64.4 -> 62.5 node visits; spreads compared
            // across all five: 64.4; diagonal tangent directions (t +- b)/sqrt2 added: 86.9 — their strips are
            // wide along both axes of the boxes)
            const float w = (hi - lo) * (k >= 3 ? 1e6f : 1.0f), m = 0.5f * lo + 0.5f * hi;
            // a usable split: finite, and the middle strictly inside (both sides non-empty)
            if (w > best && w < INFINITY && lo < m && m < hi) {
                best = w;
                axis = k;
                mid = m;
            }
        }
    }
    g.axis = axis;
    g.mid = mid;
}

// flags[p] = 1 if position p goes to the left child (flags[T] = 0, the scan's total slot)
__global__ __launch_bounds__(kBlock) void k_rb_flags(const uint32_t* __restrict__ idx, const uint32_t* __restrict__ sb,
                                                     const uint32_t* __restrict__ tabE, const float4* __restrict__ cen,
                                                     const RbSeg* __restrict__ seg, size_t T, uint32_t* __restrict__ flags) {
    const size_t p = (size_t)blockIdx.x * kBlock + threadIdx.x;
    if (p > T) return;
    uint32_t fl = 0u;
    if (p < T && sb[p] != kInact) {
        const uint32_t s = sb[p];
        const RbSeg& g = seg[s];
        if (g.axis >= 0) {
            fl = rb_key(cen[idx[p]], g, g.axis) < g.mid ? 1u : 0u;
        } else {
            fl = (p - s) < (tabE[s] - s) / 2u ? 1u : 0u;
        }
    }
    flags[p] = fl;
}

struct RbTabs {
    uint32_t *e, *par;
};

// stable partition into idx2 / sb2; the segment's first position also writes its node (id gap_id(gamma),
// range, leaf children, the link from its parent) and the next level's segments.  The tree root's segment
// (only at the first level, when the whole tree is rebuilt) takes id 0 and publishes its gap in *groot.
__global__ __launch_bounds__(kBlock) void k_rb_scatter(const uint32_t* __restrict__ idx, const uint32_t* __restrict__ sb,
                                                       const uint32_t* __restrict__ L, size_t T, RbTabs cur, RbTabs nxt,
                                                       uint32_t* __restrict__ idx2, uint32_t* __restrict__ sb2,
                                                       BNode* __restrict__ nodes, int4* __restrict__ ranges,
                                                       unsigned* __restrict__ cnt) {
    const size_t p = (size_t)blockIdx.x * kBlock + threadIdx.x;
    if (p >= T) return;
    const uint32_t s = sb[p];
    if (s == kInact) {
        idx2[p] = idx[p];
        sb2[p] = kInact;
        return;
    }
    const uint32_t e = cur.e[s];
    const uint32_t Ls = L[s], nl = L[e] - Ls, m = s + nl;
    const uint32_t lp = L[p];
    const bool left = L[p + 1] != lp;
    const uint32_t np = left ? s + (lp - Ls) : m + ((uint32_t)p - s) - (lp - Ls);
    idx2[np] = idx[p];
    const uint32_t cb = left ? s : m, ce = left ? m : e;
    sb2[np] = (ce - cb >= 2u) ? cb : kInact;
    if (p != s) return;
    // ---- the segment's node
    const uint32_t par = cur.par[s];
    const uint32_t gamma = m - 1u;
    uint32_t id;
    if (par == kRootPar) {
        id = 0u;
        cnt[1] = gamma;
    } else {
        id = gap_id(gamma, cnt[1]);
    }
    float* fn = nodes[id].f;
    if (m - s >= 2u) {
        nxt.e[s] = m;
        nxt.par[s] = (id << 1) | 0u;
    } else {
        fn[6] = __int_as_float(~(int)s);
    }
    if (e - m >= 2u) {
        nxt.e[m] = e;
        nxt.par[m] = (id << 1) | 1u;
    } else {
        fn[7] = __int_as_float(~(int)m);
    }
    if (par != kRootPar) nodes[par >> 1].f[6 + (par & 1u)] = __int_as_float((int)id);
    ranges[id] = make_int4((int)s, (int)e - 1, (int)gamma, 0);
    const unsigned k = (m - s >= 2u ? 1u : 0u) + (e - m >= 2u ? 1u : 0u);
    if (k) atomicAdd(&cnt[0], k);
}

static unsigned rb_blocks(size_t n) { return (unsigned)((n + kBlock - 1) / kBlock); }

int resplit_tree(msh_tree* tree, const double* d_v, const uint32_t* d_f, size_t T, uint32_t* d_order, int log2K) {
    if (T < 3 || log2K <= 0) return MSH_OK;
    hipStream_t s = tree->stream;
    Workspace& ws = tree->ws;
    const uint32_t K = log2K >= 31 ? 0x7FFFFFFFu : (1u << log2K);
    struct Tmp {
        void* p = nullptr;
        ~Tmp() { if (p) (void)dfree(p); }
    } t_cen, t_area, t_P, t_btot, t_idx2, t_sb, t_sb2, t_flags, t_seg, t_tab, t_cnt, t_nodes, t_ranges;
    const int nsb = (int)((T + kRbTile - 1) / kRbTile);
    const size_t nn = T - 1;
    MSH_HIP(dmalloc(&t_cen.p, T * sizeof(float4)));
    MSH_HIP(dmalloc(&t_area.p, T * sizeof(double4)));
    MSH_HIP(dmalloc(&t_P.p, (T + 1) * sizeof(double4)));
    MSH_HIP(dmalloc(&t_btot.p, (size_t)nsb * sizeof(double4)));
    MSH_HIP(dmalloc(&t_idx2.p, T * sizeof(uint32_t)));
    MSH_HIP(dmalloc(&t_sb.p, T * sizeof(uint32_t)));
    MSH_HIP(dmalloc(&t_sb2.p, T * sizeof(uint32_t)));
    MSH_HIP(dmalloc(&t_flags.p, (T + 1) * sizeof(uint32_t)));
    MSH_HIP(dmalloc(&t_seg.p, T * sizeof(RbSeg)));
    MSH_HIP(dmalloc(&t_tab.p, 4 * T * sizeof(uint32_t)));
    MSH_HIP(dmalloc(&t_cnt.p, 64 * sizeof(unsigned)));
    MSH_HIP(dmalloc(&t_nodes.p, nn * sizeof(BNode)));
    MSH_HIP(dmalloc(&t_ranges.p, nn * sizeof(int4)));
    float4* cen = static_cast<float4*>(t_cen.p);
    double4* area = static_cast<double4*>(t_area.p);
    double4* P = static_cast<double4*>(t_P.p);
    double4* btot = static_cast<double4*>(t_btot.p);
    uint32_t* idx[2] = {d_order, static_cast<uint32_t*>(t_idx2.p)};
    uint32_t* sbb[2] = {static_cast<uint32_t*>(t_sb.p), static_cast<uint32_t*>(t_sb2.p)};
    uint32_t* flags = static_cast<uint32_t*>(t_flags.p);
    RbSeg* seg = static_cast<RbSeg*>(t_seg.p);
    uint32_t* tab = static_cast<uint32_t*>(t_tab.p);
    RbTabs tabs[2] = {{tab, tab + T}, {tab + 2 * T, tab + 3 * T}};
    unsigned* cnt = static_cast<unsigned*>(t_cnt.p);  // [0] next level's segments, [1] the root's gap
    BNode* nodes2 = static_cast<BNode*>(t_nodes.p);
    int4* ranges2 = static_cast<int4*>(t_ranges.p);
    const unsigned nb = rb_blocks(T);
    const int4* ranges = ws.ranges.as<int4>();

    MSH_HIP(hipMemsetAsync(nodes2, 0, nn * sizeof(BNode), s));
    k_rb_prims<<<nb, kBlock, 0, s>>>(d_v, d_f, T, tree->origin[0], tree->origin[1], tree->origin[2], cen, area);
    k_rb_cut<<<nb, kBlock, 0, s>>>(tree->d_nodes, ranges, T, K, sbb[0], tabs[0].e, tabs[0].par);
    k_rb_bignodes<<<rb_blocks(nn), kBlock, 0, s>>>(tree->d_nodes, ranges, nn, K, nodes2, ranges2, cnt + 1);
    MSH_HIP(hipGetLastError());
    int cur = 0, levels = 0;
    for (int level = 0;; ++level) {
        k_rb_scan_blocks<<<(unsigned)nsb, kBlock, 0, s>>>(idx[cur], sbb[cur], area, T, P, btot);
        k_rb_scan_tops<<<1, kBlock, 0, s>>>(btot, nsb);
        k_rb_scan_add<<<nb, kBlock, 0, s>>>(P, T, btot);
        k_rb_frame<<<nb, kBlock, 0, s>>>(sbb[cur], tabs[cur].e, P, T, seg);
        k_rb_minmax<<<nb, kBlock, 0, s>>>(idx[cur], sbb[cur], cen, T, seg);
        k_rb_choose<<<nb, kBlock, 0, s>>>(sbb[cur], T, level, seg);
        k_rb_flags<<<rb_blocks(T + 1), kBlock, 0, s>>>(idx[cur], sbb[cur], tabs[cur].e, cen, seg, T, flags);
        MSH_HIP(hipGetLastError());
        MSH_TRY(exclusive_scan_u32(flags, T + 1, ws, s));
        MSH_HIP(hipMemsetAsync(cnt, 0, sizeof(unsigned), s));
        k_rb_scatter<<<nb, kBlock, 0, s>>>(idx[cur], sbb[cur], flags, T, tabs[cur], tabs[cur ^ 1], idx[cur ^ 1],
                                           sbb[cur ^ 1], nodes2, ranges2, cnt);
        MSH_HIP(hipGetLastError());
        unsigned h = 0;
        MSH_HIP(hipMemcpyAsync(&h, cnt, sizeof(unsigned), hipMemcpyDeviceToHost, s));
        MSH_HIP(hipStreamSynchronize(s));
        cur ^= 1;
        levels = level + 1;
        if (h == 0) break;
        if (level > 4096) {
            set_error("tree re-split: no convergence");
            return MSH_EDEVICE;
        }
    }
    if (cur != 0) MSH_HIP(hipMemcpyAsync(d_order, idx[cur], T * sizeof(uint32_t), hipMemcpyDeviceToDevice, s));
    MSH_HIP(hipMemcpyAsync(ws.ranges.ptr, ranges2, nn * sizeof(int4), hipMemcpyDeviceToDevice, s));
    MSH_HIP(hipStreamSynchronize(s));
    std::swap(tree->d_nodes, *reinterpret_cast<BNode**>(&t_nodes.p));  // the old array is freed on return
    // a whole rebuilt tree is exactly `levels` deep; otherwise the LBVH part above the rebuilt subtrees is at
    // most max_depth deep and every re-split level adds at most one
    tree->max_depth = K >= T ? levels : tree->max_depth + levels;
    return MSH_OK;
}

}  // namespace msh
