// K2 + K3 — closest-point traversal with fused fp64 refinement (replaces
// spatialsearchmodule.cpp:165-220 aabbtree_nearest and CGAL's closest_point_and_primitive), plus the
// normal-weighted metric variant (K7, aabb_normals.cpp:112-190) and the vertex nearest-neighbour
// variant (K8, search.ClosestPointTree).
//
// Execution shape (gfx950):
//   * persistent grid (≈5 workgroups of 256 lanes per CU, the LDS-stack limit); each WAVE dequeues
//     64-query tiles from one of 8 XCD-group counters (group = blockIdx % 8, which labels the blocks
//     sharing an XCD), each counter owning a contiguous eighth of the Morton-sorted queries — an XCD's
//     L2 then serves one spatial region of the BVH; exhausted groups steal from the others.
//   * one lane per query, queries visited in Morton order (perm) for wave coherence;
//   * near-child-first depth-first traversal: one 64-B node read tests both children (fp32 boxes,
//     distance evaluated in fp64 so the cull is conservative), leaves are tested immediately in fp64
//     with CGAL's construction, the far child is pushed with its lower-bound distance;
//   * per-lane stack: 16 entries in LDS ([depth][lane] layout, conflict-free), deeper entries spill to
//     a per-lane global area sized from the tree depth measured at build time;
//   * ties: the lexicographic minimum of (squared distance, face index) — deterministic and independent
//     of traversal order (boxes at distance <= best*(1+2^-40) are visited, so equal-distance faces are
//     all examined).
#include <algorithm>
#include <mutex>

#include "internal.h"

namespace msh {

struct KnnArgs {
    const BNode* nodes;
    const void* leaves;
    size_t T;
    const double* q;
    const double* n;
    const uint32_t* perm;
    size_t S;
    uint32_t* out_face;
    uint32_t* out_part;
    double* out_pt;
    double* out_dist;
    double eps;
    unsigned* counters;
    unsigned ntiles;
    uint2* spill;
    int spill_depth;
    unsigned long long* stats;
};

__device__ inline unsigned dequeue_tile(unsigned* counters, unsigned ntiles, unsigned group) {
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

// ---- leaf policies ----
struct TriPol {
    const TriRec* __restrict__ tris;
    D3 q;
    double best;
    uint32_t best_face;
    int best_leaf;
    __device__ double limit() const { return best * kSlack; }
    __device__ void test(int leaf) {
        D3 a, b, c;
        uint32_t face;
        load_tri(tris, leaf, a, b, c, face);
        D3 o;
        int part;
        const double d2 = closest_on_triangle(q, a, b, c, o, part);
        if (d2 < best || (d2 == best && face < best_face)) {
            best = d2;
            best_face = face;
            best_leaf = leaf;
        }
    }
};

// metric = ||q - p|| + eps (1 - n_q . n_tri)  (AABB_n_tree.h:40-84).  The penalty is bounded below by
// pmin = min(eps(1-|n_q|), eps(1+|n_q|)), so a face can only win inside the ball of radius best - pmin.
struct NrmPol {
    const TriRec* __restrict__ tris;
    D3 q, qn;
    double eps, pmin;
    double best;
    uint32_t best_face;
    int best_leaf;
    __device__ double limit() const {
        if (best == INFINITY) return INFINITY;
        double r = best - pmin;
        r += 1e-12 * (fabs(best) + fabs(pmin));
        if (r < 0.0) r = 0.0;
        return r * r * kSlack;
    }
    __device__ void test(int leaf) {
        D3 a, b, c;
        uint32_t face;
        load_tri(tris, leaf, a, b, c, face);
        D3 o;
        int part;
        const double d2 = closest_on_triangle(q, a, b, c, o, part);
        double pa, pb, pc, pd;
        plane_of(a, b, c, pa, pb, pc, pd);
        const double sn = sqrt(pa * pa + pb * pb + pc * pc);
        const D3 tn = D3{pa / sn, pb / sn, pc / sn};
        const double met = sqrt(d2) + eps * (1 - vdot(qn, tn));
        if (met < best || (met == best && face < best_face)) {
            best = met;
            best_face = face;
            best_leaf = leaf;
        }
    }
};

struct PtPol {
    const PtRec* __restrict__ pts;
    D3 q;
    double best;
    uint32_t best_face;
    int best_leaf;
    __device__ double limit() const { return best * kSlack; }
    __device__ void test(int leaf) {
        const double2* p = reinterpret_cast<const double2*>(pts + leaf);
        const double2 x0 = p[0], x1 = p[1];
        const uint32_t idx = (uint32_t)__double_as_longlong(x1.y);
        const double d2 = sqdist(q, D3{x0.x, x0.y, x1.x});
        if (d2 < best || (d2 == best && idx < best_face)) {
            best = d2;
            best_face = idx;
            best_leaf = leaf;
        }
    }
};

// Near-child-first depth-first traversal.  lds: this lane's column of the LDS stack (stride kBlock).
template <class Pol, bool STATS>
__device__ inline void traverse(const BNode* __restrict__ nodes, size_t T, const D3& q, Pol& pol, uint2* __restrict__ lds,
                                uint2* __restrict__ spill, unsigned& n_nodes, unsigned& n_leaves) {
    if (T == 1) {
        pol.test(0);
        if (STATS) ++n_leaves;
        return;
    }
    int node = 0;
    int sp = 0;
    // every internal node is entered at most once per query; the cap only bounds a corrupt tree
    for (size_t guard = 0; guard < T; ++guard) {
        const BNode nd = load_node(nodes, node);
        if (STATS) ++n_nodes;
        const double d0 = box_d2(q, nd.a.x, nd.a.y, nd.a.z, nd.a.w, nd.b.x, nd.b.y);
        const double d1 = box_d2(q, nd.b.z, nd.b.w, nd.c.x, nd.c.y, nd.c.z, nd.c.w);
        const int c0 = nd.d.x, c1 = nd.d.y;
        double lim = pol.limit();
        bool h0 = d0 <= lim, h1 = d1 <= lim;
        if (h0 && c0 < 0) {
            pol.test(~c0);
            if (STATS) ++n_leaves;
            h0 = false;
            lim = pol.limit();
        }
        if (h1 && c1 < 0) {
            pol.test(~c1);
            if (STATS) ++n_leaves;
            h1 = false;
            lim = pol.limit();
        }
        h0 = h0 && d0 <= lim;
        h1 = h1 && d1 <= lim;
        if (h0 && h1) {
            int nearc = c0, farc = c1;
            double dfar = d1;
            if (d1 < d0) { nearc = c1; farc = c0; dfar = d0; }
            const uint2 e = make_uint2((unsigned)farc, __float_as_uint(__double2float_rd(dfar)));
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
            if ((double)__uint_as_float(e.y) <= pol.limit()) {
                node = (int)e.x;
                found = true;
                break;
            }
        }
        if (!found) break;
    }
}

template <int MODE, bool STATS>
__global__ __launch_bounds__(kBlock) void k_knn(KnnArgs a) {
    __shared__ uint2 stk[kStack * kBlock];
    const int tid = threadIdx.x, lane = tid & 63;
    uint2* lds = stk + tid;
    uint2* spill = a.spill ? a.spill + ((size_t)blockIdx.x * kBlock + tid) * (size_t)a.spill_depth : nullptr;
    const unsigned group = blockIdx.x & 7u;
    unsigned n_nodes = 0, n_leaves = 0;
    for (;;) {
        unsigned tile = 0;
        if (lane == 0) tile = dequeue_tile(a.counters, a.ntiles, group);
        tile = __shfl(tile, 0);
        if (tile >= a.ntiles) break;
        const size_t i = (size_t)tile * 64 + lane;
        if (i >= a.S) continue;
        const size_t qi = a.perm ? (size_t)a.perm[i] : i;
        const D3 q = D3{a.q[3 * qi], a.q[3 * qi + 1], a.q[3 * qi + 2]};
        if (MODE == 0) {
            TriPol pol{static_cast<const TriRec*>(a.leaves), q, INFINITY, 0xFFFFFFFFu, -1};
            traverse<TriPol, STATS>(a.nodes, a.T, q, pol, lds, spill, n_nodes, n_leaves);
            if (!STATS) {
                D3 ta, tb, tc, o = D3{NAN, NAN, NAN};
                uint32_t face = 0xFFFFFFFFu;
                int part = 0;
                if (pol.best_leaf >= 0) {  // < 0 only for a non-finite query
                    load_tri(pol.tris, pol.best_leaf, ta, tb, tc, face);
                    closest_on_triangle(q, ta, tb, tc, o, part);
                }
                a.out_face[qi] = face;
                if (a.out_part) a.out_part[qi] = (uint32_t)part;
                a.out_pt[3 * qi] = o.x;
                a.out_pt[3 * qi + 1] = o.y;
                a.out_pt[3 * qi + 2] = o.z;
            }
        } else if (MODE == 1) {
            const D3 qn = D3{a.n[3 * qi], a.n[3 * qi + 1], a.n[3 * qi + 2]};
            const double nq = sqrt(vdot(qn, qn));
            const double pmin = fmin(a.eps * (1 - nq), a.eps * (1 + nq));
            NrmPol pol{static_cast<const TriRec*>(a.leaves), q, qn, a.eps, pmin, INFINITY, 0xFFFFFFFFu, -1};
            traverse<NrmPol, STATS>(a.nodes, a.T, q, pol, lds, spill, n_nodes, n_leaves);
            D3 ta, tb, tc, o = D3{NAN, NAN, NAN};
            uint32_t face = 0xFFFFFFFFu;
            int part = 0;
            if (pol.best_leaf >= 0) {
                load_tri(pol.tris, pol.best_leaf, ta, tb, tc, face);
                closest_on_triangle(q, ta, tb, tc, o, part);
            }
            a.out_face[qi] = face;
            a.out_pt[3 * qi] = o.x;
            a.out_pt[3 * qi + 1] = o.y;
            a.out_pt[3 * qi + 2] = o.z;
        } else {
            PtPol pol{static_cast<const PtRec*>(a.leaves), q, INFINITY, 0xFFFFFFFFu, -1};
            traverse<PtPol, STATS>(a.nodes, a.T, q, pol, lds, spill, n_nodes, n_leaves);
            a.out_face[qi] = pol.best_face;
            a.out_dist[qi] = sqrt(pol.best);
        }
    }
    if (STATS) {
        atomicAdd(&a.stats[0], (unsigned long long)n_nodes);
        atomicAdd(&a.stats[1], (unsigned long long)n_leaves);
    }
}

__global__ __launch_bounds__(kBlock) void k_query_morton(const double* __restrict__ q, size_t S, float lx, float ly, float lz,
                                                         float hx, float hy, float hz, uint32_t* __restrict__ keys,
                                                         uint32_t* __restrict__ vals) {
    const size_t i = (size_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= S) return;
    const float ex = hx - lx, ey = hy - ly, ez = hz - lz;
    float nx = ex > 0.f ? ((float)q[3 * i] - lx) / ex : 0.5f;
    float ny = ey > 0.f ? ((float)q[3 * i + 1] - ly) / ey : 0.5f;
    float nz = ez > 0.f ? ((float)q[3 * i + 2] - lz) / ez : 0.5f;
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
    keys[i] = (ex10((uint32_t)nx) << 2) | (ex10((uint32_t)ny) << 1) | ex10((uint32_t)nz);
    vals[i] = (uint32_t)i;
}

int query_morton(const msh_tree* tree, const double* d_q, size_t S, uint32_t* keys, uint32_t* vals, hipStream_t s) {
    if (S == 0) return MSH_OK;
    TimedLaunch tl("morton", s);
    k_query_morton<<<(unsigned)((S + kBlock - 1) / kBlock), kBlock, 0, s>>>(
        d_q, S, tree->scene_lo[0], tree->scene_lo[1], tree->scene_lo[2], tree->scene_hi[0], tree->scene_hi[1],
        tree->scene_hi[2], keys, vals);
    MSH_HIP(hipGetLastError());
    return MSH_OK;
}

static int device_cus(int dev) {
    static std::mutex mu;
    static int cache[64] = {0};
    std::lock_guard<std::mutex> g(mu);
    if (dev < 0 || dev >= 64) return 256;
    if (!cache[dev]) {
        int n = 0;
        if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
        cache[dev] = n;
    }
    return cache[dev];
}

// Common launch: grid, counters, spill area.
template <int MODE, bool STATS>
static int launch_knn(msh_tree* tree, KnnArgs a, hipStream_t s, const char* timer) {
    if (a.S == 0) return MSH_OK;
    const unsigned ntiles = (unsigned)((a.S + 63) / 64);
    const unsigned want = (ntiles + 3) / 4;
    const unsigned nblk = std::min<unsigned>(want, (unsigned)device_cus(tree->device) * 5u);
    a.ntiles = ntiles;
    // counters (8 x 128 B) + spill
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
    k_knn<MODE, STATS><<<nblk, kBlock, 0, s>>>(a);
    MSH_HIP(hipGetLastError());
    return MSH_OK;
}

int launch_nearest(const msh_tree* tree, const double* d_q, const uint32_t* d_perm, size_t S, uint32_t* d_face,
                   uint32_t* d_part, double* d_pt, hipStream_t s) {
    KnnArgs a{};
    a.nodes = tree->d_nodes; a.leaves = tree->d_leaves; a.T = tree->T;
    a.q = d_q; a.perm = d_perm; a.S = S;
    a.out_face = d_face; a.out_part = d_part; a.out_pt = d_pt;
    return launch_knn<0, false>(const_cast<msh_tree*>(tree), a, s, "nearest");
}

int launch_nearest_stats(const msh_tree* tree, const double* d_q, const uint32_t* d_perm, size_t S,
                         unsigned long long* d_counts, hipStream_t s) {
    KnnArgs a{};
    a.nodes = tree->d_nodes; a.leaves = tree->d_leaves; a.T = tree->T;
    a.q = d_q; a.perm = d_perm; a.S = S;
    a.stats = d_counts;
    return launch_knn<0, true>(const_cast<msh_tree*>(tree), a, s, "nearest_stats");
}

int launch_nnearest(const msh_tree* tree, const double* d_q, const double* d_n, const uint32_t* d_perm, size_t S,
                    uint32_t* d_face, double* d_pt, hipStream_t s) {
    KnnArgs a{};
    a.nodes = tree->d_nodes; a.leaves = tree->d_leaves; a.T = tree->T;
    a.q = d_q; a.n = d_n; a.perm = d_perm; a.S = S; a.eps = tree->eps;
    a.out_face = d_face; a.out_pt = d_pt;
    return launch_knn<1, false>(const_cast<msh_tree*>(tree), a, s, "nnearest");
}

int launch_points_nearest(const msh_tree* tree, const double* d_q, const uint32_t* d_perm, size_t S, uint32_t* d_idx,
                          double* d_dist, hipStream_t s) {
    KnnArgs a{};
    a.nodes = tree->d_nodes; a.leaves = tree->d_leaves; a.T = tree->T;
    a.q = d_q; a.perm = d_perm; a.S = S;
    a.out_face = d_idx; a.out_dist = d_dist;
    return launch_knn<2, false>(const_cast<msh_tree*>(tree), a, s, "points_nearest");
}

}  // namespace msh
