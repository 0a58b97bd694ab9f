// K4 — nearest_alongnormal: nearest hit of the rays (p, n) and (p, -n)
//      (replaces spatialsearchmodule.cpp:222-323: two CGAL all_intersections lists per point, serial)
// K5 — visibility any-hit over (camera x vertex) rays
//      (replaces visibility.cpp:75-115 VisibilityTask: tree.do_intersect(Ray) per camera and vertex)
//
// Ray semantics (shared with the oracle restatement): a CGAL Ray_3(p, v) is stored as two points
// (p, p + v) and its predicates use (p + v) - p as direction; the ray is closed (t >= 0) and so are
// the triangles.  A ray hits a triangle iff its supporting line passes the three edges with consistent
// orientation (edge determinants flip sign exactly for the shared edge of two triangles, so a ray
// through a shared edge is never lost) and the plane crossing parameter is >= 0.
// Hit point: CGAL's construction for a proper hit, intersection(Plane_3(a, b, c), Line_3(p, p + v))
// (Intersections_3 Plane_3/Line_3: num = A px + B py + C pz + D, den = A dx + B dy + C dz,
// point = ((den px - num dx) / den, ...)), with the plane from plane_from_pointsC3.  A ray lying in the
// triangle's plane (CGAL returns a Segment_3) enters it at the clipped parameter; the reference's
// segment branch (:295-307) is not restated: it intersects the segment's line with the ray's line in
// the xy projection, but the segment lies ON the ray's line, so its denominator is the 2-D cross
// product of two parallel vectors (0 up to rounding) and its point is not finite.
//
// Execution shape: one lane per ray, persistent near-first traversal over the same 64-B nodes as K2:
// box tests are conservative fp32 slab tests of the ray against both children's oriented boxes (the ray
// projected once per node onto the node frame; make_rayf / ray_child_slabs), and alongnormal bounds each
// child's distance from p along the line (ray_child_line_dist2: the line's interval in it).  alongnormal rays
// are sorted by their source like K2's queries, each lane reading its ray at perm[slot], and their walks start
// from the closest-point entry cut when the tree holds one (traverse_along_pend); visibility rays run
// vertex-major per camera over a Morton order of the vertices (cached per tree), so neighbouring lanes cast
// neighbouring, nearly parallel rays.
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

// 0: miss; 1: proper hit at parameter t; 2: coplanar hit entering at parameter t
__device__ inline int ray_tri(const D3& p, const D3& d, const D3& a, const D3& b, const D3& c, double& tout) {
    const D3 u = vsub(a, p), v = vsub(b, p), w = vsub(c, p);
    const double s0 = det3(u, v, d), s1 = det3(v, w, d), s2 = det3(w, u, d);
    const bool pos = s0 >= 0.0 && s1 >= 0.0 && s2 >= 0.0;
    const bool neg = s0 <= 0.0 && s1 <= 0.0 && s2 <= 0.0;
    if (!pos && !neg) return 0;
    const D3 n = vcross(vsub(b, a), vsub(c, a));
    const double num = vdot(n, u);
    const double den = vdot(n, d);
    if (den == 0.0 || (s0 == 0.0 && s1 == 0.0 && s2 == 0.0)) {
        if (num != 0.0) return 0;
        return coplanar_ray_tri(p, d, a, b, c, tout) ? 2 : 0;
    }
    const double t = num / den;
    if (t < 0.0) return 0;
    tout = t;
    return 1;
}

// CGAL intersection(Plane_3(a, b, c), Line_3(p, p + v)) with direction d = (p + v) - p; false if the
// line is parallel to the plane in this arithmetic
__device__ inline bool cgal_plane_line(const D3& p, const D3& d, const D3& a, const D3& b, const D3& c, D3& out) {
    double A, B, C, D;
    plane_of(a, b, c, A, B, C, D);
    const double num = A * p.x + B * p.y + C * p.z + D;
    const double den = A * d.x + B * d.y + C * d.z;
    if (den == 0.0) return false;
    out = D3{(den * p.x - num * d.x) / den, (den * p.y - num * d.y) / den, (den * p.z - num * d.z) / den};
    return true;
}

__device__ inline D3 ray_dir(const D3& p, const D3& v) { return vsub(vadd(p, v), p); }

// ---- generic traversal: the policy decides box hits (and ordering key) and leaf tests ----
// PF: each next node is loaded into the lane's LDS slot (nb; node_prefetch) as soon as it is chosen; D: LDS stack depth
template <class Pol, bool STATS, bool PF = false, int D = kStack>
__device__ inline void traverse_rays(const BNode* __restrict__ nodes, size_t T, Pol& pol, uint2* __restrict__ lds,
                                     uint2* __restrict__ spill, unsigned& n_nodes, unsigned& n_leaves,
                                     const float4* nb = nullptr, uint32_t wsl = 0) {
    if (T == 1) {
        pol.test(0);
        if (STATS) ++n_leaves;
        return;
    }
    int node = 0, sp = 0;
    if (PF) node_prefetch(nodes, 0, wsl);
    for (size_t guard = 0; guard < T; ++guard) {
        const NodeV nd = PF ? node_from_lds(nb) : load_node(nodes, node);
        if (STATS) ++n_nodes;
        bool h0, h1;
        float k0, k1;
        pol.children(nd, h0, h1, k0, k1);
        const int c0 = nd.child(0), c1 = nd.child(1);
        if (h0 && c0 < 0) {
            pol.test(~c0);
            if (STATS) ++n_leaves;
            h0 = false;
            if (pol.done()) return;
        }
        if (h1 && c1 < 0) {
            pol.test(~c1);
            if (STATS) ++n_leaves;
            h1 = false;
            if (pol.done()) return;
        }
        h0 = h0 && pol.keep(k0);
        h1 = h1 && pol.keep(k1);
        if (h0 && h1) {
            int nearc = c0, farc = c1;
            float kf = k1;
            if (k1 < k0) { nearc = c1; farc = c0; kf = k0; }
            const uint2 e = make_uint2((unsigned)farc, __float_as_uint(kf));
            stack_put<D>(lds, spill, sp, e);
            ++sp;
            node = nearc;
            if (PF) node_prefetch(nodes, node, wsl);
            continue;
        }
        if (h0 || h1) {
            node = h0 ? c0 : c1;
            if (PF) node_prefetch(nodes, node, wsl);
            continue;
        }
        bool found = false;
        while (sp > 0) {
            --sp;
            const uint2 e = stack_get<D>(lds, spill, sp);
            if (pol.keep(__uint_as_float(e.y))) {
                node = (int)e.x;
                found = true;
                break;
            }
        }
        if (!found) break;
        if (PF) node_prefetch(nodes, node, wsl);
    }
}

// nearest hit along +-n (the line through p); key = a lower bound of the squared distance from p to a hit inside the
// child (the line's interval in it, ray_child_line_dist2), which also prunes against the best hit so far
struct AlongPol {
    const TriRec* __restrict__ tris;
    D3 p, n;      // the rays (p, n) and (p, -n); directions ray_dir(p, +-n) are formed per leaf test
    RayF rf;      // the line, fp32 model (its parameter is the distance from p: the children's distance bounds)
    double best;  // distance
    uint32_t best_face;
    int best_leaf;  // the hit point is rebuilt from it at the end (hit()), not carried through the walk
    float limf;     // best^2 (1 + 2^-40) rounded up to fp32 (the unit of the keys), refreshed when best improves
    float capf;     // the entry cut's first phase: the squared radius its start list covers (else +inf)
    __device__ void relim() {
        limf = best == INFINITY ? capf : fminf(__double2float_ru(best * best * kSlack), capf);
    }
    __device__ void children(const NodeV& nd, bool& h0, bool& h1, float& k0, float& k1) const {
        ray_child_line_dist2(nd, rf, h0, h1, k0, k1);
        h0 = h0 && k0 <= limf;
        h1 = h1 && k1 <= limf;
    }
    __device__ bool keep(float key) const { return key <= limf; }
    __device__ bool done() const { return false; }
    // hit point and distance of the ray along +n (k = 0) or -n (k = 1); false: no hit
    __device__ bool along(int k, const D3& a, const D3& b, const D3& c, D3& hit, double& dist) const {
        return along_pn(k, p, n, a, b, c, hit, dist);
    }
    __device__ static bool along_pn(int k, const D3& p, const D3& n, const D3& a, const D3& b, const D3& c, D3& hit,
                                    double& dist) {
        const D3 d = ray_dir(p, k == 0 ? n : D3{-n.x, -n.y, -n.z});
        double t;
        const int kind = ray_tri(p, d, a, b, c, t);
        if (!kind) return false;
        if (kind == 2 || !cgal_plane_line(p, d, a, b, c, hit)) hit = vadd(p, vscale(t, d));
        dist = sqrt(sqdist(hit, p));
        return true;
    }
    __device__ void test(int leaf) {
        D3 a, b, c;
        uint32_t face;
        load_tri(tris, leaf, a, b, c, face);
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            D3 hit;
            double dist;
            if (!along(k, a, b, c, hit, dist)) continue;
            if (dist < best || (dist == best && face < best_face)) {
                best = dist;
                best_face = face;
                best_leaf = leaf;
            }
        }
        relim();
    }
    // the winning hit: the first direction of the best leaf at the best distance (the one test() kept)
    __device__ D3 hit() const {
        D3 out = D3{NAN, NAN, NAN};
        if (best_leaf < 0) return out;
        D3 a, b, c;
        uint32_t face;
        load_tri(tris, best_leaf, a, b, c, face);
        for (int k = 0; k < 2; ++k) {
            D3 h;
            double dist;
            if (along(k, a, b, c, h, dist) && dist == best) return h;
        }
        return out;
    }
};

// nearest_alongnormal with the wave leaf list (K2's scheme, nearest.hip k_knn): a lane appends the leaf children that
// pass its node test to a ring of (leaf << 6 | owner lane) entries in LDS shared by the wave and keeps walking (until
// kAlongPend of its leaves wait); whenever 64 entries wait the wave tests them in a full round, one entry per lane --
// the owner's (p, n) by ds_bpermute, both directions through one copy of the fp64 code -- and the results go back
// through LDS: an atomic min of the distance's bits per owner, then among the entries that reached it an atomic min
// of (face << 32 | leaf): the lexicographic (distance, face) rule of AlongPol::test.  Per-lane leaf tests ran with
// 31 % of the lanes active per VALU instruction (PMC, profiles/r06_c5_pmc_*): the lanes without a leaf idled through
// the two fp64 ray/triangle constructions of the lanes with one.
#ifndef MSH_ALONG_PEND
#define MSH_ALONG_PEND 1
#endif
#ifndef MSH_ALONG_LIST
#define MSH_ALONG_LIST 0
#endif
constexpr int kAlongPend = MSH_ALONG_PEND;
constexpr unsigned kARing = 256;  // ring entries per wave: < 64 left after a full round + <= 128 per step
__device__ inline unsigned lanes_below_r(unsigned long long m) {
    return __builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
}
template <bool STATS>
__device__ inline void traverse_along_list(const BNode* __restrict__ nodes, size_t T, AlongPol& pol, bool active,
                                           uint2* __restrict__ lds, uint2* __restrict__ spill, uint32_t* __restrict__ ring,
                                           unsigned long long* __restrict__ bd, unsigned long long* __restrict__ bfl,
                                           unsigned& n_nodes, unsigned& n_leaves) {
    const int lane = threadIdx.x & 63;
    int node = 0, sp = 0;
    int nq = 0;             // this lane's entries appended since all of them were last evaluated (a bound)
    unsigned last_pos = 0;  // ring counter of this lane's newest entry
    unsigned head = 0, tail = 0;
    size_t guard = 0;
    if (active && T == 1) {  // a single leaf: no node to walk
        node = ~0;
    }
    auto run_rounds = [&](unsigned upto) {
        while (head != upto) {
            const unsigned n = min(64u, upto - head);
            bd[lane] = (unsigned long long)__double_as_longlong(pol.best);
            bfl[lane] = ~0ull;
            const bool valid = (unsigned)lane < n;
            const uint32_t en = ring[(head + (valid ? (unsigned)lane : 0u)) & (kARing - 1)];
            const int src = (int)(en & 63u);
            const int leaf = (int)(en >> 6);
            const D3 p = D3{__shfl(pol.p.x, src), __shfl(pol.p.y, src), __shfl(pol.p.z, src)};
            const D3 nn = D3{__shfl(pol.n.x, src), __shfl(pol.n.y, src), __shfl(pol.n.z, src)};
            D3 a, b, c;
            uint32_t face;
            load_tri(pol.tris, leaf, a, b, c, face);
            double dist = INFINITY;
#pragma nounroll
            for (int k = 0; k < 2; ++k) {
                D3 hit;
                double dk;
                if (AlongPol::along_pn(k, p, nn, a, b, c, hit, dk) && dk < dist) dist = dk;
            }
            const unsigned long long kb = (unsigned long long)__double_as_longlong(dist);
            asm volatile("" ::: "memory");
            if (valid && dist < INFINITY) atomicMin(&bd[src], kb);
            asm volatile("" ::: "memory");
            if (valid && dist < INFINITY && bd[src] == kb) atomicMin(&bfl[src], ((unsigned long long)face << 32) | (unsigned)leaf);
            asm volatile("" ::: "memory");
            const unsigned long long nb = bd[lane], nf = bfl[lane];
            const double nd = __longlong_as_double((long long)nb);
            const uint32_t nface = (uint32_t)(nf >> 32);
            if (nf != ~0ull && (nd < pol.best || (nd == pol.best && nface < pol.best_face))) {
                pol.best = nd;
                pol.best_face = nface;
                pol.best_leaf = (int)(uint32_t)nf;
                pol.relim();
            }
            asm volatile("" ::: "memory");
            if (STATS && valid) ++n_leaves;
            head += n;
        }
        if ((int)(last_pos - head) < 0) nq = 0;  // every entry of this lane is evaluated
    };
    for (;;) {
        const bool can = active && nq < kAlongPend;
        const bool any = __ballot(can) != 0ull;
        if (!any && tail == head) break;
        int l0 = -1, l1 = -1;
        if (can) {
            if (node < 0) {  // a parked leaf (or the single leaf of a one-leaf tree)
                l0 = ~node;
                node = 0;
                active = T > 1 && sp > 0;
                if (active) {
                    active = false;
                    while (sp > 0) {
                        --sp;
                        const uint2 e = stack_get(lds, spill, sp);
                        if (pol.keep(__uint_as_float(e.y))) {
                            node = (int)e.x;
                            active = true;
                            break;
                        }
                    }
                }
            } else {
                const NodeV nd = load_node(nodes, node);
                if (STATS) ++n_nodes;
                bool h0, h1;
                float k0, k1;
                pol.children(nd, h0, h1, k0, k1);
                const int c0 = nd.child(0), c1 = nd.child(1);
                const bool lf0 = h0 && c0 < 0, lf1 = h1 && c1 < 0;
                const bool in0 = h0 && c0 >= 0, in1 = h1 && c1 >= 0;
                if (lf0 && lf1 && nq + 1 >= kAlongPend) {  // room for one: queue the nearer, park the farther
                    const bool first1 = k1 < k0;
                    l0 = first1 ? ~c1 : ~c0;
                    node = first1 ? c0 : c1;  // negative: a parked leaf, handed over by the next step
                } else {
                    if (lf0) l0 = ~c0;
                    if (lf1) { if (l0 < 0) l0 = ~c1; else l1 = ~c1; }
                    bool more = true;
                    if (in0 && in1) {
                        int nearc = c0, farc = c1;
                        float kf = k1;
                        if (k1 < k0) { nearc = c1; farc = c0; kf = k0; }
                        stack_put(lds, spill, sp, make_uint2((unsigned)farc, __float_as_uint(kf)));
                        ++sp;
                        node = nearc;
                    } else if (in0) {
                        node = c0;
                    } else if (in1) {
                        node = c1;
                    } else {
                        more = false;
                        while (sp > 0) {
                            --sp;
                            const uint2 e = stack_get(lds, spill, sp);
                            if (pol.keep(__uint_as_float(e.y))) {
                                node = (int)e.x;
                                more = true;
                                break;
                            }
                        }
                    }
                    active = more;
                }
                if (++guard >= T) active = false;  // each node is entered once: a corrupt tree
            }
        }
        // append this step's leaves (at most two per lane) to the ring, in lane order
        const unsigned long long m1 = __ballot(l0 >= 0), m2 = __ballot(l1 >= 0);
        const unsigned pos = tail + lanes_below_r(m1) + lanes_below_r(m2);
        if (l0 >= 0) {
            ring[pos & (kARing - 1)] = ((uint32_t)l0 << 6) | (uint32_t)lane;
            last_pos = pos;
            ++nq;
        }
        if (l1 >= 0) {
            ring[(pos + 1) & (kARing - 1)] = ((uint32_t)l1 << 6) | (uint32_t)lane;
            last_pos = pos + 1;
            ++nq;
        }
        tail += (unsigned)(__popcll(m1) + __popcll(m2));
        const unsigned upto = any ? head + ((tail - head) & ~63u) : tail;
        if (upto != head) run_rounds(upto);
    }
}

// nearest_alongnormal with postponed leaf tests and no leaf list: a lane that reaches a leaf within reach keeps it
// pending and stops; once every walking lane of the wave holds one, they all test their own leaf together (one call
// site of the fp64 code), so the construction runs with every lane that has a leaf instead of one lane at a time.
// A lane pends at most one leaf: its bound is never stale (the wave leaf list, which lets lanes walk on with up to
// kAlongPend leaves waiting, walked 34.4 nodes per ray instead of 29.5 at kAlongPend >= 4; at 1 it ran 4.75 ms against
// 5.02 for per-lane tests, profiles/r06_c5_along_list_pend_ab.jsonl, and this form needs neither its LDS ring nor the
// owners' rows fetched by ds_bpermute).
// The alongnormal kernel's LDS stack depth.  12 entries (24 KB per block) + the node slots (16 KB) would keep a block
// at 40 KB, 4 blocks per CU: at 4 waves per SIMD (128 VGPRs, two reloads in the walk) C5 ran 4.53-4.61 ms against
// 4.50-4.56 at 3 waves with 16 entries (profiles/r06_c5_along_waves_ab.jsonl).
#ifndef MSH_ALONG_STACK
#define MSH_ALONG_STACK 16
#endif
constexpr int kAlongStack = MSH_ALONG_STACK;
// visibility: the node prefetch into LDS with a 12-entry stack (24 KB + 16 KB of node slots per block: 4 blocks per
// CU, the kernel's 4 waves per SIMD) measured 58.8-59.8 against 50.9-51.4 ms for C5's 160M rays
// (profiles/r06_c5_vis_pf_ab.jsonl): off
#ifndef MSH_VIS_PF
#define MSH_VIS_PF 0
#endif
constexpr int kVisStack = MSH_VIS_PF ? 12 : kStack;
// PF: the lane's next node is loaded into its LDS slot as soon as it is chosen (node_prefetch, as k_knn's list
// path), so its latency overlaps the wave's leaf phases and the loop's bookkeeping
#ifndef MSH_ALONG_PF
#define MSH_ALONG_PF 1
#endif
#ifndef MSH_RAY_TILE_PF
#define MSH_RAY_TILE_PF 1
#endif
// alongnormal walks start from the closest-point entry cut when the tree holds one (traverse_along_pend)
#ifndef MSH_ALONG_CUT
#define MSH_ALONG_CUT 1
#endif
// rec / rho (round 6): the ray's cell of the closest-point entry cut and the radius around p its start list covers (every
// subtree left out of it is farther than rho from p: k_rays).  The walk first runs from the list with the bound capped
// at rho; a hit within rho is then the answer (every face with a hit that near lies in the list's subtrees, and they
// were walked with the usual bound below the cap).  Otherwise the walk runs again from the root, keeping its best hit.
template <bool STATS>
__device__ inline void traverse_along_pend(const BNode* __restrict__ nodes, size_t T, AlongPol& pol, bool active,
                                           uint2* __restrict__ lds, uint2* __restrict__ spill, unsigned& n_nodes,
                                           unsigned& n_leaves, const float4* nb, uint32_t wsl,
                                           const uint32_t* __restrict__ rec = nullptr, bool wide = false,
                                           float rho = -1.f) {
    int node = 0, sp = 0;
    int pend = -1;  // this lane's leaf waiting for the wave's leaf phase
    size_t guard = 0;
    if (active && T == 1) {
        pend = 0;
        active = false;
    }
    auto fetch = [&]() {
        if (MSH_ALONG_PF && node >= 0) node_prefetch(nodes, node, wsl);
    };
    bool phase_a = false;
    if (active && rec) {  // the start list, nearest first: the first entry is the node, the others stacked (key 0)
        int ent[kCutK];
        int m = 0;
#pragma unroll
        for (int k = 0; k < kCutK; ++k) {
            const uint32_t e = wide ? rec[2 + 2 * k] : rec[1 + k];
            const bool ok = wide ? e != kCutEmpty : (int)e >= 0;
            ent[k] = ok ? (wide ? (int)e : __builtin_amdgcn_sbfe((int)e, 0, 21)) : 0;
            if (ok) m = k + 1;
        }
        if (m > 0) {
#pragma unroll
            for (int k = kCutK - 1; k >= 1; --k)
                if (k < m) {
                    stack_put<kAlongStack>(lds, spill, sp, make_uint2((unsigned)ent[k], 0u));
                    ++sp;
                }
            node = ent[0];
            phase_a = true;
        }
    }
    if (active) fetch();
    for (;;) {
        if (phase_a && !active && pend < 0) {  // the start list is exhausted
            phase_a = false;
            if (!(pol.best <= (double)rho)) {  // no hit within rho: the whole tree, from the root
                pol.capf = INFINITY;
                pol.relim();
                node = 0;
                sp = 0;
                guard = 0;
                active = true;
                fetch();
            }
        }
        const bool can = active && pend < 0;
        if (__ballot(can) == 0ull) {
            if (__ballot(pend >= 0) == 0ull) break;
            if (pend >= 0) {  // every walking lane holds a leaf: all of them test theirs
                pol.test(pend);
                if (STATS) ++n_leaves;
                pend = -1;
            }
            continue;
        }
        if (!can) continue;
        if (node < 0) {  // a parked leaf: it is this step's leaf; the walk goes on from the stack
            pend = ~node;
            node = 0;
        } else {
            const NodeV nd = MSH_ALONG_PF ? node_from_lds(nb) : load_node(nodes, node);
            if (STATS) ++n_nodes;
            bool h0, h1;
            float k0, k1;
            pol.children(nd, h0, h1, k0, k1);
            const int c0 = nd.child(0), c1 = nd.child(1);
            const bool lf0 = h0 && c0 < 0, lf1 = h1 && c1 < 0;
            const bool in0 = h0 && c0 >= 0, in1 = h1 && c1 >= 0;
            if (lf0 && lf1) {  // two leaves: the nearer now, the farther parked as the next step's node
                const bool first1 = k1 < k0;
                pend = first1 ? ~c1 : ~c0;
                node = first1 ? c0 : c1;
                if (++guard >= T) active = false;
                continue;
            }
            if (lf0) pend = ~c0;
            if (lf1) pend = ~c1;
            if (in0 && in1) {
                int nearc = c0, farc = c1;
                float kf = k1;
                if (k1 < k0) { nearc = c1; farc = c0; kf = k0; }
                stack_put<kAlongStack>(lds, spill, sp, make_uint2((unsigned)farc, __float_as_uint(kf)));
                ++sp;
                node = nearc;
                fetch();
                if (++guard >= T) active = false;
                continue;
            }
            if (in0 || in1) {
                node = in0 ? c0 : c1;
                fetch();
                if (++guard >= T) active = false;
                continue;
            }
            if (++guard >= T) {
                active = false;
                continue;
            }
        }
        // nothing to descend into: the next entry of the stack within the bound (the pending leaf, if any, is tested
        // before it is used: the bound may only tighten, so popping now with the older bound is conservative)
        bool more = false;
        while (sp > 0) {
            --sp;
            const uint2 e = stack_get<kAlongStack>(lds, spill, sp);
            if (pol.keep(__uint_as_float(e.y))) {
                node = (int)e.x;
                more = true;
                break;
            }
        }
        active = more;
        if (more) fetch();
    }
}

// any hit of the closed ray src + t d, t >= 0; key = entry parameter
struct AnyPol {
    const TriRec* __restrict__ tris;
    D3 src, d;
    RayF rf;
    bool hit;
    __device__ void children(const NodeV& nd, bool& h0, bool& h1, float& k0, float& k1) const {
        ray_child_slabs(nd, rf, h0, h1, k0, k1);
    }
    __device__ bool keep(float) const { return !hit; }
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
    // alongnormal (slot order when res != nullptr)
    const double* p;
    const double* n;
    size_t S;
    const uint32_t* perm;  // slot -> caller's row (sorted rays), nullptr: identity
    bool lazy;             // p / n are the caller's rows, read at perm[slot] (not gathered into slot order)
    double* out_dist;
    uint32_t* out_face;
    double* out_pt;
    // visibility: cameras x vertices [v0, v0 + nv); output row stride nv
    const double* v;
    const uint32_t* vorder;  // Morton order of the vertices (nullptr: identity)
    size_t P, v0, nv;
    const double* cams;
    const double* normals;
    const double* sensors;
    double min_dist;
    uint32_t* vis;
    double* ndc;
    // common
    unsigned long long* stats;  // STATS launches: [0] nodes loaded, [1] leaf tests (outputs not written)
    unsigned* counters;
    unsigned ntiles;
    uint2* spill;
    int spill_depth;
    double org[3];  // tree origin
    double M;       // the tree's half-diagonal (hits lie within M of org)
    // alongnormal: the tree's closest-point entry cut (traverse_along_pend's first phase); nullptr: from the root
    const uint32_t* cut;
    int cut_wide, cut_G;
    double cut_lo[3], cut_iw[3];
    double cut_r;  // the cells' half-diagonal as the cut's build took it, rounded down
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

__device__ inline bool finite_d3(const D3& x) { return isfinite(x.x) && isfinite(x.y) && isfinite(x.z); }

// waves per SIMD: visibility 4 (127 VGPRs, no spills); alongnormal 3 (168 VGPRs, 48 KB of LDS per block with the node
// slots; at 4 the per-lane fp64 leaf test spilled 37 VGPRs: C5 7.41 vs 6.62 ms in round 2, 5.74 vs 4.98 ms in round 6
// before the postponed leaf tests, profiles/r06_c5_along_ab.jsonl)
#ifndef MSH_ALONG_WAVES
#define MSH_ALONG_WAVES 3
#endif
template <int MODE, bool STATS>  // MODE 0 alongnormal, 1 visibility
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(MODE == 0 ? MSH_ALONG_WAVES : 4))) void k_rays(RayArgs a) {
    unsigned n_nodes = 0, n_leaves = 0;
    __shared__ uint2 stk[(MODE == 0 ? kAlongStack : kVisStack) * kBlock];
    // alongnormal: each wave's leaf ring + per-owner (distance bits, face << 32 | leaf) slots
    __shared__ uint32_t rsh[MODE == 0 && MSH_ALONG_LIST ? 4 * (kARing + 64 * 4) : 1];
    const int tid = threadIdx.x, lane = tid & 63;
    uint2* lds = stk + tid;
    uint32_t* ring = rsh + (MODE == 0 && MSH_ALONG_LIST ? (tid >> 6) * (kARing + 64 * 4) : 0);
    [[maybe_unused]] unsigned long long* rbd = reinterpret_cast<unsigned long long*>(ring + kARing);
    [[maybe_unused]] unsigned long long* rbfl = rbd + 64;
    // alongnormal: each wave's node slots (node_prefetch: LDS address from a wave-uniform index, so M0 is scalar)
    constexpr bool kPF = MODE == 0 ? MSH_ALONG_PF : MSH_VIS_PF;
    __shared__ float4 nbuf[kPF ? 4 * kBlock : 1];
    const int wv_u = __builtin_amdgcn_readfirstlane(tid >> 6);
    const uint32_t wsl = (uint32_t)(size_t)(__attribute__((address_space(3))) float4*)(nbuf + (kPF ? wv_u * 256 : 0));
    const float4* nb = nbuf + (kPF ? (tid >> 6) * 256 + lane : 0);
    uint2* spill = a.spill ? a.spill + (size_t)blockIdx.x * kBlock * (size_t)a.spill_depth + tid : nullptr;
    const unsigned group = blockIdx.x & 7u;
    const D3 org = D3{a.org[0], a.org[1], a.org[2]};
#if MSH_RAY_TILE_PF
    // the next tile of the wave's group is claimed while the current one's rays load (nearest.hip MSH_TILE_PF)
    const unsigned glo = (unsigned)(((unsigned long long)a.ntiles * group) >> 3);
    const unsigned ghi = (unsigned)(((unsigned long long)a.ntiles * (group + 1)) >> 3);
    unsigned nxt = ~0u;
#endif
    for (;;) {
        unsigned tile = 0;
#if MSH_RAY_TILE_PF
        if (lane == 0) tile = (nxt != ~0u && glo + nxt < ghi) ? glo + nxt : dequeue_tile_r(a.counters, a.ntiles, group);
#else
        if (lane == 0) tile = dequeue_tile_r(a.counters, a.ntiles, group);
#endif
        tile = __shfl(tile, 0);
        if (tile >= a.ntiles) break;
        const size_t i = (size_t)tile * 64 + lane;
#if MSH_RAY_TILE_PF
        if (lane == 0) nxt = glo < ghi ? atomicAdd(&a.counters[group * 32], 1u) : ~0u;
#endif
        if (MODE == 0) {
            // every lane stays in the wave's loop (the leaf rounds use all 64); a lane past the rays only helps
            const bool live = i < a.S;
            const size_t r = live && a.perm ? (size_t)a.perm[i] : i;  // the caller's row
            const size_t ri = a.lazy ? r : i;
            const D3 p = live ? D3{a.p[3 * ri], a.p[3 * ri + 1], a.p[3 * ri + 2]} : D3{0.0, 0.0, 0.0};
            const D3 n = live ? D3{a.n[3 * ri], a.n[3 * ri + 1], a.n[3 * ri + 2]} : D3{0.0, 0.0, 1.0};
            const D3 dp = ray_dir(p, n), pr = vsub(p, org);
            AlongPol pol{a.tris, p, n, make_rayf(pr, dp, a.M, true), INFINITY, MSH_NO_FACE, -1, INFINITY, INFINITY};
            const bool go = live && finite_d3(p) && finite_d3(dp);
            // the entry cut's cell of p: its start list covers every face within rho of p, rho = R - |p - c| with R
            // the radius the build kept around the centre c (64-B records hold it; else d(c) + 2r, d(c): c's distance
            // to its hint face, the face the build found closest to c); both rounded down
            const uint32_t* rec = nullptr;
            float rho = -1.f;
            if (a.cut && go) {
                const double G = (double)a.cut_G;
                const double ux = (p.x - a.cut_lo[0]) * a.cut_iw[0], uy = (p.y - a.cut_lo[1]) * a.cut_iw[1],
                             uz = (p.z - a.cut_lo[2]) * a.cut_iw[2];
                if (ux >= 0.0 && ux < G && uy >= 0.0 && uy < G && uz >= 0.0 && uz < G) {
                    const unsigned ix = (unsigned)ux, iy = (unsigned)uy, iz = (unsigned)uz;
                    const uint32_t* r = a.cut + (((size_t)iz * a.cut_G + iy) * a.cut_G + ix) * (a.cut_wide ? 16 : 8);
                    const int hint = (int)r[0];
                    if (hint >= 0) {
                        const D3 c = D3{a.cut_lo[0] + ((double)ix + 0.5) / a.cut_iw[0],
                                        a.cut_lo[1] + ((double)iy + 0.5) / a.cut_iw[1],
                                        a.cut_lo[2] + ((double)iz + 0.5) / a.cut_iw[2]};
                        double R;
                        if (a.cut_wide) {
                            R = (double)__uint_as_float(r[1]);  // the build's radius (k_cut_level)
                        } else {  // 32-B records have no room for it: d(c) from the hint face
                            D3 ta, tb, tc, o;
                            uint32_t f;
                            int part;
                            load_tri(a.tris, hint, ta, tb, tc, f);
                            R = (sqrt(closest_on_triangle(c, ta, tb, tc, o, part)) + 2.0 * a.cut_r) * (1.0 - 1e-9);
                        }
                        const double rr = (R - sqrt(sqdist(p, c))) * (1.0 - 1e-9);
                        if (rr > 0.0) {
                            rec = r;
                            rho = __double2float_rd(rr);
                            pol.capf = __double2float_ru((double)rho * (double)rho * kSlack);
                            pol.relim();
                        }
                    }
                }
            }
#if MSH_ALONG_LIST
            traverse_along_list<STATS>(a.nodes, a.T, pol, live && finite_d3(p) && finite_d3(dp), lds, spill, ring, rbd,
                                       rbfl, n_nodes, n_leaves);
#else
            traverse_along_pend<STATS>(a.nodes, a.T, pol, go, lds, spill, n_nodes, n_leaves, nb, wsl, rec,
                                       a.cut_wide != 0, rho);
#endif
            if (STATS || !live) continue;
            const double dist = pol.best == INFINITY ? 1e100 : pol.best;
            a.out_dist[r] = dist;  // scattered stores to the caller's row
            a.out_face[r] = pol.best_face;
            const D3 h = pol.hit();
            a.out_pt[3 * r] = h.x;
            a.out_pt[3 * r + 1] = h.y;
            a.out_pt[3 * r + 2] = h.z;
        } else {
            if (i >= a.S) continue;
            const size_t ic = i / a.nv, k = i - ic * a.nv;
            const size_t iv = a.vorder ? (size_t)a.vorder[k] : a.v0 + k;  // vertex (global index)
            const size_t o = ic * a.nv + (iv - a.v0);                        // output element
            const D3 cam = D3{a.cams[3 * ic], a.cams[3 * ic + 1], a.cams[3 * ic + 2]};
            const D3 vv = D3{a.v[3 * iv], a.v[3 * iv + 1], a.v[3 * iv + 2]};
            D3 dir = vsub(cam, vv);
            const double len = sqrt(vdot(dir, dir));
            dir = D3{dir.x / len, dir.y / len, dir.z / len};
            const D3 src = vadd(vv, vscale(a.min_dist, dir));
            const D3 d = ray_dir(src, dir);
            AnyPol pol{a.tris, src, d, make_rayf(vsub(src, org), d, a.M, false), false};
            if (finite_d3(src) && finite_d3(d))
                traverse_rays<AnyPol, STATS, kPF, kVisStack>(a.nodes, a.T, pol, lds, spill, n_nodes, n_leaves, nb, wsl);
            if (STATS) continue;
            const uint32_t reach = pol.hit ? 0u : 1u;
            a.ndc[o] = a.normals ? vdot(D3{a.normals[3 * iv], a.normals[3 * iv + 1], a.normals[3 * iv + 2]}, dir) : 0.0;
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
            a.vis[o] = out;
        }
    }
    // a lane that stopped may still have a node prefetch in flight: it lands before the block's LDS is released
    if constexpr (kPF) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (STATS) {
        atomicAdd(&a.stats[0], (unsigned long long)n_nodes);
        atomicAdd(&a.stats[1], (unsigned long long)n_leaves);
    }
}

static int device_cus_r(int dev) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
    return n;
}

template <int MODE, bool STATS>
static int launch_rays(msh_tree* tree, RayArgs a, size_t nrays, hipStream_t s, const char* timer) {
    if (nrays == 0) return MSH_OK;
    if (nrays > (size_t)0xFFFFFFFFull * 64) {
        set_error("too many rays (%zu)", nrays);
        return MSH_EINVAL;
    }
    a.S = nrays;
    for (int k = 0; k < 3; ++k) a.org[k] = tree->origin[k];
    a.M = tree->half_diag;
    a.ntiles = (unsigned)((nrays + 63) / 64);
    const unsigned nblk = std::min<unsigned>((a.ntiles + 3) / 4, (unsigned)device_cus_r(tree->device) * 5u);
    MSH_TRY(tree->ws.counters.reserve(9 * 32 * sizeof(unsigned)));
    a.counters = tree->ws.counters.as<unsigned>();
    MSH_HIP(hipMemsetAsync(a.counters, 0, 8 * 32 * sizeof(unsigned), s));
    a.spill = nullptr;
    a.spill_depth = 0;
    const int lds_depth = MODE == 0 ? kAlongStack : kVisStack;
    const int need = tree->max_depth + 1 + (a.cut ? kCutK : 0);  // + the entry cut's start list
    if (need > lds_depth) {
        a.spill_depth = need - lds_depth + 1;
        MSH_TRY(tree->ws.spill.reserve((size_t)nblk * kBlock * (size_t)a.spill_depth * sizeof(uint2)));
        a.spill = tree->ws.spill.as<uint2>();
    }
    TimedLaunch tl(timer, s);
    k_rays<MODE, STATS><<<nblk, kBlock, 0, s>>>(a);
    MSH_HIP(hipGetLastError());
    return MSH_OK;
}

// the tree's closest-point entry cut for the alongnormal walks (traverse_along_pend's first phase)
static void along_cut(const msh_tree* tree, RayArgs& a) {
    if (!MSH_ALONG_CUT || !tree->d_cut || tree->B != 1 || tree->cut_G <= 0) return;
    a.cut = tree->d_cut;
    a.cut_wide = tree->cut_wide;
    a.cut_G = tree->cut_G;
    double w2 = 0.0;
    for (int k = 0; k < 3; ++k) {
        a.cut_lo[k] = tree->cut_lo[k];
        a.cut_iw[k] = tree->cut_iw[k];
        const double w = 1.0 / tree->cut_iw[k];
        w2 += w * w;
    }
    a.cut_r = 0.5 * sqrt(w2) * 1.001 * (1.0 - 1e-9);  // k_cut_level's r, rounded down
}

int launch_alongnormal(const msh_tree* tree, const QueryOrder& ord, size_t S, const SlotOut& o, hipStream_t s) {
    msh_tree* t = const_cast<msh_tree*>(tree);
    RayArgs a{};
    along_cut(tree, a);
    a.nodes = tree->d_nodes; a.tris = static_cast<const TriRec*>(tree->d_leaves); a.T = tree->T;
    a.p = ord.q; a.n = ord.n;
    a.perm = ord.perm;  // rays run in slot order and store their answers to the caller's rows
    a.lazy = !ord.gathered;
    a.out_dist = o.w; a.out_face = o.face; a.out_pt = o.pt;
    return launch_rays<0, false>(t, a, S, s, "alongnormal");
}

// Morton order of main-mesh vertices [v0, v0 + n) in the scene box (visibility sources): keys of vertex
// v0 + i and values v0 + i (global indices)
__global__ __launch_bounds__(kBlock) void k_vertex_morton(const double* __restrict__ v, size_t v0, size_t n, float lx,
                                                          float ly, float lz, float hx, float hy, float hz,
                                                          uint32_t* __restrict__ keys, uint32_t* __restrict__ vals) {
    const size_t i = (size_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const float e[3] = {hx - lx, hy - ly, hz - lz}, l[3] = {lx, ly, lz};
    uint32_t c[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        float x = e[k] > 0.f ? ((float)v[3 * (v0 + i) + k] - l[k]) / e[k] : 0.5f;
        x = fminf(fmaxf(x * 1024.f, 0.f), 1023.f);
        uint32_t b = (uint32_t)x;
        b = (b * 0x00010001u) & 0xFF0000FFu;
        b = (b * 0x00000101u) & 0x0F00F00Fu;
        b = (b * 0x00000011u) & 0xC30C30C3u;
        b = (b * 0x00000005u) & 0x49249249u;
        c[k] = b;
    }
    keys[i] = (c[0] << 2) | (c[1] << 1) | c[2];
    vals[i] = (uint32_t)(v0 + i);
}

// Morton order of the vertex range [v0, v0 + nv), cached on the handle: the whole mesh in d_vorder, the
// last vertex shard asked for (visibility_sharded: one range per rank) in d_vorder_shard.  A shard's order
// is the whole mesh's order restricted to the shard (the same keys, a stable sort), so a shard's rays run
// as coherently as the whole mesh's.  The buffer is published on the handle only after the sort has been
// enqueued successfully (a failed build leaves no half-initialised order behind).
static int vertex_order(msh_tree* t, size_t v0, size_t nv, const uint32_t** order, hipStream_t s) {
    *order = nullptr;
    if (nv < 4096) return MSH_OK;  // small ranges: caller order
    const bool whole = v0 == 0 && nv == t->P;
    if (whole && t->d_vorder) { *order = t->d_vorder; return MSH_OK; }
    if (!whole && t->d_vorder_shard && t->vshard_v0 == v0 && t->vshard_nv == nv) {
        *order = t->d_vorder_shard;
        return MSH_OK;
    }
    Workspace& ws = t->ws;
    MSH_TRY(ws.keys.reserve(nv * sizeof(uint32_t)));
    MSH_TRY(ws.keys_alt.reserve(nv * sizeof(uint32_t)));
    MSH_TRY(ws.vals_alt.reserve(nv * sizeof(uint32_t)));
    uint32_t* buf = nullptr;
    MSH_HIP(dmalloc(&buf, nv * sizeof(uint32_t)));
    k_vertex_morton<<<(unsigned)((nv + kBlock - 1) / kBlock), kBlock, 0, s>>>(
        t->d_v, v0, nv, t->scene_lo[0], t->scene_lo[1], t->scene_lo[2], t->scene_hi[0], t->scene_hi[1],
        t->scene_hi[2], ws.keys.as<uint32_t>(), buf);
    int st = hipGetLastError() == hipSuccess ? MSH_OK : MSH_EDEVICE;
    if (st == MSH_OK)
        st = radix_sort_pairs(ws.keys.as<uint32_t>(), buf, ws.keys_alt.as<uint32_t>(), ws.vals_alt.as<uint32_t>(), nv,
                              30, ws, s);
    if (st != MSH_OK) {
        if (st == MSH_EDEVICE) set_error("vertex Morton order: kernel launch failed");
        (void)hipStreamSynchronize(s);  // the buffer may still be in use by enqueued work
        (void)dfree(buf);
        return st;
    }
    if (whole) {
        t->d_vorder = buf;
    } else {
        if (t->d_vorder_shard) {
            // the previous shard's launches may still run on another caller stream: wait for the end of the
            // handle's last launch sequence (ws_done, recorded on whatever stream it ran) and for this stream
            if (t->ws_done) (void)hipEventSynchronize(t->ws_done);
            (void)hipStreamSynchronize(s);
            (void)dfree(t->d_vorder_shard);
        }
        t->d_vorder_shard = buf;
        t->vshard_v0 = v0;
        t->vshard_nv = nv;
    }
    *order = buf;
    return MSH_OK;
}

int launch_visibility(const msh_tree* tree, const double* d_cams, size_t C, const double* d_normals,
                      const double* d_sensors, double min_dist, size_t v0, size_t nv, uint32_t* d_vis, double* d_ndc,
                      hipStream_t s) {
    msh_tree* t = const_cast<msh_tree*>(tree);
    RayArgs a{};
    a.nodes = tree->d_nodes; a.tris = static_cast<const TriRec*>(tree->d_leaves); a.T = tree->T;
    a.v = tree->d_v; a.P = tree->P; a.v0 = v0; a.nv = nv;
    a.cams = d_cams; a.normals = d_normals; a.sensors = d_sensors;
    a.min_dist = min_dist; a.vis = d_vis; a.ndc = d_ndc;
    if (nv == 0 || C == 0) return MSH_OK;
    MSH_TRY(vertex_order(t, v0, nv, &a.vorder, s));  // Morton-ordered sources (whole mesh or shard)
    return launch_rays<1, false>(t, a, C * nv, s, "visibility");
}

int launch_alongnormal_stats(const msh_tree* tree, const QueryOrder& ord, size_t S, unsigned long long* d_counts,
                             hipStream_t s) {
    msh_tree* t = const_cast<msh_tree*>(tree);
    RayArgs a{};
    along_cut(tree, a);
    a.nodes = tree->d_nodes; a.tris = static_cast<const TriRec*>(tree->d_leaves); a.T = tree->T;
    a.p = ord.q; a.n = ord.n;
    a.perm = ord.gathered ? nullptr : ord.perm;
    a.lazy = !ord.gathered;
    a.stats = d_counts;
    return launch_rays<0, true>(t, a, S, s, "alongnormal_stats");
}

int launch_visibility_stats(const msh_tree* tree, const double* d_cams, size_t C, double min_dist,
                            unsigned long long* d_counts, hipStream_t s) {
    msh_tree* t = const_cast<msh_tree*>(tree);
    RayArgs a{};
    a.nodes = tree->d_nodes; a.tris = static_cast<const TriRec*>(tree->d_leaves); a.T = tree->T;
    a.v = tree->d_v; a.P = tree->P; a.v0 = 0; a.nv = tree->P;
    a.cams = d_cams; a.min_dist = min_dist;
    a.stats = d_counts;
    if (C == 0 || tree->P == 0) return MSH_OK;
    MSH_TRY(vertex_order(t, 0, tree->P, &a.vorder, s));
    return launch_rays<1, true>(t, a, C * tree->P, s, "visibility_stats");
}

}  // namespace msh
