// K2 + K3 — closest-point traversal with fused fp64 refinement (replaces
// spatialsearchmodule.cpp:165-220 aabbtree_nearest and CGAL's closest_point_and_primitive), plus the
// normal-weighted metric variant (K7, aabb_normals.cpp:112-190), the vertex nearest-neighbour variant
// (K8, search.ClosestPointTree) and the barycentric variant (K9: nearest + Heidrich weights of the
// closest point, mesh.py:218-222 / geometry/barycentric_coordinates_of_projection.py:9-49).
//
// Query pipeline (sorted launches):
//   k_query_morton -> radix sort (sort.hip) -> the closest-point traversal reads query row perm[i] for slot
//   i straight from the caller's array and stores its answer straight to the caller's row perm[i] (face,
//   part, point: scattered 4 + 4 + 24-B stores); only the leader phases also write a 32-B slot-order
//   record, because followers take their hints from them.  The ray, normals-metric and point-tree paths
//   gather the rows into slot order (k_gather_rows) and restore the caller's order from slot-order records
//   (k_unpermute).  Unsorted launches read and write the caller's arrays directly.
//
// Execution shape (gfx950):
//   Pass 1 (k_knn): persistent grid; each WAVE dequeues 64-query tiles from one of 8 XCD-group
//     counters (group = blockIdx % 8 labels the blocks sharing an XCD; each counter owns a contiguous
//     eighth of the Morton-sorted queries, so an XCD's L2 serves one region of the BVH; exhausted
//     groups steal).  One lane per query, near-child-first depth-first traversal: one 64-B node read
//     bounds both children by their fp32 oriented boxes; the far child is pushed (16-entry LDS stack
//     per lane, [depth][lane] layout, deeper entries spill to a lane-interleaved global area sized
//     from the tree depth).  Leaf children that survive the bound go to the wave leaf list, a ring in LDS
//     the wave evaluates in full rounds of 64 with CGAL's exact fp64 construction (postponed leaves,
//     Aila & Laine, dealt to every lane of the wave).  Pass 1 runs over super-leader slots, then leader
//     slots, then followers, each starting from the leaf of its nearest leader's answer.
//     The fp32 pruning radius is cached per lane and refreshed only when the best distance changes.
//     A lane that exceeds `budget` node steps stops and appends its query (with its exact best so far)
//     to a deferred list: queries near the centre of a closed surface are equidistant from most of it
//     and would otherwise hold their whole wave for ~10^6 steps.
//   Pass 2 (k_knn_coop): one WAVE per deferred query, dealt from an atomic counter.  The wave walks a
//     last-in-first-out list of subtrees in LDS, 64 entries at a time (one per lane): children within the
//     bound are pushed back (compacted by ballot), leaf children are tested on the spot, and the wave
//     shares the best bound (wave min) after every round.  A list that would outgrow LDS is dealt to the
//     lanes' own stacks for depth-first walks.
// Ties: the lexicographic minimum of (squared distance, face index) — deterministic and independent of
// traversal order or of how the work was split (every box within best*(1+2^-40) is visited).
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <vector>
#include <type_traits>

#include "internal.h"


namespace msh {

struct DeferRec {
    uint32_t slot;
    uint32_t face;
    int32_t leaf;
    uint32_t roff;   // first of the query's resume entries (KnnArgs::resume)
    double best;
    uint32_t rcnt;   // resume entries: pass 1's unexplored work (0: pass 2 starts at the root)
    uint32_t sbound; // pass 2, an item split over waves: their shared bound, fp32 bits rounded up (atomicMin)
};
static_assert(sizeof(DeferRec) == 32, "DeferRec must be 32 B");

// Pass 2 ends with its longest item: on C3 every deferred query lies near the sphere's centre, and their walks grow
// steeply as they approach it (12.5M shard: 8,239 items of 250 node visits on average, the longest 19,688;
// profiles/r06_c3_shard_pass2_r5_vs_r6.jsonl, r06_c3_p2_items.json).  So the items whose pass-1 distance is within
// kP2Heavy of the largest one (k_p2_plan) are split over kP2Split waves, dealt before the others: part p takes every
// kP2Split-th of the item's resume entries, the parts share their bound through DeferRec::sbound, and k_knn_combine
// merges their candidates.  (Splitting every item: 12.5M shard pass 2 0.63 -> 0.50 ms at 2 parts, 0.68 at 4; 100M
// 1.14 -> 3.2 ms at 4: the parts' fixed costs.)
#ifndef MSH_P2_SPLIT
#define MSH_P2_SPLIT 8
#endif
#ifndef MSH_P2_HEAVY
#define MSH_P2_HEAVY 0.97
#endif
constexpr unsigned kP2Split = MSH_P2_SPLIT;
constexpr double kP2Heavy = MSH_P2_HEAVY;      // split items with sqrt(best) >= kP2Heavy sqrt(the largest best)
constexpr unsigned kP2SplitItems = 1u << 16;  // at most this many items split: 8 MB of candidates
constexpr uint32_t kP2Whole = 0xFFFFFFFFu;    // DeferRec::sbound of an item run whole (k_p2_plan)
struct P2Cand {
    double best;
    uint32_t face;
    int32_t leaf;
};

// MODE: 0 closest point (face, part, point), 1 normals metric (face, point), 2 vertex NN (index,
// distance), 3 closest point + barycentric weights (face, point, weights)
struct KnnArgs {
    const BNode* nodes;
    const void* leaves;
    size_t T;
    const double* q;       // query rows in slot order (Morton-sorted copy, or the caller's array)
    const double* n;       // MODE 1: query normals in slot order
    const uint32_t* perm;  // slot -> caller's query index (nullptr: identity)
    const uint32_t* qperm; // non-null: q holds the caller's rows and slot i reads row qperm[i]
    uint32_t* inv_w;       // with qperm: pass 1 records inv_w[qperm[i]] = i
    size_t S;
    QRes* res;             // slot-order records (sorted path); nullptr: write the caller's arrays below
    double* res_w;         // MODE 3 slot-order barycentric weights (3 per slot)
    uint32_t* out_face;
    uint32_t* out_part;
    double* out_pt;
    double* out_dist;
    double* out_w;
    double eps;
    double org[3];  // tree origin: fp32 node bounds are relative to it
    double tm;      // tree_margin(tree->half_diag): the node bounds' share of the query margin (make_qf)
    // batched trees (msh_batch_build): slot i belongs to mesh i / qper (the batched sort is mesh-major),
    // whose root is node mesh * npm and whose origin is orgs[3 * mesh]; orgs == nullptr: single tree
    const double* orgs;
    size_t qper;
    size_t npm;
    size_t root0;  // batched trees: root of the launch's first mesh (a launch over meshes [mesh0, ...): mesh0 * npm)
    unsigned* counters;
    unsigned ntiles;
    uint2* spill;
    int spill_depth;
    unsigned long long* stats;
    unsigned budget;
    // leader / follower ordering (sorted closest-point launches, MODE 0 and 3): phase 0 = every slot,
    // unhinted; phase 1 = leader slots (i % kLead == 0); phase 2 = the other slots, each starting from the
    // leaf of the nearest leader's closest point in its 64-slot window (see leader_leaf)
    int phase;
    // direct: the sorted path writes each answer straight to the caller's row perm[i] (no k_unpermute);
    // slot-order records are kept only for the leader phases, whose records are the followers' hints
    bool direct;
    // rec_leaf: slot-order records are hints only (direct stores, or instrumented launches), so their part
    // field carries the winner's leaf index instead of its part code (leader_leaf)
    bool rec_leaf;
    bool list;      // closest-point modes: wave leaf list (trees of < 2^26 leaves) instead of per-lane queues
    // entry cut (list path; single trees): a query inside the grid starts from its cell's record -- the cell's hint
    // leaf and up to kCutK start entries -- instead of the root (build_entry_cut); nullptr: from the root
    const uint32_t* cut;
    int cut_wide;  // records of 64 B with 8-B entries (trees of > 2^20 leaves); else 32 B with 4-B entries
    int cut_G;
    double cut_lo[3], cut_iw[3];
    size_t nunits;  // work units of this phase (slots it covers)
    DeferRec* deferred;
    unsigned* n_deferred;
    unsigned max_deferred;
    // pass-1 work a deferred query leaves (list path): its pending node and its stack as (ref, fp32 bound bits),
    // appended to one arena, from which pass 2 resumes instead of walking again from the root; a query that does
    // not fit keeps rcnt = 0
    uint2* resume;
    unsigned* n_resume;
    unsigned resume_cap;
    // pass 2: the heavy items (k_p2_plan: heavy[0, *n_heavy)) run as kP2Split parts whose candidates go to cand
    // (k_knn_combine); max_best: pass 1's largest deferred best (d2 bits)
    P2Cand* cand;
    unsigned* heavy;
    unsigned* n_heavy;
    unsigned long long* max_best;
};

// root node and fp32 query of slot i (batched trees: its mesh's root and origin)
__device__ inline int query_root(const KnnArgs& a, size_t i, const D3& q, QF& qf) {
    if (a.orgs) {
        const size_t mb = i / a.qper;
        const double o[3] = {a.orgs[3 * mb], a.orgs[3 * mb + 1], a.orgs[3 * mb + 2]};
        qf = make_qf(q, o, a.tm);
        return (int)(a.root0 + mb * a.npm);
    }
    const double o[3] = {a.org[0], a.org[1], a.org[2]};
    qf = make_qf(q, o, a.tm);
    return 0;
}

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

__device__ inline bool finite3(const D3& q) { return isfinite(q.x) && isfinite(q.y) && isfinite(q.z); }

// ---- leaf policies ----
// limit(): squared radius (in box-distance units) inside which a primitive can still beat or tie the
// best.  `shared` is a bound published by other lanes working on the same query (pass 2); it is always
// >= the final best, so pruning with min(best, shared) keeps the result exact.  limf caches
// limit() rounded up to fp32 (the unit of the node bounds); relim() refreshes it whenever best or
// shared changes, so a traversal step compares against a register instead of re-deriving it.
struct TriPol {
    const TriRec* __restrict__ tris;
    D3 q;
    double best, shared;
    uint32_t best_face;
    int best_leaf;
    float limf;
    __device__ double limit() const { return fmin(best, shared) * kSlack; }
    __device__ void relim() { limf = __double2float_ru(limit()); }
    // CGAL's exact fp64 construction for every leaf that passed its node's oriented-box bound.  (An fp32
    // Ericson pretest before it, tri_d2_lo, rejected some leaves early but cost more than it saved: C3
    // pass 1 137 -> 117 ms without it.)
    __device__ void test(int leaf) {
        uint32_t face;
        const double d2 = eval(leaf, q, face);
        if (offer(d2, face, leaf)) relim();
    }
    // exact squared distance from x (this lane's query or another lane's) to the leaf's triangle
    __device__ double eval(int leaf, const D3& x, uint32_t& face) const {
        D3 a, b, c;
        load_tri(tris, leaf, a, b, c, face);
        D3 o;
        int part;
        return closest_on_triangle(x, a, b, c, o, part);
    }
    // lexicographic (d2, face) update; the caller refreshes limf
    __device__ bool offer(double d2, uint32_t face, int leaf) {
        if (d2 < best || (d2 == best && face < best_face)) {
            best = d2;
            best_face = face;
            best_leaf = leaf;
            return true;
        }
        return false;
    }
};

// metric = ||q - p|| + eps (1 - n_q . n_tri)  (AABB_n_tree.h:40-84).  The penalty is bounded below by
// pmin = min(eps(1-|n_q|), eps(1+|n_q|)), so a face can only win inside the ball of radius best - pmin.
struct NrmPol {
    const TriRec* __restrict__ tris;
    D3 q, qn;
    double eps, pmin;
    double best, shared;
    uint32_t best_face;
    int best_leaf;
    float limf;
    __device__ double limit() const {
        const double b = fmin(best, shared);
        if (b == INFINITY) return INFINITY;
        double r = b - pmin;
        r += 1e-12 * (fabs(b) + fabs(pmin));
        if (r < 0.0) r = 0.0;
        return r * r * kSlack;
    }
    __device__ void relim() { limf = __double2float_ru(limit()); }
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
            relim();
        }
    }
};

struct PtPol {
    const PtRec* __restrict__ pts;
    D3 q;
    double best, shared;
    uint32_t best_face;
    int best_leaf;
    float limf;
    __device__ double limit() const { return fmin(best, shared) * kSlack; }
    __device__ void relim() { limf = __double2float_ru(limit()); }
    __device__ void test(int leaf) {
        const double2* p = reinterpret_cast<const double2*>(pts + leaf);
        const double2 x0 = p[0], x1 = p[1];
        const uint32_t idx = (uint32_t)__double_as_longlong(x1.y);
        const double d2 = sqdist(q, D3{x0.x, x0.y, x1.x});
        if (d2 < best || (d2 == best && idx < best_face)) {
            best = d2;
            best_face = idx;
            best_leaf = leaf;
            relim();
        }
    }
};

// Stack entries (node or ~leaf ref, fp32 bound bits): 8 B, or 4 B for trees of <= 2^20 leaves — the bound's top
// 11 bits (sign 0, exponent, 2 mantissa bits: the bound truncated, so still a lower bound; a pop it fails to prune
// only visits a node whose children are then bounded exactly) over the ref's 21 bits, one v_bfi to pack, a v_and
// and a v_bfe to unpack.
struct Ent8 {
    typedef uint2 T;
    __device__ static T make(uint32_t ref, uint32_t bb) { return make_uint2(ref, bb); }
    __device__ static int ref(T e) { return (int)e.x; }
    __device__ static float bound(T e) { return __uint_as_float(e.y); }
};
struct Ent4 {
    typedef uint32_t T;
    __device__ static T make(uint32_t ref, uint32_t bb) { return (bb & 0xFFE00000u) | (ref & 0x001FFFFFu); }
    __device__ static int ref(T e) { return __builtin_amdgcn_sbfe((int)e, 0, 21); }
    __device__ static float bound(T e) { return __uint_as_float(e & 0xFFE00000u); }
};

// Per-lane depth-first walker.  lds: this lane's column of the LDS stack (stride kBlock).
template <class E = Ent8>
struct WalkerT {
    typedef typename E::T Ent;
    int node;
    int sp;
    __device__ inline void push(uint32_t ref, uint32_t bb, Ent* __restrict__ lds, uint2* __restrict__ spill) {
        stack_put(lds, spill, sp, E::make(ref, bb));
        ++sp;
    }
    // pop until an entry survives the current limit; false when the stack is exhausted
    template <class Pol>
    __device__ inline bool pop(const Pol& pol, Ent* __restrict__ lds, uint2* __restrict__ spill) {
        while (sp > 0) {
            --sp;
            const Ent e = stack_get(lds, spill, sp);
            if (E::bound(e) <= pol.limf) {
                node = E::ref(e);
                return true;
            }
        }
        return false;
    }
    // Visit `node`: bound its two children by their fp32 oriented boxes (node_child_bounds), test leaf
    // children, descend into the nearer internal child and push the farther one.  Returns false when the
    // traversal is complete.
    template <class Pol, bool STATS>
    __device__ inline bool step(const BNode* __restrict__ nodes, const QF& qf, Pol& pol, Ent* __restrict__ lds,
                                uint2* __restrict__ spill, unsigned& n_nodes, unsigned& n_leaves) {
        const NodeV nd = load_node(nodes, node);
        if (STATS) ++n_nodes;
        float d0, d1;
        node_child_bounds(nd, qf, d0, d1);
        const int c0 = nd.child(0), c1 = nd.child(1);
        bool h0 = d0 <= pol.limf, h1 = d1 <= pol.limf;
        if (h0 && c0 < 0) {
            pol.test(~c0);
            if (STATS) ++n_leaves;
            h0 = false;
        }
        if (h1 && c1 < 0) {
            pol.test(~c1);
            if (STATS) ++n_leaves;
            h1 = false;
        }
        h0 = h0 && d0 <= pol.limf;
        h1 = h1 && d1 <= pol.limf;
        if (h0 && h1) {
            int nearc = c0, farc = c1;
            float dfar = d1;
            if (d1 < d0) { nearc = c1; farc = c0; dfar = d0; }
            push((unsigned)farc, __float_as_uint(dfar), lds, spill);
            node = nearc;
            return true;
        }
        if (h0) { node = c0; return true; }
        if (h1) { node = c1; return true; }
        return pop(pol, lds, spill);
    }
    // As step(), but leaf children that survive the bound are handed back in p0/p1 instead of being
    // tested here, so the caller can run leaf tests for many lanes of the wave at once.  `room` = leaves the
    // caller can still queue (>= 1): when a node has two leaf children and there is room for one, the farther
    // leaf is parked on the stack as an entry (~leaf, bound); a parked leaf popped later becomes `node`
    // (negative) and is handed back by the next step without a node load.  So a lane keeps traversing while
    // its queue has room for one leaf, instead of stopping as soon as a node could add two.
    // One push site and one pop site (each is a divergent loop or branch in the wave-synchronous caller, so
    // every extra copy runs serially for the lanes that take it); a parked leaf goes straight to `node`,
    // since the stack entry it would get is the one the following pop returns.
    // PF: the node was prefetched into this lane's LDS slot (nb; node_prefetch), and the next one is prefetched
    // before returning
    template <class Pol, bool STATS, bool PF = false>
    __device__ inline bool step_collect(const BNode* __restrict__ nodes, const QF& qf, const Pol& pol,
                                        Ent* __restrict__ lds, uint2* __restrict__ spill, unsigned& n_nodes, int& p0,
                                        int& p1, int room = 2, const float4* nb = nullptr, uint32_t wsl = 0) {
        bool more = false;  // `node` holds the next entry; otherwise pop
        if (node < 0) {
            p0 = ~node;
        } else {
            const NodeV nd = PF ? node_from_lds(nb) : load_node(nodes, node);
            if (STATS) ++n_nodes;
            float d0, d1;
            node_child_bounds(nd, qf, d0, d1);
            const int c0 = nd.child(0), c1 = nd.child(1);
            const float lim = pol.limf;
            const bool h0 = d0 <= lim, h1 = d1 <= lim;
            const bool l0 = h0 && c0 < 0, l1 = h1 && c1 < 0;  // leaf children within the bound
            const bool i0 = h0 && c0 >= 0, i1 = h1 && c1 >= 0;  // internal children within the bound
            const bool first1 = d1 < d0;                         // child 1 is the nearer
            if (l0 && l1) {
                if (room < 2) {  // two leaves, room for one: queue the nearer, park the farther
                    p0 = first1 ? ~c1 : ~c0;
                    node = first1 ? c0 : c1;
                    more = true;
                } else {
                    p0 = ~c0;
                    p1 = ~c1;
                }
            } else {
                if (l0) p0 = ~c0;
                if (l1) p0 = ~c1;
                if (i0 && i1) push((unsigned)(first1 ? c0 : c1), __float_as_uint(first1 ? d0 : d1), lds, spill);
                if (i0 || i1) {
                    node = (i0 && i1) ? (first1 ? c1 : c0) : (i0 ? c0 : c1);
                    more = true;
                }
            }
        }
        const bool r = more || pop(pol, lds, spill);
        if (PF && r && node >= 0) node_prefetch(nodes, node, wsl);
        return r;
    }
};
typedef WalkerT<Ent8> Walker;

// Heidrich's barycentric coordinates of p's projection into triangle (a, b, c), with the operation
// order of the reference's numpy code (barycentric_coordinates_of_projection.py:31-47, called with
// q = a, u = b - a, v = c - a by mesh.py:222): n = u x v, s = n.n (0 -> numpy.spacing(1)),
// b2 = ((u x w).n) / s, b1 = ((w x v).n) / s with w = p - a, weights (1 - b1 - b2, b1, b2).
__device__ inline D3 heidrich_bary(const D3& p, const D3& a, const D3& b, const D3& c) {
    const D3 u = vsub(b, a), v = vsub(c, a);
    const D3 n = vcross(u, v);
    double s = n.x * n.x + n.y * n.y + n.z * n.z;
    if (s == 0.0) s = 2.220446049250313e-16;  // numpy.spacing(1)
    const double inv = 1.0 / s;
    const D3 w = vsub(p, a);
    const double b2 = vdot(vcross(u, w), n) * inv;
    const double b1 = vdot(vcross(w, v), n) * inv;
    return D3{1.0 - b1 - b2, b1, b2};
}

// Outputs of slot i from its policy (winner's leaf -> point / part recomputed exactly).
template <int MODE, class Pol>
__device__ inline void write_result(const KnnArgs& a, size_t i, const D3& q, const Pol& pol) {
    const bool rec = a.res && (!a.direct || a.phase == 1 || a.phase == 3 || a.phase == 4);  // slot-order record
    const bool out = !a.res || a.direct;                                      // caller's arrays
    const size_t r = a.res ? (size_t)a.perm[i] : i;                           // caller's row
    if constexpr (MODE == 2) {
        const double dist = pol.best_leaf >= 0 ? sqrt(pol.best) : NAN;
        if (rec) store_qres(a.res + i, pol.best_face, 0u, dist, 0.0, 0.0);
        if (out) {
            a.out_face[r] = pol.best_face;
            a.out_dist[r] = dist;
        }
        return;
    }
    const TriRec* tris = static_cast<const TriRec*>(a.leaves);
    D3 ta, tb, tc, o = D3{NAN, NAN, NAN}, w = D3{NAN, NAN, NAN};
    uint32_t face = MSH_NO_FACE;
    int part = 0;
    if (pol.best_leaf >= 0) {  // < 0 only for a non-finite query
        load_tri(tris, pol.best_leaf, ta, tb, tc, face);
        closest_on_triangle(q, ta, tb, tc, o, part);
        if (MODE == 3) w = heidrich_bary(o, ta, tb, tc);
    }
    if (rec) {
        store_qres(a.res + i, face, a.rec_leaf ? (uint32_t)pol.best_leaf : (uint32_t)part, o.x, o.y, o.z);
        if (MODE == 3 && !a.direct) {
            a.res_w[3 * i] = w.x;
            a.res_w[3 * i + 1] = w.y;
            a.res_w[3 * i + 2] = w.z;
        }
    }
    if (!out) return;
    a.out_face[r] = face;
    if (MODE == 0 && a.out_part) a.out_part[r] = (uint32_t)part;
    a.out_pt[3 * r] = o.x;
    a.out_pt[3 * r + 1] = o.y;
    a.out_pt[3 * r + 2] = o.z;
    if (MODE == 3) {
        a.out_w[3 * r] = w.x;
        a.out_w[3 * r + 1] = w.y;
        a.out_w[3 * r + 2] = w.z;
    }
}

template <int MODE>
struct PolOf { using T = TriPol; };
template <>
struct PolOf<1> { using T = NrmPol; };
template <>
struct PolOf<2> { using T = PtPol; };

template <int MODE>
__device__ inline typename PolOf<MODE>::T make_pol(const KnnArgs& a, size_t i, const D3& q) {
    typename PolOf<MODE>::T pol;
    if constexpr (MODE == 2) {
        pol.pts = static_cast<const PtRec*>(a.leaves);
    } else {
        pol.tris = static_cast<const TriRec*>(a.leaves);
    }
    pol.q = q;
    if constexpr (MODE == 1) {
        pol.qn = D3{a.n[3 * i], a.n[3 * i + 1], a.n[3 * i + 2]};
        const double nq = sqrt(vdot(pol.qn, pol.qn));
        pol.eps = a.eps;
        pol.pmin = fmin(a.eps * (1 - nq), a.eps * (1 + nq));
    }
    pol.best = INFINITY;
    pol.shared = INFINITY;
    pol.best_face = MSH_NO_FACE;
    pol.best_leaf = -1;
    pol.limf = INFINITY;
    return pol;
}


__device__ inline D3 load_q(const KnnArgs& a, size_t i) {
    const size_t r = a.qperm ? (size_t)a.qperm[i] : i;
    return D3{a.q[3 * r], a.q[3 * r + 1], a.q[3 * r + 2]};
}

// ---- pass-1 constants (each measured on C3 100M; A/B records in profiles/r02_*_ab.jsonl, r03_*_ab.jsonl) ----
// Leader ordering: one leader slot per kLead slots (4: -4 %, 16: -1 %, none: -22 %; with the entry cut and the node
// prefetch, 16: -1.5 %, 16 with 128-slot follower windows: -1.5 to -2 %, profiles/r04_c3_prefetch_asm_lead_ab.jsonl), one super-leader per kLead2
// slots; super-leaders run first and unhinted, leaders take their hint from the kLWin super-leaders of their
// window (4: -1.1 %), followers from the leaders of their kFWin-slot window (32: +-0, 128: -3 %).
#ifndef MSH_KLEAD
#define MSH_KLEAD 8
#endif
#ifndef MSH_KFWIN
#define MSH_KFWIN 64
#endif
#ifndef MSH_FOLLOW_CELL
#define MSH_FOLLOW_CELL 0
#endif
#ifndef MSH_RESUME
#define MSH_RESUME 1
#endif
constexpr unsigned kLead = MSH_KLEAD;
constexpr unsigned kLead2 = 256;
constexpr size_t kFWin = MSH_KFWIN;
constexpr size_t kLWin = 8;
static_assert(kLead2 % kLead == 0 && kLead2 / kLead >= 2, "kLead2: a multiple of kLead");
// Per-lane leaf queues (the path of trees with >= 2^26 leaves, and of the normals-metric and point modes): up
// to kLeafQ leaves per lane, a lane traverses while its queue has room for one more (a second leaf child is
// parked on its stack); leaf phases run as soon as one lane is blocked; the uncompacted phases (MODE 1, 2) test
// at most kLeafRound leaves per lane each.
constexpr int kLeafQ = 4;
constexpr int kLeafRound = 2;

// slot of work unit k in the launch's phase: 3 super-leaders, 1 leaders (without the super-leaders), 4 every leader
// (trees with cell hints: no super-leader launch), 2 followers, 0 every slot
__device__ inline size_t slot_of(const KnnArgs& a, size_t k) {
    if (a.phase == 3) return k * kLead2;
    if (a.phase == 4) return k * kLead;
    if (a.phase == 1) {
        constexpr size_t r = kLead2 / kLead;
        return kLead * (k + k / (r - 1) + 1);
    }
    if (a.phase == 2) {
        const size_t g = k / (kLead - 1);
        return g * kLead + (k - g * (kLead - 1)) + 1;
    }
    return k;
}

// The leaf holding the closest point p_L of the leader (at slots base, base + stride, ... < base + window of
// the window containing i) nearest to q, or -1.  A hinted slot starts by testing that leaf exactly, as if the
// traversal had reached it first: a real candidate (d^2, face, leaf), so no hint can be too tight, and its
// exact distance is at most |q - p_L| (host model: 14 % fewer leaf tests than a |q - p_L| bound; C3: the
// hint leaf is the answer for 17 % of the followers).  Leaders of another mesh (batched trees) and deferred
// leaders (NO_FACE until pass 2 answers them) are skipped.
__device__ inline int leader_leaf(const KnnArgs& a, size_t i, const D3& q, size_t window, size_t stride) {
    const size_t base = (i / window) * window;
    const size_t mesh = a.orgs ? i / a.qper : 0;
    double h = INFINITY;
    int leaf = -1;
    for (size_t L = 0; L < window; L += stride) {
        const size_t li = base + L;
        if (li >= a.S) break;
        if (a.orgs && li / a.qper != mesh) continue;
        const uint4 r0 = reinterpret_cast<const uint4*>(a.res + li)[0];
        if (r0.x == MSH_NO_FACE) continue;
        const double2 r1 = reinterpret_cast<const double2*>(a.res + li)[1];
        const double x = __longlong_as_double((long long)(((unsigned long long)r0.w << 32) | r0.z));
        const double dx = q.x - x, dy = q.y - r1.x, dz = q.z - r1.y;
        const double d2 = dx * dx + dy * dy + dz * dz;
        if (d2 < h) {
            h = d2;
            leaf = (int)r0.y;
        }
    }
    return leaf;
}

// number of set bits of m below this lane (v_mbcnt: no per-lane mask register)
__device__ inline unsigned lanes_below(unsigned long long m) {
    return __builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
}

// Wave leaf list (closest-point modes): lanes append the leaf children that survive their node's bound to a
// ring of (leaf << 6 | owner lane) entries in LDS shared by the wave, and the wave evaluates them in rounds of
// 64 — one entry per lane, every round full except when nobody can move — instead of per-lane queues flushed
// part-empty.  A lane stops traversing while kPend of its leaves wait.  Each round's results reach their
// owners through LDS: an atomic min of the squared distance's bits per owner, then an atomic min of
// (face << 32 | leaf) among the entries that reached it: the lexicographic (d2, face) rule.
// kPend (C3, M q/s): 3: 1236, 4: 1346, 8: 1593, 16: 1677, 32: 1706, unbounded: 1689; per-lane queues 1541.
#ifndef MSH_KPEND
#define MSH_KPEND 32
#endif
constexpr int kPend = MSH_KPEND;
// Tile prefetch (round 6): a wave claims its next tile while the current one's rows load.  dequeue_tile is two
// dependent round trips to the group's counter (a load, then the atomic), paid at every tile start with the wave
// idle: C3 100M pass 1 38.4-39.5 -> 36.3-36.4 ms, 2.35-2.41 -> 2.53-2.54 G q/s; the 12.5M shard 6.92-6.95 -> 6.76-6.78
// ms (profiles/r06_c3_tile_prefetch_ab.jsonl)
#ifndef MSH_TILE_PF
#define MSH_TILE_PF 1
#endif

constexpr unsigned kRing = 256;     // ring entries per wave: < 64 left after full rounds + <= 128 per step
constexpr size_t kListMaxLeaves = (size_t)1 << 26;  // leaf index bits of a ring entry
constexpr size_t kLeadMinLeaves = 4096;  // smaller trees skip the leader phases (C1: 0.56 -> 0.29 ms)

// Pass 1 runs 4 waves per SIMD (not the normals metric, MODE 1, whose larger live set would spill in the node
// step): the register budget drops from 139 to 128 VGPRs at the cost of a few spills of loop-invariant values
// outside the node step (C3: +10 % over the compiler's 3 waves; 5 waves spill in the loop: -30 %; 5 waves also
// need <= 32 KB of LDS per block).
#ifndef MSH_KNN_WAVES
#define MSH_KNN_WAVES 4
#endif
#define MSH_KNN_ATTR __attribute__((amdgpu_waves_per_eu(MODE == 1 ? 1 : MSH_KNN_WAVES)))
// Entry cut.  The grid cell of q (centre c, half-diagonal r) holds up to kCutK tree entries (node or ~leaf)
// whose bound from c is within (d(c) + 2r)^2, d(c) = c's exact distance to the mesh, and which together cover
// every such subtree; any other subtree lies farther than d(c) + 2r from c, so farther than d(c) + r >= d(q)
// from q, and can hold neither q's closest face nor a tie.  Each entry carries max(s, 0)^2 rounded down,
// s = sqrt(bound from c) - r: a lower bound of the squared distance from q to its subtree.  The entries go
// on the stack with it, nearest to c popped first, and the walk starts from the first entry within the
// current limit.  false: no entry survives the hint's bound (the hint is the answer).
constexpr size_t kNoCell = ~(size_t)0;
// grid cell of q, or kNoCell outside the grid (or without a cut)
__device__ inline size_t cut_cell(const KnnArgs& a, const D3& q) {
    if (!a.cut) return kNoCell;
    const double G = (double)a.cut_G;
    const double ux = (q.x - a.cut_lo[0]) * a.cut_iw[0], uy = (q.y - a.cut_lo[1]) * a.cut_iw[1],
                 uz = (q.z - a.cut_lo[2]) * a.cut_iw[2];
    if (!(ux >= 0.0 && ux < G && uy >= 0.0 && uy < G && uz >= 0.0 && uz < G)) return kNoCell;
    return ((size_t)(unsigned)uz * (size_t)a.cut_G + (unsigned)uy) * (size_t)a.cut_G + (unsigned)ux;
}
// the cell's record: word 0 its hint leaf (-1: none), then kCutK entries nearest-first -- 4-B entries in the stack's
// own packing (Ent4: the bound's top 11 bits over a 21-bit ref; empty entries have the sign bit set) in a 32-B
// record, or (ref, bound bits) pairs from word 2 of a 64-B record (empty: ref kCutEmpty)
__device__ inline const uint32_t* cut_rec(const KnnArgs& a, size_t cell) {
    return a.cut + cell * (a.cut_wide ? 16 : 8);
}
template <class Pol, class W>
__device__ inline bool cut_start(const KnnArgs& a, size_t cell, const Pol& pol, W& w, typename W::Ent* __restrict__ lds,
                                 uint2* __restrict__ spill) {
    const uint32_t* r = cut_rec(a, cell);
    if (a.cut_wide) {
        const uint4* c = reinterpret_cast<const uint4*>(r);
        uint4 e[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) e[j] = c[j];
        auto put = [&](uint32_t ref, uint32_t sb) {
            if (ref != kCutEmpty) w.push(ref, sb, lds, spill);
        };
#pragma unroll
        for (int j = 3; j >= 1; --j) {
            put(e[j].z, e[j].w);
            put(e[j].x, e[j].y);
        }
        put(e[0].z, e[0].w);  // entry 0 (words 2, 3)
    } else {
        const uint4* c = reinterpret_cast<const uint4*>(r);
        const uint4 e0 = c[0], e1 = c[1];
        const uint32_t e[kCutK] = {e0.y, e0.z, e0.w, e1.x, e1.y, e1.z, e1.w};
#pragma unroll
        for (int j = kCutK - 1; j >= 0; --j)
            if ((int)e[j] >= 0) w.push((uint32_t)Ent4::ref(e[j]), e[j] & 0xFFE00000u, lds, spill);
    }
    return w.pop(pol, lds, spill);
}

// PF (list path, trees of <= 2^20 leaves): 4-B stack entries (Ent4) and each lane's next node prefetched into LDS
// (node_prefetch); the 16 KB the node slots take per block come out of the stack.  C3: 1889 -> 1945 M q/s in one
// session, wave-cycles waiting on memory 55.7 -> 46.7 % at +10 VALU instructions per query
// (profiles/r04_c3_node_prefetch_lds_ab.jsonl).
template <int MODE, bool STATS, bool LIST, bool PF>
__global__ __launch_bounds__(kBlock) MSH_KNN_ATTR void k_knn(KnnArgs a) {
    constexpr bool kCompact = MODE == 0 || MODE == 3;  // per-lane queues dealt to the wave (else: per-lane rounds)
    constexpr bool kList = (MODE == 0 || MODE == 3) && LIST;  // a separate instantiation: its own registers
    constexpr bool kPF = kList && PF;  // 4-B stack entries and nodes prefetched into LDS
    typedef typename std::conditional<kPF, Ent4, Ent8>::type E;
    __shared__ typename E::T stk[kStack * kBlock];
    __shared__ float4 nbuf[kPF ? 4 * kBlock : 1];
    // compacted leaf phases: kLeafQ entries per lane; the wave leaf list shares this space (a.list)
    constexpr size_t kEntWords = kCompact && !kList ? (size_t)kBlock * kLeafQ * 2 : 1;
    constexpr size_t kListWords = kList ? 4 * (kRing + 64 * 4) : 1;  // per wave: ring + bd/bfl (u64 per lane each)
    __shared__ uint32_t lsh[kEntWords > kListWords ? kEntWords : kListWords];
    uint2* lent = reinterpret_cast<uint2*>(lsh);
    const int tid = threadIdx.x, lane = tid & 63;
    typename E::T* lds = stk + tid;
    // the wave's node slots (kPF): LDS byte address from a wave-uniform wave index, so M0 is set by scalar code
    const int wv_u = __builtin_amdgcn_readfirstlane(tid >> 6);
    const uint32_t wsl = (uint32_t)(size_t)(__attribute__((address_space(3))) float4*)(nbuf + (kPF ? wv_u * 256 : 0));
    const float4* nb = nbuf + (kPF ? (tid >> 6) * 256 + lane : 0);
    uint2* ent = lent + (kCompact ? (tid >> 6) * 64 * kLeafQ : 0);
    uint2* spill = a.spill ? a.spill + (size_t)blockIdx.x * kBlock * (size_t)a.spill_depth + tid : nullptr;
    const unsigned group = blockIdx.x & 7u;
    unsigned long long u_trav_it = 0, u_trav_lanes = 0, u_leaf_it = 0, u_leaf_lanes = 0;  // STATS: wave iterations
    unsigned n_nodes = 0, n_leaves = 0;
    unsigned n_impr = 0, n_hinted = 0, n_hint_won = 0;  // STATS: improving leaf tests, hinted queries, hint = answer
#if MSH_TILE_PF
    // lane 0 claims the wave's next tile of its own group while the current one's rows load (an atomic whose return
    // is waited for with the tile's first loads), instead of at the next tile's start
    const unsigned glo = (unsigned)(((unsigned long long)a.ntiles * group) >> 3);
    const unsigned ghi = (unsigned)(((unsigned long long)a.ntiles * (group + 1)) >> 3);
    unsigned nxt = ~0u;
#endif
    for (;;) {
        unsigned tile = 0;
#if MSH_TILE_PF
        if (lane == 0) tile = (nxt != ~0u && glo + nxt < ghi) ? glo + nxt : dequeue_tile(a.counters, a.ntiles, group);
#else
        if (lane == 0) tile = dequeue_tile(a.counters, a.ntiles, group);
#endif
        tile = __shfl(tile, 0);
        if (tile >= a.ntiles) break;
        // every lane of the wave stays in the tile's loops (compacted leaf phases deal entries to all 64 lanes);
        // a lane without a query (past the phase's units, or a non-finite row) only helps
        const size_t k = (size_t)tile * 64 + lane;
        size_t i = 0;
        bool live = k < a.nunits;
        if (live) {
            i = slot_of(a, k);
            live = i < a.S;
        }
        const D3 q = live ? load_q(a, i) : D3{0.0, 0.0, 0.0};
#if MSH_TILE_PF
        if (lane == 0) nxt = glo < ghi ? atomicAdd(&a.counters[group * 32], 1u) : ~0u;
#endif
        if (live && a.inv_w && !a.direct) a.inv_w[a.qperm[i]] = (uint32_t)i;
        auto pol = make_pol<MODE>(a, i, q);
        const bool fin = live && finite3(q);
        if (live && !fin) {  // no distance is defined: NO_FACE / NaN, no traversal
            if (!STATS || a.res) write_result<MODE>(a, i, q, pol);
        }
        int hint_leaf = -1;  // STATS
        const size_t cell = kList && fin ? cut_cell(a, q) : kNoCell;
        if constexpr (MODE == 0 || MODE == 3) {
            if (kList && a.cut && cell != kNoCell && a.phase != 2) {
                // slots without a leader (super-leaders, leaders, unled launches) inside the grid: the cell's hint
                // leaf (the closest face found for its centre), within U(c) + r of q's own answer
                const int lf = (int)cut_rec(a, cell)[0];
                if (STATS) hint_leaf = lf;
                if (lf >= 0) {
                    pol.test(lf);
                    if (STATS) {
                        ++n_leaves;
                        ++n_hinted;
                    }
                }
            } else if (fin && (a.phase == 2 || a.phase == 1)) {
                const int lf = a.phase == 2 ? leader_leaf(a, i, q, kFWin, kLead) : leader_leaf(a, i, q, kLWin * kLead2, kLead2);
                if (STATS) hint_leaf = lf;
#if MSH_FOLLOW_CELL
                // followers inside the grid also test their cell's hint leaf (one call site: a loop of two)
                const int lc = (kList && a.cut && cell != kNoCell) ? (int)cut_rec(a, cell)[0] : -1;
#pragma nounroll
                for (int j = 0; j < 2; ++j) {
                    const int h = j == 0 ? lf : (lc != lf ? lc : -1);
                    if (h >= 0) {
                        pol.test(h);
                        if (STATS) ++n_leaves;
                    }
                }
                if (STATS && lf >= 0) ++n_hinted;
#else
                if (lf >= 0) {
                    pol.test(lf);
                    if (STATS) {
                        ++n_leaves;
                        ++n_hinted;
                    }
                }
#endif
            }
        }
        if (a.T == 1) {
            if (fin) {
                pol.test(0);
                if (STATS) ++n_leaves;
                if (!STATS || a.res) write_result<MODE>(a, i, q, pol);
            }
            continue;
        }
        if constexpr (kList) {
          {
            QF qf;
            const int root = query_root(a, i, q, qf);
            WalkerT<E> w{root, 0};
            bool start = fin;
            if (cell != kNoCell) start = cut_start(a, cell, pol, w, lds, spill);
            if (kPF && start && w.node >= 0) node_prefetch(a.nodes, w.node, wsl);
            uint32_t* ring = lsh + (tid >> 6) * (kRing + 64 * 4);
            unsigned long long* bd = reinterpret_cast<unsigned long long*>(ring + kRing);  // per owner: d2 bits
            unsigned long long* bfl = bd + 64;                                              // (face << 32 | leaf)
            bool active = start, want_defer = false, deferred = false;
            int nq = 0;              // this lane's leaves appended since all of them were last evaluated (a bound)
            unsigned last_pos = 0;   // ring counter of this lane's newest entry
            unsigned head = 0, tail = 0;  // wave-uniform ring counters: entries [head, tail) wait
            unsigned steps = 0;
            const unsigned max_steps = (unsigned)min(a.T, (size_t)UINT_MAX);
            unsigned tot = 0;  // STATS: node steps of this lane, restarts included
            // Evaluate ring entries [head, upto) in rounds of 64, one per lane: each lane tests its entry's leaf
            // against its owner's query (ds_bpermute); the owners publish their best before each round and take
            // the round's lexicographic (d2, face) minimum back from LDS.
            auto run_rounds = [&](unsigned upto) {
                while (head != upto) {
                    const unsigned n = min(64u, upto - head);
                    bd[lane] = (unsigned long long)__double_as_longlong(pol.best);
                    bfl[lane] = ~0ull;
                    const bool valid = (unsigned)lane < n;
                    const uint32_t en = ring[(head + (valid ? (unsigned)lane : 0u)) & (kRing - 1)];
                    const int src = (int)(en & 63u);
                    const int leaf = (int)(en >> 6);
                    const D3 x = D3{__shfl(pol.q.x, src), __shfl(pol.q.y, src), __shfl(pol.q.z, src)};
                    uint32_t f;
                    const double d2 = pol.eval(leaf, x, f);
                    const unsigned long long kb = (unsigned long long)__double_as_longlong(d2);
                    asm volatile("" ::: "memory");
                    if (valid) atomicMin(&bd[src], kb);
                    asm volatile("" ::: "memory");
                    if (valid && bd[src] == kb) atomicMin(&bfl[src], ((unsigned long long)f << 32) | (unsigned)leaf);
                    asm volatile("" ::: "memory");
                    const unsigned long long nb = bd[lane], nf = bfl[lane];
                    const double nd = __longlong_as_double((long long)nb);
                    const uint32_t nface = (uint32_t)(nf >> 32);
                    if (nf != ~0ull && (nd < pol.best || (nd == pol.best && nface < pol.best_face))) {
                        pol.best = nd;
                        pol.best_face = nface;
                        pol.best_leaf = (int)(uint32_t)nf;
                        pol.relim();
                        if (STATS) ++n_impr;
                    }
                    asm volatile("" ::: "memory");
                    if (STATS) {
                        if (valid) ++n_leaves;
                        if (lane == 0) {
                            ++u_leaf_it;
                            u_leaf_lanes += n;
                        }
                    }
                    head += n;
                }
                if ((int)(last_pos - head) < 0) nq = 0;  // every entry of this lane is evaluated
            };
            unsigned dslot = 0;  // this lane's deferred-list slot (deferred)
            for (;;) {
                // a lane past its budget defers once its own leaves are evaluated (pass 2 then owns the query); its
                // records are written after the tile's loop, so the loop holds no copy of the construction
                if (want_defer && nq == 0) {
                    want_defer = false;
                    dslot = atomicAdd(a.n_deferred, 1u);
                    if (dslot < a.max_deferred) {
                        active = false;
                        deferred = true;
                    }
                    // deferred list full: finish here without a budget
                }
                const bool can = active && !want_defer && nq < kPend;
                const bool any = __ballot(can) != 0ull;
                if (!any && tail == head) break;  // nothing queued and nobody can move: the tile is done
                if (STATS) {
                    const int nt = __popcll(__ballot(can));
                    if (lane == 0 && any) {
                        ++u_trav_it;
                        u_trav_lanes += nt;
                    }
                }
                int l0 = -1, l1 = -1;
                if (can) {
                    active = w.template step_collect<decltype(pol), STATS, kPF>(a.nodes, qf, pol, lds, spill, n_nodes,
                                                                                  l0, l1, kPend - nq, nb, wsl);
                    ++steps;
                    if (STATS) ++tot;
                    if (active && steps >= max_steps) active = false;  // each node is entered once: corrupt tree
                    if (active && steps == a.budget) want_defer = true;
                }
                // append this step's leaves (at most two per lane) to the ring, in lane order
                if (l0 < 0) {
                    l0 = l1;
                    l1 = -1;
                }
                const unsigned long long m1 = __ballot(l0 >= 0), m2 = __ballot(l1 >= 0);
                const unsigned pos = tail + lanes_below(m1) + lanes_below(m2);
                if (l0 >= 0) {
                    ring[pos & (kRing - 1)] = ((uint32_t)l0 << 6) | (uint32_t)lane;
                    last_pos = pos;
                    ++nq;
                }
                if (l1 >= 0) {
                    ring[(pos + 1) & (kRing - 1)] = ((uint32_t)l1 << 6) | (uint32_t)lane;
                    last_pos = pos + 1;
                    ++nq;
                }
                tail += (unsigned)(__popcll(m1) + __popcll(m2));
                // full rounds while lanes can move; everything once nobody can
                const unsigned upto = any ? head + ((tail - head) & ~63u) : tail;
                if (upto != head) run_rounds(upto);
            }
            if (deferred) {
                if ((a.phase == 1 || a.phase == 3 || a.phase == 4) && a.res) {
                    // later phases take hints from this slot before pass 2 answers it: publish the closest point of
                    // the best face so far (a point on the mesh), or NO_FACE when it has none yet
                    D3 o = D3{NAN, NAN, NAN};
                    uint32_t f = MSH_NO_FACE;
                    if (pol.best_leaf >= 0) {
                        D3 ta, tb, tc;
                        int part;
                        load_tri(static_cast<const TriRec*>(a.leaves), pol.best_leaf, ta, tb, tc, f);
                        closest_on_triangle(q, ta, tb, tc, o, part);
                    }
                    store_qres(a.res + i, f, (uint32_t)pol.best_leaf, o.x, o.y, o.z);
                }
                DeferRec r;
                r.slot = (uint32_t)i;
                r.face = pol.best_face;
                r.leaf = pol.best_leaf;
                r.roff = 0;
                r.best = pol.best;
                r.rcnt = 0;
                r.sbound = 0x7F800000u;  // +inf
                if (a.max_best) atomicMax(a.max_best, (unsigned long long)__double_as_longlong(pol.best));
                if (a.resume) {
                    // what is left of this walk: the pending entry (w.node, not yet visited: bound 0) above the stack
                    const unsigned cnt = (unsigned)w.sp + 1;
                    const unsigned off = atomicAdd(a.n_resume, cnt);
                    if (off + cnt <= a.resume_cap) {
                        uint2* dst = a.resume + off;
                        for (int j = 0; j < w.sp; ++j) {
                            const typename E::T e = stack_get(lds, spill, j);
                            dst[j] = make_uint2((uint32_t)E::ref(e), __float_as_uint(E::bound(e)));
                        }
                        dst[w.sp] = make_uint2((uint32_t)w.node, 0u);
                        r.roff = off;
                        r.rcnt = cnt;
                    }
                }
                a.deferred[dslot] = r;
            }
            if (STATS) {  // per-tile step profile of this phase (stats[8 + 9 * phase slot ...])
                unsigned mx = tot, sm = tot;
                for (int o = 32; o > 0; o >>= 1) {
                    mx = max(mx, (unsigned)__shfl_xor((int)mx, o));
                    sm += (unsigned)__shfl_xor((int)sm, o);
                }
                unsigned long long* h = a.stats + 8 + 9 * (a.phase == 3 ? 0 : ((a.phase == 1 || a.phase == 4) ? 1 : 2));
                if (lane == 0) {
                    atomicAdd(h + 0, 1ull);
                    atomicAdd(h + 1, (unsigned long long)mx);
                    atomicAdd(h + 2, (unsigned long long)sm);
                    atomicAdd(h + 3, (unsigned long long)min(mx, 128u));
                    atomicAdd(h + 4, (unsigned long long)min(mx, 256u));
                    atomicAdd(h + 5, (unsigned long long)min(mx, 512u));
                }
                if (tot > 128) atomicAdd(h + 6, 1ull);
                if (tot > 256) atomicAdd(h + 7, 1ull);
                if (tot > 512) atomicAdd(h + 8, 1ull);
            }
            if (STATS && fin && hint_leaf >= 0 && pol.best_leaf == hint_leaf) ++n_hint_won;
            if (deferred) continue;
            if (fin && (!STATS || a.res)) write_result<MODE>(a, i, q, pol);
            continue;
          }
        }
        if constexpr (!kList) {
        {
            QF qf;
            const int root = query_root(a, i, q, qf);
            Walker w{root, 0};
            bool active = fin, deferred = false;
            // leaf children waiting for a wave-wide leaf phase: a per-lane queue of up to kLeafQ leaves
            int q0 = -1, q1 = -1, q2 = -1, q3 = -1, nq = 0;
            // a shift register (no dynamic index, so the queue stays in VGPRs, not in scratch)
            auto enqueue = [&](int x) {
                if (x < 0) return;
                if (kLeafQ > 3) q3 = q2;
                q2 = q1;
                q1 = q0;
                q0 = x;
                ++nq;
            };
            // tests up to `most` queued leaves, newest first (one copy of the fp64 construction in the code: a
            // loop over the queue, not one per entry)
            auto test_queue = [&](int most) {
                const int n = min(nq, most);
#pragma nounroll
                for (int k = 0; k < n; ++k) {
                    pol.test(q0);
                    q0 = q1;
                    q1 = q2;
                    if (kLeafQ > 3) q2 = q3;
                }
                nq -= n;
            };
            unsigned steps = 0;
            const unsigned max_steps = (unsigned)min(a.T, (size_t)UINT_MAX);
            unsigned tot = 0;  // STATS: node steps of this lane, restarts included
            // Wave-synchronous loop.  Lanes that reach leaves queue them; a lane keeps traversing while
            // its queue has room for one more leaf.  Leaf tests run as soon as one lane is blocked (or nobody
            // can traverse), so the expensive fp64 leaf path executes for many lanes at once instead of
            // stalling the wave on one lane every iteration (Aila & Laine 2009, "postponed leaf" while-while).
            for (;;) {
                const bool can = active && nq <= kLeafQ - 1;
                const bool has = nq > 0;
                const unsigned long long bl = __ballot(has);
                const unsigned long long bt = __ballot(can);
                if ((bl | bt) == 0ull) break;
                const bool flush = bt == 0ull || __ballot(has && !can) != 0ull;
                if (bl != 0ull && flush) {
                    if constexpr (kCompact) {
                        // Compacted leaf phase: the wave's queued leaves (newest first per lane) are dealt to
                        // its 64 lanes, one (leaf, owner) entry each; a lane tests its entry against the
                        // owner's query (ds_bpermute) and each owner takes its entries' (d2, face) back.  The
                        // fp64 construction then runs with (nearly) every lane busy instead of only the
                        // lanes that hold leaves.
                        const unsigned long long lt = (1ull << lane) - 1ull;
                        const unsigned long long m1 = bl, m2 = __ballot(nq >= 2), m3 = __ballot(nq >= 3),
                                                 m4 = kLeafQ > 3 ? __ballot(nq >= 4) : 0ull;
                        const int pos = __popcll(m1 & lt) + __popcll(m2 & lt) + __popcll(m3 & lt) + __popcll(m4 & lt);
                        const int E = __popcll(m1) + __popcll(m2) + __popcll(m3) + __popcll(m4);
                        if (nq >= 1) ent[pos] = make_uint2((unsigned)q0, (unsigned)lane);
                        if (nq >= 2) ent[pos + 1] = make_uint2((unsigned)q1, (unsigned)lane);
                        if (nq >= 3) ent[pos + 2] = make_uint2((unsigned)q2, (unsigned)lane);
                        if (kLeafQ > 3 && nq >= 4) ent[pos + 3] = make_uint2((unsigned)q3, (unsigned)lane);
                        asm volatile("" ::: "memory");  // the wave's LDS accesses run in order
                        bool better = false;
                        for (int base = 0; base < E; base += 64) {
                            const uint2 en = ent[min(base + lane, E - 1)];  // lanes past E repeat the last entry
                            const int src = (int)en.y;
                            const D3 x = D3{__shfl(pol.q.x, src), __shfl(pol.q.y, src), __shfl(pol.q.z, src)};
                            uint32_t f;
                            const double d2 = pol.eval((int)en.x, x, f);
                            if (STATS && base + lane < E) ++n_leaves;
#pragma unroll
                            for (int e = 0; e < kLeafQ; ++e) {
                                const int at = pos + e - base;
                                const bool mine = e < nq && at >= 0 && at < 64;
                                const int from = mine ? at : lane;
                                const double dk = __shfl(d2, from);
                                const uint32_t fk = (uint32_t)__shfl((int)f, from);
                                if (mine) {
                                    const bool b = pol.offer(dk, fk, e == 0 ? q0 : (e == 1 ? q1 : (e == 2 ? q2 : q3)));
                                    better |= b;
                                    if (STATS && b) ++n_impr;
                                }
                            }
                        }
                        asm volatile("" ::: "memory");
                        if (better) pol.relim();
                        if (STATS && lane == 0) {
                            u_leaf_it += (unsigned long long)((E + 63) / 64);
                            u_leaf_lanes += (unsigned long long)E;
                        }
                        nq = 0;
                    } else {
                        if (STATS && lane == 0) {
                            ++u_leaf_it;
                            u_leaf_lanes += __popcll(bl);
                        }
                        if (has) {
                            if (STATS) n_leaves += min(nq, kLeafRound);
                            test_queue(kLeafRound);
                        }
                    }
                    continue;
                }
                if (STATS && lane == 0) {
                    ++u_trav_it;
                    u_trav_lanes += __popcll(bt);
                }
                if (can) {
                    int l0 = -1, l1 = -1;
                    active = w.step_collect<decltype(pol), STATS>(a.nodes, qf, pol, lds, spill, n_nodes, l0, l1,
                                                                  kLeafQ - nq);
                    enqueue(l0);
                    enqueue(l1);
                    ++steps;
                    if (STATS) ++tot;
                    if (active && steps >= max_steps) active = false;  // each node is entered once: corrupt tree
                    if (active && steps == a.budget) {
                        const unsigned slot = atomicAdd(a.n_deferred, 1u);
                        if (slot < a.max_deferred) {
                            if (STATS) n_leaves += nq;
                            test_queue(kLeafQ);
                            if ((a.phase == 1 || a.phase == 3 || a.phase == 4) && a.res) {
                                // later phases take hints from this slot before pass 2 answers it: publish the
                                // closest point of the best face so far (a point on the mesh, so a valid upper
                                // bound for its neighbours), or NO_FACE when it has none yet
                                if constexpr (MODE == 0 || MODE == 3) {
                                    D3 o = D3{NAN, NAN, NAN};
                                    uint32_t f = MSH_NO_FACE;
                                    if (pol.best_leaf >= 0) {
                                        D3 ta, tb, tc;
                                        int part;
                                        load_tri(static_cast<const TriRec*>(a.leaves), pol.best_leaf, ta, tb, tc, f);
                                        closest_on_triangle(q, ta, tb, tc, o, part);
                                    }
                                    store_qres(a.res + i, f, (uint32_t)pol.best_leaf, o.x, o.y, o.z);
                                } else {
                                    store_qres(a.res + i, MSH_NO_FACE, 0u, NAN, NAN, NAN);
                                }
                            }
                            DeferRec r;
                            r.slot = (uint32_t)i;
                            r.face = pol.best_face;
                            r.leaf = pol.best_leaf;
                            r.roff = 0;
                            r.best = pol.best;
                            r.rcnt = 0;
                            r.sbound = 0x7F800000u;  // +inf
                            if (a.max_best) atomicMax(a.max_best, (unsigned long long)__double_as_longlong(pol.best));
                            a.deferred[slot] = r;
                            active = false;
                            deferred = true;  // pass 2 owns this query
                        }
                        // deferred list full: finish here without a budget
                    }
                }
            }
            if (STATS) {  // per-tile step profile of this phase (stats[8 + 9 * phase slot ...])
                unsigned mx = tot, sm = tot;
                for (int o = 32; o > 0; o >>= 1) {
                    mx = max(mx, (unsigned)__shfl_xor((int)mx, o));
                    sm += (unsigned)__shfl_xor((int)sm, o);
                }
                unsigned long long* h = a.stats + 8 + 9 * (a.phase == 3 ? 0 : ((a.phase == 1 || a.phase == 4) ? 1 : 2));
                if (lane == 0) {
                    atomicAdd(h + 0, 1ull);
                    atomicAdd(h + 1, (unsigned long long)mx);
                    atomicAdd(h + 2, (unsigned long long)sm);
                    atomicAdd(h + 3, (unsigned long long)min(mx, 128u));
                    atomicAdd(h + 4, (unsigned long long)min(mx, 256u));
                    atomicAdd(h + 5, (unsigned long long)min(mx, 512u));
                }
                if (tot > 128) atomicAdd(h + 6, 1ull);
                if (tot > 256) atomicAdd(h + 7, 1ull);
                if (tot > 512) atomicAdd(h + 8, 1ull);
            }
            if (deferred) continue;
        }
        if (STATS && fin && hint_leaf >= 0 && pol.best_leaf == hint_leaf) ++n_hint_won;
        if (fin && (!STATS || a.res)) write_result<MODE>(a, i, q, pol);
        }
    }
    // a lane that stopped (deferred) may still have a node prefetch in flight: it lands before the block's LDS is
    // released
    if constexpr (kPF) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (STATS) {
        atomicAdd(&a.stats[0], (unsigned long long)n_nodes);
        atomicAdd(&a.stats[1], (unsigned long long)n_leaves);
        atomicAdd(&a.stats[36], (unsigned long long)n_impr);
        atomicAdd(&a.stats[37], (unsigned long long)n_hinted);
        atomicAdd(&a.stats[38], (unsigned long long)n_hint_won);
        if (lane == 0) {
            atomicAdd(&a.stats[2], u_trav_it);
            atomicAdd(&a.stats[3], u_trav_lanes);
            atomicAdd(&a.stats[4], u_leaf_it);
            atomicAdd(&a.stats[5], u_leaf_lanes);
        }
    }
}

// lexicographic min of (best, face) over the wave; every lane ends with the winner
__device__ inline void wave_lexmin(double& best, uint32_t& face, int& leaf) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
        const double b2 = __shfl_xor(best, o, 64);
        const uint32_t f2 = (uint32_t)__shfl_xor((int)face, o, 64);
        const int l2 = __shfl_xor(leaf, o, 64);
        if (b2 < best || (b2 == best && f2 < face)) {
            best = b2;
            face = f2;
            leaf = l2;
        }
    }
}

__device__ inline double wave_min(double x) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) x = fmin(x, __shfl_xor(x, o, 64));
    return x;
}

constexpr int kFront = 512;  // pass 2: 2 kFront work-list entries per wave (LDS)

template <int MODE, bool STATS>
__global__ __launch_bounds__(kBlock) void k_knn_coop(KnnArgs a) {
    __shared__ uint2 stk[kStack * kBlock];
    __shared__ uint2 front[4][2][kFront];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    uint2* lds = stk + tid;
    uint2* spill = a.spill ? a.spill + (size_t)blockIdx.x * kBlock * (size_t)a.spill_depth + tid : nullptr;
    const unsigned total = min(*a.n_deferred, a.max_deferred);
    const unsigned long long lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    unsigned n_nodes = 0, n_leaves = 0;
    unsigned* next_item = a.n_deferred + 32;  // items are dealt dynamically: their costs vary widely
    // work units: the heavy items' K parts first (consecutive units: the parts run side by side), then every item in
    // order, the heavy ones skipped
    constexpr unsigned K = (MODE == 0 || MODE == 3) ? kP2Split : 1u;
    const unsigned nsplit = (K > 1 && a.cand) ? min(*a.n_heavy, kP2SplitItems) : 0u;
    const unsigned nunit = nsplit * K + total;
    for (;;) {
        unsigned unit = 0;
        if (lane == 0) unit = atomicAdd(next_item, 1u);
        unit = __shfl(unit, 0);
        if (unit >= nunit) break;
        const bool split = unit < nsplit * K;
        const unsigned hidx = split ? unit / K : 0u;
        const unsigned item = split ? a.heavy[hidx] : unit - nsplit * K;
        const unsigned part = split ? unit % K : 0u, kk = split ? K : 1u;
        if (!split && nsplit && a.deferred[item].sbound != kP2Whole) continue;  // a heavy item: its parts ran above
        const unsigned item_nodes0 = n_nodes, item_leaves0 = n_leaves;
        const DeferRec r = a.deferred[item];
        const size_t i = r.slot;
        const D3 q = load_q(a, i);
        QF qf;
        const int root = query_root(a, i, q, qf);
        auto pol = make_pol<MODE>(a, i, q);
        pol.shared = r.best;  // pass-1 best: an upper bound of the final best
        unsigned rounds = 0;
        // an item's parts share their bound: every 8th round a part publishes its own and takes the others'
        auto share = [&]() {
            if (!split || (++rounds & 7u) != 0u) return;
            unsigned old = 0;
            if (lane == 0) old = atomicMin(&a.deferred[item].sbound, __float_as_uint(__double2float_ru(pol.shared)));
            old = (unsigned)__shfl((int)old, 0);
            pol.shared = fmin(pol.shared, (double)__uint_as_float(old));
        };
        if (lane == 0) {
            pol.best = r.best;
            pol.best_face = r.face;
            pol.best_leaf = r.leaf;
        }
        pol.relim();
        // Subtree work list, last in first out, expanded 64 entries at a time (one per lane): children
        // within the bound go back on the list (compacted by ballot), leaf children are tested on the spot.
        // Taking the 64 newest entries keeps the walk deep-first, so good leaves (and the shared bound)
        // come early.  Most items finish here at full wave width; a list that would outgrow LDS is dealt
        // to the lanes' own stacks for depth-first walks.
        uint2* W = &front[wv][0][0];  // kWork contiguous entries
        constexpr int kWork = 2 * kFront;
        // pass 1's unexplored entries (oldest first, its pending node on top), or the root
        // (a split item's part p: entries p, p + K, p + 2K, ... in their order; the root, when pass 1 left none, to part 0)
        const int rc = (int)r.rcnt;
        int top = 1;
        if (rc > 0 && rc <= kWork - 128) {
            const int cnt = rc > (int)part ? (rc - (int)part + (int)kk - 1) / (int)kk : 0;
            for (int m = lane; m < cnt; m += 64) W[m] = a.resume[r.roff + part + (unsigned)m * kk];
            top = cnt;
        } else if (part != 0) {
            top = 0;
        } else if (lane == 0) {
            W[0] = make_uint2((unsigned)root, 0u);
        }
        __builtin_amdgcn_wave_barrier();
        while (top > 0 && top <= kWork - 128) {
            const int nt = min(64, top);
            const int base = top - nt;
            bool k0 = false, k1 = false;
            uint2 e0, e1;
            int lf0 = -1, lf1 = -1;  // leaves to test: a resumed leaf entry, or leaf children within the bound
            if (lane < nt) {
                const uint2 e = W[base + lane];
                if (__uint_as_float(e.y) <= pol.limf) {
                    if ((int)e.x < 0) {
                        lf0 = ~(int)e.x;
                    } else {
                        const NodeV nd = load_node(a.nodes, (int)e.x);
                        ++n_nodes;
                        float d0, d1;
                        node_child_bounds(nd, qf, d0, d1);
                        const int c0 = nd.child(0), c1 = nd.child(1);
                        if (d0 <= pol.limf) {
                            if (c0 < 0) lf0 = ~c0;
                            else { k0 = true; e0 = make_uint2((unsigned)c0, __float_as_uint(d0)); }
                        }
                        if (d1 <= pol.limf) {
                            if (c1 < 0) lf1 = ~c1;
                            else { k1 = true; e1 = make_uint2((unsigned)c1, __float_as_uint(d1)); }
                        }
                    }
                }
            }
#pragma nounroll
            for (int j = 0; j < 2; ++j) {  // one call site of the construction
                const int lf = j == 0 ? lf0 : lf1;
                if (lf >= 0) {
                    pol.test(lf);
                    ++n_leaves;
                }
            }
            __builtin_amdgcn_wave_barrier();
            const unsigned long long b0 = __ballot(k0), b1 = __ballot(k1);
            const int p0 = base + __popcll(b0 & lt) + __popcll(b1 & lt);
            if (k0) W[p0] = e0;
            if (k1) W[p0 + (k0 ? 1 : 0)] = e1;
            top = base + __popcll(b0) + __popcll(b1);
            __builtin_amdgcn_wave_barrier();
            pol.shared = fmin(pol.shared, wave_min(pol.best));
            share();
            pol.relim();
        }
        // overflow: deal the list to the lanes (entry j -> lane j % 64), then depth-first walks
        const int n = top;
        Walker w{0, 0};
        if (lane < n)
            for (int j = lane + ((n - 1 - lane) / 64) * 64; j >= lane; j -= 64) w.push(W[j].x, W[j].y, lds, spill);
        bool active = w.pop(pol, lds, spill);
        while (__any(active)) {
            if (active) active = w.step<decltype(pol), false>(a.nodes, qf, pol, lds, spill, n_nodes, n_leaves);
            pol.shared = fmin(pol.shared, wave_min(pol.best));
            share();
            pol.relim();
        }
        double best = pol.best;
        uint32_t face = pol.best_face;
        int leaf = pol.best_leaf;
        wave_lexmin(best, face, leaf);
        if (split) {  // the part's candidate; k_knn_combine merges the item's parts and writes the answer
            if (lane == 0 && !STATS) a.cand[(size_t)hidx * K + part] = P2Cand{best, face, leaf};
        } else if (lane == 0 && !STATS) {
            pol.best = best;
            pol.best_face = face;
            pol.best_leaf = leaf;
            write_result<MODE>(a, i, q, pol);
        }
        if (STATS) {  // per-item work: stats[44] sum and stats[45] max of node + leaf visits over the wave
            unsigned w = (n_nodes - item_nodes0) + (n_leaves - item_leaves0);
            for (int o = 32; o > 0; o >>= 1) w += (unsigned)__shfl_xor((int)w, o);
            if (lane == 0) {
                atomicAdd(&a.stats[44], (unsigned long long)w);
                atomicMax(&a.stats[45], (unsigned long long)w);
                atomicAdd(&a.stats[46], 1ull);
                a.deferred[item].sbound = w;  // development dump (MESH_AMD_P2_DUMP): the item's visits
            }
        }
        __builtin_amdgcn_wave_barrier();
    }
    if (STATS) {
        atomicAdd(&a.stats[0], (unsigned long long)n_nodes);
        atomicAdd(&a.stats[1], (unsigned long long)n_leaves);
        if (lane == 0) atomicAdd(&a.stats[6], 1ull);  // waves x deferred items (pass-2 work units)
    }
}

// pass 2's plan: the deferred items whose pass-1 distance is within kP2Heavy of the largest are listed in heavy[]
// (sbound +inf, the parts' shared bound); every other item is marked to run whole (sbound kP2Whole)
__global__ __launch_bounds__(kBlock) void k_p2_plan(KnnArgs a) {
    const unsigned total = min(*a.n_deferred, a.max_deferred);
    const double mb = __longlong_as_double((long long)*a.max_best);
    const double thr = mb * (kP2Heavy * kP2Heavy);
    for (unsigned k = blockIdx.x * kBlock + threadIdx.x; k < total; k += gridDim.x * kBlock) {
        uint32_t mark = kP2Whole;
        if (a.deferred[k].best >= thr) {
            const unsigned h = atomicAdd(a.n_heavy, 1u);
            if (h < kP2SplitItems) {
                a.heavy[h] = k;
                mark = 0x7F800000u;
            }
        }
        a.deferred[k].sbound = mark;
    }
}

// the answers of the split pass-2 items: the lexicographic (d2, face) minimum of their parts' candidates (each
// part starts from the pass-1 candidate, so every part holds a real one)
template <int MODE>
__global__ __launch_bounds__(kBlock) void k_knn_combine(KnnArgs a) {
    if constexpr (MODE == 0 || MODE == 3) {
        const unsigned nsplit = min(*a.n_heavy, kP2SplitItems);
        const unsigned h = blockIdx.x * kBlock + threadIdx.x;
        if (h >= nsplit) return;
        const DeferRec r = a.deferred[a.heavy[h]];
        const size_t i = r.slot;
        const D3 q = load_q(a, i);
        auto pol = make_pol<MODE>(a, i, q);
        pol.best = r.best;
        pol.best_face = r.face;
        pol.best_leaf = r.leaf;
#pragma unroll
        for (unsigned p = 0; p < kP2Split; ++p) {
            const P2Cand c = a.cand[(size_t)h * kP2Split + p];
            if (c.leaf >= 0) pol.offer(c.best, c.face, c.leaf);
        }
        write_result<MODE>(a, i, q, pol);
    }
}

// ---- query ordering: Morton codes, slot-order gather, scatter back ----
__global__ __launch_bounds__(kBlock) void k_query_morton(const double* __restrict__ q, size_t S, float lx, float ly, float lz,
                                                         float hx, float hy, float hz, uint32_t* __restrict__ keys,
                                                         uint32_t* __restrict__ vals) {
    const size_t i = (size_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= S) return;
    keys[i] = query_morton30(q[3 * i], q[3 * i + 1], q[3 * i + 2], lx, ly, lz, hx, hy, hz);
    vals[i] = (uint32_t)i;
}

constexpr float kQueryBoxMargin = 0.1f;
void query_box(const msh_tree* tree, float* lo, float* hi) {
    for (int k = 0; k < 3; ++k) {
        const float e = tree->scene_hi[k] - tree->scene_lo[k];
        lo[k] = tree->scene_lo[k] - kQueryBoxMargin * e;
        hi[k] = tree->scene_hi[k] + kQueryBoxMargin * e;
    }
}

int query_morton(const msh_tree* tree, const double* d_q, size_t S, uint32_t* keys, uint32_t* vals, hipStream_t s) {
    if (S == 0) return MSH_OK;
    TimedLaunch tl("morton", s);
    // The cells span the scene box widened by 10 % of its extent on each side: queries just outside the
    // mesh box (scan points, a query box a little larger than the mesh) keep their spatial order instead of
    // being clamped onto the boundary cells in the caller's order (C3: 25 % of the queries lie outside
    // the unit sphere's box; 1143 -> 1154-1158 M q/s for 5-20 % margins; a reduction over the queries to
    // fit the box exactly cost 0.9 ms and gained nothing net)
    float lo[3], hi[3];
    query_box(tree, lo, hi);
    k_query_morton<<<(unsigned)((S + kBlock - 1) / kBlock), kBlock, 0, s>>>(d_q, S, lo[0], lo[1], lo[2], hi[0], hi[1],
                                                                           hi[2], keys, vals);
    MSH_HIP(hipGetLastError());
    return MSH_OK;
}

// slot i <- row perm[i] of the caller's (S, 3) array (two arrays at once when b != nullptr);
// inv[perm[i]] = i
__global__ __launch_bounds__(kBlock) void k_gather_rows(const double* __restrict__ a, const double* __restrict__ b,
                                                        const uint32_t* __restrict__ perm, size_t S,
                                                        double* __restrict__ as, double* __restrict__ bs,
                                                        uint32_t* __restrict__ inv) {
    const size_t i = (size_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= S) return;
    const size_t j = perm[i];
    as[3 * i] = a[3 * j];
    as[3 * i + 1] = a[3 * j + 1];
    as[3 * i + 2] = a[3 * j + 2];
    if (b) {
        bs[3 * i] = b[3 * j];
        bs[3 * i + 1] = b[3 * j + 1];
        bs[3 * i + 2] = b[3 * j + 2];
    }
    if (inv) inv[j] = (uint32_t)i;
}

int gather_rows(const double* d_a, const double* d_b, const uint32_t* d_perm, size_t S, double* d_as, double* d_bs,
                uint32_t* d_inv, hipStream_t s) {
    if (S == 0) return MSH_OK;
    TimedLaunch tl("gather", s);
    k_gather_rows<<<(unsigned)((S + kBlock - 1) / kBlock), kBlock, 0, s>>>(d_a, d_b, d_perm, S, d_as, d_bs, d_inv);
    MSH_HIP(hipGetLastError());
    return MSH_OK;
}

// row j of the outputs <- slot inv[j]: face / part / point (or distance) from the 32-B record, nw
// extra doubles per row from w
__global__ __launch_bounds__(kBlock) void k_unpermute(const QRes* __restrict__ res, const double* __restrict__ w, int nw,
                                                      const uint32_t* __restrict__ inv, size_t S, SlotOut o) {
    const size_t j = (size_t)blockIdx.x * kBlock + threadIdx.x;
    if (j >= S) return;
    const size_t i = inv[j];
    const uint4 r0 = reinterpret_cast<const uint4*>(res + i)[0];
    const double2 r1 = reinterpret_cast<const double2*>(res + i)[1];
    const double x = __longlong_as_double((long long)(((unsigned long long)r0.w << 32) | r0.z));
    if (o.face) o.face[j] = r0.x;
    if (o.part) o.part[j] = r0.y;
    if (o.dist) o.dist[j] = x;
    if (o.pt) {
        o.pt[3 * j] = x;
        o.pt[3 * j + 1] = r1.x;
        o.pt[3 * j + 2] = r1.y;
    }
    for (int k = 0; k < nw; ++k) o.w[(size_t)nw * j + k] = w[(size_t)nw * i + k];
}

int unpermute_results(const QRes* d_res, const double* d_w, int nw, const uint32_t* d_inv, size_t S, const SlotOut& o,
                      hipStream_t s) {
    if (S == 0) return MSH_OK;
    TimedLaunch tl("unpermute", s);
    k_unpermute<<<(unsigned)((S + kBlock - 1) / kBlock), kBlock, 0, s>>>(d_res, d_w, nw, d_inv, S, o);
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

#ifndef MSH_BUDGET
#define MSH_BUDGET 512
#endif
constexpr unsigned kBudget = MSH_BUDGET;  // pass-1 node steps per lane before a query is deferred
// super-leaders: their launch has few tiles (C3: 6104 for 8192 wave slots), so its slowest tile sets its
// length; with 256 steps the launch takes 1.4 instead of 2.9 ms and pass 2 gets ~18k more (cheap) items
// (+0.4 ms).  A deferred super-leader publishes its best point so far as its leaders' hint.
constexpr unsigned kBudget3 = 256;
constexpr unsigned kBudget1 = MSH_BUDGET;  // leaders (C3: 13.8 -> 12.6 ms, pass 2 +0.5 ms)
constexpr unsigned kKnnBlocksPerCU = 4;  // resident pass-1 blocks per CU (persistent grid)

// Common launch: grid, counters, spill area, deferred list; pass 1 then pass 2 (both also in STATS
// mode, so the instrumented counts describe the traversal that is timed).
template <int MODE, bool STATS>
static int launch_knn(msh_tree* tree, KnnArgs a, hipStream_t s, const char* timer) {
    if (a.S == 0) return MSH_OK;
    for (int k = 0; k < 3; ++k) a.org[k] = tree->origin[k];
    const unsigned ncu = (unsigned)device_cus(tree->device);
    Workspace& ws = tree->ws;
    // counters: 8 group counters (one 128-B line each) + the deferred count + pass 2's item counter + the resume arena's
    // + the largest deferred best + the heavy items' count
    MSH_TRY(ws.counters.reserve(13 * 32 * sizeof(unsigned)));
    a.counters = ws.counters.as<unsigned>();
    a.n_deferred = a.counters + 8 * 32;
    a.n_resume = a.counters + 10 * 32;
    MSH_HIP(hipMemsetAsync(a.counters, 0, 13 * 32 * sizeof(unsigned), s));  // + the pass-2 item counter
    const size_t n_lead = (a.S + kLead - 1) / kLead;
    const unsigned max_tiles = (unsigned)((a.S + 63) / 64);
    const unsigned nblk_max = std::min<unsigned>((max_tiles + 3) / 4, ncu * kKnnBlocksPerCU);
    // pass 2 lanes carry up to 2 kFront/64 dealt subtrees on top of a depth-first path
    const unsigned nblk2 = ncu * 2;  // pass 2: 2 blocks per CU
    const int need = tree->max_depth + 1 + 2 * kFront / 64 + 1 + (a.cut ? kCutK : 0);
    a.spill = nullptr;
    a.spill_depth = 0;
    if (need > kStack) {
        a.spill_depth = need - kStack + 1;
        MSH_TRY(ws.spill.reserve((size_t)std::max(nblk_max, nblk2) * kBlock * (size_t)a.spill_depth * sizeof(uint2)));
        a.spill = ws.spill.as<uint2>();
    }
    a.budget = kBudget;
    bool list_pf = false;  // list path with the LDS node prefetch and 4-B stack entries (k_knn PF)
    {
        // test hook: 0 per-lane leaf queues (the path of trees of >= 2^26 leaves), 2 the list without the node
        // prefetch (the path of trees of more than 2^20 leaves)
        const char* e = getenv("MESH_AMD_LEAF_LIST");
        const int hook = e ? atoi(e) : 1;
        a.list = (MODE == 0 || MODE == 3) && hook != 0 && tree->B * tree->T < kListMaxLeaves;
        list_pf = a.list && hook != 2 && tree->B * tree->T <= kEnt4MaxLeaves;
    }
    // leader ordering: closest-point launches over a sorted slot order (records in a.res); leader phases only for
    // trees of >= kLeadMinLeaves leaves (on a small tree the hint saves little and the three dependent launches
    // serialise their slowest tiles: C1 0.56 -> 0.29 ms), and only without the entry cut's cell hints: every query inside the cut's grid starts from its cell's entries
    // with the hint leaf of the cell centre, and the leader launch's hints for the followers no longer pay for the
    // launch (C3 100M: 1985-1990 -> 2150-2179 M q/s without leader phases; one N = 8 shard of 12.5M rows 9.0 ->
    // 7.55 ms, profiles/r05_ab_leaders_sort_resume.jsonl); batched trees and trees without a cut keep them
    const bool lead = kLead > 1 && (MODE == 0 || MODE == 3) && a.res != nullptr && a.S >= 64 * (size_t)kLead &&
                      a.T >= kLeadMinLeaves && !(a.list && a.cut);
    a.max_deferred = (unsigned)std::min<size_t>(a.S, (a.S / 16) + 65536);
    DevBuf& dbuf = ws.flags;
    MSH_TRY(dbuf.reserve((size_t)a.max_deferred * sizeof(DeferRec)));
    a.deferred = dbuf.as<DeferRec>();
    a.resume = nullptr;
    a.resume_cap = 0;
    a.cand = nullptr;
    a.heavy = nullptr;
    a.n_heavy = a.counters + 12 * 32;
    a.max_best = reinterpret_cast<unsigned long long*>(a.counters + 11 * 32);
    const unsigned split_cap = std::min<unsigned>(a.max_deferred, kP2SplitItems);
    if (kP2Split > 1 && (MODE == 0 || MODE == 3) && !STATS) {
        MSH_TRY(ws.p2cand.reserve((size_t)split_cap * (kP2Split * sizeof(P2Cand) + sizeof(unsigned))));
        a.cand = ws.p2cand.as<P2Cand>();
        a.heavy = reinterpret_cast<unsigned*>(a.cand + (size_t)split_cap * kP2Split);
    }
#if MSH_RESUME
    if (a.list) {  // resume arena: ~48 entries per expected deferral (C3: 75k deferred of 100M queries), >= 1M entries
        const size_t cap = std::min<size_t>((size_t)1 << 26, std::max<size_t>((size_t)1 << 20, 48 * (a.S / 1024 + 1024)));
        MSH_TRY(ws.resume.reserve(cap * sizeof(uint2)));
        a.resume = ws.resume.as<uint2>();
        a.resume_cap = (unsigned)cap;
    }
#endif
    auto pass1 = [&](int phase, size_t nunits, const char* name) -> int {
        a.phase = phase;
        a.budget = phase == 3 ? kBudget3 : ((phase == 1 || phase == 4) ? kBudget1 : kBudget);
        // small trees: a query that walks T/16 nodes (the centre of a coarse closed mesh) goes to the
        // wave-cooperative pass 2 instead of holding its tile for up to T serial steps (C1, 840 faces:
        // traversal 1.15 -> 0.56 ms; with no leader phases below, 0.29 ms)
        a.budget = std::min<unsigned>(a.budget, (unsigned)std::max<size_t>(64, a.T / 16));
        a.nunits = nunits;
        a.ntiles = (unsigned)((nunits + 63) / 64);
        const unsigned nblk = std::min<unsigned>((a.ntiles + 3) / 4, ncu * kKnnBlocksPerCU);
        if (nblk == 0) return MSH_OK;
        TimedLaunch t1(name, s);
        if (a.list)
            if (list_pf)
                k_knn<MODE, STATS, (MODE == 0 || MODE == 3), (MODE == 0 || MODE == 3)><<<nblk, kBlock, 0, s>>>(a);
            else
                k_knn<MODE, STATS, (MODE == 0 || MODE == 3), false><<<nblk, kBlock, 0, s>>>(a);
        else
            k_knn<MODE, STATS, false, false><<<nblk, kBlock, 0, s>>>(a);
        MSH_HIP(hipGetLastError());
        return MSH_OK;
    };
    {
        TimedLaunch tl(timer, s);
        {
            TimedLaunch t1(STATS ? "knn_pass1_stats" : "knn_pass1", s);
            if (lead) {
                if (a.list && a.cut) {
                    // cell hints serve every leader inside the entry cut's grid, so the super-leaders would only
                    // hint leaders outside it: one leader launch over every leader slot (phase 4; outside the
                    // grid unhinted) instead of a super-leader launch the chip cannot fill
                    MSH_TRY(pass1(4, n_lead, STATS ? "knn_lead_stats" : "knn_lead"));
                } else if (kLead2 > 0) {
                    constexpr size_t l2 = kLead2 ? kLead2 : 1;
                    const size_t n_super = (a.S + l2 - 1) / l2;
                    MSH_TRY(pass1(3, n_super, STATS ? "knn_lead2_stats" : "knn_lead2"));
                    MSH_HIP(hipMemsetAsync(a.counters, 0, 8 * 32 * sizeof(unsigned), s));
                    MSH_TRY(pass1(1, n_lead - n_super, STATS ? "knn_lead_stats" : "knn_lead"));
                } else {
                    MSH_TRY(pass1(1, n_lead, STATS ? "knn_lead_stats" : "knn_lead"));
                }
                MSH_HIP(hipMemsetAsync(a.counters, 0, 8 * 32 * sizeof(unsigned), s));  // group counters only
                MSH_TRY(pass1(2, a.S - n_lead, STATS ? "knn_follow_stats" : "knn_follow"));
            } else {
                MSH_TRY(pass1(0, a.S, STATS ? "knn_all_stats" : "knn_all"));
            }
        }
        {
            TimedLaunch t2(STATS ? "knn_pass2_stats" : "knn_pass2", s);
            if (a.cand) {
                k_p2_plan<<<64, kBlock, 0, s>>>(a);
                MSH_HIP(hipGetLastError());
            }
            k_knn_coop<MODE, STATS><<<nblk2, kBlock, 0, s>>>(a);
            MSH_HIP(hipGetLastError());
            if (a.cand) {
                k_knn_combine<MODE><<<(split_cap + kBlock - 1) / kBlock, kBlock, 0, s>>>(a);
                MSH_HIP(hipGetLastError());
            }
        }
        if (STATS && getenv("MESH_AMD_P2_DUMP")) {  // development: the deferred items with their pass-2 visits
            unsigned nd = 0;
            MSH_HIP(hipMemcpyAsync(&nd, a.n_deferred, sizeof(unsigned), hipMemcpyDeviceToHost, s));
            MSH_HIP(hipStreamSynchronize(s));
            nd = std::min(nd, a.max_deferred);
            std::vector<DeferRec> h(nd);
            if (nd) MSH_HIP(hipMemcpy(h.data(), a.deferred, nd * sizeof(DeferRec), hipMemcpyDeviceToHost));
            if (FILE* f = fopen(getenv("MESH_AMD_P2_DUMP"), "wb")) {
                fwrite(h.data(), sizeof(DeferRec), nd, f);
                fclose(f);
            }
        }
    }
    return MSH_OK;
}


// Slot-order plumbing shared by the point-query launchers: with a permutation the kernels write 32-B
// records (plus nw weights) into the workspace and k_unpermute scatters them to the caller's arrays.
template <int MODE, bool STATS>
static int run_knn(msh_tree* tree, KnnArgs a, const QueryOrder& ord, const SlotOut& o, int nw, hipStream_t s,
                   const char* timer) {
    if (a.S == 0) return MSH_OK;
    a.q = ord.q;
    a.perm = ord.perm;
    if (!ord.gathered) {
        a.qperm = ord.perm;
        a.inv_w = const_cast<uint32_t*>(ord.inv);
    }
    Workspace& ws = tree->ws;
    if (ord.perm) {  // STATS launches keep the records too: followers take their hints from them
        MSH_TRY(ws.res.reserve(a.S * sizeof(QRes)));
        a.res = ws.res.as<QRes>();
        a.direct = !STATS && (MODE == 0 || MODE == 3);
        a.rec_leaf = a.direct || STATS;
        if (nw && !a.direct) {
            MSH_TRY(ws.res_w.reserve(a.S * (size_t)nw * sizeof(double)));
            a.res_w = ws.res_w.as<double>();
        }
        if (a.direct) {
            a.out_face = o.face;
            a.out_part = o.part;
            a.out_pt = o.pt;
            a.out_dist = o.dist;
            a.out_w = o.w;
        }
    } else {
        a.out_face = o.face;
        a.out_part = o.part;
        a.out_pt = o.pt;
        a.out_dist = o.dist;
        a.out_w = o.w;
    }
    MSH_TRY((launch_knn<MODE, STATS>(tree, a, s, timer)));
    if (ord.perm && !STATS && !a.direct) MSH_TRY(unpermute_results(a.res, a.res_w, nw, ord.inv, a.S, o, s));
    return MSH_OK;
}

static KnnArgs tree_args(const msh_tree* tree, size_t S) {
    KnnArgs a{};
    a.nodes = tree->d_nodes;
    a.leaves = tree->d_leaves;
    a.T = tree->T;
    a.S = S;
    a.tm = tree_margin(tree->half_diag);
    return a;
}

// the entry cut of a single tree (list path of the closest-point modes)
static void cut_args(const msh_tree* tree, KnnArgs& a) {
    if (!tree->d_cut || tree->B != 1) return;
    a.cut = tree->d_cut;
    a.cut_wide = tree->cut_wide;
    a.cut_G = tree->cut_G;
    for (int k = 0; k < 3; ++k) {
        a.cut_lo[k] = tree->cut_lo[k];
        a.cut_iw[k] = tree->cut_iw[k];
    }
}

int launch_nearest(const msh_tree* tree, const QueryOrder& ord, size_t S, const SlotOut& o, hipStream_t s) {
    KnnArgs a = tree_args(tree, S);
    cut_args(tree, a);
    SlotOut oo = o;
    oo.dist = nullptr;
    if (o.w) {
        oo.part = nullptr;
        return run_knn<3, false>(const_cast<msh_tree*>(tree), a, ord, oo, 3, s, "nearest");
    }
    return run_knn<0, false>(const_cast<msh_tree*>(tree), a, ord, oo, 0, s, "nearest");
}

int launch_nearest_batch(const msh_tree* tree, const QueryOrder& ord, size_t n, size_t S, const SlotOut& o,
                         hipStream_t s, size_t mesh0) {
    KnnArgs a = tree_args(tree, n);
    a.orgs = tree->d_orgs + 3 * mesh0;
    a.qper = S;
    a.npm = tree->T - 1;
    a.root0 = mesh0 * a.npm;
    SlotOut oo = o;
    oo.dist = nullptr;
    if (o.w) {
        oo.part = nullptr;
        return run_knn<3, false>(const_cast<msh_tree*>(tree), a, ord, oo, 3, s, "nearest_batch");
    }
    return run_knn<0, false>(const_cast<msh_tree*>(tree), a, ord, oo, 0, s, "nearest_batch");
}

int launch_nearest_stats(const msh_tree* tree, const QueryOrder& ord, size_t S, unsigned long long* d_counts,
                         hipStream_t s) {
    KnnArgs a = tree_args(tree, S);
    cut_args(tree, a);
    a.stats = d_counts;
    return run_knn<0, true>(const_cast<msh_tree*>(tree), a, ord, SlotOut{}, 0, s, "nearest_stats");
}

int launch_nnearest(const msh_tree* tree, const QueryOrder& ord, size_t S, const SlotOut& o, hipStream_t s) {
    KnnArgs a = tree_args(tree, S);
    a.n = ord.n;
    a.eps = tree->eps;
    SlotOut oo = o;
    oo.part = nullptr;
    oo.dist = nullptr;
    oo.w = nullptr;
    return run_knn<1, false>(const_cast<msh_tree*>(tree), a, ord, oo, 0, s, "nnearest");
}

int launch_points_nearest(const msh_tree* tree, const QueryOrder& ord, size_t S, const SlotOut& o, hipStream_t s) {
    KnnArgs a = tree_args(tree, S);
    SlotOut oo{};
    oo.face = o.face;
    oo.dist = o.dist;
    return run_knn<2, false>(const_cast<msh_tree*>(tree), a, ord, oo, 0, s, "points_nearest");
}

// ---- entry cut (build time) ----
// cell (ix, iy, iz) = row (iz G + iy) G + ix; centre lo + (i + 1/2) w per axis
__global__ __launch_bounds__(kBlock) void k_cut_centres(int G, double lx, double ly, double lz, double wx, double wy,
                                                        double wz, double* __restrict__ q) {
    const size_t n = (size_t)G * G * G;
    const size_t cell = (size_t)blockIdx.x * kBlock + threadIdx.x;
    if (cell >= n) return;
    const size_t ix = cell % (size_t)G, iy = (cell / (size_t)G) % (size_t)G, iz = cell / ((size_t)G * G);
    q[3 * cell] = lx + ((double)ix + 0.5) * wx;
    q[3 * cell + 1] = ly + ((double)iy + 0.5) * wy;
    q[3 * cell + 2] = lz + ((double)iz + 0.5) * wz;
}

// The entry cut, one thread per cell of a G^3 grid (cell (ix, iy, iz) = row (iz G + iy) G + ix), from the root (or from
// the records of the installed half-resolution grid, d_half below), with
// U(c) = the exact distance from the centre c to its closest point (pts[cell], the centre's own query; its face's leaf
// is hint[cell]).
// R = (U(c) + 2r) (1 + 1e-6), r the cell's half-diagonal + 0.1 %.  For q in the cell, d(q) <= U(c) + r, so a subtree
// farther than R from c holds neither q's answer nor a tie.  Entries (internal nodes or ~leaves) are replaced by their
// children whose bound from c is within R, in passes over the list, while it keeps at most kCutK entries; a child
// outside R is dropped (the cull is the traversal's own: bound > fp32(R^2 (1 + 2^-40)) rounded up).  An entry's bound
// from c: its box bound when its parent node was expanded, raised to the smaller of its children's bounds when its own
// node is loaded -- each a lower bound of the squared distance from c to what it holds.  (Exact leaf distances as the
// leaves' bounds, dropping leaves beyond R: 0.4 % fewer leaf tests per query for 10 ms more of build on C3,
// profiles/r06_c3_cut_build_probe.jsonl.)  An entry that cannot be expanded is retried only once the list shrank.
// Out (E4: 32-B records of 4-B entries, trees of <= 2^20 leaves; else 64-B records: word 1 the radius R around c the
// list covers, then (ref, bound bits) pairs): word 0 the hint leaf, then the entries nearest-first with max(s, 0)^2
// rounded down to fp32, s = sqrt(bound) (1 - 1e-5) - r (1 + 1e-5): a lower bound of the squared distance from any q
// of the cell.
template <bool E4>
__global__ __launch_bounds__(kBlock) void k_cut_level(const BNode* __restrict__ nodes, const TriRec* __restrict__ tris,
                                                      double ox, double oy, double oz, double tm, int G, double lx,
                                                      double ly, double lz, double wx, double wy, double wz,
                                                      const double* __restrict__ pts, const int* __restrict__ hint,
                                                      uint32_t* __restrict__ rec, const uint32_t* __restrict__ crec) {
    constexpr int kw = E4 ? 8 : 16;  // record words
    // a wave takes a 4 x 4 x 4 brick of cells (bricks in row order): its cells' start lists share their nodes, and
    // under a half-resolution grid it reads 8 records
    const size_t gid = (size_t)blockIdx.x * kBlock + threadIdx.x;
    const size_t GB = ((size_t)G + 3) / 4, brick = gid >> 6;
    const unsigned ln = (unsigned)(gid & 63);
    if (brick >= GB * GB * GB) return;
    const size_t ix = (brick % GB) * 4 + (ln & 3), iy = ((brick / GB) % GB) * 4 + ((ln >> 2) & 3),
                 iz = (brick / (GB * GB)) * 4 + (ln >> 4);
    if (ix >= (size_t)G || iy >= (size_t)G || iz >= (size_t)G) return;
    const size_t cell = (iz * G + iy) * G + ix;
    const D3 c = D3{lx + ((double)ix + 0.5) * wx, ly + ((double)iy + 0.5) * wy, lz + ((double)iz + 0.5) * wz};
    const double r = 0.5 * sqrt(wx * wx + wy * wy + wz * wz) * 1.001;
    int ref[kCutK];
    float bd[kCutK];  // bound from c; -1: not formed yet (the root)
    int stuck[kCutK];  // list size at which the entry could not be expanded (0: not stuck): retried only once smaller
    const int best_leaf = hint[cell];
    ref[0] = 0;
    bd[0] = -1.f;
    stuck[0] = 0;
    int m = 1;
    // U(c): the distance from c to its answer's point (pts: the centre walks' closest points; NaN without an answer)
    const D3 pc = D3{pts[3 * cell], pts[3 * cell + 1], pts[3 * cell + 2]};
    float limf = INFINITY;
    {
        const double R = (sqrt(sqdist(c, pc)) + 2.0 * r) * (1.0 + 1e-6);
        if (R < INFINITY) limf = __double2float_ru(R * R * kSlack);  // NaN / inf (no answer): the root only
    }
    if (crec) {
        // start from the enclosing cell of the half-resolution grid (G = 2 Gc, the same box): a subtree its record left
        // out lies farther than d(q) from every q of that cell, this one's included.  Its entries keep their records'
        // bounds -- already lower bounds for every q of the larger cell -- as (sqrt(b) + r)^2, which the store below
        // maps back to <= sqrt(b); a node's bound is raised when it is loaded
        const size_t Gc = (size_t)G / 2;
        const uint32_t* cr = crec + (((iz >> 1) * Gc + (iy >> 1)) * Gc + (ix >> 1)) * kw;
        m = 0;
        for (int k = 0; k < kCutK; ++k) {
            uint32_t rv, bb;
            if (E4) {
                const uint32_t e = cr[1 + k];
                if (e & 0x80000000u) break;  // empty: the list ends
                rv = (uint32_t)Ent4::ref(e);
                bb = __float_as_uint(Ent4::bound(e));
            } else {
                rv = cr[2 + 2 * k];
                if (rv == kCutEmpty) break;
                bb = cr[3 + 2 * k];
            }
            if (__uint_as_float(bb) > limf) continue;  // farther than R from c (its bound holds from c too)
            const float sb = sqrtf(__uint_as_float(bb)) + (float)r;
            ref[m] = (int)rv;
            bd[m] = sb * sb;  // its rounding is far inside the store's 1e-5 shrink
            stuck[m] = 0;
            ++m;
        }
        if (m == 0) {
            ref[0] = 0;
            bd[0] = -1.f;
            m = 1;
        }
    }
    const double o3[3] = {ox, oy, oz};
    const QF qf = make_qf(c, o3, tm);
    if (m > 0 && limf < INFINITY) {
        for (int pass = 0; pass < 256; ++pass) {
            bool changed = false;
            const int m0 = m;
            for (int k = 0; k < m0 && k < m; ++k) {
                if (ref[k] < 0) continue;  // a leaf: final, with its box bound
                if (stuck[k] && m >= stuck[k]) continue;  // no room has been freed since it was stuck: no reload
                const NodeV nd = load_node(nodes, ref[k]);
                float d0, d1;
                node_child_bounds(nd, qf, d0, d1);
                bd[k] = fmaxf(bd[k], fminf(d0, d1));
                const bool h0 = d0 <= limf, h1 = d1 <= limf;
                const int cnt = (int)h0 + (int)h1;
                if (m - 1 + cnt > kCutK) {
                    stuck[k] = m;
                    continue;
                }
                changed = true;
                if (cnt == 0) {  // nothing within R below this entry
                    ref[k] = ref[m - 1];
                    bd[k] = bd[m - 1];
                    stuck[k] = stuck[m - 1];
                    --m;
                    continue;
                }
                const int c0 = nd.child(0), c1 = nd.child(1);
                stuck[k] = 0;
                if (h0) {
                    ref[k] = c0;
                    bd[k] = d0;
                    if (h1) {
                        ref[m] = c1;
                        bd[m] = d1;
                        stuck[m] = 0;
                        ++m;
                    }
                } else {
                    ref[k] = c1;
                    bd[k] = d1;
                }
            }
            if (!changed || m == 0) break;
        }
    }
    if (m == 0) {  // no answer for c, or (cannot happen for a consistent tree) nothing within R: the root
        ref[0] = 0;
        bd[0] = 0.f;
        m = 1;
    }
    for (int k = 1; k < m; ++k)  // nearest first
        for (int j = k; j > 0 && bd[j] < bd[j - 1]; --j) {
            const int tr = ref[j];
            ref[j] = ref[j - 1];
            ref[j - 1] = tr;
            const float tb = bd[j];
            bd[j] = bd[j - 1];
            bd[j - 1] = tb;
        }
    uint32_t* out = rec + cell * kw;
    out[0] = (uint32_t)best_leaf;
    // 64-B records: word 1 the radius R around c the list covers (every subtree left out lies farther from c), fp32
    // rounded down (0: none) -- the alongnormal walks' first phase reads it (rays.hip)
    if (!E4) out[1] = limf < INFINITY ? __float_as_uint(__double2float_rd(sqrt((double)limf / kSlack) * (1.0 - 1e-7))) : 0u;
    for (int k = 0; k < kCutK; ++k) {
        uint32_t ev = 0xFFFFFFFFu, rv = kCutEmpty, bb = 0u;
        if (k < m) {
            const double b = bd[k] > 0.f ? (double)bd[k] : 0.0;
            const double sv = sqrt(b) * (1.0 - 1e-5) - r * (1.0 + 1e-5);
            bb = __float_as_uint(sv > 0.0 ? __double2float_rd(sv * sv) : 0.f);
            ev = Ent4::make((uint32_t)ref[k], bb);
            rv = (uint32_t)ref[k];
        }
        if (E4) {
            out[1 + k] = ev;
        } else {
            out[2 + 2 * k] = rv;
            out[3 + 2 * k] = bb;
        }
    }
}

__global__ __launch_bounds__(kBlock) void k_face_leaf(const TriRec* __restrict__ tris, size_t T, uint32_t* __restrict__ inv) {
    const size_t l = (size_t)blockIdx.x * kBlock + threadIdx.x;
    if (l >= T) return;
    D3 x, y, z;
    uint32_t face;
    load_tri(tris, (int)l, x, y, z, face);
    if (face < T) inv[face] = (uint32_t)l;
}
__global__ __launch_bounds__(kBlock) void k_cut_hint(const uint32_t* __restrict__ face, size_t n, size_t T,
                                                     const uint32_t* __restrict__ inv, int* __restrict__ hint) {
    const size_t c = (size_t)blockIdx.x * kBlock + threadIdx.x;
    if (c >= n) return;
    const uint32_t f = face[c];
    hint[c] = f < T ? (int)inv[f] : -1;
}

// The closest point and part code of each row on a GIVEN face: the fp64 construction the traversal's answer store
// runs for its winning face (write_result), so for a row the traversal answered with face f this gives the
// traversal's point and part bit for bit.  Rows with face MSH_NO_FACE (or >= T) get NaN and part 0, as the
// traversal's non-finite rows do.  The narrow result exchange (mesh_amd/distributed.py NarrowRing) all-gathers
// faces only and rebuilds the other ranks' points with it.  inv: face -> leaf (k_face_leaf).
__global__ __launch_bounds__(kBlock) void k_points_from_faces(const TriRec* __restrict__ tris, const uint32_t* __restrict__ inv,
                                                              size_t T, const double* __restrict__ q, size_t S,
                                                              const uint32_t* __restrict__ face, uint32_t* __restrict__ part,
                                                              double* __restrict__ pt) {
    const size_t i = (size_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= S) return;
    const uint32_t f = face[i];
    D3 o = D3{NAN, NAN, NAN};
    int pc = 0;
    if (f < T) {
        D3 ta, tb, tc;
        uint32_t ff;
        load_tri(tris, (int)inv[f], ta, tb, tc, ff);
        closest_on_triangle(D3{q[3 * i], q[3 * i + 1], q[3 * i + 2]}, ta, tb, tc, o, pc);
    }
    if (part) part[i] = (uint32_t)pc;
    pt[3 * i] = o.x;
    pt[3 * i + 1] = o.y;
    pt[3 * i + 2] = o.z;
}

int face_leaf_map(const msh_tree* tree, uint32_t* d_inv, hipStream_t s) {
    const size_t T = tree->T;
    k_face_leaf<<<(unsigned)((T + kBlock - 1) / kBlock), kBlock, 0, s>>>(static_cast<const TriRec*>(tree->d_leaves), T,
                                                                          d_inv);
    MSH_HIP(hipGetLastError());
    return MSH_OK;
}

int points_from_faces(const msh_tree* tree, const uint32_t* d_inv, const double* d_q, size_t S, const uint32_t* d_face,
                      uint32_t* d_part, double* d_pt, hipStream_t s) {
    if (S == 0) return MSH_OK;
    TimedLaunch tl("points_from_faces", s);
    k_points_from_faces<<<(unsigned)((S + kBlock - 1) / kBlock), kBlock, 0, s>>>(
        static_cast<const TriRec*>(tree->d_leaves), d_inv, tree->T, d_q, S, d_face, d_part, d_pt);
    MSH_HIP(hipGetLastError());
    return MSH_OK;
}

int cut_hints(const msh_tree* tree, const uint32_t* d_face, size_t n, uint32_t* d_inv, int* d_hint, hipStream_t s) {
    const size_t T = tree->T;
    k_face_leaf<<<(unsigned)((T + kBlock - 1) / kBlock), kBlock, 0, s>>>(static_cast<const TriRec*>(tree->d_leaves), T,
                                                                          d_inv);
    MSH_HIP(hipGetLastError());
    k_cut_hint<<<(unsigned)((n + kBlock - 1) / kBlock), kBlock, 0, s>>>(d_face, n, T, d_inv, d_hint);
    MSH_HIP(hipGetLastError());
    return MSH_OK;
}

int cut_centres(int G, const double* lo, const double* w, double* d_q, hipStream_t s) {
    const size_t n = (size_t)G * G * G;
    k_cut_centres<<<(unsigned)((n + kBlock - 1) / kBlock), kBlock, 0, s>>>(G, lo[0], lo[1], lo[2], w[0], w[1], w[2], d_q);
    MSH_HIP(hipGetLastError());
    return MSH_OK;
}

int cut_level(const msh_tree* tree, int G, const double* lo, const double* w, const double* d_pts, const int* d_hint,
              uint32_t* d_rec, bool e4, hipStream_t s, const uint32_t* d_half) {
    const size_t GB = ((size_t)G + 3) / 4;  // 4^3-cell bricks, one per wave
    const unsigned nb = (unsigned)((GB * GB * GB * 64 + kBlock - 1) / kBlock);
    const TriRec* tris = static_cast<const TriRec*>(tree->d_leaves);
    const double tm = tree_margin(tree->half_diag);
    TimedLaunch tl("cut_level", s);
    if (e4)
        k_cut_level<true><<<nb, kBlock, 0, s>>>(tree->d_nodes, tris, tree->origin[0], tree->origin[1], tree->origin[2], tm,
                                               G, lo[0], lo[1], lo[2], w[0], w[1], w[2], d_pts, d_hint, d_rec, d_half);
    else
        k_cut_level<false><<<nb, kBlock, 0, s>>>(tree->d_nodes, tris, tree->origin[0], tree->origin[1], tree->origin[2], tm,
                                                G, lo[0], lo[1], lo[2], w[0], w[1], w[2], d_pts, d_hint, d_rec, d_half);
    MSH_HIP(hipGetLastError());
    return MSH_OK;
}

}  // namespace msh
