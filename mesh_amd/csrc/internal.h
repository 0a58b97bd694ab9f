// Host-side internals of libmeshsearch: the handle, device buffers, error plumbing and the kernel
// launchers implemented in the .hip translation units.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include <string>
#include <vector>

#include "../../include/meshsearch.h"
#include "common.h"

namespace msh {

void set_error(const char* fmt, ...);

#define MSH_HIP(expr)                                                                           \
    do {                                                                                        \
        hipError_t _e = (expr);                                                                 \
        if (_e != hipSuccess) {                                                                 \
            ::msh::set_error("HIP error %s at %s:%d: %s", hipGetErrorName(_e), __FILE__, __LINE__, #expr); \
            return (_e == hipErrorOutOfMemory) ? MSH_ENOMEM : MSH_EDEVICE;                       \
        }                                                                                       \
    } while (0)

#define MSH_TRY(expr)               \
    do {                            \
        int _s = (expr);            \
        if (_s != MSH_OK) return _s; \
    } while (0)

// Device allocations through the library's cache (api.cpp DevCache): dfree keeps the block for the next request of a
// similar size on its device (after waiting for the device, as hipFree does).
hipError_t dmalloc_raw(void** p, size_t bytes);
hipError_t dfree(void* p);
template <class T>
inline hipError_t dmalloc(T** p, size_t bytes) {
    void* v = nullptr;
    const hipError_t e = dmalloc_raw(&v, bytes);
    *p = static_cast<T*>(v);
    return e;
}
size_t dcache_trim();
size_t dcache_bytes();

// Grow-only device scratch buffer.  Owning and move-only: a scope's buffers are freed when it ends (hipFree
// waits for the device, so a buffer still read by queued launches is not released under them).
struct DevBuf {
    void* ptr = nullptr;
    size_t bytes = 0;
    DevBuf() = default;
    DevBuf(const DevBuf&) = delete;
    DevBuf& operator=(const DevBuf&) = delete;
    DevBuf(DevBuf&& o) noexcept : ptr(o.ptr), bytes(o.bytes) { o.ptr = nullptr; o.bytes = 0; }
    DevBuf& operator=(DevBuf&& o) noexcept {
        if (this != &o) {
            release();
            ptr = o.ptr;
            bytes = o.bytes;
            o.ptr = nullptr;
            o.bytes = 0;
        }
        return *this;
    }
    ~DevBuf() { release(); }
    int reserve(size_t need);
    void release();
    template <class T>
    T* as() const { return static_cast<T*>(ptr); }
};

// Reusable per-handle scratch (query keys / permutation / sort temporaries / slot-order queries and
// results / staging).
struct Workspace {
    DevBuf keys, vals, keys_alt, vals_alt, hist, scan, q, n, out_a, out_b, out_c, out_d, flags, counters, spill, stats,
        ranges, qs, ns, inv, res, res_w, resume, p2cand;
    void release();
    size_t bytes() const;
};

enum Kind { kTriangles = 0, kNormals = 1, kPoints = 2 };

// 32-B slot-order result record written (coalesced) by the traversal kernels: face / index, part code,
// point (or distance in x for point trees).
struct alignas(16) QRes {
    uint32_t face, part;
    double x, y, z;
};
static_assert(sizeof(QRes) == 32, "QRes must be 32 B");
// one record as two 16-B stores
__device__ inline void store_qres(QRes* r, uint32_t face, uint32_t part, double x, double y, double z) {
    const unsigned long long xb = (unsigned long long)__double_as_longlong(x);
    reinterpret_cast<uint4*>(r)[0] = make_uint4(face, part, (uint32_t)xb, (uint32_t)(xb >> 32));
    reinterpret_cast<double2*>(r)[1] = make_double2(y, z);
}

// Caller-order output arrays of a point query (nullptr = not wanted).  w: per-row extra doubles
// (barycentric weights, or the ray distance).
struct SlotOut {
    uint32_t* face;
    uint32_t* part;
    double* pt;
    double* dist;
    double* w;
};

// Order in which a launch visits its queries: q (and n) are the rows in slot order; perm maps a slot
// to the caller's row and inv back (both nullptr: identity, the caller's arrays are used directly).
// gathered == false: q (and n) are still the caller's rows; the traversal reads row perm[i] for slot i
// and records inv itself (closest-point launches)
struct QueryOrder {
    const double* q;
    const double* n;
    const uint32_t* perm;
    const uint32_t* inv;
    bool gathered = true;
};

}  // namespace msh

struct msh_tree {
    int device = 0;
    int kind = msh::kTriangles;
    double eps = 0.0;
    size_t P = 0;        // main-mesh vertices
    size_t T = 0;        // leaf primitives
    size_t T_main = 0;   // main-mesh faces (visibility: extra faces follow)
    size_t B = 1;        // meshes in a batched tree (msh_batch_build; P, T are per mesh); 1 otherwise
    double* d_v = nullptr;         // (P,3) main vertices (visibility sources)
    msh::BNode* d_nodes = nullptr; // T-1 internal nodes (nullptr when T == 1)
    void* d_leaves = nullptr;      // T TriRec or PtRec in Morton order
    float scene_lo[3] = {0, 0, 0}, scene_hi[3] = {0, 0, 0};  // bbox of all primitives
    double origin[3] = {0, 0, 0};  // fp64 scene-box centre: all fp32 node bounds are relative to it
    double half_diag = 0.0;        // largest half-diagonal of the (per-mesh) boxes around their origins
    double* d_orgs = nullptr;      // (B,3) per-mesh origins on the device (B = 1: a copy of origin)
    double* d_boxes = nullptr;     // (B,6) per-mesh boxes (batched trees: query Morton codes)
    uint32_t* d_vorder = nullptr;  // Morton order of the main vertices (lazily built for visibility)
    uint32_t* d_vorder_shard = nullptr;  // Morton order of vertices [vshard_v0, +vshard_nv) (last shard asked for)
    size_t vshard_v0 = 0, vshard_nv = 0;
    hipStream_t stream = nullptr;
    hipEvent_t ws_done = nullptr;  // recorded after the last launch that used `ws` (stream ordering)
    // host-call staging (lazily created, grow-only): two pinned host slabs, two device slabs, copy
    // streams and their events (api.cpp pipelined())
    void* h_stage[2] = {nullptr, nullptr};
    void* d_stage[3] = {nullptr, nullptr, nullptr};  // device slabs: a ring of 3 (pipelined)
    size_t stage_bytes = 0;   // device slabs
    size_t hstage_bytes = 0;  // host slabs (inputs only when results go straight into pinned arrays)
    hipStream_t s_up = nullptr, s_down = nullptr;
    hipEvent_t e_up[3] = {nullptr, nullptr, nullptr}, e_run[3] = {nullptr, nullptr, nullptr},
               e_down[3] = {nullptr, nullptr, nullptr};
    double build_ms = 0.0;
    int max_depth = 0;             // bound of the deepest leaf (root children = 1): k_karras prefix lengths
    // entry cut (single triangle trees; api.cpp build_entry_cut): a G^3 grid over the scene box widened by 1/4, one
    // record per cell -- its hint leaf and kCutK start entries, 32 B (4-B entries, trees of <= 2^20 leaves) or 64 B
    // (cut_wide) --; d_cut == nullptr: every query starts at the root
    uint32_t* d_cut = nullptr;
    int cut_wide = 0;
    uint32_t* d_face_leaf = nullptr;  // face -> leaf (msh_tree_points_from_faces_device; built on first use)
    int cut_G = 0;
    // lazily built on the first closest-point query (msh_tree_set_entry_cut): requested grid (< 0 automatic,
    // 0 off), state (0 pending, 1 built, 2 off / not applicable, 3 failed), GPU build time
    int cut_req = -1;
    int cut_state = 0;
    bool cut_force = false;   // msh_tree_set_entry_cut was called: build at the next query, whatever its size
    uint64_t cut_rows = 0;    // closest-point rows answered while the automatic cut waits (ensure_entry_cut)
    int cut_fails = 0;        // failed automatic builds (retried after another threshold of rows, at most twice)
    bool cut_fine = false;    // the built grid is the fine automatic one (or a requested one): no upgrade
    double cut_ms = 0.0;
    double cut_lo[3] = {0, 0, 0}, cut_iw[3] = {0, 0, 0};
    msh::Workspace ws;
    // copies of this tree on the other devices of msh_set_devices / msh_set_device_list (owned; freed with it):
    // host-buffer calls split their rows over this handle and its replicas
    std::vector<msh_tree*> replicas;
    // batched builds return before their last kernels finish (api.cpp msh_batch_build): the build's temporaries
    // (device pointers and its workspace) are freed, and build_ms read, once pend_done has passed (finish_pending)
    bool pending = false;
    std::vector<void*> pend_free;
    msh::Workspace pend_ws;
    hipEvent_t pend_e0 = nullptr, pend_done = nullptr;
};

namespace msh {

// ---- radix sort (sort.hip): stable LSD sort of (u32 key, u32 value) pairs on the low `bits` bits.
// Result ends in keys/vals (the alt buffers are temporaries) — or, with in_alt and an odd number of
// passes, in keys_alt/vals_alt (*in_alt = true) without the copy back.  lo_bit: first key bit sorted.
int radix_sort_pairs(uint32_t* keys, uint32_t* vals, uint32_t* keys_alt, uint32_t* vals_alt, size_t n, int bits,
                     Workspace& ws, hipStream_t s, int lo_bit = 0, bool* in_alt = nullptr);
// exclusive scan of u32 (in place), n elements
int exclusive_scan_u32(uint32_t* data, size_t n, Workspace& ws, hipStream_t s);

// ---- LBVH build (build.hip) ----
// prim_lo/prim_hi: (T,3) fp64 bounds per primitive on device.  Builds nodes and the Morton order
// `order` (sorted position -> primitive id).  scene box written to tree.
int build_lbvh(msh_tree* tree, const double* d_prim_lo, const double* d_prim_hi, size_t T, uint32_t* d_order);
// Batched LBVH over tree->B meshes of T primitives each (bounds (B*T,3), mesh b's primitives at
// [bT, (b+1)T)): per-mesh boxes/origins, Morton codes, two-phase stable radix sort (Morton, then mesh),
// per-mesh Karras emission with global child references, refit.
int build_lbvh_batch(msh_tree* tree, const double* d_prim_lo, const double* d_prim_hi, size_t T, uint32_t* d_order);
int tri_bounds_batch(const double* d_v, size_t P, const uint32_t* d_f, size_t B, size_t T, double* d_lo, double* d_hi,
                     hipStream_t s);
int pack_tri_leaves_batch(const double* d_v, size_t P, const uint32_t* d_f, const uint32_t* d_order, size_t B, size_t T,
                          TriRec* d_out, hipStream_t s);
// Morton codes of (B*S,3) queries in their mesh's box (query i belongs to mesh mesh0 + i / S) + iota values.
int query_morton_batch(const msh_tree* tree, const double* d_q, size_t n, size_t S, uint32_t* keys, uint32_t* vals,
                       hipStream_t s, size_t mesh0 = 0);
// keys[j] = vals[j] / per (the mesh of element vals[j]), for the second, per-mesh sort phase
int mesh_keys(const uint32_t* vals, size_t n, size_t per, uint32_t* keys, hipStream_t s);
// largest distance from origin to a corner of box (lo xyz, hi xyz): msh_tree::half_diag
double half_diagonal(const double* box, const double* origin);
// device copy of tree->origin (single-mesh trees; blob unpack)
int upload_origin(msh_tree* tree, hipStream_t s);
// Top-down re-split of every LBVH subtree over at most 2^log2K leaves (refine.hip): the same node ids,
// ranges and leaf-order conventions as build_lbvh, which it must follow (triangle trees; before leaf packing).
int resplit_tree(msh_tree* tree, const double* d_v, const uint32_t* d_f, size_t T, uint32_t* d_order, int log2K);
// Oriented-box pass over the packed leaves (needs the node ranges recorded by build_lbvh).  defer: leave its
// temporaries to tree->pend_free instead of synchronising and freeing them (asynchronous batched builds).
int build_obb(msh_tree* tree, bool triangles, bool defer = false);
int tri_bounds(const double* d_v, const uint32_t* d_f, size_t T, double* d_lo, double* d_hi, hipStream_t s);
int pack_tri_leaves(const double* d_v, const uint32_t* d_f, const uint32_t* d_order, size_t T, uint32_t face_base,
                    TriRec* d_out, hipStream_t s);
int pack_point_leaves(const double* d_v, const uint32_t* d_order, size_t P, PtRec* d_out, hipStream_t s);
int point_bounds(const double* d_v, size_t P, double* d_lo, double* d_hi, hipStream_t s);

// ---- queries (nearest.hip) ----
// 30-bit Morton codes of query points in the tree's scene box + iota values.
int query_morton(const msh_tree* tree, const double* d_q, size_t S, uint32_t* keys, uint32_t* vals, hipStream_t s);
// the box query Morton codes are taken in: the scene box widened by 10 % of its extent per side
void query_box(const msh_tree* tree, float* lo, float* hi);
// Query order (sort.hip): the S rows stably sorted by the top 30 - lo_bit bits (<= 24) of their Morton codes in the
// box lo..hi; the permutation (slot -> row) ends in ws.vals.  Uses ws.keys, ws.keys_alt, ws.vals_alt, ws.hist.
int query_sort(const float* lo, const float* hi, const double* d_q, size_t S, int lo_bit, Workspace& ws, hipStream_t s);
// slot i <- rows perm[i] of a (and b when non-null); inv[perm[i]] = i
int gather_rows(const double* d_a, const double* d_b, const uint32_t* d_perm, size_t S, double* d_as, double* d_bs,
                uint32_t* d_inv, hipStream_t s);
// caller row j <- slot inv[j] (record fields + nw doubles per row from d_w)
int unpermute_results(const QRes* d_res, const double* d_w, int nw, const uint32_t* d_inv, size_t S, const SlotOut& o,
                      hipStream_t s);
// Entry cut of a single triangle tree (nearest.hip k_cut_level): the records of a G^3 grid from the cell centres' exact
// answers (closest points d_pts, their leaves d_hint); e4: 32-B records of 4-B entries (trees of <= 2^20 leaves), else 64-B records.
// kCutK start entries per cell (the hint takes the record's eighth word; round 5: 8 entries of 8 B + a separate hint;
// 4 entries: 1773-1800 M q/s against 8, 16: 1285, C3, profiles/r03_c3_entry_cut_ab.jsonl)
constexpr int kCutK = 7;
constexpr uint32_t kCutEmpty = 0x7FFFFFFFu;  // empty 64-B record entry: not a node id (ids < T - 1 <= 2^31 - 2) nor a ~leaf
constexpr size_t kEnt4MaxLeaves = (size_t)1 << 20;  // 4-B stack / cut entries: refs in [-2^20, 2^20), 21 bits
int cut_centres(int G, const double* lo, const double* w, double* d_q, hipStream_t s);
// d_half: the records of the G/2 grid over the same box (same record size), each cell then starts from its enclosing
// half-resolution cell's entries instead of the root; nullptr: from the root
int cut_level(const msh_tree* tree, int G, const double* lo, const double* w, const double* d_pts, const int* d_hint,
              uint32_t* d_rec, bool e4, hipStream_t s, const uint32_t* d_half = nullptr);
// d_inv[face] = the leaf holding it (T words)
int face_leaf_map(const msh_tree* tree, uint32_t* d_inv, hipStream_t s);
// closest point (and part) of each row q[i] on face d_face[i] (the traversal's answer construction); d_inv from
// face_leaf_map
int points_from_faces(const msh_tree* tree, const uint32_t* d_inv, const double* d_q, size_t S, const uint32_t* d_face,
                      uint32_t* d_part, double* d_pt, hipStream_t s);
// d_hint[cell] = the leaf holding face d_face[cell] (d_inv: T scratch words)
int cut_hints(const msh_tree* tree, const uint32_t* d_face, size_t n, uint32_t* d_inv, int* d_hint, hipStream_t s);
// closest point: o.face, o.part (nullable), o.pt; with o.w (3 per row) the barycentric variant (part unused)
int launch_nearest(const msh_tree* tree, const QueryOrder& ord, size_t S, const SlotOut& o, hipStream_t s);
// batched trees: n = (meshes) * S queries, slot i answered on mesh mesh0 + i / S (the batched sort is mesh-major)
int launch_nearest_batch(const msh_tree* tree, const QueryOrder& ord, size_t n, size_t S, const SlotOut& o,
                         hipStream_t s, size_t mesh0 = 0);
int launch_nearest_stats(const msh_tree* tree, const QueryOrder& ord, size_t S, unsigned long long* d_counts,
                         hipStream_t s);
// normals metric: o.face, o.pt; ord.n = query normals in slot order
int launch_nnearest(const msh_tree* tree, const QueryOrder& ord, size_t S, const SlotOut& o, hipStream_t s);
// vertex NN: o.face (index), o.dist
int launch_points_nearest(const msh_tree* tree, const QueryOrder& ord, size_t S, const SlotOut& o, hipStream_t s);

// ---- rays (rays.hip) ----
// alongnormal: ord.q / ord.n = sources / normals in slot order; o.w = distance (1 per row), o.face, o.pt
int launch_alongnormal(const msh_tree* tree, const QueryOrder& ord, size_t S, const SlotOut& o, hipStream_t s);
// visibility of vertices [v0, v0 + nv) from C cameras: vis / ndc are (C, nv)
int launch_visibility(const msh_tree* tree, const double* d_cams, size_t C, const double* d_normals,
                      const double* d_sensors, double min_dist, size_t v0, size_t nv, uint32_t* d_vis, double* d_ndc,
                      hipStream_t s);

// instrumented (untimed, outputs not written): d_counts[0] += internal nodes loaded, [1] += leaf tests
int launch_alongnormal_stats(const msh_tree* tree, const QueryOrder& ord, size_t S, unsigned long long* d_counts,
                             hipStream_t s);
int launch_visibility_stats(const msh_tree* tree, const double* d_cams, size_t C, double min_dist,
                            unsigned long long* d_counts, hipStream_t s);

// ---- triangle-triangle (tritri.hip) ----
// flags[i] = 1 iff query triangle i intersects any tree triangle (self: skip shared-vertex pairs and
// the query triangles are the tree's own leaves in face order).
int launch_tri_intersect(const msh_tree* tree, const TriRec* d_qtris, size_t Tq, int self_mode, uint32_t* d_flags,
                         hipStream_t s);

// ---- mesh geometry (geometry.hip) ----
// area-weighted vertex normals of (P,3) v over (T,3) f: sum of the faces' cross products in ascending
// face order per vertex, normalised (mesh.py:208-216)
// d_err (device u32, zeroed by the caller) is set when a face index is >= P (those faces are ignored)
int vertex_normals(const double* d_v, size_t P, const uint32_t* d_f, size_t T, double* d_vn, Workspace& ws,
                   hipStream_t s, uint32_t* d_err);

// ---- timing ----
struct TimedLaunch {
    const char* name;
    hipStream_t s;
    hipEvent_t a = nullptr, b = nullptr;
    TimedLaunch(const char* n, hipStream_t st);
    ~TimedLaunch();
};

}  // namespace msh
