/*
 * meshsearch.h — C ABI of the MI355X-native point-to-mesh spatial search engine (libmeshsearch.so).
 *
 * Drop-in replacement for the three CPython extensions of psbody-mesh 0.4 that wrap CGAL 4.7's
 * AABB_tree (KanaLab/mesh: mesh/src/spatialsearchmodule.cpp, mesh/src/aabb_normals.cpp,
 * mesh/src/py_visibility.cpp) and for the scipy KDTree behind search.ClosestPointTree.  Every entry
 * point takes plain pointers and sizes; no Python, numpy or torch type crosses this boundary.
 * The Python shims in mesh_amd/ (spatialsearch.py, aabb_normals.py, visibility.py, search.py) bind
 * these functions with ctypes; INTEGRATION.md shows the binding a psbody-mesh maintainer would add.
 *
 * Conventions
 *  - Arrays are C-contiguous row-major: points/normals (N,3) double, faces (T,3) uint32.
 *  - Every function returns MSH_OK (0) or an error code; msh_last_error() gives the message of the
 *    last failure on the calling thread.  MSH_EINVAL maps to ValueError (bad shape / index),
 *    MSH_EDEVICE / MSH_ENOMEM to RuntimeError (HIP failure), as the reference raises
 *    (spatialsearchmodule.cpp:82-97 ValueError; cgal_error_emulation.hpp:19-33 RuntimeError).
 *  - Host-buffer entry points (no _device suffix) copy inputs to HBM, run the HIP kernels and copy
 *    results back; they are synchronous.  *_device entry points take HBM pointers and a hipStream_t
 *    (passed as void*, NULL = the handle's own stream, a blocking stream that orders with the legacy default
 *    stream — so NULL also serves a caller whose work is queued on the default stream) and are asynchronous
 *    on that stream.
 *  - A handle owns device copies of the mesh and its BVH (the reference's TreeAndTri owns host
 *    copies, nearest_triangle.hpp:28-32); input arrays are not retained.  Calls on one handle must be
 *    serialised by the caller (host threads); on the device, launches that share a handle's scratch
 *    are ordered with an event, whatever streams they are issued on.  Different handles are
 *    independent.
 *  - Query counts per call are limited to 2^32 - 1 (device slot indices are 32-bit).
 *  - There is no CPU fallback: without a usable gfx950 device every compute entry point fails with
 *    MSH_EDEVICE.
 */
#ifndef MESHSEARCH_H_
#define MESHSEARCH_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MSH_OK 0
#define MSH_EINVAL 1
#define MSH_EDEVICE 2
#define MSH_ENOMEM 3

#define MSH_NO_FACE 0xFFFFFFFFu

typedef struct msh_tree msh_tree;

typedef struct msh_tree_info {
    int device;          /* HIP device ordinal holding the tree */
    int kind;            /* 0 triangles (spatialsearch), 1 normals metric (aabb_normals), 2 points */
    uint64_t n_points;   /* P: vertices of the main mesh */
    uint64_t n_faces;    /* T: leaf primitives (main + extra mesh faces, or points) */
    uint64_t n_main_faces;
    uint64_t n_nodes;    /* internal LBVH nodes (T-1) */
    uint64_t bytes;      /* device bytes owned by the handle (mesh + BVH) */
    double eps;
    float scene_lo[3], scene_hi[3];
    double build_ms;     /* GPU time of the build (Morton + radix sort + emission + re-split + oriented boxes) */
    uint64_t n_meshes;   /* meshes in a batched tree (msh_batch_build), 1 otherwise */
    uint32_t node_bytes; /* bytes of one internal node as stored in HBM (one traversal step reads it) */
    uint32_t leaf_bytes; /* bytes of one leaf record (triangle: 9 x f64 + face id; point: 3 x f64 + id) */
    int32_t max_depth;   /* upper bound of the deepest leaf below the root (sizes traversal stacks) */
} msh_tree_info;

/* Layout of a packed tree blob (msh_tree_blob_*), readable on the host without a device. */
typedef struct msh_blob_info {
    int32_t kind, max_depth;
    uint64_t n_points, n_faces, n_main_faces;
    uint64_t off_vertices, off_nodes, off_leaves, total;
    uint32_t node_bytes, leaf_bytes;
    double origin[3];
} msh_blob_info;

/* ---- library / device ---- */
const char* msh_last_error(void);
int msh_version(void);
/* Identity of the built kernels: the first 16 hex digits of the SHA-256 of mesh_amd/csrc's sources (and any
 * extra compile flags).  Profiles are keyed by it, so a measurement is only ever paired with the code it
 * measured (bench.py roofline.traffic). */
const char* msh_build_id(void);
int msh_device_count(int* n);
/* Device used by subsequent builds on the calling thread (default: current HIP device).  It also drops the
 * thread's device list (msh_set_devices / msh_set_device_list): later trees are built on this device alone. */
int msh_set_device(int device);
/* In-process multi-device handles (SURVEY §8(b) msh_set_devices; the reference's drop-in call
 * Mesh.closest_faces_and_points -> AabbTree.nearest, mesh.py:454-455 / search.py:26-30, has no device argument).
 * Trees built afterwards on the calling thread are built on the first device and replicated to the others
 * (blob pack + peer copy + unpack); the host-buffer entry points (msh_tree_nearest, _nearest_bary,
 * _nearest_alongnormal, msh_ntree_nearest, msh_points_nearest: contiguous row ranges; msh_visibility: camera
 * ranges) then split their rows over the devices, one host thread and one chunk pipeline per device, so each
 * device's host link carries its share.  Calls below 32 MB of rows stay on the first device.  The answers equal
 * the one-device answers bit for bit (disjoint row ranges of the same arrays).  *_device entry points, batched
 * trees and the intersection tests stay on the handle's own device.  Untested across devices: the GPU box this
 * library is tested on has one device, so the peer copy and the per-device pipelines have run only as replicas on
 * one device, and the devices' pageable <-> pinned staging copies share one host copy pool (one job at a time).
 *   msh_set_devices(G): devices d, d + 1, ..., d + G - 1 from the current device d (G = 1: one device again);
 *   msh_set_device_list(devices, G): an explicit list (an entry may repeat: several replicas on one device);
 *   msh_tree_devices: the devices of a handle (G = 1 + replicas; devices may be NULL);
 *   msh_device_plan: the row split of S rows over G devices, begins[0..G] (host only, no device needed). */
int msh_set_devices(int G);
int msh_set_device_list(const int* devices, int G);
int msh_tree_devices(const msh_tree* tree, int* devices, int cap, int* G);
int msh_device_plan(uint64_t S, int G, uint64_t* begins);

/* ---- spatialsearch (spatialsearchmodule.cpp) ---- */
/* aabbtree_compute(v, f) -> capsule: spatialsearchmodule.cpp:74-127 (TreeAndTri build :108-123).
 * GPU LBVH build: Morton codes of triangle centroids, LDS radix sort, Karras emission, subtrees of <= 2^16
 * leaves re-split top down along the surface, and 64-B nodes holding both children's oriented boxes (exact fp64
 * extents rounded outward, quantised outward); no refit pass. */
int msh_tree_build(const double* v, size_t P, const uint32_t* f, size_t T, msh_tree** out);
/* visibility_compute(v=, f=, extra_v=, extra_f=) builds over main + extra triangles:
 * py_visibility.cpp:114-163.  extra may be NULL/0. */
int msh_tree_build_ex(const double* v, size_t P, const uint32_t* f, size_t T, const double* ev, size_t EP,
                      const uint32_t* ef, size_t ET, msh_tree** out);
/* capsule destructor: spatialsearchmodule.cpp:68-72 */
void msh_tree_free(msh_tree* tree);
int msh_tree_get_info(const msh_tree* tree, msh_tree_info* info);

/* aabbtree_nearest(tree, q) -> (face (1,S) u32, part (1,S) u32, point (S,3) f64):
 * spatialsearchmodule.cpp:165-220, per query nearest_one :129-140.  part may be NULL.
 * Closest face = lexicographic minimum of (squared distance, face index); point = CGAL's
 * construction for that face (project on plane, edge, vertex); part = iev::nearest_primitive code. */
int msh_tree_nearest(msh_tree* tree, const double* q, size_t S, uint32_t* face, uint32_t* part, double* pt);
int msh_tree_nearest_device(msh_tree* tree, const double* d_q, size_t S, uint32_t* d_face, uint32_t* d_part,
                            double* d_pt, void* stream);
/* Instrumented traversal (not timed, same two-pass traversal as msh_tree_nearest_device): total internal
 * nodes popped and leaf triangles tested over the S queries, for the algorithmic-bytes figure of the
 * roofline. */
int msh_tree_nearest_stats(msh_tree* tree, const double* d_q, size_t S, uint64_t* nodes, uint64_t* leaves);
/* nearest + barycentric weights of the closest point in its face (Heidrich's projection, the reference's
 * Mesh.barycentric_coordinates_for_points, mesh.py:218-222 / barycentric_coordinates_of_projection.py:9-49,
 * as called by landmarks.py:61-62): face (S,) u32, point (S,3) f64, w (S,3) f64 for vertices f[face]. */
int msh_tree_nearest_bary(msh_tree* tree, const double* q, size_t S, uint32_t* face, double* pt, double* w);
int msh_tree_nearest_bary_device(msh_tree* tree, const double* d_q, size_t S, uint32_t* d_face, double* d_pt,
                                 double* d_w, void* stream);

/* The closest point (and part code) of each row q[i] on a GIVEN face face[i] -- the construction msh_tree_nearest
 * stores for the face it finds (CGAL's closest point on the triangle, spatialsearchmodule.cpp:129-140 /
 * nearest_point_triangle_3.h:22-154), so for rows answered with face f it reproduces the answer's point and part bit
 * for bit.  face MSH_NO_FACE (or >= T): point NaN, part 0.  The narrow multi-GPU result exchange
 * (mesh_amd/distributed.py NarrowRing) all-gathers faces only (4 B per row instead of 32) and rebuilds the other
 * ranks' points with it.  Device pointers; asynchronous on `stream`; part may be NULL. */
int msh_tree_points_from_faces_device(msh_tree* tree, const double* d_q, size_t S, const uint32_t* d_face,
                                      uint32_t* d_part, double* d_pt, void* stream);

/* The order in which the closest-point path visits the S query rows (d_perm[slot] = row): stable by the
 * Hilbert index of each row's cell in a 256^3 grid over the tree's scene box widened by 10 % per side (the cell is
 * the top 24 bits of the row's 30-bit Morton code, mapped to the Hilbert curve of the same cells; then 3 LDS radix
 * passes of 8 bits).  No reference counterpart (test and diagnostic entry point).  Asynchronous on `stream`. */
int msh_tree_query_order(msh_tree* tree, const double* d_q, size_t S, uint32_t* d_perm, void* stream);

/* Entry cut of a triangle tree (no reference counterpart: derived acceleration data).  A grid
 * of G^3 cells over the scene box widened by 1/4, one record per cell -- its hint leaf and 7 start entries: 32 B for
 * trees of up to 2^20 faces, 64 B beyond (which also hold the radius each list covers) -- from which closest-point
 * queries start their walks instead of the root, and so do nearest_alongnormal rays (their walk first covers that
 * radius around p, and starts again from the root only when no hit lies that near); it changes where a walk starts,
 * never an answer.  It is built lazily by a closest-point or alongnormal call of the handle (msh_tree_nearest*,
 * msh_tree_nearest_bary*, msh_tree_nearest_alongnormal*, and their _stats).  The automatic grid comes in two sizes: the
 * coarse one (about 8 cells per face, at most 2^23 cells: C3 G = 200, 256 MB, ~11 ms) once the handle's calls have
 * brought at least one row per 16 of its cells (C3: 500k rows; a few small calls on a large mesh walk from the root
 * instead of paying the build), the fine one (twice the coarse resolution: about 64 cells per face, C3 G = 400,
 * 2.05 GB) once they have brought 16 rows per fine cell (C3: ~1G rows), or at the next call after
 * msh_tree_set_entry_cut(t, -1) (a caller that keeps the tree for many batches).  The fine grid is built from the
 * coarse one (its cells' start lists and centre walks begin there); asked for with no grid installed, the coarse grid
 * is built first and freed after (C3: ~57 ms for both).  build_ms counts both.  A grid asked for with msh_tree_set_entry_cut is built by the
 * next call whatever its size.  Trees used only for visibility or the normals metric never hold it; trees of
 * < 4096 faces never get one.  The call that builds it is synchronous, also for the *_device entry points (the cut's
 * build waits for its own cell-centre queries): a caller that captures *_device calls in a graph or needs them
 * asynchronous calls msh_tree_set_entry_cut and makes one small query first (or sets G = 0).
 *   G < 0: the fine automatic grid at the next call (the default policy above until then);
 *   G = 0: no cut (frees one already built); queries start at the root;
 *   G > 0: G^3 cells.
 * Calling it (any G != 0, also the current one) makes the next closest-point call build the grid if it is not
 * built yet; changing G frees the current cut first.  A cut that cannot be built (device memory) is not an error:
 * its queries start at the root (a failed upgrade keeps the coarse grid); an automatic grid is tried again after
 * another threshold of rows (at most twice, state 0 meanwhile), then the handle records the failure (state 3), as
 * it does at once for a grid asked for with msh_tree_set_entry_cut. */
int msh_tree_set_entry_cut(msh_tree* tree, int G);
/* state: 0 not built yet, 1 built, 2 off (G = 0, or a tree it does not apply to), 3 build failed (a handle with
 * replicas reports a replica's failed or pending state over its own);
 * G: cells per axis of the built cut (0 if none); bytes: device bytes it holds; build_ms: GPU time of its
 * build (cell-centre queries + cut + hints).  Any output pointer may be NULL. */
int msh_tree_entry_cut_info(const msh_tree* tree, int* state, int* G, uint64_t* bytes, double* build_ms);

/* aabbtree_nearest_alongnormal(tree, p, n) -> (dist (S,) f64, face (S,) u32, point (S,3) f64):
 * spatialsearchmodule.cpp:222-323.  Nearest hit of the rays (p, n) and (p, -n); hit point = CGAL's
 * Plane_3 / Line_3 construction.  No hit: dist = 1e100 (as the reference), face = MSH_NO_FACE,
 * point = NaN (reference: uninitialised). */
int msh_tree_nearest_alongnormal(msh_tree* tree, const double* p, const double* n, size_t S, double* dist,
                                 uint32_t* face, double* pt);
int msh_tree_nearest_alongnormal_device(msh_tree* tree, const double* d_p, const double* d_n, size_t S,
                                        double* d_dist, uint32_t* d_face, double* d_pt, void* stream);
/* Instrumented ray traversals (not timed; same traversal as the entry points above): total internal nodes
 * loaded and leaf triangles tested, for the algorithmic-bytes figure of the ray roofline. */
int msh_tree_nearest_alongnormal_stats(msh_tree* tree, const double* d_p, const double* d_n, size_t S, uint64_t* nodes,
                                       uint64_t* leaves);
int msh_visibility_stats(msh_tree* tree, const double* d_cams, size_t C, double min_dist, uint64_t* nodes,
                         uint64_t* leaves);

/* aabbtree_intersections_indices(tree, qv, qf) -> ascending query-face indices (K,) u32 whose
 * triangle intersects any mesh triangle: spatialsearchmodule.cpp:326-417 (unregistered there,
 * SURVEY App. B).  out must hold Tq entries; *K receives the count. */
int msh_tree_intersections(msh_tree* tree, const double* qv, size_t Pq, const uint32_t* qf, size_t Tq, uint32_t* out,
                           size_t* K);

/* ---- aabb_normals (aabb_normals.cpp, AABB_n_tree.h) ---- */
/* aabbtree_n_compute(v, f, eps): aabb_normals.cpp:63-110 */
int msh_ntree_build(const double* v, size_t P, const uint32_t* f, size_t T, double eps, msh_tree** out);
/* aabbtree_n_nearest(tree, v, n) -> (face (1,S) u32, point (S,3) f64): aabb_normals.cpp:112-190.
 * Metric ||q - p|| + eps (1 - n_q . n_tri) (AABB_n_tree.h:40-84); lexicographic min (metric, face). */
int msh_ntree_nearest(msh_tree* tree, const double* q, const double* n, size_t S, uint32_t* face, double* pt);
/* aabbtree_n_selfintersects(tree) -> int: aabb_normals.cpp:192-207; pairs sharing an exactly equal
 * vertex coordinate are skipped (AABB_n_tree.h:107-116). */
int msh_ntree_selfintersects(msh_tree* tree, int64_t* count);

/* ---- visibility (py_visibility.cpp, visibility.cpp) ---- */
/* visibility_compute(cams, tree|v,f, n, sensors, extra_v, extra_f, min_dist) -> (vis (C,P) u32,
 * n_dot_cam (C,P) f64): py_visibility.cpp:81-219, VisibilityTask visibility.cpp:75-115.
 * Visibility is computed for the tree's main-mesh vertices.  normals (P,3) and sensors (C,9) may be
 * NULL; without normals ndc is zero-filled (reference: uninitialised).  The tree is borrowed, never
 * freed (fixes the double free at py_visibility.cpp:212). */
int msh_visibility(msh_tree* tree, const double* cams, size_t C, const double* normals, const double* sensors,
                   double min_dist, uint32_t* vis, double* ndc);
/* Device-resident shard of visibility_compute: vertices [v_begin, v_begin + v_count) of the main mesh
 * (the multi-GPU split of the (C x P) ray grid by vertex range, visibility.cpp:136-173).  d_normals is
 * indexed by global vertex (P,3); d_vis / d_ndc are (C, v_count). */
int msh_visibility_device(msh_tree* tree, const double* d_cams, size_t C, const double* d_normals,
                          const double* d_sensors, double min_dist, size_t v_begin, size_t v_count, uint32_t* d_vis,
                          double* d_ndc, void* stream);

/* ---- mesh geometry feeding the path ---- */
/* Mesh.estimate_vertex_normals (mesh.py:208-216): per vertex, the sum in ascending face order of the
 * faces' cross products (v1 - v0) x (v2 - v0) (tri_normals.py:23-24), divided by its norm (0 -> 1). */
int msh_vertex_normals(const double* v, size_t P, const uint32_t* f, size_t T, double* vn);
/* device pointers; returns when the result is in d_vn (stream may be NULL).  A face index >= P is
 * detected on the device: MSH_EINVAL, d_vn unspecified, no out-of-bounds access. */
int msh_vertex_normals_device(const double* d_v, size_t P, const uint32_t* d_f, size_t T, double* d_vn, void* stream);

/* ---- batched trees: scan-to-mesh registration over many meshes (BASELINE configs[3], C4) ----
 * The reference answers this with one AabbTree per mesh (search.py:21-30, one aabbtree_compute +
 * aabbtree_nearest per mesh).  Here B meshes sharing one topology are built in ONE batched LBVH build
 * (per-mesh Morton order, Karras emission and refit in single launches over all B*T faces) and queried
 * in one launch.  v: (B,P,3) f64, f: (T,3) u32 shared by all meshes, T >= 2.  Face indices returned
 * are mesh-local (as a per-mesh AabbTree would return). */
int msh_batch_build(const double* v, size_t B, size_t P, const uint32_t* f, size_t T, msh_tree** out);
/* q: (B,S,3) f64, S queries per mesh -> face (B,S) u32, part (B,S) u32 (may be NULL), point (B,S,3) f64;
 * per mesh identical to msh_tree_nearest on that mesh alone. */
int msh_batch_nearest(msh_tree* tree, const double* q, size_t S, uint32_t* face, uint32_t* part, double* pt);
int msh_batch_nearest_device(msh_tree* tree, const double* d_q, size_t S, uint32_t* d_face, uint32_t* d_part,
                             double* d_pt, void* stream);
/* registration-ready variant: face (B,S), point (B,S,3), barycentric weights (B,S,3) (see
 * msh_tree_nearest_bary) */
int msh_batch_nearest_bary(msh_tree* tree, const double* q, size_t S, uint32_t* face, double* pt, double* w);
int msh_batch_nearest_bary_device(msh_tree* tree, const double* d_q, size_t S, uint32_t* d_face, double* d_pt,
                                  double* d_w, void* stream);

/* ---- ClosestPointTree (search.py:52-65, scipy.spatial.KDTree) ---- */
int msh_points_build(const double* v, size_t P, msh_tree** out);
/* nearest vertex: lexicographic min (squared distance, vertex index); dist = sqrt(d2) */
int msh_points_nearest(msh_tree* tree, const double* q, size_t S, uint32_t* idx, double* dist);

/* ---- multi-GPU replication (RCCL broadcast of a built BVH over xGMI) ---- */
/* Size of the flat device blob holding the mesh + BVH of a handle. */
int msh_tree_blob_size(const msh_tree* tree, size_t* bytes);
/* Pack the handle's device buffers into d_dst (HBM, on the handle's device, blob_size bytes). */
int msh_tree_blob_pack(const msh_tree* tree, void* d_dst, void* stream);
/* Create a handle on `device` from a packed blob already resident in that device's HBM
 * (e.g. after an RCCL broadcast).  The blob is copied; the caller keeps ownership of d_src. */
int msh_tree_blob_unpack(const void* d_src, size_t bytes, int device, void* stream, msh_tree** out);
/* Host-side blob header (no device): write the header of a blob for the given sizes into dst (cap
 * bytes), or parse + validate a header copied to host memory (magic, layout, version, length). */
int msh_blob_header_write(int kind, uint64_t P, uint64_t T, uint64_t T_main, void* dst, size_t cap,
                          msh_blob_info* info);
int msh_blob_header_parse(const void* src, size_t bytes, msh_blob_info* info);

/* ---- mesh files feeding the path (host parsing) ----
 * OBJ: replaces psbody.mesh.serialization.loadobj (mesh/src/py_loadobj.cpp:62-243).  sizes[9] = v rows,
 * vt rows, vt columns, vn rows, f rows, ft rows, fn rows, groups, landmarks.  Arrays are row-major
 * (rows x 3, vt rows x vt columns); groups and landmarks are enumerated in name order (std::map, as the
 * reference).  Errors: "Could not load file". */
typedef struct msh_obj msh_obj;
int msh_obj_load(const char* path, msh_obj** out);
int msh_obj_sizes(const msh_obj* obj, uint64_t* sizes);
int msh_obj_arrays(const msh_obj* obj, double* v, double* vt, double* vn, uint32_t* f, uint32_t* ft, uint32_t* fn);
const char* msh_obj_mtl_path(const msh_obj* obj);
int msh_obj_group(const msh_obj* obj, size_t k, const char** name, uint64_t* n_faces, const uint32_t** faces);
int msh_obj_landmark(const msh_obj* obj, size_t k, const char** name, uint32_t* vertex);
void msh_obj_free(msh_obj* obj);
/* PLY: replaces psbody.mesh.serialization.plyutils.read (mesh/src/plyutils.c:64-139 over rply.c).
 * sizes[4] = vertices, faces, has colour, has normals; v / colour / normals (P,3), tri (F,3) as double
 * (items 0..2 of each face list).  Errors: "Failed to open PLY file.", "plyread_mex: Bad raw header.",
 * "Read failed. <path>". */
typedef struct msh_ply msh_ply;
int msh_ply_load(const char* path, msh_ply** out);
int msh_ply_sizes(const msh_ply* ply, uint64_t* sizes);
int msh_ply_arrays(const msh_ply* ply, double* v, double* tri, double* color, double* normals);
void msh_ply_free(msh_ply* ply);

/* ---- kernel timing (HIP events on the launch stream; used by bench.py's roofline) ---- */
int msh_timing_enable(int on);
/* Total milliseconds and launch count of kernel `name` ("nearest", "sort", "morton") since reset. */
int msh_timing_get(const char* name, double* ms, int64_t* count);
int msh_timing_reset(void);

/* ---- page-locked result pool (host-buffer entry points) ----
 * Replaces nothing in the reference: its methods return fresh numpy arrays (PyArray_SimpleNew,
 * spatialsearchmodule.cpp:196-206), which the shims keep doing for small calls.  For large calls the
 * shims carve the result arrays out of one block of this pool instead, so the host-buffer entry points
 * copy results from HBM straight into them (no pinned staging copy, and no first-touch page faults of
 * fresh pages: on C3, 3.2 GB of results per call).  A block returns to the pool when the last array
 * over it dies.
 *  - msh_host_alloc: a block of >= bytes (2 MB granules), reusing a free block of at most 5/4 the
 *    size; blocks are page-locked with hipHostMalloc.  MSH_ENOMEM when the pool would outgrow its
 *    cap (MESH_AMD_PINNED_POOL_MB, default 16384; 0 disables the pool) even after releasing its free
 *    blocks: the caller then allocates ordinary pageable arrays.
 *  - msh_host_free: returns a block (any pointer msh_host_alloc gave) to the pool; NULL is ignored.
 *  - msh_host_pool_trim: releases every free block, and the idle staging slabs the host-array entry points
 *    share between handles; msh_host_pool_bytes: bytes held (live + free).
 * Host-buffer entry points recognise output arrays that lie inside one live block. */
int msh_host_alloc(size_t bytes, void** out);
void msh_host_free(void* p);
int msh_host_pool_trim(void);
size_t msh_host_pool_bytes(void);

/* ---- device memory kept between handles (no reference counterpart) ----
 * Three process-wide caches keep device memory after the handles that used it are freed, so a caller that builds
 * a tree per call (Mesh.closest_faces_and_points, mesh.py:454-455) does not reallocate it every call:
 *  - every device block the library frees (tree buffers, build temporaries, scratch) is cached for the next
 *    request of a similar size on its device, up to MESH_AMD_DEVICE_CACHE_MB (default 16384; 0 turns it off);
 *  - the query workspace of a freed triangle tree (sort keys, permutations, spill stacks, deferred lists:
 *    ~80 B per query of its largest call, ~8 GB at 100M queries), one idle workspace per device, handed to the
 *    next triangle tree built on that device;
 *  - up to two idle sets of host-call staging slabs per device (three device slabs of chunk x row bytes each,
 *    plus two page-locked host slabs).
 * msh_device_pool_trim frees all three (idle entries only: memory held by live handles stays with them);
 * msh_device_pool_bytes reports the device bytes they hold (any pointer may be NULL).  A process that
 * shares the GPU with other allocators (torch) calls the trim after freeing its handles.  A device allocation of
 * the library that fails for memory first releases the idle workspace, the idle staging slabs' device slabs and
 * the cached blocks of its device, then tries once more. */
int msh_device_pool_trim(void);
int msh_device_pool_bytes(uint64_t* workspace, uint64_t* staging, uint64_t* cached);

#ifdef __cplusplus
}
#endif
#endif /* MESHSEARCH_H_ */
