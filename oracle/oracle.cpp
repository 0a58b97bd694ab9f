// ORACLE — TEST INFRASTRUCTURE ONLY.
//
// CPU restatement of the algorithms behind psbody-mesh's point-to-mesh spatial search
// (the CGAL 4.7 AABB_tree wrapped by mesh/src/spatialsearchmodule.cpp, aabb_normals.cpp,
// visibility.cpp).  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg
// may load this library, and only as the checker / CPU baseline — never as the product path.
//
// CGAL 4.7 itself is absent from /root/reference (.MISSING_LARGE_BLOBS:1) and Boost headers
// are absent from the image, so the reference's native path cannot be compiled here.  This
// file restates CGAL's published algorithm (Simple_cartesian<double> kernel, AABB_tree build /
// traversal / Projection_traits, internal/AABB_tree/nearest_point_triangle_3.h) and the
// reference's own variants.  Parity is pinned by the reference's own known-answer tests
// (tests/golden/ref_tests.json, generated from the literal values of tests/test_mesh.py:89-109,
// tests/test_aabb_n_tree.py:29-89, tests/test_visibility.py:13-53, tests/test_intersections.py:27)
// and, for ClosestPointTree, by scipy.spatial.KDTree.
//
// Compiled with -ffp-contract=off: the reference was built by g++ -O3 for baseline x86-64 (no
// FMA), so every construction here is evaluated with separately rounded * and +.
//
// Entry points (extern "C", ctypes-friendly):
//   closest point:   ora_cgal_tree_build / ora_cgal_tree_nearest (CGAL semantics, KD hint)
//                    ora_brute_nearest   (exhaustive, lexicographic min (d², face))
//                    ora_point_triangle  (one query / one face: point, part, d²)
//   normals metric:  ora_cgal_ntree_nearest (CGAL AABB_n_tree semantics), ora_brute_nnearest
//   rays:            ora_cgal_tree_alongnormal, ora_cgal_tree_visibility (CGAL tree traversal,
//                    the C5 CPU baseline), ora_brute_alongnormal, ora_brute_visibility
//   tri-tri:         ora_tri_tri_overlap, ora_brute_intersections, ora_brute_selfintersects
//   vertex NN:       ora_brute_vertex_nn
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <limits>
#include <vector>
#ifdef _OPENMP
#include <omp.h>
#endif

namespace {

struct P3 {
    double x, y, z;
};

inline P3 mk(const double* p) { return P3{p[0], p[1], p[2]}; }
// CGAL Construct_vector_3(a, b) == b - a
inline P3 vec(const P3& a, const P3& b) { return P3{b.x - a.x, b.y - a.y, b.z - a.z}; }
inline P3 sub(const P3& a, const P3& b) { return P3{a.x - b.x, a.y - b.y, a.z - b.z}; }
inline P3 add(const P3& a, const P3& b) { return P3{a.x + b.x, a.y + b.y, a.z + b.z}; }
inline P3 scale(double s, const P3& a) { return P3{s * a.x, s * a.y, s * a.z}; }
// Cartesian Compute_scalar_product_3: x*x' + y*y' + z*z' (left-assoc)
inline double dot(const P3& a, const P3& b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
// Cartesian Construct_cross_product_vector_3
inline P3 cross(const P3& v, const P3& w) {
    return P3{v.y * w.z - v.z * w.y, v.z * w.x - v.x * w.z, v.x * w.y - v.y * w.x};
}
// squared_distanceC3: square(px-qx) + square(py-qy) + square(pz-qz)
inline double sqd(const P3& p, const P3& q) {
    double dx = p.x - q.x, dy = p.y - q.y, dz = p.z - q.z;
    return dx * dx + dy * dy + dz * dz;
}
inline bool peq(const P3& a, const P3& b) { return a.x == b.x && a.y == b.y && a.z == b.z; }

// plane_from_pointsC3(p, q, r): coefficients (a, b, c, d)
inline void plane_of(const P3& p, const P3& q, const P3& r, double& a, double& b, double& c, double& d) {
    double rpx = p.x - r.x, rpy = p.y - r.y, rpz = p.z - r.z;
    double rqx = q.x - r.x, rqy = q.y - r.y, rqz = q.z - r.z;
    a = rpy * rqz - rqy * rpz;
    b = rpz * rqx - rqz * rpx;
    c = rpx * rqy - rqx * rpy;
    d = -a * r.x - b * r.y - c * r.z;
}

// projection_planeC3
inline P3 project_plane(double a, double b, double c, double d, const P3& p) {
    double num = a * p.x + b * p.y + c * p.z + d;
    double den = a * a + b * b + c * c;
    double lambda = num / den;
    return P3{p.x - lambda * a, p.y - lambda * b, p.z - lambda * c};
}

// Construct_projected_point_3(Line_3(p1, p2), q): line point p1, direction p2 - p1
inline P3 project_line(const P3& p1, const P3& p2, const P3& q) {
    double ldx = p2.x - p1.x, ldy = p2.y - p1.y, ldz = p2.z - p1.z;
    double dpx = q.x - p1.x, dpy = q.y - p1.y, dpz = q.z - p1.z;
    double lambda = (ldx * dpx + ldy * dpy + ldz * dpz) / (ldx * ldx + ldy * ldy + ldz * ldz);
    return P3{p1.x + lambda * ldx, p1.y + lambda * ldy, p1.z + lambda * ldz};
}

// iev::is_inside_triangle_3_aux (nearest_point_triangle_3.h:22-60)
inline bool edge_aux(const P3& w, const P3& p1, const P3& p2, const P3& q, P3& result, bool& outside) {
    const P3 v = cross(vec(p1, p2), vec(p1, q));
    if (dot(v, w) < 0.0) {
        if (dot(vec(p1, q), vec(p1, p2)) >= 0.0 && dot(vec(p2, q), vec(p2, p1)) >= 0.0) {
            result = project_line(p1, p2, q);
            return true;
        }
        outside = true;
    }
    return false;
}

// nearest_point_3(origin, p1, p2, p3) (nearest_point_triangle_3.h:72-101)
inline int nearest_vertex(const P3& o, const P3& p1, const P3& p2, const P3& p3) {
    const double d1 = sqd(o, p1), d2 = sqd(o, p2), d3 = sqd(o, p3);
    if (d2 >= d1 && d3 >= d1) return 0;
    if (d3 >= d2) return 1;
    return 2;
}

// Closest point of closed segment [a, b] to p (used only for degenerate triangles).
inline P3 seg_closest(const P3& a, const P3& b, const P3& p) {
    P3 ab = vec(a, b);
    double den = dot(ab, ab);
    if (!(den > 0.0)) return a;
    double t = dot(vec(a, p), ab) / den;
    if (t <= 0.0) return a;
    if (t >= 1.0) return b;
    return P3{a.x + t * ab.x, a.y + t * ab.y, a.z + t * ab.z};
}

// Closest point of triangle t0 t1 t2 to origin, CGAL construction:
// project on the supporting plane, then edge / vertex fallback of the projected point.
// part: 0 interior, 1/2/3 edge t0t1/t1t2/t2t0, 4/5/6 vertex t0/t1/t2
// (iev::nearest_primitive, nearest_point_triangle_3.h:113-154).
// Degenerate triangles (zero plane normal): reference behaviour is NaN; the
// build and this oracle both fall back to the nearest point over the three closed edges.
inline double closest_on_triangle(const P3& o, const P3& t0, const P3& t1, const P3& t2, P3& out, int& part) {
    double a, b, c, d;
    plane_of(t0, t1, t2, a, b, c, d);
    if (a * a + b * b + c * c == 0.0) {
        P3 c0 = seg_closest(t0, t1, o), c1 = seg_closest(t1, t2, o), c2 = seg_closest(t2, t0, o);
        double d0 = sqd(o, c0), d1 = sqd(o, c1), d2 = sqd(o, c2);
        out = c0; part = 1;
        double best = d0;
        if (d1 < best) { best = d1; out = c1; part = 2; }
        if (d2 < best) { best = d2; out = c2; part = 3; }
        if (peq(out, t0)) part = 4; else if (peq(out, t1)) part = 5; else if (peq(out, t2)) part = 6;
        return best;
    }
    const P3 p = project_plane(a, b, c, d, o);
    const P3 w = cross(vec(t0, t1), vec(t1, t2));
    bool outside = false;
    P3 r;
    if (edge_aux(w, t0, t1, p, r, outside)) { out = r; part = 1; }
    else if (edge_aux(w, t1, t2, p, r, outside)) { out = r; part = 2; }
    else if (edge_aux(w, t2, t0, p, r, outside)) { out = r; part = 3; }
    else if (outside) {
        int k = nearest_vertex(p, t0, t1, t2);
        out = k == 0 ? t0 : (k == 1 ? t1 : t2);
        part = 4 + k;
    } else {
        out = p; part = 0;
    }
    return sqd(o, out);
}

// CGAL internal::nearest_point_3(origin, triangle, bound): returns the triangle's closest point
// if its squared distance is <= that of bound, else bound.
inline P3 cgal_nearest_point_bounded(const P3& o, const P3& t0, const P3& t1, const P3& t2, const P3& bound) {
    const double bound_sq = sqd(o, bound);
    double a, b, c, d;
    plane_of(t0, t1, t2, a, b, c, d);
    if (a * a + b * b + c * c == 0.0) {
        P3 q; int part;
        double dd = closest_on_triangle(o, t0, t1, t2, q, part);
        return dd > bound_sq ? bound : q;
    }
    const P3 proj = project_plane(a, b, c, d, o);
    if (sqd(o, proj) > bound_sq) return bound;
    const P3 w = cross(vec(t0, t1), vec(t1, t2));
    bool outside = false;
    P3 moved;
    if (edge_aux(w, t0, t1, proj, moved, outside) || edge_aux(w, t1, t2, proj, moved, outside) ||
        edge_aux(w, t2, t0, proj, moved, outside)) {
        // on an edge
    } else if (outside) {
        int k = nearest_vertex(proj, t0, t1, t2);
        moved = k == 0 ? t0 : (k == 1 ? t1 : t2);
    } else {
        return proj;
    }
    if (sqd(o, moved) > bound_sq) return bound;
    return moved;
}

struct Mesh {
    std::vector<P3> tri;  // 3 * T vertices
    size_t T = 0;
    void load(const double* v, const uint32_t* f, size_t T_) {
        T = T_;
        tri.resize(3 * T);
        for (size_t t = 0; t < T; ++t)
            for (int k = 0; k < 3; ++k) tri[3 * t + k] = mk(v + 3 * (size_t)f[3 * t + k]);
    }
};

struct Box {
    double lo[3], hi[3];
};

// ---------------------------------------------------------------------------------------------
// CGAL AABB_tree restatement (AABB_tree::build / AABB_node::expand / AABB_traits::Sort_primitives)
// Nodes: n-1 for n primitives; each node's bbox is the exact double union of its triangles' bboxes;
// split at first + n/2 by std::nth_element on the reference point (vertex 0) along the longest axis.
struct CgalNode {
    Box box;
    int32_t left, right;  // node index, or ~primitive position when a leaf
};

struct CgalTree {
    Mesh mesh;
    std::vector<uint32_t> prim;  // primitive order (face ids)
    std::vector<CgalNode> nodes;
    // KD hint (accelerate_distance_queries): nearest reference point (vertex 0) of any primitive.
    std::vector<uint32_t> kd_idx;
    struct KdNode { int axis; double split; int32_t lo, hi; uint32_t b, e; };
    std::vector<KdNode> kd;
    double eps = 0.0;
    bool has_hint = false;

    Box prim_box(uint32_t f) const {
        const P3* t = &mesh.tri[3 * (size_t)f];
        Box b;
        b.lo[0] = std::min(std::min(t[0].x, t[1].x), t[2].x); b.hi[0] = std::max(std::max(t[0].x, t[1].x), t[2].x);
        b.lo[1] = std::min(std::min(t[0].y, t[1].y), t[2].y); b.hi[1] = std::max(std::max(t[0].y, t[1].y), t[2].y);
        b.lo[2] = std::min(std::min(t[0].z, t[1].z), t[2].z); b.hi[2] = std::max(std::max(t[0].z, t[1].z), t[2].z);
        return b;
    }

    void expand(size_t node, size_t first, size_t beyond, size_t range) {
        Box b = prim_box(prim[first]);
        for (size_t i = first + 1; i < beyond; ++i) {
            Box c = prim_box(prim[i]);
            for (int k = 0; k < 3; ++k) { b.lo[k] = std::min(b.lo[k], c.lo[k]); b.hi[k] = std::max(b.hi[k], c.hi[k]); }
        }
        nodes[node].box = b;
        // AABB_traits::longest_axis
        const double dx = b.hi[0] - b.lo[0], dy = b.hi[1] - b.lo[1], dz = b.hi[2] - b.lo[2];
        int axis = (dx >= dy) ? (dx >= dz ? 0 : 2) : (dy >= dz ? 1 : 2);
        const P3* tri = mesh.tri.data();
        auto key = [tri, axis](uint32_t f) {
            const P3& r = tri[3 * (size_t)f];
            return axis == 0 ? r.x : (axis == 1 ? r.y : r.z);
        };
        std::nth_element(prim.begin() + first, prim.begin() + first + (beyond - first) / 2, prim.begin() + beyond,
                         [&key](uint32_t a, uint32_t c) { return key(a) < key(c); });
        switch (range) {
            case 2:
                nodes[node].left = ~(int32_t)first;
                nodes[node].right = ~(int32_t)(first + 1);
                break;
            case 3:
                nodes[node].left = ~(int32_t)first;
                nodes[node].right = (int32_t)(node + 1);
                expand(node + 1, first + 1, beyond, 2);
                break;
            default: {
                const size_t nr = range / 2;
                nodes[node].left = (int32_t)(node + 1);
                nodes[node].right = (int32_t)(node + nr);
                expand(node + 1, first, first + nr, nr);
                expand(node + nr, first + nr, beyond, range - nr);
            }
        }
    }

    void build(const double* v, const uint32_t* f, size_t T, bool hint) {
        mesh.load(v, f, T);
        prim.resize(T);
        for (size_t i = 0; i < T; ++i) prim[i] = (uint32_t)i;
        nodes.clear();
        if (T > 1) {
            nodes.resize(T - 1);
            expand(0, 0, T, T);
        }
        has_hint = hint;
        if (hint) build_kd();
    }

    // --- KD hint: simple kd-tree over reference points, exact 1-NN (ties: first found) ---
    void build_kd() {
        kd_idx.resize(mesh.T);
        for (size_t i = 0; i < mesh.T; ++i) kd_idx[i] = (uint32_t)i;
        kd.clear();
        kd_build(0, (uint32_t)mesh.T);
    }
    int32_t kd_build(uint32_t b, uint32_t e) {
        int32_t id = (int32_t)kd.size();
        kd.push_back(KdNode{-1, 0.0, -1, -1, b, e});
        if (e - b <= 10) return id;
        double lo[3] = {1e300, 1e300, 1e300}, hi[3] = {-1e300, -1e300, -1e300};
        for (uint32_t i = b; i < e; ++i) {
            const P3& r = mesh.tri[3 * (size_t)kd_idx[i]];
            lo[0] = std::min(lo[0], r.x); hi[0] = std::max(hi[0], r.x);
            lo[1] = std::min(lo[1], r.y); hi[1] = std::max(hi[1], r.y);
            lo[2] = std::min(lo[2], r.z); hi[2] = std::max(hi[2], r.z);
        }
        int axis = 0;
        for (int k = 1; k < 3; ++k) if (hi[k] - lo[k] > hi[axis] - lo[axis]) axis = k;
        uint32_t m = (b + e) / 2;
        const P3* tri = mesh.tri.data();
        auto c = [tri, axis](uint32_t f) { const P3& r = tri[3 * (size_t)f]; return axis == 0 ? r.x : (axis == 1 ? r.y : r.z); };
        std::nth_element(kd_idx.begin() + b, kd_idx.begin() + m, kd_idx.begin() + e,
                         [&c](uint32_t x, uint32_t y) { return c(x) < c(y); });
        double split = c(kd_idx[m]);
        int32_t l = kd_build(b, m);
        int32_t h = kd_build(m, e);
        kd[id].axis = axis; kd[id].split = split; kd[id].lo = l; kd[id].hi = h;
        return id;
    }
    void kd_search(int32_t n, const P3& q, double& best, uint32_t& bid) const {
        const KdNode& k = kd[n];
        if (k.axis < 0) {
            for (uint32_t i = k.b; i < k.e; ++i) {
                double d = sqd(q, mesh.tri[3 * (size_t)kd_idx[i]]);
                if (d < best) { best = d; bid = kd_idx[i]; }
            }
            return;
        }
        double qc = k.axis == 0 ? q.x : (k.axis == 1 ? q.y : q.z);
        double diff = qc - k.split;
        int32_t nearc = diff < 0 ? k.lo : k.hi, farc = diff < 0 ? k.hi : k.lo;
        kd_search(nearc, q, best, bid);
        if (diff * diff <= best) kd_search(farc, q, best, bid);
    }

    // --- Projection_traits traversal (AABB_node::traversal, left child first) ---
    struct Proj {
        P3 point;
        uint32_t prim;
    };
    static bool sphere_box(const P3& c, double r2, const Box& b) {
        // Bbox_3 / Sphere_3 do_intersect: squared distance to the box <= squared radius (closed)
        double dist = 0.0, d;
        if (c.x < b.lo[0]) { d = b.lo[0] - c.x; dist += d * d; } else if (c.x > b.hi[0]) { d = c.x - b.hi[0]; dist += d * d; }
        if (c.y < b.lo[1]) { d = b.lo[1] - c.y; dist += d * d; } else if (c.y > b.hi[1]) { d = c.y - b.hi[1]; dist += d * d; }
        if (c.z < b.lo[2]) { d = b.lo[2] - c.z; dist += d * d; } else if (c.z > b.hi[2]) { d = c.z - b.hi[2]; dist += d * d; }
        return dist <= r2;
    }
    void proj_intersection(const P3& q, uint32_t f, Proj& st) const {
        const P3* t = &mesh.tri[3 * (size_t)f];
        P3 np = cgal_nearest_point_bounded(q, t[0], t[1], t[2], st.point);
        if (!peq(np, st.point)) { st.prim = f; st.point = np; }
    }
    bool proj_do_intersect(const P3& q, const CgalNode& n, const Proj& st) const {
        return sphere_box(q, sqd(q, st.point), n.box);
    }
    void traverse(const P3& q, size_t node, size_t nb, Proj& st, uint64_t* visits) const {
        const CgalNode& n = nodes[node];
        if (visits) ++*visits;
        switch (nb) {
            case 2:
                proj_intersection(q, prim[~n.left], st);
                proj_intersection(q, prim[~n.right], st);
                break;
            case 3:
                proj_intersection(q, prim[~n.left], st);
                if (proj_do_intersect(q, nodes[n.right], st)) traverse(q, n.right, 2, st, visits);
                break;
            default:
                if (proj_do_intersect(q, nodes[n.left], st)) {
                    traverse(q, n.left, nb / 2, st, visits);
                    if (proj_do_intersect(q, nodes[n.right], st)) traverse(q, n.right, nb - nb / 2, st, visits);
                } else if (proj_do_intersect(q, nodes[n.right], st)) {
                    traverse(q, n.right, nb - nb / 2, st, visits);
                }
        }
    }
    Proj nearest(const P3& q, uint64_t* visits) const {
        Proj st;
        if (has_hint) {
            double best = std::numeric_limits<double>::infinity();
            uint32_t bid = 0;
            kd_search(0, q, best, bid);
            st.point = mesh.tri[3 * (size_t)bid]; st.prim = bid;
        } else {
            st.point = mesh.tri[3 * (size_t)prim[0]]; st.prim = prim[0];
        }
        if (mesh.T == 1) proj_intersection(q, prim[0], st);
        else traverse(q, 0, mesh.T, st, visits);
        return st;
    }

    // --- AABB_n_tree (AABB_n_tree.h): metric ||q-p|| + eps (1 - n_q . n_tri) ---
    struct ProjN {
        P3 point, normal;
        uint32_t prim;
    };
    P3 unit_normal(uint32_t f) const {
        const P3* t = &mesh.tri[3 * (size_t)f];
        double a, b, c, d;
        plane_of(t[0], t[1], t[2], a, b, c, d);
        double s = std::sqrt(a * a + b * b + c * c);
        return P3{a / s, b / s, c / s};
    }
    // nearest_pointnormal_3 (AABB_n_tree.h:47-84)
    void projn_intersection(const P3& q, const P3& qn, uint32_t f, ProjN& st) const {
        const P3* t = &mesh.tri[3 * (size_t)f];
        const double dist_n_bound = eps * (1 - dot(qn, st.normal));
        const P3 tn = unit_normal(f);
        const double dist_n_tri = eps * (1 - dot(qn, tn));
        const double dist_bound = std::sqrt(sqd(q, st.point)) + dist_n_bound;
        if (dist_n_tri > dist_bound) return;
        double a, b, c, d;
        plane_of(t[0], t[1], t[2], a, b, c, d);
        const P3 proj = project_plane(a, b, c, d, q);
        const double dist_proj = std::sqrt(sqd(q, proj)) + dist_n_tri;
        P3 np;
        if (dist_proj > dist_bound) return;
        const P3 w = cross(vec(t[0], t[1]), vec(t[1], t[2]));
        bool outside = false;
        P3 moved;
        if (edge_aux(w, t[0], t[1], proj, moved, outside) || edge_aux(w, t[1], t[2], proj, moved, outside) ||
            edge_aux(w, t[2], t[0], proj, moved, outside)) {
        } else if (outside) {
            int k = nearest_vertex(proj, t[0], t[1], t[2]);
            moved = t[k];
        } else {
            np = proj;
            if (!peq(np, st.point)) { st.point = np; st.normal = tn; st.prim = f; }
            return;
        }
        const double dist_moved = std::sqrt(sqd(q, moved)) + dist_n_tri;
        if (dist_moved > dist_bound) return;
        if (!peq(moved, st.point)) { st.point = moved; st.normal = tn; st.prim = f; }
    }
    bool projn_do_intersect(const P3& q, const P3& qn, const CgalNode& n, const ProjN& st) const {
        double safe = std::sqrt(sqd(q, st.point)) + eps * (1 - dot(qn, st.normal));
        return sphere_box(q, safe * safe, n.box);
    }
    void ntraverse(const P3& q, const P3& qn, size_t node, size_t nb, ProjN& st) const {
        const CgalNode& n = nodes[node];
        switch (nb) {
            case 2:
                projn_intersection(q, qn, prim[~n.left], st);
                projn_intersection(q, qn, prim[~n.right], st);
                break;
            case 3:
                projn_intersection(q, qn, prim[~n.left], st);
                if (projn_do_intersect(q, qn, nodes[n.right], st)) ntraverse(q, qn, n.right, 2, st);
                break;
            default:
                if (projn_do_intersect(q, qn, nodes[n.left], st)) {
                    ntraverse(q, qn, n.left, nb / 2, st);
                    if (projn_do_intersect(q, qn, nodes[n.right], st)) ntraverse(q, qn, n.right, nb - nb / 2, st);
                } else if (projn_do_intersect(q, qn, nodes[n.right], st)) {
                    ntraverse(q, qn, n.right, nb - nb / 2, st);
                }
        }
    }
    // --- Ray traversal (AABB_tree::all_intersections / do_intersect with a Ray_3 query) ---
    // Ray_3 / Bbox_3 do_intersect: closed slab test, t in [0, +inf) (CGAL's
    // do_intersect_bbox_segment_aux with the far end unbounded), in double.
    static bool ray_box(const P3& p, const P3& d, const Box& b) {
        double tmin = 0.0, tmax = std::numeric_limits<double>::infinity();
        const double pc[3] = {p.x, p.y, p.z}, dc[3] = {d.x, d.y, d.z};
        for (int k = 0; k < 3; ++k) {
            if (dc[k] == 0.0) {
                if (pc[k] < b.lo[k] || pc[k] > b.hi[k]) return false;
                continue;
            }
            double t0 = (b.lo[k] - pc[k]) / dc[k], t1 = (b.hi[k] - pc[k]) / dc[k];
            if (t0 > t1) std::swap(t0, t1);
            tmin = std::max(tmin, t0);
            tmax = std::min(tmax, t1);
            if (tmin > tmax) return false;
        }
        return true;
    }
    struct RayHit { double t; uint32_t prim; int kind; };
    // Listing_primitive_traits: every primitive hit, appended in left-first traversal order.
    template <class F>
    bool ray_traverse(const P3& p, const P3& d, size_t node, size_t nb, F& on_prim) const {
        const CgalNode& n = nodes[node];
        switch (nb) {
            case 2:
                if (on_prim(prim[~n.left])) return true;
                return on_prim(prim[~n.right]);
            case 3:
                if (on_prim(prim[~n.left])) return true;
                if (ray_box(p, d, nodes[n.right].box)) return ray_traverse(p, d, n.right, 2, on_prim);
                return false;
            default:
                if (ray_box(p, d, nodes[n.left].box) && ray_traverse(p, d, n.left, nb / 2, on_prim)) return true;
                if (ray_box(p, d, nodes[n.right].box)) return ray_traverse(p, d, n.right, nb - nb / 2, on_prim);
                return false;
        }
    }
    // on_prim returns true to stop (do_intersect's first-hit exit).
    template <class F>
    void ray_query(const P3& p, const P3& d, F& on_prim) const {
        if (mesh.T == 1) { on_prim(prim[0]); return; }
        // AABB_tree::traversal tests the root box before descending
        if (!nodes.empty() && ray_box(p, d, nodes[0].box)) ray_traverse(p, d, 0, mesh.T, on_prim);
    }

    ProjN nnearest(const P3& q, const P3& qn) const {
        // hint = any_reference_point_and_id(): first primitive in tree order (AABB_n_tree.h:279)
        ProjN st;
        st.prim = prim[0];
        st.point = mesh.tri[3 * (size_t)prim[0]];
        st.normal = unit_normal(prim[0]);
        if (mesh.T == 1) projn_intersection(q, qn, prim[0], st);
        else ntraverse(q, qn, 0, mesh.T, st);
        return st;
    }
};

// ---------------------------------------------------------------------------------------------
// Rays.  A CGAL Ray_3(p, v) is stored as two points (p, p + v); predicates use (p+v) - p as the
// direction.  Closed triangle, closed ray (t >= 0).  Hit iff the ray line passes the three edges
// with consistent orientation (shared edges are watertight: the edge determinant flips sign exactly)
// and the plane crossing parameter is >= 0.  Coplanar rays: entry point of the ray into the
// closed triangle (clipping in the plane).
inline double det3(const P3& a, const P3& b, const P3& c) { return dot(cross(a, b), c); }

// returns true and t (hit = p + t*d) if the closed ray hits the closed triangle
inline bool coplanar_ray_tri(const P3& p, const P3& d, const P3& a, const P3& b, const P3& c, double& tout) {
    P3 n = cross(vec(a, b), vec(a, c));
    if (n.x == 0.0 && n.y == 0.0 && n.z == 0.0) return false;
    double tlo = 0.0, thi = std::numeric_limits<double>::infinity();
    const P3 v[3] = {a, b, c};
    for (int e = 0; e < 3; ++e) {
        const P3& s = v[e];
        const P3& t = v[(e + 1) % 3];
        // inside half-plane: dot(n, cross(t - s, x - s)) >= 0 ; x = p + t d -> f0 + t f1
        P3 et = vec(s, t);
        double f0 = dot(n, cross(et, vec(s, p)));
        double f1 = dot(n, cross(et, d));
        if (f1 == 0.0) {
            if (f0 < 0.0) return false;
        } else {
            double tt = -f0 / f1;
            if (f1 > 0.0) tlo = std::max(tlo, tt);
            else thi = std::min(thi, tt);
        }
    }
    if (tlo > thi) return false;
    tout = tlo;
    return true;
}

// 0: miss; 1: proper hit at parameter t; 2: coplanar hit (CGAL returns a Segment_3) entering at t
inline int ray_tri_kind(const P3& p, const P3& d, const P3& a, const P3& b, const P3& c, double& tout) {
    const P3 u = vec(p, a), v = vec(p, b), w = vec(p, c);
    const double s0 = det3(u, v, d), s1 = det3(v, w, d), s2 = det3(w, u, d);
    const bool pos = s0 >= 0.0 && s1 >= 0.0 && s2 >= 0.0;
    const bool neg = s0 <= 0.0 && s1 <= 0.0 && s2 <= 0.0;
    if (!pos && !neg) return 0;
    const P3 n = cross(vec(a, b), vec(a, c));
    const double num = dot(n, u);
    const double den = dot(n, d);
    if (den == 0.0 || (s0 == 0.0 && s1 == 0.0 && s2 == 0.0)) {
        if (num != 0.0) return 0;  // parallel, off-plane
        return coplanar_ray_tri(p, d, a, b, c, tout) ? 2 : 0;
    }
    const double t = num / den;
    if (t < 0.0) return 0;
    tout = t;
    return 1;
}
inline bool ray_tri(const P3& p, const P3& d, const P3& a, const P3& b, const P3& c, double& tout) {
    return ray_tri_kind(p, d, a, b, c, tout) != 0;
}

// The point CGAL 4.7 returns for a proper Triangle_3 / Ray_3 hit: t3r3_intersection_aux intersects
// r.supporting_line() = Line_3(p, p + v) (point p, direction d = (p + v) - p) with
// t.supporting_plane() = Plane_3(a, b, c) (plane_from_pointsC3), Intersections_3 Plane_3/Line_3:
//   num = A px + B py + C pz + D,  den = A dx + B dy + C dz,
//   point = Point_3(den px - num dx, den py - num dy, den pz - num dz, den)  (homogeneous; /den).
// Call sites: spatialsearchmodule.cpp:277-278 (all_intersections), visibility.cpp:93 (do_intersect).
// false when den == 0 in this arithmetic (CGAL then returns the Line_3 itself, i.e. no Point_3).
inline bool cgal_plane_line(const P3& p, const P3& d, const P3& a, const P3& b, const P3& c, P3& out) {
    double A, B, C, D;
    plane_of(a, b, c, A, B, C, D);
    const double num = A * p.x + B * p.y + C * p.z + D;
    const double den = A * d.x + B * d.y + C * d.z;
    if (den == 0.0) return false;
    out = P3{(den * p.x - num * d.x) / den, (den * p.y - num * d.y) / den, (den * p.z - num * d.z) / den};
    return true;
}

inline P3 ray_dir(const P3& p, const P3& v) {
    const P3 q = add(p, v);
    return vec(p, q);
}

// ---------------------------------------------------------------------------------------------
// Triangle-triangle overlap (closed), orientation-predicate test in the style of Guigue &
// Devillers (2003) — the algorithm CGAL's Triangle_3/Triangle_3 do_intersect implements.
inline bool seg_seg_2d(double ax, double ay, double bx, double by, double cx, double cy, double dx, double dy) {
    auto o2 = [](double px, double py, double qx, double qy, double rx, double ry) {
        return (qx - px) * (ry - py) - (qy - py) * (rx - px);
    };
    double o1 = o2(ax, ay, bx, by, cx, cy), o2v = o2(ax, ay, bx, by, dx, dy);
    double o3 = o2(cx, cy, dx, dy, ax, ay), o4 = o2(cx, cy, dx, dy, bx, by);
    if (((o1 > 0 && o2v < 0) || (o1 < 0 && o2v > 0)) && ((o3 > 0 && o4 < 0) || (o3 < 0 && o4 > 0))) return true;
    auto onseg = [](double px, double py, double qx, double qy, double rx, double ry) {
        return std::min(px, qx) <= rx && rx <= std::max(px, qx) && std::min(py, qy) <= ry && ry <= std::max(py, qy);
    };
    if (o1 == 0 && onseg(ax, ay, bx, by, cx, cy)) return true;
    if (o2v == 0 && onseg(ax, ay, bx, by, dx, dy)) return true;
    if (o3 == 0 && onseg(cx, cy, dx, dy, ax, ay)) return true;
    if (o4 == 0 && onseg(cx, cy, dx, dy, bx, by)) return true;
    return false;
}
inline bool pt_in_tri_2d(double px, double py, const double* t) {
    auto o2 = [](double ax, double ay, double bx, double by, double cx, double cy) {
        return (bx - ax) * (cy - ay) - (by - ay) * (cx - ax);
    };
    double d0 = o2(t[0], t[1], t[2], t[3], px, py);
    double d1 = o2(t[2], t[3], t[4], t[5], px, py);
    double d2 = o2(t[4], t[5], t[0], t[1], px, py);
    return (d0 >= 0 && d1 >= 0 && d2 >= 0) || (d0 <= 0 && d1 <= 0 && d2 <= 0);
}
bool coplanar_tri_tri(const P3& p1, const P3& q1, const P3& r1, const P3& p2, const P3& q2, const P3& r2, const P3& n) {
    // drop the dominant axis of the normal
    double ax = std::fabs(n.x), ay = std::fabs(n.y), az = std::fabs(n.z);
    int drop = (ax > az && ax >= ay) ? 0 : ((ay > az && ay > ax) ? 1 : 2);
    auto pr = [drop](const P3& p, double* o) {
        if (drop == 0) { o[0] = p.y; o[1] = p.z; }
        else if (drop == 1) { o[0] = p.x; o[1] = p.z; }
        else { o[0] = p.x; o[1] = p.y; }
    };
    double t1[6], t2[6];
    pr(p1, t1); pr(q1, t1 + 2); pr(r1, t1 + 4);
    pr(p2, t2); pr(q2, t2 + 2); pr(r2, t2 + 4);
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j)
            if (seg_seg_2d(t1[2 * i], t1[2 * i + 1], t1[(2 * i + 2) % 6], t1[(2 * i + 3) % 6], t2[2 * j], t2[2 * j + 1],
                           t2[(2 * j + 2) % 6], t2[(2 * j + 3) % 6]))
                return true;
    if (pt_in_tri_2d(t1[0], t1[1], t2)) return true;
    if (pt_in_tri_2d(t2[0], t2[1], t1)) return true;
    return false;
}
inline bool check_min_max(const P3& p1, const P3& q1, const P3& r1, const P3& p2, const P3& q2, const P3& r2) {
    P3 n = cross(sub(p2, q1), sub(p1, q1));
    if (dot(sub(q2, q1), n) > 0.0) return false;
    n = cross(sub(p2, p1), sub(r1, p1));
    if (dot(sub(r2, p1), n) > 0.0) return false;
    return true;
}
inline bool tri_tri_3d(const P3& p1, const P3& q1, const P3& r1, const P3& p2, const P3& q2, const P3& r2, double dp2,
                       double dq2, double dr2, const P3& n1) {
    if (dp2 > 0.0) {
        if (dq2 > 0.0) return check_min_max(p1, r1, q1, r2, p2, q2);
        if (dr2 > 0.0) return check_min_max(p1, r1, q1, q2, r2, p2);
        return check_min_max(p1, q1, r1, p2, q2, r2);
    }
    if (dp2 < 0.0) {
        if (dq2 < 0.0) return check_min_max(p1, q1, r1, r2, p2, q2);
        if (dr2 < 0.0) return check_min_max(p1, q1, r1, q2, r2, p2);
        return check_min_max(p1, r1, q1, p2, q2, r2);
    }
    if (dq2 < 0.0) {
        if (dr2 >= 0.0) return check_min_max(p1, r1, q1, q2, r2, p2);
        return check_min_max(p1, q1, r1, p2, q2, r2);
    }
    if (dq2 > 0.0) {
        if (dr2 > 0.0) return check_min_max(p1, r1, q1, p2, q2, r2);
        return check_min_max(p1, q1, r1, q2, r2, p2);
    }
    if (dr2 > 0.0) return check_min_max(p1, q1, r1, r2, p2, q2);
    if (dr2 < 0.0) return check_min_max(p1, r1, q1, r2, p2, q2);
    return coplanar_tri_tri(p1, q1, r1, p2, q2, r2, n1);
}
bool tri_tri_overlap(const P3& p1, const P3& q1, const P3& r1, const P3& p2, const P3& q2, const P3& r2) {
    const P3 n2 = cross(sub(p2, r2), sub(q2, r2));
    const double dp1 = dot(sub(p1, r2), n2), dq1 = dot(sub(q1, r2), n2), dr1 = dot(sub(r1, r2), n2);
    if (dp1 * dq1 > 0.0 && dp1 * dr1 > 0.0) return false;
    const P3 n1 = cross(sub(q1, p1), sub(r1, p1));
    const double dp2 = dot(sub(p2, r1), n1), dq2 = dot(sub(q2, r1), n1), dr2 = dot(sub(r2, r1), n1);
    if (dp2 * dq2 > 0.0 && dp2 * dr2 > 0.0) return false;
    if (dp1 > 0.0) {
        if (dq1 > 0.0) return tri_tri_3d(r1, p1, q1, p2, r2, q2, dp2, dr2, dq2, n1);
        if (dr1 > 0.0) return tri_tri_3d(q1, r1, p1, p2, r2, q2, dp2, dr2, dq2, n1);
        return tri_tri_3d(p1, q1, r1, p2, q2, r2, dp2, dq2, dr2, n1);
    }
    if (dp1 < 0.0) {
        if (dq1 < 0.0) return tri_tri_3d(r1, p1, q1, p2, q2, r2, dp2, dq2, dr2, n1);
        if (dr1 < 0.0) return tri_tri_3d(q1, r1, p1, p2, q2, r2, dp2, dq2, dr2, n1);
        return tri_tri_3d(p1, q1, r1, p2, r2, q2, dp2, dr2, dq2, n1);
    }
    if (dq1 < 0.0) {
        if (dr1 >= 0.0) return tri_tri_3d(q1, r1, p1, p2, r2, q2, dp2, dr2, dq2, n1);
        return tri_tri_3d(p1, q1, r1, p2, q2, r2, dp2, dq2, dr2, n1);
    }
    if (dq1 > 0.0) {
        if (dr1 > 0.0) return tri_tri_3d(p1, q1, r1, p2, r2, q2, dp2, dr2, dq2, n1);
        return tri_tri_3d(q1, r1, p1, p2, q2, r2, dp2, dq2, dr2, n1);
    }
    if (dr1 > 0.0) return tri_tri_3d(r1, p1, q1, p2, q2, r2, dp2, dq2, dr2, n1);
    if (dr1 < 0.0) return tri_tri_3d(r1, p1, q1, p2, r2, q2, dp2, dr2, dq2, n1);
    return coplanar_tri_tri(p1, q1, r1, p2, q2, r2, n1);
}

void set_threads(int threads) {
#ifdef _OPENMP
    if (threads > 0) omp_set_num_threads(threads);
#else
    (void)threads;
#endif
}

}  // namespace

extern "C" {

int ora_version(void) { return 1; }

// ---- single query / single face: CGAL construction, part code, squared distance ----
double ora_point_triangle(const double* q, const double* a, const double* b, const double* c, double* pt, uint32_t* part) {
    P3 o; int pp;
    double d2 = closest_on_triangle(mk(q), mk(a), mk(b), mk(c), o, pp);
    pt[0] = o.x; pt[1] = o.y; pt[2] = o.z;
    *part = (uint32_t)pp;
    return d2;
}

// ---- CGAL-faithful tree (spatialsearchmodule.cpp:108-123 build; :129-140 per query) ----
void* ora_cgal_tree_build(const double* v, size_t P, const uint32_t* f, size_t T, int with_hint, double eps) {
    (void)P;
    CgalTree* t = new CgalTree();
    t->eps = eps;
    t->build(v, f, T, with_hint != 0);
    return t;
}
void ora_cgal_tree_free(void* h) { delete static_cast<CgalTree*>(h); }

// aabbtree_nearest: face, part (nearest_primitive on the winning face), point.  visits (nullable):
// total node visits, for the instrumented baseline.
void ora_cgal_tree_nearest(void* h, const double* q, size_t S, uint32_t* face, uint32_t* part, double* pt, int threads,
                           uint64_t* visits) {
    const CgalTree* t = static_cast<CgalTree*>(h);
    set_threads(threads);
    uint64_t total = 0;
#pragma omp parallel for schedule(dynamic, 256) reduction(+ : total)
    for (long s = 0; s < (long)S; ++s) {
        const P3 qq = mk(q + 3 * s);
        uint64_t vv = 0;
        CgalTree::Proj r = t->nearest(qq, visits ? &vv : nullptr);
        total += vv;
        face[s] = r.prim;
        pt[3 * s] = r.point.x; pt[3 * s + 1] = r.point.y; pt[3 * s + 2] = r.point.z;
        if (part) {
            P3 o; int pp;
            const P3* tri = &t->mesh.tri[3 * (size_t)r.prim];
            closest_on_triangle(qq, tri[0], tri[1], tri[2], o, pp);
            part[s] = (uint32_t)pp;
        }
    }
    if (visits) *visits = total;
}

// aabbtree_n_nearest (aabb_normals.cpp:112-190)
void ora_cgal_ntree_nearest(void* h, const double* q, const double* n, size_t S, uint32_t* face, double* pt, int threads) {
    const CgalTree* t = static_cast<CgalTree*>(h);
    set_threads(threads);
#pragma omp parallel for schedule(dynamic, 256)
    for (long s = 0; s < (long)S; ++s) {
        CgalTree::ProjN r = t->nnearest(mk(q + 3 * s), mk(n + 3 * s));
        face[s] = r.prim;
        pt[3 * s] = r.point.x; pt[3 * s + 1] = r.point.y; pt[3 * s + 2] = r.point.z;
    }
}

// ---- nearest_alongnormal through the CGAL tree (spatialsearchmodule.cpp:272-321): all_intersections
// of Ray_3(p, n) then Ray_3(p, -n) in traversal order, first minimum distance (std::min_element, :314).
// Same hit constructions as ora_brute_alongnormal; differs from it only in which face wins an exact tie.
void ora_cgal_tree_alongnormal(void* h, const double* p, const double* n, size_t S, double* dist, uint32_t* face,
                               double* pt, int threads, uint64_t* tests) {
    const CgalTree* t = static_cast<CgalTree*>(h);
    set_threads(threads);
    uint64_t total = 0;
#pragma omp parallel for schedule(dynamic, 256) reduction(+ : total)
    for (long s = 0; s < (long)S; ++s) {
        const P3 pp = mk(p + 3 * s), nn = mk(n + 3 * s);
        const P3 nneg{-nn.x, -nn.y, -nn.z};
        double best = 1e100;
        uint32_t bf = 0xFFFFFFFFu;
        P3 bp{NAN, NAN, NAN};
        bool any = false;
        uint64_t ntest = 0;
        for (int k = 0; k < 2; ++k) {
            const P3 d = ray_dir(pp, k ? nneg : nn);
            auto on_prim = [&](uint32_t f) {
                ++ntest;
                const P3 &ta = t->mesh.tri[3 * (size_t)f], &tb = t->mesh.tri[3 * (size_t)f + 1],
                         &tc = t->mesh.tri[3 * (size_t)f + 2];
                double tt;
                const int kind = ray_tri_kind(pp, d, ta, tb, tc, tt);
                if (!kind) return false;
                P3 hit;
                if (kind == 2 || !cgal_plane_line(pp, d, ta, tb, tc, hit)) hit = add(pp, scale(tt, d));
                const double dd = std::sqrt(sqd(hit, pp));
                if (!any || dd < best) { best = dd; bf = f; bp = hit; any = true; }
                return false;
            };
            t->ray_query(pp, d, on_prim);
        }
        total += ntest;
        dist[s] = best;
        face[s] = bf;
        pt[3 * s] = bp.x; pt[3 * s + 1] = bp.y; pt[3 * s + 2] = bp.z;
    }
    if (tests) *tests = total;
}

// ---- visibility_compute through the CGAL tree (visibility.cpp:75-115): tree.do_intersect(Ray) stops at
// the first hit.  The tree holds main + extra triangles (py_visibility.cpp:140-163); v are the main
// vertices.  Cameras in the outer loop as the reference's VisibilityTask; vertices in parallel.
void ora_cgal_tree_visibility(void* h, const double* v, size_t P, const double* cams, size_t C, const double* normals,
                              const double* sensors, double min_dist, uint32_t* vis, double* ndc, int threads) {
    const CgalTree* t = static_cast<CgalTree*>(h);
    set_threads(threads);
    // (camera, vertex) pairs in camera-major order, as VisibilityTask visits them; parallel over both.
#pragma omp parallel for schedule(dynamic, 64)
    for (long o = 0; o < (long)(C * P); ++o) {
        const size_t ic = (size_t)o / P, iv = (size_t)o % P;
        const P3 cam = mk(cams + 3 * ic);
        P3 xoff{0, 0, 0}, yoff{0, 0, 0}, zoff{0, 0, 0};
        double planeoff = 0.0;
        if (sensors) {
            const double* s = sensors + 9 * ic;
            xoff = P3{s[0], s[1], s[2]};
            yoff = P3{s[3], s[4], s[5]};
            zoff = P3{-s[6], -s[7], -s[8]};
            planeoff = dot(zoff, add(cam, zoff));
        }
        const P3 vv = mk(v + 3 * iv);
        P3 dir = vec(vv, cam);
        const double len = std::sqrt(dot(dir, dir));
        dir = P3{dir.x / len, dir.y / len, dir.z / len};
        const P3 src = add(vv, scale(min_dist, dir));
        const P3 d = ray_dir(src, dir);
        bool hit = false;
        auto on_prim = [&](uint32_t f) {
            double tt;
            hit = ray_tri(src, d, t->mesh.tri[3 * (size_t)f], t->mesh.tri[3 * (size_t)f + 1],
                          t->mesh.tri[3 * (size_t)f + 2], tt);
            return hit;
        };
        t->ray_query(src, d, on_prim);
        const uint32_t reach = hit ? 0u : 1u;
        ndc[o] = normals ? dot(mk(normals + 3 * iv), dir) : 0.0;
        if (sensors) {
            if (reach) {
                const double tp = -(dot(zoff, vv) - planeoff) / dot(zoff, dir);
                const P3 pi = sub(add(vv, scale(tp, dir)), add(cam, zoff));
                vis[o] = (std::fabs(dot(pi, xoff)) < dot(xoff, xoff) && std::fabs(dot(pi, yoff)) < dot(yoff, yoff)) ? 1u : 0u;
            } else {
                vis[o] = 0u;
            }
        } else {
            vis[o] = reach;
        }
    }
}

// ---- exhaustive closest point: lexicographic min (d², face) ----
void ora_brute_nearest(const double* v, size_t P, const uint32_t* f, size_t T, const double* q, size_t S, uint32_t* face,
                       uint32_t* part, double* pt, double* d2out, int threads) {
    (void)P;
    Mesh m;
    m.load(v, f, T);
    set_threads(threads);
#pragma omp parallel for schedule(dynamic, 64)
    for (long s = 0; s < (long)S; ++s) {
        const P3 qq = mk(q + 3 * s);
        double best = std::numeric_limits<double>::infinity();
        uint32_t bf = 0;
        P3 bp{0, 0, 0};
        int bpart = 0;
        for (size_t t = 0; t < T; ++t) {
            P3 o; int pp;
            double d2 = closest_on_triangle(qq, m.tri[3 * t], m.tri[3 * t + 1], m.tri[3 * t + 2], o, pp);
            if (d2 < best) { best = d2; bf = (uint32_t)t; bp = o; bpart = pp; }
        }
        face[s] = bf;
        if (part) part[s] = (uint32_t)bpart;
        pt[3 * s] = bp.x; pt[3 * s + 1] = bp.y; pt[3 * s + 2] = bp.z;
        if (d2out) d2out[s] = best;
    }
}

// ---- exhaustive normals metric: lexicographic min (sqrt(d²) + eps (1 - n.n_tri), face) ----
void ora_brute_nnearest(const double* v, size_t P, const uint32_t* f, size_t T, double eps, const double* q,
                        const double* n, size_t S, uint32_t* face, double* pt, double* metric, int threads) {
    (void)P;
    Mesh m;
    m.load(v, f, T);
    set_threads(threads);
#pragma omp parallel for schedule(dynamic, 64)
    for (long s = 0; s < (long)S; ++s) {
        const P3 qq = mk(q + 3 * s), qn = mk(n + 3 * s);
        double best = std::numeric_limits<double>::infinity();
        uint32_t bf = 0;
        P3 bp{0, 0, 0};
        for (size_t t = 0; t < T; ++t) {
            const P3* tr = &m.tri[3 * t];
            double a, b, c, d;
            plane_of(tr[0], tr[1], tr[2], a, b, c, d);
            double sn = std::sqrt(a * a + b * b + c * c);
            P3 tn{a / sn, b / sn, c / sn};
            P3 o; int pp;
            double d2 = closest_on_triangle(qq, tr[0], tr[1], tr[2], o, pp);
            double met = std::sqrt(d2) + eps * (1 - dot(qn, tn));
            if (met < best) { best = met; bf = (uint32_t)t; bp = o; }
        }
        face[s] = bf;
        pt[3 * s] = bp.x; pt[3 * s + 1] = bp.y; pt[3 * s + 2] = bp.z;
        if (metric) metric[s] = best;
    }
}

// ---- nearest_alongnormal (spatialsearchmodule.cpp:222-323): rays (p, n) and (p, -n), min distance.
// Exhaustive; ties -> lexicographic min (distance, face).  No hit: dist = 1e100, face = 0xFFFFFFFF,
// point = NaN (the reference leaves them uninitialised).
void ora_brute_alongnormal(const double* v, size_t P, const uint32_t* f, size_t T, const double* p, const double* n,
                           size_t S, double* dist, uint32_t* face, double* pt, int threads) {
    (void)P;
    Mesh m;
    m.load(v, f, T);
    set_threads(threads);
#pragma omp parallel for schedule(dynamic, 64)
    for (long s = 0; s < (long)S; ++s) {
        const P3 pp = mk(p + 3 * s), nn = mk(n + 3 * s);
        const P3 nneg{-nn.x, -nn.y, -nn.z};
        const P3 dirs[2] = {ray_dir(pp, nn), ray_dir(pp, nneg)};
        double best = 1e100;
        uint32_t bf = 0xFFFFFFFFu;
        P3 bp{NAN, NAN, NAN};
        for (size_t t = 0; t < T; ++t) {
            for (int k = 0; k < 2; ++k) {
                double tt;
                const P3 &ta = m.tri[3 * t], &tb = m.tri[3 * t + 1], &tc = m.tri[3 * t + 2];
                const int kind = ray_tri_kind(pp, dirs[k], ta, tb, tc, tt);
                if (!kind) continue;
                // proper hit: CGAL's plane/line construction; coplanar (Segment_3): entry point of the
                // clipped ray (the reference's xy formula at :295-307 divides by the 2-D cross product of
                // two parallel vectors and is not restated)
                P3 hit;
                if (kind == 2 || !cgal_plane_line(pp, dirs[k], ta, tb, tc, hit)) hit = add(pp, scale(tt, dirs[k]));
                double d = std::sqrt(sqd(hit, pp));
                if (d < best || (d == best && (uint32_t)t < bf)) { best = d; bf = (uint32_t)t; bp = hit; }
            }
        }
        dist[s] = best;
        face[s] = bf;
        pt[3 * s] = bp.x; pt[3 * s + 1] = bp.y; pt[3 * s + 2] = bp.z;
    }
}

// ---- visibility_compute (visibility.cpp:75-115) over main + extra triangles, exhaustive any-hit.
// v: main-mesh vertices (P,3); tris: all triangles as (Tall, 9) coordinates.
void ora_brute_visibility(const double* v, size_t P, const double* tris, size_t Tall, const double* cams, size_t C,
                          const double* normals, const double* sensors, double min_dist, uint32_t* vis, double* ndc,
                          int threads) {
    set_threads(threads);
    for (size_t ic = 0; ic < C; ++ic) {
        const P3 cam = mk(cams + 3 * ic);
        P3 xoff{0, 0, 0}, yoff{0, 0, 0}, zoff{0, 0, 0};
        double planeoff = 0.0;
        if (sensors) {
            const double* s = sensors + 9 * ic;
            xoff = P3{s[0], s[1], s[2]};
            yoff = P3{s[3], s[4], s[5]};
            zoff = P3{-s[6], -s[7], -s[8]};
            planeoff = dot(zoff, add(cam, zoff));
        }
#pragma omp parallel for schedule(dynamic, 64)
        for (long iv = 0; iv < (long)P; ++iv) {
            const P3 vv = mk(v + 3 * iv);
            P3 dir = vec(vv, cam);
            const double len = std::sqrt(dot(dir, dir));
            dir = P3{dir.x / len, dir.y / len, dir.z / len};
            const P3 src = add(vv, scale(min_dist, dir));
            const P3 d = ray_dir(src, dir);
            bool hit = false;
            for (size_t t = 0; t < Tall && !hit; ++t) {
                const double* tr = tris + 9 * t;
                double tt;
                hit = ray_tri(src, d, mk(tr), mk(tr + 3), mk(tr + 6), tt);
            }
            uint32_t reach = hit ? 0u : 1u;
            const size_t o = iv + ic * P;
            ndc[o] = normals ? dot(mk(normals + 3 * iv), dir) : 0.0;
            if (sensors) {
                if (reach) {
                    const double t = -(dot(zoff, vv) - planeoff) / dot(zoff, dir);
                    const P3 pi = sub(add(vv, scale(t, dir)), add(cam, zoff));
                    vis[o] = (std::fabs(dot(pi, xoff)) < dot(xoff, xoff) && std::fabs(dot(pi, yoff)) < dot(yoff, yoff)) ? 1u : 0u;
                } else {
                    vis[o] = 0u;
                }
            } else {
                vis[o] = reach;
            }
        }
    }
}

// ---- triangle-triangle ----
int ora_tri_tri_overlap(const double* t1, const double* t2) {
    return tri_tri_overlap(mk(t1), mk(t1 + 3), mk(t1 + 6), mk(t2), mk(t2 + 3), mk(t2 + 6)) ? 1 : 0;
}

// intersections_indices (spatialsearchmodule.cpp:326-417): ascending query-face indices whose
// triangle intersects any mesh triangle.  Returns K; out has capacity Tq.
size_t ora_brute_intersections(const double* v, size_t P, const uint32_t* f, size_t T, const double* qv, size_t Pq,
                               const uint32_t* qf, size_t Tq, uint32_t* out, int threads) {
    (void)P; (void)Pq;
    Mesh m, qm;
    m.load(v, f, T);
    qm.load(qv, qf, Tq);
    std::vector<uint8_t> flag(Tq, 0);
    set_threads(threads);
#pragma omp parallel for schedule(dynamic, 16)
    for (long i = 0; i < (long)Tq; ++i) {
        const P3* a = &qm.tri[3 * i];
        for (size_t t = 0; t < T; ++t) {
            const P3* b = &m.tri[3 * t];
            if (tri_tri_overlap(a[0], a[1], a[2], b[0], b[1], b[2])) { flag[i] = 1; break; }
        }
    }
    size_t K = 0;
    for (size_t i = 0; i < Tq; ++i) if (flag[i]) out[K++] = (uint32_t)i;
    return K;
}

// aabbtree_n_selfintersects (aabb_normals.cpp:192-207; AABB_n_tree.h:107-116): number of triangles
// that intersect another triangle sharing no exactly-equal vertex coordinate.
long ora_brute_selfintersects(const double* v, size_t P, const uint32_t* f, size_t T, int threads) {
    (void)P;
    Mesh m;
    m.load(v, f, T);
    long count = 0;
    set_threads(threads);
#pragma omp parallel for schedule(dynamic, 16) reduction(+ : count)
    for (long i = 0; i < (long)T; ++i) {
        const P3* a = &m.tri[3 * i];
        for (size_t t = 0; t < T; ++t) {
            const P3* b = &m.tri[3 * t];
            bool share = false;
            for (int x = 0; x < 3; ++x)
                for (int y = 0; y < 3; ++y) share |= peq(a[x], b[y]);
            if (share) continue;
            if (tri_tri_overlap(a[0], a[1], a[2], b[0], b[1], b[2])) { ++count; break; }
        }
    }
    return count;
}

// ---- vertex nearest neighbour (ClosestPointTree, search.py:52-65): lexicographic min (d², index) ----
void ora_brute_vertex_nn(const double* v, size_t P, const double* q, size_t S, uint32_t* idx, double* dist, int threads) {
    set_threads(threads);
#pragma omp parallel for schedule(dynamic, 64)
    for (long s = 0; s < (long)S; ++s) {
        const P3 qq = mk(q + 3 * s);
        double best = std::numeric_limits<double>::infinity();
        uint32_t bi = 0;
        for (size_t i = 0; i < P; ++i) {
            double d2 = sqd(qq, mk(v + 3 * i));
            if (d2 < best) { best = d2; bi = (uint32_t)i; }
        }
        idx[s] = bi;
        dist[s] = std::sqrt(best);
    }
}

}  // extern "C"
