// Host-side performance model of the traversal (development tool, not product code): builds the same
// Karras LBVH as mesh_amd/csrc/build.hip (30-bit Morton codes of box centres in the scene box, stable
// sort, Karras emission, exact subtree boxes) or alternative trees, and replays the near-first
// closest-point traversal to count node visits / leaf tests per query.  Used to choose tree layouts
// without spending GPU time.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <limits>
#include <numeric>
#include <vector>

namespace {

struct Node {
    double lo[2][3], hi[2][3];
    int c[2];
};

struct Tree {
    std::vector<Node> nodes;
    std::vector<int> order;  // leaf position -> face
    int root_leaf = -1;
};

uint32_t ex10(uint32_t v) {
    v = (v * 0x00010001u) & 0xFF0000FFu;
    v = (v * 0x00000101u) & 0x0F00F00Fu;
    v = (v * 0x00000011u) & 0xC30C30C3u;
    v = (v * 0x00000005u) & 0x49249249u;
    return v;
}

int delta(const std::vector<uint32_t>& k, int n, int i, int j) {
    if (j < 0 || j >= n) return -1;
    if (k[i] != k[j]) return __builtin_clz(k[i] ^ k[j]);
    return 32 + __builtin_clz((uint32_t)i ^ (uint32_t)j);
}

void prim_bounds(const double* v, const uint32_t* f, int T, std::vector<double>& lo, std::vector<double>& hi) {
    lo.resize(3 * T);
    hi.resize(3 * T);
    for (int t = 0; t < T; ++t)
        for (int k = 0; k < 3; ++k) {
            double a = v[3 * f[3 * t] + k], b = v[3 * f[3 * t + 1] + k], c = v[3 * f[3 * t + 2] + k];
            lo[3 * t + k] = std::min(std::min(a, b), c);
            hi[3 * t + k] = std::max(std::max(a, b), c);
        }
}

void fill_boxes(Tree& tr, int x, const std::vector<double>& plo, const std::vector<double>& phi, double* olo, double* ohi) {
    for (int s = 0; s < 2; ++s) {
        int c = tr.nodes[x].c[s];
        double clo[3], chi[3];
        if (c >= 0) fill_boxes(tr, c, plo, phi, clo, chi);
        else {
            int f = tr.order[~c];
            for (int k = 0; k < 3; ++k) { clo[k] = plo[3 * f + k]; chi[k] = phi[3 * f + k]; }
        }
        for (int k = 0; k < 3; ++k) { tr.nodes[x].lo[s][k] = clo[k]; tr.nodes[x].hi[s][k] = chi[k]; }
    }
    for (int k = 0; k < 3; ++k) {
        olo[k] = std::min(tr.nodes[x].lo[0][k], tr.nodes[x].lo[1][k]);
        ohi[k] = std::max(tr.nodes[x].hi[0][k], tr.nodes[x].hi[1][k]);
    }
}

Tree build_lbvh(const double* v, const uint32_t* f, int T) {
    std::vector<double> lo, hi;
    prim_bounds(v, f, T, lo, hi);
    double box[6] = {1e300, 1e300, 1e300, -1e300, -1e300, -1e300};
    for (int t = 0; t < T; ++t)
        for (int k = 0; k < 3; ++k) { box[k] = std::min(box[k], lo[3 * t + k]); box[3 + k] = std::max(box[3 + k], hi[3 * t + k]); }
    std::vector<uint32_t> key(T);
    for (int t = 0; t < T; ++t) {
        uint32_t c[3];
        for (int k = 0; k < 3; ++k) {
            double e = box[3 + k] - box[k];
            double m = 0.5 * (lo[3 * t + k] + hi[3 * t + k]);
            double nrm = e > 0 ? (m - box[k]) / e : 0.5;
            nrm = std::min(std::max(nrm * 1024.0, 0.0), 1023.0);
            c[k] = (uint32_t)nrm;
        }
        key[t] = (ex10(c[0]) << 2) | (ex10(c[1]) << 1) | ex10(c[2]);
    }
    Tree tr;
    tr.order.resize(T);
    std::iota(tr.order.begin(), tr.order.end(), 0);
    std::stable_sort(tr.order.begin(), tr.order.end(), [&](int a, int b) { return key[a] < key[b]; });
    std::vector<uint32_t> sk(T);
    for (int i = 0; i < T; ++i) sk[i] = key[tr.order[i]];
    if (T == 1) { tr.root_leaf = 0; return tr; }
    tr.nodes.resize(T - 1);
    for (int i = 0; i < T - 1; ++i) {
        int d = (delta(sk, T, i, i + 1) - delta(sk, T, i, i - 1)) >= 0 ? 1 : -1;
        int dmin = delta(sk, T, i, i - d);
        int lmax = 2;
        while (delta(sk, T, i, i + lmax * d) > dmin) lmax <<= 1;
        int l = 0;
        for (int t = lmax >> 1; t >= 1; t >>= 1)
            if (delta(sk, T, i, i + (l + t) * d) > dmin) l += t;
        int j = i + l * d;
        int dn = delta(sk, T, i, j);
        int s = 0, t = l;
        do {
            t = (t + 1) >> 1;
            if (delta(sk, T, i, i + (s + t) * d) > dn) s += t;
        } while (t > 1);
        int g = i + s * d + (d < 0 ? -1 : 0);
        tr.nodes[i].c[0] = (std::min(i, j) == g) ? ~g : g;
        tr.nodes[i].c[1] = (std::max(i, j) == g + 1) ? ~(g + 1) : g + 1;
    }
    double a[3], b[3];
    fill_boxes(tr, 0, lo, hi, a, b);
    return tr;
}

// median split on the longest axis of the centroid box (CGAL-like), leaves are single triangles
int build_median_rec(Tree& tr, std::vector<int>& idx, int b, int e, const std::vector<double>& lo,
                     const std::vector<double>& hi) {
    if (e - b == 1) return ~b;
    int node = (int)tr.nodes.size();
    tr.nodes.push_back(Node{});
    double cl[3] = {1e300, 1e300, 1e300}, ch[3] = {-1e300, -1e300, -1e300};
    for (int i = b; i < e; ++i)
        for (int k = 0; k < 3; ++k) {
            double c = 0.5 * (lo[3 * idx[i] + k] + hi[3 * idx[i] + k]);
            cl[k] = std::min(cl[k], c);
            ch[k] = std::max(ch[k], c);
        }
    int ax = 0;
    for (int k = 1; k < 3; ++k) if (ch[k] - cl[k] > ch[ax] - cl[ax]) ax = k;
    int m = (b + e) / 2;
    std::nth_element(idx.begin() + b, idx.begin() + m, idx.begin() + e, [&](int x, int y) {
        return lo[3 * x + ax] + hi[3 * x + ax] < lo[3 * y + ax] + hi[3 * y + ax];
    });
    int l = build_median_rec(tr, idx, b, m, lo, hi);
    int r = build_median_rec(tr, idx, m, e, lo, hi);
    tr.nodes[node].c[0] = l;
    tr.nodes[node].c[1] = r;
    return node;
}

Tree build_median(const double* v, const uint32_t* f, int T) {
    std::vector<double> lo, hi;
    prim_bounds(v, f, T, lo, hi);
    Tree tr;
    std::vector<int> idx(T);
    std::iota(idx.begin(), idx.end(), 0);
    if (T == 1) { tr.order = idx; tr.root_leaf = 0; return tr; }
    build_median_rec(tr, idx, 0, T, lo, hi);
    tr.order = idx;
    double a[3], b[3];
    fill_boxes(tr, 0, lo, hi, a, b);
    return tr;
}

double box_d2(const double* q, const double* lo, const double* hi) {
    double s = 0;
    for (int k = 0; k < 3; ++k) {
        double g = std::max(std::max(lo[k] - q[k], q[k] - hi[k]), 0.0);
        s += g * g;
    }
    return s;
}

double seg_d2(const double* p, const double* a, const double* b) {
    double ab[3], ap[3];
    for (int k = 0; k < 3; ++k) { ab[k] = b[k] - a[k]; ap[k] = p[k] - a[k]; }
    double den = ab[0] * ab[0] + ab[1] * ab[1] + ab[2] * ab[2];
    double t = den > 0 ? (ap[0] * ab[0] + ap[1] * ab[1] + ap[2] * ab[2]) / den : 0;
    t = std::min(std::max(t, 0.0), 1.0);
    double d = 0;
    for (int k = 0; k < 3; ++k) { double x = a[k] + t * ab[k] - p[k]; d += x * x; }
    return d;
}

double tri_d2(const double* p, const double* a, const double* b, const double* c) {
    double ab[3], ac[3], n[3];
    for (int k = 0; k < 3; ++k) { ab[k] = b[k] - a[k]; ac[k] = c[k] - a[k]; }
    n[0] = ab[1] * ac[2] - ab[2] * ac[1]; n[1] = ab[2] * ac[0] - ab[0] * ac[2]; n[2] = ab[0] * ac[1] - ab[1] * ac[0];
    double nn = n[0] * n[0] + n[1] * n[1] + n[2] * n[2];
    double best = std::min(seg_d2(p, a, b), std::min(seg_d2(p, b, c), seg_d2(p, c, a)));
    if (nn > 0) {
        double ap[3] = {p[0] - a[0], p[1] - a[1], p[2] - a[2]};
        double s = (ap[0] * n[0] + ap[1] * n[1] + ap[2] * n[2]) / nn;
        double pr[3] = {p[0] - s * n[0] - a[0], p[1] - s * n[1] - a[1], p[2] - s * n[2] - a[2]};
        double d00 = ab[0] * ab[0] + ab[1] * ab[1] + ab[2] * ab[2], d01 = ab[0] * ac[0] + ab[1] * ac[1] + ab[2] * ac[2];
        double d11 = ac[0] * ac[0] + ac[1] * ac[1] + ac[2] * ac[2];
        double d20 = pr[0] * ab[0] + pr[1] * ab[1] + pr[2] * ab[2], d21 = pr[0] * ac[0] + pr[1] * ac[1] + pr[2] * ac[2];
        double den = d00 * d11 - d01 * d01;
        double vv = (d11 * d20 - d01 * d21) / den, w = (d00 * d21 - d01 * d20) / den;
        if (vv >= 0 && w >= 0 && vv + w <= 1) best = std::min(best, s * s * nn);
    }
    return best;
}

}  // namespace

extern "C" {

// kind 0 = LBVH (as built on the GPU), 1 = median split.  Outputs per-query node visits and leaf tests.
void model_counts(const double* v, const uint32_t* f, int T, const double* q, long S, int kind, uint32_t* nodes_out,
                  uint32_t* leaves_out, int* depth_out) {
    Tree tr = kind == 0 ? build_lbvh(v, f, T) : build_median(v, f, T);
    // depth
    int maxd = 0;
    {
        std::vector<std::pair<int, int>> st{{0, 1}};
        while (!st.empty()) {
            auto [x, d] = st.back();
            st.pop_back();
            for (int s = 0; s < 2; ++s) {
                int c = tr.nodes[x].c[s];
                if (c >= 0) st.push_back({c, d + 1});
                else maxd = std::max(maxd, d);
            }
        }
    }
    *depth_out = maxd;
#pragma omp parallel for schedule(dynamic, 64)
    for (long i = 0; i < S; ++i) {
        const double* qq = q + 3 * i;
        double best = std::numeric_limits<double>::infinity();
        uint32_t nn = 0, nl = 0;
        std::vector<std::pair<int, double>> st;
        int node = 0;
        for (;;) {
            const Node& n = tr.nodes[node];
            ++nn;
            double d[2];
            bool h[2];
            for (int s = 0; s < 2; ++s) {
                d[s] = box_d2(qq, n.lo[s], n.hi[s]);
                h[s] = d[s] <= best;
                if (h[s] && n.c[s] < 0) {
                    int fc = tr.order[~n.c[s]];
                    const uint32_t* ff = f + 3 * fc;
                    best = std::min(best, tri_d2(qq, v + 3 * ff[0], v + 3 * ff[1], v + 3 * ff[2]));
                    ++nl;
                    h[s] = false;
                }
            }
            h[0] = h[0] && d[0] <= best;
            h[1] = h[1] && d[1] <= best;
            if (h[0] && h[1]) {
                int nr = d[1] < d[0] ? 1 : 0;
                st.push_back({n.c[1 - nr], d[1 - nr]});
                node = n.c[nr];
                continue;
            }
            if (h[0]) { node = n.c[0]; continue; }
            if (h[1]) { node = n.c[1]; continue; }
            bool found = false;
            while (!st.empty()) {
                auto e = st.back();
                st.pop_back();
                if (e.second <= best) { node = e.first; found = true; break; }
            }
            if (!found) break;
        }
        nodes_out[i] = nn;
        leaves_out[i] = nl;
    }
}
}

// ---- OBB experiment: per child an oriented box aligned with the area-weighted normal of its triangles
namespace {
struct OBB {
    double ax[3][3];  // rows: unit axes
    double lo[3], hi[3];
};
void range_of(const Tree& tr, int c, int& b, int& e) {
    // leaves of the subtree rooted at c are contiguous in Morton order for the LBVH: find extremes
    if (c < 0) { b = e = ~c; return; }
    int lb, le, rb, re;
    range_of(tr, tr.nodes[c].c[0], lb, le);
    range_of(tr, tr.nodes[c].c[1], rb, re);
    b = std::min(lb, rb);
    e = std::max(le, re);
}
OBB make_obb(const Tree& tr, const double* v, const uint32_t* f, int b, int e, int mode) {
    OBB o;
    double n[3] = {0, 0, 0};
    for (int i = b; i <= e; ++i) {
        const uint32_t* ff = f + 3 * tr.order[i];
        const double *A = v + 3 * ff[0], *B = v + 3 * ff[1], *C = v + 3 * ff[2];
        double ab[3] = {B[0] - A[0], B[1] - A[1], B[2] - A[2]}, ac[3] = {C[0] - A[0], C[1] - A[1], C[2] - A[2]};
        n[0] += ab[1] * ac[2] - ab[2] * ac[1]; n[1] += ab[2] * ac[0] - ab[0] * ac[2]; n[2] += ab[0] * ac[1] - ab[1] * ac[0];
    }
    double nl = std::sqrt(n[0] * n[0] + n[1] * n[1] + n[2] * n[2]);
    if (mode == 0 || !(nl > 0)) { n[0] = 1; n[1] = 0; n[2] = 0; nl = 1; }
    for (int k = 0; k < 3; ++k) o.ax[0][k] = n[k] / nl;
    double t[3] = {0, 0, 0};
    int m = std::fabs(o.ax[0][0]) < 0.9 ? 0 : 1;
    t[m] = 1;
    // t1 = normalize(t - (t.n) n)
    double d = t[0] * o.ax[0][0] + t[1] * o.ax[0][1] + t[2] * o.ax[0][2];
    for (int k = 0; k < 3; ++k) t[k] -= d * o.ax[0][k];
    double tl = std::sqrt(t[0] * t[0] + t[1] * t[1] + t[2] * t[2]);
    for (int k = 0; k < 3; ++k) o.ax[1][k] = t[k] / tl;
    o.ax[2][0] = o.ax[0][1] * o.ax[1][2] - o.ax[0][2] * o.ax[1][1];
    o.ax[2][1] = o.ax[0][2] * o.ax[1][0] - o.ax[0][0] * o.ax[1][2];
    o.ax[2][2] = o.ax[0][0] * o.ax[1][1] - o.ax[0][1] * o.ax[1][0];
    for (int a = 0; a < 3; ++a) { o.lo[a] = 1e300; o.hi[a] = -1e300; }
    for (int i = b; i <= e; ++i) {
        const uint32_t* ff = f + 3 * tr.order[i];
        for (int c = 0; c < 3; ++c) {
            const double* P = v + 3 * ff[c];
            for (int a = 0; a < 3; ++a) {
                double p = P[0] * o.ax[a][0] + P[1] * o.ax[a][1] + P[2] * o.ax[a][2];
                o.lo[a] = std::min(o.lo[a], p);
                o.hi[a] = std::max(o.hi[a], p);
            }
        }
    }
    return o;
}
double obb_d2(const double* q, const OBB& o) {
    double s = 0;
    for (int a = 0; a < 3; ++a) {
        double p = q[0] * o.ax[a][0] + q[1] * o.ax[a][1] + q[2] * o.ax[a][2];
        double g = std::max(std::max(o.lo[a] - p, p - o.hi[a]), 0.0);
        s += g * g;
    }
    return s;
}
}  // namespace

extern "C" void model_counts_obb_init(const double* v, const uint32_t* f, int T, const double* q, long S, int mode,
                                      uint32_t* nodes_out, uint32_t* leaves_out, const double* init_best);
extern "C" void model_counts_obb(const double* v, const uint32_t* f, int T, const double* q, long S, int mode,
                                 uint32_t* nodes_out, uint32_t* leaves_out) {
    model_counts_obb_init(v, f, T, q, S, mode, nodes_out, leaves_out, nullptr);
}
// init_best (nullable): per-query initial squared bound (an upper bound of the answer)
static thread_local int* g_first_leaf = nullptr;
extern "C" void model_counts_obb_first(const double* v, const uint32_t* f, int T, const double* q, long S, int mode,
                                       uint32_t* nodes_out, uint32_t* leaves_out, const double* init_best,
                                       int* first_face);
extern "C" void model_counts_obb_init(const double* v, const uint32_t* f, int T, const double* q, long S, int mode,
                                      uint32_t* nodes_out, uint32_t* leaves_out, const double* init_best) {
    model_counts_obb_first(v, f, T, q, S, mode, nodes_out, leaves_out, init_best, nullptr);
}
// first_face (nullable): face of the first leaf each query tests
extern "C" void model_counts_obb_first(const double* v, const uint32_t* f, int T, const double* q, long S, int mode,
                                       uint32_t* nodes_out, uint32_t* leaves_out, const double* init_best,
                                       int* first_face) {
    Tree tr = (mode % 100) >= 10 ? build_median(v, f, T) : build_lbvh(v, f, T);  // mode + 10: median-split tree
    mode = (mode / 100) * 100 + (mode % 10);
    std::vector<OBB> ob(2 * (T - 1));
    for (int x = 0; x < T - 1; ++x) {
        int pb, pe;
        range_of(tr, x, pb, pe);
        OBB parent = make_obb(tr, v, f, pb, pe, 1);
        for (int s = 0; s < 2; ++s) {
            int b, e;
            range_of(tr, tr.nodes[x].c[s], b, e);
            if (mode == 3 || mode == 4) {
                OBB o = parent;
                for (int a = 0; a < 3; ++a) { o.lo[a] = 1e300; o.hi[a] = -1e300; }
                for (int i = b; i <= e; ++i) {
                    const uint32_t* ff = f + 3 * tr.order[i];
                    for (int c = 0; c < 3; ++c) {
                        const double* P = v + 3 * ff[c];
                        for (int a = 0; a < 3; ++a) {
                            double pp = P[0] * o.ax[a][0] + P[1] * o.ax[a][1] + P[2] * o.ax[a][2];
                            o.lo[a] = std::min(o.lo[a], pp); o.hi[a] = std::max(o.hi[a], pp);
                        }
                    }
                }
                ob[2 * x + s] = o;
            } else {
                ob[2 * x + s] = make_obb(tr, v, f, b, e, 1);
            }
        }
    }
    const bool hint = mode >= 100;  // mode + 100: second pass starting from the final best distance
    mode %= 100;
#pragma omp parallel for schedule(dynamic, 64)
    for (long i = 0; i < S; ++i) {
      const double* qq = q + 3 * i;
      double final_best = std::numeric_limits<double>::infinity();
      for (int pass = 0; pass < (hint ? 2 : 1); ++pass) {
        double best = pass == 1 ? final_best * (1 + 1e-12) : std::numeric_limits<double>::infinity();
        if (init_best) best = init_best[i];
        uint32_t nn = 0, nl = 0;
        std::vector<std::pair<int, double>> st;
        int node = 0;
        for (;;) {
            const Node& n = tr.nodes[node];
            ++nn;
            double d[2];
            bool h[2];
            for (int s = 0; s < 2; ++s) {
                d[s] = (mode == 1 || mode == 4) ? std::max(box_d2(qq, n.lo[s], n.hi[s]), obb_d2(qq, ob[2 * node + s]))
                                                 : obb_d2(qq, ob[2 * node + s]);
                h[s] = d[s] <= best;
                if (h[s] && n.c[s] < 0) {
                    int fc = tr.order[~n.c[s]];
                    const uint32_t* ff = f + 3 * fc;
                    best = std::min(best, tri_d2(qq, v + 3 * ff[0], v + 3 * ff[1], v + 3 * ff[2]));
                    if (first_face && nl == 0) first_face[i] = fc;
                    ++nl;
                    h[s] = false;
                }
            }
            h[0] = h[0] && d[0] <= best;
            h[1] = h[1] && d[1] <= best;
            if (h[0] && h[1]) {
                int nr = d[1] < d[0] ? 1 : 0;
                st.push_back({n.c[1 - nr], d[1 - nr]});
                node = n.c[nr];
                continue;
            }
            if (h[0]) { node = n.c[0]; continue; }
            if (h[1]) { node = n.c[1]; continue; }
            bool found = false;
            while (!st.empty()) {
                auto e = st.back();
                st.pop_back();
                if (e.second <= best) { node = e.first; found = true; break; }
            }
            if (!found) break;
        }
        final_best = best;
        nodes_out[i] = nn;
        leaves_out[i] = nl;
      }
    }
}

// ---- packet (wave-uniform) traversal experiment: 64 queries share one node stack; a child is entered
// when any lane's bound passes.  Outputs per packet: uniform node visits, uniform leaf visits and the
// per-lane leaf tests summed over the packet.  mode as model_counts_obb (1 = max(AABB, OBB)).
extern "C" void model_packets_init(const double* v, const uint32_t* f, int T, const double* q, long npk, int mode,
                                   uint32_t* steps_out, uint32_t* leafv_out, uint32_t* leaft_out,
                                   const double* init_best);
extern "C" void model_packets(const double* v, const uint32_t* f, int T, const double* q, long npk, int mode,
                              uint32_t* steps_out, uint32_t* leafv_out, uint32_t* leaft_out) {
    model_packets_init(v, f, T, q, npk, mode, steps_out, leafv_out, leaft_out, nullptr);
}
// init_best (nullable): per-query initial squared bound
extern "C" void model_packets_init(const double* v, const uint32_t* f, int T, const double* q, long npk, int mode,
                                   uint32_t* steps_out, uint32_t* leafv_out, uint32_t* leaft_out,
                                   const double* init_best) {
    Tree tr = build_lbvh(v, f, T);
    std::vector<OBB> ob(2 * (T - 1));
#pragma omp parallel for schedule(dynamic, 256)
    for (int x = 0; x < T - 1; ++x) {
        for (int s = 0; s < 2; ++s) {
            int b, e;
            range_of(tr, tr.nodes[x].c[s], b, e);
            ob[2 * x + s] = make_obb(tr, v, f, b, e, 1);
        }
    }
#pragma omp parallel for schedule(dynamic, 4)
    for (long p = 0; p < npk; ++p) {
        const double* qq = q + 3 * 64 * p;
        double best[64];
        for (int l = 0; l < 64; ++l)
            best[l] = init_best ? init_best[64 * p + l] : std::numeric_limits<double>::infinity();
        uint32_t ns = 0, nlv = 0, nlt = 0;
        struct E { int node; double d[64]; };
        std::vector<E> st;
        int node = 0;
        for (;;) {
            const Node& n = tr.nodes[node];
            ++ns;
            double d[2][64];
            bool need[2] = {false, false};
            for (int s = 0; s < 2; ++s) {
                for (int l = 0; l < 64; ++l) {
                    const double* ql = qq + 3 * l;
                    d[s][l] = mode == 1 ? std::max(box_d2(ql, n.lo[s], n.hi[s]), obb_d2(ql, ob[2 * node + s]))
                                        : box_d2(ql, n.lo[s], n.hi[s]);
                }
                if (n.c[s] < 0) {
                    int fc = tr.order[~n.c[s]];
                    const uint32_t* ff = f + 3 * fc;
                    bool any = false;
                    for (int l = 0; l < 64; ++l)
                        if (d[s][l] <= best[l]) {
                            any = true;
                            ++nlt;
                            best[l] = std::min(best[l], tri_d2(qq + 3 * l, v + 3 * ff[0], v + 3 * ff[1], v + 3 * ff[2]));
                        }
                    if (any) ++nlv;
                }
            }
            int cnt[2] = {0, 0}, nearer0 = 0;
            for (int s = 0; s < 2; ++s) {
                if (n.c[s] < 0) continue;
                for (int l = 0; l < 64; ++l)
                    if (d[s][l] <= best[l]) { need[s] = true; ++cnt[s]; }
            }
            for (int l = 0; l < 64; ++l) nearer0 += d[0][l] <= d[1][l];
            if (need[0] && need[1]) {
                int nr = nearer0 >= 32 ? 0 : 1;
                E e;
                e.node = n.c[1 - nr];
                for (int l = 0; l < 64; ++l) e.d[l] = d[1 - nr][l];
                st.push_back(e);
                node = n.c[nr];
                continue;
            }
            if (need[0]) { node = n.c[0]; continue; }
            if (need[1]) { node = n.c[1]; continue; }
            bool found = false;
            while (!st.empty()) {
                E e = st.back();
                st.pop_back();
                bool any = false;
                for (int l = 0; l < 64; ++l) any |= e.d[l] <= best[l];
                if (any) { node = e.node; found = true; break; }
            }
            if (!found) break;
        }
        steps_out[p] = ns;
        leafv_out[p] = nlv;
        leaft_out[p] = nlt;
    }
}

// ---- BVH4 experiment: collapse the binary LBVH (node x -> grandchildren), oriented boxes of slots
// (0,1) in the frame of binary child A's range and slots (2,3) in child B's.  Per-lane depth-first,
// nearest child first.  Outputs per query: BVH4 nodes visited and leaf tests.
extern "C" void model_counts_bvh4(const double* v, const uint32_t* f, int T, const double* q, long S,
                                  uint32_t* nodes_out, uint32_t* leaves_out) {
    Tree tr = build_lbvh(v, f, T);
    struct Slot { int c; double lo[3], hi[3]; OBB o; };
    struct N4 { Slot s[4]; int n; };
    std::vector<int> map(T - 1, -1);
    std::vector<N4> n4;
    std::vector<int> todo{0};
    map[0] = 0;
    n4.push_back({});
    auto box_of = [&](int parent, int side, double* lo, double* hi) {
        for (int k = 0; k < 3; ++k) { lo[k] = tr.nodes[parent].lo[side][k]; hi[k] = tr.nodes[parent].hi[side][k]; }
    };
    while (!todo.empty()) {
        int x = todo.back();
        todo.pop_back();
        N4 nd{};
        nd.n = 0;
        for (int side = 0; side < 2; ++side) {
            int a = tr.nodes[x].c[side];
            int gb, ge;
            range_of(tr, a, gb, ge);
            OBB frame = make_obb(tr, v, f, gb, ge, 1);
            auto add = [&](int c, int par, int sd) {
                Slot s;
                s.c = c;
                box_of(par, sd, s.lo, s.hi);
                int b, e;
                range_of(tr, c, b, e);
                s.o = frame;
                for (int k = 0; k < 3; ++k) { s.o.lo[k] = 1e300; s.o.hi[k] = -1e300; }
                for (int i = b; i <= e; ++i) {
                    const uint32_t* ff = f + 3 * tr.order[i];
                    for (int cc = 0; cc < 3; ++cc) {
                        const double* P = v + 3 * ff[cc];
                        for (int k = 0; k < 3; ++k) {
                            double pp = P[0] * s.o.ax[k][0] + P[1] * s.o.ax[k][1] + P[2] * s.o.ax[k][2];
                            s.o.lo[k] = std::min(s.o.lo[k], pp); s.o.hi[k] = std::max(s.o.hi[k], pp);
                        }
                    }
                }
                nd.s[nd.n++] = s;
            };
            if (a < 0) add(a, x, side);
            else { add(tr.nodes[a].c[0], a, 0); add(tr.nodes[a].c[1], a, 1); }
        }
        for (int k = 0; k < nd.n; ++k) {
            int c = nd.s[k].c;
            if (c >= 0) {
                map[c] = (int)n4.size();
                n4.push_back({});
                todo.push_back(c);
                nd.s[k].c = map[c];
            }
        }
        n4[map[x]] = nd;
    }
#pragma omp parallel for schedule(dynamic, 64)
    for (long i = 0; i < S; ++i) {
        const double* qq = q + 3 * i;
        double best = std::numeric_limits<double>::infinity();
        uint32_t nn = 0, nl = 0;
        std::vector<std::pair<int, double>> st;
        int node = 0;
        for (;;) {
            const N4& n = n4[node];
            ++nn;
            std::pair<double, int> h[4];
            int nh = 0;
            double dd[4];
            for (int s = 0; s < n.n; ++s) {
                dd[s] = std::max(box_d2(qq, n.s[s].lo, n.s[s].hi), obb_d2(qq, n.s[s].o));
            }
            for (int s = 0; s < n.n; ++s) {
                if (dd[s] <= best && n.s[s].c < 0) {
                    int fc = tr.order[~n.s[s].c];
                    const uint32_t* ff = f + 3 * fc;
                    best = std::min(best, tri_d2(qq, v + 3 * ff[0], v + 3 * ff[1], v + 3 * ff[2]));
                    ++nl;
                }
            }
            for (int s = 0; s < n.n; ++s)
                if (n.s[s].c >= 0 && dd[s] <= best) h[nh++] = {dd[s], n.s[s].c};
            std::sort(h, h + nh);
            if (nh > 0) {
                for (int k = nh - 1; k >= 1; --k) st.push_back({h[k].second, h[k].first});
                node = h[0].second;
                continue;
            }
            bool found = false;
            while (!st.empty()) {
                auto e = st.back();
                st.pop_back();
                if (e.second <= best) { node = e.first; found = true; break; }
            }
            if (!found) break;
        }
        nodes_out[i] = nn;
        leaves_out[i] = nl;
    }
}

// ---- entry-cut experiment: a uniform grid of G^3 cells over the box [blo, bhi]; every cell stores the
// frontier of tree nodes that any point of the cell may need (a node is kept when its oriented-box bound
// from the cell centre is <= d*(centre) + 2 r, r = the cell's half-diagonal; descent stops at depth Dcut or
// when expanding would make the frontier larger than K).  Per query: nodes loaded from the root with a
// near-perfect initial bound (d* (1 + 1e-9)), vs nodes loaded starting from its cell's frontier (every
// frontier node is loaded once), and the frontier size.  depth_hist (64 bins, may be null): nodes loaded
// from the root, by depth, summed over queries.
namespace {
struct ObbTree {
    Tree tr;
    std::vector<OBB> ob;
    std::vector<int> depth;
};
ObbTree make_obb_tree(const double* v, const uint32_t* f, int T) {
    ObbTree t;
    t.tr = build_lbvh(v, f, T);
    t.ob.resize(2 * (T - 1));
#pragma omp parallel for schedule(dynamic, 256)
    for (int x = 0; x < T - 1; ++x)
        for (int s = 0; s < 2; ++s) {
            int b, e;
            range_of(t.tr, t.tr.nodes[x].c[s], b, e);
            t.ob[2 * x + s] = make_obb(t.tr, v, f, b, e, 1);
        }
    t.depth.assign(T - 1, 0);
    std::vector<int> st{0};
    while (!st.empty()) {
        int x = st.back();
        st.pop_back();
        for (int s = 0; s < 2; ++s) {
            int c = t.tr.nodes[x].c[s];
            if (c >= 0) { t.depth[c] = t.depth[x] + 1; st.push_back(c); }
        }
    }
    return t;
}
// nodes loaded by a near-first traversal from the given start nodes with initial squared bound b0;
// returns final best
double walk(const ObbTree& t, const double* v, const uint32_t* f, const double* q, const std::vector<int>& start,
            double b0, uint32_t& nn, uint32_t& nl, uint64_t* hist) {
    double best = b0;
    std::vector<std::pair<int, double>> st;
    for (int k = (int)start.size() - 1; k >= 0; --k) st.push_back({start[k], 0.0});
    int node;
    for (;;) {
        bool found = false;
        while (!st.empty()) {
            auto e = st.back();
            st.pop_back();
            if (e.second <= best) { node = e.first; found = true; break; }
        }
        if (!found) break;
        for (;;) {
            const Node& n = t.tr.nodes[node];
            ++nn;
            if (hist) hist[std::min(t.depth[node], 63)]++;
            double d[2];
            bool h[2];
            for (int s = 0; s < 2; ++s) {
                d[s] = obb_d2(q, t.ob[2 * node + s]);
                h[s] = d[s] <= best;
                if (h[s] && n.c[s] < 0) {
                    int fc = t.tr.order[~n.c[s]];
                    const uint32_t* ff = f + 3 * fc;
                    best = std::min(best, tri_d2(q, v + 3 * ff[0], v + 3 * ff[1], v + 3 * ff[2]));
                    ++nl;
                    h[s] = false;
                }
            }
            h[0] = h[0] && d[0] <= best;
            h[1] = h[1] && d[1] <= best;
            if (h[0] && h[1]) {
                int nr = d[1] < d[0] ? 1 : 0;
                st.push_back({n.c[1 - nr], d[1 - nr]});
                node = n.c[nr];
                continue;
            }
            if (h[0]) { node = n.c[0]; continue; }
            if (h[1]) { node = n.c[1]; continue; }
            break;
        }
    }
    return best;
}
double exact_d2(const ObbTree& t, const double* v, const uint32_t* f, const double* q) {
    uint32_t a = 0, b = 0;
    return walk(t, v, f, q, std::vector<int>{0}, std::numeric_limits<double>::infinity(), a, b, nullptr);
}
// frontier of a cell: BFS by depth from the root, keeping nodes whose bound from c is <= lim (squared)
std::vector<int> cell_cut(const ObbTree& t, const double* c, double lim, int dcut, int K) {
    std::vector<int> cur{0};
    for (int d = 0; d < dcut; ++d) {
        std::vector<int> nxt;
        bool leafy = false;
        for (int x : cur) {
            for (int s = 0; s < 2; ++s) {
                int ch = t.tr.nodes[x].c[s];
                if (obb_d2(c, t.ob[2 * x + s]) > lim) continue;
                if (ch < 0) { leafy = true; continue; }
                nxt.push_back(ch);
            }
        }
        if (leafy || (int)nxt.size() > K || nxt.empty()) break;  // keep cur
        cur.swap(nxt);
    }
    return cur;
}
}  // namespace

extern "C" void model_entry_cut(const double* v, const uint32_t* f, int T, const double* q, long S, const double* blo,
                                const double* bhi, int G, int dcut, int K, uint32_t* root_nodes, uint32_t* cut_nodes,
                                uint32_t* cut_size, uint64_t* depth_hist) {
    ObbTree t = make_obb_tree(v, f, T);
    std::vector<uint64_t> hist(64, 0);
#pragma omp parallel
    {
        std::vector<uint64_t> h(64, 0);
#pragma omp for schedule(dynamic, 64)
        for (long i = 0; i < S; ++i) {
            const double* qq = q + 3 * i;
            const double d2 = exact_d2(t, v, f, qq);
            uint32_t nn = 0, nl = 0;
            walk(t, v, f, qq, std::vector<int>{0}, d2 * (1 + 1e-9), nn, nl, h.data());
            root_nodes[i] = nn;
            // cell of q
            double c[3], r2 = 0;
            bool inside = true;
            for (int k = 0; k < 3; ++k) {
                const double w = (bhi[k] - blo[k]) / G;
                int ci = (int)std::floor((qq[k] - blo[k]) / w);
                if (ci < 0 || ci >= G) inside = false;
                ci = std::min(std::max(ci, 0), G - 1);
                c[k] = blo[k] + (ci + 0.5) * w;
                r2 += 0.25 * w * w;
            }
            if (!inside) { cut_nodes[i] = nn; cut_size[i] = 0; continue; }
            const double r = std::sqrt(r2);
            const double dc = std::sqrt(exact_d2(t, v, f, c));
            const double lim = (dc + 2 * r) * (dc + 2 * r) * (1 + 1e-9);
            std::vector<int> cut = cell_cut(t, c, lim, dcut, K);
            uint32_t cn = 0, cl = 0;
            walk(t, v, f, qq, cut, d2 * (1 + 1e-9), cn, cl, nullptr);
            cut_nodes[i] = cn;
            cut_size[i] = (uint32_t)cut.size();
        }
#pragma omp critical
        for (int k = 0; k < 64; ++k) hist[k] += h[k];
    }
    if (depth_hist)
        for (int k = 0; k < 64; ++k) depth_hist[k] = hist[k];
}

// ---- follower hint experiment: slots in Morton order; every 8th slot is a leader answered exactly; the
// other slots start from a hint of their 64-slot window's 8 leaders: kind 0 = min |q - p_L|^2 (the
// leader's closest point, as k_knn does), 1 = d^2(q, face of the leader whose p_L is nearest), 2 = min over
// the 8 leaders' faces of d^2(q, face), 3 = the exact answer (perfect bound).  Outputs per follower slot:
// nodes loaded and leaf tests (leaders: 0).
extern "C" void model_follower_hints(const double* v, const uint32_t* f, int T, const double* q, long S, int kind,
                                     uint32_t* nodes_out, uint32_t* leaves_out) {
    ObbTree t = make_obb_tree(v, f, T);
    std::vector<int> face(S, -1);
    std::vector<double> pt(3 * S, 0.0);
    // leaders: exact closest face and point (brute force over the tree walk, then a point by projection)
    auto closest = [&](const double* qq, int& bf, double* bp) {
        double best = std::numeric_limits<double>::infinity();
        std::vector<std::pair<int, double>> st{{0, 0.0}};
        bf = -1;
        while (!st.empty()) {
            auto e = st.back();
            st.pop_back();
            if (e.second > best) continue;
            const Node& n = t.tr.nodes[e.first];
            for (int s = 0; s < 2; ++s) {
                double d = obb_d2(qq, t.ob[2 * e.first + s]);
                if (d > best) continue;
                if (n.c[s] < 0) {
                    int fc = t.tr.order[~n.c[s]];
                    const uint32_t* ff = f + 3 * fc;
                    double d2 = tri_d2(qq, v + 3 * ff[0], v + 3 * ff[1], v + 3 * ff[2]);
                    if (d2 < best) { best = d2; bf = fc; }
                } else {
                    st.push_back({n.c[s], d});
                }
            }
        }
        // closest point on face bf: sample by minimising over a projection (use segment/plane logic of tri_d2)
        const uint32_t* ff = f + 3 * bf;
        const double *A = v + 3 * ff[0], *B = v + 3 * ff[1], *C = v + 3 * ff[2];
        // barycentric projection clamp (Ericson)
        double ab[3], ac[3], ap[3];
        for (int k = 0; k < 3; ++k) { ab[k] = B[k] - A[k]; ac[k] = C[k] - A[k]; ap[k] = qq[k] - A[k]; }
        auto dot = [](const double* x, const double* y) { return x[0] * y[0] + x[1] * y[1] + x[2] * y[2]; };
        double d1 = dot(ab, ap), d2 = dot(ac, ap);
        double res[3];
        if (d1 <= 0 && d2 <= 0) { for (int k = 0; k < 3; ++k) res[k] = A[k]; }
        else {
            double bp_[3]; for (int k = 0; k < 3; ++k) bp_[k] = qq[k] - B[k];
            double d3 = dot(ab, bp_), d4 = dot(ac, bp_);
            double cp[3]; for (int k = 0; k < 3; ++k) cp[k] = qq[k] - C[k];
            double d5 = dot(ab, cp), d6 = dot(ac, cp);
            double vc = d1 * d4 - d3 * d2, vb = d5 * d2 - d1 * d6, va = d3 * d6 - d5 * d4;
            if (d3 >= 0 && d4 <= d3) { for (int k = 0; k < 3; ++k) res[k] = B[k]; }
            else if (vc <= 0 && d1 >= 0 && d3 <= 0) { double w = d1 / (d1 - d3); for (int k = 0; k < 3; ++k) res[k] = A[k] + w * ab[k]; }
            else if (d6 >= 0 && d5 <= d6) { for (int k = 0; k < 3; ++k) res[k] = C[k]; }
            else if (vb <= 0 && d2 >= 0 && d6 <= 0) { double w = d2 / (d2 - d6); for (int k = 0; k < 3; ++k) res[k] = A[k] + w * ac[k]; }
            else if (va <= 0 && (d4 - d3) >= 0 && (d5 - d6) >= 0) { double w = (d4 - d3) / ((d4 - d3) + (d5 - d6)); for (int k = 0; k < 3; ++k) res[k] = B[k] + w * (C[k] - B[k]); }
            else { double den = 1.0 / (va + vb + vc); double vv = vb * den, ww = vc * den; for (int k = 0; k < 3; ++k) res[k] = A[k] + ab[k] * vv + ac[k] * ww; }
        }
        for (int k = 0; k < 3; ++k) bp[k] = res[k];
        return best;
    };
#pragma omp parallel for schedule(dynamic, 64)
    for (long i = 0; i < S; i += 8) closest(q + 3 * i, face[i], &pt[3 * i]);
#pragma omp parallel for schedule(dynamic, 64)
    for (long i = 0; i < S; ++i) {
        nodes_out[i] = leaves_out[i] = 0;
        if (i % 8 == 0) continue;
        const double* qq = q + 3 * i;
        const long base = (i / 64) * 64;
        double h = std::numeric_limits<double>::infinity();
        if (kind == 3) {
            int bf; double bp[3];
            h = closest(qq, bf, bp) * (1 + 1e-9);
        } else {
            int nearest_l = -1;
            double hp = std::numeric_limits<double>::infinity();
            for (long L = base; L < base + 64 && L < S; L += 8) {
                double dx = qq[0] - pt[3 * L], dy = qq[1] - pt[3 * L + 1], dz = qq[2] - pt[3 * L + 2];
                double d2 = dx * dx + dy * dy + dz * dz;
                if (d2 < hp) { hp = d2; nearest_l = (int)L; }
                if (kind == 2) {
                    const uint32_t* ff = f + 3 * face[L];
                    h = std::min(h, tri_d2(qq, v + 3 * ff[0], v + 3 * ff[1], v + 3 * ff[2]));
                }
            }
            if (kind == 0) h = hp;
            if (kind == 1) {
                const uint32_t* ff = f + 3 * face[nearest_l];
                h = tri_d2(qq, v + 3 * ff[0], v + 3 * ff[1], v + 3 * ff[2]);
            }
            h *= 1 + 1e-9;
        }
        uint32_t nn = 0, nl = 0;
        walk(t, v, f, qq, std::vector<int>{0}, h, nn, nl, nullptr);
        nodes_out[i] = nn;
        leaves_out[i] = nl;
    }
}

// ---- postponed leaves: the near-first walk with leaf tests delayed until `qmax` leaves are queued or the
// stack runs dry (k_knn's per-lane queue between wave-wide leaf phases); hint kind 0 (min |q - p_L|^2 of
// 8 leaders in the 64-slot window, leaders exact) as model_follower_hints.  Outputs per follower slot.
extern "C" void model_postponed(const double* v, const uint32_t* f, int T, const double* q, long S, int qmax,
                                uint32_t* nodes_out, uint32_t* leaves_out) {
    ObbTree t = make_obb_tree(v, f, T);
    std::vector<double> pt(3 * S, 0.0);
    // leaders' closest points from an exact walk + brute projection via tri_d2's minimiser (vertex/edge/face):
    // reuse model_follower_hints' point by a fine sampling-free approach: closest point = q - (q - p) where
    // p is found by testing the exact best face with a barycentric clamp
    auto best_face = [&](const double* qq) {
        double best = std::numeric_limits<double>::infinity();
        int bf = -1;
        std::vector<std::pair<int, double>> st{{0, 0.0}};
        while (!st.empty()) {
            auto e = st.back();
            st.pop_back();
            if (e.second > best) continue;
            const Node& n = t.tr.nodes[e.first];
            for (int s = 0; s < 2; ++s) {
                double d = obb_d2(qq, t.ob[2 * e.first + s]);
                if (d > best) continue;
                if (n.c[s] < 0) {
                    int fc = t.tr.order[~n.c[s]];
                    const uint32_t* ff = f + 3 * fc;
                    double d2 = tri_d2(qq, v + 3 * ff[0], v + 3 * ff[1], v + 3 * ff[2]);
                    if (d2 < best) { best = d2; bf = fc; }
                } else st.push_back({n.c[s], d});
            }
        }
        return bf;
    };
    auto closest_pt = [&](const double* qq, int bf, double* res) {
        const uint32_t* ff = f + 3 * bf;
        const double *A = v + 3 * ff[0], *B = v + 3 * ff[1], *C = v + 3 * ff[2];
        // minimise over a fine barycentric grid refined by projection (adequate for a hint model)
        double bestd = 1e300;
        for (int i = 0; i <= 40; ++i)
            for (int j = 0; i + j <= 40; ++j) {
                double a = i / 40.0, b = j / 40.0, c = 1 - a - b, p[3], d = 0;
                for (int k = 0; k < 3; ++k) { p[k] = a * A[k] + b * B[k] + c * C[k]; d += (p[k] - qq[k]) * (p[k] - qq[k]); }
                if (d < bestd) { bestd = d; for (int k = 0; k < 3; ++k) res[k] = p[k]; }
            }
    };
#pragma omp parallel for schedule(dynamic, 64)
    for (long i = 0; i < S; i += 8) closest_pt(q + 3 * i, best_face(q + 3 * i), &pt[3 * i]);
#pragma omp parallel for schedule(dynamic, 64)
    for (long i = 0; i < S; ++i) {
        nodes_out[i] = leaves_out[i] = 0;
        if (i % 8 == 0) continue;
        const double* qq = q + 3 * i;
        const long base = (i / 64) * 64;
        double best = std::numeric_limits<double>::infinity();
        for (long L = base; L < base + 64 && L < S; L += 8) {
            double dx = qq[0] - pt[3 * L], dy = qq[1] - pt[3 * L + 1], dz = qq[2] - pt[3 * L + 2];
            best = std::min(best, dx * dx + dy * dy + dz * dz);
        }
        best *= 1 + 1e-9;
        uint32_t nn = 0, nl = 0;
        std::vector<std::pair<int, double>> st;
        std::vector<int> queue;
        auto flush = [&]() {
            for (int lf : queue) {
                int fc = t.tr.order[lf];
                const uint32_t* ff = f + 3 * fc;
                best = std::min(best, tri_d2(qq, v + 3 * ff[0], v + 3 * ff[1], v + 3 * ff[2]));
                ++nl;
            }
            queue.clear();
        };
        int node = 0;
        bool have = true;
        for (;;) {
            if (!have) {
                bool found = false;
                while (!st.empty()) {
                    auto e = st.back();
                    st.pop_back();
                    if (e.second <= best) { node = e.first; found = true; break; }
                }
                if (!found) {
                    if (queue.empty()) break;
                    flush();
                    continue;
                }
            }
            have = true;
            if ((int)queue.size() > qmax - 2) flush();
            const Node& n = t.tr.nodes[node];
            ++nn;
            double d[2];
            bool h[2];
            for (int s = 0; s < 2; ++s) {
                d[s] = obb_d2(qq, t.ob[2 * node + s]);
                h[s] = d[s] <= best;
                if (h[s] && n.c[s] < 0) {
                    if (qmax == 0) {
                        int fc = t.tr.order[~n.c[s]];
                        const uint32_t* ff = f + 3 * fc;
                        best = std::min(best, tri_d2(qq, v + 3 * ff[0], v + 3 * ff[1], v + 3 * ff[2]));
                        ++nl;
                    } else {
                        queue.push_back(~n.c[s]);
                    }
                    h[s] = false;
                }
            }
            h[0] = h[0] && d[0] <= best;
            h[1] = h[1] && d[1] <= best;
            if (h[0] && h[1]) {
                int nr = d[1] < d[0] ? 1 : 0;
                st.push_back({n.c[1 - nr], d[1 - nr]});
                node = n.c[nr];
                continue;
            }
            if (h[0]) { node = n.c[0]; continue; }
            if (h[1]) { node = n.c[1]; continue; }
            have = false;
        }
        nodes_out[i] = nn;
        leaves_out[i] = nl;
    }
}

// ---- node encoding experiment: both children's oriented boxes in the PARENT's frame (k_obb_*: the frame
// from the area-weighted normal of the node's Morton range, t from the x or y axis), and their extents
// quantised like build.hip encode_node.  enc: 0 exact fp64 extents, 1 8-bit codes with a power-of-two scale
// (254 * 2^e >= range, the product format), 2 8-bit codes with scale range / 255 (any fp32), 3 16-bit
// codes with scale range / 65535.  init_best (nullable) as model_counts_obb_init.
namespace {
struct QBox { double ax[3][3]; double lo[2][3], hi[2][3]; };
}
Tree build_tree_kind(const double* v, const uint32_t* f, int T, int kind);
extern "C" void model_encoded_tree(const double* v, const uint32_t* f, int T, const double* q, long S, int enc,
                                   const double* init_best, uint32_t* nodes_out, uint32_t* leaves_out, int tree_kind);
extern "C" void model_encoded(const double* v, const uint32_t* f, int T, const double* q, long S, int enc,
                              const double* init_best, uint32_t* nodes_out, uint32_t* leaves_out) {
    model_encoded_tree(v, f, T, q, S, enc, init_best, nodes_out, leaves_out, 0);
}
extern "C" void model_encoded_tree(const double* v, const uint32_t* f, int T, const double* q, long S, int enc,
                                   const double* init_best, uint32_t* nodes_out, uint32_t* leaves_out, int tree_kind) {
    Tree tr = build_tree_kind(v, f, T, tree_kind);
    std::vector<QBox> nb(T - 1);
#pragma omp parallel for schedule(dynamic, 256)
    for (int x = 0; x < T - 1; ++x) {
        int b, e;
        range_of(tr, x, b, e);
        double s[3] = {0, 0, 0};
        for (int i = b; i <= e; ++i) {
            const uint32_t* ff = f + 3 * tr.order[i];
            const double *A = v + 3 * ff[0], *B = v + 3 * ff[1], *C = v + 3 * ff[2];
            double ab[3] = {B[0] - A[0], B[1] - A[1], B[2] - A[2]}, ac[3] = {C[0] - A[0], C[1] - A[1], C[2] - A[2]};
            s[0] += ab[1] * ac[2] - ab[2] * ac[1]; s[1] += ab[2] * ac[0] - ab[0] * ac[2]; s[2] += ab[0] * ac[1] - ab[1] * ac[0];
        }
        double len = std::sqrt(s[0] * s[0] + s[1] * s[1] + s[2] * s[2]);
        double n[3] = {1, 0, 0};
        if (len > 0) for (int k = 0; k < 3; ++k) n[k] = s[k] / len;
        double ee[3] = {0, 0, 0};
        ee[std::fabs(n[0]) < 0.9 ? 0 : 1] = 1;
        double d = ee[0] * n[0] + ee[1] * n[1] + ee[2] * n[2], t[3];
        for (int k = 0; k < 3; ++k) t[k] = ee[k] - d * n[k];
        double tl = std::sqrt(t[0] * t[0] + t[1] * t[1] + t[2] * t[2]);
        for (int k = 0; k < 3; ++k) t[k] /= tl;
        QBox& qb = nb[x];
        for (int k = 0; k < 3; ++k) { qb.ax[0][k] = n[k]; qb.ax[1][k] = t[k]; }
        qb.ax[2][0] = n[1] * t[2] - n[2] * t[1]; qb.ax[2][1] = n[2] * t[0] - n[0] * t[2]; qb.ax[2][2] = n[0] * t[1] - n[1] * t[0];
        for (int sd = 0; sd < 2; ++sd) {
            int cb, ce;
            range_of(tr, tr.nodes[x].c[sd], cb, ce);
            for (int a = 0; a < 3; ++a) { qb.lo[sd][a] = 1e300; qb.hi[sd][a] = -1e300; }
            for (int i = cb; i <= ce; ++i) {
                const uint32_t* ff = f + 3 * tr.order[i];
                for (int c = 0; c < 3; ++c) {
                    const double* P = v + 3 * ff[c];
                    for (int a = 0; a < 3; ++a) {
                        double p = P[0] * qb.ax[a][0] + P[1] * qb.ax[a][1] + P[2] * qb.ax[a][2];
                        qb.lo[sd][a] = std::min(qb.lo[sd][a], p);
                        qb.hi[sd][a] = std::max(qb.hi[sd][a], p);
                    }
                }
            }
        }
        if (enc == 0) continue;
        for (int a = 0; a < 3; ++a) {
            double base = std::min(qb.lo[0][a], qb.lo[1][a]);
            double top = std::max(qb.hi[0][a], qb.hi[1][a]);
            double range = top - base, sc;
            if (enc == 1) { int e2 = range > 0 ? (int)std::ceil(std::log2(range / 254.0)) : -126; sc = std::ldexp(1.0, e2); }
            else if (enc == 2) sc = range > 0 ? range / 255.0 : 1e-30;
            else sc = range > 0 ? range / 65535.0 : 1e-30;
            for (int sd = 0; sd < 2; ++sd) {
                qb.lo[sd][a] = base + std::floor((qb.lo[sd][a] - base) / sc) * sc;
                qb.hi[sd][a] = base + std::ceil((qb.hi[sd][a] - base) / sc) * sc;
            }
        }
    }
#pragma omp parallel for schedule(dynamic, 64)
    for (long i = 0; i < S; ++i) {
        const double* qq = q + 3 * i;
        double best = init_best ? init_best[i] : std::numeric_limits<double>::infinity();
        uint32_t nn = 0, nl = 0;
        std::vector<std::pair<int, double>> st;
        int node = 0;
        for (;;) {
            const Node& n = tr.nodes[node];
            const QBox& qb = nb[node];
            ++nn;
            double pr[3];
            for (int a = 0; a < 3; ++a) pr[a] = qq[0] * qb.ax[a][0] + qq[1] * qb.ax[a][1] + qq[2] * qb.ax[a][2];
            double dd[2];
            bool h[2];
            for (int s = 0; s < 2; ++s) {
                double acc = 0;
                for (int a = 0; a < 3; ++a) {
                    double g = std::max(std::max(qb.lo[s][a] - pr[a], pr[a] - qb.hi[s][a]), 0.0);
                    acc += g * g;
                }
                dd[s] = acc;
                h[s] = acc <= best;
                if (h[s] && n.c[s] < 0) {
                    int fc = tr.order[~n.c[s]];
                    const uint32_t* ff = f + 3 * fc;
                    best = std::min(best, tri_d2(qq, v + 3 * ff[0], v + 3 * ff[1], v + 3 * ff[2]));
                    ++nl;
                    h[s] = false;
                }
            }
            h[0] = h[0] && dd[0] <= best;
            h[1] = h[1] && dd[1] <= best;
            if (h[0] && h[1]) {
                int nr = dd[1] < dd[0] ? 1 : 0;
                st.push_back({n.c[1 - nr], dd[1 - nr]});
                node = n.c[nr];
                continue;
            }
            if (h[0]) { node = n.c[0]; continue; }
            if (h[1]) { node = n.c[1]; continue; }
            bool found = false;
            while (!st.empty()) {
                auto e = st.back();
                st.pop_back();
                if (e.second <= best) { node = e.first; found = true; break; }
            }
            if (!found) break;
        }
        nodes_out[i] = nn;
        leaves_out[i] = nl;
    }
}


// ---- tree builders for the encoding experiment: 0 LBVH (build.hip), 1 median split on the longest axis of
// the centroid AABB (CGAL-like), 2 median split along the longest tangent axis of the node's own frame
// (area-weighted normal n; centroids projected on t, b; split on the larger spread), 3 as 2 but split at the
// spatial midpoint of that axis (object partition, unbalanced allowed)
namespace {
const double* g_v = nullptr;
const uint32_t* g_f = nullptr;
int g_bins = 16;
int build_oriented_rec(Tree& tr, std::vector<int>& idx, int b, int e, const std::vector<double>& cen,
                       const std::vector<double>& area, int mode) {
    if (e - b == 1) return ~b;
    int node = (int)tr.nodes.size();
    tr.nodes.push_back(Node{});
    double s[3] = {0, 0, 0};
    for (int i = b; i < e; ++i)
        for (int k = 0; k < 3; ++k) s[k] += area[3 * idx[i] + k];
    double len = std::sqrt(s[0] * s[0] + s[1] * s[1] + s[2] * s[2]);
    double n[3] = {1, 0, 0};
    if (len > 1e-9 * (e - b) * 1e-12) for (int k = 0; k < 3; ++k) n[k] = s[k] / len;
    // candidate axes: for a closed/curved patch use the 3 principal directions of the centroid spread
    // (covariance eigenvectors via power iteration); otherwise the tangent plane
    double m[3] = {0, 0, 0};
    for (int i = b; i < e; ++i)
        for (int k = 0; k < 3; ++k) m[k] += cen[3 * idx[i] + k];
    for (int k = 0; k < 3; ++k) m[k] /= (e - b);
    double C[3][3] = {{0}};
    for (int i = b; i < e; ++i) {
        double d[3];
        for (int k = 0; k < 3; ++k) d[k] = cen[3 * idx[i] + k] - m[k];
        for (int a = 0; a < 3; ++a)
            for (int c = 0; c < 3; ++c) C[a][c] += d[a] * d[c];
    }
    double ax[3] = {1, 1, 1};
    if (mode == 10 || mode == 11) {
        // binned SAH over the candidate axes x, y, z, t, b: cost N_L * SA_L + N_R * SA_R of the children's boxes
        // in the node frame (n, t, b) (mode 11: lateral area t-extent * b-extent only)
        double fr[3][3] = {{1, 0, 0}, {0, 1, 0}, {0, 0, 1}};
        if (len > 0) {
            double ee[3] = {0, 0, 0};
            ee[std::fabs(n[0]) < 0.9 ? 0 : 1] = 1;
            double d = ee[0] * n[0] + ee[1] * n[1] + ee[2] * n[2], t[3];
            for (int k = 0; k < 3; ++k) t[k] = ee[k] - d * n[k];
            double tl = std::sqrt(t[0] * t[0] + t[1] * t[1] + t[2] * t[2]);
            for (int k = 0; k < 3; ++k) t[k] /= tl;
            double bb[3] = {n[1] * t[2] - n[2] * t[1], n[2] * t[0] - n[0] * t[2], n[0] * t[1] - n[1] * t[0]};
            for (int k = 0; k < 3; ++k) { fr[0][k] = n[k]; fr[1][k] = t[k]; fr[2][k] = bb[k]; }
        }
        double cands[5][3] = {{1, 0, 0}, {0, 1, 0}, {0, 0, 1}, {fr[1][0], fr[1][1], fr[1][2]}, {fr[2][0], fr[2][1], fr[2][2]}};
        const int NB = g_bins;
        double best_cost = 1e300; int best_axis = -1; double best_split = 0;
        for (int c = 0; c < 5; ++c) {
            double lo = 1e300, hi = -1e300;
            for (int i = b; i < e; ++i) {
                double k = cen[3 * idx[i]] * cands[c][0] + cen[3 * idx[i] + 1] * cands[c][1] + cen[3 * idx[i] + 2] * cands[c][2];
                lo = std::min(lo, k); hi = std::max(hi, k);
            }
            if (!(hi > lo)) continue;
            std::vector<double> bmin(NB * 3, 1e300), bmax(NB * 3, -1e300);
            std::vector<int> bcnt(NB, 0);
            for (int i = b; i < e; ++i) {
                int t = idx[i];
                double k = cen[3 * t] * cands[c][0] + cen[3 * t + 1] * cands[c][1] + cen[3 * t + 2] * cands[c][2];
                int bi = std::min(NB - 1, (int)((k - lo) / (hi - lo) * NB));
                bcnt[bi]++;
                for (int vv = 0; vv < 3; ++vv) {
                    const double* P = g_v + 3 * g_f[3 * t + vv];
                    for (int a = 0; a < 3; ++a) {
                        double pr = P[0] * fr[a][0] + P[1] * fr[a][1] + P[2] * fr[a][2];
                        bmin[3 * bi + a] = std::min(bmin[3 * bi + a], pr);
                        bmax[3 * bi + a] = std::max(bmax[3 * bi + a], pr);
                    }
                }
            }
            auto sa = [&](const double* mn, const double* mx) {
                double x = mx[0] - mn[0], y = mx[1] - mn[1], z = mx[2] - mn[2];
                return mode == 11 ? y * z : 2 * (x * y + y * z + z * x);
            };
            std::vector<double> lcost(NB, 0);
            double mn[3] = {1e300, 1e300, 1e300}, mx[3] = {-1e300, -1e300, -1e300};
            int cntL = 0;
            for (int sp = 1; sp < NB; ++sp) {
                for (int a = 0; a < 3; ++a) { mn[a] = std::min(mn[a], bmin[3 * (sp - 1) + a]); mx[a] = std::max(mx[a], bmax[3 * (sp - 1) + a]); }
                cntL += bcnt[sp - 1];
                lcost[sp] = cntL ? cntL * sa(mn, mx) : -1;
            }
            double mn2[3] = {1e300, 1e300, 1e300}, mx2[3] = {-1e300, -1e300, -1e300};
            int cntR = 0;
            for (int sp = NB - 1; sp >= 1; --sp) {
                for (int a = 0; a < 3; ++a) { mn2[a] = std::min(mn2[a], bmin[3 * sp + a]); mx2[a] = std::max(mx2[a], bmax[3 * sp + a]); }
                cntR += bcnt[sp];
                if (cntR == 0 || lcost[sp] < 0) continue;
                double cst = lcost[sp] + cntR * sa(mn2, mx2);
                if (cst < best_cost) { best_cost = cst; best_axis = c; best_split = lo + (hi - lo) * sp / NB; }
            }
        }
        if (best_axis >= 0) {
            for (int k = 0; k < 3; ++k) ax[k] = cands[best_axis][k];
            auto key2 = [&](int x) { return cen[3 * x] * ax[0] + cen[3 * x + 1] * ax[1] + cen[3 * x + 2] * ax[2]; };
            auto it = std::partition(idx.begin() + b, idx.begin() + e, [&](int x) { return key2(x) < best_split; });
            int mid = (int)(it - idx.begin());
            if (mid == b || mid == e) { mid = (b + e) / 2; std::nth_element(idx.begin() + b, idx.begin() + mid, idx.begin() + e, [&](int x, int y) { return key2(x) < key2(y); }); }
            int l = build_oriented_rec(tr, idx, b, mid, cen, area, mode);
            int r = build_oriented_rec(tr, idx, mid, e, cen, area, mode);
            tr.nodes[node].c[0] = l;
            tr.nodes[node].c[1] = r;
            return node;
        }
        int mid = (b + e) / 2;
        int l = build_oriented_rec(tr, idx, b, mid, cen, area, mode);
        int r = build_oriented_rec(tr, idx, mid, e, cen, area, mode);
        tr.nodes[node].c[0] = l;
        tr.nodes[node].c[1] = r;
        return node;
    }
    if (mode == 5 || mode == 6 || mode == 7) {
        // 5: longest axis of the centroid AABB, split at its spatial middle; 6: the longest centroid spread
        // among x, y, z and the node frame's two tangent axes, split at the median
        double cands[5][3] = {{1, 0, 0}, {0, 1, 0}, {0, 0, 1}, {0, 0, 0}, {0, 0, 0}};
        int nc = 3;
        if ((mode == 6 || mode == 7) && len > 0) {
            double ee[3] = {0, 0, 0};
            ee[std::fabs(n[0]) < 0.9 ? 0 : 1] = 1;
            double d = ee[0] * n[0] + ee[1] * n[1] + ee[2] * n[2], t[3];
            for (int k = 0; k < 3; ++k) t[k] = ee[k] - d * n[k];
            double tl = std::sqrt(t[0] * t[0] + t[1] * t[1] + t[2] * t[2]);
            for (int k = 0; k < 3; ++k) t[k] /= tl;
            double bb[3] = {n[1] * t[2] - n[2] * t[1], n[2] * t[0] - n[0] * t[2], n[0] * t[1] - n[1] * t[0]};
            for (int k = 0; k < 3; ++k) { cands[3][k] = t[k]; cands[4][k] = bb[k]; }
            nc = 5;
        }
        double bestw = -1;
        for (int c = 0; c < nc; ++c) {
            double lo = 1e300, hi = -1e300;
            for (int i = b; i < e; ++i) {
                double k = cen[3 * idx[i]] * cands[c][0] + cen[3 * idx[i] + 1] * cands[c][1] + cen[3 * idx[i] + 2] * cands[c][2];
                lo = std::min(lo, k); hi = std::max(hi, k);
            }
            if (hi - lo > bestw) { bestw = hi - lo; for (int k = 0; k < 3; ++k) ax[k] = cands[c][k]; }
        }
    } else
    for (int it = 0; it < 50; ++it) {
        double y[3];
        for (int a = 0; a < 3; ++a) y[a] = C[a][0] * ax[0] + C[a][1] * ax[1] + C[a][2] * ax[2];
        double l = std::sqrt(y[0] * y[0] + y[1] * y[1] + y[2] * y[2]);
        if (!(l > 0)) break;
        for (int a = 0; a < 3; ++a) ax[a] = y[a] / l;
    }
    (void)n;
    auto key = [&](int x) { return cen[3 * x] * ax[0] + cen[3 * x + 1] * ax[1] + cen[3 * x + 2] * ax[2]; };
    int mid = (b + e) / 2;
    if (mode == 3 || mode == 5 || mode == 7) {
        double lo = 1e300, hi = -1e300;
        for (int i = b; i < e; ++i) { double k = key(idx[i]); lo = std::min(lo, k); hi = std::max(hi, k); }
        double c = 0.5 * (lo + hi);
        auto it = std::partition(idx.begin() + b, idx.begin() + e, [&](int x) { return key(x) < c; });
        mid = (int)(it - idx.begin());
        if (mid == b || mid == e) mid = (b + e) / 2;
        std::nth_element(idx.begin() + b, idx.begin() + mid, idx.begin() + e, [&](int x, int y) { return key(x) < key(y); });
    } else {
        std::nth_element(idx.begin() + b, idx.begin() + mid, idx.begin() + e, [&](int x, int y) { return key(x) < key(y); });
    }
    int l = build_oriented_rec(tr, idx, b, mid, cen, area, mode);
    int r = build_oriented_rec(tr, idx, mid, e, cen, area, mode);
    tr.nodes[node].c[0] = l;
    tr.nodes[node].c[1] = r;
    return node;
}
}  // namespace
namespace {
// hybrid: the LBVH's nodes over more than K leaves, its subtrees over at most K leaves rebuilt with mode 7
int hybrid_rec(const Tree& lb, int c, Tree& out, std::vector<int>& idx, const std::vector<double>& cen,
               const std::vector<double>& area, int K, int mode) {
    if (c < 0) return c;  // a leaf: position ~c
    int b, e;
    range_of(lb, c, b, e);
    if (e - b + 1 <= K) return build_oriented_rec(out, idx, b, e + 1, cen, area, mode);
    int node = (int)out.nodes.size();
    out.nodes.push_back(Node{});
    int l = hybrid_rec(lb, lb.nodes[c].c[0], out, idx, cen, area, K, mode);
    int r = hybrid_rec(lb, lb.nodes[c].c[1], out, idx, cen, area, K, mode);
    out.nodes[node].c[0] = l;
    out.nodes[node].c[1] = r;
    return node;
}
}  // namespace
Tree build_tree_kind(const double* v, const uint32_t* f, int T, int kind) {
    if (kind == 0) return build_lbvh(v, f, T);
    if (kind == 1) return build_median(v, f, T);
    std::vector<double> cen(3 * T), area(3 * T);
    for (int t = 0; t < T; ++t) {
        const double *A = v + 3 * f[3 * t], *B = v + 3 * f[3 * t + 1], *C = v + 3 * f[3 * t + 2];
        double ab[3] = {B[0] - A[0], B[1] - A[1], B[2] - A[2]}, ac[3] = {C[0] - A[0], C[1] - A[1], C[2] - A[2]};
        area[3 * t] = ab[1] * ac[2] - ab[2] * ac[1];
        area[3 * t + 1] = ab[2] * ac[0] - ab[0] * ac[2];
        area[3 * t + 2] = ab[0] * ac[1] - ab[1] * ac[0];
        for (int k = 0; k < 3; ++k) cen[3 * t + k] = (A[k] + B[k] + C[k]) / 3.0;
    }
    Tree tr;
    std::vector<int> idx(T);
    std::iota(idx.begin(), idx.end(), 0);
    tr.nodes.reserve(T);
    g_v = v;
    g_f = f;
    if (kind >= 100) {  // 100 + log2 K: hybrid over the LBVH (split mode 7); 200 + log2 K: mode 10; 300: mode 11
        Tree lb = build_lbvh(v, f, T);
        idx = lb.order;
        const int m = kind >= 300 ? 11 : (kind >= 200 ? 10 : 7);
        hybrid_rec(lb, 0, tr, idx, cen, area, 1 << (kind % 100), m);
    } else {
        build_oriented_rec(tr, idx, 0, T, cen, area, kind);
    }
    tr.order = idx;
    return tr;
}


// ---- leaf screen experiment: lower bound of the triangle distance from the plane distance and the three
// edge half-planes (max of the in-plane signed edge distances), exact arithmetic; counts, over the leaf
// tests of a walk with initial bound b0, how many the screen would reject against the best at that moment.
namespace {
double tri_lb2(const double* q, const double* A, const double* B, const double* C) {
    double a[3], b[3], c[3];
    for (int k = 0; k < 3; ++k) { a[k] = A[k] - q[k]; b[k] = B[k] - q[k]; c[k] = C[k] - q[k]; }
    double ab[3] = {b[0] - a[0], b[1] - a[1], b[2] - a[2]}, ac[3] = {c[0] - a[0], c[1] - a[1], c[2] - a[2]};
    double n[3] = {ab[1] * ac[2] - ab[2] * ac[1], ab[2] * ac[0] - ab[0] * ac[2], ab[0] * ac[1] - ab[1] * ac[0]};
    double nl = std::sqrt(n[0] * n[0] + n[1] * n[1] + n[2] * n[2]);
    if (!(nl > 0)) return 0;
    double h = (n[0] * a[0] + n[1] * a[1] + n[2] * a[2]) / nl;
    const double* P[3] = {a, b, c};
    double smax = 0;
    for (int e = 0; e < 3; ++e) {
        const double* p1 = P[e];
        const double* p2 = P[(e + 1) % 3];
        double d[3] = {p2[0] - p1[0], p2[1] - p1[1], p2[2] - p1[2]};
        double m[3] = {d[1] * n[2] - d[2] * n[1], d[2] * n[0] - d[0] * n[2], d[0] * n[1] - d[1] * n[0]};
        double ml = std::sqrt(m[0] * m[0] + m[1] * m[1] + m[2] * m[2]);
        if (!(ml > 0)) continue;
        double sd = -(m[0] * p1[0] + m[1] * p1[1] + m[2] * p1[2]) / ml;
        smax = std::max(smax, sd);
    }
    return h * h + smax * smax;
}
}  // namespace
extern "C" void model_leaf_screen(const double* v, const uint32_t* f, int T, const double* q, long S, const double* b0,
                                  uint32_t* tests_out, uint32_t* rejects_out, uint32_t* improves_out) {
    ObbTree t = make_obb_tree(v, f, T);
#pragma omp parallel for schedule(dynamic, 64)
    for (long i = 0; i < S; ++i) {
        const double* qq = q + 3 * i;
        double best = b0 ? b0[i] : std::numeric_limits<double>::infinity();
        uint32_t nt = 0, nr = 0, ni = 0;
        std::vector<std::pair<int, double>> st{{0, 0.0}};
        while (!st.empty()) {
            auto e = st.back();
            st.pop_back();
            if (e.second > best) continue;
            int node = e.first;
            for (;;) {
                const Node& n = t.tr.nodes[node];
                double d[2];
                bool h[2];
                for (int s2 = 0; s2 < 2; ++s2) {
                    d[s2] = obb_d2(qq, t.ob[2 * node + s2]);
                    h[s2] = d[s2] <= best;
                    if (h[s2] && n.c[s2] < 0) {
                        int fc = t.tr.order[~n.c[s2]];
                        const uint32_t* ff = f + 3 * fc;
                        const double* A = v + 3 * ff[0]; const double* B = v + 3 * ff[1]; const double* C = v + 3 * ff[2];
                        double lb = tri_lb2(qq, A, B, C);
                        double dd = tri_d2(qq, A, B, C);
                        ++nt;
                        if (lb > best * (1 + 1e-6)) ++nr;
                        if (dd < best) { ++ni; best = dd; }
                        h[s2] = false;
                    }
                }
                h[0] = h[0] && d[0] <= best;
                h[1] = h[1] && d[1] <= best;
                if (h[0] && h[1]) {
                    int nr2 = d[1] < d[0] ? 1 : 0;
                    st.push_back({n.c[1 - nr2], d[1 - nr2]});
                    node = n.c[nr2];
                    continue;
                }
                if (h[0]) { node = n.c[0]; continue; }
                if (h[1]) { node = n.c[1]; continue; }
                break;
            }
        }
        tests_out[i] = nt;
        rejects_out[i] = nr;
        improves_out[i] = ni;
    }
}
