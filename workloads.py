"""Synthetic workloads of BASELINE.md §3 (no network: meshes and queries are generated, seeded).

C1  sphere.obj fixture (tests/golden/meshes.npz), 100k uniform queries in the bbox + 10% (seed 0)
C2  SMPL-topology stand-in: UV sphere 84 slices x 82 rings + 2 poles = 6,890 v / 13,776 f, ellipsoid
    0.6 x 1.7 x 0.3 m with seeded low-frequency radial noise (seed 1); queries = area-weighted surface
    samples + N(0, 1 cm) (seed 2)
C3  class-I geodesic icosphere, frequency 224 = 1,003,520 f / 501,762 v, unit radius; queries uniform
    in [-1.1, 1.1]^3 (seed 3)
C4  4096 x UV surface 72 x 70 + 2 = 5,042 v / 10,080 f with per-mesh radii + noise (seed 4 + i)
C5  geodesic icosphere frequency 500 = 5,000,000 f, radially bumped r = 1 + 0.1 sin(5θ) sin(4φ)
"""
import os

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))


def sphere_fixture():
    g = np.load(os.path.join(ROOT, "tests", "golden", "meshes.npz"))
    return g["sphere_v"], g["sphere_f"]


def uniform_in_box(lo, hi, n, seed, margin=0.1):
    lo = np.asarray(lo, np.float64)
    hi = np.asarray(hi, np.float64)
    ext = hi - lo
    return np.random.default_rng(seed).uniform(lo - margin * ext, hi + margin * ext, (n, 3))


def c1_queries(n=100000):
    v, f = sphere_fixture()
    return uniform_in_box(v.min(0), v.max(0), n, seed=0)


def uv_sphere(slices, rings):
    """UV sphere: `rings` latitude rings of `slices` vertices + 2 poles; F = 2 * slices * rings."""
    th = np.pi * (np.arange(1, rings + 1) / (rings + 1.0))  # polar angle of each ring
    ph = 2 * np.pi * (np.arange(slices) / float(slices))
    T, PH = np.meshgrid(th, ph, indexing="ij")
    ring_v = np.stack([np.sin(T) * np.cos(PH), np.sin(T) * np.sin(PH), np.cos(T)], -1).reshape(-1, 3)
    v = np.vstack([[0, 0, 1.0], ring_v, [0, 0, -1.0]])
    top, bot = 0, v.shape[0] - 1
    idx = lambda r, s: 1 + r * slices + (s % slices)  # noqa: E731
    f = []
    for s in range(slices):
        f.append([top, idx(0, s), idx(0, s + 1)])
    for r in range(rings - 1):
        for s in range(slices):
            a, b, c, d = idx(r, s), idx(r, s + 1), idx(r + 1, s), idx(r + 1, s + 1)
            f.append([a, c, b])
            f.append([b, c, d])
    for s in range(slices):
        f.append([bot, idx(rings - 1, s + 1), idx(rings - 1, s)])
    return v, np.array(f, dtype=np.uint32)


def _radial_noise(v, rng, amp=0.03, nfreq=4):
    r = np.ones(v.shape[0])
    for _ in range(nfreq):
        k = rng.normal(size=3) * 2.0
        r += amp * np.sin(v @ k + rng.uniform(0, 2 * np.pi))
    return v * r[:, None]


def c2_mesh():
    v, f = uv_sphere(84, 82)
    rng = np.random.default_rng(1)
    v = _radial_noise(v, rng) * np.array([0.3, 0.85, 0.15])  # 0.6 x 1.7 x 0.3 m
    return v, f


def surface_samples(v, f, n, seed, sigma):
    rng = np.random.default_rng(seed)
    tri = v[f.astype(np.int64)]
    area = 0.5 * np.linalg.norm(np.cross(tri[:, 1] - tri[:, 0], tri[:, 2] - tri[:, 0]), axis=1)
    fi = rng.choice(f.shape[0], size=n, p=area / area.sum())
    r1 = np.sqrt(rng.uniform(size=n))
    r2 = rng.uniform(size=n)
    t = tri[fi]
    p = (1 - r1)[:, None] * t[:, 0] + (r1 * (1 - r2))[:, None] * t[:, 1] + (r1 * r2)[:, None] * t[:, 2]
    return p + rng.normal(scale=sigma, size=p.shape), fi


def c2_queries(n=10_000_000, seed=2):
    v, f = c2_mesh()
    return surface_samples(v, f, n, seed, 0.01)[0]


_ICO_CACHE = {}


def icosahedron():
    t = (1.0 + 5 ** 0.5) / 2.0
    v = np.array([[-1, t, 0], [1, t, 0], [-1, -t, 0], [1, -t, 0], [0, -1, t], [0, 1, t], [0, -1, -t], [0, 1, -t],
                  [t, 0, -1], [t, 0, 1], [-t, 0, -1], [-t, 0, 1]], dtype=np.float64)
    v /= np.linalg.norm(v, axis=1)[:, None]
    f = np.array([[0, 11, 5], [0, 5, 1], [0, 1, 7], [0, 7, 10], [0, 10, 11], [1, 5, 9], [5, 11, 4], [11, 10, 2],
                  [10, 7, 6], [7, 1, 8], [3, 9, 4], [3, 4, 2], [3, 2, 6], [3, 6, 8], [3, 8, 9], [4, 9, 5],
                  [2, 4, 11], [6, 2, 10], [8, 6, 7], [9, 8, 1]], dtype=np.int64)
    return v, f


def geodesic_icosphere(freq):
    """Class-I geodesic sphere: 20 freq^2 faces, 10 freq^2 + 2 vertices, unit radius."""
    if freq in _ICO_CACHE:
        return _ICO_CACHE[freq]
    V0, F0 = icosahedron()
    n = freq
    # barycentric lattice (i, j) with i + j <= n on each face
    ii, jj = np.meshgrid(np.arange(n + 1), np.arange(n + 1), indexing="ij")
    keep = ii + jj <= n
    ii, jj = ii[keep], jj[keep]
    lat_index = -np.ones((n + 1, n + 1), dtype=np.int64)
    lat_index[ii, jj] = np.arange(ii.size)
    a, b, c = V0[F0[:, 0]], V0[F0[:, 1]], V0[F0[:, 2]]
    wa = (n - ii - jj) / float(n)
    wb = ii / float(n)
    wc = jj / float(n)
    # exact integer lattice keys for dedupe: global vertex = sum of integer weights on icosahedron ids
    pts = (wa[None, :, None] * a[:, None, :] + wb[None, :, None] * b[:, None, :] + wc[None, :, None] * c[:, None, :])
    key = np.round(pts.reshape(-1, 3) * 1e9).astype(np.int64)
    _, first, inv = np.unique(key, axis=0, return_index=True, return_inverse=True)
    inv = inv.reshape(-1)
    verts = pts.reshape(-1, 3)[first]
    verts /= np.linalg.norm(verts, axis=1)[:, None]
    # triangles on the lattice
    up_i, up_j = np.meshgrid(np.arange(n), np.arange(n), indexing="ij")
    m = up_i + up_j <= n - 1
    ui, uj = up_i[m], up_j[m]
    up = np.stack([lat_index[ui, uj], lat_index[ui + 1, uj], lat_index[ui, uj + 1]], -1)
    m2 = up_i + up_j <= n - 2
    di, dj = up_i[m2], up_j[m2]
    down = np.stack([lat_index[di + 1, dj], lat_index[di + 1, dj + 1], lat_index[di, dj + 1]], -1)
    local = np.vstack([up, down])
    npts = ii.size
    faces = (local[None, :, :] + (np.arange(20) * npts)[:, None, None]).reshape(-1, 3)
    faces = inv[faces].astype(np.uint32)
    _ICO_CACHE[freq] = (verts, faces)
    return verts, faces


def c3_mesh():
    return geodesic_icosphere(224)


def c3_workload_name(freq, S):
    """config.workload of bench.py (and the key its PMC profile is matched on): one C3 query stream of S
    rows per step, sharded contiguously over the GPUs."""
    return ("C3: geodesic icosphere freq %d (%d faces, %d vertices), %d uniform queries in [-1.1,1.1]^3 (seed 3) "
            "per step, sharded contiguously over the GPUs" % (freq, 20 * freq ** 2, 10 * freq ** 2 + 2, S))


def c3_stream(S, device, seed=3):
    """The C3 query stream (BASELINE configs[2]): S rows uniform in [-1.1, 1.1]^3 drawn by torch's generator
    for `device` with `seed` — the same rows on every device of one kind, so every rank can draw the whole
    stream and keep its shard (c3_shard) instead of receiving it.  (S, 3) float64, contiguous."""
    import torch
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    return (torch.rand((S, 3), generator=g, dtype=torch.float64, device=device) * 2.2 - 1.1).contiguous()


def c3_shard(q, rank, world):
    """Rank `rank`'s contiguous shard of the (S, 3) stream q (mesh_amd.distributed.shard_range) as a view
    (rows of a C-contiguous array: contiguous), with its [start, stop)."""
    from mesh_amd.distributed import shard_range
    a, b = shard_range(q.shape[0], rank, world)
    return q[a:b], (a, b)


def c5_mesh():
    v, f = geodesic_icosphere(500)
    th = np.arccos(np.clip(v[:, 2], -1, 1))
    ph = np.arctan2(v[:, 1], v[:, 0])
    r = 1 + 0.1 * np.sin(5 * th) * np.sin(4 * ph)
    return v * r[:, None], f


def c4_mesh(i):
    v, f = uv_sphere(72, 70)
    rng = np.random.default_rng(4 + i)
    radii = rng.uniform(0.07, 0.12, size=3)
    return _radial_noise(v, rng) * radii, f


def c4_batch(B=4096, S=10_000, seed=4):
    """C4 (BASELINE configs[3]): B meshes of the 72x70+2 UV topology (5,042 v / 10,080 f), per-mesh
    shape c4_mesh(i), and S scan points per mesh = surface samples + N(0, 0.005 diag) noise.
    Returns v (B,P,3), f (T,3), q (B,S,3)."""
    f = c4_mesh(0)[1]
    v = np.stack([c4_mesh(i)[0] for i in range(B)])
    q = np.empty((B, S, 3))
    for i in range(B):
        diag = float(np.linalg.norm(v[i].max(0) - v[i].min(0)))
        q[i] = surface_samples(v[i], f, S, seed=seed * 100003 + i, sigma=0.005 * diag)[0]
    return v, f, q


def c4_batch_range(lo, hi, B=4096, S=10_000, seed=4):
    """Meshes [lo, hi) of c4_batch(B, S, seed), each identical to its row there, inside full-size (B, ...) arrays
    whose other rows are left unset: a rank of C4's mesh-range split generates only its own meshes."""
    f = c4_mesh(0)[1]
    P = c4_mesh(0)[0].shape[0]
    v = np.empty((B, P, 3))
    q = np.empty((B, S, 3))
    for i in range(lo, hi):
        v[i] = c4_mesh(i)[0]
        diag = float(np.linalg.norm(v[i].max(0) - v[i].min(0)))
        q[i] = surface_samples(v[i], f, S, seed=seed * 100003 + i, sigma=0.005 * diag)[0]
    return v, f, q


def fibonacci_cameras(C=64, radius=3.0):
    """C5 cameras: C points of a Fibonacci sphere of the given radius."""
    k = np.arange(C) + 0.5
    z = 1 - 2 * k / C
    r = np.sqrt(1 - z * z)
    ph = np.pi * (1 + 5 ** 0.5) * k
    return radius * np.stack([r * np.cos(ph), r * np.sin(ph), z], 1)


def c5_rays(v, f, n=10_000_000, seed=5, sigma=0.01):
    """C5 nearest_alongnormal rays: area-weighted surface samples s on face fi, offset by delta ~ N(0, sigma)
    along the unit face normal nrm; the ray direction is nrm.  Returns p = s + delta * nrm, nrm, delta, fi."""
    rng = np.random.default_rng(seed)
    tri = v[f.astype(np.int64)]
    cr = np.cross(tri[:, 1] - tri[:, 0], tri[:, 2] - tri[:, 0])
    area = np.linalg.norm(cr, axis=1)
    fi = rng.choice(f.shape[0], size=n, p=area / area.sum())
    r1 = np.sqrt(rng.uniform(size=n))
    r2 = rng.uniform(size=n)
    t = tri[fi]
    s = (1 - r1)[:, None] * t[:, 0] + (r1 * (1 - r2))[:, None] * t[:, 1] + (r1 * r2)[:, None] * t[:, 2]
    del t
    nrm = cr[fi] / area[fi][:, None]
    delta = rng.normal(scale=sigma, size=n)
    return s + delta[:, None] * nrm, nrm, delta, fi
