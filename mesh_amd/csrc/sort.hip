// Stable LSD radix sort of (u32 key, u32 value) pairs and a device-wide exclusive scan, written for
// gfx950 wave64.  Used twice on the hot path: Morton order of triangle centroids (LBVH build, K1) and
// Morton order of query points (traversal coherence, K2).
//
// One pass = 8 key bits, three launches:
//   k_hist     each 256-thread workgroup counts the digits of a 4096-key tile in per-wave LDS
//              histograms (coalesced 4-B loads), writes its 256 counts digit-major: hist[d*nb + b]
//   scan       exclusive scan of hist  ->  global output offset of (digit, tile)
//   k_scatter  the tile is re-read wave by wave in index order; each key's rank among equal digits is
//              found with eight 64-lane ballots (no LDS atomics, deterministic, stable), per-wave digit
//              counters live in LDS; the tile is staged in LDS in its locally sorted order and written
//              out linearly, so each digit's run of the tile is one contiguous, coalesced store.
// HBM traffic per pass: read keys+values twice (8 B + 4 B), write keys+values once (8 B).
#include <algorithm>

#include "internal.h"

namespace msh {

constexpr int kSortItems = 16;
constexpr int kSortTile = kBlock * kSortItems;  // 4096 keys per workgroup
constexpr int kWaveItems = 64 * kSortItems;     // 1024 keys per wave

__global__ __launch_bounds__(kBlock) void k_hist(const uint32_t* __restrict__ keys, size_t n, int shift,
                                                 uint32_t* __restrict__ hist, unsigned nb) {
    __shared__ uint32_t h[4][256];
    const int tid = threadIdx.x, w = tid >> 6;
    for (int i = tid; i < 1024; i += kBlock) (&h[0][0])[i] = 0;
    __syncthreads();
    const size_t base = (size_t)blockIdx.x * kSortTile;
#pragma unroll
    for (int k = 0; k < kSortItems; ++k) {
        const size_t i = base + (size_t)k * kBlock + tid;
        if (i < n) atomicAdd(&h[w][(keys[i] >> shift) & 255u], 1u);
    }
    __syncthreads();
    const uint32_t c = h[0][tid] + h[1][tid] + h[2][tid] + h[3][tid];
    hist[(size_t)tid * nb + blockIdx.x] = c;
}

__device__ inline uint32_t block_exclusive_scan(uint32_t x, uint32_t* sh, uint32_t& total);

__global__ __launch_bounds__(kBlock) void k_scatter(const uint32_t* __restrict__ keys, const uint32_t* __restrict__ vals,
                                                    uint32_t* __restrict__ okeys, uint32_t* __restrict__ ovals, size_t n,
                                                    int shift, const uint32_t* __restrict__ offs, unsigned nb) {
    __shared__ uint32_t wcnt[4][256];
    __shared__ uint32_t gbase[256];   // global start of (digit, this tile) minus the digit's local start
    __shared__ uint32_t lstart[256];  // local (in-tile) start of each digit
    __shared__ uint32_t scan_sh[4];
    __shared__ uint32_t lk[kSortTile], lv[kSortTile];
    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
    wcnt[0][tid] = 0; wcnt[1][tid] = 0; wcnt[2][tid] = 0; wcnt[3][tid] = 0;
    const uint32_t g_off = offs[(size_t)tid * nb + blockIdx.x];
    __syncthreads();
    const size_t tile0 = (size_t)blockIdx.x * kSortTile;
    const size_t base = tile0 + (size_t)w * kWaveItems;
    const unsigned long long lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    uint32_t kk[kSortItems], vv[kSortItems], rr[kSortItems];
#pragma unroll
    for (int it = 0; it < kSortItems; ++it) {
        const size_t i = base + (size_t)it * 64 + lane;
        const bool valid = i < n;
        const uint32_t key = valid ? keys[i] : 0u;
        const uint32_t val = valid ? vals[i] : 0u;
        const uint32_t d = (key >> shift) & 255u;
        unsigned long long peers = __ballot(valid);
#pragma unroll
        for (int b = 0; b < 8; ++b) {
            const bool bit = (d >> b) & 1u;
            const unsigned long long m = __ballot(bit);
            peers &= bit ? m : ~m;
        }
        const uint32_t below = (uint32_t)__popcll(peers & lt);
        const uint32_t cnt = (uint32_t)__popcll(peers);
        const uint32_t prev = valid ? wcnt[w][d] : 0u;
        const bool leader = valid && ((peers & lt) == 0ull);
        if (leader) wcnt[w][d] = prev + cnt;
        kk[it] = key;
        vv[it] = val;
        rr[it] = prev + below;
    }
    __syncthreads();
    {
        // digit tid: local start = exclusive scan of the tile's digit counts; per-wave starts inside it
        const uint32_t c0 = wcnt[0][tid], c1 = wcnt[1][tid], c2 = wcnt[2][tid], c3 = wcnt[3][tid];
        uint32_t total;
        const uint32_t ls = block_exclusive_scan(c0 + c1 + c2 + c3, scan_sh, total);
        lstart[tid] = ls;
        gbase[tid] = g_off - ls;
        wcnt[0][tid] = ls;
        wcnt[1][tid] = ls + c0;
        wcnt[2][tid] = ls + c0 + c1;
        wcnt[3][tid] = ls + c0 + c1 + c2;
    }
    __syncthreads();
    // stage the tile in LDS in its locally sorted (stable) order ...
#pragma unroll
    for (int it = 0; it < kSortItems; ++it) {
        const size_t i = base + (size_t)it * 64 + lane;
        if (i < n) {
            const uint32_t d = (kk[it] >> shift) & 255u;
            const uint32_t p = wcnt[w][d] + rr[it];
            lk[p] = kk[it];
            lv[p] = vv[it];
        }
    }
    __syncthreads();
    // ... and write it out linearly: consecutive lanes write consecutive addresses of one digit's run
    const uint32_t tn = (uint32_t)(n - tile0 < (size_t)kSortTile ? n - tile0 : (size_t)kSortTile);
    for (uint32_t p = tid; p < tn; p += kBlock) {
        const uint32_t key = lk[p];
        const uint32_t dst = gbase[(key >> shift) & 255u] + p;
        okeys[dst] = key;
        ovals[dst] = lv[p];
    }
}

// ---- exclusive scan (u32), 4096 elements per workgroup, recursive over block sums ----
__device__ inline uint32_t block_exclusive_scan(uint32_t x, uint32_t* sh, uint32_t& total) {
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    uint32_t incl = x;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(incl, o, 64);
        if (lane >= o) incl += y;
    }
    if (lane == 63) sh[w] = incl;
    __syncthreads();
    uint32_t woff = 0;
    for (int k = 0; k < w; ++k) woff += sh[k];
    total = sh[0] + sh[1] + sh[2] + sh[3];
    __syncthreads();
    return woff + incl - x;
}

__global__ __launch_bounds__(kBlock) void k_scan_block(uint32_t* __restrict__ data, size_t n, uint32_t* __restrict__ sums) {
    __shared__ uint32_t sh[4];
    const size_t base = (size_t)blockIdx.x * kSortTile + (size_t)threadIdx.x * kSortItems;
    uint32_t v[kSortItems];
    uint32_t s = 0;
#pragma unroll
    for (int k = 0; k < kSortItems; ++k) {
        v[k] = (base + k < n) ? data[base + k] : 0u;
        s += v[k];
    }
    uint32_t total;
    uint32_t run = block_exclusive_scan(s, sh, total);
#pragma unroll
    for (int k = 0; k < kSortItems; ++k) {
        if (base + k < n) data[base + k] = run;
        run += v[k];
    }
    if (threadIdx.x == 0 && sums) sums[blockIdx.x] = total;
}

__global__ __launch_bounds__(kBlock) void k_scan_add(uint32_t* __restrict__ data, size_t n, const uint32_t* __restrict__ sums) {
    const uint32_t add = sums[blockIdx.x];
    const size_t base = (size_t)blockIdx.x * kSortTile;
#pragma unroll
    for (int k = 0; k < kSortItems; ++k) {
        const size_t i = base + (size_t)k * kBlock + threadIdx.x;
        if (i < n) data[i] += add;
    }
}

static size_t scan_scratch_elems(size_t n) {
    size_t total = 0;
    while (n > (size_t)kSortTile) {
        n = (n + kSortTile - 1) / kSortTile;
        total += n;
    }
    return total + 1;
}

static int scan_rec(uint32_t* data, size_t n, uint32_t* scratch, hipStream_t s) {
    const size_t nb = (n + kSortTile - 1) / kSortTile;
    if (nb <= 1) {
        k_scan_block<<<1, kBlock, 0, s>>>(data, n, nullptr);
        MSH_HIP(hipGetLastError());
        return MSH_OK;
    }
    uint32_t* sums = scratch;
    k_scan_block<<<(unsigned)nb, kBlock, 0, s>>>(data, n, sums);
    MSH_HIP(hipGetLastError());
    MSH_TRY(scan_rec(sums, nb, scratch + nb, s));
    k_scan_add<<<(unsigned)nb, kBlock, 0, s>>>(data, n, sums);
    MSH_HIP(hipGetLastError());
    return MSH_OK;
}

int exclusive_scan_u32(uint32_t* data, size_t n, Workspace& ws, hipStream_t s) {
    if (n == 0) return MSH_OK;
    MSH_TRY(ws.scan.reserve(scan_scratch_elems(n) * sizeof(uint32_t)));
    return scan_rec(data, n, ws.scan.as<uint32_t>(), s);
}

int radix_sort_pairs(uint32_t* keys, uint32_t* vals, uint32_t* keys_alt, uint32_t* vals_alt, size_t n, int bits,
                     Workspace& ws, hipStream_t s, int lo_bit, bool* in_alt) {
    if (n <= 1) return MSH_OK;
    if (n > 0xFFFFFFFFull) {
        set_error("radix sort: %zu elements exceed the 32-bit offset range", n);
        return MSH_EINVAL;
    }
    TimedLaunch tl("sort", s);
    const unsigned nb = (unsigned)((n + kSortTile - 1) / kSortTile);
    MSH_TRY(ws.hist.reserve((size_t)nb * 256 * sizeof(uint32_t)));
    uint32_t* hist = ws.hist.as<uint32_t>();
    uint32_t *src_k = keys, *src_v = vals, *dst_k = keys_alt, *dst_v = vals_alt;
    int passes = 0;
    for (int shift = lo_bit; shift < lo_bit + bits; shift += 8, ++passes) {
        k_hist<<<nb, kBlock, 0, s>>>(src_k, n, shift, hist, nb);
        MSH_HIP(hipGetLastError());
        MSH_TRY(exclusive_scan_u32(hist, (size_t)nb * 256, ws, s));
        k_scatter<<<nb, kBlock, 0, s>>>(src_k, src_v, dst_k, dst_v, n, shift, hist, nb);
        MSH_HIP(hipGetLastError());
        uint32_t* t;
        t = src_k; src_k = dst_k; dst_k = t;
        t = src_v; src_v = dst_v; dst_v = t;
    }
    if (in_alt) *in_alt = (passes & 1) != 0;
    if ((passes & 1) && !in_alt) {
        MSH_HIP(hipMemcpyAsync(keys, src_k, n * sizeof(uint32_t), hipMemcpyDeviceToDevice, s));
        MSH_HIP(hipMemcpyAsync(vals, src_v, n * sizeof(uint32_t), hipMemcpyDeviceToDevice, s));
    }
    return MSH_OK;
}

// ---- query order: one-sweep LSD sort of 24-bit query Morton keys (decoupled look-back) ----
// The closest-point path sorts its queries by the top 24 bits of their 30-bit Morton codes (8 bits per pass,
// 3 passes).  Instead of a histogram launch, a device-wide scan and a scatter launch per pass (radix_sort_pairs),
// one launch computes every key AND all three digit histograms up front (k_os_keys), and each pass is ONE
// launch whose tiles find their output offsets by decoupled look-back (Merrill & Garland, "Single-pass Parallel
// Prefix Scan with Decoupled Look-back"; the Onesweep radix sort of Adinets & Merrill applies it per digit):
// a tile takes the next tile id from a counter (so every earlier tile is already running), publishes its own
// per-digit counts, then walks back over earlier tiles' published words — counts (flag 1) or inclusive
// prefixes (flag 2) — until it meets a prefix.  Per key: 24 B of query row in and 4 B of key out (keys +
// histograms), then 4 + 8 B, 8 + 8 B and 8 + 4 B (the last pass writes only the permutation).  Status words
// carry flag << 30 | count, so n < 2^30 (larger calls use radix_sort_pairs).
constexpr uint32_t kOsAgg = 1u << 30, kOsPrefix = 2u << 30, kOsCount = (1u << 30) - 1u;
constexpr int kOsPasses = 3;
constexpr unsigned kOsHistBlocks = 1024;  // persistent grid of k_os_keys (its histograms are added atomically)

__global__ __launch_bounds__(kBlock) void k_os_keys(const double* __restrict__ q, size_t n, float lx, float ly, float lz,
                                                    float hx, float hy, float hz, int lo_bit, uint32_t* __restrict__ keys,
                                                    uint32_t* __restrict__ ghist) {
    __shared__ uint32_t h[kOsPasses][4][256];
    const int tid = threadIdx.x, w = tid >> 6;
    for (int k = tid; k < kOsPasses * 4 * 256; k += kBlock) (&h[0][0][0])[k] = 0;
    __syncthreads();
    const size_t ntiles = (n + kSortTile - 1) / kSortTile;
    for (size_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
#pragma unroll 4
        for (int k = 0; k < kSortItems; ++k) {
            const size_t i = tile * kSortTile + (size_t)k * kBlock + tid;
            if (i >= n) break;
            const uint32_t key = (query_morton30(q[3 * i], q[3 * i + 1], q[3 * i + 2], lx, ly, lz, hx, hy, hz) >> lo_bit) &
                                 0xFFFFFFu;
            keys[i] = key;
            atomicAdd(&h[0][w][key & 255u], 1u);
            atomicAdd(&h[1][w][(key >> 8) & 255u], 1u);
            atomicAdd(&h[2][w][key >> 16], 1u);
        }
    }
    __syncthreads();
#pragma unroll
    for (int d = 0; d < kOsPasses; ++d) {
        const uint32_t c = h[d][0][tid] + h[d][1][tid] + h[d][2][tid] + h[d][3][tid];
        if (c) atomicAdd(&ghist[d * 256 + tid], c);
    }
}

// One pass over digit (key >> shift) & 255.  FIRST: the values are the key indices (not read); LAST: only the
// values (the permutation) are written.
template <bool FIRST, bool LAST>
__global__ __launch_bounds__(kBlock) void k_os_pass(const uint32_t* __restrict__ keys, const uint32_t* __restrict__ vals,
                                                    uint32_t* __restrict__ okeys, uint32_t* __restrict__ ovals, size_t n,
                                                    int shift, const uint32_t* __restrict__ ghist, uint32_t* status,
                                                    unsigned* tile_ctr) {
    __shared__ uint32_t wcnt[4][256];
    __shared__ uint32_t gbase[256];
    __shared__ uint32_t scan_sh[4];
    __shared__ uint32_t lk[kSortTile], lv[kSortTile];
    __shared__ unsigned s_tile;
    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
    if (tid == 0) s_tile = atomicAdd(tile_ctr, 1u);
    wcnt[0][tid] = 0; wcnt[1][tid] = 0; wcnt[2][tid] = 0; wcnt[3][tid] = 0;
    __syncthreads();
    const size_t tile = s_tile;
    const size_t tile0 = tile * kSortTile;
    const size_t base = tile0 + (size_t)w * kWaveItems;
    const unsigned long long lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    uint32_t kk[kSortItems], vv[kSortItems], rr[kSortItems];
#pragma unroll
    for (int it = 0; it < kSortItems; ++it) {
        const size_t i = base + (size_t)it * 64 + lane;
        const bool valid = i < n;
        const uint32_t key = valid ? keys[i] : 0u;
        const uint32_t val = FIRST ? (uint32_t)i : (valid ? vals[i] : 0u);
        const uint32_t d = (key >> shift) & 255u;
        unsigned long long peers = __ballot(valid);
#pragma unroll
        for (int b = 0; b < 8; ++b) {
            const bool bit = (d >> b) & 1u;
            const unsigned long long m = __ballot(bit);
            peers &= bit ? m : ~m;
        }
        const uint32_t below = (uint32_t)__popcll(peers & lt);
        const uint32_t cnt = (uint32_t)__popcll(peers);
        const uint32_t prev = valid ? wcnt[w][d] : 0u;
        if (valid && (peers & lt) == 0ull) wcnt[w][d] = prev + cnt;
        kk[it] = key;
        vv[it] = val;
        rr[it] = prev + below;
    }
    __syncthreads();
    {
        // thread tid owns digit tid: this tile's count, published at once (flag 1), then the look-back
        const uint32_t c0 = wcnt[0][tid], c1 = wcnt[1][tid], c2 = wcnt[2][tid], c3 = wcnt[3][tid];
        const uint32_t c = c0 + c1 + c2 + c3;
        uint32_t* my = status + tile * 256 + tid;
        __hip_atomic_store(my, (tile == 0 ? kOsPrefix : kOsAgg) | c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        uint32_t excl = 0;
        for (size_t t = tile; t > 0;) {
            --t;
            uint32_t v;
            do {
                v = __hip_atomic_load(status + t * 256 + tid, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            } while ((v & ~kOsCount) == 0u);
            excl += v & kOsCount;
            if (v & kOsPrefix) break;
        }
        if (tile > 0) __hip_atomic_store(my, kOsPrefix | (excl + c), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        uint32_t total;
        const uint32_t ls = block_exclusive_scan(c, scan_sh, total);            // digit's start inside the tile
        const uint32_t gs = block_exclusive_scan(ghist[tid], scan_sh, total);   // digit's start in the output
        gbase[tid] = gs + excl - ls;
        wcnt[0][tid] = ls;
        wcnt[1][tid] = ls + c0;
        wcnt[2][tid] = ls + c0 + c1;
        wcnt[3][tid] = ls + c0 + c1 + c2;
    }
    __syncthreads();
#pragma unroll
    for (int it = 0; it < kSortItems; ++it) {
        const size_t i = base + (size_t)it * 64 + lane;
        if (i < n) {
            const uint32_t p = wcnt[w][(kk[it] >> shift) & 255u] + rr[it];
            lk[p] = kk[it];
            lv[p] = vv[it];
        }
    }
    __syncthreads();
    const uint32_t tn = (uint32_t)(n - tile0 < (size_t)kSortTile ? n - tile0 : (size_t)kSortTile);
    for (uint32_t p = tid; p < tn; p += kBlock) {
        const uint32_t key = lk[p];
        const uint32_t dst = gbase[(key >> shift) & 255u] + p;
        if (!LAST) okeys[dst] = key;
        ovals[dst] = lv[p];
    }
}

int query_sort(const double* d_q, size_t n, const float* lo, const float* hi, int lo_bit, uint32_t* keys,
               uint32_t* keys_alt, uint32_t* perm, uint32_t* perm_alt, Workspace& ws, hipStream_t s, bool* in_alt) {
    *in_alt = false;
    if (n == 0) return MSH_OK;
    if (n > (size_t)kOsCount) {
        set_error("query sort: %zu keys exceed the one-sweep status range", n);
        return MSH_EINVAL;
    }
    const unsigned nt = (unsigned)((n + kSortTile - 1) / kSortTile);
    // ghist (3 x 256) | tile counters (3, one 128-B line each) | status (3 passes x nt tiles x 256 digits)
    const size_t words = kOsPasses * 256 + kOsPasses * 32 + (size_t)kOsPasses * nt * 256;
    MSH_TRY(ws.hist.reserve(words * sizeof(uint32_t)));
    uint32_t* ghist = ws.hist.as<uint32_t>();
    unsigned* ctr = ghist + kOsPasses * 256;
    uint32_t* status = ctr + kOsPasses * 32;
    MSH_HIP(hipMemsetAsync(ghist, 0, words * sizeof(uint32_t), s));
    {
        TimedLaunch tl("morton", s);
        const unsigned nb = std::min<unsigned>(nt, kOsHistBlocks);
        k_os_keys<<<nb, kBlock, 0, s>>>(d_q, n, lo[0], lo[1], lo[2], hi[0], hi[1], hi[2], lo_bit, keys, ghist);
        MSH_HIP(hipGetLastError());
    }
    TimedLaunch tl("sort", s);
    k_os_pass<true, false><<<nt, kBlock, 0, s>>>(keys, nullptr, keys_alt, perm_alt, n, 0, ghist, status, ctr);
    MSH_HIP(hipGetLastError());
    k_os_pass<false, false><<<nt, kBlock, 0, s>>>(keys_alt, perm_alt, keys, perm, n, 8, ghist + 256,
                                                  status + (size_t)nt * 256, ctr + 32);
    MSH_HIP(hipGetLastError());
    k_os_pass<false, true><<<nt, kBlock, 0, s>>>(keys, perm, nullptr, perm_alt, n, 16, ghist + 512,
                                                 status + 2 * (size_t)nt * 256, ctr + 64);
    MSH_HIP(hipGetLastError());
    *in_alt = true;  // the permutation is in perm_alt
    return MSH_OK;
}

}  // namespace msh
