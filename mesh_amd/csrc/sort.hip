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

}  // namespace msh
