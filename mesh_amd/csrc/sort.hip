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

// The first level of exclusive_scan_u32 only, when the consumer finishes it (tile_offset): *nsums chunk totals in
// ws.scan, or *nsums = 0 with data fully scanned.
static int scan_chunks(uint32_t* data, size_t n, Workspace& ws, hipStream_t s, const uint32_t** sums, unsigned* nsums,
                       unsigned max_sums) {
    const size_t nc = (n + kSortTile - 1) / kSortTile;
    *sums = nullptr;
    *nsums = 0;
    if (nc <= 1 || nc > max_sums) return exclusive_scan_u32(data, n, ws, s);
    MSH_TRY(ws.scan.reserve(nc * sizeof(uint32_t)));
    k_scan_block<<<(unsigned)nc, kBlock, 0, s>>>(data, n, ws.scan.as<uint32_t>());
    MSH_HIP(hipGetLastError());
    *sums = ws.scan.as<uint32_t>();
    *nsums = (unsigned)nc;
    return MSH_OK;
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


// ---- query order: stable sort of query rows by the top 24 bits of their 30-bit Morton codes ----
// Specialised for the query path (3 passes of 8 bits, values = row indices), so the passes move fewer bytes than
// radix_sort_pairs does with the same ballot ranking:
//   k_qkeys      Morton key of every row + the first pass's per-tile digit counts (no separate histogram read);
//   pass 1       u32 keys in, rows implied by the index (no value array is written or read), packed u64 out
//                (key << 32 | row: one 8-B store per element, so a digit run of a tile is twice as long in
//                bytes as two 4-B arrays);
//   pass 2       packed in, packed out;   pass 3  packed in, rows only out (the keys are not needed after it).
// Tiles of kQsNT x 16 elements: with 512-thread blocks a tile's 256 digit runs average 32 elements (256 B
// packed), so the scattered stores are mostly whole lines.  HBM bytes per element: 24 (rows) + 4 (keys) in
// k_qkeys; 4 + 8 in pass 1; 8 (histogram) + 8 + 8 in pass 2; 8 + 8 + 4 in pass 3.
// 512-thread blocks, 8192-key tiles: 73 KB of LDS, so two blocks per CU overlap each other's load, rank and write
// phases (1024 threads and 16384-key tiles took 145 KB, one block per CU): C3 100M rows 1.94-1.98 -> 1.77 ms per sort,
// 12.5M rows 0.267 -> 0.226 ms (profiles/r05_ab_sort_fold_nt.jsonl); a stable sort, so the same order either way
#ifndef MSH_QSORT_NT
#define MSH_QSORT_NT 512
#endif
// Query order along the Hilbert curve of the 256^3 cells instead of the Morton curve: C3 100M 1985-1990 ->
// 2033-2058 M q/s, 12.5M rows 1390 -> 1401-1416 M q/s (profiles/r05_ab_leaders_sort_resume.jsonl)
#ifndef MSH_QORDER_HILBERT
#define MSH_QORDER_HILBERT 1
#endif
constexpr int kQsNT = MSH_QSORT_NT;

// 24-bit Hilbert index of a cell of the 256^3 grid: Skilling's transform ("Programming the Hilbert curve", 2004: the
// axes to the transposed form, then the transposed bits interleaved, axis 0 first at each level; numpy copy in
// scripts/sort_debug.py hilbert24) run as the state machine it amounts to.  Consecutive indices are face-adjacent
// cells, so a tile of consecutive queries never jumps across the box the way a Morton tile does at the octree's
// block boundaries.  kHilbertTable[state * 8 + octant] = index digit | next state << 3 over the Morton code's 3-bit
// octants from the top; scripts/hilbert_table.py derives the 24 states from the transform and checks the table
// against it on all 2^24 cells (tests/test_hilbert_table.py).  k_qkeys expands it to two octants per step in LDS
// (hilbert_pairs): four dependent LDS reads per key instead of ~200 VALU operations of the transform (C3 100M rows:
// 0.59 -> 0.56 ms per key launch, profiles/r05_ab_hilbert_lut.jsonl).
__constant__ uint8_t kHilbertTable[192] = {8, 17, 27, 2, 39, 46, 52, 5,
 56, 71, 73, 86, 91, 20, 10, 13,
 48, 1, 103, 110, 115, 18, 12, 21,
 126, 129, 29, 26, 79, 80, 140, 3,
 148, 43, 37, 34, 127, 128, 78, 81,
 156, 45, 35, 42, 31, 6, 160, 105,
 72, 87, 139, 4, 57, 70, 50, 53,
 0, 171, 111, 76, 49, 58, 102, 61,
 180, 143, 83, 184, 69, 54, 66, 97,
 16, 123, 9, 74, 47, 60, 38, 77,
 132, 95, 85, 14, 67, 144, 82, 33,
 142, 55, 185, 96, 93, 116, 90, 11,
 188, 107, 175, 176, 101, 98, 62, 65,
 164, 109, 119, 22, 99, 106, 152, 41,
 174, 177, 63, 64, 117, 114, 92, 19,
 30, 125, 161, 122, 7, 172, 104, 75,
 130, 25, 133, 166, 179, 136, 84, 191,
 94, 15, 141, 28, 145, 32, 138, 51,
 146, 155, 149, 36, 137, 24, 190, 167,
 154, 157, 147, 44, 169, 182, 120, 135,
 162, 165, 121, 134, 187, 108, 168, 183,
 118, 173, 23, 124, 153, 170, 40, 59,
 178, 113, 131, 88, 181, 158, 68, 151,
 186, 163, 89, 112, 189, 100, 150, 159};
constexpr int kHilbertPairs = 24 * 64;
// pairs[state * 64 + two octants] = two index digits | next state << 6, built by the block from kHilbertTable
__device__ inline void hilbert_pairs(uint16_t* pairs, int tid, int nt) {
    for (int i = tid; i < kHilbertPairs; i += nt) {
        const uint32_t e1 = kHilbertTable[(i >> 6) * 8 + ((i >> 3) & 7)];
        const uint32_t e2 = kHilbertTable[(e1 >> 3) * 8 + (i & 7)];
        pairs[i] = (uint16_t)(((e1 & 7u) << 3) | (e2 & 7u) | ((e2 >> 3) << 6));
    }
}
__device__ inline uint32_t hilbert24(uint32_t m, const uint16_t* pairs) {
    uint32_t st = 0, h = 0;
#pragma unroll
    for (int L = 3; L >= 0; --L) {
        const uint32_t e = pairs[st * 64 + ((m >> (6 * L)) & 63u)];
        h = (h << 6) | (e & 63u);
        st = e >> 6;
    }
    return h;
}
constexpr int kQsItems = 16;
// Most chunk sums a scatter block scans itself (scan_chunks; at most 2 per thread), else the recursive scan.  Each
// block pays for loading and scanning them, so only small sorts fold: C3 12.5M rows (48 sums) 0.278 -> 0.267 ms per
// sort, 100M rows (382 sums) 1.95 -> 2.00 ms (profiles/r05_ab_sort_scan_fold.jsonl; 16384-key tiles then); with
// 8192-key tiles 128 sums = 16.8M rows.
#ifndef MSH_QSORT_FOLD_MAX
#define MSH_QSORT_FOLD_MAX 128
#endif
constexpr unsigned kQsMaxSums = MSH_QSORT_FOLD_MAX;
static_assert(kQsMaxSums <= 2 * MSH_QSORT_NT, "tile_offset scans 2 sums per thread");

// Global start of (digit tid, this tile) for the first 256 threads.  With nsums == 0 offs holds the full exclusive
// scan; otherwise offs holds scans local to 4096-entry chunks and sums the chunk totals, whose exclusive prefix the
// block forms in LDS (sp, free until the tile is staged) -- the scan's recursive launches folded into the consumer.
// Ends with a barrier (the caller's LDS zeroing is complete after it).
template <int NT>
__device__ inline uint32_t tile_offset(const uint32_t* __restrict__ offs, unsigned nb, const uint32_t* __restrict__ sums,
                                       unsigned nsums, uint32_t* sp) {
    constexpr int NW = NT / 64;
    __shared__ uint32_t wsum[NW];
    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
    const size_t idx = (size_t)tid * nb + blockIdx.x;
    uint32_t g = tid < 256 ? offs[idx] : 0u;
    if (nsums == 0) {
        __syncthreads();
        return g;
    }
    const unsigned j = 2u * (unsigned)tid;
    const uint32_t a = j < nsums ? sums[j] : 0u, b = j + 1 < nsums ? sums[j + 1] : 0u;
    const uint32_t x = a + b;
    uint32_t incl = x;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(incl, o, 64);
        if (lane >= o) incl += y;
    }
    if (lane == 63) wsum[w] = incl;
    __syncthreads();
    uint32_t ex = incl - x;
    for (int k = 0; k < w; ++k) ex += wsum[k];
    if (j < nsums) sp[j] = ex;
    if (j + 1 < nsums) sp[j + 1] = ex + a;
    __syncthreads();
    if (tid < 256) g += sp[idx / (size_t)kSortTile];
    __syncthreads();
    return g;
}
constexpr int kQsTile = kQsNT * kQsItems;

template <int NT, int ITEMS>
__global__ __launch_bounds__(NT) void k_qkeys(const double* __restrict__ q, size_t n, int lo_bit, float lx, float ly,
                                              float lz, float hx, float hy, float hz, uint32_t* __restrict__ keys,
                                              uint32_t* __restrict__ hist, unsigned nb) {
    constexpr int NW = NT / 64;
    __shared__ uint32_t h[NW][256];
    __shared__ uint16_t pairs[MSH_QORDER_HILBERT ? kHilbertPairs : 1];
    const int tid = threadIdx.x, w = tid >> 6;
    for (int i = tid; i < NW * 256; i += NT) (&h[0][0])[i] = 0;
    if (MSH_QORDER_HILBERT) hilbert_pairs(pairs, tid, NT);
    __syncthreads();
    const size_t base = (size_t)blockIdx.x * (NT * ITEMS);
#pragma unroll 4
    for (int k = 0; k < ITEMS; ++k) {
        const size_t i = base + (size_t)k * NT + tid;
        if (i < n) {
            uint32_t key = query_morton30(q[3 * i], q[3 * i + 1], q[3 * i + 2], lx, ly, lz, hx, hy, hz) >> lo_bit;
            if (MSH_QORDER_HILBERT) key = hilbert24(key, pairs);  // the same 256^3 cells (lo_bit == 6), Hilbert order
            keys[i] = key;
            atomicAdd(&h[w][key & 255u], 1u);
        }
    }
    __syncthreads();
    for (int d = tid; d < 256; d += NT) {
        uint32_t c = 0;
#pragma unroll
        for (int x = 0; x < NW; ++x) c += h[x][d];
        hist[(size_t)d * nb + blockIdx.x] = c;
    }
}

template <int NT, int ITEMS>
__global__ __launch_bounds__(NT) void k_qhist64(const unsigned long long* __restrict__ in, size_t n, int shift,
                                                uint32_t* __restrict__ hist, unsigned nb) {
    constexpr int NW = NT / 64;
    __shared__ uint32_t h[NW][256];
    const int tid = threadIdx.x, w = tid >> 6;
    for (int i = tid; i < NW * 256; i += NT) (&h[0][0])[i] = 0;
    __syncthreads();
    const size_t base = (size_t)blockIdx.x * (NT * ITEMS);
    unsigned long long e[ITEMS];
#pragma unroll
    for (int k = 0; k < ITEMS; ++k) {
        const size_t i = base + (size_t)k * NT + tid;
        e[k] = i < n ? in[i] : ~0ull;
    }
#pragma unroll
    for (int k = 0; k < ITEMS; ++k)
        if (e[k] != ~0ull) atomicAdd(&h[w][(uint32_t)(e[k] >> (32 + shift)) & 255u], 1u);
    __syncthreads();
    for (int d = tid; d < 256; d += NT) {
        uint32_t c = 0;
#pragma unroll
        for (int x = 0; x < NW; ++x) c += h[x][d];
        hist[(size_t)d * nb + blockIdx.x] = c;
    }
}

// One stable pass on digit (key >> shift) & 255.  IN64: packed input, else u32 keys whose row is the index.
// OUT64: packed output, else the rows only.  Ranking as k_scatter: eight ballots per element give its rank among
// the wave's equal digits; per-wave digit counts are scanned over the block, the tile is staged in LDS in its
// sorted order and written out linearly (each digit run of the tile contiguous).
template <int NT, int ITEMS, bool IN64, bool OUT64>
__global__ __launch_bounds__(NT) void k_qscatter(const void* __restrict__ in, void* __restrict__ out, size_t n, int shift,
                                                 const uint32_t* __restrict__ offs, unsigned nb,
                                                 const uint32_t* __restrict__ sums, unsigned nsums) {
    constexpr int NW = NT / 64, TILE = NT * ITEMS, WI = 64 * ITEMS;
    static_assert(NT >= 256, "one thread per digit");
    __shared__ uint32_t wcnt[NW][256];
    __shared__ uint32_t gbase[256];
    __shared__ uint32_t ssum[4];
    __shared__ unsigned long long stage[TILE];
    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
    for (int i = tid; i < NW * 256; i += NT) (&wcnt[0][0])[i] = 0;
    const size_t tile0 = (size_t)blockIdx.x * TILE;
    const size_t base = tile0 + (size_t)w * WI;
    const unsigned long long lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    const unsigned long long* in64 = static_cast<const unsigned long long*>(in);
    const uint32_t* in32 = static_cast<const uint32_t*>(in);
    unsigned long long ee[ITEMS];
    uint32_t rr[ITEMS];
#pragma unroll
    for (int it = 0; it < ITEMS; ++it) {
        const size_t i = base + (size_t)it * 64 + lane;
        ee[it] = i < n ? (IN64 ? in64[i] : (((unsigned long long)in32[i] << 32) | (uint32_t)i)) : 0ull;
    }
    // after the tile's loads are issued, so the offsets' loads and scan overlap them (its barriers also order
    // the counters' zeroing before the ranking)
    const uint32_t g_off = tile_offset<NT>(offs, nb, sums, nsums, reinterpret_cast<uint32_t*>(stage));
#pragma unroll
    for (int it = 0; it < ITEMS; ++it) {
        const size_t i = base + (size_t)it * 64 + lane;
        const bool valid = i < n;
        const uint32_t d = (uint32_t)(ee[it] >> (32 + shift)) & 255u;
        unsigned long long peers = __ballot(valid);
#pragma unroll
        for (int b = 0; b < 8; ++b) {
            const bool bit = (d >> b) & 1u;
            const unsigned long long m = __ballot(bit);
            peers &= bit ? m : ~m;
        }
        const uint32_t prev = valid ? wcnt[w][d] : 0u;
        if (valid && (peers & lt) == 0ull) wcnt[w][d] = prev + (uint32_t)__popcll(peers);
        rr[it] = prev + (uint32_t)__popcll(peers & lt);
    }
    __syncthreads();
    // digit tid (< 256): the tile's count, its exclusive scan over the digits, then each wave's start inside the run
    uint32_t tot = 0;
    if (tid < 256) {
#pragma unroll
        for (int x = 0; x < NW; ++x) tot += wcnt[x][tid];
    }
    uint32_t incl = tot;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(incl, o, 64);
        if (lane >= o) incl += y;
    }
    if (w < 4 && lane == 63) ssum[w] = incl;
    __syncthreads();
    if (tid < 256) {
        uint32_t run = incl - tot;
        for (int k = 0; k < w; ++k) run += ssum[k];
        gbase[tid] = g_off - run;
#pragma unroll
        for (int x = 0; x < NW; ++x) {
            const uint32_t c = wcnt[x][tid];
            wcnt[x][tid] = run;
            run += c;
        }
    }
    __syncthreads();
#pragma unroll
    for (int it = 0; it < ITEMS; ++it) {
        const size_t i = base + (size_t)it * 64 + lane;
        if (i < n) stage[wcnt[w][(uint32_t)(ee[it] >> (32 + shift)) & 255u] + rr[it]] = ee[it];
    }
    __syncthreads();
    const uint32_t tn = (uint32_t)(n - tile0 < (size_t)TILE ? n - tile0 : (size_t)TILE);
    for (uint32_t p = tid; p < tn; p += NT) {
        const unsigned long long e = stage[p];
        const uint32_t dst = gbase[(uint32_t)(e >> (32 + shift)) & 255u] + p;
        if (OUT64) static_cast<unsigned long long*>(out)[dst] = e;
        else static_cast<uint32_t*>(out)[dst] = (uint32_t)e;
    }
}

// Split-array form of the middle passes (MSH_QSORT_SPLIT): keys and rows in two u32 arrays, so a histogram pass
// reads 4 B per element instead of the packed 8 B (a digit run of an 8192-key tile averages 128 B per array).
template <int NT, int ITEMS>
__global__ __launch_bounds__(NT) void k_qhist32(const uint32_t* __restrict__ keys, size_t n, int shift,
                                                uint32_t* __restrict__ hist, unsigned nb) {
    constexpr int NW = NT / 64;
    __shared__ uint32_t h[NW][256];
    const int tid = threadIdx.x, w = tid >> 6;
    for (int i = tid; i < NW * 256; i += NT) (&h[0][0])[i] = 0;
    __syncthreads();
    const size_t base = (size_t)blockIdx.x * (NT * ITEMS);
    uint32_t e[ITEMS];
#pragma unroll
    for (int k = 0; k < ITEMS; ++k) {
        const size_t i = base + (size_t)k * NT + tid;
        e[k] = i < n ? keys[i] : 0xFFFFFFFFu;
    }
#pragma unroll
    for (int k = 0; k < ITEMS; ++k)
        if (e[k] != 0xFFFFFFFFu) atomicAdd(&h[w][(e[k] >> shift) & 255u], 1u);
    __syncthreads();
    for (int d = tid; d < 256; d += NT) {
        uint32_t c = 0;
#pragma unroll
        for (int x = 0; x < NW; ++x) c += h[x][d];
        hist[(size_t)d * nb + blockIdx.x] = c;
    }
}

// ROWS_IN: rows from rin (else the index); KEYS_OUT: keys written to kout (else the rows only).  Staged and ranked as
// k_qscatter.
template <int NT, int ITEMS, bool ROWS_IN, bool KEYS_OUT>
__global__ __launch_bounds__(NT) void k_qscatter2(const uint32_t* __restrict__ kin, const uint32_t* __restrict__ rin,
                                                  uint32_t* __restrict__ kout, uint32_t* __restrict__ rout, size_t n,
                                                  int shift, const uint32_t* __restrict__ offs, unsigned nb,
                                                  const uint32_t* __restrict__ sums, unsigned nsums) {
    constexpr int NW = NT / 64, TILE = NT * ITEMS, WI = 64 * ITEMS;
    static_assert(NT >= 256, "one thread per digit");
    __shared__ uint32_t wcnt[NW][256];
    __shared__ uint32_t gbase[256];
    __shared__ uint32_t ssum[4];
    __shared__ unsigned long long stage[TILE];
    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
    for (int i = tid; i < NW * 256; i += NT) (&wcnt[0][0])[i] = 0;
    const size_t tile0 = (size_t)blockIdx.x * TILE;
    const size_t base = tile0 + (size_t)w * WI;
    const unsigned long long lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    unsigned long long ee[ITEMS];
    uint32_t rr[ITEMS];
#pragma unroll
    for (int it = 0; it < ITEMS; ++it) {
        const size_t i = base + (size_t)it * 64 + lane;
        ee[it] = i < n ? (((unsigned long long)kin[i] << 32) | (ROWS_IN ? rin[i] : (uint32_t)i)) : 0ull;
    }
    // after the tile's loads are issued, so the offsets' loads and scan overlap them (its barriers also order
    // the counters' zeroing before the ranking)
    const uint32_t g_off = tile_offset<NT>(offs, nb, sums, nsums, reinterpret_cast<uint32_t*>(stage));
#pragma unroll
    for (int it = 0; it < ITEMS; ++it) {
        const size_t i = base + (size_t)it * 64 + lane;
        const bool valid = i < n;
        const uint32_t d = (uint32_t)(ee[it] >> (32 + shift)) & 255u;
        unsigned long long peers = __ballot(valid);
#pragma unroll
        for (int b = 0; b < 8; ++b) {
            const bool bit = (d >> b) & 1u;
            const unsigned long long m = __ballot(bit);
            peers &= bit ? m : ~m;
        }
        const uint32_t prev = valid ? wcnt[w][d] : 0u;
        if (valid && (peers & lt) == 0ull) wcnt[w][d] = prev + (uint32_t)__popcll(peers);
        rr[it] = prev + (uint32_t)__popcll(peers & lt);
    }
    __syncthreads();
    uint32_t tot = 0;
    if (tid < 256) {
#pragma unroll
        for (int x = 0; x < NW; ++x) tot += wcnt[x][tid];
    }
    uint32_t incl = tot;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(incl, o, 64);
        if (lane >= o) incl += y;
    }
    if (w < 4 && lane == 63) ssum[w] = incl;
    __syncthreads();
    if (tid < 256) {
        uint32_t run = incl - tot;
        for (int k = 0; k < w; ++k) run += ssum[k];
        gbase[tid] = g_off - run;
#pragma unroll
        for (int x = 0; x < NW; ++x) {
            const uint32_t c = wcnt[x][tid];
            wcnt[x][tid] = run;
            run += c;
        }
    }
    __syncthreads();
#pragma unroll
    for (int it = 0; it < ITEMS; ++it) {
        const size_t i = base + (size_t)it * 64 + lane;
        if (i < n) stage[wcnt[w][(uint32_t)(ee[it] >> (32 + shift)) & 255u] + rr[it]] = ee[it];
    }
    __syncthreads();
    const uint32_t tn = (uint32_t)(n - tile0 < (size_t)TILE ? n - tile0 : (size_t)TILE);
    for (uint32_t p = tid; p < tn; p += NT) {
        const unsigned long long e = stage[p];
        const uint32_t dst = gbase[(uint32_t)(e >> (32 + shift)) & 255u] + p;
        if (KEYS_OUT) kout[dst] = (uint32_t)(e >> 32);
        rout[dst] = (uint32_t)e;
    }
}

#ifndef MSH_QSORT_SPLIT
#define MSH_QSORT_SPLIT 1
#endif

int query_sort(const float* lo, const float* hi, const double* d_q, size_t S, int lo_bit, Workspace& ws, hipStream_t s) {
    if (S == 0) return MSH_OK;
    if (S > 0xFFFFFFFFull || lo_bit < 6) {
        set_error("query sort: %zu rows (at most 2^32 - 1) on Morton bits from %d (keys of at most 24 bits)", S, lo_bit);
        return MSH_EINVAL;
    }
    const unsigned nb = (unsigned)((S + kQsTile - 1) / kQsTile);
    MSH_TRY(ws.keys.reserve(S * sizeof(uint32_t)));
    MSH_TRY(ws.vals.reserve(S * sizeof(uint32_t)));
    MSH_TRY(ws.keys_alt.reserve(S * sizeof(unsigned long long)));
    MSH_TRY(ws.vals_alt.reserve(S * sizeof(unsigned long long)));
    MSH_TRY(ws.hist.reserve((size_t)nb * 256 * sizeof(uint32_t)));
    uint32_t* hist = ws.hist.as<uint32_t>();
    unsigned long long* A = ws.keys_alt.as<unsigned long long>();
    unsigned long long* B = ws.vals_alt.as<unsigned long long>();
    {
        TimedLaunch tl("morton", s);
        k_qkeys<kQsNT, kQsItems><<<nb, kQsNT, 0, s>>>(d_q, S, lo_bit, lo[0], lo[1], lo[2], hi[0], hi[1], hi[2],
                                                     ws.keys.as<uint32_t>(), hist, nb);
        MSH_HIP(hipGetLastError());
    }
    TimedLaunch tl("sort", s);
    const uint32_t* sums;
    unsigned nsums;
    MSH_TRY(scan_chunks(hist, (size_t)nb * 256, ws, s, &sums, &nsums, kQsMaxSums));
    if (MSH_QSORT_SPLIT) {
        uint32_t* k0 = ws.keys.as<uint32_t>();
        uint32_t* k1 = ws.keys_alt.as<uint32_t>();
        uint32_t* r1 = k1 + S;
        uint32_t* k2 = ws.vals_alt.as<uint32_t>();
        uint32_t* r2 = k2 + S;
        k_qscatter2<kQsNT, kQsItems, false, true><<<nb, kQsNT, 0, s>>>(k0, nullptr, k1, r1, S, 0, hist, nb, sums, nsums);
        MSH_HIP(hipGetLastError());
        k_qhist32<kQsNT, kQsItems><<<nb, kQsNT, 0, s>>>(k1, S, 8, hist, nb);
        MSH_HIP(hipGetLastError());
        MSH_TRY(scan_chunks(hist, (size_t)nb * 256, ws, s, &sums, &nsums, kQsMaxSums));
        k_qscatter2<kQsNT, kQsItems, true, true><<<nb, kQsNT, 0, s>>>(k1, r1, k2, r2, S, 8, hist, nb, sums, nsums);
        MSH_HIP(hipGetLastError());
        k_qhist32<kQsNT, kQsItems><<<nb, kQsNT, 0, s>>>(k2, S, 16, hist, nb);
        MSH_HIP(hipGetLastError());
        MSH_TRY(scan_chunks(hist, (size_t)nb * 256, ws, s, &sums, &nsums, kQsMaxSums));
        k_qscatter2<kQsNT, kQsItems, true, false><<<nb, kQsNT, 0, s>>>(k2, r2, nullptr, ws.vals.as<uint32_t>(), S, 16,
                                                                        hist, nb, sums, nsums);
        MSH_HIP(hipGetLastError());
        return MSH_OK;
    }
    k_qscatter<kQsNT, kQsItems, false, true><<<nb, kQsNT, 0, s>>>(ws.keys.ptr, A, S, 0, hist, nb, sums, nsums);
    MSH_HIP(hipGetLastError());
    k_qhist64<kQsNT, kQsItems><<<nb, kQsNT, 0, s>>>(A, S, 8, hist, nb);
    MSH_HIP(hipGetLastError());
    MSH_TRY(scan_chunks(hist, (size_t)nb * 256, ws, s, &sums, &nsums, kQsMaxSums));
    k_qscatter<kQsNT, kQsItems, true, true><<<nb, kQsNT, 0, s>>>(A, B, S, 8, hist, nb, sums, nsums);
    MSH_HIP(hipGetLastError());
    k_qhist64<kQsNT, kQsItems><<<nb, kQsNT, 0, s>>>(B, S, 16, hist, nb);
    MSH_HIP(hipGetLastError());
    MSH_TRY(scan_chunks(hist, (size_t)nb * 256, ws, s, &sums, &nsums, kQsMaxSums));
    k_qscatter<kQsNT, kQsItems, true, false><<<nb, kQsNT, 0, s>>>(B, ws.vals.ptr, S, 16, hist, nb, sums, nsums);
    MSH_HIP(hipGetLastError());
    return MSH_OK;
}

}  // namespace msh
