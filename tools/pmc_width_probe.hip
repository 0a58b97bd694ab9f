// What do rocprofv3's FETCH_SIZE and WRITE_SIZE report on gfx950 for loads and stores of 4, 8 and 16 B per lane?
// MI355X_MICROARCH.md calibrates only 16-B-per-lane streams.  Six kernels each move 512 MB of a buffer far larger than
// the Infinity Cache, coalesced (lane l of a wave touches consecutive elements): k_ld<W> reads it (one store per
// block keeps the loads alive), k_st<W> writes it; plus the traversal's pattern, k_st_scatter<W>: one W-byte store
// per lane (W = 4, 8) to a random row of a 24-B-per-row table (as k_knn stores a row's face, part and point).  Run under
// `rocprofv3 --pmc FETCH_SIZE` and `--pmc WRITE_SIZE` (separate passes); scripts/pmc_width_probe.sh prints the
// counter bytes over the bytes moved per kernel.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

constexpr size_t kBytes = (size_t)512 << 20;

template <int W>
struct Vec;
template <>
struct Vec<4> { typedef uint32_t T; };
template <>
struct Vec<8> { typedef uint2 T; };
template <>
struct Vec<16> { typedef uint4 T; };

template <int W>
__global__ void k_ld(const typename Vec<W>::T* __restrict__ a, size_t n, uint32_t* __restrict__ sink) {
    uint32_t acc = 0;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const typename Vec<W>::T v = a[i];
        acc ^= reinterpret_cast<const uint32_t*>(&v)[0];
    }
    if (acc == 0x9E3779B9u) sink[blockIdx.x] = acc;  // practically never: keeps the loads
}

template <int W>
__global__ void k_st(typename Vec<W>::T* __restrict__ a, size_t n) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        typename Vec<W>::T v;
        for (int k = 0; k < W / 4; ++k) reinterpret_cast<uint32_t*>(&v)[k] = (uint32_t)i;
        a[i] = v;
    }
}

// one W-B store per lane at a pseudo-random row (24-B rows) of a table of `rows` rows
template <int W>
__global__ void k_st_scatter(char* __restrict__ table, size_t rows, size_t n) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const size_t r = (i * 0x9E3779B97F4A7C15ull >> 17) % rows;
        typename Vec<W>::T v;
        for (int k = 0; k < W / 4; ++k) reinterpret_cast<uint32_t*>(&v)[k] = (uint32_t)i;
        *reinterpret_cast<typename Vec<W>::T*>(table + 24 * r + 8) = v;
    }
}

int main() {
    char *a = nullptr, *table = nullptr;
    uint32_t* sink = nullptr;
    const size_t rows = ((size_t)2 << 30) / 24;  // a 2 GB table
    if (hipMalloc(&a, kBytes) != hipSuccess || hipMalloc(&table, rows * 24) != hipSuccess ||
        hipMalloc(&sink, 1 << 20) != hipSuccess) {
        fprintf(stderr, "hipMalloc failed\n");
        return 2;
    }
    hipMemset(a, 1, kBytes);
    const int grid = 256 * 8, block = 256;
    // order of dispatches: ld4 ld8 ld16 st4 st8 st16 sc4 sc8
    k_ld<4><<<grid, block>>>(reinterpret_cast<const uint32_t*>(a), kBytes / 4, sink);
    k_ld<8><<<grid, block>>>(reinterpret_cast<const uint2*>(a), kBytes / 8, sink);
    k_ld<16><<<grid, block>>>(reinterpret_cast<const uint4*>(a), kBytes / 16, sink);
    k_st<4><<<grid, block>>>(reinterpret_cast<uint32_t*>(a), kBytes / 4);
    k_st<8><<<grid, block>>>(reinterpret_cast<uint2*>(a), kBytes / 8);
    k_st<16><<<grid, block>>>(reinterpret_cast<uint4*>(a), kBytes / 16);
    const size_t ns = (size_t)64 << 20;  // 64M scattered stores each
    k_st_scatter<4><<<grid, block>>>(table, rows, ns);
    k_st_scatter<8><<<grid, block>>>(table, rows, ns);
    if (hipDeviceSynchronize() != hipSuccess) {
        fprintf(stderr, "kernel failed\n");
        return 3;
    }
    printf("bytes per coalesced kernel %zu, scattered stores %zu of 4 / 8 B\n", kBytes, ns);
    hipFree(a);
    hipFree(table);
    hipFree(sink);
    return 0;
}
