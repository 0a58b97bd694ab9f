// Where does global_load_lds_dwordx4 with an immediate offset write in LDS?  One wave: lane l loads the 16 B at
// src + 64 l + 16 (instruction offset 16 applied to the global address) with the LDS base at byte 256 of a zeroed
// 4 KB buffer; the LDS image is copied out and the host prints the byte offset where lane 0's 16 B landed
// (256 + 16 if the offset also moves the LDS destination, 256 if it does not).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__global__ void k(const uint32_t* src, uint32_t* out) {
    __shared__ uint32_t buf[1024];
    for (int i = threadIdx.x; i < 1024; i += 64) buf[i] = 0;
    __syncthreads();
    typedef __attribute__((address_space(3))) void* LP;
    __builtin_amdgcn_global_load_lds(src + 16 * threadIdx.x, (LP)(buf + 64), 16, 16, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int i = threadIdx.x; i < 1024; i += 64) out[i] = buf[i];
}

int main() {
    uint32_t h[64 * 16 + 64];
    for (int i = 0; i < 64 * 16 + 64; ++i) h[i] = 0x10000u + i;
    uint32_t *ds, *dout;
    if (hipMalloc(&ds, sizeof(h)) != hipSuccess || hipMalloc(&dout, 4096) != hipSuccess) return 2;
    hipMemcpy(ds, h, sizeof(h), hipMemcpyHostToDevice);
    k<<<1, 64>>>(ds, dout);
    uint32_t o[1024];
    if (hipMemcpy(o, dout, 4096, hipMemcpyDeviceToHost) != hipSuccess) return 3;
    for (int i = 0; i < 1024; ++i)
        if (o[i] == 0x10000u + 4) { printf("lane 0's first word (src word 4) at LDS byte %d\n", 4 * i); break; }
    for (int i = 0; i < 1024; ++i)
        if (o[i] == 0x10000u + 16 + 4) { printf("lane 1's first word at LDS byte %d\n", 4 * i); break; }
    return 0;
}
