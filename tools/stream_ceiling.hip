// stream_ceiling.hip -- measurement tool (not product code): the plain HBM
// read-stream rate of this MI355X, to put the checksum kernel's GB/s next to a
// measured ceiling as well as the 8 TB/s spec peak.  Each lane streams
// 16-byte loads (UNROLL in flight) and folds them into one word per thread.
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef const u32x4 __attribute__((address_space(1))) *gptr;

template <int UNROLL, bool NT>
__global__ void __launch_bounds__(256) k_read(const u32x4 *__restrict__ in,
                                              uint64_t n16, uint32_t *out)
{
    const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t nth = (uint64_t)gridDim.x * blockDim.x;
    gptr p = (gptr)in;
    uint32_t acc = 0;
    uint64_t i = tid;
    for (; i + (UNROLL - 1) * nth < n16; i += UNROLL * nth) {
        u32x4 v[UNROLL];
#pragma unroll
        for (int u = 0; u < UNROLL; ++u)
            v[u] = NT ? __builtin_nontemporal_load(p + i + u * nth) : p[i + u * nth];
#pragma unroll
        for (int u = 0; u < UNROLL; ++u)
            acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
    }
    for (; i < n16; i += nth) {
        u32x4 v = p[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u)
        out[tid] = acc; // practically never; keeps the loads live
}

extern "C" int stream_read(const void *buf, uint64_t bytes, int grid, int unroll,
                           int nt, void *out, void *stream)
{
    const uint64_t n16 = bytes / 16;
    hipStream_t st = (hipStream_t)stream;
#define L(U, N)                                                                \
    hipLaunchKernelGGL((k_read<U, N>), dim3(grid), dim3(256), 0, st,           \
                       (const u32x4 *)buf, n16, (uint32_t *)out)
    if (unroll == 1) { if (nt) L(1, true); else L(1, false); }
    else if (unroll == 2) { if (nt) L(2, true); else L(2, false); }
    else if (unroll == 4) { if (nt) L(4, true); else L(4, false); }
    else { if (nt) L(8, true); else L(8, false); }
#undef L
    return (int)hipGetLastError();
}
