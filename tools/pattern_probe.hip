// pattern_probe.hip -- measurement tool (not product code): HBM read rate of
// global_load_dwordx4 under the lane patterns a chunk-dealing kernel can use.
// Each wave reads one block of 64*K consecutive 16-byte chunks as K load
// instructions; within the block, lane l's k-th chunk is
//     ((l / W) * K + k) * W + (l % W)
// i.e. W-lane groups each own K*W consecutive chunks.  W = 64 is the fully
// coalesced row pattern (flat / seg kernels); W = 1 gives every lane K
// consecutive chunks (a 16*K-byte segment per lane, stride 16*K between
// lanes within one instruction).  One-shot grid, 256-thread blocks.
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef const u32x4 __attribute__((address_space(1))) *gptr;

template <int W, int K>
__global__ void __launch_bounds__(256) k_probe(const u32x4 *__restrict__ in, uint64_t nblk,
                                               uint32_t *out, uint32_t shift)
{
    const int lane = threadIdx.x & 63;
    const uint64_t wave = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (wave >= nblk)
        return;
    // shift (in chunks) moves every wave's block off its 64 / 128-byte
    // alignment: each W-lane segment then straddles cache lines.
    gptr p = (gptr)in + wave * 64 * K + shift;
    const int q = lane / W, gl = lane % W;
    u32x4 v[K];
#pragma unroll
    for (int k = 0; k < K; ++k)
        v[k] = __builtin_nontemporal_load(p + (q * K + k) * W + gl);
    uint32_t acc = 0;
#pragma unroll
    for (int k = 0; k < K; ++k)
        acc += v[k].x + v[k].y + v[k].z + v[k].w;
    if (acc == 0x12345678u)
        out[lane] = acc;
}

extern "C" int probe_read(const void *buf, uint64_t bytes, int w, int k, void *out,
                          void *stream, int shift)
{
    const uint64_t nblk = bytes / (1024ull * k) - 1; // room for the shift
    const int grid = (int)((nblk + 3) / 4);
    hipStream_t st = (hipStream_t)stream;
#define L(W_, K_)                                                              \
    if (w == W_ && k == K_) {                                                  \
        hipLaunchKernelGGL((k_probe<W_, K_>), dim3(grid), dim3(256), 0, st,    \
                           (const u32x4 *)buf, nblk, (uint32_t *)out, (uint32_t)shift);         \
        return (int)hipGetLastError();                                         \
    }
    L(64, 4) L(16, 4) L(8, 4) L(4, 4) L(2, 4) L(1, 4) L(8, 2) L(16, 2)
    L(64, 2) L(4, 2) L(1, 2) L(64, 8) L(4, 8) L(1, 8)
#undef L
    return -1;
}
