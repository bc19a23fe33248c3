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

// Slot-read ceiling (measurement only): the lines a netmap ring of mixed
// sizes touches -- packet i at base + i * stride + off, lens[i] bytes -- read
// with G lanes per packet and the cheapest addressing (no checksum, no owner
// lookup): each lane loads chunks k, k + G, ... of its packet's aligned chunk
// range, two loads in flight per step.
template <int G, bool NT>
__global__ void __launch_bounds__(256) k_slot_read(const uint8_t *__restrict__ base,
                                                   uint64_t stride, uint32_t off,
                                                   const uint16_t *__restrict__ lens,
                                                   uint64_t n, uint32_t *out)
{
    const uint64_t gid = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) / G;
    const uint64_t ngr = (uint64_t)gridDim.x * blockDim.x / G;
    const uint32_t k = threadIdx.x % G;
    uint32_t acc = 0;
    for (uint64_t p = gid; p < n; p += ngr) {
        const uint64_t a = (uint64_t)base + p * stride + off;
        const uint64_t c0 = a & ~15ull;
        const uint32_t nch = (uint32_t)((a & 15u) + lens[p] + 15u) >> 4;
        for (uint32_t c = k; c < nch; c += 2 * G) {
            const uint32_t c2 = min(c + G, nch - 1u);
            gptr q0 = (gptr)(uintptr_t)(c0 + 16ull * c), q1 = (gptr)(uintptr_t)(c0 + 16ull * c2);
            u32x4 v0 = NT ? __builtin_nontemporal_load(q0) : *q0;
            u32x4 v1 = NT ? __builtin_nontemporal_load(q1) : *q1;
            acc ^= v0.x ^ v0.y ^ v1.z ^ v1.w;
        }
    }
    if (acc == 0x12345678u)
        out[threadIdx.x] = acc;
}

extern "C" int slot_read(const void *base, uint64_t stride, uint32_t off, const void *lens,
                         uint64_t n, int group, int grid, int nt, void *out, void *stream)
{
    hipStream_t st = (hipStream_t)stream;
#define S(GG, N)                                                               \
    hipLaunchKernelGGL((k_slot_read<GG, N>), dim3(grid), dim3(256), 0, st,     \
                       (const uint8_t *)base, stride, off, (const uint16_t *)lens, n, \
                       (uint32_t *)out)
    if (group == 4) { if (nt) S(4, true); else S(4, false); }
    else if (group == 8) { if (nt) S(8, true); else S(8, false); }
    else if (group == 16) { if (nt) S(16, true); else S(16, false); }
    else { if (nt) S(32, true); else S(32, false); }
#undef S
    return (int)hipGetLastError();
}

// Tile-read probe (measurement only): does the checksum's ragged tile
// structure -- each wave streaming its own contiguous region of R bytes in
// 1-KiB rows, 4-row groups ping-ponged -- cost HBM rate by itself?
//   mode 0: wave w reads region w (the seg kernel's layout: the resident
//           waves' streams are R bytes apart);
//   mode 1: the 4 waves of a block interleave their rows over the block's
//           4 regions (the block streams one contiguous range).
template <int GR>
__global__ void __launch_bounds__(256) k_tile_read(const uint8_t *__restrict__ base,
                                                   uint64_t region, uint64_t nregions, int mode,
                                                   uint32_t *out)
{
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint64_t reg = (uint64_t)blockIdx.x * 4 + w;
    if (reg >= nregions)
        return;
    const uint64_t rows = region / 1024;
    uint32_t acc = 0;
    for (uint64_t r = 0; r < rows; r += GR) {
        u32x4 v[GR];
#pragma unroll
        for (int u = 0; u < GR; ++u) {
            const uint64_t row = r + u;
            uint64_t off;
            if (mode == 0)
                off = reg * region + row * 1024;
            else // block-interleaved: global row index within the block's 4 regions
                off = (uint64_t)blockIdx.x * 4 * region + (row * 4 + w) * 1024;
            gptr q = (gptr)(uintptr_t)(base + off + 16 * lane);
            v[u] = __builtin_nontemporal_load(q);
        }
#pragma unroll
        for (int u = 0; u < GR; ++u)
            acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
    }
    if (acc == 0x12345678u)
        out[threadIdx.x] = acc;
}

extern "C" int tile_read(const void *base, uint64_t bytes, uint64_t region, int mode, int rows,
                         void *out, void *stream)
{
    const uint64_t nreg = bytes / region;
    const int grid = (int)((nreg + 3) / 4);
    hipStream_t st = (hipStream_t)stream;
    if (rows == 8)
        hipLaunchKernelGGL((k_tile_read<8>), dim3(grid), dim3(256), 0, st, (const uint8_t *)base,
                           region, nreg, mode, (uint32_t *)out);
    else
        hipLaunchKernelGGL((k_tile_read<4>), dim3(grid), dim3(256), 0, st, (const uint8_t *)base,
                           region, nreg, mode, (uint32_t *)out);
    return (int)hipGetLastError();
}

// Line-read ceiling (measurement only): exactly the
// 128-B lines a set of byte ranges touches -- a netmap ring's frames in their
// 2048-B slots -- each read once with nontemporal 16-B loads, 8 lanes per
// line, U lines in flight per 8-lane group, one-shot grid.  The only other
// traffic is the line list itself (a uint32 line index per 128-B line, 3 %).
// No arithmetic beyond keeping the loads live: the fastest any kernel can
// pull those lines through the memory system.
template <int U>
__global__ void __launch_bounds__(256) k_line_read(const uint8_t *__restrict__ base,
                                                   const uint32_t *__restrict__ lines,
                                                   uint64_t nlines, uint32_t *out)
{
    const uint64_t g0 = (uint64_t)blockIdx.x * 32u * U + (threadIdx.x >> 3);
    const uint32_t c = threadIdx.x & 7u;
    u32x4 v[U];
    uint32_t li[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const uint64_t l = g0 + 32u * u;
        li[u] = l < nlines ? lines[l] : 0xFFFFFFFFu;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const uint64_t a = (uint64_t)(li[u] == 0xFFFFFFFFu ? 0u : li[u]) * 128u + 16u * c;
        v[u] = __builtin_nontemporal_load((gptr)(uintptr_t)(base + a));
    }
    uint32_t acc = 0;
#pragma unroll
    for (int u = 0; u < U; ++u)
        acc ^= li[u] == 0xFFFFFFFFu ? 0u : (v[u].x ^ v[u].y ^ v[u].z ^ v[u].w);
    if (acc == 0x12345678u)
        out[threadIdx.x] = acc;
}

extern "C" int line_read(const void *base, const void *lines, uint64_t nlines, int unroll,
                         void *out, void *stream)
{
    hipStream_t st = (hipStream_t)stream;
    const uint64_t per_block = 32ull * (uint64_t)unroll;
    const int grid = (int)((nlines + per_block - 1) / per_block);
#define LR(U)                                                                  \
    hipLaunchKernelGGL((k_line_read<U>), dim3(grid), dim3(256), 0, st, (const uint8_t *)base, \
                       (const uint32_t *)lines, nlines, (uint32_t *)out)
    if (unroll == 1) LR(1);
    else if (unroll == 2) LR(2);
    else if (unroll == 4) LR(4);
    else LR(8);
#undef LR
    return (int)hipGetLastError();
}
