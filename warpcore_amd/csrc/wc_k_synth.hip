// wc_k_synth.hip -- synthetic payload bytes on the device (bench / tests),
// and the shader-clock probe bench.py runs beside its timed legs.
#include "wc_device.h"

namespace wc {

// ---------------------------------------------------------------------------
// Synthetic bytes.

// splitmix64 output k for state `seed` (must match oracle_synth_fill).
__device__ __forceinline__ uint64_t splitmix64_at(uint64_t seed, uint64_t k)
{
    uint64_t z = seed + (k + 1ull) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__global__ void __launch_bounds__(256)
k_synth(uint8_t *__restrict__ buf, uint64_t nbytes, uint64_t seed)
{
    const uint64_t words = nbytes / 8;
    const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t nth = (uint64_t)gridDim.x * blockDim.x;
    // Two words (16 B) per thread per step; buf is 16-byte aligned by contract.
    for (uint64_t w = 2 * tid; w < words; w += 2 * nth) {
        if (w + 1 < words) {
            uint64_t v[2] = {splitmix64_at(seed, w), splitmix64_at(seed, w + 1)};
            *reinterpret_cast<u32x4 *>(buf + 8 * w) = *reinterpret_cast<const u32x4 *>(v);
        } else {
            *reinterpret_cast<uint64_t *>(buf + 8 * w) = splitmix64_at(seed, w);
        }
    }
    if (tid == 0 && (nbytes & 7u)) {
        const uint64_t v = splitmix64_at(seed, words);
        for (uint32_t b = 0; b < (nbytes & 7u); ++b)
            buf[8 * words + b] = (uint8_t)(v >> (8 * b));
    }
}

hipError_t launch_synth(void *buf, uint64_t nbytes, uint64_t seed, int grid, hipStream_t st)
{
    hipLaunchKernelGGL(k_synth, dim3(grid), dim3(256), 0, st, (uint8_t *)buf, nbytes, seed);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Shader-clock probe.  One wave, beside a workload on another stream: lane 0
// records n pairs (the 100-MHz constant wall clock, the shader clock
// counter) every `interval` wall ticks; the ratio of successive deltas is
// the shader clock while the workload ran (DVFS moves it between ~1.5 and
// ~2.4 GHz on MI355X, and clock-sensitive kernels move with it; DESIGN.md
// section 5.1).  It always ends after n samples.
__global__ void __launch_bounds__(64) k_sclk_probe(uint64_t *__restrict__ out, int n,
                                                   uint64_t interval)
{
    if (threadIdx.x != 0)
        return;
    for (int i = 0; i < n; ++i) {
        const uint64_t t0 = wall_clock64();
        while (wall_clock64() - t0 < interval)
            __builtin_amdgcn_s_sleep(1);
        const uint64_t w = wall_clock64(), c = clock64();
        out[2 * i] = w;
        out[2 * i + 1] = c;
    }
}

hipError_t launch_sclk_probe(uint64_t *out, int n, uint64_t interval, hipStream_t st)
{
    hipLaunchKernelGGL(k_sclk_probe, dim3(1), dim3(64), 0, st, out, n, interval);
    return hipGetLastError();
}

} // namespace wc
