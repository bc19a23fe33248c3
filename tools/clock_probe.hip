// clock_probe.hip -- a one-wave sampler of the shader clock (tools only).
// Launched on its own stream beside a workload, lane 0 records pairs
// (s_memrealtime: the 100 MHz constant wall clock, s_memtime: the shader
// clock counter) every `interval` wall ticks for `n` samples; the ratio of
// their deltas is the shader clock while the workload ran.  Bounded: it
// always ends after n samples.
#include <hip/hip_runtime.h>
#include <stdint.h>

extern "C" __global__ void k_clock_probe(uint64_t *out, int n, uint64_t interval)
{
    if (threadIdx.x != 0)
        return;
    for (int i = 0; i < n; ++i) {
        const uint64_t t0 = wall_clock64();
        while (wall_clock64() - t0 < interval)
            __builtin_amdgcn_s_sleep(1);
        out[2 * i] = wall_clock64();
        out[2 * i + 1] = clock64();
    }
}

extern "C" int clock_probe_launch(uint64_t *out, int n, uint64_t interval, void *stream)
{
    hipLaunchKernelGGL(k_clock_probe, dim3(1), dim3(64), 0, (hipStream_t)stream, out, n,
                       interval);
    return (int)hipGetLastError();
}
