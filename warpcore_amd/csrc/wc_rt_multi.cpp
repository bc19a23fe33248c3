// wc_rt_multi.cpp -- multi-GPU batches from one host thread (SURVEY.md
// 8(e)): an even contiguous packet split over the shard executors, no
// data-path collective; RCCL only for the optional result gather.

#include "wc_rt.h"
#include "wc_rccl.h"

#include <algorithm>

namespace wc {
namespace rt __attribute__((visibility("hidden"))) {

// Run fn(g) for every shard with its device current; the caller's device is
// restored.  Snapshot of the shard devices taken under the lock (the batch
// calls take it themselves).
template <class F>
int for_each_shard(F &&fn)
{
    int devs[kMaxDevices];
    int G = 0;
    {
        std::lock_guard<FairMutex> lk(g_mu);
        G = g_multi_n;
        for (int g = 0; g < G; ++g)
            devs[g] = g_shard[g].dev;
    }
    if (G == 0)
        return WC_EINVAL; // wc_gpu_init_multi first
    int cur = 0;
    if (hipGetDevice(&cur) != hipSuccess)
        return WC_ENODEV;
    int rc = WC_OK;
    for (int g = 0; g < G && rc == WC_OK; ++g) {
        rc = hip_err(hipSetDevice(devs[g]));
        if (rc == WC_OK)
            rc = fn(g);
    }
    (void)hipSetDevice(cur);
    return rc;
}

} // namespace rt
} // namespace wc

using namespace wc::rt;

extern "C" {

// ---------------------------------------------------------------------------
// Multi-GPU: an even contiguous packet split over the shard
// executors, no data-path collective; RCCL only for the optional result
// gather.

int wc_shard_range(uint64_t n, int g, int ngpus, uint64_t *lo, uint64_t *hi)
{
    if (ngpus < 1 || g < 0 || g >= ngpus || !lo || !hi)
        return WC_EINVAL;
    shard_range(n, g, ngpus, lo, hi);
    return WC_OK;
}

int wc_gpu_init_multi(int ngpus, const int *devices)
{
    std::lock_guard<FairMutex> lk(g_mu);
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0)
        return WC_ENODEV;
    if (ngpus <= 0) {
        if (devices)
            return WC_EINVAL;
        ngpus = ndev;
    }
    if (ngpus > kMaxDevices)
        return WC_EINVAL;
    int devs[kMaxDevices];
    for (int g = 0; g < ngpus; ++g) {
        devs[g] = devices ? devices[g] : g;
        if (devs[g] < 0 || devs[g] >= ndev || devs[g] >= kMaxDevices)
            return WC_EINVAL;
    }
    int cur = 0;
    if (hipGetDevice(&cur) != hipSuccess)
        return WC_ENODEV;
    // A new shard set replaces the old one (its pipelines and communicators).
    wc::rccl_fini();
    for (int g = 0; g < g_multi_n; ++g) {
        (void)hipSetDevice(g_shard[g].dev);
        pipe_free(g_shard[g].pipe);
        g_shard[g] = ShardExec{};
    }
    g_multi_n = 0;
    // All or nothing: a shard that fails to come up (its device's scratch or
    // its pipeline) tears down the ones built before it, so a later
    // wc_cksum_host_multi never runs on a half-built executor -- it falls
    // back to the current device, as before any wc_gpu_init_multi.
    int rc = WC_OK;
    int built = 0;
    for (int g = 0; g < ngpus && rc == WC_OK; ++g) {
        Device *D = nullptr;
        rc = init_locked(devs[g], &D); // sets device devs[g]
        g_shard[g].dev = devs[g];
        if (rc == WC_OK)
            rc = pipe_init_locked(g_shard[g].pipe);
        built = g + 1; // pipe_free below also frees a partly built pipe
    }
    if (rc != WC_OK) {
        for (int g = 0; g < built; ++g) {
            (void)hipSetDevice(g_shard[g].dev);
            pipe_free(g_shard[g].pipe);
            g_shard[g] = ShardExec{};
        }
    } else {
        g_multi_n = ngpus;
    }
    (void)hipSetDevice(cur);
    return rc;
}

int wc_gpu_multi_count(void)
{
    std::lock_guard<FairMutex> lk(g_mu);
    return g_multi_n;
}

int wc_cksum_host_multi(const void *h_base, uint64_t h_bytes, const uint64_t *h_off,
                        const uint16_t *h_len, uint64_t n, uint16_t *h_out, int kind)
{
    if (kind != WC_CKSUM_IP && kind != WC_CKSUM_PAYLOAD)
        return WC_EINVAL;
    if (n == 0)
        return WC_OK;
    if (!h_base || !h_off || !h_len || !h_out)
        return WC_EINVAL;
    int G = 0;
    {
        std::lock_guard<FairMutex> lk(g_mu);
        G = g_multi_n;
    }
    if (G == 0)
        return wc_cksum_host(h_base, h_bytes, h_off, h_len, n, h_out, kind);
    bool ascending = true;
    uint64_t total = 0;
    if (!host_batch_ok((const uint8_t *)h_base, h_bytes, h_off, h_len, n, kind, &ascending,
                       &total))
        return WC_EINVAL;
    {
        std::lock_guard<FairMutex> lk(g_mu);
        G = g_multi_n;
        int cur = 0;
        if (hipGetDevice(&cur) != hipSuccess)
            return WC_ENODEV;
        const bool registered = registered_dptr_locked(h_base, h_bytes) != nullptr;
        if (registered && n <= kZcPkts && total <= (uint64_t)g_cfg.zc_bytes) {
            // Small registered batch: one zero-copy launch on shard 0, with
            // the region's address as shard 0's device sees it.
            Device *D = nullptr;
            int rc = init_locked(g_shard[0].dev, &D); // sets shard 0's device
            const uint8_t *dbase = rc == WC_OK ? registered_dptr_locked(h_base, h_bytes) : nullptr;
            if (rc == WC_OK && !dbase)
                rc = WC_EINVAL;
            if (rc == WC_OK)
                rc = host_zero_copy(*D, dbase, h_off, h_len, n, (uint8_t *)h_out, kind);
            (void)hipSetDevice(cur);
            return rc;
        }
        PipeRun runs[kMaxDevices];
        for (int g = 0; g < G; ++g) {
            PipeRun &r = runs[g];
            r.D = &g_dev[g_shard[g].dev];
            r.P = &g_shard[g].pipe;
            r.dev = g_shard[g].dev;
            r.hb = (const uint8_t *)h_base;
            r.registered = registered;
            r.ascending = ascending;
            r.h_off = h_off;
            r.h_len = h_len;
            r.h_out = (uint8_t *)h_out;
            r.kind = kind;
            shard_range(n, g, G, &r.i, &r.hi);
        }
        // One thread, G pipelines: each pass stages one chunk per unfinished
        // shard, so every device's copies and kernels overlap the staging of
        // the others.
        int rc = WC_OK;
        for (bool more = true; more && rc == WC_OK;) {
            more = false;
            for (int g = 0; g < G && rc == WC_OK; ++g) {
                if (runs[g].done())
                    continue;
                more = true;
                rc = hip_err(hipSetDevice(runs[g].dev));
                if (rc == WC_OK)
                    rc = runs[g].step();
            }
        }
        for (int g = 0; g < G; ++g) {
            (void)hipSetDevice(runs[g].dev);
            if (rc == WC_OK)
                rc = runs[g].finish();
        }
        if (rc != WC_OK)
            for (int g = 0; g < G; ++g) {
                (void)hipSetDevice(runs[g].dev);
                (void)runs[g].fail(rc);
            }
        (void)hipSetDevice(cur);
        return rc;
    }
}

int wc_cksum_strided_multi(const void *const *d_base, uint64_t stride, uint16_t len,
                           const uint64_t *n, uint16_t *const *d_out, int kind,
                           void *const *streams)
{
    if (!d_base || !n || !d_out)
        return WC_EINVAL;
    return for_each_shard([&](int g) {
        return wc_cksum_strided(d_base[g], stride, len, n[g], d_out[g], kind,
                                streams ? streams[g] : nullptr);
    });
}

int wc_cksum_ragged_multi(const void *const *d_base, const uint64_t *const *d_off,
                          const uint16_t *const *d_len, const uint64_t *n,
                          uint16_t *const *d_out, int kind, void *const *streams)
{
    if (!d_base || !d_off || !d_len || !n || !d_out)
        return WC_EINVAL;
    return for_each_shard([&](int g) {
        return wc_cksum_ragged(d_base[g], d_off[g], d_len[g], n[g], d_out[g], kind,
                               streams ? streams[g] : nullptr);
    });
}

int wc_gather_results_multi(uint16_t *const *d_shard_out, const uint64_t *n,
                            uint16_t *const *d_all, void *const *streams)
{
    if (!d_shard_out || !n || !d_all)
        return WC_EINVAL;
    std::lock_guard<FairMutex> lk(g_mu);
    if (g_multi_n == 0)
        return WC_EINVAL;
    int devs[kMaxDevices];
    for (int g = 0; g < g_multi_n; ++g)
        devs[g] = g_shard[g].dev;
    int cur = 0;
    if (hipGetDevice(&cur) != hipSuccess)
        return WC_ENODEV;
    const int rc = wc::rccl_allgatherv_u16(g_multi_n, devs, d_shard_out, n, d_all, streams);
    (void)hipSetDevice(cur);
    return rc;
}

} // extern "C"
