// wc_rt_host.cpp -- host-memory batches (wc_cksum_host, wc_cksum_ip_udp_host,
// wc_rx_verdict_host, wc_host_register): the resident server or one
// zero-copy launch for a small registered batch, else the pipelined path
// (hipMemcpyAsync H2D, kernel, D2H) through pinned staging.

#include "wc_rt.h"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <thread>
#include <vector>

namespace wc {
namespace rt __attribute__((visibility("hidden"))) {

// ---------------------------------------------------------------------------
// Host-memory pipeline.

// Frees whatever a (possibly partly built) pipeline holds.
void pipe_free(HostPipe &P)
{
    for (int s = 0; s < kPipe; ++s) {
        if (P.st[s])
            (void)hipStreamSynchronize(P.st[s]);
        (void)hipFree(P.d_bytes[s]);
        (void)hipFree(P.d_off[s]);
        (void)hipFree(P.d_len[s]);
        (void)hipFree(P.d_out[s]);
        (void)hipFree(P.d_out2[s]);
        (void)hipHostFree(P.h_bytes[s]);
        (void)hipHostFree(P.h_off[s]);
        (void)hipHostFree(P.h_len[s]);
        (void)hipHostFree(P.h_out[s]);
        (void)hipHostFree(P.h_out2[s]);
        if (P.done[s])
            (void)hipEventDestroy(P.done[s]);
        if (P.st[s])
            (void)hipStreamDestroy(P.st[s]);
    }
    P = HostPipe{};
}

// Streams, events and staging of one host pipeline, created on the current
// device.
int pipe_init_locked(HostPipe &P)
{
    if (P.ready)
        return WC_OK;
    for (int s = 0; s < kPipe; ++s) {
        if (hipStreamCreateWithFlags(&P.st[s], hipStreamNonBlocking) != hipSuccess ||
            hipEventCreateWithFlags(&P.done[s], hipEventDisableTiming) != hipSuccess ||
            hipMalloc((void **)&P.d_bytes[s], kChunkBytes + 64) != hipSuccess ||
            hipMalloc((void **)&P.d_off[s], kChunkPkts * 8) != hipSuccess ||
            hipMalloc((void **)&P.d_len[s], kChunkPkts * 2) != hipSuccess ||
            hipMalloc((void **)&P.d_out[s], kChunkPkts * 2) != hipSuccess ||
            hipMalloc((void **)&P.d_out2[s], kChunkPkts * 2) != hipSuccess ||
            hipHostMalloc((void **)&P.h_bytes[s], kChunkBytes + 64, 0) != hipSuccess ||
            hipHostMalloc((void **)&P.h_off[s], kChunkPkts * 8, 0) != hipSuccess ||
            hipHostMalloc((void **)&P.h_len[s], kChunkPkts * 2, 0) != hipSuccess ||
            hipHostMalloc((void **)&P.h_out[s], kChunkPkts * 2, 0) != hipSuccess ||
            hipHostMalloc((void **)&P.h_out2[s], kChunkPkts * 2, 0) != hipSuccess) {
            pipe_free(P);
            return WC_ENOMEM;
        }
    }
    P.ready = true;
    return WC_OK;
}

int zc_init_locked(Device &D)
{
    ZeroCopy &Z = D.zc;
    if (Z.ready)
        return WC_OK;
    const unsigned fl = hipHostMallocMapped | hipHostMallocCoherent;
    if (hipStreamCreateWithFlags(&Z.st, hipStreamNonBlocking) != hipSuccess ||
        hipHostMalloc((void **)&Z.h_off, kZcPkts * 8, fl) != hipSuccess ||
        hipHostMalloc((void **)&Z.h_len, kZcPkts * 2, fl) != hipSuccess ||
        hipHostMalloc((void **)&Z.h_out, kZcPkts * 2, fl) != hipSuccess ||
        hipHostMalloc((void **)&Z.h_out2, kZcPkts * 2, fl) != hipSuccess ||
        hipHostGetDevicePointer((void **)&Z.d_off, Z.h_off, 0) != hipSuccess ||
        hipHostGetDevicePointer((void **)&Z.d_len, Z.h_len, 0) != hipSuccess ||
        hipHostGetDevicePointer((void **)&Z.d_out, Z.h_out, 0) != hipSuccess ||
        hipHostGetDevicePointer((void **)&Z.d_out2, Z.h_out2, 0) != hipSuccess)
        return WC_ENOMEM;
    Z.ready = true;
    return WC_OK;
}

// Address on the CURRENT device of host range [p, p + bytes) if it lies
// inside one registered region, else nullptr.  The region was registered
// portable and mapped; its device address is looked up for this device the
// first time (a batch may run on a shard device other than the one current
// at wc_host_register).
const uint8_t *registered_dptr_locked(const void *p, uint64_t bytes)
{
    const uintptr_t a = (uintptr_t)p;
    auto it = g_registered.upper_bound(a);
    if (it == g_registered.begin())
        return nullptr;
    --it;
    if (a < it->first || a + bytes > it->first + it->second.bytes)
        return nullptr;
    int dev = 0;
    if (current_device(&dev) != WC_OK)
        return nullptr;
    const uint8_t *&d = it->second.dptr[dev];
    if (!d) {
        void *dp = nullptr;
        if (hipHostGetDevicePointer(&dp, (void *)it->first, 0) != hipSuccess)
            return nullptr;
        d = (const uint8_t *)dp;
    }
    return d + (a - it->first);
}

// Bytes the reference reads for one packet (payload_cksum reads the IPv4
// header fields up to byte 19 whatever len is, in_cksum.c:149-151).
uint64_t span_of(uint16_t len, int kind)
{
    return kind == WC_CKSUM_PAYLOAD || kind == kKindFused ? std::max<uint64_t>(len, 20) : len;
}

// Bytes the fused TX pair reads of the packet at p (whose first
// span_of(len, kKindFused) bytes are known to be readable): payload_cksum's,
// and the IPv4 header's hl bytes ip_cksum sums (ip4.c:184-186) when they run
// past them (options behind a short len).
uint64_t fused_span(const uint8_t *p, uint16_t len)
{
    const uint64_t s = span_of(len, kKindFused);
    if (s >= 60) // (no IPv4 header is longer: the packet's byte need not be read)
        return s;
    return (p[0] >> 4) == 4 ? std::max<uint64_t>(s, (uint64_t)(p[0] & 15u) * 4u) : s;
}

// Result bytes per packet in the main result array: a uint16 checksum, or a
// uint8 RX verdict.
int out_size(int kind) { return kind == kKindRx ? 1 : 2; }

// One device launch over a ragged batch of `kind` (a checksum kind, RX
// verdicts -- lengths are frame lengths --, or the fused pair, whose header
// checksums go to d_out_hdr).
int run_ragged_any(Device &D, const Config &C, const uint8_t *d_base, const uint64_t *d_off,
                   const uint16_t *d_len, uint64_t n, void *d_out, int kind, bool zero_copy,
                   hipStream_t st, uint16_t *d_out_hdr = nullptr)
{
    if (kind == kKindRx)
        return hip_err(rx_launch(D, C, d_base, d_off, d_len, n, (uint8_t *)d_out, nullptr, st));
    const bool fused = kind == kKindFused;
    const int k = fused ? WC_CKSUM_PAYLOAD : kind;
    const Plan p = plan_ragged(D, C, n, k, zero_copy, fused);
    wc::LaunchArgs a{d_base, 0,       0,    d_off, d_len, n,
                     (uint16_t *)d_out, nullptr, k, true,  false, C.nt != 0,
                     C.flat_tpw, fused ? d_out_hdr : nullptr};
    return run(D, C, a, p, st);
}

// Small registered batch: one launch reading host memory in place.
int host_zero_copy(Device &D, const uint8_t *dbase, const uint64_t *h_off,
                   const uint16_t *h_len, uint64_t n, uint8_t *h_out, int kind,
                   uint16_t *h_out2)
{
    int rc = zc_init_locked(D);
    if (rc)
        return rc;
    ZeroCopy &Z = D.zc;
    memcpy(Z.h_off, h_off, n * 8);
    memcpy(Z.h_len, h_len, n * 2);
    rc = run_ragged_any(D, g_cfg, dbase, Z.d_off, Z.d_len, n, Z.d_out, kind, true, Z.st,
                        Z.d_out2);
    if (rc)
        return rc;
    hipError_t e = hipStreamSynchronize(Z.st);
    if (e != hipSuccess)
        return hip_err(e);
    memcpy(h_out, (const void *)Z.h_out, n * out_size(kind));
    if (kind == kKindFused)
        memcpy(h_out2, (const void *)Z.h_out2, n * 2);
    return WC_OK;
}

int zs_init_locked(Device &D)
{
    ZcStream &S = D.zs;
    if (S.ready)
        return WC_OK;
    const unsigned fl = hipHostMallocMapped | hipHostMallocCoherent;
    bool ok = hipStreamCreateWithFlags(&S.st, hipStreamNonBlocking) == hipSuccess;
    for (int b = 0; b < 2 && ok; ++b)
        ok = hipEventCreateWithFlags(&S.done[b], hipEventDisableTiming) == hipSuccess &&
             hipHostMalloc((void **)&S.h_off[b], kZsPkts * 8, fl) == hipSuccess &&
             hipHostMalloc((void **)&S.h_len[b], kZsPkts * 2, fl) == hipSuccess &&
             hipHostMalloc((void **)&S.h_out[b], kZsPkts * 2, fl) == hipSuccess &&
             hipHostMalloc((void **)&S.h_out2[b], kZsPkts * 2, fl) == hipSuccess &&
             hipHostGetDevicePointer((void **)&S.d_off[b], S.h_off[b], 0) == hipSuccess &&
             hipHostGetDevicePointer((void **)&S.d_len[b], S.h_len[b], 0) == hipSuccess &&
             hipHostGetDevicePointer((void **)&S.d_out[b], S.h_out[b], 0) == hipSuccess &&
             hipHostGetDevicePointer((void **)&S.d_out2[b], S.h_out2[b], 0) == hipSuccess;
    if (!ok) {
        zs_free(S);
        return WC_ENOMEM;
    }
    S.ready = true;
    return WC_OK;
}

void zs_free(ZcStream &S)
{
    if (S.st)
        (void)hipStreamSynchronize(S.st);
    for (int b = 0; b < 2; ++b) {
        if (S.done[b])
            (void)hipEventDestroy(S.done[b]);
        (void)hipHostFree(S.h_off[b]);
        (void)hipHostFree(S.h_len[b]);
        (void)hipHostFree(S.h_out[b]);
        (void)hipHostFree(S.h_out2[b]);
    }
    if (S.st)
        (void)hipStreamDestroy(S.st);
    S = ZcStream{};
}

// A large batch in a registered region (ZcStream): chunk k's launch reads
// its packets in place while the host writes chunk k + 1's offsets and
// lengths into the other buffer and copies chunk k - 1's results out.
int host_zc_stream(Device &D, const uint8_t *dbase, const uint64_t *h_off,
                   const uint16_t *h_len, uint64_t n, uint8_t *h_out, int kind,
                   uint16_t *h_out2)
{
    int rc = zs_init_locked(D);
    if (rc)
        return rc;
    ZcStream &S = D.zs;
    const int osz = out_size(kind);
    uint64_t pend_lo[2] = {}, pend_n[2] = {};
    bool pend[2] = {};
    auto drain = [&](int b) -> int {
        if (!pend[b])
            return WC_OK;
        const hipError_t e = hipEventSynchronize(S.done[b]);
        if (e != hipSuccess)
            return hip_err(e);
        memcpy(h_out + pend_lo[b] * osz, (const void *)S.h_out[b], pend_n[b] * osz);
        if (kind == kKindFused)
            memcpy(h_out2 + pend_lo[b], (const void *)S.h_out2[b], pend_n[b] * 2);
        pend[b] = false;
        return WC_OK;
    };
    int b = 0;
    const uint64_t per = g_cfg.zs_pkts;
    for (uint64_t i = 0; i < n && rc == WC_OK; i += per, b ^= 1) {
        const uint64_t cnt = std::min(per, n - i);
        rc = drain(b); // (chunk k - 2's results: its buffers are free again)
        if (rc)
            break;
        memcpy(S.h_off[b], h_off + i, cnt * 8);
        memcpy(S.h_len[b], h_len + i, cnt * 2);
        rc = run_ragged_any(D, g_cfg, dbase, S.d_off[b], S.d_len[b], cnt, S.d_out[b], kind, true,
                            S.st, S.d_out2[b]);
        if (rc == WC_OK)
            rc = hip_err(hipEventRecord(S.done[b], S.st));
        if (rc == WC_OK) {
            pend[b] = true;
            pend_lo[b] = i;
            pend_n[b] = cnt;
        }
    }
    if (rc == WC_OK)
        rc = drain(b); // the older of the two in flight first
    if (rc == WC_OK)
        rc = drain(b ^ 1);
    if (rc != WC_OK) // (nothing may still write the mapped buffers the next call refills)
        (void)hipStreamSynchronize(S.st);
    return rc;
}

// Library-owned staging workers.  Pageable input reaches the GPU through
// the pinned staging ring, and copying it there was the end-to-end path's
// limit on one thread (24.6-28.9 GB/s against ~55 GB/s for DMA from
// registered memory) -- for every shard of
// wc_cksum_host_multi alike, since the engine thread stages them all.  The
// copy of each chunk is split over W workers plus the calling thread
// (WC_STAGE_THREADS, default min(8, cores - 1); 0 = the calling thread
// alone).  Created at the first pageable chunk, joined at exit.
class StagePool {
public:
    explicit StagePool(int workers)
    {
        for (int i = 0; i < workers; ++i)
            th_.emplace_back([this] { loop(); });
    }
    ~StagePool()
    {
        {
            std::lock_guard<std::mutex> lk(mu_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto &t : th_)
            t.join();
    }
    int width() const { return (int)th_.size() + 1; }
    // fn(0) .. fn(parts - 1), the calling thread taking its share; returns
    // when all are done.
    void run(int parts, const std::function<void(int)> &fn)
    {
        if (parts <= 1 || th_.empty()) {
            for (int i = 0; i < parts; ++i)
                fn(i);
            return;
        }
        std::unique_lock<std::mutex> lk(mu_);
        job_ = &fn;
        parts_ = parts;
        next_ = 0;
        pending_ = parts;
        ++gen_;
        cv_.notify_all();
        while (next_ < parts_) {
            const int i = next_++;
            lk.unlock();
            fn(i);
            lk.lock();
            --pending_;
        }
        done_.wait(lk, [this] { return pending_ == 0; });
        job_ = nullptr;
    }

private:
    void loop()
    {
        uint64_t seen = 0;
        std::unique_lock<std::mutex> lk(mu_);
        for (;;) {
            cv_.wait(lk, [&] { return stop_ || (gen_ != seen && job_ && next_ < parts_); });
            if (stop_)
                return;
            seen = gen_;
            while (job_ && next_ < parts_) {
                const int i = next_++;
                const std::function<void(int)> *fn = job_;
                lk.unlock();
                (*fn)(i);
                lk.lock();
                if (--pending_ == 0)
                    done_.notify_all();
            }
        }
    }
    std::vector<std::thread> th_;
    std::mutex mu_;
    std::condition_variable cv_, done_;
    const std::function<void(int)> *job_ = nullptr;
    int parts_ = 0, next_ = 0, pending_ = 0;
    uint64_t gen_ = 0;
    bool stop_ = false;
};

StagePool &stage_pool()
{
    static StagePool pool([] {
        const char *v = getenv("WC_STAGE_THREADS");
        if (v && *v)
            return std::max(0, atoi(v));
        const int hw = (int)std::thread::hardware_concurrency();
        return std::max(0, std::min(8, hw - 1));
    }());
    return pool;
}

// memcpy of `bytes` split over the staging pool (pieces of >= 2 MiB).
void stage_copy(void *dst, const void *src, uint64_t bytes)
{
    StagePool &P = stage_pool();
    constexpr uint64_t kPiece = 2ull << 20;
    const int parts = (int)std::min<uint64_t>((uint64_t)P.width(), (bytes + kPiece - 1) / kPiece);
    if (parts <= 1) {
        memcpy(dst, src, bytes);
        return;
    }
    const uint64_t step = ((bytes + parts - 1) / parts + 63) & ~63ull;
    P.run(parts, [&](int i) {
        const uint64_t lo = std::min(bytes, (uint64_t)i * step);
        const uint64_t hi = std::min(bytes, lo + step);
        memcpy((uint8_t *)dst + lo, (const uint8_t *)src + lo, hi - lo);
    });
}

// Pipelined path: chunks of packets go through kPipe streams, each chunk
// H2D -> kernel -> D2H.  An ascending batch ships the byte range its chunk
// covers (straight from registered memory, else via pinned staging); any
// other order is gathered packet by packet into pinned staging first.
//
// A PipeRun walks packets [i, hi) of a batch through one HostPipe on one
// device, one chunk per step(), so a single host thread can interleave the
// runs of several devices (wc_cksum_host_multi): while it stages device g's
// next chunk, the other devices' copies and kernels are in flight.
// Bytes packet j's check reads (the fused pair: also its IPv4 header).
uint64_t PipeRun::span(uint64_t j) const
{
    return kind == kKindFused ? fused_span(hb + h_off[j], h_len[j]) : span_of(h_len[j], kind);
}

// Wait for a slot's chunk and copy its results out.
int PipeRun::drain(int s)
{
    if (!pend[s])
        return WC_OK;
    hipError_t e = hipEventSynchronize(P->done[s]);
    if (e != hipSuccess)
        return hip_err(e);
    const int osz = out_size(kind);
    memcpy(h_out + pend_lo[s] * osz, P->h_out[s], pend_n[s] * osz);
    if (kind == kKindFused)
        memcpy(h_out2 + pend_lo[s], P->h_out2[s], pend_n[s] * 2);
    pend[s] = false;
    return WC_OK;
}

// On any error, wait for every slot's in-flight copies and kernel before
// returning: they use the library's pinned staging, which the next call
// rewrites with plain memcpy.
int PipeRun::fail(int rc)
{
    for (int s = 0; s < kPipe; ++s) {
        (void)hipStreamSynchronize(P->st[s]);
        pend[s] = false;
    }
    return rc;
}

// Stage and enqueue the next chunk (caller: current device = dev).
int PipeRun::step()
{
    int rc = drain(slot);
    if (rc)
        return rc;
    const uint64_t i0 = i;
    uint64_t j = i, bytes = 0;
    const uint8_t *src = nullptr;
    if (ascending) {
        const uint64_t lo = h_off[i];
        uint64_t top = lo;
        while (j < hi && j - i0 < kChunkPkts) {
            const uint64_t e = h_off[j] + span(j);
            if (std::max(top, e) - lo > kChunkBytes && j > i0)
                break;
            top = std::max(top, e);
            P->h_off[slot][j - i0] = h_off[j] - lo;
            P->h_len[slot][j - i0] = h_len[j];
            ++j;
        }
        bytes = top - lo;
        src = hb + lo;
        if (!registered) {
            stage_copy(P->h_bytes[slot], src, bytes);
            src = P->h_bytes[slot];
        }
    } else {
        // Rebased offsets first (a prefix sum), then the packet copies
        // in parallel ranges of the staging pool.
        while (j < hi && j - i0 < kChunkPkts) {
            const uint64_t sp = span(j);
            if (bytes + sp > kChunkBytes && j > i0)
                break;
            P->h_off[slot][j - i0] = bytes;
            P->h_len[slot][j - i0] = h_len[j];
            bytes += sp;
            ++j;
        }
        const uint64_t cnt = j - i0;
        StagePool &pool = stage_pool();
        const int parts = (int)std::min<uint64_t>((uint64_t)pool.width(), (cnt + 4095) / 4096);
        uint8_t *dst = P->h_bytes[slot];
        const uint64_t *roff = P->h_off[slot];
        auto gather = [&](int t) {
            const uint64_t a = cnt * (uint64_t)t / (uint64_t)parts;
            const uint64_t b = cnt * (uint64_t)(t + 1) / (uint64_t)parts;
            for (uint64_t q = a; q < b; ++q)
                memcpy(dst + roff[q], hb + h_off[i0 + q], span(i0 + q));
        };
        pool.run(std::max(parts, 1), gather);
        src = P->h_bytes[slot];
    }
    const uint64_t cnt = j - i0;
    hipStream_t st = P->st[slot];
    hipError_t e = hipMemcpyAsync(P->d_bytes[slot], src, bytes, hipMemcpyHostToDevice, st);
    if (e == hipSuccess)
        e = hipMemcpyAsync(P->d_off[slot], P->h_off[slot], cnt * 8, hipMemcpyHostToDevice,
                           st);
    if (e == hipSuccess)
        e = hipMemcpyAsync(P->d_len[slot], P->h_len[slot], cnt * 2, hipMemcpyHostToDevice,
                           st);
    if (e != hipSuccess)
        return hip_err(e);
    rc = run_ragged_any(*D, g_cfg, P->d_bytes[slot], P->d_off[slot], P->d_len[slot], cnt,
                        P->d_out[slot], kind, false, st, P->d_out2[slot]);
    if (rc)
        return rc;
    e = hipMemcpyAsync(P->h_out[slot], P->d_out[slot], cnt * out_size(kind),
                       hipMemcpyDeviceToHost, st);
    if (e == hipSuccess && kind == kKindFused)
        e = hipMemcpyAsync(P->h_out2[slot], P->d_out2[slot], cnt * 2, hipMemcpyDeviceToHost,
                           st);
    if (e == hipSuccess)
        e = hipEventRecord(P->done[slot], st);
    if (e != hipSuccess)
        return hip_err(e);
    pend[slot] = true;
    pend_lo[slot] = i0;
    pend_n[slot] = cnt;
    i = j;
    slot = (slot + 1) % kPipe;
    return WC_OK;
}

int PipeRun::finish()
{
    for (int s = 0; s < kPipe; ++s) {
        int rc = drain((slot + s) % kPipe);
        if (rc)
            return rc;
    }
    return WC_OK;
}

// Every packet of a host batch inside [0, h_bytes); its order and bytes.
bool host_batch_ok(const uint8_t *hb, uint64_t h_bytes, const uint64_t *h_off,
                   const uint16_t *h_len, uint64_t n, int kind, bool *ascending, uint64_t *total,
                   uint64_t *range)
{
    bool asc = true;
    uint64_t tot = 0, lo = ~0ull, hi = 0;
    for (uint64_t i = 0; i < n; ++i) {
        const uint64_t o = h_off[i];
        uint64_t sp = span_of(h_len[i], kind);
        if (o > h_bytes || sp > h_bytes - o)
            return false;
        if (kind == kKindFused) { // (its first sp >= 20 bytes are in range)
            sp = fused_span(hb + o, h_len[i]);
            if (sp > h_bytes - o)
                return false;
        }
        asc &= i == 0 || o >= h_off[i - 1];
        tot += sp;
        lo = std::min(lo, o);
        hi = std::max(hi, o + sp);
    }
    *ascending = asc;
    *total = tot;
    if (range)
        *range = n ? hi - lo : 0;
    return true;
}

void shard_range(uint64_t n, int g, int G, uint64_t *lo, uint64_t *hi)
{
    // n * g / G without overflow for any uint64 n
    *lo = (uint64_t)((unsigned __int128)n * (unsigned)g / (unsigned)G);
    *hi = (uint64_t)((unsigned __int128)n * (unsigned)(g + 1) / (unsigned)G);
}

int host_pipeline(Device &D, const uint8_t *hb, bool registered, bool ascending,
                  const uint64_t *h_off, const uint16_t *h_len, uint64_t n,
                  uint8_t *h_out, int kind, uint16_t *h_out2)
{
    PipeRun r;
    r.D = &D;
    r.P = &D.pipe;
    r.hb = hb;
    r.registered = registered;
    r.ascending = ascending;
    r.h_off = h_off;
    r.h_len = h_len;
    r.h_out = h_out;
    r.h_out2 = h_out2;
    r.kind = kind;
    r.hi = n;
    while (!r.done()) {
        const int rc = r.step();
        if (rc)
            return r.fail(rc);
    }
    const int rc = r.finish();
    return rc ? r.fail(rc) : WC_OK;
}


// wc_cksum_host / wc_rx_verdict_host / wc_cksum_ip_udp_host: a host-memory
// batch on the current device -- the resident server or one zero-copy launch
// for a small registered batch, else the pipeline.  h_out2: the fused pair's
// header checksums.
int host_batch(const void *h_base, uint64_t h_bytes, const uint64_t *h_off,
               const uint16_t *h_len, uint64_t n, uint8_t *h_out, int kind,
               uint16_t *h_out2 = nullptr)
{
    if (n == 0)
        return WC_OK;
    if (!h_base || !h_off || !h_len || !h_out || (kind == kKindFused && !h_out2))
        return WC_EINVAL;
    bool ascending = true;
    uint64_t total = 0, range = 0;
    if (!host_batch_ok((const uint8_t *)h_base, h_bytes, h_off, h_len, n, kind, &ascending,
                       &total, &range))
        return WC_EINVAL;
    // Packets covering less than 7/8 of their byte range (netmap slots: 1472
    // of 2048 B) are sparse: the pipeline would ship the gaps too.
    const bool sparse = total < range - range / 8;

    std::lock_guard<FairMutex> lk(g_mu);
    Device *D = nullptr;
    int rc = init_locked(-1, &D);
    if (rc)
        return rc;
    const uint8_t *dbase = registered_dptr_locked(h_base, h_bytes);
    if (dbase && g_cfg.serve && server_enabled_locked() && n <= (uint64_t)g_cfg.serve_max) {
        bool fits = true; // (a fused header adds at most 40 bytes to the span)
        for (uint64_t i = 0; i < n && fits; ++i)
            fits = span_of(h_len[i], kind) + (kind == kKindFused ? 40u : 0u) <= wc::kSrvMaxBytes;
        int dev = 0;
        if (fits && current_device(&dev) == WC_OK) {
            rc = serve_batch(*D, dev, dbase, h_off, h_len, n, h_out, kind, h_out2);
            if (rc != kSrvFallback)
                return rc;
        }
    }
    if (dbase && n <= kZcPkts && total <= (uint64_t)g_cfg.zc_bytes)
        return host_zero_copy(*D, dbase, h_off, h_len, n, h_out, kind, h_out2);
    // A large registered batch: sparse or in any order, the kernels read its
    // packets in place (only the lines they touch cross the link); dense and
    // ascending, the pipeline's range DMA is a little faster (C2 bytes from a
    // registered region: 54.5 vs 52.9 GB/s, the three sparse ring calls 39 ->
    // 46-47 GB/s: profiles/e2e_r06b.log).
    if (dbase && g_cfg.zc_stream && (sparse || !ascending))
        return host_zc_stream(*D, dbase, h_off, h_len, n, h_out, kind, h_out2);
    rc = pipe_init_locked(D->pipe);
    if (rc)
        return rc;
    // (pageable and sparse: gathered packet by packet into the staging, not
    // the whole range with its gaps)
    return host_pipeline(*D, (const uint8_t *)h_base, dbase != nullptr, ascending && !sparse,
                         h_off, h_len, n, h_out, kind, h_out2);
}

} // namespace rt
} // namespace wc

using namespace wc::rt;

extern "C" {

int wc_host_register(void *h_ptr, uint64_t bytes)
{
    if (!h_ptr || !bytes)
        return WC_EINVAL;
    std::lock_guard<FairMutex> lk(g_mu);
    Device *D = nullptr;
    int rc = init_locked(-1, &D);
    if (rc)
        return rc;
    // The resident server grid would hold up a device-wide synchronisation
    // that (un)registering may do until the idle watcher stopped it -- and
    // the watcher waits for g_mu, held here.  Stop it first; the next small
    // call starts it again.
    server_stop_all_locked();
    // Registering a base address again always pins the pages mapped there
    // NOW: the caller may have freed the old region without
    // wc_host_unregister and got a new buffer at the same address, whose
    // pages the old registration (and its cached device addresses) do not
    // cover.  So the old registration is dropped and the range registered
    // afresh; if that fails, the old range is registered again so a live
    // region keeps working, and the error is returned.
    uint64_t old_bytes = 0;
    auto it = g_registered.find((uintptr_t)h_ptr);
    if (it != g_registered.end()) {
        old_bytes = it->second.bytes;
        g_registered.erase(it);
        (void)hipHostUnregister(h_ptr);
    }
    const unsigned flags = hipHostRegisterMapped | hipHostRegisterPortable;
    auto pin = [&](uint64_t nb) -> hipError_t {
        // Portable: every device (wc_cksum_host_multi's shards) may DMA from it.
        hipError_t e = hipHostRegister(h_ptr, nb, flags);
        if (e != hipSuccess)
            return e;
        void *dptr = nullptr;
        e = hipHostGetDevicePointer(&dptr, h_ptr, 0);
        if (e != hipSuccess) {
            (void)hipHostUnregister(h_ptr);
            return e;
        }
        Registration reg;
        reg.bytes = nb;
        int dev = 0;
        if (current_device(&dev) == WC_OK)
            reg.dptr[dev] = (const uint8_t *)dptr;
        g_registered[(uintptr_t)h_ptr] = reg;
        return hipSuccess;
    };
    const hipError_t e = pin(bytes);
    if (e != hipSuccess && old_bytes)
        (void)pin(old_bytes);
    return hip_err(e);
}

int wc_host_unregister(void *h_ptr)
{
    if (!h_ptr)
        return WC_EINVAL;
    std::lock_guard<FairMutex> lk(g_mu);
    auto it = g_registered.find((uintptr_t)h_ptr);
    if (it == g_registered.end())
        return WC_EINVAL;
    g_registered.erase(it);
    server_stop_all_locked(); // (see wc_host_register)
    return hip_err(hipHostUnregister(h_ptr));
}

int wc_cksum_host(const void *h_base, uint64_t h_bytes, const uint64_t *h_off,
                  const uint16_t *h_len, uint64_t n, uint16_t *h_out, int kind)
{
    if (kind != WC_CKSUM_IP && kind != WC_CKSUM_PAYLOAD)
        return WC_EINVAL;
    return host_batch(h_base, h_bytes, h_off, h_len, n, (uint8_t *)h_out, kind);
}

int wc_cksum_ip_udp_host(const void *h_base, uint64_t h_bytes, const uint64_t *h_off,
                         const uint16_t *h_len, uint64_t n, uint16_t *h_out_ip_hdr,
                         uint16_t *h_out_payload)
{
    if (n && (!h_out_ip_hdr || !h_out_payload))
        return WC_EINVAL;
    return host_batch(h_base, h_bytes, h_off, h_len, n, (uint8_t *)h_out_payload, kKindFused,
                      h_out_ip_hdr);
}

int wc_rx_verdict_host(const void *h_base, uint64_t h_bytes, const uint64_t *h_off,
                       const uint16_t *h_frame_len, uint64_t n, uint8_t *h_verdict,
                       uint64_t *h_drops)
{
    if (n && !h_verdict)
        return WC_EINVAL;
    const int rc = host_batch(h_base, h_bytes, h_off, h_frame_len, n, h_verdict, kKindRx);
    if (rc == WC_OK && h_drops) {
        uint64_t d = 0;
        for (uint64_t i = 0; i < n; ++i)
            d += WC_RX_IS_DROP(h_verdict[i]);
        *h_drops = d;
    }
    return rc;
}

} // extern "C"
