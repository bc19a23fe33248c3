// wc_rt_server.cpp -- host side of the resident small-batch server
// (wc_k_serve.hip): its lifetime, request posting,
// the idle watcher, pause / resume and its counters.

#include "wc_rt.h"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>

namespace wc {
namespace rt __attribute__((visibility("hidden"))) {

ServerStats g_srv_stats;

// wc_server_pause depth (under g_mu): while > 0 no grid is resident and small
// registered batches take the zero-copy launch.
int g_srv_paused = 0;

bool server_enabled_locked() { return g_srv_paused == 0; }

// ---------------------------------------------------------------------------
// The resident small-batch server (wc_k_serve.hip).  A small batch in a
// registered region is answered by a persistent grid that polls request
// records in mapped pinned memory: no launch, no stream synchronisation, no
// copy per call.  The grid is started by the first such call, kept while
// calls keep coming, and stopped (stop flag in every record, then the stream
// drained) by the idle watcher after WC_SERVE_IDLE_US without a call, by
// wc_gpu_fini, or at process exit -- so it never outlives its process.  If it
// ever fails to answer, the call falls back to the zero-copy launch and the
// server stays off for the process.

constexpr uint64_t kSrvSafetyMs = 4000; // the grid drains itself after this idle time

std::atomic<bool> g_srv_quit{false};
std::thread g_srv_watcher;
bool g_srv_hooks = false; // watcher started, atexit registered

// The grid's stream must not share a hardware queue with other work.  HIP
// maps a process's streams onto a few shared hardware queues per priority
// level (GPU_MAX_HW_QUEUES, 4 here), and a queue runs its commands in order:
// every kernel or copy of another stream that lands on the grid's queue waits
// until the grid leaves -- and the idle watcher that stops it needs g_mu,
// which a host call waiting for such a kernel holds, so the wait lasted until
// the grid's own 4-s drain (tests/c/thread_engines.c: 2-3 host calls per
// engine in 8 s).  The grid's stream takes the highest priority, whose queues
// are not shared with normal-priority streams (the library's own and, by
// default, the caller's); it stays non-blocking, so work on the null stream
// (torch's default) never waits for the grid either.  (A CU-masked stream
// would get a queue of its own too, but HIP creates those as blocking
// streams.)
hipError_t server_stream_create(hipStream_t *st)
{
    int least = 0, greatest = 0;
    if (g_cfg.serve_prio && hipDeviceGetStreamPriorityRange(&least, &greatest) == hipSuccess &&
        greatest != least)
        return hipStreamCreateWithPriority(st, hipStreamNonBlocking, greatest);
    return hipStreamCreateWithFlags(st, hipStreamNonBlocking);
}

int server_init_locked(Device &D)
{
    Server &S = D.srv;
    if (S.ready)
        return WC_OK;
    const unsigned fl = hipHostMallocMapped | hipHostMallocCoherent;
    if (server_stream_create(&S.st) != hipSuccess ||
        hipHostMalloc((void **)&S.h_rec, wc::kSrvMaxPkts * sizeof(wc::SrvRec), fl) != hipSuccess ||
        hipHostMalloc((void **)&S.h_res, wc::kSrvMaxPkts * sizeof(wc::SrvRes), fl) != hipSuccess ||
        hipHostMalloc((void **)&S.h_hb, 64, fl) != hipSuccess ||
        hipHostGetDevicePointer((void **)&S.d_rec, S.h_rec, 0) != hipSuccess ||
        hipHostGetDevicePointer((void **)&S.d_res, S.h_res, 0) != hipSuccess ||
        hipHostGetDevicePointer((void **)&S.d_hb, S.h_hb, 0) != hipSuccess)
        return WC_ENOMEM;
    memset(S.h_rec, 0, wc::kSrvMaxPkts * sizeof(wc::SrvRec));
    memset((void *)S.h_res, 0, wc::kSrvMaxPkts * sizeof(wc::SrvRes));
    memset(S.h_hb, 0, 64);
    S.ready = true;
    return WC_OK;
}

// Launch the grid with every record rewritten to {S.seq, no stop} first:
// nothing pending, stop flags cleared, the heartbeat at S.seq.
int server_launch_locked(Device &D)
{
    Server &S = D.srv;
    for (uint32_t k = 0; k < wc::kSrvMaxPkts; ++k) {
        S.h_rec[k].addr = 0;
        S.h_rec[k].info = 0;
        __atomic_store_n(&S.h_rec[k].seq, S.seq, __ATOMIC_RELEASE);
    }
    __atomic_store_n(S.h_hb, S.seq, __ATOMIC_RELEASE);
    const uint64_t idle_ticks = kSrvSafetyMs * D.clock_khz;
    const hipError_t e =
        wc::launch_serve(S.d_rec, S.d_res, S.d_hb, S.seq, S.waves, idle_ticks, S.st);
    if (e != hipSuccess)
        return hip_err(e);
    S.running = true;
    S.posted = std::chrono::steady_clock::now();
    ++g_srv_stats.launches;
    return WC_OK;
}

// Stop flag in every polled record, then wait for the grid to drain.
void server_stop_locked(Device &D, int dev)
{
    Server &S = D.srv;
    if (!S.running)
        return;
    for (int k = 0; k < S.waves && k < (int)wc::kSrvMaxPkts; ++k)
        __atomic_store_n(&S.h_rec[k].info, 1u << 24, __ATOMIC_RELEASE);
    int cur = -1;
    (void)hipGetDevice(&cur);
    (void)hipSetDevice(dev);
    (void)hipStreamSynchronize(S.st);
    if (cur >= 0)
        (void)hipSetDevice(cur);
    S.running = false;
}

void server_stop_all_locked()
{
    for (int d = 0; d < kMaxDevices; ++d)
        if (g_dev[d].ok && g_dev[d].srv.running)
            server_stop_locked(g_dev[d], d);
}

void server_watch()
{
    while (!g_srv_quit.load()) {
        std::this_thread::sleep_for(std::chrono::milliseconds(2));
        std::lock_guard<FairMutex> lk(g_mu);
        const auto now = std::chrono::steady_clock::now();
        for (int d = 0; d < kMaxDevices; ++d) {
            Device &D = g_dev[d];
            if (D.ok && D.srv.running &&
                now - D.srv.last > std::chrono::microseconds(g_cfg.serve_idle_us))
                server_stop_locked(D, d);
        }
    }
}

void server_atexit()
{
    g_srv_quit.store(true);
    if (g_srv_watcher.joinable())
        g_srv_watcher.join();
    std::lock_guard<FairMutex> lk(g_mu);
    server_stop_all_locked();
}

// The next request number (0 is the records' initial value: never used).
uint32_t server_next_seq(Server &S)
{
    S.seq = S.seq + 1 == 0 ? 1 : S.seq + 1;
    return S.seq;
}

// Post request `seq`: the heartbeat first, then one record per packet, last
// packet first -- a wave that sees its first record current finds every
// later one of the request current too (stores become visible in program
// order).
void server_post(Server &S, uint32_t seq, const uint8_t *dbase, const uint64_t *h_off,
                 const uint16_t *h_len, uint64_t n, uint32_t rkind)
{
    __atomic_store_n(S.h_hb, seq, __ATOMIC_RELEASE);
    for (uint64_t k = n; k-- > 0;) {
        wc::SrvRec &r = S.h_rec[k];
        r.addr = (uint64_t)(dbase + h_off[k]) | (n << wc::kSrvAddrBits);
        r.info = (uint32_t)h_len[k] | (rkind << 16);
        __atomic_store_n(&r.seq, seq, __ATOMIC_RELEASE);
    }
    S.posted = std::chrono::steady_clock::now();
}

// One small registered batch through the server (caller holds g_mu, the
// device is current).  Returns kSrvFallback when the server can't take it.
// h_out2: the fused pair's header checksums (kind kKindFused).
int serve_batch(Device &D, int dev, const uint8_t *dbase, const uint64_t *h_off,
                const uint16_t *h_len, uint64_t n, uint8_t *h_out, int kind,
                uint16_t *h_out2)
{
    Server &S = D.srv;
    if (S.broken) {
        ++g_srv_stats.fallbacks;
        return kSrvFallback;
    }
    // The record packs the count above a 48-bit address: every packet's
    // (offsets come in any order).
    for (uint64_t k = 0; k < n; ++k)
        if ((uint64_t)dbase + h_off[k] >= (1ull << wc::kSrvAddrBits)) {
            ++g_srv_stats.fallbacks;
            return kSrvFallback;
        }
    int rc = server_init_locked(D);
    if (rc)
        return rc;
    if (!g_srv_hooks) {
        g_srv_hooks = true;
        g_srv_watcher = std::thread(server_watch);
        std::atexit(server_atexit);
    }
    // A grid left without a request for half its own drain time is stopped
    // and started afresh: it may be about to leave (each wave leaves once
    // kSrvSafetyMs passed without a request it or the heartbeat showed), and
    // a request posted to a grid that is half gone would not be answered in
    // full.  (The idle watcher normally stops it within WC_SERVE_IDLE_US.)
    if (S.running && std::chrono::steady_clock::now() - S.posted >
                         std::chrono::milliseconds(kSrvSafetyMs / 2))
        server_stop_locked(D, dev);
    if (!S.running) {
        S.waves = g_cfg.serve_waves;
        rc = server_launch_locked(D);
        if (rc)
            return rc;
    }
    const uint32_t rkind = kind == kKindRx      ? wc::kSrvKindRx
                           : kind == kKindFused ? wc::kSrvKindFused
                                                : (uint32_t)kind;
    uint32_t seq = server_next_seq(S);
    server_post(S, seq, dbase, h_off, h_len, n, rkind);
    auto t0 = std::chrono::steady_clock::now();
    bool relaunched = false;
    for (uint64_t k = 0; k < n; ++k) {
        for (uint32_t spin = 1;; ++spin) {
            if (__atomic_load_n(&S.h_res[k].seq, __ATOMIC_ACQUIRE) == seq)
                break;
            __builtin_ia32_pause();
            if (spin % 4096)
                continue;
            const auto dt = std::chrono::steady_clock::now() - t0;
            if (dt > std::chrono::milliseconds(50) && !relaunched &&
                hipStreamQuery(S.st) == hipSuccess) {
                // The grid is gone (it cannot leave part-way: see above):
                // start it afresh -- every record reset, so no wave takes a
                // stale record for a request -- and post the batch again.
                relaunched = true;
                S.running = false;
                rc = server_launch_locked(D);
                if (rc)
                    return rc;
                seq = server_next_seq(S);
                server_post(S, seq, dbase, h_off, h_len, n, rkind);
                t0 = std::chrono::steady_clock::now();
                k = 0;
                spin = 0;
                continue;
            }
            if (dt > std::chrono::milliseconds(2000)) {
                fprintf(stderr, "wccksum: resident server did not answer; using launches\n");
                server_stop_locked(D, dev);
                S.broken = true;
                ++g_srv_stats.fallbacks;
                return kSrvFallback;
            }
        }
    }
    if (kind == kKindRx) {
        for (uint64_t k = 0; k < n; ++k)
            h_out[k] = (uint8_t)S.h_res[k].value;
    } else {
        uint16_t *o = (uint16_t *)h_out;
        for (uint64_t k = 0; k < n; ++k)
            o[k] = (uint16_t)S.h_res[k].value;
        if (kind == kKindFused)
            for (uint64_t k = 0; k < n; ++k)
                h_out2[k] = (uint16_t)(S.h_res[k].value >> 16);
    }
    S.last = std::chrono::steady_clock::now();
    ++g_srv_stats.served;
    return WC_OK;
}

} // namespace rt
} // namespace wc

using namespace wc::rt;

extern "C" {

int wc_server_pause(void)
{
    std::lock_guard<FairMutex> lk(g_mu);
    ++g_srv_paused;
    // Stop flags into the polled records, then the grid's stream drained:
    // when this returns no wave of the grid is left on any device.
    server_stop_all_locked();
    return WC_OK;
}

int wc_server_resume(void)
{
    std::lock_guard<FairMutex> lk(g_mu);
    if (g_srv_paused == 0)
        return WC_EINVAL;
    --g_srv_paused;
    return WC_OK;
}

int wc_server_stats(uint64_t *served, uint64_t *fallbacks, uint64_t *launches)
{
    std::lock_guard<FairMutex> lk(g_mu);
    if (served)
        *served = g_srv_stats.served;
    if (fallbacks)
        *fallbacks = g_srv_stats.fallbacks;
    if (launches)
        *launches = g_srv_stats.launches;
    return WC_OK;
}

} // extern "C"
