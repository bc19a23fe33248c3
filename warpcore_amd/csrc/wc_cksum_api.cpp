// wc_cksum_api.cpp -- the C ABI of libwccksum.so (include/warpcore_gpu/wc_cksum.h).
//
// Host-side runtime around the gfx950 kernels: device selection and
// per-device scratch, the launch planner (group shape + grid), the scalar
// drop-ins for the reference's ip_cksum / payload_cksum
// (/root/reference/lib/src/in_cksum.h:32-36), the device-resident batch calls
// and the pipelined host-memory path.  There is no CPU checksum anywhere in
// this library: if no gfx950 device is usable, batch calls return WC_ENODEV
// and the scalar drop-ins abort (the reference's die(), util.h:280-340).

#include "warpcore_gpu/wc_cksum.h"

#include "wc_cksum_kernels.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <string>

namespace {

constexpr int kMaxDevices = 64;
constexpr int kPipe = 3;                          // host-path pipeline depth
constexpr uint64_t kChunkBytes = 64ull << 20;     // host-path bytes per chunk
constexpr uint64_t kChunkPkts = 1ull << 20;       // host-path packets per chunk
constexpr uint64_t kScalarStage = 65536 + 64;     // one max-size packet

struct HostPipe {
    hipStream_t st[kPipe] = {};
    hipEvent_t done[kPipe] = {};
    uint8_t *d_bytes[kPipe] = {};
    uint64_t *d_off[kPipe] = {};
    uint16_t *d_len[kPipe] = {};
    uint16_t *d_out[kPipe] = {};
    uint8_t *h_bytes[kPipe] = {};  // pinned staging for unregistered input
    uint64_t *h_off[kPipe] = {};   // pinned, rebased offsets
    uint16_t *h_len[kPipe] = {};
    uint16_t *h_out[kPipe] = {};
    bool ready = false;
};

struct Device {
    bool ok = false;
    int cus = 0;
    hipStream_t scalar_st = nullptr;
    uint8_t *h_stage = nullptr;  // pinned + mapped scalar staging
    uint8_t *d_stage = nullptr;
    uint16_t *h_res = nullptr;
    uint16_t *d_res = nullptr;
    HostPipe pipe;
};

std::mutex g_mu;
Device g_dev[kMaxDevices];
std::map<uintptr_t, uint64_t> g_registered; // host base -> bytes

int hip_err(hipError_t e) { return e == hipSuccess ? WC_OK : -(int)e; }

int env_int(const char *name, int dflt)
{
    const char *v = getenv(name);
    return (v && *v) ? atoi(v) : dflt;
}

int current_device(int *dev)
{
    int d = 0;
    hipError_t e = hipGetDevice(&d);
    if (e != hipSuccess)
        return hip_err(e);
    if (d < 0 || d >= kMaxDevices)
        return WC_ENODEV;
    *dev = d;
    return WC_OK;
}

// Create per-device state (caller holds g_mu).
int init_locked(int device, Device **out)
{
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0)
        return WC_ENODEV;
    if (device >= 0) {
        if (device >= ndev || device >= kMaxDevices)
            return WC_EINVAL;
        hipError_t e = hipSetDevice(device);
        if (e != hipSuccess)
            return hip_err(e);
    } else {
        int rc = current_device(&device);
        if (rc)
            return rc;
    }
    Device &D = g_dev[device];
    if (!D.ok) {
        hipDeviceProp_t prop;
        hipError_t e = hipGetDeviceProperties(&prop, device);
        if (e != hipSuccess)
            return hip_err(e);
        if (strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
            fprintf(stderr, "wccksum: device %d is %s, this build targets gfx950\n",
                    device, prop.gcnArchName);
            return WC_ENODEV;
        }
        D.cus = prop.multiProcessorCount;
        e = hipStreamCreateWithFlags(&D.scalar_st, hipStreamNonBlocking);
        if (e != hipSuccess)
            return hip_err(e);
        e = hipHostMalloc((void **)&D.h_stage, kScalarStage,
                          hipHostMallocMapped | hipHostMallocCoherent);
        if (e != hipSuccess)
            return WC_ENOMEM;
        e = hipHostMalloc((void **)&D.h_res, 64,
                          hipHostMallocMapped | hipHostMallocCoherent);
        if (e != hipSuccess)
            return WC_ENOMEM;
        if (hipHostGetDevicePointer((void **)&D.d_stage, D.h_stage, 0) != hipSuccess ||
            hipHostGetDevicePointer((void **)&D.d_res, D.h_res, 0) != hipSuccess)
            return WC_ENOMEM;
        D.ok = true;
    }
    *out = &D;
    return WC_OK;
}

int ensure_device(Device **out)
{
    std::lock_guard<std::mutex> lk(g_mu);
    return init_locked(-1, out);
}

// ---------------------------------------------------------------------------
// Planner.

wc::Shape shape_for_chunks(uint32_t nch)
{
    // Smallest group covering the packet in one pass, with U packets per
    // group so every lane keeps ~4-18 16-byte loads in flight (tuned on
    // MI355X: DESIGN.md section 5, profiles/tune_r01_*.log).
    if (nch <= 4)
        return {4, 1, 8};
    if (nch <= 8)
        return {8, 1, 4};
    if (nch <= 16)
        return {16, 1, 4};
    if (nch <= 32)
        return {16, 2, 4};
    if (nch <= 48)
        return {16, 3, 4};
    if (nch <= 96)
        return {16, 6, 4};
    if (nch <= 128)
        return {32, 4, 1};
    if (nch <= 256)
        return {64, 4, 1};
    if (nch <= 576)
        return {32, 18, 1};
    return {64, 9, 1};
}

bool shape_override(wc::Shape *sh)
{
    const char *v = getenv("WC_SHAPE");
    if (!v || !*v)
        return false;
    int g = 0, c = 0, u = 0;
    if (sscanf(v, "%d,%d,%d", &g, &c, &u) != 3)
        return false;
    sh->group = g;
    sh->cpl = c;
    sh->unroll = u;
    return true;
}

int grid_for(const Device &D, const wc::Shape &sh, uint64_t n)
{
    const uint64_t ppw = (uint64_t)(64 / sh.group) * sh.unroll;
    const uint64_t waves = (n + ppw - 1) / ppw;
    const uint64_t blocks = (waves + 3) / 4;
    // One-shot grid by default: every block handles one wave-iteration per
    // wave and retires (measured faster than a resident grid-stride loop on
    // MI355X: DESIGN.md section 5).  WC_BLOCKS_PER_CU / WC_GRID cap it into a
    // grid-stride launch for experiments.
    uint64_t cap = 0x7FFFFFFFull;
    const int per_cu = env_int("WC_BLOCKS_PER_CU", 0);
    if (per_cu > 0)
        cap = (uint64_t)D.cus * (uint64_t)per_cu;
    const int fixed = env_int("WC_GRID", 0);
    if (fixed > 0)
        cap = (uint64_t)fixed;
    return (int)std::max<uint64_t>(1, std::min(blocks, cap));
}

struct Plan {
    wc::Shape shape;
    bool full;
    int grid;
};

Plan plan_strided(const Device &D, uint64_t base, uint64_t stride, uint32_t len,
                  uint64_t n, int kind)
{
    Plan p;
    const uint32_t span = kind == WC_CKSUM_PAYLOAD ? std::max(len, 20u) : len;
    // Worst-case start phase within a 16-byte chunk over the batch.
    const uint32_t phase = (stride % 16 == 0) ? (uint32_t)(base % 16) : 15u;
    const uint32_t nch = (phase + span + 15u) / 16u;
    p.shape = shape_for_chunks(nch);
    shape_override(&p.shape);
    p.full = kind == WC_CKSUM_IP && base % 16 == 0 && stride % 16 == 0 &&
             len % 16 == 0;
    p.grid = grid_for(D, p.shape, n);
    return p;
}

Plan plan_ragged(const Device &D, uint64_t n)
{
    (void)D;
    (void)n;
    Plan p;
    // The chunk-balanced flat kernel (group = 0 marks it; unroll = 64-chunk
    // rows per ping-pong group, WC_FLAT_UN overrides).
    p.shape = {0, 1, env_int("WC_FLAT_UN", 2)};
    p.full = false;
    p.grid = 0;
    return p;
}

bool nontemporal() { return env_int("WC_NT", 1) != 0; }
int flat_tpw() { return env_int("WC_FLAT_TPW", 1); }

int run(const Device &D, const wc::LaunchArgs &a, const Plan &p, hipStream_t st)
{
    (void)D;
    hipError_t e = p.shape.group == 0 ? wc::launch_flat(a, p.shape.unroll, st)
                                      : wc::launch_cksum(a, p.shape, p.grid, st);
    return hip_err(e);
}

int batch_strided(const void *d_base, uint64_t stride, uint16_t len, uint64_t n,
                  uint16_t *d_out, uint64_t *d_bad, int kind, void *stream,
                  uint16_t *d_out_hdr = nullptr)
{
    if (kind != WC_CKSUM_IP && kind != WC_CKSUM_PAYLOAD)
        return WC_EINVAL;
    if (n == 0)
        return WC_OK;
    if (!d_base || (!d_out && !d_bad))
        return WC_EINVAL;
    Device *D = nullptr;
    int rc = ensure_device(&D);
    if (rc)
        return rc;
    const Plan p = plan_strided(*D, (uint64_t)d_base, stride, len, n, kind);
    wc::LaunchArgs a{d_base, stride, len,  nullptr,  nullptr, n,
                     d_out,  d_bad,  kind, false,    p.full,  nontemporal(),
                     0,      d_out_hdr};
    return run(*D, a, p, (hipStream_t)stream);
}

int batch_ragged(const void *d_base, const uint64_t *d_off, const uint16_t *d_len,
                 uint64_t n, uint16_t *d_out, uint64_t *d_bad, int kind,
                 void *stream, uint16_t *d_out_hdr = nullptr)
{
    if (kind != WC_CKSUM_IP && kind != WC_CKSUM_PAYLOAD)
        return WC_EINVAL;
    if (n == 0)
        return WC_OK;
    if (!d_base || !d_off || !d_len || (!d_out && !d_bad))
        return WC_EINVAL;
    Device *D = nullptr;
    int rc = ensure_device(&D);
    if (rc)
        return rc;
    const Plan p = plan_ragged(*D, n);
    wc::LaunchArgs a{d_base, 0,     0,    d_off, d_len, n,
                     d_out,  d_bad, kind, true,  false, nontemporal(), flat_tpw(),
                     d_out_hdr, env_int("WC_DIAG_NOLOAD", 0) != 0};
    return run(*D, a, p, (hipStream_t)stream);
}

[[noreturn]] void die(const char *what, int rc)
{
    fprintf(stderr, "wccksum: %s failed: %s (%d)\n", what, wc_strerror(rc), rc);
    abort();
}

uint16_t scalar_cksum(const void *buf, uint16_t len, int kind, const char *who)
{
    std::lock_guard<std::mutex> lk(g_mu);
    Device *D = nullptr;
    int rc = init_locked(-1, &D);
    if (rc)
        die(who, rc);
    // payload_cksum reads the IPv4 header fields up to byte 19 whatever len is
    // (in_cksum.c:149-151); stage the same bytes the reference reads.
    const size_t span =
        kind == WC_CKSUM_PAYLOAD ? std::max<size_t>(len, 20) : (size_t)len;
    memcpy(D->h_stage, buf, span);
    Plan p = plan_strided(*D, (uint64_t)D->d_stage, 0, len, 1, kind);
    wc::LaunchArgs a{D->d_stage, 0,   len,  nullptr, nullptr, 1,
                     D->d_res,   nullptr, kind, false,   p.full,  false};
    rc = run(*D, a, p, D->scalar_st);
    if (rc)
        die(who, rc);
    hipError_t e = hipStreamSynchronize(D->scalar_st);
    if (e != hipSuccess)
        die(who, hip_err(e));
    return *(volatile uint16_t *)D->h_res;
}

// ---------------------------------------------------------------------------
// Host-memory pipeline.

int pipe_init_locked(Device &D)
{
    HostPipe &P = D.pipe;
    if (P.ready)
        return WC_OK;
    for (int s = 0; s < kPipe; ++s) {
        if (hipStreamCreateWithFlags(&P.st[s], hipStreamNonBlocking) != hipSuccess ||
            hipEventCreateWithFlags(&P.done[s], hipEventDisableTiming) != hipSuccess)
            return WC_ENOMEM;
        if (hipMalloc((void **)&P.d_bytes[s], kChunkBytes + 64) != hipSuccess ||
            hipMalloc((void **)&P.d_off[s], kChunkPkts * 8) != hipSuccess ||
            hipMalloc((void **)&P.d_len[s], kChunkPkts * 2) != hipSuccess ||
            hipMalloc((void **)&P.d_out[s], kChunkPkts * 2) != hipSuccess)
            return WC_ENOMEM;
        if (hipHostMalloc((void **)&P.h_bytes[s], kChunkBytes + 64, 0) != hipSuccess ||
            hipHostMalloc((void **)&P.h_off[s], kChunkPkts * 8, 0) != hipSuccess ||
            hipHostMalloc((void **)&P.h_len[s], kChunkPkts * 2, 0) != hipSuccess ||
            hipHostMalloc((void **)&P.h_out[s], kChunkPkts * 2, 0) != hipSuccess)
            return WC_ENOMEM;
    }
    P.ready = true;
    return WC_OK;
}

bool is_registered_locked(const void *p, uint64_t bytes)
{
    const uintptr_t a = (uintptr_t)p;
    auto it = g_registered.upper_bound(a);
    if (it == g_registered.begin())
        return false;
    --it;
    return a >= it->first && a + bytes <= it->first + it->second;
}

} // namespace

// ===========================================================================
// Exported C ABI.

extern "C" {

uint16_t ip_cksum(const void *buf, uint16_t len)
{
    return scalar_cksum(buf, len, WC_CKSUM_IP, "ip_cksum");
}

uint16_t payload_cksum(const void *buf, uint16_t len)
{
    return scalar_cksum(buf, len, WC_CKSUM_PAYLOAD, "payload_cksum");
}

int wc_cksum_strided(const void *d_base, uint64_t stride, uint16_t len,
                     uint64_t n, uint16_t *d_out, int kind, void *stream)
{
    if (!d_out && n)
        return WC_EINVAL;
    return batch_strided(d_base, stride, len, n, d_out, nullptr, kind, stream);
}

int wc_cksum_ragged(const void *d_base, const uint64_t *d_off,
                    const uint16_t *d_len, uint64_t n, uint16_t *d_out,
                    int kind, void *stream)
{
    if (!d_out && n)
        return WC_EINVAL;
    return batch_ragged(d_base, d_off, d_len, n, d_out, nullptr, kind, stream);
}

int wc_verify_strided(const void *d_base, uint64_t stride, uint16_t len,
                      uint64_t n, uint16_t *d_out, uint64_t *d_bad, int kind,
                      void *stream)
{
    if (!d_bad && n)
        return WC_EINVAL;
    return batch_strided(d_base, stride, len, n, d_out, d_bad, kind, stream);
}

int wc_verify_ragged(const void *d_base, const uint64_t *d_off,
                     const uint16_t *d_len, uint64_t n, uint16_t *d_out,
                     uint64_t *d_bad, int kind, void *stream)
{
    if (!d_bad && n)
        return WC_EINVAL;
    return batch_ragged(d_base, d_off, d_len, n, d_out, d_bad, kind, stream);
}

int wc_cksum_ip_udp_strided(const void *d_base, uint64_t stride, uint16_t len,
                            uint64_t n, uint16_t *d_out_ip_hdr,
                            uint16_t *d_out_payload, void *stream)
{
    if (n && (!d_out_ip_hdr || !d_out_payload))
        return WC_EINVAL;
    return batch_strided(d_base, stride, len, n, d_out_payload, nullptr,
                         WC_CKSUM_PAYLOAD, stream, d_out_ip_hdr);
}

int wc_cksum_ip_udp_ragged(const void *d_base, const uint64_t *d_off,
                           const uint16_t *d_len, uint64_t n, uint16_t *d_out_ip_hdr,
                           uint16_t *d_out_payload, void *stream)
{
    if (n && (!d_out_ip_hdr || !d_out_payload))
        return WC_EINVAL;
    return batch_ragged(d_base, d_off, d_len, n, d_out_payload, nullptr,
                        WC_CKSUM_PAYLOAD, stream, d_out_ip_hdr);
}

int wc_host_register(void *h_ptr, uint64_t bytes)
{
    if (!h_ptr || !bytes)
        return WC_EINVAL;
    std::lock_guard<std::mutex> lk(g_mu);
    Device *D = nullptr;
    int rc = init_locked(-1, &D);
    if (rc)
        return rc;
    hipError_t e = hipHostRegister(h_ptr, bytes, hipHostRegisterDefault);
    if (e != hipSuccess)
        return hip_err(e);
    g_registered[(uintptr_t)h_ptr] = bytes;
    return WC_OK;
}

int wc_host_unregister(void *h_ptr)
{
    if (!h_ptr)
        return WC_EINVAL;
    std::lock_guard<std::mutex> lk(g_mu);
    auto it = g_registered.find((uintptr_t)h_ptr);
    if (it == g_registered.end())
        return WC_EINVAL;
    g_registered.erase(it);
    return hip_err(hipHostUnregister(h_ptr));
}

int wc_cksum_host(const void *h_base, uint64_t h_bytes, const uint64_t *h_off,
                  const uint16_t *h_len, uint64_t n, uint16_t *h_out, int kind)
{
    if (kind != WC_CKSUM_IP && kind != WC_CKSUM_PAYLOAD)
        return WC_EINVAL;
    if (n == 0)
        return WC_OK;
    if (!h_base || !h_off || !h_len || !h_out)
        return WC_EINVAL;

    std::lock_guard<std::mutex> lk(g_mu);
    Device *D = nullptr;
    int rc = init_locked(-1, &D);
    if (rc)
        return rc;
    rc = pipe_init_locked(*D);
    if (rc)
        return rc;
    HostPipe &P = D->pipe;
    const bool direct = is_registered_locked(h_base, h_bytes);
    const uint8_t *hb = (const uint8_t *)h_base;

    // Bytes each packet needs (payload_cksum reads >= 20 header bytes).
    auto span_of = [kind](uint16_t l) -> uint64_t {
        return kind == WC_CKSUM_PAYLOAD ? std::max<uint64_t>(l, 20) : l;
    };

    // Pipeline over chunks of packets listed in ascending address order; a
    // chunk is the byte range its packets cover.
    uint64_t i = 0;
    int slot = 0;
    uint64_t pend_lo[kPipe] = {}, pend_n[kPipe] = {};
    bool pend[kPipe] = {};
    auto drain = [&](int s) -> int {
        if (!pend[s])
            return WC_OK;
        hipError_t e = hipEventSynchronize(P.done[s]);
        if (e != hipSuccess)
            return hip_err(e);
        memcpy(h_out + pend_lo[s], P.h_out[s], pend_n[s] * 2);
        pend[s] = false;
        return WC_OK;
    };

    while (i < n) {
        rc = drain(slot);
        if (rc)
            return rc;
        const uint64_t lo = h_off[i];
        uint64_t hi = lo, j = i;
        while (j < n && j - i < kChunkPkts) {
            const uint64_t o = h_off[j];
            const uint64_t e = o + span_of(h_len[j]);
            if (o < lo || e > h_bytes) // descending order or out of range
                return WC_EINVAL;
            if (std::max(hi, e) - lo > kChunkBytes) {
                if (j == i)
                    return WC_EINVAL;
                break;
            }
            hi = std::max(hi, e);
            ++j;
        }
        const uint64_t cnt = j - i, bytes = hi - lo;
        for (uint64_t k = 0; k < cnt; ++k) {
            P.h_off[slot][k] = h_off[i + k] - lo;
            P.h_len[slot][k] = h_len[i + k];
        }
        hipStream_t st = P.st[slot];
        const uint8_t *src = hb + lo;
        if (!direct) {
            memcpy(P.h_bytes[slot], src, bytes);
            src = P.h_bytes[slot];
        }
        hipError_t e = hipMemcpyAsync(P.d_bytes[slot], src, bytes,
                                      hipMemcpyHostToDevice, st);
        if (e == hipSuccess)
            e = hipMemcpyAsync(P.d_off[slot], P.h_off[slot], cnt * 8,
                               hipMemcpyHostToDevice, st);
        if (e == hipSuccess)
            e = hipMemcpyAsync(P.d_len[slot], P.h_len[slot], cnt * 2,
                               hipMemcpyHostToDevice, st);
        if (e != hipSuccess)
            return hip_err(e);
        const Plan p = plan_ragged(*D, cnt);
        wc::LaunchArgs a{P.d_bytes[slot], 0,    0,    P.d_off[slot], P.d_len[slot],
                         cnt,             P.d_out[slot], nullptr, kind, true,
                         false,           nontemporal(), flat_tpw()};
        rc = run(*D, a, p, st);
        if (rc)
            return rc;
        e = hipMemcpyAsync(P.h_out[slot], P.d_out[slot], cnt * 2,
                           hipMemcpyDeviceToHost, st);
        if (e == hipSuccess)
            e = hipEventRecord(P.done[slot], st);
        if (e != hipSuccess)
            return hip_err(e);
        pend[slot] = true;
        pend_lo[slot] = i;
        pend_n[slot] = cnt;
        i = j;
        slot = (slot + 1) % kPipe;
    }
    for (int s = 0; s < kPipe; ++s) {
        rc = drain((slot + s) % kPipe);
        if (rc)
            return rc;
    }
    return WC_OK;
}

int wc_gpu_init(int device)
{
    std::lock_guard<std::mutex> lk(g_mu);
    Device *D = nullptr;
    return init_locked(device, &D);
}

int wc_gpu_fini(void)
{
    std::lock_guard<std::mutex> lk(g_mu);
    for (auto &D : g_dev) {
        if (!D.ok)
            continue;
        HostPipe &P = D.pipe;
        if (P.ready) {
            for (int s = 0; s < kPipe; ++s) {
                (void)hipStreamSynchronize(P.st[s]);
                (void)hipFree(P.d_bytes[s]);
                (void)hipFree(P.d_off[s]);
                (void)hipFree(P.d_len[s]);
                (void)hipFree(P.d_out[s]);
                (void)hipHostFree(P.h_bytes[s]);
                (void)hipHostFree(P.h_off[s]);
                (void)hipHostFree(P.h_len[s]);
                (void)hipHostFree(P.h_out[s]);
                (void)hipEventDestroy(P.done[s]);
                (void)hipStreamDestroy(P.st[s]);
            }
            P = HostPipe{};
        }
        (void)hipStreamSynchronize(D.scalar_st);
        (void)hipStreamDestroy(D.scalar_st);
        (void)hipHostFree(D.h_stage);
        (void)hipHostFree(D.h_res);
        D = Device{};
    }
    return WC_OK;
}

int wc_synth_fill(void *d_buf, uint64_t nbytes, uint64_t seed, void *stream)
{
    if (!nbytes)
        return WC_OK;
    if (!d_buf || ((uintptr_t)d_buf & 15u))
        return WC_EINVAL;
    Device *D = nullptr;
    int rc = ensure_device(&D);
    if (rc)
        return rc;
    const uint64_t threads = (nbytes / 16) + 1;
    const int grid = (int)std::min<uint64_t>((threads + 255) / 256,
                                             (uint64_t)D->cus * 8);
    return hip_err(wc::launch_synth(d_buf, nbytes, seed, grid, (hipStream_t)stream));
}

int wc_plan_strided(uint64_t base_addr, uint64_t stride, uint16_t len,
                    uint64_t n, int kind, int *group, int *chunks_per_lane,
                    int *unroll, int *grid)
{
    if (kind != WC_CKSUM_IP && kind != WC_CKSUM_PAYLOAD)
        return WC_EINVAL;
    Device *D = nullptr;
    int rc = ensure_device(&D);
    if (rc)
        return rc;
    const Plan p = plan_strided(*D, base_addr, stride, len, n, kind);
    if (group)
        *group = p.shape.group;
    if (chunks_per_lane)
        *chunks_per_lane = p.shape.cpl;
    if (unroll)
        *unroll = p.shape.unroll;
    if (grid)
        *grid = p.grid;
    return WC_OK;
}

const char *wc_strerror(int err)
{
    switch (err) {
    case WC_OK:
        return "success";
    case WC_EINVAL:
        return "invalid argument";
    case WC_ENODEV:
        return "no usable gfx950 device";
    case WC_ENOMEM:
        return "out of memory";
    default:
        if (err < 0 && err > -10000)
            return hipGetErrorString((hipError_t)(-err));
        return "unknown error";
    }
}

const char *wc_version(void) { return "wccksum 0.1.0 (gfx950)"; }

} // extern "C"
