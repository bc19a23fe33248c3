// wc_k_serve.hip -- the resident small-batch server on gfx950: a persistent
// grid that serves wc_cksum_host / wc_rx_verdict_host calls on small batches
// in a registered (page-locked, mapped) host region without a kernel launch,
// a stream synchronisation or any copy per call (DESIGN.md section 5,
// "Small host batches").
//
// The reference's batch points hand over one netmap ring or one w_iov_sq at a
// time (backend_netmap.c:348-358 TX, 379-391 RX): tens of packets, where a
// launch + completion round trip (~15-20 us) costs more than one CPU core's
// checksum.  Here the kernel stays resident between calls:
//   * the host writes one 16-byte record per packet into mapped pinned memory
//     (device address of the packet in the registered region, its length, the
//     kind, and the request number `seq`, stored last);
//   * wave w (one 64-lane workgroup per wave, W of them) polls record w with
//     a cache-bypassing load; when its seq changes, it takes packets w, w + W,
//     w + 2W, ... while their records carry the same seq (the host writes
//     records from the last to the first, so those are already visible);
//   * per packet the whole wave loads the packet's chunks straight out of the
//     host region over PCIe (after one system-scope acquire per request, which
//     invalidates this CU's caches), sums them exactly as the group kernel's
//     64-lane groups do (byte-lane sums, in_cksum.c:107-167), and stores
//     {result, seq} to the packet's 8-byte result slot in mapped host memory
//     with one system-scope store;
//   * the host spins on the n result slots.
// Kinds: ip_cksum, payload_cksum, the RX verdict of an Ethernet frame
// (eth_rx -> ip4_rx / ip6_rx -> udp_rx: eth.c:75-86, ip4.c:95-138,
// ip6.c:91-111, udp.c:99-139; the same decisions, in the same order, as
// k_rx_verdict and oracle_rx_verdict), and the fused TX pair --
// payload_cksum and the IPv4 header's ip_cksum of one packet from one read
// of its bytes (mk_ip4_hdr + udp_tx, ip4.c:184-186, udp.c:209-213).
// Exit: every wave leaves when its record carries the stop flag (the host's
// idle watcher, wc_gpu_fini, a host-side restart set it), or once the wall
// clock has run `idle_ticks` past the last request ANY wave saw: a wave whose
// own records stayed quiet re-reads the host's heartbeat word (the latest
// request number) before it leaves, so light traffic that never reaches a
// wave does not thin the grid out -- the grid drains as a whole, and always
// drains.
#include "wc_device.h"

namespace wc {
namespace {

// enum wc_rx_verdict (wc_cksum.h)
constexpr uint32_t kSvOk = 0, kSvOkNoCksum = 1, kSvBadIpCksum = 2, kSvBadUdpCksum = 3,
                   kSvShort = 4, kSvFragment = 5, kSvBadVersion = 6, kSvNotUdp = 7,
                   kSvNotIp = 8, kSvTruncated = 9;

constexpr int kSvLoads = 4; // chunk loads per lane: 256 chunks cover any packet of kSrvMaxBytes
static_assert((15u + kSrvMaxBytes + 15u) / 16u <= 64u * kSvLoads, "server packet size");

// 16 bytes of host memory past every cache (sc0 sc1): the poll of a record.
__device__ __forceinline__ u32x4 load_sys16(const void *p)
{
    u32x4 v;
    asm volatile("global_load_dwordx4 %0, %1, off sc0 sc1\n\ts_waitcnt vmcnt(0)"
                 : "=v"(v)
                 : "v"(p)
                 : "memory");
    return v;
}

// One host word past every cache: the heartbeat.
__device__ __forceinline__ uint32_t load_sys4(const uint32_t *p)
{
    uint32_t v;
    asm volatile("global_load_dword %0, %1, off sc0 sc1\n\ts_waitcnt vmcnt(0)"
                 : "=v"(v)
                 : "v"(p)
                 : "memory");
    return (uint32_t)__builtin_amdgcn_readfirstlane((int)v);
}

struct Rec {
    uint64_t addr;
    uint32_t len, kind, stop, seq, n; // n: the request's packet count
};

__device__ __forceinline__ void rec_addr(Rec &x, uint32_t lo, uint32_t hi)
{
    x.addr = (uint64_t)lo | ((uint64_t)(hi & ((1u << (kSrvAddrBits - 32)) - 1u)) << 32);
    x.n = hi >> (kSrvAddrBits - 32);
}

__device__ __forceinline__ Rec rec_load(const SrvRec *r)
{
    u32x4 v = load_sys16(r);
    // every lane loaded the same record: make it wave-uniform (SGPRs)
    v.x = (uint32_t)__builtin_amdgcn_readfirstlane((int)v.x);
    v.y = (uint32_t)__builtin_amdgcn_readfirstlane((int)v.y);
    v.z = (uint32_t)__builtin_amdgcn_readfirstlane((int)v.z);
    v.w = (uint32_t)__builtin_amdgcn_readfirstlane((int)v.w);
    Rec x;
    rec_addr(x, v.x, v.y);
    x.len = v.z & 0xFFFFu;
    x.kind = (v.z >> 16) & 0xFFu;
    x.stop = v.z >> 24;
    x.seq = v.w;
    return x;
}

// The packet's (frame's) chunks, whole-wave: lane l holds chunks l + 64 j.
// Only chunks overlapping [a, a + span) are loaded (others: the zero chunk).
__device__ __forceinline__ void sv_load(uint64_t a, uint32_t span, int lane, u32x4 (&d)[kSvLoads])
{
    const uint64_t c0 = a & ~15ull;
    const uint32_t nch = span ? ((uint32_t)(a & 15u) + span + 15u) >> 4 : 0u;
    const uint64_t zero = (uint64_t)(uintptr_t)&kZeroChunk;
#pragma unroll
    for (int j = 0; j < kSvLoads; ++j) {
        const uint32_t k = (uint32_t)lane + 64u * j;
        d[j] = load_chunk<false>(k < nch ? c0 + 16ull * k : zero);
    }
}

// Byte o of the packet from lane-held chunks (o uniform and s + o < 1024:
// the chunk sits in d[0] of lane (s + o) >> 4): one v_readlane, no LDS round
// trip -- the RX parse reads a dozen header bytes one after the other.
__device__ __forceinline__ uint32_t sv_byte(const u32x4 (&d)[kSvLoads], uint32_t s, uint32_t o)
{
    const uint32_t pos = (uint32_t)__builtin_amdgcn_readfirstlane((int)(s + o));
    const uint32_t j = (pos >> 2) & 3u;
    const uint32_t dw = j == 0 ? d[0].x : j == 1 ? d[0].y : j == 2 ? d[0].z : d[0].w;
    const uint32_t v = (uint32_t)__builtin_amdgcn_readlane((int)dw, (int)(pos >> 4));
    return (v >> (8u * (pos & 3u))) & 0xFFu;
}

// Exact sum (reference accumulator, mod 2^32) of packet bytes [rs, re) --
// plus, for payload_cksum, the pseudo-header fields of a v4 / v6 header
// (in_cksum.c:140-167) -- over chunks that start s bytes before the packet
// (s < 32: an IP header 14 bytes into a frame).  A chunk wholly before the
// packet adds nothing; its offset is clamped to -16, where accum_arith's
// masks are defined and give it no byte.
template <int KIND>
__device__ __forceinline__ uint32_t sv_sum(const u32x4 (&d)[kSvLoads], uint32_t s, int lane,
                                           int rs, int re, uint32_t v4, bool odd)
{
    uint32_t E = 0, O = 0;
#pragma unroll
    for (int j = 0; j < kSvLoads; ++j)
        accum_arith<KIND>(d[j], max(16 * (lane + 64 * j) - (int)s, -16), rs, re, v4, E, O);
    return group_sum<64>(combine(E, O, odd));
}

// Bytes a packet's check reads: payload_cksum reads the IPv4 header fields
// up to byte 19 whatever len is (in_cksum.c:149-151); an RX frame its length.
__device__ __forceinline__ uint32_t sv_span(uint32_t len, uint32_t kind)
{
    return kind == WC_KIND_PAYLOAD || kind == kSrvKindFused ? max(len, 20u) : len;
}

// ip_cksum / payload_cksum of [a, a + len) (in_cksum.c:133-167) from its
// loaded chunks.
__device__ __forceinline__ uint32_t sv_cksum(const u32x4 (&d)[kSvLoads], uint64_t a, uint32_t len,
                                             uint32_t kind, int lane)
{
    const uint32_t s = (uint32_t)__builtin_amdgcn_readfirstlane((int)(a & 15u));
    if (kind != WC_KIND_PAYLOAD)
        return fold_not(sv_sum<WC_KIND_IP>(d, s, lane, 0, (int)len, 0u, a & 1u));
    const PseudoHdr ph =
        pseudo_hdr(sv_byte(d, s, 0), sv_byte(d, s, 2), sv_byte(d, s, 3), sv_byte(d, s, 6));
    return fold_not(sv_sum<WC_KIND_PAYLOAD>(d, s, lane, (int)ph.hl, (int)len, ph.v4, a & 1u) +
                    ph.special);
}

// The fused TX pair of packet [a, a + len): payload_cksum(pkt, len) in the
// low half, ip_cksum(pkt, hl) of an IPv4 header in the high half (0 for
// IPv6, which has no header checksum) -- what mk_ip4_hdr and udp_tx store
// (ip4.c:184-186, udp.c:209-213).  An IPv4 header longer than the bytes
// loaded with the packet (options past a short len) is loaded again on its
// own (rare: the host checked [a, a + hl) lies in the region).
__device__ __forceinline__ uint32_t sv_fused(const u32x4 (&d)[kSvLoads], uint64_t a, uint32_t len,
                                             int lane)
{
    const uint32_t s = (uint32_t)__builtin_amdgcn_readfirstlane((int)(a & 15u));
    const PseudoHdr ph =
        pseudo_hdr(sv_byte(d, s, 0), sv_byte(d, s, 2), sv_byte(d, s, 3), sv_byte(d, s, 6));
    const uint32_t pay = fold_not(
        sv_sum<WC_KIND_PAYLOAD>(d, s, lane, (int)ph.hl, (int)len, ph.v4, a & 1u) + ph.special);
    if (!ph.v4)
        return pay;
    uint32_t hs;
    if (ph.hl <= max(len, 20u)) {
        hs = sv_sum<WC_KIND_IP>(d, s, lane, 0, (int)ph.hl, 0u, a & 1u);
    } else {
        u32x4 e[kSvLoads];
        sv_load(a, ph.hl, lane, e);
        hs = sv_sum<WC_KIND_IP>(e, s, lane, 0, (int)ph.hl, 0u, a & 1u);
    }
    return pay | ((uint32_t)fold_not(hs) << 16);
}

// The RX verdict of frame [fa, fa + flen), the reference's check order
// (oracle_rx_verdict, k_rx_verdict): only bytes inside the frame are used.
__device__ __forceinline__ uint32_t sv_rx(const u32x4 (&d)[kSvLoads], uint64_t fa, uint32_t flen,
                                          int lane)
{
    const uint32_t s = (uint32_t)__builtin_amdgcn_readfirstlane((int)(fa & 15u));
    auto B = [&](uint32_t o) { return sv_byte(d, s, o); };
    if (flen < 14u)
        return kSvTruncated;
    const uint32_t type = (B(12) << 8) | B(13); // eth.c:75-86
    if (type != 0x0800u && type != 0x86DDu)
        return kSvNotIp;
    const uint32_t room = flen - 14u;
    if (room < 1u)
        return kSvTruncated;
    const bool v4 = type == 0x0800u;
    const uint32_t b0 = B(14);
    if ((b0 >> 4) != (v4 ? 4u : 6u)) // ip4.c:95-98, ip6.c:91-95
        return kSvBadVersion;
    const uint64_t ip = fa + 14u;
    const uint32_t si = s + 14u; // the IP header's position in the chunk stream
    uint32_t hl, ip_plen, proto;
    if (v4) {
        hl = (b0 & 15u) * 4u;
        if (room < max(hl, 20u))
            return kSvTruncated;
        // ip_cksum(ip, hl) (ip4.c:110-115)
        if (fold_not(sv_sum<WC_KIND_IP>(d, si, lane, 0, (int)hl, 0u, ip & 1u)) != 0)
            return kSvBadIpCksum;
        if ((B(20) & 0x1Fu) || B(21)) // ip->off & IP4_OFFMASK (ip4.c:123-127)
            return kSvFragment;
        proto = B(23);
        ip_plen = (((B(16) << 8) | B(17)) - hl) & 0xFFFFu; // udp.c:104
    } else {
        hl = 40u;
        if (room < 40u)
            return kSvTruncated;
        proto = B(20);                    // next_hdr (ip6.c:105)
        ip_plen = (B(18) << 8) | B(19);   // udp.c:114
    }
    if (proto != 17u)
        return kSvNotUdp;
    if (ip_plen < 8u) // udp.c:123-126
        return kSvShort;
    if (room < hl + 8u)
        return kSvTruncated;
    const uint32_t u = 14u + hl; // the UDP header
    const uint32_t ulen = (B(u + 4) << 8) | B(u + 5);
    const uint32_t udp_len = min(ulen, ip_plen); // udp.c:128
    if (B(u + 6) == 0u && B(u + 7) == 0u)       // udp.c:132
        return kSvOkNoCksum;
    const uint32_t plen = udp_len + hl;
    if (room < max(plen, 20u))
        return kSvTruncated;
    // payload_cksum(ip, udp_len + hl) (udp.c:134)
    const PseudoHdr ph = pseudo_hdr(b0, B(16), B(17), B(20));
    const uint32_t S =
        sv_sum<WC_KIND_PAYLOAD>(d, si, lane, (int)ph.hl, (int)plen, ph.v4, ip & 1u) + ph.special;
    return fold_not(S) != 0 ? kSvBadUdpCksum : kSvOk;
}

__global__ void __launch_bounds__(64) k_serve(const SrvRec *__restrict__ recs,
                                              SrvRes *__restrict__ res,
                                              const uint32_t *__restrict__ hb, uint32_t seq0,
                                              uint64_t idle_ticks)
{
    const int lane = threadIdx.x;
    const uint32_t w = blockIdx.x, W = gridDim.x;
    uint32_t last = seq0, hb_seen = seq0;
    uint64_t t_last = (uint64_t)wall_clock64();
    for (;;) {
        Rec r = rec_load(&recs[w]);
        if (r.stop)
            return;
        if (r.seq == last) {
            const uint64_t now = (uint64_t)wall_clock64();
            if (now - t_last > idle_ticks) {
                // Quiet for idle_ticks here; leave only if the whole grid
                // was (no request since this wave last looked), else keep
                // serving: a wave that exits while the others stay would
                // leave its share of a later, larger request unanswered.
                const uint32_t h = load_sys4(hb);
                if (h == hb_seen)
                    return;
                hb_seen = h;
                t_last = now;
            }
            __builtin_amdgcn_s_sleep(2);
            continue;
        }
        // A new request: one system-scope acquire (invalidates this CU's
        // caches), then the packets' bytes are read fresh from host memory.
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
        const uint32_t seq = r.seq;
        // This wave's packets are w + j W, j = 0, 1, ...: their records are
        // fetched 64 at a time in one load (lane i reads the record of packet
        // j0 + 1 + i); the host wrote them all before record w, so they are
        // current when w is.  Two packets are processed at a time, both
        // packets' loads in flight before either is summed.
        Rec r0 = r;
        uint32_t j = 0;
        for (bool more = true; more;) {
            const uint32_t j0 = j; // r0 is packet j0's record
            const uint32_t kx = w + (j0 + 1u + (uint32_t)lane) * W;
            // (two 8-byte system-scope loads the compiler waits for only at
            // first use: in flight with packet j0's loads; records written
            // before the one already seen need no single-snapshot load)
            // Only this wave's packets of the request are read: n (in every
            // record) gives their count, so a request of n <= W packets reads
            // no further record at all.
            const uint32_t nrec = r.n > w ? (r.n - w + W - 1u) / W : 0u;
            uint64_t rlo = 0, rhi = 0;
            if (j0 + 1u + (uint32_t)lane < nrec && kx < kSrvMaxPkts) {
                const uint64_t *rp = (const uint64_t *)&recs[kx];
                rlo = __hip_atomic_load(rp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                rhi = __hip_atomic_load(rp + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            }
            const u32x4 rv = {(uint32_t)rlo, (uint32_t)(rlo >> 32), (uint32_t)rhi,
                              (uint32_t)(rhi >> 32)};
            auto rec_at = [&](uint32_t jj) { // packet jj's record, j0 < jj <= j0 + 64
                Rec x;
                const int l = (int)(jj - j0 - 1u);
                rec_addr(x, (uint32_t)__builtin_amdgcn_readlane((int)rv.x, l),
                         (uint32_t)__builtin_amdgcn_readlane((int)rv.y, l));
                const uint32_t z = (uint32_t)__builtin_amdgcn_readlane((int)rv.z, l);
                x.len = z & 0xFFFFu;
                x.kind = (z >> 16) & 0xFFu;
                x.stop = z >> 24;
                x.seq = jj < nrec && w + jj * W < kSrvMaxPkts
                            ? (uint32_t)__builtin_amdgcn_readlane((int)rv.w, l) : ~seq;
                return x;
            };
            more = false;
            while (r0.seq == seq) {
                u32x4 d0[kSvLoads], d1[kSvLoads];
                sv_load(r0.addr, sv_span(r0.len, r0.kind), lane, d0);
                const bool last_in_batch = j == j0 + 64u; // r1 would need the next batch
                const Rec r1 = last_in_batch ? Rec{0, 0, 0, 0, ~seq, 0} : rec_at(j + 1u);
                const bool two = r1.seq == seq;
                if (two)
                    sv_load(r1.addr, sv_span(r1.len, r1.kind), lane, d1);
                auto answer = [&](const Rec &x, const u32x4 (&d)[kSvLoads], uint32_t k) {
                    const uint32_t v = x.kind == kSrvKindRx      ? sv_rx(d, x.addr, x.len, lane)
                                       : x.kind == kSrvKindFused ? sv_fused(d, x.addr, x.len, lane)
                                                                 : sv_cksum(d, x.addr, x.len,
                                                                            x.kind, lane);
                    if (lane == 0)
                        __hip_atomic_store((uint64_t *)&res[k],
                                           (uint64_t)v | ((uint64_t)seq << 32), __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_SYSTEM);
                };
                answer(r0, d0, w + j * W);
                if (last_in_batch) { // packet j + 1's record is in the next batch
                    j += 1u;
                    more = w + j * W < kSrvMaxPkts;
                    if (more)
                        r0 = rec_load(&recs[w + j * W]);
                    break;
                }
                if (!two)
                    break;
                answer(r1, d1, w + (j + 1u) * W);
                j += 2u;
                if (j > j0 + 64u) { // both of packets j0 + 63, j0 + 64 done
                    more = w + j * W < kSrvMaxPkts;
                    if (more)
                        r0 = rec_load(&recs[w + j * W]);
                    break;
                }
                r0 = rec_at(j);
            }
        }
        last = seq;
        t_last = (uint64_t)wall_clock64();
    }
}

} // namespace

hipError_t launch_serve(const SrvRec *d_recs, SrvRes *d_res, const uint32_t *d_hb, uint32_t seq0,
                        int waves, uint64_t idle_ticks, hipStream_t st)
{
    hipLaunchKernelGGL(k_serve, dim3(waves), dim3(64), 0, st, d_recs, d_res, d_hb, seq0,
                       idle_ticks);
    return hipGetLastError();
}

} // namespace wc
