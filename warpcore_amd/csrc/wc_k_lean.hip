// wc_k_lean.hip -- aligned strided batches whose packets fit one pass of the
// group: the lean group kernel k_cksum_lean.
//
// Preconditions (wc_cksum_api.cpp plan_strided): base, stride and len are
// multiples of 16, len / 16 <= G * CPL, PPW * stride < 2^32, and for
// payload_cksum len >= 48.  Every chunk is then a whole 16-byte chunk of one
// packet, every packet starts at an even address, and the reference's
// accumulator is a plain word sum:
//   ip_cksum       V = the little-endian words of [0, len)      (in_cksum.c:107-120)
//   payload_cksum  V = words of [8, len) + per-packet terms      (in_cksum.c:140-164)
// where the per-packet terms (payload_as_ip in wc_flat.h: IPv4 with IHL 5
// minus bytes 8..11 plus proto << 8, IPv6 plus the payload-length word,
// then the plen re-swap / next_hdr << 24) come from the packet's first chunk,
// which the group's lane 0 holds -- no cross-lane header exchange.  A packet
// those terms do not cover (IPv4 with options or IHL < 5) is recomputed
// exactly by the lane that stores its result (lane_payload_exact).
//
// What makes it lean: the wave's first packet address is scalar (SGPRs) and
// each lane's chunk a 32-bit offset from it, so the prologue before the
// first load is mostly scalar; 4 v_dot2 per chunk instead of 8 v_dot4
// byte-lane sums; no masks unless the tail wave or a pass the packet does
// not fill needs them (the planner picks shapes the packet fills).  Tiny packets are the case it
// is for: C3 64 B spends most of a wave's life before its first load and
// after its last (profiles/ab_r02_lane_store.log).
#include "wc_seg.h"

namespace wc {
namespace {

typedef const uint8_t __attribute__((address_space(1))) *gbyte_ptr;

template <bool NT>
__device__ __forceinline__ u32x4 load_at(gbyte_ptr b, uint32_t off)
{
    gchunk_ptr p = (gchunk_ptr)(b + off);
    if constexpr (NT)
        return __builtin_nontemporal_load(p);
    else
        return *p;
}

__device__ __forceinline__ uint32_t wsum4(const u32x4 &d, uint32_t acc)
{
    return wsum(d.w, wsum(d.z, wsum(d.y, wsum(d.x, acc))));
}

// payload_cksum's per-packet terms from the packet's first chunk c (bytes
// 0..15), for the word sum over [8, len): see payload_as_ip (wc_flat.h).
// ok = false for an IPv4 header that is not 20 bytes long.
__device__ __forceinline__ uint32_t lean_extra(const u32x4 &c, bool &ok)
{
    const uint32_t b0 = c.x & 0xFFu;
    const PseudoHdr ph = pseudo_hdr(b0, (c.x >> 16) & 0xFFu, c.x >> 24, (c.y >> 16) & 0xFFu);
    ok = !ph.v4 || ph.hl == 20u;
    return ph.v4 ? ph.special - ((c.z & 0xFFu) + ((c.z >> 16) & 0xFFu) + ((c.z >> 24) << 8))
                 : ph.special + (c.y & 0xFFFFu);
}

// Bytes [lo, hi) of a dword whose first byte is window byte b, as a mask.
__device__ __forceinline__ uint32_t range_mask(int b, int lo, int hi)
{
    const int l = min(max(lo - b, 0), 4), h = min(max(hi - b, 0), 4);
    return (uint32_t)(((1ull << (8 * h)) - 1ull) & ~((1ull << (8 * l)) - 1ull));
}

// PH: the packets share an even start phase p != 0 in their 16-byte chunks
// (stride % 16 == 0, e.g. IP packets at +14 in netmap slots), and / or len is
// not a multiple of 16.  The wave then reads each packet's chunk-aligned
// window [a - p, a - p + 16 nch), and every lane ANDs its chunks with masks
// that are the same for every packet -- computed once per kernel -- before
// the word sums: with an even phase the window's little-endian words are the
// packet's, and a masked odd tail byte is its low byte, as in_cksum.c:107-120
// adds it.  payload_cksum's header words (packet bytes 0..11) come from the
// unmasked window dwords of group lanes 0 and 1, one DPP broadcast each.
template <int G, int CPL, int U, int KIND, bool NT, bool PH>
__global__ void __launch_bounds__(256)
k_cksum_lean(const uint8_t *__restrict__ base, uint64_t stride, uint32_t len, uint64_t n,
             uint16_t *__restrict__ out, unsigned long long *__restrict__ bad, int variant_arg,
             uint32_t phase)
{
    const int variant = tuning_variant(variant_arg); // 0 outside the tuning build
    constexpr int GPW = 64 / G;
    constexpr uint32_t PPW = (uint32_t)GPW * U;
    constexpr uint32_t PASS = (uint32_t)G * CPL;
    constexpr bool PL = KIND == WC_KIND_PAYLOAD;
    static_assert(PPW <= 64, "one result store per wave-iteration");

    const int lane = threadIdx.x & 63;
    const uint32_t gl = (uint32_t)lane & (G - 1u);
    const uint32_t grp = (uint32_t)lane / G;
    // Wave-uniform in SGPRs: the wave index and so the first packet's address.
    const uint32_t wib = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t nwaves = (uint64_t)gridDim.x * 4u;
    const uint32_t ph = PH ? phase : 0u;
    const uint32_t nch = PH ? (ph + len + 15u) >> 4 : len >> 4;
    const bool fills = !PH && nch == PASS; // uniform: every chunk slot holds packet bytes
    const uint32_t lo = grp * (uint32_t)stride + 16u * gl;
    const uint32_t ustep = (uint32_t)GPW * (uint32_t)stride;
    uint32_t nbad = 0;
    // PH: this lane's byte masks for its chunk slots (window bytes
    // [ph + 8, ph + len) for payload_cksum, which sums from byte 8 on).
    uint32_t msk[PH ? CPL : 1][4];
    if constexpr (PH) {
        const int rlo = (int)ph + (PL ? 8 : 0), rhi = (int)(ph + len);
#pragma unroll
        for (int c = 0; c < CPL; ++c)
#pragma unroll
            for (int j = 0; j < 4; ++j)
                msk[c][j] = range_mask(16 * (int)(gl + (uint32_t)c * G) + 4 * j, rlo, rhi);
    }

    for (uint64_t wave = xcd_block(variant) * 4u + wib; wave * PPW < n; wave += nwaves) {
        const uint64_t p0 = wave * PPW;
        const gbyte_ptr gb = (gbyte_ptr)(base - ph + p0 * stride);
        u32x4 d[U][CPL];
        if (fills && p0 + PPW <= n) { // uniform: no masks
#pragma unroll
            for (int u = 0; u < U; ++u)
#pragma unroll
                for (int c = 0; c < CPL; ++c)
                    d[u][c] = load_at<NT>(gb, lo + (uint32_t)u * ustep + 16u * G * c);
        } else {
            // The tail wave, or a pass the packets do not fill: a dead slot
            // re-reads another chunk of its own packet (the wave's first
            // packet past the batch end) and is zeroed -- spread over the
            // packets' lines, not one hot line for every dead lane.
#pragma unroll
            for (int u = 0; u < U; ++u)
#pragma unroll
                for (int c = 0; c < CPL; ++c) {
                    const uint32_t k = gl + (uint32_t)c * G;
                    const bool pv = p0 + (uint64_t)u * GPW + grp < n;
                    const bool live = pv && k < nch;
                    const uint32_t kk = k < nch ? k : (k - nch < nch ? k - nch : 0u);
                    const uint32_t off =
                        pv ? grp * (uint32_t)stride + (uint32_t)u * ustep + 16u * kk : 16u * kk;
                    const u32x4 x = load_at<NT>(gb, off);
                    d[u][c] = live ? x : u32x4{0u, 0u, 0u, 0u};
                }
        }
        if constexpr (CPL * U < 16)
            __builtin_amdgcn_sched_barrier(0); // every load before the first sum

        // Per packet-round u: the group's word sum, handed to lane j = its
        // packet's store lane (packet p0 + j) together with, for
        // payload_cksum, the packet's first 12 bytes from the group leader.
        // The per-packet terms and the fold then run once per wave-iteration
        // for all 64 packets, not once per round (64-B payload_cksum 10.5 ->
        // 10.0-10.1 us, ip_cksum 9.8-10.0 -> 9.7 us in tune.py A/B,
        // profiles/ab_r03_lean_xpose.log).
        uint32_t Vs = 0, hx = 0, hy = 0, hz = 0;
        const int src = (lane % GPW) * G;
#pragma unroll
        for (int u = 0; u < U; ++u) {
            uint32_t V = 0;
            uint32_t h0 = 0, h1 = 0, h2 = 0; // packet bytes 0..11 (payload_cksum)
            if constexpr (PH && PL) {
                // before the masks: window dwords ph / 4 .. ph / 4 + 3 of
                // group lanes 0 / 1, shifted to the packet start
                uint32_t w[4];
                using Seq = std::make_integer_sequence<int, 4>;
                switch (ph >> 2) {
                case 0: hdr_words_uni<G, 0>(d[u][0], w, Seq{}); break;
                case 1: hdr_words_uni<G, 1>(d[u][0], w, Seq{}); break;
                case 2: hdr_words_uni<G, 2>(d[u][0], w, Seq{}); break;
                default: hdr_words_uni<G, 3>(d[u][0], w, Seq{}); break;
                }
                const uint32_t sh = 8u * (ph & 3u);
                h0 = __builtin_amdgcn_alignbit(w[1], w[0], sh);
                h1 = __builtin_amdgcn_alignbit(w[2], w[1], sh);
                h2 = __builtin_amdgcn_alignbit(w[3], w[2], sh);
            } else if constexpr (PL) {
                h0 = d[u][0].x;
                h1 = d[u][0].y;
                h2 = d[u][0].z;
            }
#pragma unroll
            for (int c = 0; c < CPL; ++c) {
                if constexpr (PH)
                    V = wsum4(u32x4{d[u][c].x & msk[c][0], d[u][c].y & msk[c][1],
                                    d[u][c].z & msk[c][2], d[u][c].w & msk[c][3]},
                              V);
                else if (PL && c == 0) // payload_cksum sums from byte 8 on
                    V = gl == 0 ? wsum(d[u][0].w, wsum(d[u][0].z, V)) : wsum4(d[u][0], V);
                else
                    V = wsum4(d[u][c], V);
            }
            V = group_sum<G>(V);
            const bool mine = lane / GPW == u;
            const uint32_t v = __shfl(V, src, 64);
            Vs = mine ? v : Vs;
            if constexpr (PL) {
                const uint32_t x = __shfl(h0, src, 64);
                const uint32_t y = __shfl(h1, src, 64);
                const uint32_t z = __shfl(h2, src, 64);
                hx = mine ? x : hx;
                hy = mine ? y : hy;
                hz = mine ? z : hz;
            }
        }
        uint32_t res;
        if constexpr (PL) {
            bool ok = true;
            Vs += lean_extra(u32x4{hx, hy, hz, 0u}, ok);
            res = (uint32_t)fold_not(Vs) | (ok ? 0u : 0x10000u);
        } else {
            res = fold_not(Vs);
        }
        const uint64_t i = p0 + (uint64_t)lane;
        if (lane < (int)PPW && i < n) {
            uint16_t r = (uint16_t)res;
            if constexpr (PL)
                if (res >> 16) // IPv4 header with options / IHL < 5: exact, by this lane
                    r = lane_payload_exact<NT>((uint64_t)base + i * stride, len);
            if (out)
                out[i] = r;
            nbad += r != 0;
        }
    }
    if (bad) {
        nbad = group_sum<64>(nbad);
        if (lane == 0 && nbad)
            atomicAdd(bad, (unsigned long long)nbad);
    }
}

template <int G, int CPL, int U>
hipError_t launch_lean_shape(const LaunchArgs &a, int grid, hipStream_t st)
{
    // PH: an even start phase, or a length that is not whole chunks
    // (nontemporal loads only, the planner's default).
    const uint32_t phase = (uint32_t)((uintptr_t)a.base & 15u);
    const bool ph = phase != 0 || a.len % 16 != 0;
    if (ph && (phase % 2 != 0 || a.stride % 16 != 0 || !a.nontemporal))
        return hipErrorInvalidValue;
#define WC_LEAN_K(K, N, P)                                                     \
    hipLaunchKernelGGL((k_cksum_lean<G, CPL, U, K, N, P>), dim3(grid), dim3(256), 0, st, \
                       (const uint8_t *)a.base, a.stride, a.len, a.n, a.out,           \
                       (unsigned long long *)a.bad, a.variant, phase)
    if (a.kind == WC_KIND_PAYLOAD) {
        if (ph)
            WC_LEAN_K(WC_KIND_PAYLOAD, true, true);
        else if (a.nontemporal)
            WC_LEAN_K(WC_KIND_PAYLOAD, true, false);
        else
            WC_LEAN_K(WC_KIND_PAYLOAD, false, false);
    } else {
        if (ph)
            WC_LEAN_K(WC_KIND_IP, true, true);
        else if (a.nontemporal)
            WC_LEAN_K(WC_KIND_IP, true, false);
        else
            WC_LEAN_K(WC_KIND_IP, false, false);
    }
#undef WC_LEAN_K
    return hipGetLastError();
}

} // namespace

hipError_t launch_lean(const LaunchArgs &a, const Shape &sh, int grid, hipStream_t st)
{
#define WC_SHAPE(G_, C_, U_)                                                   \
    if (sh.group == G_ && sh.cpl == C_ && sh.unroll == U_)                     \
        return launch_lean_shape<G_, C_, U_>(a, grid, st);
    WC_LEAN_SHAPE_LIST
#undef WC_SHAPE
    return hipErrorInvalidValue;
}

} // namespace wc
