// wc_k_strided.hip -- strided batches on gfx950: the group-per-packet kernel
// k_cksum and its launch table.
#include "wc_device.h"

#include <type_traits>

namespace wc {

// ---------------------------------------------------------------------------
// Strided batches: group-per-packet kernel.
//   G     lanes per packet (power of two, 4..64)
//   CPL   16-byte chunk loads per lane per pass (a pass covers G*CPL chunks)
//   U     packets per group per iteration (more bytes in flight for small
//         packets)
//   KIND  WC_KIND_IP / WC_KIND_PAYLOAD
//   FULL  every packet starts 16-byte aligned and len % 16 == 0 (IP only):
//         no masks, no tables
//   NT    nontemporal loads
//   HDR   (payload only) also store ip_cksum(ip, ip4_hl) of each IPv4 packet
//         into out_hdr (0 for IPv6, which has no header checksum)
//   RAGGED packet i is [base + offs[i], + lens[i]) instead: the small-batch
//         ragged variant (a few packets per wave, so a batch far smaller than
//         the GPU still puts every packet's loads in flight at once)
// Packet i is [base + i*stride, + len).  The grid is one-shot by default
// (each wave does one iteration); a capped grid strides.  waves_per_eu(3)
// caps the kernel at 168 VGPRs: payload (16,6,4) otherwise takes 170, which
// leaves 2 waves per SIMD and cost 10 % of HBM throughput (80 -> 88 % of peak,
// profiles/ab_r01_c2_payload_waves.log).
template <int G, int CPL, int U, int KIND, bool FULL, bool NT, bool HDR, bool RAGGED>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3)))
k_cksum(const uint8_t *__restrict__ base, uint64_t stride, uint32_t len,
        const uint64_t *__restrict__ offs, const uint16_t *__restrict__ lens,
        uint64_t n, uint16_t *__restrict__ out, unsigned long long *__restrict__ bad,
        uint16_t *__restrict__ out_hdr, int variant_arg)
{
    const int variant = tuning_variant(variant_arg); // 0 outside the tuning build
    static_assert(!(RAGGED && (FULL || HDR)), "ragged group variant: masked, no header");
    static_assert(!HDR || KIND == WC_KIND_PAYLOAD, "header checksum rides on payload");
    static_assert(G >= 4 && G <= 64 && (G & (G - 1)) == 0, "group width");
    static_assert(!(FULL && KIND == WC_KIND_PAYLOAD), "payload needs masks");
    constexpr int GPW = 64 / G;
    constexpr uint64_t PPW = (uint64_t)GPW * U;
    constexpr int PASS = G * CPL;
    // payload_cksum as ip_cksum over [8, len) plus per-packet terms from the
    // header (payload_as_ip, wc_flat.h; the lean kernel's scheme): the
    // chunk sums no longer wait for the header hand-off, and their masks are
    // ip_cksum's.  A round with a packet the terms do not cover (IPv4 with
    // options or IHL < 5, a packet shorter than its header) is summed again
    // from the same registers with the header ranges (wave-uniform, rare in
    // real traffic).  The fused header variant keeps the header-range
    // accumulate (it sums [0, hl) too), and so do all shapes but the 96-chunk
    // passes (32 x 3, 16 x 6: MTU packets), where it measured faster -- 1500 B
    // in 2048-B slots at +14 85.9 -> 89.7 %, C2 92.3 -> 92.7 % -- and not
    // slower elsewhere (2048-B slots at +14: 128 B 41.4 -> 37.3 %, 576 B 78 ->
    // 75.6 %, 1024 B on 16 x 5 77.3 -> 69.1 %, 9000 B on 32 x 18 92 -> 26 %:
    // profiles/ab_r03_strided_asip.log).
    // (Tuning build: WC_VARIANT bit 27 turns ASIP on for every shape.)
    constexpr bool ASIP_CT = KIND == WC_KIND_PAYLOAD && !HDR && G * CPL == 96;
#ifdef WC_TUNING
    constexpr bool ASIP_ANY = KIND == WC_KIND_PAYLOAD && !HDR;
#else
    constexpr bool ASIP_ANY = ASIP_CT;
#endif
    const bool ASIP = ASIP_CT || (ASIP_ANY && (variant & (1 << 27)));

    const int lane = threadIdx.x & 63;
    const int gl = lane & (G - 1);
    const int grp = lane / G;
    const int lead = lane & ~(G - 1);
    const uint64_t wave = xcd_block(variant) * (blockDim.x >> 6) + (threadIdx.x >> 6);
    const uint64_t nwaves = (uint64_t)gridDim.x * (blockDim.x >> 6);
    uint32_t nbad = 0;
    const uint64_t zero = (uint64_t)(uintptr_t)&kZeroChunk;
    // A wave-iteration's results are PPW consecutive uint16s: with PPW <= 64
    // one store instruction of lane j = packet p0 + j writes them (one
    // coalesced store instead of U partial ones from the group leaders).  The
    // leaders' scattered 2-byte stores cost C3 64 B 2 of its 11.5 us.
    // WC_VARIANT bit 128 keeps the leader stores (A/B).
    constexpr bool kLaneStore = PPW <= 64;
    const bool lane_store = kLaneStore && !(variant & 128);

    for (uint64_t p0 = wave * PPW; p0 < n; p0 += nwaves * PPW) {
        uint32_t res = 0, res_h = 0;
        uint64_t c0[U];
        uint32_t nch[U], plen[U];
        int s[U];
        bool valid[U];
        u32x4 d[U][CPL];

        // Strided: packet p0 + u GPW + grp sits GPW * stride after the one
        // of u - 1 (one 64-bit multiply per wave, not per packet: the
        // address setup runs before the first load).
        const uint64_t a_first = (uint64_t)base + p0 * stride;
        uint64_t a_u = a_first + (uint64_t)grp * stride;
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t i = p0 + (uint64_t)u * GPW + grp;
            valid[u] = i < n;
            uint64_t a;
            if constexpr (RAGGED) {
                const uint64_t ii = valid[u] ? i : p0;
                a = (uint64_t)base + offs[ii];
                plen[u] = lens[ii];
            } else {
                a = valid[u] ? a_u : a_first;
                a_u += (uint64_t)GPW * stride;
                plen[u] = len;
            }
            // payload_cksum reads the IPv4 header fields up to byte 19 even
            // for a shorter len (in_cksum.c:149-151), so cover them too.
            const uint32_t span = KIND == WC_KIND_PAYLOAD ? max(plen[u], 20u) : plen[u];
            s[u] = (int)(a & 15u);
            c0[u] = a & ~15ull;
            nch[u] = valid[u] ? ((uint32_t)s[u] + span + 15u) >> 4 : 0u;
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int c = 0; c < CPL; ++c) {
                const uint32_t k = (uint32_t)(gl + c * G);
                // Unconditional load (no branch per chunk): dead slots read a
                // zero chunk.
                d[u][c] = load_chunk<NT>(k < nch[u] ? c0[u] + 16ull * k : zero);
            }
        // Every load of the iteration is issued before any sum: without the
        // barrier hipcc hoisted the first packet's dot4s between the loads,
        // with a vmcnt(0) after the first one, so the (4,1,4) and (8,3,2)
        // shapes paid two memory latencies per wave (256 B: 86 -> 89-90 % of
        // HBM peak).  The long shapes keep hipcc's own order, which measured
        // better for C2 (90.8 vs 90.0 %, profiles/ab_r02_sched_barrier.log).
        if constexpr (CPL * U < 16)
            __builtin_amdgcn_sched_barrier(0);

#pragma unroll
        for (int u = 0; u < U; ++u) {
            PseudoHdr ph{0u, 1u, 0u};
            uint32_t extra = 0;
            bool ok = true;
            if constexpr (KIND == WC_KIND_PAYLOAD) {
                // Header bytes 0..11 sit in the group's chunks 0/1, i.e. in
                // d[u][0] of group lanes 0 and 1.
                const int su = s[u];
                uint32_t b0, b2, b3, b6, x1 = 0, x2 = 0;
                auto exchange = [&] { // ds_bpermute from the lane holding each byte
                    b0 = __shfl(pick_byte(d[u][0], su), lead + (su >> 4), 64);
                    b2 = __shfl(pick_byte(d[u][0], (su + 2) & 15), lead + ((su + 2) >> 4), 64);
                    b3 = __shfl(pick_byte(d[u][0], (su + 3) & 15), lead + ((su + 3) >> 4), 64);
                    b6 = __shfl(pick_byte(d[u][0], (su + 6) & 15), lead + ((su + 6) >> 4), 64);
                };
                if (variant & (1 << 29)) { // timing probe (tuning build): no hand-off, wrong results
                    b0 = 0x45u;
                    b2 = 0u;
                    b3 = 64u;
                    b6 = 17u;
                } else if (!RAGGED && (stride & 15u) == 0 && !(variant & (1 << 30))) {
                    // One start phase for the batch: the window dwords and
                    // their lanes are wave-uniform (tuning build: WC_VARIANT
                    // bit 30 takes the per-lane path below instead).
                    constexpr int NW = ASIP_ANY ? 4 : 3;
                    uint32_t w[NW];
                    const int su0 = __builtin_amdgcn_readfirstlane(su);
                    using Seq = std::make_integer_sequence<int, NW>;
                    switch (su0 >> 2) {
                    case 0: hdr_words_uni<G, 0>(d[u][0], w, Seq{}); break;
                    case 1: hdr_words_uni<G, 1>(d[u][0], w, Seq{}); break;
                    case 2: hdr_words_uni<G, 2>(d[u][0], w, Seq{}); break;
                    default: hdr_words_uni<G, 3>(d[u][0], w, Seq{}); break;
                    }
                    const uint32_t sh = 8u * (uint32_t)(su0 & 3);
                    const uint32_t x0 = __builtin_amdgcn_alignbit(w[1], w[0], sh); // 0..3
                    x1 = __builtin_amdgcn_alignbit(w[2], w[1], sh);                // 4..7
                    if constexpr (ASIP_ANY)
                        x2 = __builtin_amdgcn_alignbit(w[3], w[2], sh); // 8..11
                    b0 = x0 & 0xFFu;
                    b2 = (x0 >> 16) & 0xFFu;
                    b3 = x0 >> 24;
                    b6 = (x1 >> 16) & 0xFFu;
                } else if (ASIP_ANY || !(variant & (1 << 19))) {
                    // DPP broadcasts of the window dwords that hold packet
                    // bytes 0..7 (0..11 for ASIP) (window dword k is dword
                    // k & 3 of group lane k >> 2); the ds_bpermute exchange
                    // (WC_VARIANT bit 19) cost 2048-B netmap slots 4 points,
                    // packed 64-192 B 2-5 points (profiles/ab_r02_hdr_dpp.log).
                    constexpr int NW = ASIP_ANY ? 4 : 3;
                    uint32_t w[NW];
#pragma unroll
                    for (int j = 0; j < NW; ++j) {
                        const int k = (su >> 2) + j;
                        const uint32_t mine = pick_dword(d[u][0], k & 3);
                        // both broadcasts run with every lane active
                        const uint32_t f0 = group_bcast<G, 0>(mine);
                        const uint32_t f1 = group_bcast<G, 1>(mine);
                        w[j] = (k >> 2) ? f1 : f0;
                    }
                    const uint32_t sh = 8u * (uint32_t)(su & 3);
                    const uint32_t x0 = __builtin_amdgcn_alignbit(w[1], w[0], sh); // 0..3
                    x1 = __builtin_amdgcn_alignbit(w[2], w[1], sh);                // 4..7
                    if constexpr (ASIP_ANY)
                        x2 = __builtin_amdgcn_alignbit(w[3], w[2], sh); // 8..11
                    b0 = x0 & 0xFFu;
                    b2 = (x0 >> 16) & 0xFFu;
                    b3 = x0 >> 24;
                    b6 = (x1 >> 16) & 0xFFu;
                } else {
                    exchange();
                }
                ph = pseudo_hdr(b0, b2, b3, b6);
                if (ASIP) {
                    ok = ph.v4 ? ph.hl == 20u && plen[u] >= 20u : plen[u] >= 40u;
                    extra = ph.v4 ? ph.special - ((x2 & 0xFFu) + ((x2 >> 16) & 0xFFu) +
                                                  ((x2 >> 24) << 8))
                                  : ph.special + (x1 & 0xFFFFu);
                }
            }
            const int re = (int)plen[u];
            uint32_t E = 0, O = 0, Eh = 0, Oh = 0;
            // The chunk sums of [rs, re) with kind K's weights, extra passes
            // for packets longer than one (e.g. 9000 B jumbo frames) reloaded.
            auto sum_packet = [&](auto kind, int rs) {
                constexpr int K = decltype(kind)::value;
#pragma unroll
                for (int c = 0; c < CPL; ++c)
                    accum_strided<K, FULL, HDR>(d[u][c], 16 * (gl + c * G) - s[u], rs, re,
                                                (uint32_t)(gl + c * G) < nch[u], ph.v4, E, O,
                                                Eh, Oh);
                for (uint32_t kb = PASS; kb < nch[u]; kb += PASS) {
                    u32x4 t[CPL];
#pragma unroll
                    for (int c = 0; c < CPL; ++c) {
                        const uint32_t k = kb + (uint32_t)(gl + c * G);
                        t[c] = load_chunk<NT>(k < nch[u] ? c0[u] + 16ull * k : zero);
                    }
#pragma unroll
                    for (int c = 0; c < CPL; ++c)
                        accum_strided<K, FULL, HDR>(t[c], 16 * (int)(kb + gl + c * G) - s[u],
                                                    rs, re, kb + (uint32_t)(gl + c * G) < nch[u],
                                                    ph.v4, E, O, Eh, Oh);
                }
            };
            uint32_t S;
            if (ASIP) {
                sum_packet(std::integral_constant<int, WC_KIND_IP>{}, 8);
                S = combine(E, O, s[u] & 1) + (gl == 0 ? extra : 0u);
                if (__ballot(valid[u] && !ok)) { // rare: redo the round with header ranges
                    E = O = 0;
                    sum_packet(std::integral_constant<int, WC_KIND_PAYLOAD>{}, (int)ph.hl);
                    S = combine(E, O, s[u] & 1) + (gl == 0 ? ph.special : 0u);
                }
            } else {
                sum_packet(std::integral_constant<int, KIND>{}, KIND == WC_KIND_PAYLOAD ? (int)ph.hl : 0);
                S = combine(E, O, s[u] & 1) + (gl == 0 ? ph.special : 0u);
            }
            S = group_sum<G>(S);
            uint32_t Sh = 0;
            if constexpr (HDR)
                Sh = group_sum<G>(combine(Eh, Oh, s[u] & 1));
            const uint32_t rr = fold_not(S);
            if (lane_store) {
                // Lane j of the wave takes packet p0 + j's result from its
                // group (every lane of a group holds the sum).
                const int src = (lane % GPW) * G;
                const uint32_t r = __shfl(rr, src, 64);
                if (lane / GPW == u)
                    res = r;
                if constexpr (HDR) {
                    const uint32_t rh = __shfl(ph.v4 ? (uint32_t)fold_not(Sh) : 0u, src, 64);
                    if (lane / GPW == u)
                        res_h = rh;
                }
                continue;
            }
            if (gl == 0 && valid[u]) {
                const uint64_t i = p0 + (uint64_t)u * GPW + grp;
                const uint16_t r = (uint16_t)rr;
                if (out && !(variant & 64)) // WC_VARIANT bit 64: no result store (timing only)
                    out[i] = r;
                nbad += r != 0;
                if constexpr (HDR)
                    out_hdr[i] = ph.v4 ? fold_not(Sh) : 0; // ip4.c:110-115
            }
        }
        if (lane_store) {
            const uint64_t i = p0 + (uint64_t)lane;
            if (lane < (int)PPW && i < n) {
                const uint16_t r = (uint16_t)res;
                if (out && !(variant & 64)) // WC_VARIANT bit 64: no result store (timing only)
                    out[i] = r; // (a nontemporal store measured the same)
                nbad += r != 0;
                if constexpr (HDR)
                    out_hdr[i] = (uint16_t)res_h; // ip4.c:110-115
            }
        }
    }

    if (bad) {
        // Wave-level total of the leaders' counts, one atomic per wave.
        nbad = group_sum<64>(nbad);
        if (lane == 0 && nbad)
            atomicAdd(bad, (unsigned long long)nbad);
    }
}

// ---------------------------------------------------------------------------
// Launch table.

template <int G, int CPL, int U, int KIND, bool FULL, bool NT, bool HDR = false,
          bool RAGGED = false>
static hipError_t launch_one(const LaunchArgs &a, int grid, hipStream_t st)
{
    hipLaunchKernelGGL((k_cksum<G, CPL, U, KIND, FULL, NT, HDR, RAGGED>), dim3(grid),
                       dim3(256), 0, st, (const uint8_t *)a.base, a.stride, a.len, a.offs,
                       a.lens, a.n, a.out, (unsigned long long *)a.bad, a.out_hdr, a.variant);
    return hipGetLastError();
}

template <int G, int CPL, int U>
static hipError_t launch_shape(const LaunchArgs &a, int grid, hipStream_t st)
{
    const bool nt = a.nontemporal;
    if (a.kind == WC_KIND_PAYLOAD && a.out_hdr)
        return nt ? launch_one<G, CPL, U, WC_KIND_PAYLOAD, false, true, true>(a, grid, st)
                  : launch_one<G, CPL, U, WC_KIND_PAYLOAD, false, false, true>(a, grid, st);
    if (a.kind == WC_KIND_PAYLOAD)
        return nt ? launch_one<G, CPL, U, WC_KIND_PAYLOAD, false, true>(a, grid, st)
                  : launch_one<G, CPL, U, WC_KIND_PAYLOAD, false, false>(a, grid, st);
    if (a.full)
        return nt ? launch_one<G, CPL, U, WC_KIND_IP, true, true>(a, grid, st)
                  : launch_one<G, CPL, U, WC_KIND_IP, true, false>(a, grid, st);
    return nt ? launch_one<G, CPL, U, WC_KIND_IP, false, true>(a, grid, st)
              : launch_one<G, CPL, U, WC_KIND_IP, false, false>(a, grid, st);
}

template <int G, int CPL, int U>
static hipError_t launch_ragged_shape(const LaunchArgs &a, int grid, hipStream_t st)
{
    if (a.kind == WC_KIND_PAYLOAD)
        return launch_one<G, CPL, U, WC_KIND_PAYLOAD, false, true, false, true>(a, grid, st);
    return launch_one<G, CPL, U, WC_KIND_IP, false, true, false, true>(a, grid, st);
}

hipError_t launch_cksum(const LaunchArgs &a, const Shape &sh, int grid, hipStream_t st)
{
    if (a.ragged) {
        if (a.out_hdr)
            return hipErrorInvalidValue;
#define WC_SHAPE(G_, C_, U_)                                                   \
    if (sh.group == G_ && sh.cpl == C_ && sh.unroll == U_)                     \
        return launch_ragged_shape<G_, C_, U_>(a, grid, st);
        WC_RAGGED_SHAPE_LIST
#undef WC_SHAPE
        return hipErrorInvalidValue;
    }
#define WC_SHAPE(G_, C_, U_)                                                   \
    if (sh.group == G_ && sh.cpl == C_ && sh.unroll == U_)                     \
        return launch_shape<G_, C_, U_>(a, grid, st);
    WC_SHAPE_LIST
#undef WC_SHAPE
    return hipErrorInvalidValue;
}

} // namespace wc
