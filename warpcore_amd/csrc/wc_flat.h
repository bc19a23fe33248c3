// wc_flat.h -- device code of the chunk-balanced "flat" tile path, shared by
// k_cksum_flat (wc_k_flat.hip) and the flat fallback of k_cksum_seg
// (wc_k_seg.hip).
#pragma once

#include "wc_device.h"

namespace wc {
namespace {

// ---------------------------------------------------------------------------
// Ragged batches: chunk-balanced "flat" kernel.
//
// A wave owns a tile of 64 consecutive packets (lane l holds packet l's
// metadata, loaded coalesced).  The tile's 16-byte chunks are numbered
// 0..T-1 in packet order (wave prefix sum of the per-packet chunk counts) and
// dealt to the lanes one 64-chunk ROW at a time, so every lane streams a chunk
// whatever the length mix (Zipf, jumbo frames, empty packets).  Per row:
//   * owner lookup: each packet whose run of chunks starts inside the row
//     marks that slot in LDS (tagged with the row number, so nothing needs
//     clearing); a ballot of the marks gives the run starts, and
//     rank(owner) = rank(first run) + mbcnt(starts at or below the lane);
//   * the owner's descriptor (chunk base, start phase, length, header info)
//     comes from the tile's LDS table, indexed by the rank of the packet
//     among the tile's non-empty packets;
//   * byte weights come from the LDS tables above;
//   * the lanes' exact partial sums go through a DPP inclusive prefix sum and
//     each packet lane adds P[last slot] - P[first slot - 1] of its run to a
//     register accumulator -- no atomics, no same-address LDS traffic.
// Row groups (UN interleaved rows, each load fully coalesced) are
// ping-ponged, and the next tile's metadata (and, for payload_cksum, its
// header bytes) is prefetched while the current tile streams.

struct FlatDesc {          // 16 bytes per non-empty packet of the tile, in LDS
    uint32_t vb_lo, vb_hi; // chunk q of the packet sits at vb + 16 q
    uint32_t rel;          // packet start in the tile's slot-byte space
    uint32_t info;         // len | hl << 16 | v4 << 24
};

template <int UN, int PK = 1>
struct FlatRows {
    u32x4 d[UN][PK];
    uint32_t own[UN];
};

template <int UN>
struct FlatLds {
    FlatDesc desc[64];
    uint32_t mark[UN][64]; // run-start tags, one array per row of a group
    uint32_t pre[64 * UN]; // inclusive prefix sums of the group's chunk sums
    u32x4 pm[17];          // VSUM byte masks: 0xFF in bytes [0, k)
    u32x4 nm[17];          //                  0xFF in bytes [k, 16)
};

// Intra-wave LDS hand-offs need no fence: one wave's LDS instructions execute
// in issue order.  wave_barrier only stops hipcc moving LDS accesses across.
__device__ __forceinline__ void wave_order()
{
    __builtin_amdgcn_wave_barrier();
}

// Owner lookup + loads for the UN rows of a group starting at slot g0.  A
// slot is PK consecutive 16-byte chunks of one packet (PK = 2: every lane
// streams 32 contiguous bytes per row, and the owner lookup, scan and
// hand-offs below are paid once per 2 chunks).
// SKIP: a descriptor whose info has bit 31 set is skipped -- its slots read
// the zero chunk (the RX verdict kernel marks frames its header parse rules
// out after the first row group is in flight).
template <int UN, bool NT, bool NOLOAD = false, int PK = 1, int KIND = WC_KIND_IP,
          bool SKIP = false>
__device__ __forceinline__ void flat_issue(FlatRows<UN, PK> &R, FlatLds<UN> &L,
                                           uint32_t g0, int lane, uint32_t cp,
                                           uint32_t ce, uint32_t rank,
                                           uint32_t last_rank, uint32_t total)
{
    uint32_t first[UN];
#pragma unroll
    for (int u = 0; u < UN; ++u) {
        const uint32_t row0 = g0 + 64u * u;
        // Packet lane: its run inside this row is [lo, hi); a run that starts
        // inside the row (not at its first slot) marks its first slot with
        // the row's tag.
        const uint32_t lo = max(cp, row0), hi = min(ce, row0 + 64u);
        const bool part = lo < hi;
        if (part && lo > row0)
            L.mark[u][lo - row0] = row0 >> 6;
        // Rank of the packet covering the row's first slot; a row past the
        // tile's end has none and takes the last packet (its loads are
        // clamped to the tile's last chunk, which that packet owns).
        const uint64_t firstm = __ballot(part && lo == row0);
        first[u] = firstm ? __builtin_amdgcn_readlane(rank, (int)__builtin_ctzll(firstm))
                          : last_rank;
    }
    wave_order();
#pragma unroll
    for (int u = 0; u < UN; ++u) {
        const uint32_t row0 = g0 + 64u * u;
        const bool st = L.mark[u][lane] == (row0 >> 6);
        const uint32_t own = min(first[u] + mbcnt64(__ballot(st)) + (st ? 1u : 0u), last_rank);
        R.own[u] = own;
        // Unconditional load (slots past the tile's end re-read its last
        // chunk and are zeroed in flat_accum): a straight-line issue stream
        // lets hipcc wait for exactly the older row group.
        const uint32_t q = min(row0 + (uint32_t)lane, total - 1u);
        if constexpr (PK == 1 && SKIP) {
            const FlatDesc g = L.desc[own];
            const uint64_t vb = (uint64_t)g.vb_lo | ((uint64_t)g.vb_hi << 32);
            R.d[u][0] = load_chunk<NT>((g.info >> 31) ? (uint64_t)(uintptr_t)&kZeroChunk
                                                       : vb + 16ull * q);
        } else if constexpr (PK == 1) {
            const uint64_t vb = *reinterpret_cast<const uint64_t *>(&L.desc[own]);
            if constexpr (NOLOAD) // diagnostic build: same stream, no HBM traffic
                R.d[u][0] = u32x4{(uint32_t)vb, q, (uint32_t)(vb >> 32), q ^ 0x5a5a5a5au};
            else
                R.d[u][0] = load_chunk<NT>(vb + 16ull * q);
        } else {
            // The slot's chunks past the packet's last one re-read that
            // chunk (never a page the packet does not touch); their weights
            // are zero in flat_accum.
            const FlatDesc g = L.desc[own];
            const uint64_t vb = (uint64_t)g.vb_lo | ((uint64_t)g.vb_hi << 32);
            const uint32_t len = g.info & 0xFFFFu;
            const uint32_t span = KIND == WC_KIND_PAYLOAD ? max(len, 20u) : len;
            const uint32_t cend = (g.rel >> 4) + (((g.rel & 15u) + span + 15u) >> 4);
#pragma unroll
            for (int j = 0; j < PK; ++j) {
                const uint32_t c = min((uint32_t)PK * q + (uint32_t)j, cend - 1u);
                R.d[u][j] = load_chunk<NT>(vb + 16ull * c);
            }
        }
    }
}

// VSUM (ip_cksum ranges, one chunk per slot): each chunk contributes V =
// the sum of its little-endian words at even addresses (4 v_dot2 of the
// masked dwords; masks from the pm / nm tables, one v_and3 per dword), not
// the exact byte-lane pair (E, O) -- half the VALU per chunk.  For an even
// start V is the reference's accumulator; for an odd one the caller folds
// rotl32(V, 8) instead, bit-exact by the residue argument of the seg path
// (wc_k_seg.hip).
template <int UN, int KIND, bool ARITH = false, int PK = 1, bool VSUM = false>
__device__ __forceinline__ void flat_accum(const FlatRows<UN, PK> &R, FlatLds<UN> &L,
                                           const WeightLut *M, uint32_t g0,
                                           int lane, uint32_t cp, uint32_t ce,
                                           uint32_t total, uint32_t &acc)
{
    static_assert(!VSUM || (PK == 1 && KIND == WC_KIND_IP), "VSUM: ip_cksum, one chunk a slot");
    uint32_t P[UN];
#pragma unroll
    for (int u = 0; u < UN; ++u) {
        const uint32_t q = g0 + 64u * u + (uint32_t)lane;
        const FlatDesc &g = L.desc[R.own[u]];
        const uint32_t rel = g.rel, info = g.info;
        if constexpr (VSUM) {
            const int co = (int)(16u * q - rel);
            const int rs = (int)((info >> 16) & 0xFFu), re = (int)(info & 0xFFFFu);
            const int lo = min(max(rs - co, 0), 16), hi = min(max(re - co, 0), 16);
            const u32x4 x = R.d[u][0] & L.pm[hi] & L.nm[lo];
            const uint32_t V = wsum(x.w, wsum(x.z, wsum(x.y, wsum(x.x, 0u))));
            P[u] = q < total ? V : 0u;
            continue;
        }
        uint32_t E = 0, O = 0;
#pragma unroll
        for (int j = 0; j < PK; ++j) {
            const int co = (int)(16u * ((uint32_t)PK * q + (uint32_t)j) - rel);
            if constexpr (ARITH)
                accum_arith<KIND>(R.d[u][j], co, (int)((info >> 16) & 0xFFu),
                                  (int)(info & 0xFFFFu), (info >> 24) & 1u, E, O);
            else
                accum_masked<KIND>(R.d[u][j], co, (int)((info >> 16) & 0xFFu),
                                   (int)(info & 0xFFFFu), (info >> 24) & 1u, *M, E, O);
        }
        P[u] = q < total ? combine(E, O, rel & 1u) : 0u;
    }
    // Inclusive prefix sums of the UN rows, step-interleaved so each row's DPP
    // step fills the others' hazard slots; then the rows are chained.
#define WC_SCAN_STEP(CTRL, ROWS)                                               \
    _Pragma("unroll") for (int u = 0; u < UN; ++u) P[u] += dpp0<CTRL, ROWS>(P[u]);
    WC_SCAN_STEP(kDppRowShr + 1, 0xF)
    WC_SCAN_STEP(kDppRowShr + 2, 0xF)
    WC_SCAN_STEP(kDppRowShr + 4, 0xF)
    WC_SCAN_STEP(kDppRowShr + 8, 0xF)
    WC_SCAN_STEP(kDppRowBcast15, 0xA)
    WC_SCAN_STEP(kDppRowBcast31, 0xC)
#undef WC_SCAN_STEP
    uint32_t carry = 0;
#pragma unroll
    for (int u = 0; u < UN; ++u) {
        const uint32_t tot = __builtin_amdgcn_readlane(P[u], 63);
        L.pre[64 * u + lane] = P[u] + carry;
        carry += tot;
    }
    wave_order();
    // Packet lane: Σ over its run [rlo, rhi) of the group.
    constexpr uint32_t kGrp = 64u * UN;
    const uint32_t rlo = max(cp, g0), rhi = min(ce, g0 + kGrp);
    const uint32_t e_last = min(rhi - g0 - 1u, kGrp - 1u);
    const uint32_t e_before = rlo > g0 ? min(rlo - g0 - 1u, kGrp - 1u) : 0u;
    const uint32_t pe = L.pre[e_last];
    const uint32_t pb = L.pre[e_before];
    if (rlo < rhi)
        acc += pe - (rlo > g0 ? pb : 0u);
    wave_order(); // pre is rewritten by the next group
}

// payload_cksum's header bytes, prefetched a tile ahead: ONE 16-byte load at
// the 4-byte boundary at or below the packet start (a scattered load moves a
// whole cache line per lane, so one load instead of several byte loads).  It
// covers packet bytes 0..12, inside the header the reference reads anyway
// (in_cksum.c:142-160), so it never touches a page the reference would not.
// The bytes are picked out at their use (hdr_h0 / hdr_h1), not at the load:
// extracting them right away made hipcc wait for the load -- and for every
// stream load issued before it -- at the prefetch.
typedef uint32_t u32x4a4 __attribute__((ext_vector_type(4), aligned(4)));

struct HdrRaw {
    u32x4 d;
};

__device__ __forceinline__ HdrRaw load_hdr(uint64_t a)
{
    return HdrRaw{*(const u32x4a4 __attribute__((address_space(1))) *)(uintptr_t)(a & ~3ull)};
}

// b0 | b2 << 8 | b3 << 16 | b6 << 24 of the packet at a.
__device__ __forceinline__ uint32_t hdr_h0(const HdrRaw &h, uint64_t a)
{
    const uint32_t sh = 8u * (uint32_t)(a & 3u);
    const uint32_t w0 = __builtin_amdgcn_alignbit(h.d.y, h.d.x, sh); // bytes 0..3
    const uint32_t w1 = __builtin_amdgcn_alignbit(h.d.z, h.d.y, sh); // bytes 4..7
    return __builtin_amdgcn_perm(w1, w0, 0x06030200u);
}

// b4 | b5 << 8 | b9 << 16 of the packet at a.
__device__ __forceinline__ uint32_t hdr_h1(const HdrRaw &h, uint64_t a)
{
    const uint32_t sh = 8u * (uint32_t)(a & 3u);
    const uint32_t w1 = __builtin_amdgcn_alignbit(h.d.z, h.d.y, sh); // bytes 4..7
    const uint32_t w2 = __builtin_amdgcn_alignbit(h.d.w, h.d.z, sh); // bytes 8..11
    return __builtin_amdgcn_perm(w2, w1, 0x0C050100u);
}

__device__ __forceinline__ PseudoHdr hdr_pseudo(const HdrRaw &h, uint64_t a)
{
    const uint32_t h0 = hdr_h0(h, a);
    return pseudo_hdr(h0 & 0xFFu, (h0 >> 8) & 0xFFu, (h0 >> 16) & 0xFFu, h0 >> 24);
}

// payload_cksum as an ip_cksum-style sum over [8, len) plus per-packet terms.
// The pseudo-header's src/dst fields end where a standard header ends (IPv4
// @12..19 with IHL 5, IPv6 @8..39, in_cksum.c:150-151, 158-159), so the
// reference's accumulator (in_cksum.c:140-164) is, exactly and mod 2^32:
//   IPv4, hl = 20:  words[8, len) - (b8 + b10 + (b11 << 8)) + special
//                   (words[8, 12) = b8 + (b9 << 8) + b10 + (b11 << 8), and the
//                   reference adds proto = b9 << 8 itself, in_cksum.c:149)
//   IPv6:           words[8, len) + (b4 | b5 << 8) + special   (in_cksum.c:160)
// where words[...] are little-endian 16-bit words counted from the packet
// start (8 is even, so the flat path's exact byte-lane sums E / O combine to
// them) and special is the plen re-swap / next_hdr << 24 term.  Chunks then
// need only the range masks of ip_cksum -- no pseudo-header weight tables --
// which is half the masking work of the generic payload accumulate.  Returns
// false (generic path) for an IPv4 header with options or a malformed IHL,
// and for a packet shorter than its header.
__device__ __forceinline__ bool payload_as_ip(const HdrRaw &h, uint64_t a, uint32_t len,
                                              const PseudoHdr &ph, uint32_t &extra)
{
    const uint32_t sh = 8u * (uint32_t)(a & 3u);
    const uint32_t w1 = __builtin_amdgcn_alignbit(h.d.z, h.d.y, sh); // bytes 4..7
    const uint32_t w2 = __builtin_amdgcn_alignbit(h.d.w, h.d.z, sh); // bytes 8..11
    if (ph.v4)
        extra = ph.special - ((w2 & 0xFFu) + ((w2 >> 16) & 0xFFu) + ((w2 >> 24) << 8));
    else
        extra = ph.special + (w1 & 0xFFFFu);
    return ph.v4 ? (ph.hl == 20u && len >= 20u) : len >= 40u;
}

// Fused IPv4 header checksum for the flat kernel: the packet's own lane sums
// its header [0, hl) (at most 5 chunks) -- ip_cksum(ip, hl), ip4.c:110-115.
template <bool NT>
__device__ __forceinline__ uint16_t lane_hdr_cksum(uint64_t a, uint32_t hl,
                                                   const WeightLut *M)
{
    const uint32_t s = (uint32_t)(a & 15u);
    const uint64_t c0 = a & ~15ull;
    const uint32_t nh = (s + hl + 15u) >> 4;
    uint32_t E = 0, O = 0;
    for (uint32_t k = 0; k < nh; ++k) {
        const u32x4 d = load_chunk<false>(c0 + 16ull * k);
        const int co = (int)(16u * k) - (int)s;
        if (M) // the flat kernel's LDS tables, or arithmetic masks
            accum_masked<WC_KIND_IP>(d, co, 0, (int)hl, 0u, *M, E, O);
        else
            accum_arith<WC_KIND_IP>(d, co, 0, (int)hl, 0u, E, O);
    }
    return fold_not(combine(E, O, s & 1u));
}

// Per-tile layout of the flat path: slot range [cp, ce) of this lane's
// packet within the tile, the tile's slot count, and the packet's rank among
// the tile's non-empty packets.  Slot q's chunk j is the packet's chunk
// PK (q - cp) + j, at vb + 16 (PK q + j).
struct FlatTile {
    uint32_t cp, ce, total, rank, last_rank;
    uint32_t ends; // ce - 1 if another non-empty packet follows this one, else ~0 (GathSrc)
};

template <int UN, int PK, bool VSUM = false>
__device__ __forceinline__ FlatTile flat_tile_setup(FlatLds<UN> &L, int lane, uint64_t a,
                                                    uint32_t len, uint32_t span, bool valid,
                                                    uint32_t info)
{
    if constexpr (VSUM) {
        if (lane < 17) {
            const uint32_t k = (uint32_t)lane;
            L.pm[k] = u32x4{head_mask(k, 0), head_mask(k, 1), head_mask(k, 2), head_mask(k, 3)};
        } else if (lane < 34) {
            const uint32_t k = (uint32_t)lane - 17u;
            L.nm[k] = u32x4{~head_mask(k, 0), ~head_mask(k, 1), ~head_mask(k, 2),
                            ~head_mask(k, 3)};
        }
    }
    const uint32_t s = (uint32_t)(a & 15u);
    const uint32_t nch = valid ? (s + span + 15u) >> 4 : 0u;
    const uint32_t nsl = (nch + PK - 1u) / PK; // slots of PK chunks
    FlatTile t;
    t.ce = wave_incl_sum(nsl);
    t.cp = t.ce - nsl;
    t.total = lane_u32(t.ce, 63);
    const uint64_t nonempty = __ballot(nch != 0);
    t.rank = mbcnt64(nonempty);
    t.last_rank = nonempty ? (uint32_t)__builtin_popcountll(nonempty) - 1u : 0u;
    t.ends = nch != 0 && t.rank < t.last_rank ? t.ce - 1u : 0xFFFFFFFFu;
    const uint64_t vb = (a & ~15ull) - 16ull * PK * t.cp;
    if (nch != 0)
        L.desc[t.rank] = FlatDesc{(uint32_t)vb, (uint32_t)(vb >> 32), s + 16u * PK * t.cp, info};
    // Row marks carry the row's number within the tile; reset them to a
    // tag no row has so the previous tile's marks can't match.
#pragma unroll
    for (int u = 0; u < UN; ++u)
        L.mark[u][lane] = 0xFFFFFFFFu;
    wave_order();
    return t;
}

// The tile's row groups after the first one (A, already issued): ping-pong
// A / B (no register copies), group g+1's loads in flight while group g is
// summed; sched_barrier keeps each issue ahead of the other group's sum.
// While a third group still holds tile slots; then a tail of one or two
// groups.  Every issued group is summed: a load left pending at the loop's
// exit makes hipcc wait vmcnt(0) at the loop head on every iteration
// (measured in the ISA with a mid-loop exit).
template <int UN, int KIND, bool NT, bool NOLOAD, bool ARITH, int PK, bool VSUM = false>
__device__ __forceinline__ void flat_tile_loop(FlatRows<UN, PK> &A, FlatLds<UN> &L,
                                               const WeightLut *lut, int lane,
                                               const FlatTile &t, uint32_t &acc)
{
    constexpr uint32_t kGrp = 64u * UN;
    FlatRows<UN, PK> B;
    uint32_t j = 0;
    for (; j + 2 * kGrp < t.total; j += 2 * kGrp) {
        flat_issue<UN, NT, NOLOAD, PK, KIND>(B, L, j + kGrp, lane, t.cp, t.ce, t.rank,
                                             t.last_rank, t.total);
        __builtin_amdgcn_sched_barrier(0);
        flat_accum<UN, KIND, ARITH, PK, VSUM>(A, L, lut, j, lane, t.cp, t.ce, t.total, acc);
        __builtin_amdgcn_sched_barrier(0);
        flat_issue<UN, NT, NOLOAD, PK, KIND>(A, L, j + 2 * kGrp, lane, t.cp, t.ce, t.rank,
                                             t.last_rank, t.total);
        __builtin_amdgcn_sched_barrier(0);
        flat_accum<UN, KIND, ARITH, PK, VSUM>(B, L, lut, j + kGrp, lane, t.cp, t.ce, t.total, acc);
        __builtin_amdgcn_sched_barrier(0);
    }
    if (j + kGrp < t.total) {
        flat_issue<UN, NT, NOLOAD, PK, KIND>(B, L, j + kGrp, lane, t.cp, t.ce, t.rank,
                                             t.last_rank, t.total);
        __builtin_amdgcn_sched_barrier(0);
        flat_accum<UN, KIND, ARITH, PK, VSUM>(A, L, lut, j, lane, t.cp, t.ce, t.total, acc);
        __builtin_amdgcn_sched_barrier(0);
        flat_accum<UN, KIND, ARITH, PK, VSUM>(B, L, lut, j + kGrp, lane, t.cp, t.ce, t.total, acc);
    } else {
        flat_accum<UN, KIND, ARITH, PK, VSUM>(A, L, lut, j, lane, t.cp, t.ce, t.total, acc);
    }
}

// One 64-packet tile of the flat kernel: returns this lane's packet's exact
// reference accumulator (in_cksum.c:140-167 / 107-120, mod 2^32) -- the
// caller folds it.  `after_first_issue` runs once the tile's first row group
// is in flight (the caller's next-tile prefetch goes there).
template <int UN, int KIND, bool NT, bool NOLOAD, bool ARITH, class F, int PK = 1,
          bool VSUM = false>
__device__ __forceinline__ uint32_t flat_tile_sum(FlatLds<UN> &L, const WeightLut *lut,
                                                  int lane, uint64_t a, uint32_t len,
                                                  bool valid, const PseudoHdr &ph,
                                                  F &&after_first_issue)
{
    static_assert(PK == 1 || !NOLOAD, "diagnostic build: one chunk per slot");
    const uint32_t span = KIND == WC_KIND_PAYLOAD ? max(len, 20u) : len;
    const FlatTile t = flat_tile_setup<UN, PK, VSUM>(L, lane, a, len, span, valid,
                                                     len | (ph.hl << 16) | (ph.v4 << 24));
    uint32_t acc = ph.special;
    FlatRows<UN, PK> A;
    if (t.total != 0)
        flat_issue<UN, NT, NOLOAD, PK, KIND>(A, L, 0, lane, t.cp, t.ce, t.rank, t.last_rank,
                                             t.total);
    after_first_issue();
    if (t.total != 0)
        flat_tile_loop<UN, KIND, NT, NOLOAD, ARITH, PK, VSUM>(A, L, lut, lane, t, acc);
    if constexpr (VSUM) {
        static_assert(KIND == WC_KIND_IP, "VSUM: plain ip_cksum");
        if (a & 1u) // residue of the odd-start accumulator (fold-exact)
            acc = __builtin_amdgcn_alignbit(acc, acc, 24);
    }
    return acc;
}

// flat_tile_sum for payload_cksum batches: a tile whose packets all pass
// payload_as_ip runs as ip_cksum over [8, len) with per-packet terms (the
// range start 8 rides in the descriptor's hl field); any other tile takes
// the generic payload accumulate.  Tile-uniform choice.
template <int UN, bool NT, bool ARITH, class F, int PK = 1>
__device__ __forceinline__ uint32_t flat_tile_sum_payload(FlatLds<UN> &L, const WeightLut *lut,
                                                          int lane, uint64_t a, uint32_t len,
                                                          bool valid, const PseudoHdr &ph,
                                                          const HdrRaw &hdr, F &&after_first_issue)
{
    uint32_t extra = 0;
    const bool fast = !valid || payload_as_ip(hdr, a, len, ph, extra);
    if (!__ballot(!fast))
        return flat_tile_sum<UN, WC_KIND_IP, NT, false, ARITH, F, PK>(
            L, lut, lane, a, len, valid, PseudoHdr{8u, 0u, extra}, (F &&)after_first_issue);
    return flat_tile_sum<UN, WC_KIND_PAYLOAD, NT, false, ARITH, F, PK>(
        L, lut, lane, a, len, valid, ph, (F &&)after_first_issue);
}

} // namespace
} // namespace wc
