// wc_seg.h -- device code of the segmented-prefix tile path (seg_tile with
// its dense and gathered chunk sources), the grouped tile path and the
// per-lane exact payload sum: shared by k_cksum_seg (wc_k_seg.hip) and the
// RX verdict kernel (wc_k_rx.hip).  DESIGN.md section 4.4.
#pragma once

#include "wc_flat.h"

#include <type_traits>

namespace wc {
namespace {

// ---------------------------------------------------------------------------
// Ragged batches, dense tiles: the "segmented prefix" path.
//
// When a tile's 64 packets lie in order inside one dense byte range (starts
// and ends non-decreasing, gaps < 4 KiB, range <= 9/8 of the tile's bytes +
// 2 KiB -- the packed Zipf layout of C4, an RX ring drained into one buffer),
// the wave streams that range itself: row r of the tile is the 64 chunks
// [A0 + 1024 r, + 1024), every load fully coalesced and its address known
// without any per-chunk owner lookup.  Every chunk is summed with constant
// weights, a wave prefix sum gives the running sum at every chunk boundary,
// and each packet lane takes the difference of the running sums at its end
// and its start, adding its partial first / last chunk from its own cached
// re-load.  Bytes outside every packet cancel in the differences.  A gap of
// less than 4 KiB between two packets lies in pages that hold packet bytes,
// so the stream never touches an unmapped page.  Other tiles take the flat
// path above.
//
// Both kinds keep ONE running sum: V = sum of the little-endian words at even
// addresses (v_dot2_u32_u16, 4 per chunk).  For an even-start packet V is the
// reference's accumulator (in_cksum.c:107-120; < 2^31, no wrap).  For an odd
// start the reference's X = O + 256 E satisfies X == 256 V == rotl32(V, 8)
// (mod 0xFFFF, as 2^16 == 2^32 == 1) and X == 0 iff V == 0; the end-around
// fold (in_cksum.c:74-80) maps positive numbers to [1, 0xFFFF] by their
// residue, so fold(rotl32(V, 8)) is bit-exact.
//
// payload_cksum (in_cksum.c:140-167) needs no header pass and no header load
// either.  Its pseudo-header src/dst fields end where a standard header ends
// (IPv4 @12..19 with IHL 5, IPv6 @8..39), so body + src/dst is essentially ONE
// range of the running sum, taken as [a + 8, a + len) for both versions.  The
// header bytes 0..11 come out of the stream itself (the lane picks up its
// packet's first two staged chunks, seg_accum): IPv6 adds its payload length
// word @4, IPv4 takes out bytes 8..11 and adds proto << 8 (@9), and an IPv4
// header with options (or a malformed IHL < 5) corrects the range by the
// bytes between byte 20 and hl, from a few masked loads of those lanes alone.
// Then the non-linear term `special` (IPv4 plen, IPv6 next_hdr << 24) is
// added.  The reference adds it in a uint32 that may wrap (next_hdr << 24,
// in_cksum.c:157).  For an even start V is the exact accumulator, so
// V + special wraps exactly as the reference does.  For an odd start the
// residue is exact as long as the reference's sum does not wrap; a tile
// holding an odd-start packet that could wrap (IPv6, next_hdr >= ~254 at
// 1500 B) is redone on the exact flat path (seg_wrap_risk), as is one holding
// a packet shorter than its header.  A separate scattered header load per
// packet cost 14 % of the C4 time (one more cache line per lane, not latency:
// profiles/ab_r01_c4_payload_hdr.log).

// V of a chunk's first q bytes (q = 16: all of them).
template <bool MASK>
__device__ __forceinline__ uint32_t seg_chunk(const u32x4 &d, uint32_t q)
{
    uint32_t v = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j)
        v = wsum(MASK ? pick_dword(d, j) & head_mask(q, j) : pick_dword(d, j), v);
    return v;
}

// V of the bytes at packet offsets [lo, hi) inside a chunk that starts co
// bytes after the packet start.
__device__ __forceinline__ uint32_t seg_range(const u32x4 &d, int co, int lo, int hi)
{
    const int l = min(max(lo - co, 0), 16);
    const int h = max(min(max(hi - co, 0), 16), l);
    const uint32_t kb = (1u << h) - (1u << l);
    uint32_t v = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j)
        v = wsum(pick_dword(d, j) & (expand_nibble(kb, j) * 0xFFu), v);
    return v;
}

template <int UNS>
struct SegRows {
    u32x4 d[UNS];
};

template <int UNS, bool NT>
__device__ __forceinline__ void seg_issue(SegRows<UNS> &R, uint64_t A0, uint32_t g0, int lane,
                                          uint32_t T, uint64_t zero)
{
#pragma unroll
    for (int u = 0; u < UNS; ++u) {
        const uint32_t q = g0 + 64u * u + (uint32_t)lane;
        R.d[u] = load_chunk<NT>(q < T ? A0 + 16ull * q : zero);
    }
}

// Sum the UNS rows of the group at slot g0: row prefix sums (DPP), chained
// through LDS; packet lanes whose start / end chunk falls in the group pick
// up the running sum before it and the chunk itself.  `carry` is the running
// sum before the group (wave-uniform).  With HC >= 2 (payload_cksum) the lane
// also picks up its packet's first HC chunks c0, c0 + 1 (, c0 + 2) -- its
// header bytes 0..11 (0..19 with the fused header checksum), and the start
// chunk cs, which is c0 or c0 + 1.
template <int UNS, int HC, bool CLAMP>
__device__ __forceinline__ void seg_accum(const SegRows<UNS> &R, uint32_t *pre, u32x4 *stage,
                                          uint32_t g0, int lane, uint32_t T, uint32_t cs,
                                          uint32_t ce, uint32_t c0, uint32_t sa, uint32_t &carry,
                                          uint32_t &Ps, uint32_t &Pe, u32x4 &hs, u32x4 &he,
                                          u32x4 &h1, u32x4 &h2)
{
    constexpr uint32_t kGrp = 64u * UNS;
    uint32_t P[UNS];
#pragma unroll
    for (int u = 0; u < UNS; ++u) {
        P[u] = seg_chunk<false>(R.d[u], 16u);
        if constexpr (CLAMP) // a gathered stream's slots past T re-read its last chunk
            P[u] = g0 + 64u * u + (uint32_t)lane < T ? P[u] : 0u;
    }
#define WC_SEG_STEP(CTRL, ROWS)                                                \
    _Pragma("unroll") for (int u = 0; u < UNS; ++u) P[u] += dpp0<CTRL, ROWS>(P[u]);
    WC_SEG_STEP(kDppRowShr + 1, 0xF)
    WC_SEG_STEP(kDppRowShr + 2, 0xF)
    WC_SEG_STEP(kDppRowShr + 4, 0xF)
    WC_SEG_STEP(kDppRowShr + 8, 0xF)
    WC_SEG_STEP(kDppRowBcast15, 0xA)
    WC_SEG_STEP(kDppRowBcast31, 0xC)
#undef WC_SEG_STEP
    uint32_t c = carry;
#pragma unroll
    for (int u = 0; u < UNS; ++u) {
        stage[64u * u + lane] = R.d[u];
        const uint32_t tot = __builtin_amdgcn_readlane(P[u], 63);
        pre[64u * u + lane] = P[u] + c;
        c += tot;
    }
    wave_order();
    const uint32_t ds = cs - g0, de = ce - g0;
    // The packet's first / last chunk, for its partial sums (exec-masked
    // LDS reads: no scattered global re-loads).
    if constexpr (HC >= 2) {
        // Header chunks c0 .. c0 + 2: bytes 0..11 (0..19 with the header
        // checksum) from the packet's start phase sa on -- the second chunk
        // only if sa > 4 (with the checksum: always), the third only if
        // sa > 12 (fewer LDS reads and bank conflicts than every lane
        // reading all three).
        const uint32_t d0 = c0 - g0; // (unsigned: c0 + 1 == g0 gives d0 + 1 == 0)
        if (d0 < kGrp)
            hs = stage[d0];
        if ((HC >= 3 || sa > 4u) && d0 + 1u < kGrp)
            h1 = stage[d0 + 1u];
        if constexpr (HC >= 3)
            if (sa > 12u && d0 + 2u < kGrp)
                h2 = stage[d0 + 2u];
    } else {
        if (ds < kGrp)
            hs = stage[ds];
    }
    if (de < kGrp)
        he = stage[de];
    const uint32_t vs = pre[min(ds - 1u, kGrp - 1u)];
    const uint32_t ve = pre[min(de - 1u, kGrp - 1u)];
    if (ds < kGrp)
        Ps = ds ? vs : carry;
    if (de < kGrp)
        Pe = de ? ve : carry;
    carry = c;
    wave_order(); // pre is rewritten by the next group
}

// Dword k (0..11) of the 48-byte window x:y:z.
__device__ __forceinline__ uint32_t win_dword(const u32x4 &x, const u32x4 &y, const u32x4 &z,
                                              uint32_t k)
{
    const u32x4 &h = k >= 8u ? z : (k & 4u ? y : x);
    return pick_dword(h, (int)(k & 3u));
}

// Packet bytes 4 m .. 4 m + 3 from the window x:y:z that holds the packet's
// first bytes from offset s on.
__device__ __forceinline__ uint32_t win_bytes(const u32x4 &x, const u32x4 &y, const u32x4 &z,
                                              uint32_t s, uint32_t m)
{
    const uint32_t k = (s >> 2) + m;
    return __builtin_amdgcn_alignbit(win_dword(x, y, z, k + 1u), win_dword(x, y, z, k),
                                     8u * (s & 3u));
}

// Packet bytes 4 m .. 4 m + 3 for m = 0 .. W - 1 from the window x:y:z that
// holds the packet's first bytes from offset s (< 16) on: the window is
// rotated by s >> 2 dwords in two select levels, then each output dword is
// one alignbit -- about 3 W + 4 VALU for all W, where W separate win_bytes
// calls select each dword out of 12 (about 14 VALU apiece).
template <int W>
__device__ __forceinline__ void win_rot(const u32x4 &x, const u32x4 &y, const u32x4 &z,
                                        uint32_t s, uint32_t (&w)[W])
{
    static_assert(W >= 1 && W <= 5, "window of 48 bytes from offset < 16");
    // Named scalars, not an array: a select between two array elements is
    // turned into a dynamic index, which puts the array in scratch.
    const bool q1 = s & 4u, q2 = s & 8u;
    const uint32_t e0 = q1 ? x.y : x.x, e1 = q1 ? x.z : x.y, e2 = q1 ? x.w : x.z,
                   e3 = q1 ? y.x : x.w, e4 = q1 ? y.y : y.x, e5 = q1 ? y.z : y.y,
                   e6 = q1 ? y.w : y.z, e7 = q1 ? z.x : y.w, e8 = q1 ? z.y : z.x;
    const uint32_t d0 = q2 ? e2 : e0, d1 = q2 ? e3 : e1, d2 = q2 ? e4 : e2, d3 = q2 ? e5 : e3,
                   d4 = q2 ? e6 : e4, d5 = q2 ? e7 : e5;
    (void)e8;
    const uint32_t sh = 8u * (s & 3u);
    w[0] = __builtin_amdgcn_alignbit(d1, d0, sh);
    if constexpr (W > 1)
        w[1] = __builtin_amdgcn_alignbit(d2, d1, sh);
    if constexpr (W > 2)
        w[2] = __builtin_amdgcn_alignbit(d3, d2, sh);
    if constexpr (W > 3)
        w[3] = __builtin_amdgcn_alignbit(d4, d3, sh);
    if constexpr (W > 4)
        w[4] = __builtin_amdgcn_alignbit(d5, d4, sh);
}

// V of a chunk's first q bytes (q <= 16) with the head masks from LDS: one
// 16-byte LDS read and 4 v_and, where head_mask computes each dword's mask
// in ~5 VALU.  pm[k] = 0xFF in bytes [0, k) (seg_init_masks).
__device__ __forceinline__ uint32_t seg_head(const u32x4 &d, uint32_t q, const u32x4 *pm)
{
    const u32x4 m = pm[q];
    return wsum(d.w & m.w, wsum(d.z & m.z, wsum(d.y & m.y, wsum(d.x & m.x, 0u))));
}

// Fill the 17 head masks (lanes 0..16 of the calling wave).
__device__ __forceinline__ void seg_init_masks(u32x4 *pm, int lane)
{
    if (lane < 17) {
        const uint32_t k = (uint32_t)lane;
        pm[k] = u32x4{head_mask(k, 0), head_mask(k, 1), head_mask(k, 2), head_mask(k, 3)};
    }
}

// Could the reference's uint32 sum for this odd-start payload packet wrap
// when `special` is added?  Before it, the sum holds at most (len + 1) / 2 + 1
// words of <= 0xFFFF (body, src/dst and proto or payload length; len >= hl),
// so only IPv6 next_hdr >= ~254 at 1500 B (never at <= 500 B) can.
__device__ __forceinline__ bool seg_wrap_risk(uint64_t a, uint32_t len, const PseudoHdr &ph)
{
    return (a & 1u) &&
           (uint64_t)ph.special + 65535ull * ((len + 1u) / 2u + 1u) >= (1ull << 32);
}

// Can the seg path sum this payload packet?  It needs the whole header inside
// the packet (len >= hl; the reference reads ~4 GiB otherwise) and, for IPv4,
// the src/dst fields too.
__device__ __forceinline__ bool seg_payload_ok(uint64_t a, uint32_t len, const PseudoHdr &ph)
{
    return len >= max(ph.hl, 20u) && !seg_wrap_risk(a, len, ph);
}

// Chunk sources of seg_tile: slot q of the tile's stream is
//   * DenseSrc: the byte range itself, chunk A0 + 16 q (zero past T);
//   * GathSrc: the tile's packets' own chunks in packet order (the flat
//     path's slot numbering, its owner lookup for the address; slots past T
//     re-read the last chunk and are zeroed in seg_accum).
template <int UNS, bool NT>
struct DenseSrc {
    static constexpr bool kClamp = false;
    uint64_t A0;
    uint32_t T;
    uint64_t zero;
    __device__ __forceinline__ void issue(SegRows<UNS> &R, uint32_t g0, int lane) const
    {
        seg_issue<UNS, NT>(R, A0, g0, lane, T, zero);
    }
};

//
// GathSrc's owner lookup ("end bits"): slot s belongs to the packet of rank
// = the number of packets whose last slot lies before s (counting only
// packets followed by another non-empty one, FlatTile::ends, so the count
// stops at the last rank for slots past the tile's end).  Per row group,
// each such packet whose last slot falls in the group sets that slot's bit
// in a 64-bit word per row (one LDS OR per packet lane); per row, the count
// is a ballot of the packets that ended before the row plus an mbcnt of the
// row's word below the lane.  Against the per-row run-start marks of
// flat_issue (a row-tagged store, two ballots, a readlane and an mbcnt per
// row), the RX kernel's inner loop went from 345 to 239 VALU and from 165
// to 91 SALU per 8 rows.
template <int UNS, bool NT, bool SKIP = false>
struct GathSrc {
    static constexpr bool kClamp = true;
    FlatLds<UNS> *L;
    FlatTile t;
    __device__ __forceinline__ void issue(SegRows<UNS> &R, uint32_t g0, int lane) const
    {
        constexpr uint32_t kGrp = 64u * UNS;
        uint64_t *M = reinterpret_cast<uint64_t *>(&L->mark[0][0]); // one word per row
        wave_order(); // (after the previous group's reads)
        if (lane < UNS) {
            uint32_t z0, z1; // materialised here, not hoisted into registers held across the tile
            asm volatile("v_mov_b32 %0, 0\n\tv_mov_b32 %1, 0" : "=v"(z0), "=v"(z1));
            M[lane] = (uint64_t)z0 | ((uint64_t)z1 << 32);
        }
        wave_order();
        const uint32_t d = t.ends - g0; // (~0 - g0: never below kGrp)
        if (d < kGrp)
            __hip_atomic_fetch_or(&M[d >> 6], 1ull << (d & 63u), __ATOMIC_RELAXED,
                                  __HIP_MEMORY_SCOPE_WORKGROUP);
        wave_order();
#pragma unroll
        for (int u = 0; u < UNS; ++u) {
            const uint64_t m = M[u]; // the same address in every lane: a broadcast read
            const uint32_t row0 = g0 + 64u * u;
            const uint32_t before = (uint32_t)__builtin_popcountll(__ballot(t.ends < row0));
            const uint32_t own = __builtin_amdgcn_mbcnt_hi(
                (uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, before));
            // Slots past the tile's end re-read its last chunk (zeroed in
            // seg_accum): a straight-line issue stream.
            const uint32_t q = min(row0 + (uint32_t)lane, t.total - 1u);
            if constexpr (SKIP) {
                const FlatDesc g = L->desc[own];
                const uint64_t vb = (uint64_t)g.vb_lo | ((uint64_t)g.vb_hi << 32);
                R.d[u] = load_chunk<NT>((g.info >> 31) ? (uint64_t)(uintptr_t)&kZeroChunk
                                                       : vb + 16ull * q);
            } else {
                const uint64_t vb = *reinterpret_cast<const uint64_t *>(&L->desc[own]);
                R.d[u] = load_chunk<NT>(vb + 16ull * q);
            }
        }
    }
};

// One tile as a stream of T chunk slots.  [a, a + len) is this lane's packet,
// starting ra bytes into the stream (dense: a - A0; gathered: 16 cp + (a &
// 15), so a packet's bytes keep their address parity and position within a
// chunk); ip_cksum sums all of it, payload_cksum the range [a + 8, a + len)
// corrected as below.  Returns the checksum, or done = false when a
// payload_cksum lane can't be summed here (header longer than the packet,
// possible uint32 wrap): the caller then takes the exact flat path for the
// tile.  On a gathered stream a packet's first and last chunks hold other
// bytes of the same cache lines; they cancel like the gaps of a dense range.
//
// LANEFIX (payload_cksum on the seg-only packed strided kernel): a lane the
// seg arithmetic can't take gets done = false on its own, the others keep
// their result, and the caller recomputes that lane's packet exactly
// (lane_payload_exact) -- no flat path in that kernel.
struct NoLate {
    __device__ __forceinline__ void operator()(uint32_t &, bool &) const {}
};

template <int UNS, int KIND, bool NT, bool HDR, class Src, bool LANEFIX = false,
          class Late = NoLate>
__device__ __forceinline__ uint16_t seg_tile(uint32_t *pre, u32x4 *stage, const u32x4 *pm,
                                             int lane, uint64_t a, uint64_t ra, uint32_t len,
                                             bool valid, uint32_t T, const Src &src,
                                             uint64_t zero, bool &done, uint16_t &rh,
                                             const Late &late = Late{})
{
    constexpr uint32_t kGrp = 64u * UNS;
    constexpr bool PL = KIND == WC_KIND_PAYLOAD;
    constexpr int HC = PL ? (HDR ? 3 : 2) : 0;
    constexpr bool CL = Src::kClamp;
    const uint32_t c0 = (uint32_t)(ra >> 4);
    const uint32_t sa = (uint32_t)(ra & 15u); // == a & 15 (dense and gathered streams)

    SegRows<UNS> A, B;
    src.issue(A, 0, lane);
    // Late: the lane's packet length (and whether it is summed at all) may be
    // decided only now, with the first row group in flight -- the stream
    // already holds the longest range the packet can have (the RX verdict
    // kernel streams each frame while its headers are still being parsed).
    late(len, valid);
    const uint64_t rs = ra + (PL ? 8u : 0u), re = ra + len;
    const uint32_t cs = (uint32_t)(rs >> 4), qs = (uint32_t)(rs & 15u);
    const uint32_t ce = (uint32_t)(re >> 4), qe = (uint32_t)(re & 15u);

    uint32_t carry = 0, Ps = 0, Pe = 0;
    u32x4 hs = {0u, 0u, 0u, 0u}, he = {0u, 0u, 0u, 0u}, h1 = {0u, 0u, 0u, 0u},
          h2 = {0u, 0u, 0u, 0u};
    // Ping-pong row groups A / B while a third group still holds tile
    // chunks; then a tail of one or two groups.  Every issued group is
    // summed (no load is left pending, so hipcc's waits stay precise) and
    // the rows summed round up to one group, not two (a 17-row tile sums
    // 20 rows instead of 24).
    uint32_t j = 0;
#define WC_SEG_ACC(R, G)                                                       \
    seg_accum<UNS, HC, CL>(R, pre, stage, G, lane, T, cs, ce, c0, sa, carry, Ps, Pe, hs, he, h1, h2)
    for (; j + 2 * kGrp < T; j += 2 * kGrp) {
        src.issue(B, j + kGrp, lane);
        __builtin_amdgcn_sched_barrier(0);
        WC_SEG_ACC(A, j);
        __builtin_amdgcn_sched_barrier(0);
        src.issue(A, j + 2 * kGrp, lane);
        __builtin_amdgcn_sched_barrier(0);
        WC_SEG_ACC(B, j + kGrp);
        __builtin_amdgcn_sched_barrier(0);
    }
    if (j + kGrp < T) {
        src.issue(B, j + kGrp, lane);
        __builtin_amdgcn_sched_barrier(0);
        WC_SEG_ACC(A, j);
        __builtin_amdgcn_sched_barrier(0);
        WC_SEG_ACC(B, j + kGrp);
        j += 2 * kGrp;
    } else {
        WC_SEG_ACC(A, j);
        j += kGrp;
    }
#undef WC_SEG_ACC
    if (cs >= j) // an empty packet at the stream's end (gathered streams)
        Ps = carry;
    if (ce >= j) // the packet ends exactly at the last row group's end
        Pe = carry;
    done = true;
    if constexpr (!PL) {
        const uint32_t v = (Pe + seg_head(he, qe, pm)) - (Ps + seg_head(hs, qs, pm));
        if (!(a & 1u))
            return fold_not(v);
        return fold_not(__builtin_amdgcn_alignbit(v, v, 24)); // rotl32(v, 8)
    } else {
        // Header bytes 0..11 from the packet's first two chunks (hs = c0, h1 =
        // c0 + 1); the start chunk cs is one of them.
        const uint32_t s = (uint32_t)(a & 15u);
        uint32_t wv[HDR ? 5 : 3]; // packet bytes 0..11 (0..19 with the header checksum)
        win_rot(hs, h1, h2, s, wv);
        const uint32_t w0 = wv[0], w1 = wv[1], w2 = wv[2];
        const PseudoHdr ph = pseudo_hdr(w0 & 0xFFu, (w0 >> 16) & 0xFFu, w0 >> 24,
                                        (w1 >> 16) & 0xFFu);
        const bool lane_bad = valid && !seg_payload_ok(a, len, ph);
        if constexpr (LANEFIX) {
            done = !lane_bad;
        } else if (__ballot(lane_bad)) {
            done = false;
            return 0;
        }
        const u32x4 hq = cs == c0 ? hs : h1;
        // V of [a + 8, a + len): IPv6 src/dst + body (hl = 40); IPv4 bytes
        // 8..11, src/dst, options, body.
        uint32_t v = (Pe + seg_head(he, qe, pm)) - (Ps + seg_head(hq, qs, pm));
        const uint32_t odd = (uint32_t)(a & 1u);
        if (ph.v4) {
            // Minus bytes 8..11 (ttl, proto, header checksum), plus proto << 8
            // (in_cksum.c:149) -- both at their address weight.
            const uint32_t b9 = (w2 >> 8) & 0xFFu;
            v -= wsum(odd ? __builtin_amdgcn_perm(w2, w2, 0x02030001u) : w2, 0u);
            v += odd ? b9 : b9 << 8;
        } else {
            // plus the payload length word @4 (in_cksum.c:160)
            const uint32_t b4 = w1 & 0xFFu, b5 = (w1 >> 8) & 0xFFu;
            v += odd ? (b4 << 8) | b5 : b4 | (b5 << 8);
        }
        // IPv4 with hl != 20: the body starts at hl, not 20 -- minus the
        // options [20, hl), or plus [hl, 20) (src/dst then count twice, as in
        // the reference).  <= 40 bytes, <= 4 chunks, loaded by those lanes.
        const bool corr = ph.v4 && ph.hl != 20u && !lane_bad; // (a bad lane's hl may pass len)
        uint32_t cv = 0;
        if (__ballot(valid && corr)) {
            const int clo = (int)min(ph.hl, 20u), chi = (int)max(ph.hl, 20u);
            const uint64_t ca = (a + (uint32_t)clo) & ~15ull;
            u32x4 xc[4];
#pragma unroll
            for (int k = 0; k < 4; ++k)
                xc[k] = load_chunk<false>(valid && corr && ca + 16ull * k < a + (uint32_t)chi
                                              ? ca + 16ull * k : zero);
#pragma unroll
            for (int k = 0; k < 4; ++k)
                cv += seg_range(xc[k], (int)(ca - a) + 16 * k, clo, chi);
            if (corr)
                v = ph.hl < 20u ? v + cv : v - cv;
        }
        if constexpr (HDR) {
            // Fused IPv4 header checksum ip_cksum(ip, hl) (ip4.c:110-115),
            // 0 for IPv6: V of bytes 0..19 from the staged chunks (each
            // dword's bytes at their address weight, as wsum of the dword,
            // byte-swapped per word for an odd start), then minus the bytes
            // [hl, 20) or plus [20, hl) summed above.  Folded like ip_cksum.
            const uint32_t w3 = wv[HDR ? 3 : 0], w4 = wv[HDR ? 4 : 0];
            const uint32_t sw = odd ? 0x02030001u : 0x03020100u;
            uint32_t vh = wsum(__builtin_amdgcn_perm(w0, w0, sw), 0u);
            vh = wsum(__builtin_amdgcn_perm(w1, w1, sw), vh);
            vh = wsum(__builtin_amdgcn_perm(w2, w2, sw), vh);
            vh = wsum(__builtin_amdgcn_perm(w3, w3, sw), vh);
            vh = wsum(__builtin_amdgcn_perm(w4, w4, sw), vh);
            if (corr)
                vh = ph.hl < 20u ? vh - cv : vh + cv;
            rh = !ph.v4 ? (uint16_t)0
                        : fold_not(odd ? __builtin_amdgcn_alignbit(vh, vh, 24) : vh);
        }
        if (!odd)
            return fold_not(v + ph.special); // exact, wrap included
        // residue of rotl32(v, 8) + special (no wrap: seg_wrap_risk), zero
        // iff both are
        const uint64_t t = (uint64_t)__builtin_amdgcn_alignbit(v, v, 24) + ph.special;
        return fold_not((uint32_t)(t & 0xFFFFu) + (uint32_t)(t >> 16));
    }
}

// ---------------------------------------------------------------------------
// Ragged batches, uniform tiles: the "grouped" path.
//
// When a tile's packets have similar chunk counts (a netmap RX ring: fixed
// 2048-B slots holding ~MTU packets at +14, backend_netmap.c:379-391), the
// wave sums it the way the strided kernel sums a batch: 16 lanes per packet,
// four packets per 64-chunk row, R = ceil(max chunks / 16) rows per quad of
// packets, 16 quads per tile.  A chunk's address is its packet's base + 16 c
// -- no owner lookup, no scan, no LDS per row -- and the lanes keep exact
// byte-lane sums (E, O), so payload_cksum needs no wrap guard.  Slots past a
// packet's end read the zero chunk.  A quad's 16 lane sums are reduced with
// a DPP row scan and its four results parked in LDS until the tile's packet
// lanes store them.  Used when the tile's chunks fill at least thr / 64 of
// its 1024 R slots (LaunchArgs::grp_thr): sparse tiles from 40/64 on (netmap
// slots: 71 -> 78 % of HBM peak); dense tiles stay on the seg path, which
// measured faster on them (rc2: 84.7 vs 82.2 %).

struct GrpDesc { // one per packet of the tile, in LDS
    uint32_t a_lo, a_hi;
    uint32_t info; // len | hl << 16 | v4 << 24
    uint32_t special;
};

struct GrpLds {
    GrpDesc gd[64];
    uint32_t res[64];
    uint32_t res_h[64]; // fused IPv4 header checksums (HDR)
};

// Issue-side walk state: quad q, row k within it, and the quad's descriptor
// as this lane sees it (its packet = 4 q + lane / 16).
struct GrpIssue {
    uint32_t q, k;
    uint64_t cb;  // packet's first aligned chunk
    uint32_t nch; // its chunk count
};

template <int UNG>
struct GrpRows {
    u32x4 d[UNG];
};

// Bytes a packet's chunks cover: payload_cksum reads the IPv4 header fields
// up to byte 19 whatever len is (in_cksum.c:149-151).
template <int KIND>
__device__ __forceinline__ uint32_t grp_span(uint32_t len)
{
    return KIND == WC_KIND_PAYLOAD && len ? max(len, 20u) : len;
}

template <int KIND>
__device__ __forceinline__ void grp_load_quad(GrpIssue &I, const GrpLds &L, int lane)
{
    const GrpDesc g = L.gd[min(4u * I.q + ((uint32_t)lane >> 4), 63u)];
    const uint64_t a = (uint64_t)g.a_lo | ((uint64_t)g.a_hi << 32);
    const uint32_t span = grp_span<KIND>(g.info & 0xFFFFu);
    I.cb = a & ~15ull;
    I.nch = I.q < 16u && span ? (uint32_t)((a & 15u) + span + 15u) >> 4 : 0u;
}

template <int UNG, int KIND, bool NT>
__device__ __forceinline__ void grp_issue(GrpRows<UNG> &R, GrpIssue &I, const GrpLds &L,
                                          int lane, uint32_t Rq, uint64_t zero)
{
#pragma unroll
    for (int u = 0; u < UNG; ++u) {
        const uint32_t c = 16u * I.k + ((uint32_t)lane & 15u);
        R.d[u] = load_chunk<NT>(c < I.nch ? I.cb + 16ull * c : zero);
        if (++I.k == Rq) { // wave-uniform
            I.k = 0;
            ++I.q;
            grp_load_quad<KIND>(I, L, lane);
        }
    }
}

// Accumulate-side walk state.
struct GrpAcc {
    uint32_t q, k;
    uint32_t s, len, hl, v4, special;
    uint32_t E, O;
    uint32_t Eh, Oh; // IP header bytes [0, hl) (HDR)
};

__device__ __forceinline__ void grp_acc_quad(GrpAcc &S, const GrpLds &L, int lane)
{
    const GrpDesc g = L.gd[min(4u * S.q + ((uint32_t)lane >> 4), 63u)];
    S.s = g.a_lo & 15u;
    S.len = S.q < 16u ? g.info & 0xFFFFu : 0u;
    S.hl = (g.info >> 16) & 0xFFu;
    S.v4 = (g.info >> 24) & 1u;
    S.special = g.special;
}

template <int UNG, int KIND, bool HDR>
__device__ __forceinline__ void grp_accum(const GrpRows<UNG> &R, GrpAcc &S, GrpLds &L, int lane,
                                          uint32_t Rq)
{
    const uint32_t gl = (uint32_t)lane & 15u;
#pragma unroll
    for (int u = 0; u < UNG; ++u) {
        if (S.q < 16u) { // wave-uniform: rows past the tile's last quad are idle
            const uint32_t c = 16u * S.k + gl;
            const uint32_t span = grp_span<KIND>(S.len);
            const uint32_t nch = span ? (S.s + span + 15u) >> 4 : 0u;
            accum_strided<KIND, false, HDR>(R.d[u], 16 * (int)c - (int)S.s,
                                            KIND == WC_KIND_PAYLOAD ? (int)S.hl : 0,
                                            (int)S.len, c < nch, S.v4, S.E, S.O, S.Eh, S.Oh);
            if (++S.k == Rq) {
                // Quad done: exact reference accumulator of each packet
                // (in_cksum.c:140-167 / 107-120, mod 2^32), row scan to lane 15.
                uint32_t x = combine(S.E, S.O, S.s & 1u) + (gl == 0 ? S.special : 0u);
                x += dpp0<kDppRowShr + 1, 0xF>(x);
                x += dpp0<kDppRowShr + 2, 0xF>(x);
                x += dpp0<kDppRowShr + 4, 0xF>(x);
                x += dpp0<kDppRowShr + 8, 0xF>(x);
                if (gl == 15u)
                    L.res[4u * S.q + ((uint32_t)lane >> 4)] = fold_not(x);
                if constexpr (HDR) {
                    // ip_cksum(ip, hl) of IPv4 packets (ip4.c:110-115)
                    uint32_t h = combine(S.Eh, S.Oh, S.s & 1u);
                    h += dpp0<kDppRowShr + 1, 0xF>(h);
                    h += dpp0<kDppRowShr + 2, 0xF>(h);
                    h += dpp0<kDppRowShr + 4, 0xF>(h);
                    h += dpp0<kDppRowShr + 8, 0xF>(h);
                    if (gl == 15u)
                        L.res_h[4u * S.q + ((uint32_t)lane >> 4)] = S.v4 ? fold_not(h) : 0u;
                    S.Eh = S.Oh = 0u;
                }
                S.E = S.O = 0u;
                S.k = 0;
                ++S.q;
                grp_acc_quad(S, L, lane);
            }
        }
    }
}

// One uniform tile.  Returns this lane's packet's checksum, or done = false
// (payload_cksum with a header longer than its packet: the caller takes the
// flat path).
template <int UNG, int KIND, bool NT, bool HDR>
__device__ __forceinline__ uint16_t grp_tile(GrpLds &L, int lane, uint64_t a, uint32_t len,
                                             bool valid, uint32_t Rq, uint64_t zero, bool &done,
                                             uint16_t &rh)
{
    // payload_cksum's header bytes: loaded first, waited for only after the
    // first row group is issued (the addresses need no header).
    HdrRaw hdr{};
    if constexpr (KIND == WC_KIND_PAYLOAD)
        hdr = load_hdr(a);
    L.gd[lane] = GrpDesc{(uint32_t)a, (uint32_t)(a >> 32), valid ? len : 0u, 0u};
    wave_order();
    GrpIssue I{0u, 0u, 0ull, 0u};
    grp_load_quad<KIND>(I, L, lane);
    GrpRows<UNG> A, B;
    grp_issue<UNG, KIND, NT>(A, I, L, lane, Rq, zero);
    __builtin_amdgcn_sched_barrier(0); // keep the header wait behind the issue
    if constexpr (KIND == WC_KIND_PAYLOAD) {
        PseudoHdr ph{0u, 1u, 0u};
        if (valid)
            ph = hdr_pseudo(hdr, a);
        if (__ballot(valid && len < max(ph.hl, 20u))) {
            done = false;
            return 0;
        }
        L.gd[lane].info |= (ph.hl << 16) | (ph.v4 << 24);
        L.gd[lane].special = ph.special;
        wave_order();
    }
    done = true;
    GrpAcc S{};
    grp_acc_quad(S, L, lane);
    const uint32_t rows = 16u * Rq;
    for (uint32_t j = 0; j < rows; j += 2u * UNG) {
        grp_issue<UNG, KIND, NT>(B, I, L, lane, Rq, zero);
        __builtin_amdgcn_sched_barrier(0);
        grp_accum<UNG, KIND, HDR>(A, S, L, lane, Rq);
        __builtin_amdgcn_sched_barrier(0);
        grp_issue<UNG, KIND, NT>(A, I, L, lane, Rq, zero);
        __builtin_amdgcn_sched_barrier(0);
        grp_accum<UNG, KIND, HDR>(B, S, L, lane, Rq);
        __builtin_amdgcn_sched_barrier(0);
    }
    wave_order();
    if constexpr (HDR)
        rh = (uint16_t)L.res_h[lane];
    return (uint16_t)L.res[lane];
}

// Dense-tile test (wave-uniform): every valid packet non-empty, starts and
// ends non-decreasing, gaps below 4 KiB, and the range at most 9/8 of the
// tile's bytes + 2 KiB.  Sets the range [A0, A0 + 16 T).
__device__ __forceinline__ bool seg_dense(int lane, uint64_t a, uint32_t len, bool valid,
                                          uint32_t nvalid, uint64_t &A0, uint32_t &T)
{
    const uint64_t e = a + len;
    const uint64_t elast = lane_u64(e, (int)nvalid - 1);
    const uint64_t s0 = valid ? a : elast, s1 = valid ? e : elast;
    const uint64_t p0 = wave_shr1_u64(s0), p1 = wave_shr1_u64(s1);
    const bool ok = !valid || (len != 0 && (lane == 0 ||
                                            (s0 >= p0 && s1 >= p1 && s0 < p1 + 4096u)));
    if (__ballot(!ok))
        return false;
    const uint32_t sum = lane_u32(wave_incl_sum(valid ? len : 0u), 63);
    A0 = lane_u64(s0, 0) & ~15ull;
    const uint64_t range = elast - A0;
    if (range > (uint64_t)sum + sum / 8u + 2048u)
        return false;
    T = (uint32_t)((range + 15u) >> 4);
    return true;
}

// payload_cksum of one packet by its own lane, exact byte-lane sums over its
// chunks (in_cksum.c:140-167, the strided kernel's edge-chunk arithmetic):
// the seg-only kernel's fallback for a packet whose header is longer than it
// or whose odd-start sum could wrap -- rare, so a serial loop.
template <bool NT>
__device__ __noinline__ uint16_t lane_payload_exact(uint64_t a, uint32_t len)
{
    const PseudoHdr ph = hdr_pseudo(load_hdr(a), a);
    const uint32_t s = (uint32_t)(a & 15u);
    const uint64_t c0 = a & ~15ull;
    const uint32_t nch = (s + max(len, 20u) + 15u) >> 4;
    uint32_t E = 0, O = 0;
    for (uint32_t k = 0; k < nch; ++k)
        accum_arith<WC_KIND_PAYLOAD>(load_chunk<NT>(c0 + 16ull * k), 16 * (int)k - (int)s,
                                     (int)ph.hl, (int)len, ph.v4, E, O);
    return fold_not(combine(E, O, s & 1u) + ph.special);
}

} // namespace
} // namespace wc
