// wc_device.h -- device helpers shared by the gfx950 (MI355X / CDNA4) kernels
// for warpcore's RFC 1071 Internet / UDP checksum (wc_k_*.hip).
//
// Reference semantics (read, not copied):
//   /root/reference/lib/src/in_cksum.c:107-120  csum_oc16: Σ of native LE
//       16-bit words into a uint32, odd trailing byte as a low byte;
//   /root/reference/lib/src/in_cksum.c:74-80    csum_oc16_reduce: fold the
//       end-around carry, complement;
//   /root/reference/lib/src/in_cksum.c:133-137  ip_cksum;
//   /root/reference/lib/src/in_cksum.c:140-167  payload_cksum (IPv4 / IPv6
//       pseudo-header, header layouts ip4.h:55-66 and ip6.h:45-57).
//
// Design:
//   * Loads are always 16-byte-aligned chunks covering [start & ~15, end)
//     (global_load_dwordx4 nt, coalesced).  An aligned chunk that overlaps the
//     packet never crosses a page, so this can't fault at an allocation edge.
//   * Each lane keeps two EXACT byte-lane sums with v_dot4_u32_u8: E = Σ bytes
//     at even addresses, O = Σ bytes at odd addresses.  The reference's uint32
//     accumulator is exactly E + 256*O (packet starts at an even address) or
//     O + 256*E (odd start), modulo 2^32 -- bit-identical for every alignment,
//     including the reference's uint32 wrap on IPv6 next_hdr << 24
//     (in_cksum.c:157).  Head/tail masking and the pseudo-header fields
//     payload_cksum adds with their natural word weight are dot4 byte weights:
//     computed from the range bounds in the strided kernel (edge chunks are
//     rare there), looked up in small LDS tables in the flat kernel.
//   * Strided batches: a GROUP of G lanes of one wave64 owns a packet (G = 64
//     is "one packet per wavefront"), every lane issuing CPL x U loads before
//     any arithmetic.  Ragged batches: the chunk-balanced flat kernel deals
//     16-byte chunks, not packets, to lanes (section 4.3).
//   * No MFMA: a pure HBM-read stream (roofline: HBM).
//
// Kernels: wc_k_strided.hip (group-per-packet, strided batches), wc_k_flat.hip
// (chunk-balanced flat kernel), wc_k_seg.hip (segmented-prefix tile kernel
// with its grouped and flat paths), wc_k_synth.hip (synthetic bytes).  Every
// helper here has internal linkage, so each kernel translation unit carries
// its own copy of the device tables.
#pragma once

#include <hip/hip_runtime.h>
#include <utility>
#include <stdint.h>

#include <algorithm>

#include "wc_cksum_kernels.h"

namespace wc {
namespace {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// dot4 byte weights: bytes 0 and 2 of a dword sit at even addresses (chunks
// are 16-byte aligned), bytes 1 and 3 at odd addresses.
constexpr uint32_t kEvenW = 0x00010001u;
constexpr uint32_t kOddW = 0x01000100u;
constexpr uint32_t kEvenB = 0x00FF00FFu;
constexpr uint32_t kOddB = 0xFF00FF00u;

__device__ __forceinline__ uint32_t dot4(uint32_t x, uint32_t w, uint32_t acc)
{
    return __builtin_amdgcn_udot4(x, w, acc, false);
}

__device__ __forceinline__ uint32_t pick_dword(const u32x4 &d, int j)
{
    return j == 0 ? d.x : j == 1 ? d.y : j == 2 ? d.z : d.w;
}

__device__ __forceinline__ uint32_t pick_byte(const u32x4 &d, int pos)
{
    return (pick_dword(d, pos >> 2) >> (8 * (pos & 3))) & 0xFFu;
}

// WC_VARIANT (experimental kernel branches for A/B timing, some of which
// drop results, e.g. bit 64 = no result store) exists only in the tuning
// build (-DWC_TUNING, libwccksum_tune.so, tools/).  The shipped library
// compiles every kernel with variant 0, so those branches are folded away and
// no environment variable can change a result.
__device__ __forceinline__ constexpr int tuning_variant(int v)
{
#ifdef WC_TUNING
    return v;
#else
    return (void)v, 0;
#endif
}

// Logical block of this workgroup, XCD-contiguous within super-blocks of
// 4096 workgroups: workgroups are placed on the 8 XCDs round-robin
// (blockIdx.x % 8), so inside each super-block XCD x gets logical blocks
// [x q + min(x, r), + q + (x < r)) -- one contiguous eighth of the
// super-block per XCD instead of interleaved 1/8-strips (q = m / 8, r = m % 8
// for a super-block of m workgroups; a bijection for any grid).  Bounding the
// span keeps the 8 XCDs' streams within a few hundred MB of each other:
// remapping the whole grid left them gigabytes apart and cost up to 8 points
// on large batches (address-translation reach).  Measured vs no remap and vs
// a whole-grid remap: profiles/ab_r01_xcd_remap.log.  WC_VARIANT bit 8 turns
// it off, bits 8..15 = k set the span to 2^k (k >= 31: whole grid) (A/B).
__device__ __forceinline__ uint64_t xcd_block(int variant)
{
    const uint32_t b = blockIdx.x, nb = gridDim.x;
    if (variant & 8)
        return b;
    const uint32_t k = ((uint32_t)variant >> 8) & 0xFFu;
    // Power-of-two spans: shifts, not a division (this runs before any
    // load of every wave, so it is on the critical path of small batches).
    uint32_t base = 0, m = nb;
    if (k < 31) {
        const uint32_t sh = k == 0 ? 12u : k;
        base = (b >> sh) << sh;
        m = min(1u << sh, nb - base);
    }
    const uint32_t l = b - base;
    const uint32_t x = l & 7u, q = m >> 3, r = m & 7u;
    return (uint64_t)(base + x * q + min(x, r) + (l >> 3));
}

// Global (addrspace 1) pointer: lets hipcc emit global_load_dwordx4 rather
// than flat loads for addresses computed as integers.
typedef const u32x4 __attribute__((address_space(1))) *gchunk_ptr;

template <bool NT>
__device__ __forceinline__ u32x4 load_chunk(uint64_t addr)
{
    gchunk_ptr p = (gchunk_ptr)(uintptr_t)addr;
    if constexpr (NT)
        return __builtin_nontemporal_load(p);
    else
        return *p;
}

typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));

// V += the dword's two little-endian 16-bit words (v_dot2_u32_u16): the sum
// of the words at even addresses of a 16-byte-aligned chunk.
__device__ __forceinline__ uint32_t wsum(uint32_t x, uint32_t acc)
{
    return __builtin_amdgcn_udot2(__builtin_bit_cast(u16x2, x), u16x2{1, 1}, acc, false);
}

// 0xFF in the bytes of dword j that are among the first q bytes of a chunk.
__device__ __forceinline__ uint32_t head_mask(uint32_t q, int j)
{
    const uint32_t nb = min(q - min(q, 4u * j), 4u);
    return nb >= 4u ? 0xFFFFFFFFu : ((1u << (8u * nb)) - 1u);
}

// in_cksum.c:74-80 -- two end-around folds always suffice for a uint32.
__device__ __forceinline__ uint16_t fold_not(uint32_t s)
{
    s = (s & 0xFFFFu) + (s >> 16);
    s = (s & 0xFFFFu) + (s >> 16);
    return (uint16_t)~s;
}

// Exact reference accumulator of a lane's byte-lane sums (mod 2^32).
__device__ __forceinline__ uint32_t combine(uint32_t E, uint32_t O, bool odd_start)
{
    return odd_start ? O + (E << 8) : E + (O << 8);
}

// payload_cksum's per-packet terms that are not byte-weighted sums
// (in_cksum.c:142-160): version / header length from byte 0 (ip4.h:75-92),
// IPv4 plen = bswap16(bswap16(ip->len) - hl) read as a native word
// (152-153), IPv6 next_hdr << 24 (157).
struct PseudoHdr {
    uint32_t hl, v4, special;
};

__device__ __forceinline__ PseudoHdr pseudo_hdr(uint32_t b0, uint32_t b2,
                                                uint32_t b3, uint32_t b6)
{
    PseudoHdr h;
    h.v4 = (b0 >> 4) == 4u;
    h.hl = h.v4 ? (b0 & 15u) * 4u : 40u;
    if (h.v4) {
        const uint32_t x = (((b2 << 8) | b3) - h.hl) & 0xFFFFu;
        h.special = ((x & 0xFFu) << 8) | (x >> 8);
    } else {
        h.special = b6 << 24;
    }
    return h;
}

// ---------------------------------------------------------------------------
// LDS weight tables.
//
// keep[lo * 17 + hi]    0xFF in byte b of a chunk iff lo <= b < hi
// hdr[v4][co + 16]      0x01 in byte b iff packet offset co + b is one of the
//                       pseudo-header fields payload_cksum adds with natural
//                       word weight: IPv4 proto @9, src/dst @12..19
//                       (in_cksum.c:149-151); IPv6 payload length @4..5,
//                       src/dst @8..39 (158-160); co in [-16, 40), entry 56 = 0
constexpr int kHdrSlots = 57;

struct WeightLut {
    u32x4 keep[17 * 17];
    u32x4 hdr[2][kHdrSlots];
};

constexpr bool hdr_field(int v4, int o)
{
    return v4 ? (o == 9 || (o >= 12 && o < 20))
              : (o == 4 || o == 5 || (o >= 8 && o < 40));
}

constexpr int kLutKeep = 17 * 17;
constexpr int kLutAll = kLutKeep + 2 * kHdrSlots;

struct WeightTable {
    uint32_t w[kLutAll][4];
};

constexpr WeightTable make_weight_table()
{
    WeightTable t{};
    for (int i = 0; i < kLutAll; ++i)
        for (int j = 0; j < 4; ++j) {
            uint32_t v = 0;
            for (int b = 0; b < 4; ++b) {
                const int pos = 4 * j + b;
                bool on = false;
                if (i < kLutKeep) {
                    on = pos >= i / 17 && pos < i % 17;
                } else {
                    const int k = i - kLutKeep, v4 = k / kHdrSlots, slot = k % kHdrSlots;
                    on = slot < kHdrSlots - 1 && hdr_field(v4, slot - 16 + pos);
                }
                v |= (on ? (i < kLutKeep ? 0xFFu : 1u) : 0u) << (8 * b);
            }
            t.w[i][j] = v;
        }
    return t;
}

// Generated at compile time; each flat-kernel block copies it into LDS (6.4 KB).
__device__ const WeightTable kWeightTable = make_weight_table();

// 16 zero bytes: the strided kernel's dead load slots read this instead of
// branching around the load.
__device__ __attribute__((aligned(16))) const uint32_t kZeroChunk[4] = {0u, 0u, 0u, 0u};

__device__ __forceinline__ void load_weight_lut(WeightLut &M)
{
    u32x4 *dst = reinterpret_cast<u32x4 *>(&M);
    const u32x4 __attribute__((address_space(1))) *src =
        (const u32x4 __attribute__((address_space(1))) *)&kWeightTable;
    for (int i = threadIdx.x; i < kLutAll; i += blockDim.x)
        dst[i] = src[i];
}

// Accumulate one 16-byte chunk whose start is `co` bytes after the packet
// start: bytes at packet offsets [rs, re) get weight 1, and for
// payload_cksum the pseudo-header field bytes get one more (so a malformed
// IHL < 5 that makes the payload overlap src/dst double-counts them, as the
// reference does).
template <int KIND>
__device__ __forceinline__ void accum_masked(const u32x4 &d, int co, int rs, int re,
                                             uint32_t v4, const WeightLut &M,
                                             uint32_t &E, uint32_t &O)
{
    const int lo = min(max(rs - co, 0), 16), hi = min(max(re - co, 0), 16);
    const u32x4 keep = M.keep[lo * 17 + hi];
    if constexpr (KIND == WC_KIND_PAYLOAD) {
        const int slot = (co >= -16 && co < 40) ? co + 16 : kHdrSlots - 1;
        // byte weights <= 2: no carries between bytes
        const u32x4 w = (keep & 0x01010101u) + M.hdr[v4][slot];
        E = dot4(d.x, w.x & kEvenB, E);
        O = dot4(d.x, w.x & kOddB, O);
        E = dot4(d.y, w.y & kEvenB, E);
        O = dot4(d.y, w.y & kOddB, O);
        E = dot4(d.z, w.z & kEvenB, E);
        O = dot4(d.z, w.z & kOddB, O);
        E = dot4(d.w, w.w & kEvenB, E);
        O = dot4(d.w, w.w & kOddB, O);
    } else {
        const u32x4 m = d & keep; // masked bytes, then the fixed byte-lane weights
        E = dot4(m.x, kEvenW, E);
        O = dot4(m.x, kOddW, O);
        E = dot4(m.y, kEvenW, E);
        O = dot4(m.y, kOddW, O);
        E = dot4(m.z, kEvenW, E);
        O = dot4(m.z, kOddW, O);
        E = dot4(m.w, kEvenW, E);
        O = dot4(m.w, kOddW, O);
    }
}

__device__ __forceinline__ void accum_full(const u32x4 &d, uint32_t &E, uint32_t &O)
{
    E = dot4(d.x, kEvenW, E);
    O = dot4(d.x, kOddW, O);
    E = dot4(d.y, kEvenW, E);
    O = dot4(d.y, kOddW, O);
    E = dot4(d.z, kEvenW, E);
    O = dot4(d.z, kOddW, O);
    E = dot4(d.w, kEvenW, E);
    O = dot4(d.w, kOddW, O);
}

// Arithmetic byte weights (no tables): bit b of a 16-bit chunk mask becomes
// weight 0x01 in byte b.  n * 0x204081 places bit k of a nibble at bits
// k, k+7, k+14, k+21 -- all distinct, so no carries -- and bits 0/8/16/24
// come from k = 0/1/2/3 alone.
__device__ __forceinline__ uint32_t expand_nibble(uint32_t bits, int j)
{
    return (((bits >> (4 * j)) & 0xFu) * 0x00204081u) & 0x01010101u;
}

// Pseudo-header field bytes of payload_cksum as bit masks over packet offsets
// (same fields as hdr_field above), pre-shifted by 16 so a chunk starting at
// co >= -16 reads its 16 bits at (co + 16).
constexpr uint64_t kHdrBitsV4 = ((1ull << 9) | (0xFFull << 12)) << 16;
constexpr uint64_t kHdrBitsV6 = ((1ull << 4) | (1ull << 5) | (0xFFFFFFFFull << 8)) << 16;

// accum_masked without the LDS tables: the weights are computed from the
// range bounds, a few VALU ops per dword (used where edge chunks are rare).
template <int KIND>
__device__ __forceinline__ void accum_arith(const u32x4 &d, int co, int rs, int re,
                                            uint32_t v4, uint32_t &E, uint32_t &O)
{
    const int lo = min(max(rs - co, 0), 16);
    const int hi = max(min(max(re - co, 0), 16), lo);
    const uint32_t kb = (1u << hi) - (1u << lo);
    uint32_t hb = 0;
    if constexpr (KIND == WC_KIND_PAYLOAD) {
        const uint32_t sh = (uint32_t)min(co + 16, 63);
        hb = (uint32_t)((v4 ? kHdrBitsV4 : kHdrBitsV6) >> sh) & 0xFFFFu;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        uint32_t w = expand_nibble(kb, j);
        if constexpr (KIND == WC_KIND_PAYLOAD)
            w += expand_nibble(hb, j); // byte weights <= 2
        const uint32_t x = pick_dword(d, j);
        E = dot4(x, w & kEvenB, E);
        O = dot4(x, w & kOddB, O);
    }
}

// One chunk of the strided kernel: chunks strictly inside the summed range
// (and past the header) take the full-weight path; the wave takes the masked
// path only when one of its lanes holds a head / tail / header chunk of its
// packet (`live`: the chunk is one of the packet's own -- slots past the end
// hold zeros and need no mask).  Edge weights are computed (accum_arith), so
// the strided kernel needs no LDS at all.  With HDR the IP header bytes
// [0, hl) also go into (Eh, Oh) for the fused IPv4 header checksum.
template <int KIND, bool FULL, bool HDR>
__device__ __forceinline__ void accum_strided(const u32x4 &d, int co, int rs, int re,
                                              bool live, uint32_t v4, uint32_t &E,
                                              uint32_t &O, uint32_t &Eh, uint32_t &Oh)
{
    if constexpr (FULL) {
        accum_full(d, E, O);
    } else {
        const int head = KIND == WC_KIND_PAYLOAD ? max(rs, 40) : rs;
        const bool edge = live && (co < head || co + 16 > re);
        if (__ballot(edge)) {
            accum_arith<KIND>(d, co, rs, re, v4, E, O);
            if constexpr (HDR)
                accum_arith<WC_KIND_IP>(d, co, 0, rs, 0u, Eh, Oh);
        } else {
            accum_full(d, E, O);
        }
    }
}

__device__ __forceinline__ uint32_t lane_u32(uint32_t v, int l)
{
    return (uint32_t)__builtin_amdgcn_readlane((int)v, l);
}

// DPP move with every source lane valid (quad_perm / mirror patterns).
template <int CTRL>
__device__ __forceinline__ uint32_t dpp_all(uint32_t v)
{
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, 0xF, 0xF, false);
}

// Sum over each aligned group of G lanes (mod 2^32), in every lane of the
// group.  DPP within a 16-lane row (quad_perm xor 1 / xor 2, row_half_mirror,
// row_mirror), readlane across rows: no LDS round trips (ds_bpermute), which
// dominated the small-packet shapes' per-packet cost.
template <int G>
__device__ __forceinline__ uint32_t group_sum(uint32_t v)
{
    if constexpr (G >= 2)
        v += dpp_all<0xB1>(v); // quad_perm [1,0,3,2]
    if constexpr (G >= 4)
        v += dpp_all<0x4E>(v); // quad_perm [2,3,0,1]
    if constexpr (G >= 8)
        v += dpp_all<0x141>(v); // row_half_mirror: the other quad of the 8
    if constexpr (G >= 16)
        v += dpp_all<0x140>(v); // row_mirror: the other half of the row
    if constexpr (G == 32) {
        const uint32_t lo = lane_u32(v, 0) + lane_u32(v, 16);
        const uint32_t hi = lane_u32(v, 32) + lane_u32(v, 48);
        v = (threadIdx.x & 32) ? hi : lo;
    } else if constexpr (G == 64) {
        v = lane_u32(v, 0) + lane_u32(v, 16) + lane_u32(v, 32) + lane_u32(v, 48);
    }
    return v;
}

constexpr int kDppRowBcast15Ctl = 0x142; // row_bcast:15 (DPP controls below)
constexpr int kDppRowShr4Ctl = 0x114;    // row_shr:4

// Lane N of each aligned group of G lanes, in every lane of the group:
// DPP quad_perm for G = 4; for G = 8 quad_perm and, in the group's second
// quad, row_shr:4 of it; row_newbcast for G = 16 (one 16-lane row), plus
// row_bcast:15 into the odd rows for G = 32 (lane 15 of rows 0 / 2 then
// holds their lane N); readlane for G = 64.  Every lane must be active.
template <int G, int N>
__device__ __forceinline__ uint32_t group_bcast(uint32_t v)
{
    static_assert(G == 4 || G == 8 || G == 16 || G == 32 || G == 64, "group width");
    static_assert(N >= 0 && N < 4, "source lane within the group's first quad");
    if constexpr (G == 64) {
        return (uint32_t)__builtin_amdgcn_readlane((int)v, N);
    } else if constexpr (G <= 8) {
        const uint32_t q = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, N * 0x55, 0xF, 0xF,
                                                                 false);
        if constexpr (G == 4)
            return q;
        const uint32_t sh = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)q, kDppRowShr4Ctl, 0xF,
                                                                  0xF, false);
        return (threadIdx.x & 4) ? sh : q;
    } else {
        const uint32_t t = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x150 + N, 0xF, 0xF,
                                                                 false);
        if constexpr (G == 16)
            return t;
        return (uint32_t)__builtin_amdgcn_update_dpp((int)t, (int)t, kDppRowBcast15Ctl, 0xA, 0xF,
                                                     false);
    }
}

// payload_cksum's header window dwords K0 .. K0 + NW - 1 of a packet whose
// start phase in its 16-byte chunk is the same for the whole batch (stride a
// multiple of 16): window dword k is dword k & 3 of group lane k >> 2, both
// known at compile time here, so each word is one broadcast from one lane and
// no per-lane select.
template <int G, int K0, int... J>
__device__ __forceinline__ void hdr_words_uni(const u32x4 &d0, uint32_t *w,
                                              std::integer_sequence<int, J...>)
{
    ((w[J] = group_bcast<G, ((K0 + J) >> 2)>(d0[(K0 + J) & 3])), ...);
}

constexpr int kFlatWaves = 4; // 256-thread blocks

// DPP controls (GFX9 family, gfx950 included).
constexpr int kDppRowShr = 0x110; // + 1..15
constexpr int kDppRowBcast15 = 0x142;
constexpr int kDppRowBcast31 = 0x143;

// Lanes whose DPP source is outside the row / disabled read 0.
template <int CTRL, int ROWS>
__device__ __forceinline__ uint32_t dpp0(uint32_t v)
{
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, ROWS, 0xF, true);
}

// Inclusive wave64 prefix sum (mod 2^32).
__device__ __forceinline__ uint32_t wave_incl_sum(uint32_t v)
{
    v += dpp0<kDppRowShr + 1, 0xF>(v);
    v += dpp0<kDppRowShr + 2, 0xF>(v);
    v += dpp0<kDppRowShr + 4, 0xF>(v);
    v += dpp0<kDppRowShr + 8, 0xF>(v);
    v += dpp0<kDppRowBcast15, 0xA>(v); // rows 1, 3 += end of rows 0, 2
    v += dpp0<kDppRowBcast31, 0xC>(v); // rows 2, 3 += end of row 1
    return v;
}

__device__ __forceinline__ uint32_t mbcnt64(uint64_t m)
{
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                     __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// Wave-uniform broadcasts and shifts without LDS round trips (readlane /
// DPP instead of ds_bpermute); lane_u32 is defined with group_sum.

__device__ __forceinline__ uint64_t lane_u64(uint64_t v, int l)
{
    return (uint64_t)lane_u32((uint32_t)v, l) | ((uint64_t)lane_u32((uint32_t)(v >> 32), l) << 32);
}

constexpr int kDppWaveShr1 = 0x138;

// v of lane - 1 (0 in lane 0).
__device__ __forceinline__ uint64_t wave_shr1_u64(uint64_t v)
{
    return (uint64_t)dpp0<kDppWaveShr1, 0xF>((uint32_t)v) |
           ((uint64_t)dpp0<kDppWaveShr1, 0xF>((uint32_t)(v >> 32)) << 32);
}

// Wave maximum (DPP max-scan; lane 63 holds the result).
__device__ __forceinline__ uint32_t wave_max(uint32_t v)
{
    v = max(v, dpp0<kDppRowShr + 1, 0xF>(v));
    v = max(v, dpp0<kDppRowShr + 2, 0xF>(v));
    v = max(v, dpp0<kDppRowShr + 4, 0xF>(v));
    v = max(v, dpp0<kDppRowShr + 8, 0xF>(v));
    v = max(v, dpp0<kDppRowBcast15, 0xA>(v));
    v = max(v, dpp0<kDppRowBcast31, 0xC>(v));
    return lane_u32(v, 63);
}

// Packet p's offset and length, or packet 0's offset and length 0 past the
// batch end -- with unconditional loads.
__device__ __forceinline__ void meta_load(const uint64_t *__restrict__ offs,
                                          const uint16_t *__restrict__ lens, uint64_t p,
                                          uint64_t n, uint64_t &off, uint32_t &len)
{
    const bool v = p < n;
    const uint64_t pc = v ? p : 0;
    off = offs[pc];
    const uint32_t l = lens[pc];
    len = v ? l : 0u;
}

} // namespace
} // namespace wc
