// wc_cksum_kernels.hip -- gfx950 (MI355X / CDNA4) kernels for warpcore's
// RFC 1071 Internet / UDP checksum.
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

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "wc_cksum_kernels.h"

namespace wc {

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
    const uint32_t span = k == 0 ? 4096u : k >= 31 ? nb : (1u << k);
    const uint32_t base = b / span * span, m = min(span, nb - base), l = b - base;
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
        uint16_t *__restrict__ out_hdr, int variant)
{
    static_assert(!(RAGGED && (FULL || HDR)), "ragged group variant: masked, no header");
    static_assert(!HDR || KIND == WC_KIND_PAYLOAD, "header checksum rides on payload");
    static_assert(G >= 4 && G <= 64 && (G & (G - 1)) == 0, "group width");
    static_assert(!(FULL && KIND == WC_KIND_PAYLOAD), "payload needs masks");
    constexpr int GPW = 64 / G;
    constexpr uint64_t PPW = (uint64_t)GPW * U;
    constexpr int PASS = G * CPL;

    const int lane = threadIdx.x & 63;
    const int gl = lane & (G - 1);
    const int grp = lane / G;
    const int lead = lane & ~(G - 1);
    const uint64_t wave = xcd_block(variant) * (blockDim.x >> 6) + (threadIdx.x >> 6);
    const uint64_t nwaves = (uint64_t)gridDim.x * (blockDim.x >> 6);
    uint32_t nbad = 0;
    const uint64_t zero = (uint64_t)(uintptr_t)&kZeroChunk;

    for (uint64_t p0 = wave * PPW; p0 < n; p0 += nwaves * PPW) {
        uint64_t c0[U];
        uint32_t nch[U], plen[U];
        int s[U];
        bool valid[U];
        u32x4 d[U][CPL];

#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t i = p0 + (uint64_t)u * GPW + grp;
            valid[u] = i < n;
            const uint64_t ii = valid[u] ? i : p0;
            uint64_t a;
            if constexpr (RAGGED) {
                a = (uint64_t)base + offs[ii];
                plen[u] = lens[ii];
            } else {
                a = (uint64_t)base + ii * stride;
                plen[u] = len;
            }
            // payload_cksum reads the IPv4 header fields up to byte 19 even
            // for a shorter len (in_cksum.c:149-151), so cover them too.
            const uint32_t span = KIND == WC_KIND_PAYLOAD ? max(plen[u], 20u) : plen[u];
            s[u] = (int)(a & 15u);
            c0[u] = a & ~15ull;
            nch[u] = valid[u] ? (uint32_t)((a + span + 15u - c0[u]) >> 4) : 0u;
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

#pragma unroll
        for (int u = 0; u < U; ++u) {
            PseudoHdr ph{0u, 1u, 0u};
            if constexpr (KIND == WC_KIND_PAYLOAD) {
                // Header bytes 0, 2, 3, 6 sit in the group's chunks 0/1, i.e.
                // in d[u][0] of group lanes 0 and 1.
                const int su = s[u];
                const uint32_t b0 = __shfl(pick_byte(d[u][0], su), lead + (su >> 4), 64);
                const uint32_t b2 = __shfl(pick_byte(d[u][0], (su + 2) & 15),
                                           lead + ((su + 2) >> 4), 64);
                const uint32_t b3 = __shfl(pick_byte(d[u][0], (su + 3) & 15),
                                           lead + ((su + 3) >> 4), 64);
                const uint32_t b6 = __shfl(pick_byte(d[u][0], (su + 6) & 15),
                                           lead + ((su + 6) >> 4), 64);
                ph = pseudo_hdr(b0, b2, b3, b6);
            }
            const int rs = (int)ph.hl, re = (int)plen[u];

            uint32_t E = 0, O = 0, Eh = 0, Oh = 0;
#pragma unroll
            for (int c = 0; c < CPL; ++c)
                accum_strided<KIND, FULL, HDR>(d[u][c], 16 * (gl + c * G) - s[u], rs, re,
                                               (uint32_t)(gl + c * G) < nch[u], ph.v4, E, O,
                                               Eh, Oh);
            // Packets longer than one pass (e.g. 9000 B jumbo frames).
            for (uint32_t kb = PASS; kb < nch[u]; kb += PASS) {
                u32x4 t[CPL];
#pragma unroll
                for (int c = 0; c < CPL; ++c) {
                    const uint32_t k = kb + (uint32_t)(gl + c * G);
                    t[c] = load_chunk<NT>(k < nch[u] ? c0[u] + 16ull * k : zero);
                }
#pragma unroll
                for (int c = 0; c < CPL; ++c)
                    accum_strided<KIND, FULL, HDR>(t[c], 16 * (int)(kb + gl + c * G) - s[u],
                                                   rs, re, kb + (uint32_t)(gl + c * G) < nch[u],
                                                   ph.v4, E, O, Eh, Oh);
            }

            uint32_t S = combine(E, O, s[u] & 1);
            S += gl == 0 ? ph.special : 0u;
            S = group_sum<G>(S);
            uint32_t Sh = 0;
            if constexpr (HDR)
                Sh = group_sum<G>(combine(Eh, Oh, s[u] & 1));
            if (gl == 0 && valid[u]) {
                const uint64_t i = p0 + (uint64_t)u * GPW + grp;
                const uint16_t r = fold_not(S);
                if (out)
                    out[i] = r;
                nbad += r != 0;
                if constexpr (HDR)
                    out_hdr[i] = ph.v4 ? fold_not(Sh) : 0; // ip4.c:110-115
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

struct FlatDesc {          // 16 bytes per non-empty packet of the tile, in LDS
    uint32_t vb_lo, vb_hi; // chunk q of the packet sits at vb + 16 q
    uint32_t rel;          // packet start in the tile's slot-byte space
    uint32_t info;         // len | hl << 16 | v4 << 24
};

template <int UN>
struct FlatRows {
    u32x4 d[UN];
    uint32_t own[UN];
};

template <int UN>
struct FlatLds {
    FlatDesc desc[64];
    uint32_t mark[UN][64]; // run-start tags, one array per row of a group
    uint32_t pre[64 * UN]; // inclusive prefix sums of the group's chunk sums
};

// Intra-wave LDS hand-offs need no fence: one wave's LDS instructions execute
// in issue order.  wave_barrier only stops hipcc moving LDS accesses across.
__device__ __forceinline__ void wave_order()
{
    __builtin_amdgcn_wave_barrier();
}

// Owner lookup + loads for the UN rows of a group starting at slot g0.
template <int UN, bool NT, bool NOLOAD = false>
__device__ __forceinline__ void flat_issue(FlatRows<UN> &R, FlatLds<UN> &L,
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
        const uint64_t vb = *reinterpret_cast<const uint64_t *>(&L.desc[own]);
        // Unconditional load (slots past the tile's end re-read its last
        // chunk and are zeroed in flat_accum): a straight-line issue stream
        // lets hipcc wait for exactly the older row group.
        const uint32_t q = min(row0 + (uint32_t)lane, total - 1u);
        if constexpr (NOLOAD) // diagnostic build: same stream, no HBM traffic
            R.d[u] = u32x4{(uint32_t)vb, q, (uint32_t)(vb >> 32), q ^ 0x5a5a5a5au};
        else
            R.d[u] = load_chunk<NT>(vb + 16ull * q);
    }
}

template <int UN, int KIND, bool ARITH = false>
__device__ __forceinline__ void flat_accum(const FlatRows<UN> &R, FlatLds<UN> &L,
                                           const WeightLut *M, uint32_t g0,
                                           int lane, uint32_t cp, uint32_t ce,
                                           uint32_t total, uint32_t &acc)
{
    uint32_t P[UN];
#pragma unroll
    for (int u = 0; u < UN; ++u) {
        const uint32_t q = g0 + 64u * u + (uint32_t)lane;
        const FlatDesc &g = L.desc[R.own[u]];
        const uint32_t rel = g.rel, info = g.info;
        uint32_t E = 0, O = 0;
        if constexpr (ARITH)
            accum_arith<KIND>(R.d[u], (int)(16u * q - rel), (int)((info >> 16) & 0xFFu),
                              (int)(info & 0xFFFFu), (info >> 24) & 1u, E, O);
        else
            accum_masked<KIND>(R.d[u], (int)(16u * q - rel), (int)((info >> 16) & 0xFFu),
                               (int)(info & 0xFFFFu), (info >> 24) & 1u, *M, E, O);
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

// One 64-packet tile of the flat kernel: returns this lane's packet's exact
// reference accumulator (in_cksum.c:140-167 / 107-120, mod 2^32) -- the
// caller folds it.  `after_first_issue` runs once the tile's first row group
// is in flight (the caller's next-tile prefetch goes there).
template <int UN, int KIND, bool NT, bool NOLOAD, bool ARITH, class F>
__device__ __forceinline__ uint32_t flat_tile_sum(FlatLds<UN> &L, const WeightLut *lut,
                                                  int lane, uint64_t a, uint32_t len,
                                                  bool valid, const PseudoHdr &ph,
                                                  F &&after_first_issue)
{
    const uint32_t s = (uint32_t)(a & 15u);
    const uint32_t span = KIND == WC_KIND_PAYLOAD ? max(len, 20u) : len;
    const uint32_t nch = valid ? (s + span + 15u) >> 4 : 0u;

    // Chunk-slot range [cp, ce) of this lane's packet within the tile;
    // rank among the tile's non-empty packets.
    const uint32_t ce = wave_incl_sum(nch);
    const uint32_t cp = ce - nch;
    const uint32_t total = lane_u32(ce, 63);
    const uint64_t nonempty = __ballot(nch != 0);
    const uint32_t rank = mbcnt64(nonempty);
    const uint32_t last_rank = nonempty ? (uint32_t)__builtin_popcountll(nonempty) - 1u : 0u;
    const uint64_t vb = (a & ~15ull) - 16ull * cp;
    if (nch != 0)
        L.desc[rank] = FlatDesc{(uint32_t)vb, (uint32_t)(vb >> 32), s + 16u * cp,
                                len | (ph.hl << 16) | (ph.v4 << 24)};
    // Row marks carry the row's number within the tile; reset them to a
    // tag no row has so the previous tile's marks can't match.
#pragma unroll
    for (int u = 0; u < UN; ++u)
        L.mark[u][lane] = 0xFFFFFFFFu;
    wave_order();

    uint32_t acc = ph.special;
    constexpr uint32_t kGrp = 64u * UN;
    FlatRows<UN> A, B;
    if (total != 0)
        flat_issue<UN, NT, NOLOAD>(A, L, 0, lane, cp, ce, rank, last_rank, total);
    after_first_issue();
    if (total != 0) {
        // Ping-pong row groups A / B (no register copies): group g+1's
        // loads are in flight while group g is summed.  No exit between
        // the halves: a half past the tile's end sums zeros, and keeping
        // each load's use in the next half stops hipcc sinking the load
        // next to it; sched_barrier keeps each issue ahead of the other
        // group's sum.
        for (uint32_t j = 0; j < total; j += 2 * kGrp) {
            flat_issue<UN, NT, NOLOAD>(B, L, j + kGrp, lane, cp, ce, rank, last_rank, total);
            __builtin_amdgcn_sched_barrier(0);
            flat_accum<UN, KIND, ARITH>(A, L, lut, j, lane, cp, ce, total, acc);
            __builtin_amdgcn_sched_barrier(0);
            flat_issue<UN, NT, NOLOAD>(A, L, j + 2 * kGrp, lane, cp, ce, rank, last_rank, total);
            __builtin_amdgcn_sched_barrier(0);
            flat_accum<UN, KIND, ARITH>(B, L, lut, j + kGrp, lane, cp, ce, total, acc);
            __builtin_amdgcn_sched_barrier(0);
        }
    }
    return acc;
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

template <int UN, int KIND, bool NT, bool HDR, bool NOLOAD = false>
__global__ void __launch_bounds__(256)
k_cksum_flat(const uint8_t *__restrict__ base, const uint64_t *__restrict__ offs,
             const uint16_t *__restrict__ lens, uint64_t n,
             uint16_t *__restrict__ out, unsigned long long *__restrict__ bad,
             uint16_t *__restrict__ out_hdr)
{
    static_assert(!HDR || KIND == WC_KIND_PAYLOAD, "header checksum rides on payload");
    __shared__ FlatLds<UN> lds_all[kFlatWaves];
    __shared__ WeightLut lut;
    load_weight_lut(lut);
    __syncthreads();

    const int lane = threadIdx.x & 63;
    const int w = threadIdx.x >> 6;
    FlatLds<UN> &L = lds_all[w];
    const uint64_t ntiles = (n + 63) / 64;
    const uint64_t nwaves = (uint64_t)gridDim.x * kFlatWaves;
    uint64_t tile = xcd_block(0) * kFlatWaves + w;
    uint32_t nbad = 0;

    // Metadata (and payload header bytes) of the first tile.  All prefetch
    // loads are unconditional (lanes past the batch end re-read packet 0):
    // a load under a branch leaves hipcc's wait counting no choice but
    // vmcnt(0), which would wait for the prefetch itself.
    uint64_t p = tile * 64 + lane;
    uint64_t off_n;
    uint32_t len_n;
    meta_load(offs, lens, p, n, off_n, len_n);
    HdrRaw hdr_n{};
    if constexpr (KIND == WC_KIND_PAYLOAD)
        hdr_n = load_hdr((uint64_t)base + off_n);

    for (; tile < ntiles; tile += nwaves) {
        p = tile * 64 + lane;
        const bool valid = p < n;
        const uint64_t off = off_n;
        const uint32_t len = len_n;
        const HdrRaw hdr = hdr_n;
        const uint64_t pn = (tile + nwaves) * 64 + lane;
        meta_load(offs, lens, pn, n, off_n, len_n); // prefetch the next tile's metadata

        const uint64_t a = (uint64_t)base + off;
        PseudoHdr ph{0u, 1u, 0u};
        if constexpr (KIND == WC_KIND_PAYLOAD)
            if (valid)
                ph = hdr_pseudo(hdr, a);
        // The next tile's header bytes: issued once its offsets are back,
        // behind this tile's first loads.
        const uint32_t acc = flat_tile_sum<UN, KIND, NT, NOLOAD, false>(
            L, &lut, lane, a, len, valid, ph, [&] {
                if constexpr (KIND == WC_KIND_PAYLOAD)
                    hdr_n = load_hdr((uint64_t)base + off_n);
            });

        const uint16_t r = fold_not(acc);
        if (valid && out)
            out[p] = r;
        nbad += valid && r != 0;
        if constexpr (HDR)
            if (valid)
                out_hdr[p] = ph.v4 ? lane_hdr_cksum<NT>(a, ph.hl, &lut) : 0;
        wave_order(); // the tables are rewritten by the next tile
    }
    if (bad) {
        nbad = group_sum<64>(nbad);
        if (lane == 0 && nbad)
            atomicAdd(bad, (unsigned long long)nbad);
    }
}

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

typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));

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
template <int UNS, int HC>
__device__ __forceinline__ void seg_accum(const SegRows<UNS> &R, uint32_t *pre, u32x4 *stage,
                                          uint32_t g0, int lane, uint32_t cs, uint32_t ce,
                                          uint32_t c0, uint32_t &carry, uint32_t &Ps,
                                          uint32_t &Pe, u32x4 &hs, u32x4 &he, u32x4 &h1,
                                          u32x4 &h2)
{
    constexpr uint32_t kGrp = 64u * UNS;
    uint32_t P[UNS];
#pragma unroll
    for (int u = 0; u < UNS; ++u)
        P[u] = seg_chunk<false>(R.d[u], 16u);
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
        const uint32_t d0 = c0 - g0; // (unsigned: c0 + 1 == g0 gives d0 + 1 == 0)
        if (d0 < kGrp)
            hs = stage[d0];
        if (d0 + 1u < kGrp)
            h1 = stage[d0 + 1u];
        if constexpr (HC >= 3)
            if (d0 + 2u < kGrp)
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

// One dense tile.  [a, a + len) is this lane's packet; ip_cksum sums all of
// it, payload_cksum the range [a + 8, a + len) corrected as below.  Returns
// the checksum, or done = false when a payload_cksum lane can't be summed
// here (header longer than the packet, possible uint32 wrap): the caller
// then takes the exact flat path for the tile.
template <int UNS, int KIND, bool NT, bool HDR>
__device__ __forceinline__ uint16_t seg_tile(uint32_t *pre, u32x4 *stage, int lane, uint64_t a,
                                             uint32_t len, bool valid, uint64_t A0, uint32_t T,
                                             uint64_t zero, bool &done, uint16_t &rh)
{
    constexpr uint32_t kGrp = 64u * UNS;
    constexpr bool PL = KIND == WC_KIND_PAYLOAD;
    constexpr int HC = PL ? (HDR ? 3 : 2) : 0;
    const uint64_t rs = a + (PL ? 8u : 0u) - A0, re = a + len - A0;
    const uint32_t cs = (uint32_t)(rs >> 4), qs = (uint32_t)(rs & 15u);
    const uint32_t ce = (uint32_t)(re >> 4), qe = (uint32_t)(re & 15u);
    const uint32_t c0 = (uint32_t)((a - A0) >> 4);

    SegRows<UNS> A, B;
    seg_issue<UNS, NT>(A, A0, 0, lane, T, zero);

    uint32_t carry = 0, Ps = 0, Pe = 0;
    u32x4 hs = {0u, 0u, 0u, 0u}, he = {0u, 0u, 0u, 0u}, h1 = {0u, 0u, 0u, 0u},
          h2 = {0u, 0u, 0u, 0u};
    uint32_t j = 0;
    for (; j < T; j += 2 * kGrp) {
        seg_issue<UNS, NT>(B, A0, j + kGrp, lane, T, zero);
        __builtin_amdgcn_sched_barrier(0);
        seg_accum<UNS, HC>(A, pre, stage, j, lane, cs, ce, c0, carry, Ps, Pe, hs, he, h1, h2);
        __builtin_amdgcn_sched_barrier(0);
        seg_issue<UNS, NT>(A, A0, j + 2 * kGrp, lane, T, zero);
        __builtin_amdgcn_sched_barrier(0);
        seg_accum<UNS, HC>(B, pre, stage, j + kGrp, lane, cs, ce, c0, carry, Ps, Pe, hs, he, h1,
                           h2);
        __builtin_amdgcn_sched_barrier(0);
    }
    if (ce >= j) // the packet ends exactly at the last row group's end
        Pe = carry;
    done = true;
    if constexpr (!PL) {
        const uint32_t v = (Pe + seg_chunk<true>(he, qe)) - (Ps + seg_chunk<true>(hs, qs));
        if (!(a & 1u))
            return fold_not(v);
        return fold_not(__builtin_amdgcn_alignbit(v, v, 24)); // rotl32(v, 8)
    } else {
        // Header bytes 0..11 from the packet's first two chunks (hs = c0, h1 =
        // c0 + 1); the start chunk cs is one of them.
        const uint32_t s = (uint32_t)(a & 15u);
        const uint32_t w0 = win_bytes(hs, h1, h2, s, 0), w1 = win_bytes(hs, h1, h2, s, 1),
                       w2 = win_bytes(hs, h1, h2, s, 2);
        const PseudoHdr ph = pseudo_hdr(w0 & 0xFFu, (w0 >> 16) & 0xFFu, w0 >> 24,
                                        (w1 >> 16) & 0xFFu);
        if (__ballot(valid && !seg_payload_ok(a, len, ph))) {
            done = false;
            return 0;
        }
        const u32x4 hq = cs == c0 ? hs : h1;
        // V of [a + 8, a + len): IPv6 src/dst + body (hl = 40); IPv4 bytes
        // 8..11, src/dst, options, body.
        uint32_t v = (Pe + seg_chunk<true>(he, qe)) - (Ps + seg_chunk<true>(hq, qs));
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
        const bool corr = ph.v4 && ph.hl != 20u;
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
            const uint32_t w3 = win_bytes(hs, h1, h2, s, 3), w4 = win_bytes(hs, h1, h2, s, 4);
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

// Ragged kernel with both paths: dense tiles stream their byte range
// (seg_tile), the others take the flat path.  (The fused header checksum
// stays on k_cksum_flat.)  STR: a strided batch (packet i at i * stride,
// slen bytes) -- packed packets at any alignment are one dense byte range,
// which the seg path streams better than the group kernel masks its
// boundary chunks; offsets and lengths are computed, not loaded.
template <int UN, int UNS, int UNG, int KIND, bool NT, bool STR, bool HDR = false>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(UNS >= 8 ? 2 : 4)))
k_cksum_seg(const uint8_t *__restrict__ base, const uint64_t *__restrict__ offs,
            const uint16_t *__restrict__ lens, uint64_t n, uint16_t *__restrict__ out,
            unsigned long long *__restrict__ bad, int grp_thr, int variant, uint64_t stride,
            uint32_t slen, uint16_t *__restrict__ out_hdr)
{
    static_assert(!HDR || KIND == WC_KIND_PAYLOAD, "header checksum rides on payload");
    union TileLds {
        FlatLds<UN> flat;
        GrpLds grp;
        struct {
            u32x4 stage[64 * UNS]; // the row group's chunks
            uint32_t pre[64 * UNS];
        } seg;
    };
    __shared__ TileLds lds_all[kFlatWaves];

    const int lane = threadIdx.x & 63;
    const int w = threadIdx.x >> 6;
    TileLds &L = lds_all[w];
    const uint64_t ntiles = (n + 63) / 64;
    const uint64_t nwaves = (uint64_t)gridDim.x * kFlatWaves;
    uint64_t tile = xcd_block(variant) * kFlatWaves + w;
    uint32_t nbad = 0;
    const uint64_t zero = (uint64_t)(uintptr_t)&kZeroChunk;

    // Unconditional metadata prefetch loads, as in k_cksum_flat.  No header
    // prefetch: the seg path reads payload_cksum's header bytes out of its
    // own stream, the grouped and flat paths load them when they run.
    auto meta = [&](uint64_t q, uint64_t &off, uint32_t &len) {
        if constexpr (STR) {
            off = (q < n ? q : 0) * stride;
            len = q < n ? slen : 0u;
        } else {
            meta_load(offs, lens, q, n, off, len);
        }
    };
    uint64_t p = tile * 64 + lane;
    uint64_t off_n;
    uint32_t len_n;
    meta(p, off_n, len_n);

    for (; tile < ntiles; tile += nwaves) {
        p = tile * 64 + lane;
        const bool valid = p < n;
        const uint32_t nvalid = (uint32_t)min<uint64_t>(64, n - tile * 64);
        const uint64_t off = off_n;
        const uint32_t len = len_n;
        const uint64_t pn = (tile + nwaves) * 64 + lane;
        meta(pn, off_n, len_n);

        const uint64_t a = (uint64_t)base + off;
        uint64_t A0 = 0;
        uint32_t T = 0;
        uint16_t r = 0;
        const bool dense = seg_dense(lane, a, len, valid, nvalid, A0, T);
        // Uniform tile?  Chunk fill of the grouped path's 1024 R slots.
        const uint32_t span = grp_span<KIND>(len);
        const uint32_t nchg = valid ? ((uint32_t)(a & 15u) + span + 15u) >> 4 : 0u;
        const uint32_t Rq = (wave_max(nchg) + 15u) >> 4;
        const uint32_t fill = lane_u32(wave_incl_sum(nchg), 63);
        const uint32_t thr = dense ? (uint32_t)(grp_thr & 0xFF) : (uint32_t)(grp_thr >> 8);
        const bool grouped = Rq != 0 && (uint64_t)fill * 64u >= (uint64_t)thr * 1024u * Rq;
        bool done = false;
        uint16_t rh = 0;
        if (grouped)
            r = grp_tile<UNG, KIND, NT, HDR>(L.grp, lane, a, len, valid, Rq, zero, done, rh);
        else if (dense)
            r = seg_tile<UNS, KIND, NT, HDR>(L.seg.pre, L.seg.stage, lane, a, len, valid, A0, T,
                                             zero, done, rh);
        if (!done) {
            PseudoHdr ph{0u, 1u, 0u};
            if constexpr (KIND == WC_KIND_PAYLOAD)
                if (valid)
                    ph = hdr_pseudo(load_hdr(a), a);
            wave_order();
            r = fold_not(flat_tile_sum<UN, KIND, NT, false, true>(L.flat, nullptr, lane, a, len,
                                                                  valid, ph, [] {}));
            if constexpr (HDR)
                rh = valid && ph.v4 ? lane_hdr_cksum<NT>(a, ph.hl, nullptr) : (uint16_t)0;
        }
        if constexpr (HDR)
            if (valid)
                out_hdr[p] = rh;
        if (valid && out)
            out[p] = r;
        nbad += valid && r != 0;
        wave_order(); // the tables are rewritten by the next tile
    }
    if (bad) {
        nbad = group_sum<64>(nbad);
        if (lane == 0 && nbad)
            atomicAdd(bad, (unsigned long long)nbad);
    }
}

// ---------------------------------------------------------------------------
// Synthetic bytes.

// splitmix64 output k for state `seed` (must match oracle_synth_fill).
__device__ __forceinline__ uint64_t splitmix64_at(uint64_t seed, uint64_t k)
{
    uint64_t z = seed + (k + 1ull) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__global__ void __launch_bounds__(256)
k_synth(uint8_t *__restrict__ buf, uint64_t nbytes, uint64_t seed)
{
    const uint64_t words = nbytes / 8;
    const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t nth = (uint64_t)gridDim.x * blockDim.x;
    // Two words (16 B) per thread per step; buf is 16-byte aligned by contract.
    for (uint64_t w = 2 * tid; w < words; w += 2 * nth) {
        if (w + 1 < words) {
            uint64_t v[2] = {splitmix64_at(seed, w), splitmix64_at(seed, w + 1)};
            *reinterpret_cast<u32x4 *>(buf + 8 * w) = *reinterpret_cast<const u32x4 *>(v);
        } else {
            *reinterpret_cast<uint64_t *>(buf + 8 * w) = splitmix64_at(seed, w);
        }
    }
    if (tid == 0 && (nbytes & 7u)) {
        const uint64_t v = splitmix64_at(seed, words);
        for (uint32_t b = 0; b < (nbytes & 7u); ++b)
            buf[8 * words + b] = (uint8_t)(v >> (8 * b));
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

template <int UN>
static hipError_t launch_flat_un(const LaunchArgs &a, hipStream_t st)
{
    const uint64_t tiles = (a.n + 63) / 64;
    const uint64_t tpw = (uint64_t)(a.tiles_per_wave > 0 ? a.tiles_per_wave : 1);
    const uint64_t waves = (tiles + tpw - 1) / tpw;
    const int grid = (int)std::max<uint64_t>(1, (waves + kFlatWaves - 1) / kFlatWaves);
    const uint8_t *b = (const uint8_t *)a.base;
    unsigned long long *bad = (unsigned long long *)a.bad;
#define WC_FLAT(K, N, H)                                                       \
    hipLaunchKernelGGL((k_cksum_flat<UN, K, N, H>), dim3(grid), dim3(256), 0,  \
                       st, b, a.offs, a.lens, a.n, a.out, bad, a.out_hdr)
    if (a.diag_noload && a.kind == WC_KIND_IP) {
        hipLaunchKernelGGL((k_cksum_flat<UN, WC_KIND_IP, true, false, true>), dim3(grid),
                           dim3(256), 0, st, b, a.offs, a.lens, a.n, a.out, bad, a.out_hdr);
        return hipGetLastError();
    }
    if (a.seg_rows && a.out_hdr && a.kind == WC_KIND_PAYLOAD && a.offs) {
        // fused IPv4 header + payload_cksum pass, default row-group sizes
        hipLaunchKernelGGL((k_cksum_seg<UN, 4, 4, WC_KIND_PAYLOAD, true, false, true>),
                           dim3(grid), dim3(256), 0, st, b, a.offs, a.lens, a.n, a.out, bad,
                           a.grp_thr, a.variant, a.stride, a.len, a.out_hdr);
        return hipGetLastError();
    }
    if (a.seg_rows && !a.out_hdr) {
#define WC_SEG_K(K, S)                                                         \
    hipLaunchKernelGGL((k_cksum_seg<UN, US, UG, K, true, S>), dim3(grid), dim3(256), 0, st, \
                       b, a.offs, a.lens, a.n, a.out, bad, a.grp_thr, a.variant, a.stride, \
                       a.len, nullptr)
#define WC_SEG(US_, UG_)                                                       \
    {                                                                          \
        constexpr int US = US_, UG = UG_;                                      \
        const bool str = a.offs == nullptr;                                    \
        if (a.kind == WC_KIND_PAYLOAD) {                                       \
            if (str)                                                           \
                WC_SEG_K(WC_KIND_PAYLOAD, true);                               \
            else                                                               \
                WC_SEG_K(WC_KIND_PAYLOAD, false);                              \
        } else {                                                               \
            if (str)                                                           \
                WC_SEG_K(WC_KIND_IP, true);                                    \
            else                                                               \
                WC_SEG_K(WC_KIND_IP, false);                                   \
        }                                                                      \
    }
        // Row-group sizes: seg path a.seg_rows (WC_SEG_ROWS), grouped path
        // a.grp_rows (WC_GRP_ROWS 4 or 2, with the default flat and seg
        // sizes only; 6 and 8 measured no faster on netmap slots).
        if (a.seg_rows == 2) {
            WC_SEG(2, 4)
        } else if (a.seg_rows == 8) {
            WC_SEG(8, 4)
        } else if (UN != 2 || a.grp_rows == 4) {
            WC_SEG(4, 4)
        } else {
            WC_SEG(4, 2)
        }
#undef WC_SEG
#undef WC_SEG_K
        return hipGetLastError();
    }
    if (a.kind == WC_KIND_PAYLOAD && a.out_hdr) {
        if (a.nontemporal)
            WC_FLAT(WC_KIND_PAYLOAD, true, true);
        else
            WC_FLAT(WC_KIND_PAYLOAD, false, true);
    } else if (a.kind == WC_KIND_PAYLOAD) {
        if (a.nontemporal)
            WC_FLAT(WC_KIND_PAYLOAD, true, false);
        else
            WC_FLAT(WC_KIND_PAYLOAD, false, false);
    } else {
        if (a.nontemporal)
            WC_FLAT(WC_KIND_IP, true, false);
        else
            WC_FLAT(WC_KIND_IP, false, false);
    }
#undef WC_FLAT
    return hipGetLastError();
}

hipError_t launch_flat(const LaunchArgs &a, int rows, hipStream_t st)
{
    switch (rows) {
    case 1:
        return launch_flat_un<1>(a, st);
    case 2:
        return launch_flat_un<2>(a, st);
    case 4:
        return launch_flat_un<4>(a, st);
    default:
        return hipErrorInvalidValue;
    }
}

hipError_t launch_synth(void *buf, uint64_t nbytes, uint64_t seed, int grid, hipStream_t st)
{
    hipLaunchKernelGGL(k_synth, dim3(grid), dim3(256), 0, st, (uint8_t *)buf, nbytes, seed);
    return hipGetLastError();
}

} // namespace wc
