// wc_k_rx.hip -- the RX verdict kernel on gfx950: for every frame of a netmap
// RX ring (or any batch of Ethernet frames), the checksum and header-format
// decision the reference's RX path makes, computed on the device from the
// frame bytes alone.
//
// Reference decisions restated (read, not copied):
//   eth_rx  /root/reference/lib/src/eth.c:75-86     EtherType dispatch
//   ip4_rx  /root/reference/lib/src/ip4.c:95-138    version, ip_cksum(ip, hl),
//                                                   fragment offset, protocol
//   ip6_rx  /root/reference/lib/src/ip6.c:91-111    version, next header
//   udp_rx  /root/reference/lib/src/udp.c:99-139    ip_plen, MIN(udp->len,
//           ip_plen), the zero-checksum skip and payload_cksum(ip, udp_len + hl)
// The codes are enum wc_rx_verdict (include/warpcore_gpu/wc_cksum.h); the CPU
// restatement is oracle_rx_verdict (oracle/wc_oracle.c).  Engine state (MAC
// and address filters, bound sockets) stays with the caller.
//
// One wave per tile of 64 frames (lane l = frame l), one-shot grid:
//   1. header fields: two aligned chunks around frame bytes 12..23 (EtherType,
//      version / IHL, lengths, fragment offset, protocol / next header);
//   2. with the IHL known: the UDP length and checksum fields, and for IPv4
//      the header's chunks -- its checksum is summed by the lane itself;
//   3. the frames whose UDP checksum must be verified go through the gathered
//      stream of the seg path (wc_seg.h, seg_tile over the tile's IP packets
//      [ip, ip + udp_len + hl) in packet order), the payload_cksum lanes it
//      can't take redone exactly by their own lane.
// Every load stays inside its frame (chunks that overlap [frame, frame +
// flen) only); whatever the reference would read past the frame is
// WC_RX_TRUNCATED.  Roofline: HBM, the checked frames' bytes once.
#include "wc_seg.h"

#ifdef WC_DIAG_STAMPS
// Timing diagnostic build only (tools/rx_stamps.py): per tile, lane 0 stores
// the 100-MHz wall clock (s_memrealtime, which hipcc keeps in program order
// with the loads and stores around it) at phase boundaries, the wave's
// hardware ids and the tile's stream length.
constexpr uint64_t kStampTiles = 1u << 16;
__device__ uint32_t g_rx_stamps[kStampTiles * 8];
#define WC_STAMP(k, v)                                                         \
    do {                                                                       \
        if (lane == 0 && tile < kStampTiles)                                   \
            g_rx_stamps[tile * 8 + (k)] = (v);                                 \
    } while (0)
#define WC_CLOCK() ((uint32_t)wall_clock64())
#else
#define WC_STAMP(k, v) ((void)0)
#define WC_CLOCK() 0u
#endif

namespace wc {
namespace {

// enum wc_rx_verdict (wc_cksum.h)
constexpr uint32_t kRxOk = 0, kRxOkNoCksum = 1, kRxBadIpCksum = 2, kRxBadUdpCksum = 3,
                   kRxShort = 4, kRxFragment = 5, kRxBadVersion = 6, kRxNotUdp = 7,
                   kRxNotIp = 8, kRxTruncated = 9;

__device__ __forceinline__ bool rx_is_drop(uint32_t v)
{
    return v != kRxOk && v != kRxOkNoCksum && v != kRxNotUdp && v != kRxNotIp;
}

struct RxParse {
    uint64_t ip;      // the frame's IP header (frame + 14)
    uint32_t plen;    // payload_cksum length udp_len + hl (need)
    uint32_t verdict; // final unless need
    bool need;        // the UDP checksum must be verified
};

// Two aligned chunks holding frame bytes from `at` on, each loaded only if it
// overlaps the frame (else the zero chunk): never a page the frame does not
// touch.
struct Win2 {
    u32x4 x, y;
};

__device__ __forceinline__ Win2 win2_load(uint64_t at, uint64_t fend, bool on, uint64_t zero)
{
    const uint64_t c = at & ~15ull;
    Win2 w;
    w.x = load_chunk<false>(on && c < fend ? c : zero);
    w.y = load_chunk<false>(on && c + 16u < fend ? c + 16u : zero);
    return w;
}

constexpr int kHdrChunks = 5; // an IPv4 header (<= 60 B) at any phase

// The header view shared by both parses: EtherType, version, IHL, lengths.
struct RxHdr {
    bool v4, v6, version_ok, hdr_in, frag, udp_in;
    uint32_t hl, room, proto, ip_plen;
};

__device__ __forceinline__ RxHdr rx_hdr(uint32_t f0, uint32_t f1, uint32_t f2, uint32_t flen)
{
    RxHdr x;
    const uint32_t etype = ((f0 & 0xFFu) << 8) | ((f0 >> 8) & 0xFFu); // eth.h:44-53
    const uint32_t b0 = (f0 >> 16) & 0xFFu;                              // vhl / vfc
    x.v4 = etype == 0x0800u;
    x.v6 = etype == 0x86DDu;
    x.room = flen >= 14u ? flen - 14u : 0u; // IP bytes inside the frame
    x.hl = x.v4 ? (b0 & 15u) * 4u : 40u;    // ip4.h:88-92, udp.c:113
    x.version_ok = (b0 >> 4) == (x.v4 ? 4u : 6u);
    // Header fields (ip4.h:55-66, ip6.h:45-57): valid once the header is in.
    x.hdr_in = (x.v4 || x.v6) && x.room >= 1u && x.version_ok &&
               x.room >= (x.v4 ? max(x.hl, 20u) : 40u);
    x.proto = x.v4 ? f2 >> 24 : f2 & 0xFFu; // p @9 / next_hdr @6
    // IP4_OFFMASK 0xff1f on the native word @6: the fragment offset (ip4.h:49)
    x.frag = x.v4 && (((f2 & 0x1Fu) | (f2 & 0xFF00u)) != 0u);
    x.ip_plen = x.v4 ? ((((f1 & 0xFFu) << 8) | ((f1 >> 8) & 0xFFu)) - x.hl) & 0xFFFFu // udp.c:104
                     : (((f1 >> 16) & 0xFFu) << 8) | (f1 >> 24);                     // udp.c:114
    x.udp_in = x.hdr_in && x.proto == 17u && x.ip_plen >= 8u && x.room >= x.hl + 8u;
    return x;
}

// The reference's decision chain (eth_rx -> ip4_rx / ip6_rx -> udp_rx); bytes
// past the frame only feed decisions that the length checks have made.
__device__ __forceinline__ RxParse rx_decide(uint64_t fa, uint32_t flen, bool valid,
                                             const RxHdr &x, uint32_t g0, uint16_t ipck)
{
    RxParse h{fa + 14u, 0u, kRxTruncated, false};
    const bool v4 = x.v4, v6 = x.v6, frag = x.frag;
    const uint32_t room = x.room, hl = x.hl, proto = x.proto, ip_plen = x.ip_plen;
    const uint32_t ulen = ((g0 & 0xFFu) << 8) | ((g0 >> 8) & 0xFFu);
    const bool ck_zero = (g0 >> 16) == 0u; // udp.c:132
    const uint32_t udp_len = min(ulen, ip_plen); // udp.c:128
    const uint32_t L = udp_len + hl;             // unwrapped; > 65535 is past any frame
    const bool version_ok = x.version_ok, hdr_in = x.hdr_in, udp_in = x.udp_in;
    uint32_t v;
    if (flen < 14u)
        v = kRxTruncated;
    else if (!v4 && !v6)
        v = kRxNotIp;
    else if (room < 1u)
        v = kRxTruncated;
    else if (!version_ok)
        v = kRxBadVersion;
    else if (!hdr_in)
        v = kRxTruncated;
    else if (v4 && ipck != 0)
        v = kRxBadIpCksum;
    else if (frag)
        v = kRxFragment;
    else if (proto != 17u)
        v = kRxNotUdp;
    else if (ip_plen < 8u)
        v = kRxShort;
    else if (!udp_in)
        v = kRxTruncated;
    else if (ck_zero)
        v = kRxOkNoCksum;
    else if (room < max(L, 20u))
        v = kRxTruncated;
    else {
        v = kRxOk;
        h.need = valid;
        h.plen = L;
    }
    h.verdict = v;
    return h;
}

// Steps 1 and 2 in ONE load round (rx_load, then rx_parse on what it
// loaded): the frame's first five aligned chunks
// (frame bytes [0, 65) at least, each chunk loaded only if it overlaps the
// frame) hold the Ethernet header, an IPv4 header of up to 40 bytes or the
// IPv6 header, and the UDP length / checksum fields after either.  A lane
// with a longer IPv4 header (options > 20 B) or a malformed IHL < 5 sets
// `slow` and is re-parsed by rx_parse_slow.  Two dependent load rounds per tile cost the mixed-size ring
// its headroom over payload_cksum alone.
__device__ __forceinline__ void rx_load(uint64_t fa, uint32_t flen, bool valid, uint64_t zero,
                                        u32x4 (&c)[5])
{
    const uint64_t fend = fa + flen;
    const uint64_t cf = fa & ~15ull;
#pragma unroll
    for (int k = 0; k < 5; ++k)
        c[k] = load_chunk<false>(valid && cf + 16ull * k < fend ? cf + 16ull * k : zero);
}

// The same five chunks, loaded transposed (HT): instruction i reads frames
// 16 i .. 16 i + 15, four lanes per frame, lane 4 f' + j its chunk j -- 64
// contiguous bytes per frame, one cache line instead of four separate
// 16-byte requests (five one-lane-per-frame loads put 320 line requests per
// tile in front of the stream's ~140).  Chunk 4 (frame bytes past 64 - sf)
// is loaded per lane, and only by lanes whose start phase sf > 2 may need it
// (the parse reads frame bytes < 14 + 40 + 8 = 62).  rx_hdr_gather then hands
// each lane its frame's chunks through LDS.
// Each lane finds its frame's address and length in a 1-KB LDS table the
// tile's lanes write first (one 16-byte store, four 16-byte reads, all
// issued back to back), not by twelve cross-lane shuffles, each a dependent
// LDS round trip before the next header load.  `tbl` is the tile's
// descriptor table, which flat_tile_setup rewrites afterwards.
__device__ __forceinline__ void rx_load_t(uint64_t fa, uint32_t flen, bool valid, uint64_t zero,
                                          int lane, u32x4 *tbl, u32x4 (&hx)[4], u32x4 &c4)
{
    const uint32_t lv = valid ? flen : 0u;
    tbl[lane] = u32x4{(uint32_t)fa, (uint32_t)(fa >> 32), lv, 0u};
    wave_order();
    u32x4 e[4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
        e[i] = tbl[16 * i + (lane >> 2)]; // frame 16 i + lane / 4
    wave_order(); // (the table is rewritten by flat_tile_setup)
    const uint64_t j16 = 16ull * (uint32_t)(lane & 3);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const uint64_t faf = (uint64_t)e[i].x | ((uint64_t)e[i].y << 32);
        const uint32_t lf = e[i].z;
        const uint64_t a = (faf & ~15ull) + j16;
        hx[i] = load_chunk<false>(lf != 0u && a < faf + lf ? a : zero);
    }
    const uint64_t a4 = (fa & ~15ull) + 64u;
    c4 = load_chunk<false>(lv != 0u && (fa & 15u) > 2u && a4 < fa + lv ? a4 : zero);
}

// The hand-off is XOR-swizzled: chunk j of frame f sits in slot
// 4 f + (j ^ ((f >> 2) & 3)).  Unswizzled (slot 4 f + j), the read of chunk k
// by lane f -- 16 B at a 64-B lane stride -- put the four lanes f, f + 4,
// f + 8, f + 12 of a ds_read_b128 lane group on the same banks (bank =
// (address / 4) mod 64): a 4-way conflict on every read, 2.85 M conflict
// cycles on the mixed-size ring against 1.28 M for the plain stream
// (profiles/pmc_r05_rx_instr.txt).  Swizzled, each 16-lane group reads 16
// distinct 16-B bank slots (its lanes are 16 distinct residues mod 16), and
// the stores stay conflict-free (each 8-lane ds_write_b128 group still
// covers 8 consecutive slots, permuted).
__device__ __forceinline__ void rx_hdr_gather(u32x4 *stage, int lane, const u32x4 (&hx)[4],
                                              const u32x4 &c4, u32x4 (&c)[5])
{
    const int ws = lane ^ ((lane >> 4) & 3); // frame 16 i + lane / 4, chunk lane % 4
#pragma unroll
    for (int i = 0; i < 4; ++i)
        stage[64 * i + ws] = hx[i];
    wave_order();
    const int rs = (lane >> 2) & 3;
#pragma unroll
    for (int k = 0; k < 4; ++k)
        c[k] = stage[4 * lane + (k ^ rs)];
    c[4] = c4;
    wave_order(); // stage is rewritten by the stream's first row group
}

__device__ __forceinline__ RxParse rx_parse(const u32x4 (&c)[5], uint64_t fa, uint32_t flen,
                                            bool valid, bool &slow)
{
    const uint32_t sf = (uint32_t)(fa & 15u);
    // frame bytes 12..23 start in chunk 0 or 1
    const uint32_t o1 = sf + 12u;
    const bool j1 = o1 >= 16u;
    const u32x4 x1 = j1 ? c[1] : c[0], y1 = j1 ? c[2] : c[1];
    uint32_t fw[3];
    win_rot(x1, y1, y1, o1 & 15u, fw);
    const RxHdr x = rx_hdr(fw[0], fw[1], fw[2], flen);
    slow = valid && x.hdr_in && x.v4 && (x.hl > 40u || x.hl < 20u);
    // UDP length / checksum at frame byte 14 + hl + 4: chunk 2, 3 or 4 (20 <= hl <= 40)
    const uint32_t u = sf + 18u + x.hl;
    const uint32_t ju = min(u >> 4, 4u);
    const u32x4 z4 = {0u, 0u, 0u, 0u};
    const u32x4 xu = ju <= 2u ? c[2] : (ju == 3u ? c[3] : c[4]);
    const u32x4 yu = ju <= 2u ? c[3] : (ju == 3u ? c[4] : z4);
    const uint32_t g0 = win_bytes(xu, yu, yu, u & 15u, 0);
    // ip_cksum(ip, hl) (ip4.c:110-115) over frame bytes [14, 14 + hl),
    // 20 <= hl <= 40 here (14 + 40 + 15 < 80: inside the five chunks): the
    // header's little-endian words summed header-relative, as csum_oc16 reads
    // them (in_cksum.c:107-120) -- two 20-byte windows rotated out of the
    // chunks, one dot2 per dword, so no address-parity fix.  (Per-chunk byte
    // masks over all five chunks took about twice the VALU.)
    const uint32_t o = sf + 14u;  // header start in the chunk stream: 14..29
    const uint32_t o2 = o + 20u;  // its second 20 bytes: 34..49
    const bool j0 = o >= 16u, j2 = o2 >= 48u;
    uint32_t h0[5], h1[5];
    win_rot(j0 ? c[1] : c[0], j0 ? c[2] : c[1], j0 ? c[3] : c[2], o & 15u, h0);
    win_rot(j2 ? c[3] : c[2], j2 ? c[4] : c[3], j2 ? z4 : c[4], o2 & 15u, h1);
    uint32_t V = 0;
#pragma unroll
    for (int m = 0; m < 5; ++m)
        V = wsum(h0[m], V);
#pragma unroll
    for (int m = 0; m < 5; ++m) // header bytes 20 + 4 m .. 23 + 4 m, if below hl
        V = wsum(x.hl > 20u + 4u * m ? h1[m] : 0u, V);
    const uint16_t ipck = fold_not(V);
    return rx_decide(fa, flen, valid, x, g0, ipck);
}

// Steps 1 and 2 in two load rounds for this lane's frame [fa, fa + flen): the
// chunks around frame bytes 12..23 first, then, with the IHL known, the UDP
// fields and the IPv4 header's chunks (any IHL).  The fallback of rx_parse.
__device__ __forceinline__ RxParse rx_parse_slow(uint64_t fa, uint32_t flen, bool valid,
                                                 uint64_t zero)
{
    const uint64_t fend = fa + flen;
    const uint64_t a1 = fa + 12u;
    const Win2 w1 = win2_load(a1, fend, valid && flen > 12u, zero);
    const uint32_t s1 = (uint32_t)(a1 & 15u);
    uint32_t fw[3]; // frame 12..15, 16..19 = ip 2..5, 20..23 = ip 6..9
    win_rot(w1.x, w1.y, w1.y, s1, fw);
    const RxHdr x = rx_hdr(fw[0], fw[1], fw[2], flen);
    const uint64_t ip = fa + 14u;
    const uint32_t hl = x.hl;
    // The UDP length / checksum fields (udp.h:41-46) at ip + hl + 4, and the
    // IPv4 header's chunks, all issued before any is used.
    const uint64_t a2 = ip + hl + 4u;
    const Win2 w2 = win2_load(a2, fend, valid && x.udp_in, zero);
    const bool hsum = valid && x.hdr_in && x.v4;
    const uint32_t sip = (uint32_t)(ip & 15u);
    const uint64_t cip = ip & ~15ull;
    const uint32_t nh = hsum ? (sip + hl + 15u) >> 4 : 0u;
    u32x4 hc[kHdrChunks];
#pragma unroll
    for (int k = 0; k < kHdrChunks; ++k)
        hc[k] = load_chunk<false>((uint32_t)k < nh ? cip + 16ull * k : zero);
    // ip_cksum(ip, hl) (ip4.c:110-115): word sum at even addresses; an odd
    // start folds rotl32(V, 8) (the seg path's residue identity; <= 30 words,
    // no wrap).
    uint32_t V = 0;
#pragma unroll
    for (int k = 0; k < kHdrChunks; ++k)
        V += seg_range(hc[k], 16 * k - (int)sip, 0, (int)hl);
    const uint16_t ipck = fold_not((ip & 1u) ? __builtin_amdgcn_alignbit(V, V, 24) : V);
    const uint32_t g0 = win_bytes(w2.x, w2.y, w2.y, (uint32_t)(a2 & 15u), 0);
    return rx_decide(fa, flen, valid, x, g0, ipck);
}


// One 64-chunk row group of 4 rows for the gathered stream (the seg
// kernel's ragged default; 2-row groups measured slower, 128 -> 131 us on the
// mixed ring: profiles/ab_r04_rx_modes.log).  Kernel modes (launch_rx_verdict),
// all giving the same verdicts:
//   EARLY  the header parse completes BEFORE the stream, which then carries
//          only the frames that need the UDP check and only their checked
//          range [ip, ip + udp_len + hl) -- one load round trip per tile
//          more; otherwise every frame with >= 28 IP bytes starts streaming
//          while the parse is in flight;
//   HT     the header chunks are loaded transposed (rx_load_t);
//   SKIP   (with !EARLY) once parsed, frames that need no check leave the
//          stream: its later row groups read the zero chunk for them.
//   TALLY  (with the default ADAPT mode, wc_cksum_api.cpp rx_launch) every
//          64th tile writes how many of its frames needed no UDP check (not
//          IP, not UDP, zero checksum, drops) and how many it held, one word
//          per tile `tally[tile / 64] = gen << 16 | ruled_out << 8 | frames`,
//          with a plain store into mapped host memory; the host picks EARLY
//          or HT for the device's next launch from the newest complete
//          tally.  No load and no atomic in the kernel: a first version kept
//          one device counter per launch that every tile read and every 8th
//          tile added to, and the same-address atomics serialised the mixed
//          ring from 113 to 458 us (profiles/ab_r05_rx_adapt.log).
// (4 waves per SIMD for every mode: capping the EARLY kernels at 96 VGPRs
// for 5 spilled 4 of them and took the mixed ring from 114 to 141 us,
// profiles/ab_r04_rx_early_waves.log.)
// One-wave workgroups: a wave's slot is handed to the next tile as soon as
// its own tile is done, not when the slowest of four is (mixed-size ring with
// ARP frames 91.8 -> 89.1 us, the others unchanged: profiles/ab_r06m_rx_waves.log).
constexpr int kRxWaves = 1;
constexpr int kRxSpan = 15; // XCD super-blocks of 2^15 tiles, as the seg kernel's

template <bool NT, bool EARLY, bool HT, bool SKIP, bool TALLY = false>
__global__ void __launch_bounds__(64 * kRxWaves) __attribute__((amdgpu_waves_per_eu(4)))
k_rx_verdict(const uint8_t *__restrict__ base, const uint64_t *__restrict__ offs,
             const uint16_t *__restrict__ flens, uint64_t n, uint8_t *__restrict__ verdict,
             unsigned long long *__restrict__ drops, uint32_t *__restrict__ tally, uint32_t gen)
{
    constexpr int UNS = 4;
    using Src = GathSrc<UNS, NT, SKIP && !EARLY>;
    struct Lds {
        FlatLds<UNS> f; // slot table, row marks, prefix sums
        u32x4 stage[64 * UNS]; // also the header chunks' transpose (HT)
        u32x4 pm[17]; // seg_head's masks
    };
    __shared__ Lds lds_all[kRxWaves];

    const int lane = threadIdx.x & 63;
    const int w = kRxWaves == 1 ? 0 : __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    Lds &L = lds_all[w];
    seg_init_masks(L.pm, lane); // read after the first row group's wave_order
    const uint64_t ntiles = (n + 63) / 64;
    const uint64_t nwaves = (uint64_t)gridDim.x * kRxWaves;
    uint64_t tile = xcd_block(kRxSpan << 8) * kRxWaves + w; // the seg kernel's XCD span
    uint32_t ndrop = 0;
    const uint64_t zero = (uint64_t)(uintptr_t)&kZeroChunk;

    uint64_t off_n;
    uint32_t flen_n;
    meta_load(offs, flens, tile * 64 + lane, n, off_n, flen_n);

    for (; tile < ntiles; tile += nwaves) {
        WC_STAMP(0, WC_CLOCK());
        const uint64_t p = tile * 64 + lane;
        const bool valid = p < n;
        const uint64_t fa = (uint64_t)base + off_n;
        const uint32_t flen = flen_n;
        meta_load(offs, flens, (tile + nwaves) * 64 + lane, n, off_n, flen_n);

        u32x4 c[5];
        u32x4 hx[4], c4;
        if constexpr (HT)
            rx_load_t(fa, flen, valid, zero, lane, reinterpret_cast<u32x4 *>(L.f.desc), hx, c4);
        else
            rx_load(fa, flen, valid, zero, c);
        WC_STAMP(1, WC_CLOCK());
#ifdef WC_DIAG_STAMPS
        if (lane == 0 && tile < kStampTiles) {
            g_rx_stamps[tile * 8 + 6] = __builtin_amdgcn_s_getreg(4 | (31 << 11));  // HW_ID
            g_rx_stamps[tile * 8 + 7] = __builtin_amdgcn_s_getreg(20 | (15 << 11)); // XCC_ID
        }
#endif
        auto headers = [&] { // this lane's frame chunks 0..4 (HT: through LDS)
            if constexpr (HT)
                rx_hdr_gather(L.stage, lane, hx, c4, c);
        };
        const uint64_t ip = fa + 14u;
        bool slow = false;
        RxParse h{};
        uint32_t v;
        if constexpr (EARLY) {
            headers();
            h = rx_parse(c, fa, flen, valid, slow);
            v = h.verdict;
            const bool need = h.need && !slow;
            if (__ballot(need)) {
                const FlatTile t = flat_tile_setup<UNS, 1>(L.f, lane, ip, h.plen, h.plen, need, 0u);
                bool done = true;
                uint16_t rh = 0;
                uint16_t r = seg_tile<UNS, WC_KIND_PAYLOAD, NT, false, Src, true>(
                    L.f.pre, L.stage, L.pm, lane, ip, 16ull * t.cp + (ip & 15u), h.plen, need,
                    t.total, Src{&L.f, t}, zero, done, rh);
                if (need && !done) // header longer than the packet, or a possible wrap
                    r = lane_payload_exact<NT>(ip, h.plen);
                if (need)
                    v = r != 0 ? kRxBadUdpCksum : kRxOk; // udp.c:134-139
                wave_order(); // the tables are rewritten by the next tile
            }
        } else {
            // Header chunks first; then every frame that may need the UDP
            // check (>= 28 IP bytes) streams its IP bytes [ip, ip + room) as
            // the seg path's gathered stream, and the parse completes once
            // that stream's first row group is in flight (seg_tile's Late
            // hook): the checked range [ip, ip + udp_len + hl) is a prefix of
            // the streamed one.  A frame that turns out not to need the check
            // was read for the first row group only (SKIP).
            const uint32_t room = flen >= 14u ? flen - 14u : 0u;
            const bool spec = valid && room >= 28u;
            if (__ballot(spec)) {
                const FlatTile t = flat_tile_setup<UNS, 1>(L.f, lane, ip, room, room, spec, 0u);
                bool need = false;
                auto late = [&](uint32_t &len, bool &on) {
                    headers();
                    h = rx_parse(c, fa, flen, valid, slow);
                    need = h.need && !slow;
                    on = need;
                    len = need ? h.plen : 0u;
                    WC_STAMP(2, WC_CLOCK());
                    if constexpr (SKIP) {
                        if (spec && !need) // its later chunks: the zero chunk
                            L.f.desc[t.rank].info = 1u << 31;
                        wave_order();
                    }
                };
                bool done = true;
                uint16_t rh = 0;
                uint16_t r = seg_tile<UNS, WC_KIND_PAYLOAD, NT, false, Src, true, decltype(late)>(
                    L.f.pre, L.stage, L.pm, lane, ip, 16ull * t.cp + (ip & 15u), room, spec,
                    t.total, Src{&L.f, t}, zero, done, rh, late);
                WC_STAMP(3, WC_CLOCK());
                WC_STAMP(5, t.total);
                if (need && !done) // header longer than the packet, or a possible wrap
                    r = lane_payload_exact<NT>(ip, h.plen);
                v = h.verdict;
                if (need)
                    v = r != 0 ? kRxBadUdpCksum : kRxOk; // udp.c:134-139
                wave_order(); // the tables are rewritten by the next tile
            } else {
                headers();
                h = rx_parse(c, fa, flen, valid, slow);
                v = h.verdict;
            }
        }
        if constexpr (TALLY) {
            if ((tile & 63u) == 0 && (tile >> 6) < kRxTallyWords) { // a sample of the mix
                const uint32_t nv = __builtin_popcountll(__ballot(valid));
                const uint32_t nout = __builtin_popcountll(__ballot(valid && !h.need));
                if (lane == 0)
                    __hip_atomic_store(&tally[tile >> 6], (gen << 16) | (nout << 8) | nv,
                                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            }
        }
        if (__ballot(slow)) { // IPv4 headers with more than 20 B of options, IHL < 5
            const RxParse hs = rx_parse_slow(fa, flen, slow, zero);
            if (slow) {
                v = hs.verdict;
                if (hs.need)
                    v = lane_payload_exact<NT>(hs.ip, hs.plen) != 0 ? kRxBadUdpCksum : kRxOk;
            }
        }
        if (valid)
            verdict[p] = (uint8_t)v;
        ndrop += valid && rx_is_drop(v);
        WC_STAMP(4, WC_CLOCK());
    }
    if (drops) {
        ndrop = group_sum<64>(ndrop);
        if (lane == 0 && ndrop)
            atomicAdd(drops, (unsigned long long)ndrop);
    }
}

} // namespace

template <bool NT, bool EARLY, bool HT, bool SKIP, bool TALLY = false>
static hipError_t launch_rx_one(const void *base, const uint64_t *offs, const uint16_t *flens,
                                uint64_t n, uint8_t *verdict, uint64_t *drops, int grid,
                                hipStream_t st, uint32_t *tally, uint32_t gen)
{
    hipLaunchKernelGGL((k_rx_verdict<NT, EARLY, HT, SKIP, TALLY>), dim3(grid), dim3(64 * kRxWaves), 0, st,
                       (const uint8_t *)base, offs, flens, n, verdict,
                       (unsigned long long *)drops, tally, gen);
    return hipGetLastError();
}

hipError_t launch_rx_verdict(const void *base, const uint64_t *offs, const uint16_t *flens,
                             uint64_t n, uint8_t *verdict, uint64_t *drops, bool nt,
                             hipStream_t st, int mode, uint32_t *tally, uint32_t gen,
                             int max_grid)
{
    const uint64_t tiles = (n + 63) / 64;
    // One tile per wave (one-shot); max_grid > 0 (WC_RX_GRID, tools) caps the
    // grid, each wave then walks several tiles with the next tile's metadata
    // prefetched.
    const uint64_t cap = max_grid > 0 ? (uint64_t)max_grid : kMaxGridBlocks;
    const int grid = (int)std::min<uint64_t>(
        cap, std::max<uint64_t>(1, (tiles + kRxWaves - 1) / kRxWaves));
    // EARLY streams only the checked frames: SKIP has nothing to skip there,
    // and is dropped so that NT and HDRT are still honoured.
    const bool early = mode & kRxEarly, ht = mode & kRxHdrT, skip = (mode & kRxSkip) && !early;
    if (tally && !skip && ht) { // ADAPT: the host chose EARLY or HT; the kernel tallies
        if (nt)
            return early ? launch_rx_one<true, true, true, false, true>(base, offs, flens, n,
                                                                        verdict, drops, grid,
                                                                        st, tally, gen)
                         : launch_rx_one<true, false, true, false, true>(base, offs, flens, n,
                                                                         verdict, drops, grid,
                                                                         st, tally, gen);
        return early ? launch_rx_one<false, true, true, false, true>(base, offs, flens, n, verdict,
                                                                     drops, grid, st, tally, gen)
                     : launch_rx_one<false, false, true, false, true>(base, offs, flens, n,
                                                                      verdict, drops, grid, st,
                                                                      tally, gen);
    }
#define WC_RX(N, E, H, S)                                                      \
    if (nt == N && early == E && ht == H && skip == S)                         \
        return launch_rx_one<N, E, H, S>(base, offs, flens, n, verdict, drops, grid, st,   \
                                         nullptr, 0u);
#define WC_RX_NT(N)                                                            \
    WC_RX(N, false, false, false) WC_RX(N, false, false, true)                 \
    WC_RX(N, false, true, false) WC_RX(N, false, true, true)                   \
    WC_RX(N, true, false, false) WC_RX(N, true, true, false)
    WC_RX_NT(true)
    WC_RX_NT(false)
#undef WC_RX_NT
#undef WC_RX
    return hipErrorInvalidValue; // (every combination is listed above)
}

} // namespace wc

#ifdef WC_DIAG_STAMPS
extern "C" int wc_diag_rx_stamps(uint32_t *host, uint64_t words)
{
    if (words > kStampTiles * 8)
        words = kStampTiles * 8;
    return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_rx_stamps), words * 4, 0,
                                    hipMemcpyDeviceToHost);
}
#endif
