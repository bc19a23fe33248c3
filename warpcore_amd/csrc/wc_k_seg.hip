// wc_k_seg.hip -- ragged (and packed strided) batches on gfx950: the
// segmented-prefix tile kernel k_cksum_seg with its grouped, gathered and
// flat tile paths, and the ragged launch entry point.
#include "wc_seg.h"

namespace wc {


// Ragged kernel with both paths: dense tiles stream their byte range
// (seg_tile), the others take the flat path.  (The fused header checksum
// stays on k_cksum_flat.)  STR: a strided batch (packet i at i * stride,
// slen bytes) -- packed packets at any alignment are one dense byte range,
// which the seg path streams better than the group kernel masks its
// boundary chunks; offsets and lengths are computed, not loaded.
template <int UN, int UNS, int UNG, int KIND, bool NT, bool STR, bool HDR = false>
#ifndef WC_SEG_WAVES
#define WC_SEG_WAVES 4 // waves per SIMD the 2/4-row variants are register-capped for
#endif
#ifndef WC_SEG_STR_WAVES
#define WC_SEG_STR_WAVES 4 // the same for packed strided ip_cksum (seg path only)
#endif
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(
    UNS >= 8 ? 2 : (STR && !HDR ? WC_SEG_STR_WAVES : WC_SEG_WAVES))))
k_cksum_seg(const uint8_t *__restrict__ base, const uint64_t *__restrict__ offs,
            const uint16_t *__restrict__ lens, uint64_t n, uint16_t *__restrict__ out,
            unsigned long long *__restrict__ bad, int grp_thr, int variant_arg, uint64_t stride,
            uint32_t slen, uint16_t *__restrict__ out_hdr, int gather)
{
    const int variant = tuning_variant(variant_arg); // 0 outside the tuning build
    static_assert(!HDR || KIND == WC_KIND_PAYLOAD, "header checksum rides on payload");
    // Packed strided batches: every tile is dense and the seg path always
    // completes (a payload_cksum lane it can't take is recomputed by its own
    // lane), so the other paths (and their registers and LDS) are not
    // compiled in.
    constexpr bool kSegOnly = STR && !HDR;
    struct SegLds {
        u32x4 stage[64 * UNS]; // the row group's chunks
        uint32_t pre[64 * UNS];
    };
    union FullLds {
        FlatLds<UN> flat;
        GrpLds grp;
        SegLds seg;
        struct {
            FlatLds<UNS> f; // slot table, row marks, prefix sums
            u32x4 stage[64 * UNS];
        } gat;
    };
    struct SegOnlyLds {
        SegLds seg;
    };
    using TileLds = typename std::conditional<kSegOnly, SegOnlyLds, FullLds>::type;
    __shared__ TileLds lds_all[kFlatWaves];
    __shared__ u32x4 head_masks[kFlatWaves][17]; // seg_head's tables, one per wave

    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); // wave-uniform: SGPR
    TileLds &L = lds_all[w];
    const u32x4 *pm = head_masks[w];
    seg_init_masks(head_masks[w], lane); // read after the first row group's wave_order
    const uint64_t ntiles = (n + 63) / 64;
    const uint64_t nwaves = (uint64_t)gridDim.x * kFlatWaves;
    // XCD super-blocks of 2^13 workgroups (32768 tiles) unless WC_VARIANT
    // sets the span: +0.5-1 point on C4, the mixed ring and packed 300 B over
    // the strided kernel's 2^12 (profiles/ab_r02_xcd_span.log).
    const int xv = (variant & 0xFF00) ? variant : (variant | (13 << 8));
    uint64_t tile = xcd_block(xv) * kFlatWaves + w;
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
        bool dense;
        if constexpr (STR) {
            // Packed strided batch (the planner's precondition: len > 0,
            // len <= stride <= len + len / 8, < 90 chunks): every tile is
            // dense, and its range follows from the stride -- no wave
            // reductions before the first load.
            dense = true;
            const uint64_t a0 = (uint64_t)base + tile * 64u * stride;
            A0 = a0 & ~15ull;
            T = (uint32_t)((a0 + (uint64_t)(nvalid - 1u) * stride + slen - A0 + 15u) >> 4);
        } else {
            dense = seg_dense(lane, a, len, valid, nvalid, A0, T);
        }
        if (!STR && gather == 2) // WC_GATHER=2 (tests): every non-uniform tile gathered
            dense = false;
        // Uniform tile?  Chunk fill of the grouped path's 1024 R slots --
        // only computed when the threshold for this kind of tile can be met
        // (dense tiles never take the grouped path by default).
        const uint32_t thr = dense ? (uint32_t)(grp_thr & 0xFF) : (uint32_t)(grp_thr >> 8);
        uint32_t Rq = 0;
        bool grouped = false;
        // The fused header variant (HDR) leaves the grouped path out: with it
        // and the gathered path it spilled; the gathered path takes its
        // uniform tiles (mixed-size ring fused 43 -> 56 %, ragged 1500-B ring
        // 80.5 -> 79.7 %: profiles/ab_r02_hdr_gather2.log).
        if (!kSegOnly && !HDR && thr <= 64u) {
            const uint32_t span = grp_span<KIND>(len);
            const uint32_t nchg = valid ? ((uint32_t)(a & 15u) + span + 15u) >> 4 : 0u;
            Rq = (wave_max(nchg) + 15u) >> 4;
            const uint32_t fill = lane_u32(wave_incl_sum(nchg), 63);
            grouped = Rq != 0 && (uint64_t)fill * 64u >= (uint64_t)thr * 1024u * Rq;
        }
        bool done = false;
        uint16_t rh = 0;
        if constexpr (kSegOnly) {
            r = seg_tile<UNS, KIND, NT, HDR, DenseSrc<UNS, NT>, true>(
                L.seg.pre, L.seg.stage, pm, lane, a, a - A0, len, valid, T,
                DenseSrc<UNS, NT>{A0, T, zero}, zero, done, rh);
            if constexpr (KIND == WC_KIND_PAYLOAD)
                if (!done)
                    r = lane_payload_exact<NT>(a, len);
        }
        else if (!HDR && grouped)
            r = grp_tile<UNG, KIND, NT, HDR>(L.grp, lane, a, len, valid, Rq, zero, done, rh);
        else if (dense)
            r = seg_tile<UNS, KIND, NT, HDR>(L.seg.pre, L.seg.stage, pm, lane, a, a - A0, len, valid,
                                             T, DenseSrc<UNS, NT>{A0, T, zero}, zero, done, rh);
        else if (!STR && gather) {
            // Gathered stream: the tile's packets' chunks in packet order
            // (sparse or unordered tiles -- a netmap ring of mixed sizes).
            const uint32_t span = KIND == WC_KIND_PAYLOAD ? max(len, 20u) : len;
            const FlatTile t = flat_tile_setup<UNS, 1>(L.gat.f, lane, a, len, span, valid, 0u);
            if (t.total != 0)
                r = seg_tile<UNS, KIND, NT, HDR>(L.gat.f.pre, L.gat.stage, pm, lane, a,
                                                 16ull * t.cp + (a & 15u), len, valid, t.total,
                                                 GathSrc<UNS, NT>{&L.gat.f, t}, zero, done, rh);
            wave_order(); // the flat path below rewrites the tables
        }
        if constexpr (!kSegOnly) if (!done) {
            PseudoHdr ph{0u, 1u, 0u};
            HdrRaw hdr{};
            if constexpr (KIND == WC_KIND_PAYLOAD) {
                hdr = load_hdr(a);
                if (valid)
                    ph = hdr_pseudo(hdr, a);
            }
            wave_order();
            auto noop = [] {};
            if constexpr (KIND == WC_KIND_PAYLOAD)
                r = fold_not(flat_tile_sum_payload<UN, NT, true>(L.flat, nullptr, lane, a, len,
                                                                 valid, ph, hdr, noop));
            else // ip_cksum: word sums (VSUM), +0.5 point on the mixed-size ring
                r = fold_not(flat_tile_sum<UN, KIND, NT, false, true, decltype(noop) &, 1,
                                           KIND == WC_KIND_IP>(L.flat, nullptr, lane, a, len,
                                                               valid, ph, noop));
            if constexpr (HDR)
                rh = valid && ph.v4 ? lane_hdr_cksum<NT>(a, ph.hl, nullptr) : (uint16_t)0;
        }
        // Both results from one block, after every path's loads: apart, hipcc
        // put an s_waitcnt vmcnt(0) between the two stores, so the second
        // waited for the first one's write (C4 fused 649 -> 641 us).  The
        // results' HBM writes themselves cost C4 ~30 us per 32 MB array
        // whatever their form -- 16-byte chunks, one 512-B run per block of
        // tiles, nt / sc1 (profiles/ab_r03_fused_store.log).
        // (Tuning build only, for the write-cost counters of DESIGN.md
        // section 10: WC_VARIANT bit 24 drops the result store, bit 25 the
        // header-checksum store -- results are then missing.)
        if (valid) {
            if constexpr (HDR)
                if (!(variant & (1 << 25)))
                    out_hdr[p] = rh;
            if (out && !(variant & (1 << 24)))
                out[p] = r;
        }
        nbad += valid && r != 0;
        wave_order(); // the tables are rewritten by the next tile
    }
    if (bad) {
        nbad = group_sum<64>(nbad);
        if (lane == 0 && nbad)
            atomicAdd(bad, (unsigned long long)nbad);
    }
}

// The flat-path fallback inside k_cksum_seg always uses 2 rows per group (the
// default); WC_FLAT_UN only changes the standalone flat kernel.
static hipError_t launch_seg_kernel(const LaunchArgs &a, hipStream_t st)
{
    constexpr int UN = 2;
    const uint64_t tiles = (a.n + 63) / 64;
    int grid = (int)std::min<uint64_t>(
        kMaxGridBlocks, std::max<uint64_t>(1, (tiles + kFlatWaves - 1) / kFlatWaves));
#ifdef WC_TUNING
    if ((a.variant >> 20) & 15) // A/B: cap the grid at k * 1024 blocks (several tiles per wave)
        grid = std::min(grid, ((a.variant >> 20) & 15) * 1024);
#endif
    const uint8_t *b = (const uint8_t *)a.base;
    unsigned long long *bad = (unsigned long long *)a.bad;
    if (a.out_hdr) {
        // fused IPv4 header + payload_cksum pass (ragged), default row-group sizes
        if (a.kind != WC_KIND_PAYLOAD || !a.offs)
            return hipErrorInvalidValue;
        hipLaunchKernelGGL((k_cksum_seg<UN, 4, 4, WC_KIND_PAYLOAD, true, false, true>),
                           dim3(grid), dim3(256), 0, st, b, a.offs, a.lens, a.n, a.out, bad,
                           a.grp_thr, a.variant, a.stride, a.len, a.out_hdr, (int)a.gather);
        return hipGetLastError();
    }
#define WC_SEG_K(K, S)                                                         \
    hipLaunchKernelGGL((k_cksum_seg<UN, US, UG, K, true, S>), dim3(grid), dim3(256), 0, st, \
                       b, a.offs, a.lens, a.n, a.out, bad, a.grp_thr, a.variant, a.stride, \
                       a.len, nullptr, (int)a.gather)
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
    // a.grp_rows (WC_GRP_ROWS 4 or 2; 6 and 8 measured no faster on netmap
    // slots).
    if (a.seg_rows == 2) {
        WC_SEG(2, 4)
    } else if (a.seg_rows == 8) {
        WC_SEG(8, 4)
    } else if (a.grp_rows == 2) {
        WC_SEG(4, 2)
    } else {
        WC_SEG(4, 4)
    }
#undef WC_SEG
#undef WC_SEG_K
    return hipGetLastError();
}

hipError_t launch_flat(const LaunchArgs &a, int rows, hipStream_t st)
{
    if (a.seg_rows && !(a.diag_noload && a.kind == WC_KIND_IP) &&
        (!a.out_hdr || (a.kind == WC_KIND_PAYLOAD && a.offs)))
        return launch_seg_kernel(a, st);
    return launch_flat_kernel(a, rows, st);
}

} // namespace wc
