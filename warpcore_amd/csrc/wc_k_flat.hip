// wc_k_flat.hip -- ragged batches on gfx950: the chunk-balanced flat kernel
// k_cksum_flat, used for WC_SEG=0 and (tuning build
// only) its diagnostic no-load build; k_cksum_seg falls back to the same tile
// path.
#include "wc_flat.h"

namespace wc {

template <int UN, int KIND, bool NT, bool HDR, bool NOLOAD = false, int PK = 1>
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
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); // wave-uniform: SGPR
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
        auto next_hdr = [&] {
            if constexpr (KIND == WC_KIND_PAYLOAD)
                hdr_n = load_hdr((uint64_t)base + off_n);
        };
        uint32_t acc;
        if constexpr (KIND == WC_KIND_PAYLOAD && !NOLOAD)
            acc = flat_tile_sum_payload<UN, NT, false, decltype(next_hdr) &, PK>(
                L, &lut, lane, a, len, valid, ph, hdr, next_hdr);
        else
            acc = flat_tile_sum<UN, KIND, NT, NOLOAD, false, decltype(next_hdr) &, PK>(
                L, &lut, lane, a, len, valid, ph, next_hdr);

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

template <int UN>
static hipError_t launch_flat_un(const LaunchArgs &a, hipStream_t st)
{
    const uint64_t tiles = (a.n + 63) / 64;
    const uint64_t tpw = (uint64_t)(a.tiles_per_wave > 0 ? a.tiles_per_wave : 1);
    const uint64_t waves = (tiles + tpw - 1) / tpw;
    const int grid = (int)std::min<uint64_t>(
        kMaxGridBlocks, std::max<uint64_t>(1, (waves + kFlatWaves - 1) / kFlatWaves));
    const uint8_t *b = (const uint8_t *)a.base;
    unsigned long long *bad = (unsigned long long *)a.bad;
#define WC_FLAT(K, N, H)                                                       \
    if (a.flat_pk == 2)                                                        \
        hipLaunchKernelGGL((k_cksum_flat<UN, K, N, H, false, 2>), dim3(grid), dim3(256), 0, \
                           st, b, a.offs, a.lens, a.n, a.out, bad, a.out_hdr); \
    else                                                                       \
        hipLaunchKernelGGL((k_cksum_flat<UN, K, N, H>), dim3(grid), dim3(256), 0, st, b, \
                           a.offs, a.lens, a.n, a.out, bad, a.out_hdr)
#ifdef WC_TUNING
    // Diagnostic no-load build (timing only, wrong results): tuning library only.
    if (a.diag_noload && a.kind == WC_KIND_IP) {
        hipLaunchKernelGGL((k_cksum_flat<UN, WC_KIND_IP, true, false, true>), dim3(grid),
                           dim3(256), 0, st, b, a.offs, a.lens, a.n, a.out, bad, a.out_hdr);
        return hipGetLastError();
    }
#endif
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

hipError_t launch_flat_kernel(const LaunchArgs &a, int rows, hipStream_t st)
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

} // namespace wc
