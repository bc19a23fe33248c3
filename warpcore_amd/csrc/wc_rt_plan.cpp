// wc_rt_plan.cpp -- the launch planner (group shape, kernel family, grid),
// the device-resident batch calls, the scalar drop-ins for the reference's
// ip_cksum / payload_cksum (/root/reference/lib/src/in_cksum.h:32-36), and
// the bench / introspection entry points.

#include "wc_rt.h"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>

namespace wc {
namespace rt __attribute__((visibility("hidden"))) {

// ---------------------------------------------------------------------------
// Planner.

wc::Shape shape_for_chunks(uint32_t nch, bool full, bool payload, bool aligned,
                           bool sparse = false)
{
    // Smallest group covering the packet in one pass, with U packets per
    // group so every lane keeps ~4-18 16-byte loads in flight (tuned on
    // MI355X: DESIGN.md section 5, profiles/tune_r01_*.log).
    if (nch <= 4)
        return {4, 1, 4};
    // Sparse batches (stride >= twice the packet's chunk span: netmap slots)
    // run at the rate of the cache lines they touch, one or two per packet;
    // shapes with more lanes per packet reach it (2048-B slots at +14,
    // profiles/ab_r03_slot_shapes.log): ip_cksum 5-6 chunks on 8 x 1 x 4
    // (64 / 72 / 80 B: 36 -> 41, 41 -> 47, 46 -> 52 %).  payload_cksum keeps
    // 4 x 2 x 2 there (8 x 1 x 4: 36 -> 28 %: its header hand-off between
    // lanes costs more the wider the group), and takes it for sparse packets
    // of up to 16 chunks too, even where that is two passes: read from HBM
    // (rotating buffers, round 4) it beats the (8,1,4) / (8,2,4) round 3
    // picked on Infinity-Cache-resident reruns -- 96 B 35.6 -> 27.2 us, 128 B
    // 49.2 -> 44.4, 160 B 49.6 -> 44.3, 200 B 50.0 -> 46.2, 240 B 48.4 ->
    // 45.9 (profiles/ab_r04_payload_small.log).
    if (nch <= 6 || (sparse && payload && nch <= 16))
        return sparse && !payload ? wc::Shape{8, 1, 4} : wc::Shape{4, 2, 2};
    if (nch <= 8)
        return {8, 1, 4};
    // 9..24 chunks: 8 lanes x 3 chunks, two packets per group -- fewer dead
    // lane slots than 16 x 2 (profiles/sweep_r01_mid_shapes.log: 256 B 78.7 -> 84.1 %,
    // 200 B 55 -> 67.5 %, 256 B at +14 50 -> 60 % of HBM peak)
    if (nch <= 16 || (nch <= 24 && !full))
        return {8, 3, 2};
    // aligned unmasked 17..30 chunks: 16 x 2 x 4 (320 B 80.8 -> 85.4 %,
    // profiles/sweep_r02_small_shapes.log)
    if (nch <= 30)
        return {16, 2, 4};
    // ~512 B: 8 lanes x 6 chunks, one packet per group (85 -> 90.8 % packed,
    // 81 -> 87 % in 2048-B slots); 576 B: (16,3,2) (85 -> 86.6 %)
    // (profiles/sweep_r01_mid_shapes.log)
    if (nch <= 34)
        return {8, 6, 1};
    // 35..48 chunks: one packet per 16-lane group when aligned unmasked
    // (704 B 90.5 -> 93.6 %, 576 B 90.7 -> 91.2 %)
    if (nch <= 48)
        return full ? wc::Shape{16, 3, 1} : wc::Shape{16, 3, 2};
    // 49..96 chunks (784..1536 B): 32-lane groups with 2-4 loads per lane
    // beat 16 x 6 for ip_cksum (profiles/sweep_r02_wide_shapes.log: C2
    // 1472 B 88.6-91 -> 93.3-95 %, 1024 B 82 -> 94 %, 2048-B slots at +14
    // +2..5 points).  Aligned unmasked (FULL) batches and masked ones differ
    // below 88 chunks.  payload_cksum (more registers per lane) keeps 16-lane
    // groups, fewer packets per group when aligned
    // (profiles/sweep_r02_payload_shapes.log: C2 payload 84 -> 92.5 %).
    if (payload && nch <= 96) {
        if (aligned)
            return {16, 6, 2};
        return nch <= 80 ? wc::Shape{16, 5, 4} : wc::Shape{32, 3, 2};
    }
    if (nch <= 56)
        return full ? wc::Shape{32, 2, 4} : wc::Shape{16, 5, 4};
    if (nch <= 63)
        return full ? wc::Shape{32, 2, 2} : wc::Shape{16, 5, 4};
    if (nch <= 77)
        return full ? wc::Shape{32, 4, 2} : wc::Shape{32, 3, 2};
    if (nch <= 87)
        return full ? wc::Shape{32, 4, 1} : wc::Shape{32, 4, 2};
    if (nch <= 128)
        return {32, 4, 1};
    if (nch <= 256)
        return {64, 4, 1};
    if (nch <= 576)
        return {32, 18, 1};
    return {64, 9, 1};
}

// Lean-kernel shape: a group whose one pass the packet fills exactly (G *
// CPL == chunks, no dead slots -- a pass the packet does not fill costs the
// masked path: 576 B in (16,3,1) ran at 70 vs 91 %), groups of >= 8 lanes
// (a 4-lane group reads 64-B half lines per load, 128 B in (4,2,2) ran at
// 75 vs 89 % in (8,1,4)) except for 64-B packets, which 4-lane groups read
// as one contiguous kilobyte per load; ~4 loads in flight per lane
// (profiles/ab_r03_lean*.log).  {0,0,0}: no such shape, not lean.  Packets
// under 4 chunks take the masked path of (4, 1, 4).
// Lean-kernel shape for packets at a start phase (PH): one pass covering the
// window, dead slots allowed (they read nothing new and are masked).
wc::Shape lean_ph_shape(uint32_t nch)
{
    if (nch <= 4)
        return {4, 1, 4};
    if (nch <= 8)
        return {8, 1, 4};
    if (nch <= 16)
        return {8, 2, 4};
    if (nch <= 24)
        return {8, 3, 2};
    if (nch <= 32)
        return {16, 2, 2};
    if (nch <= 48)
        return {16, 3, 1};
    return {0, 0, 0};
}

wc::Shape lean_shape_for(uint32_t nch)
{
    if (nch <= 4)
        return {4, 1, 4};
    for (int g = 8; g <= 64; g *= 2) {
        if (nch % (uint32_t)g)
            continue;
        const int cpl = (int)(nch / (uint32_t)g);
        if (cpl > 3)
            continue;
        return {g, cpl, cpl == 1 ? 4 : cpl == 2 ? 2 : (g <= 8 ? 2 : 1)};
    }
    return {0, 0, 0};
}

int grid_for(const Device &D, const Config &C, const wc::Shape &sh, uint64_t n)
{
    const uint64_t ppw = (uint64_t)(64 / sh.group) * sh.unroll;
    const uint64_t waves = (n + ppw - 1) / ppw;
    const uint64_t blocks = (waves + 3) / 4;
    // One-shot grid by default: every block handles one wave-iteration per
    // wave and retires (measured faster than a resident grid-stride loop on
    // MI355X: DESIGN.md section 5).  WC_BLOCKS_PER_CU / WC_GRID cap it into a
    // grid-stride launch for experiments.
    // The kernel grid-strides, so capping at wc::kMaxGridBlocks (gridDim.x *
    // 256 must fit in a uint32) stays correct for any n.
    uint64_t cap = wc::kMaxGridBlocks;
    if (C.blocks_per_cu > 0)
        cap = std::min(cap, (uint64_t)D.cus * (uint64_t)C.blocks_per_cu);
    if (C.grid > 0)
        cap = std::min(cap, (uint64_t)C.grid);
    return (int)std::max<uint64_t>(1, std::min(blocks, cap));
}


bool lean_shape_ok(const wc::Shape &sh)
{
#define WC_SHAPE(G_, C_, U_)                                                   \
    if (sh.group == G_ && sh.cpl == C_ && sh.unroll == U_)                     \
        return true;
    WC_LEAN_SHAPE_LIST
#undef WC_SHAPE
    return false;
}

Plan plan_strided(const Device &D, const Config &C, uint64_t base, uint64_t stride,
                  uint32_t len, uint64_t n, int kind, bool hdr)
{
    Plan p;
    const uint32_t span = kind == WC_CKSUM_PAYLOAD ? std::max(len, 20u) : len;
    // Worst-case start phase within a 16-byte chunk over the batch.
    const uint32_t phase = (stride % 16 == 0) ? (uint32_t)(base % 16) : 15u;
    const uint32_t nch = (phase + span + 15u) / 16u;
    p.full = kind == WC_CKSUM_IP && base % 16 == 0 && stride % 16 == 0 &&
             len % 16 == 0 && !(C.variant & 2);
    p.shape = C.have_shape ? C.shape
                           : shape_for_chunks(nch, p.full, kind == WC_CKSUM_PAYLOAD, phase == 0,
                                              stride >= 32ull * nch);
    p.grid = grid_for(D, C, p.shape, n);
    // Packed (or nearly packed) packets that the group kernel would have to
    // mask: the seg kernel streams their byte range instead (k_cksum_seg<STR>)
    // where it measured faster -- a 60-length x 2-offset sweep on MI355X
    // (profiles/sweep_r02_planner.log):
    //   stride % 64 == 0   group kernel (every packet at the same offset in
    //                      its cache lines: 256 B at +14 85 % vs seg 70-73 %)
    //   <= 5 chunks        group kernel
    //   6..14 chunks       seg, 2-row groups (120 B: 74 % vs group 51-56 %)
    //   36..48 chunks      group kernel (550-700 B: 84-89 % vs seg 83-84 %)
    //   >= 90 chunks       group kernel
    //   otherwise          seg, 4-row groups (300 B: 84 % vs group 69 %)
    // Aligned unmasked (FULL) packets of 5..16 chunks at a stride that is not
    // a multiple of 64 take the seg kernel too: the group kernel leaves most
    // of its lane slots dead there (80..240 B packed: 64-77 % vs seg 71-85 %;
    // 64 / 128 / 256 B, whose packets share cache-line phases, keep the
    // group kernel: profiles/sweep_r02_small_aligned.log), 2-row groups up to
    // 9 chunks, 4-row groups above.
    // payload_cksum: packed packets below 64 chunks take the seg kernel at any
    // stride -- it reads the header bytes from its own stream, where the group
    // kernel exchanges them between lanes (64 B 46 -> 56 %, 192 B 54 -> 82 %,
    // 576 B 74-77 -> 83-84 %, 900 B 78 -> 84 %; from 64 chunks on the group
    // kernel's 87-92 % wins: profiles/sweep_r02_payload_seg.log).
    // WC_STRIDED_SEG = 0 never, 2 always (no fused header), 1 = the table;
    // WC_SEG_ROWS forces the row-group size.
    const int sseg = C.strided_seg;
    const bool payload = kind == WC_CKSUM_PAYLOAD;
    const bool packed = len != 0 && stride >= len && stride <= len + len / 8u;
    const bool seg_table =
        payload ? nch < 64
                : stride % 64 != 0 && (p.full ? nch >= 5 && nch <= 16
                                              : nch > 5 && !(nch >= 36 && nch <= 48) && nch < 90);
    if (!hdr && n >= 64 && packed && (sseg == 2 || (sseg == 1 && seg_table))) {
        p.shape = {0, 1, C.flat_un};
        const uint32_t rows2 = payload ? 5u : (p.full ? 9u : 14u);
        p.seg_rows = C.seg_rows_set ? C.seg_rows : (nch <= rows2 ? 2 : 4);
        p.grid = 0;
    }
    // Aligned packets (base, stride and len multiples of 16) that one pass of
    // a group covers take the lean kernel (wc_k_lean.hip): scalar wave
    // addresses, word sums, payload_cksum's header terms from the group's
    // first lane.  payload_cksum needs len >= 48 there (the whole IPv4 /
    // IPv6 header inside the packet); up to WC_LEAN_MAX chunks.
    const bool aligned16 = base % 16 == 0 && stride % 16 == 0 && len % 16 == 0 && len != 0;
    // Sparse payload_cksum packets at one even start phase (netmap slots: IP
    // packets at +14) of up to 18 window chunks take it too, with per-slot
    // byte masks (PH, wc_k_lean.hip): in 2048-B slots at +14, from HBM,
    // payload 64 B 24.2 -> 22.5 us, 128 B 41.3 -> 39.8, 256 B 58.2 -> 56.1
    // against the group kernel, within 1 us of ip_cksum; ip_cksum gains
    // nothing (128 B 39.2 -> 41.2 us) and 576 B loses on both kinds (96.9 ->
    // 112.7 us), so they keep the group kernel (profiles/ab_r05_lean_phase.log).
    const bool phased = !aligned16 && C.lean_phase && C.nt && stride % 16 == 0 &&
                        base % 2 == 0 && len != 0 && !packed && sseg != 2 && payload &&
                        nch <= 18;
    if (!hdr && C.lean_max > 0 && (aligned16 || phased) && (!payload || len >= 48) &&
        nch <= (uint32_t)C.lean_max && (sseg != 2 || !packed)) {
        const wc::Shape sh = C.have_shape ? C.shape : aligned16 ? lean_shape_for(nch)
                                                                 : lean_ph_shape(nch);
        const uint64_t ppw = (uint64_t)(64 / std::max(sh.group, 1)) * sh.unroll;
        if (lean_shape_ok(sh) && nch <= (uint32_t)(sh.group * sh.cpl) && ppw <= 64 &&
            ppw * stride < (1ull << 32)) {
            p.shape = sh;
            p.lean = true;
            p.seg_rows = 0;
            p.grid = grid_for(D, C, sh, n);
        }
    }
    return p;
}

// Ragged batches take the segmented-prefix kernel k_cksum_seg (both kinds):
// dense tiles stream their byte range, sparse ones take its flat path
// (DESIGN.md section 4.4), the fused header pass (out_hdr) included (group =
// 0 marks both the seg and the flat kernel; unroll = 64-chunk rows per
// ping-pong group of the flat path, WC_FLAT_UN).  WC_SEG = 0 forces the flat
// kernel; WC_SEG_ROWS = 2 / 4 / 8 rows per seg row group.  A host zero-copy batch of
// at most kZcGroupMax packets takes the ragged group kernel instead: a flat
// wave walks its 64-packet tile's rows one PCIe latency at a time, the group
// kernel issues every packet's loads at once.  (Device-resident batches
// measured no better on the group kernel at any size -- launch cost
// dominates small ones -- so WC_FLAT_MIN defaults to 0.)
Plan plan_ragged(const Device &D, const Config &C, uint64_t n, int kind,
                 bool zero_copy, bool hdr)
{
    (void)D;
    Plan p;
    p.full = false;
    const bool small = (zero_copy && n <= (uint64_t)C.zc_group_max) ||
                       n < C.flat_min;
    if (small && !hdr) {
        p.shape = C.have_rshape ? C.rshape : wc::Shape{64, 2, 1};
        const uint64_t ppw = (uint64_t)(64 / p.shape.group) * p.shape.unroll;
        p.grid = (int)std::min<uint64_t>(
            wc::kMaxGridBlocks, std::max<uint64_t>(1, ((n + ppw - 1) / ppw + 3) / 4));
        return p;
    }
    p.shape = {0, 1, C.flat_un};
    p.grid = 0;
    if ((!zero_copy || C.zc_seg) && C.diag_noload == 0 && C.seg != 0 &&
        (!hdr || kind == WC_CKSUM_PAYLOAD))
        p.seg_rows = C.seg_rows;
    return p;
}

int run(const Device &D, const Config &C, const wc::LaunchArgs &args, const Plan &p,
        hipStream_t st)
{
    (void)D;
    wc::LaunchArgs a = args;
    a.seg_rows = p.seg_rows;
    a.grp_thr = C.grp_dense | (C.grp_sparse << 8);
    a.grp_rows = C.grp_rows;
    a.flat_pk = C.flat_pk;
    a.gather = C.gather;
    hipError_t e = p.lean              ? wc::launch_lean(a, p.shape, p.grid, st)
                   : p.shape.group == 0 ? wc::launch_flat(a, p.shape.unroll, st)
                                        : wc::launch_cksum(a, p.shape, p.grid, st);
    return hip_err(e);
}

int batch_strided(const void *d_base, uint64_t stride, uint16_t len, uint64_t n,
                  uint16_t *d_out, uint64_t *d_bad, int kind, void *stream,
                  uint16_t *d_out_hdr = nullptr)
{
    if (kind != WC_CKSUM_IP && kind != WC_CKSUM_PAYLOAD)
        return WC_EINVAL;
    if (n == 0)
        return WC_OK;
    if (!d_base || (!d_out && !d_bad))
        return WC_EINVAL;
    Device *D = nullptr;
    Config C;
    int rc = ensure_device(&D, &C);
    if (rc)
        return rc;
    // A batch larger than the piece runs as back-to-back launches of it on
    // the same stream, each planned on its own (Config::split_bytes).
    uint64_t piece = n;
    if (C.split_pkts)
        piece = std::min(n, C.split_pkts);
    else if (C.split_bytes && stride)
        piece = std::min(n, std::max<uint64_t>(1, C.split_bytes / stride));
    for (uint64_t p0 = 0; p0 < n; p0 += piece) {
        const uint64_t cnt = std::min(piece, n - p0);
        const uint8_t *b = (const uint8_t *)d_base + p0 * stride;
        const Plan p = plan_strided(*D, C, (uint64_t)b, stride, len, cnt, kind, d_out_hdr != nullptr);
        wc::LaunchArgs a{b,      stride, len,  nullptr,  nullptr, cnt,
                         d_out ? d_out + p0 : nullptr,  d_bad,  kind, false,    p.full,  C.nt != 0,
                         0,      d_out_hdr ? d_out_hdr + p0 : nullptr};
        a.variant = C.variant;
        rc = run(*D, C, a, p, (hipStream_t)stream);
        if (rc)
            return rc;
    }
    return WC_OK;
}

int batch_ragged(const void *d_base, const uint64_t *d_off, const uint16_t *d_len,
                 uint64_t n, uint16_t *d_out, uint64_t *d_bad, int kind,
                 void *stream, uint16_t *d_out_hdr = nullptr)
{
    if (kind != WC_CKSUM_IP && kind != WC_CKSUM_PAYLOAD)
        return WC_EINVAL;
    if (n == 0)
        return WC_OK;
    if (!d_base || !d_off || !d_len || (!d_out && !d_bad))
        return WC_EINVAL;
    Device *D = nullptr;
    Config C;
    int rc = ensure_device(&D, &C);
    if (rc)
        return rc;
    const uint64_t piece = C.split_pkts && n > C.split_pkts ? C.split_pkts : n;
    for (uint64_t p0 = 0; p0 < n; p0 += piece) {
        const uint64_t cnt = std::min(piece, n - p0);
        const Plan p = plan_ragged(*D, C, cnt, kind, false, d_out_hdr != nullptr);
        wc::LaunchArgs a{d_base, 0,     0,    d_off + p0, d_len + p0, cnt,
                         d_out ? d_out + p0 : nullptr,  d_bad, kind, true,  false, C.nt != 0,
                         C.flat_tpw, d_out_hdr ? d_out_hdr + p0 : nullptr, C.diag_noload != 0};
        a.variant = C.variant;
        rc = run(*D, C, a, p, (hipStream_t)stream);
        if (rc)
            return rc;
    }
    return WC_OK;
}

[[noreturn]] void die(const char *what, int rc)
{
    fprintf(stderr, "wccksum: %s failed: %s (%d)\n", what, wc_strerror(rc), rc);
    abort();
}

uint16_t scalar_cksum(const void *buf, uint16_t len, int kind, const char *who)
{
    std::lock_guard<FairMutex> lk(g_mu);
    Device *D = nullptr;
    int rc = init_locked(-1, &D);
    if (rc)
        die(who, rc);
    // payload_cksum reads the IPv4 header fields up to byte 19 whatever len is
    // (in_cksum.c:149-151); stage the same bytes the reference reads.
    const size_t span =
        kind == WC_CKSUM_PAYLOAD ? std::max<size_t>(len, 20) : (size_t)len;
    memcpy(D->h_stage, buf, span);
    // (the load flavour the planner assumed: the lean kernel's phase path,
    // which a 1-packet batch at an even staging phase may take, exists with
    // nontemporal loads only)
    Plan p = plan_strided(*D, g_cfg, (uint64_t)D->d_stage, 0, len, 1, kind);
    wc::LaunchArgs a{D->d_stage, 0,   len,  nullptr, nullptr, 1,
                     D->d_res,   nullptr, kind, false,   p.full,  g_cfg.nt != 0};
    rc = run(*D, g_cfg, a, p, D->scalar_st);
    if (rc)
        die(who, rc);
    hipError_t e = hipStreamSynchronize(D->scalar_st);
    if (e != hipSuccess)
        die(who, hip_err(e));
    return *(volatile uint16_t *)D->h_res;
}

} // namespace rt
} // namespace wc

using namespace wc::rt;

extern "C" {

uint16_t ip_cksum(const void *buf, uint16_t len)
{
    return scalar_cksum(buf, len, WC_CKSUM_IP, "ip_cksum");
}

uint16_t payload_cksum(const void *buf, uint16_t len)
{
    return scalar_cksum(buf, len, WC_CKSUM_PAYLOAD, "payload_cksum");
}

int wc_cksum_strided(const void *d_base, uint64_t stride, uint16_t len,
                     uint64_t n, uint16_t *d_out, int kind, void *stream)
{
    if (!d_out && n)
        return WC_EINVAL;
    return batch_strided(d_base, stride, len, n, d_out, nullptr, kind, stream);
}

int wc_cksum_ragged(const void *d_base, const uint64_t *d_off,
                    const uint16_t *d_len, uint64_t n, uint16_t *d_out,
                    int kind, void *stream)
{
    if (!d_out && n)
        return WC_EINVAL;
    return batch_ragged(d_base, d_off, d_len, n, d_out, nullptr, kind, stream);
}

int wc_verify_strided(const void *d_base, uint64_t stride, uint16_t len,
                      uint64_t n, uint16_t *d_out, uint64_t *d_bad, int kind,
                      void *stream)
{
    if (!d_bad && n)
        return WC_EINVAL;
    return batch_strided(d_base, stride, len, n, d_out, d_bad, kind, stream);
}

int wc_verify_ragged(const void *d_base, const uint64_t *d_off,
                     const uint16_t *d_len, uint64_t n, uint16_t *d_out,
                     uint64_t *d_bad, int kind, void *stream)
{
    if (!d_bad && n)
        return WC_EINVAL;
    return batch_ragged(d_base, d_off, d_len, n, d_out, d_bad, kind, stream);
}

int wc_cksum_ip_udp_strided(const void *d_base, uint64_t stride, uint16_t len,
                            uint64_t n, uint16_t *d_out_ip_hdr,
                            uint16_t *d_out_payload, void *stream)
{
    if (n && (!d_out_ip_hdr || !d_out_payload))
        return WC_EINVAL;
    return batch_strided(d_base, stride, len, n, d_out_payload, nullptr,
                         WC_CKSUM_PAYLOAD, stream, d_out_ip_hdr);
}

int wc_cksum_ip_udp_ragged(const void *d_base, const uint64_t *d_off,
                           const uint16_t *d_len, uint64_t n, uint16_t *d_out_ip_hdr,
                           uint16_t *d_out_payload, void *stream)
{
    if (n && (!d_out_ip_hdr || !d_out_payload))
        return WC_EINVAL;
    return batch_ragged(d_base, d_off, d_len, n, d_out_payload, nullptr,
                        WC_CKSUM_PAYLOAD, stream, d_out_ip_hdr);
}

int wc_sclk_probe(uint64_t *d_samples, int n, uint64_t interval, void *stream)
{
    if (n <= 0)
        return WC_OK;
    if (!d_samples || !interval || ((uintptr_t)d_samples & 7u))
        return WC_EINVAL;
    Device *D = nullptr;
    Config C;
    int rc = ensure_device(&D, &C);
    if (rc)
        return rc;
    return hip_err(wc::launch_sclk_probe(d_samples, n, interval, (hipStream_t)stream));
}

int wc_synth_fill(void *d_buf, uint64_t nbytes, uint64_t seed, void *stream)
{
    if (!nbytes)
        return WC_OK;
    if (!d_buf || ((uintptr_t)d_buf & 15u))
        return WC_EINVAL;
    Device *D = nullptr;
    Config C;
    int rc = ensure_device(&D, &C);
    if (rc)
        return rc;
    const uint64_t threads = (nbytes / 16) + 1;
    const int grid = (int)std::min<uint64_t>((threads + 255) / 256,
                                             (uint64_t)D->cus * 8);
    return hip_err(wc::launch_synth(d_buf, nbytes, seed, grid, (hipStream_t)stream));
}

int wc_plan_strided(uint64_t base_addr, uint64_t stride, uint16_t len,
                    uint64_t n, int kind, int *group, int *chunks_per_lane,
                    int *unroll, int *grid)
{
    if (kind != WC_CKSUM_IP && kind != WC_CKSUM_PAYLOAD)
        return WC_EINVAL;
    Device *D = nullptr;
    Config C;
    int rc = ensure_device(&D, &C);
    if (rc)
        return rc;
    const Plan p = plan_strided(*D, C, base_addr, stride, len, n, kind);
    if (group)
        *group = p.shape.group;
    if (chunks_per_lane)
        *chunks_per_lane = p.shape.cpl;
    if (unroll)
        *unroll = p.shape.unroll;
    if (grid)
        *grid = p.grid;
    return WC_OK;
}

const char *wc_plan_strided_kernel(uint64_t base_addr, uint64_t stride, uint16_t len, uint64_t n,
                                   int kind)
{
    if (kind != WC_CKSUM_IP && kind != WC_CKSUM_PAYLOAD)
        return "invalid";
    Device *D = nullptr;
    Config C;
    if (ensure_device(&D, &C))
        return "invalid";
    const Plan p = plan_strided(*D, C, base_addr, stride, len, n, kind);
    return p.lean ? "lean" : p.shape.group == 0 ? "seg" : "group";
}

} // extern "C"
