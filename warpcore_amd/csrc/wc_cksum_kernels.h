// wc_cksum_kernels.h -- internal interface between the C-ABI layer
// (wc_cksum_api.cpp) and the gfx950 kernels (wc_k_*.hip, wc_device.h).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#define WC_KIND_IP 0
#define WC_KIND_PAYLOAD 1

// Every (group width, chunk loads per lane, packets per group-iteration)
// shape the strided planner may pick (wc_cksum_api.cpp: shape_for_chunks) or
// WC_SHAPE may request; each is instantiated for ip_cksum (masked and
// aligned-unmasked) and payload_cksum, with temporal and nontemporal loads.
#define WC_SHAPE_LIST                                                          \
    WC_SHAPE(4, 1, 1)                                                          \
    WC_SHAPE(4, 1, 2)                                                          \
    WC_SHAPE(4, 1, 4)                                                          \
    WC_SHAPE(4, 1, 8)                                                          \
    WC_SHAPE(4, 2, 2)                                                          \
    WC_SHAPE(4, 2, 4)                                                          \
    WC_SHAPE(8, 1, 2)                                                          \
    WC_SHAPE(8, 2, 4)                                                          \
    WC_SHAPE(8, 3, 2)                                                          \
    WC_SHAPE(8, 3, 4)                                                          \
    WC_SHAPE(4, 5, 4)                                                          \
    WC_SHAPE(8, 5, 2)                                                          \
    WC_SHAPE(8, 6, 2)                                                          \
    WC_SHAPE(8, 6, 1)                                                          \
    WC_SHAPE(16, 3, 2)                                                         \
    WC_SHAPE(16, 1, 2)                                                         \
    WC_SHAPE(16, 2, 2)                                                         \
    WC_SHAPE(16, 3, 1)                                                         \
    WC_SHAPE(32, 1, 2)                                                         \
    WC_SHAPE(32, 1, 4)                                                         \
    WC_SHAPE(32, 2, 1)                                                         \
    WC_SHAPE(4, 1, 16)                                                         \
    WC_SHAPE(8, 1, 4)                                                          \
    WC_SHAPE(8, 1, 8)                                                          \
    WC_SHAPE(16, 1, 4)                                                         \
    WC_SHAPE(16, 1, 8)                                                         \
    WC_SHAPE(16, 2, 4)                                                         \
    WC_SHAPE(16, 3, 4)                                                         \
    WC_SHAPE(16, 4, 2)                                                         \
    WC_SHAPE(16, 4, 4)                                                         \
    WC_SHAPE(16, 5, 2)                                                         \
    WC_SHAPE(16, 5, 4)                                                         \
    WC_SHAPE(16, 6, 2)                                                         \
    WC_SHAPE(16, 6, 4)                                                         \
    WC_SHAPE(32, 2, 2)                                                         \
    WC_SHAPE(32, 2, 4)                                                         \
    WC_SHAPE(32, 3, 1)                                                         \
    WC_SHAPE(32, 3, 2)                                                         \
    WC_SHAPE(32, 3, 4)                                                         \
    WC_SHAPE(32, 3, 8)                                                         \
    WC_SHAPE(32, 4, 1)                                                         \
    WC_SHAPE(32, 4, 2)                                                         \
    WC_SHAPE(64, 2, 1)                                                         \
    WC_SHAPE(64, 2, 2)                                                         \
    WC_SHAPE(32, 18, 1)                                                        \
    WC_SHAPE(64, 4, 1)                                                         \
    WC_SHAPE(64, 9, 1)                                                         \
    WC_SHAPE(64, 9, 2)

// Shapes of the small-batch ragged group kernel (ip_cksum / payload_cksum,
// nontemporal loads).
#define WC_RAGGED_SHAPE_LIST                                                   \
    WC_SHAPE(16, 2, 2)                                                         \
    WC_SHAPE(32, 4, 1)                                                         \
    WC_SHAPE(32, 3, 2)                                                         \
    WC_SHAPE(32, 2, 1)                                                         \
    WC_SHAPE(64, 2, 1)                                                         \
    WC_SHAPE(64, 4, 1)                                                         \
    WC_SHAPE(16, 6, 4)

// Shapes of the lean kernel (aligned strided batches, one pass per packet;
// wc_k_lean.hip): the planner's FULL shapes up to 576 B plus tuning
// neighbours for small packets.
#define WC_LEAN_SHAPE_LIST                                                     \
    WC_SHAPE(4, 1, 2)                                                      \
    WC_SHAPE(4, 1, 4)                                                      \
    WC_SHAPE(4, 2, 2)                                                      \
    WC_SHAPE(4, 2, 4)                                                      \
    WC_SHAPE(4, 3, 1)                                                      \
    WC_SHAPE(8, 1, 2)                                                      \
    WC_SHAPE(8, 1, 4)                                                      \
    WC_SHAPE(8, 1, 8)                                                      \
    WC_SHAPE(8, 2, 2)                                                      \
    WC_SHAPE(8, 2, 4)                                                      \
    WC_SHAPE(8, 3, 1)                                                      \
    WC_SHAPE(8, 3, 2)                                                      \
    WC_SHAPE(8, 6, 1)                                                      \
    WC_SHAPE(16, 1, 4)                                                     \
    WC_SHAPE(16, 2, 2)                                                     \
    WC_SHAPE(16, 2, 4)                                                     \
    WC_SHAPE(16, 3, 1)                                                     \
    WC_SHAPE(16, 3, 2)                                                     \
    WC_SHAPE(16, 6, 2)                                                     \
    WC_SHAPE(32, 1, 4)                                                     \
    WC_SHAPE(32, 2, 2)                                                     \
    WC_SHAPE(32, 2, 4)                                                     \
    WC_SHAPE(32, 3, 1)                                                     \
    WC_SHAPE(32, 3, 2)                                                     \
    WC_SHAPE(32, 4, 1)                                                     \
    WC_SHAPE(32, 4, 2)                                                     \
    WC_SHAPE(32, 18, 1)                                                    \
    WC_SHAPE(64, 1, 4)                                                     \
    WC_SHAPE(64, 2, 2)                                                     \
    WC_SHAPE(64, 3, 1)                                                     \
    WC_SHAPE(64, 4, 1)

namespace wc {

// Largest grid any launcher uses: gridDim.x * 256 threads must fit in a
// uint32 on AMD.  Every kernel strides over its work, so a capped grid stays
// correct (wc_cksum_api.cpp grid_for, the ragged launchers).
constexpr uint64_t kMaxGridBlocks = (1ull << 24) - 1;

struct LaunchArgs {
    const void *base;
    uint64_t stride;
    uint32_t len;
    const uint64_t *offs;
    const uint16_t *lens;
    uint64_t n;
    uint16_t *out;
    uint64_t *bad;
    int kind;
    bool ragged; // offs/lens batch: flat kernel, or the ragged group kernel
    bool full;
    bool nontemporal;
    int tiles_per_wave; // flat kernel: 64-packet tiles each wave walks
    uint16_t *out_hdr;  // payload kind: also the IPv4 header checksums (or null)
    bool diag_noload;   // WC_DIAG_NOLOAD=1: timing-only flat build (wrong results)
    int variant = 0;    // WC_VARIANT: experimental kernel variants (A/B tuning)
    int seg_rows = 0;   // ragged: 0 = flat kernel, else k_cksum_seg with 2/4/8-row groups
    // k_cksum_seg: minimum chunk fill (in 64ths) for a tile's grouped path,
    // dense tiles | sparse tiles << 8 (65 = never)
    int grp_thr = 65 | (40 << 8);
    int grp_rows = 4; // k_cksum_seg grouped path: rows per ping-pong group (2, 4)
    int flat_pk = 1;  // flat kernel: 16-byte chunks per lane slot (1, or 2 = 32 B per lane)
    int gather = 1; // k_cksum_seg: gathered-stream path for tiles neither dense nor uniform
                    // (0 = flat path, 2 = for dense tiles too: tests)
};

struct Shape {
    int group;  // lanes per packet
    int cpl;    // 16-byte chunk loads per lane per pass
    int unroll; // packets per group per iteration
};

// Group-per-packet kernel: strided, or (a.ragged) the small-batch ragged
// variant over WC_RAGGED_SHAPE_LIST.
hipError_t launch_cksum(const LaunchArgs &a, const Shape &sh, int grid,
                        hipStream_t st);
// Aligned strided batches, one pass per packet (wc_k_lean.hip).
hipError_t launch_lean(const LaunchArgs &a, const Shape &sh, int grid, hipStream_t st);
// Ragged batches: a.seg_rows != 0 -> the segmented-prefix kernel (dense
// tiles; the rest take its flat path), else the chunk-balanced flat kernel
// (rows = 64-chunk rows per ping-pong group: 1, 2 or 4).
hipError_t launch_flat(const LaunchArgs &a, int rows, hipStream_t st);
// The standalone flat kernel (wc_k_flat.hip), behind launch_flat.
hipError_t launch_flat_kernel(const LaunchArgs &a, int rows, hipStream_t st);
hipError_t launch_synth(void *buf, uint64_t nbytes, uint64_t seed, int grid,
                        hipStream_t st);
hipError_t launch_sclk_probe(uint64_t *out, int n, uint64_t interval, hipStream_t st);
// RX verdicts of Ethernet frames [base + offs[i], + flens[i]) (wc_k_rx.hip);
// drops (optional) accumulates the frames the reference's RX path drops.
// mode: kRxEarly (parse, then stream only the checked frames) | kRxHdrT
// (transposed header loads) | kRxSkip (frames the parse rules out leave the
// stream); every mode gives the same verdicts.  `tally` (mapped host memory,
// kRxTallyWords words; ADAPT, with HT and without SKIP): every 64th tile
// stores gen << 16 | frames ruled out << 8 | frames, for the host's choice
// of EARLY or HT for the next launch.
constexpr int kRxEarly = 2, kRxHdrT = 4, kRxSkip = 8, kRxAdapt = 16;
constexpr uint32_t kRxTallyWords = 1024;
hipError_t launch_rx_verdict(const void *base, const uint64_t *offs, const uint16_t *flens,
                             uint64_t n, uint8_t *verdict, uint64_t *drops, bool nt,
                             hipStream_t st, int mode = 0, uint32_t *tally = nullptr,
                             uint32_t gen = 0, int max_grid = 0);

// Resident small-batch server (wc_k_serve.hip).  Host-mapped pinned memory:
// one record per packet, written by the host (seq last), polled / read by the
// server's waves; one result slot per packet, written by the GPU in one
// 8-byte store.  Requests are numbered by seq (never 0 after the first).
constexpr uint32_t kSrvMaxPkts = 1024;  // packets per request
constexpr uint32_t kSrvMaxBytes = 4064; // bytes one packet (frame) may span
constexpr uint32_t kSrvKindRx = 2;      // record kind beside WC_KIND_IP / _PAYLOAD
// Fused TX record: payload_cksum(pkt, len) | ip_cksum(pkt, ip4_hl) << 16 (0
// for IPv6), the two checksums mk_ip4_hdr + udp_tx compute (ip4.c:184-186,
// udp.c:209-213).
constexpr uint32_t kSrvKindFused = 3;
constexpr int kSrvAddrBits = 48;        // the packet count rides above the address
struct alignas(16) SrvRec {
    uint64_t addr; // device address of the packet / frame (< 2^48) | n << 48
    uint32_t info; // len | kind << 16 | stop << 24
    uint32_t seq;  // request number, stored last
};
struct alignas(8) SrvRes {
    uint32_t value; // checksum or RX verdict
    uint32_t seq;   // the request it answers
};
// d_hb: the host's heartbeat word (the latest request number, written before
// every request's records): a wave leaves on its own only after idle_ticks in
// which the heartbeat did not move, so the grid drains as a whole.
hipError_t launch_serve(const SrvRec *d_recs, SrvRes *d_res, const uint32_t *d_hb, uint32_t seq0,
                        int waves, uint64_t idle_ticks, hipStream_t st);

} // namespace wc
