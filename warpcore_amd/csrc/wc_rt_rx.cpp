// wc_rt_rx.cpp -- RX verdict launches (wc_rx_verdict_ragged and the host
// paths' RX batches): the default ADAPT mode picks EARLY or HT per launch
// from the tallies earlier launches' tiles stored.

#include "wc_rt.h"

#include <algorithm>
#include <cstdio>
#include <cstring>

namespace wc {
namespace rt __attribute__((visibility("hidden"))) {

std::mutex g_rx_mu;

// One RX verdict launch.  ADAPT (the default): EARLY or HT by the newest
// earlier launch on this device whose tally has arrived (>= 8 sampled tiles,
// or all it will write): EARLY when more than 1 in 8 of its sampled frames
// needed no UDP check (ARP / ICMP / TCP / zero checksums / drops), else HT;
// the previous choice stands until a tally arrives.  The kernel's tally is a
// store per 64 tiles into mapped host memory -- nothing to wait for here,
// and launches stay asynchronous (a tally read while its launch still runs
// is a partial sample).
hipError_t rx_launch(Device &D, const Config &C, const void *base, const uint64_t *offs,
                     const uint16_t *flens, uint64_t n, uint8_t *verdict, uint64_t *drops,
                     hipStream_t st)
{
    const int mode = C.rx_mode();
    if (!(mode & wc::kRxAdapt))
        return wc::launch_rx_verdict(base, offs, flens, n, verdict, drops, C.nt != 0, st, mode,
                                     nullptr, 0u, C.rx_grid);
    // (wc_gpu_fini frees the tallies under this lock too: test them inside it)
    std::lock_guard<std::mutex> lk(g_rx_mu);
    if (!D.h_rx_tally[0])
        return wc::launch_rx_verdict(base, offs, flens, n, verdict, drops, C.nt != 0, st,
                                     wc::kRxHdrT, nullptr, 0u, C.rx_grid);
    const auto t0 = std::chrono::steady_clock::now();
    uint32_t from = 0, from_words = 0, from_seen = 0, from_out = 0;
    for (uint32_t back = 1; back < (uint32_t)kRxSets && back <= D.rx_gen; ++back) {
        const uint32_t g = D.rx_gen - back;
        const int set = (int)(g % kRxSets);
        const volatile uint32_t *t = D.h_rx_tally[set];
        uint32_t words = 0, seen = 0, out = 0;
        for (uint32_t i = 0; i < D.rx_words[set]; ++i) {
            const uint32_t w = t[i];
            if ((w >> 16) != (g & 0xFFFFu))
                continue;
            ++words;
            seen += w & 0xFFu;
            out += (w >> 8) & 0xFFu;
        }
        if (words >= 8 || (words && words == D.rx_words[set])) {
            D.rx_early = out * 8u > seen;
            from = g;
            from_words = words;
            from_seen = seen;
            from_out = out;
            break;
        }
    }
    const uint32_t g = ++D.rx_gen;
    const int set = (int)(g % kRxSets);
    const uint64_t tiles = (n + 63) / 64;
    const uint32_t words = (uint32_t)std::min<uint64_t>((tiles + 63) / 64, wc::kRxTallyWords);
    // cleared first: a word older launches left there could carry this
    // launch's 16-bit tag once the tags come round (a late store of launch
    // g - 4 after the clear carries g - 4's tag and is not counted).  The
    // cleared words carry a tag no launch of this set can have -- g's
    // complement, never g's own (a plain 0 is launch g's tag whenever
    // g & 0xFFFF == 0, and its words would count as arrived, empty).
    const uint32_t cleared = ((~g) & 0xFFFFu) << 16;
    for (uint32_t i = 0; i < words; ++i)
        D.h_rx_tally[set][i] = cleared;
    D.rx_words[set] = words;
    if (C.rx_force) // (tools: the tallying kernel with the decision fixed)
        D.rx_early = C.rx_force == 2;
    const int m = wc::kRxHdrT | (D.rx_early ? wc::kRxEarly : 0);
    if (C.rx_trace == 2) { // one summary line per 512 launches
        ++D.rx_nlaunch[D.rx_early ? 1 : 0];
        D.rx_ndecided += from_words != 0;
        if ((g & 511u) == 0) {
            fprintf(stderr, "wccksum rx gen %u: last 512 launches %u HT / %u EARLY, %u decided "
                            "from an arrived tally\n",
                    g, D.rx_nlaunch[0], D.rx_nlaunch[1], D.rx_ndecided);
            D.rx_nlaunch[0] = D.rx_nlaunch[1] = D.rx_ndecided = 0;
        }
    } else if (C.rx_trace)
        fprintf(stderr, "wccksum rx gen %u: %s (tally of gen %u: %u words, %u of %u frames ruled "
                        "out; %.1f us on the host)\n",
                g, D.rx_early ? "EARLY" : "HT", from, from_words, from_out, from_seen,
                std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0)
                    .count());
    return wc::launch_rx_verdict(base, offs, flens, n, verdict, drops, C.nt != 0, st, m,
                                 D.d_rx_tally[set], g & 0xFFFFu, C.rx_grid);
}

} // namespace rt
} // namespace wc

using namespace wc::rt;

extern "C" {

int wc_rx_verdict_ragged(const void *d_base, const uint64_t *d_off, const uint16_t *d_frame_len,
                         uint64_t n, uint8_t *d_verdict, uint64_t *d_drops, void *stream)
{
    if (n == 0)
        return WC_OK;
    if (!d_base || !d_off || !d_frame_len || !d_verdict)
        return WC_EINVAL;
    Device *D = nullptr;
    Config C;
    int rc = ensure_device(&D, &C);
    if (rc)
        return rc;
    return hip_err(rx_launch(*D, C, d_base, d_off, d_frame_len, n, d_verdict, d_drops,
                             (hipStream_t)stream));
}

} // extern "C"
