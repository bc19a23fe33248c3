/*
 * wc_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of warpcore's Internet / UDP checksum (RFC 1071) used as the
 * parity checker for the MI355X HIP path and as the timed CPU baseline
 * (`cpu_baseline.kind = "port"` in bench.py).  Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load this library.  The product library
 * (warpcore_amd/libwccksum.so) never links or calls it.
 *
 * Reference being restated (read as text, never copied):
 *   /root/reference/lib/src/in_cksum.c:74-80    csum_oc16_reduce
 *   /root/reference/lib/src/in_cksum.c:107-120  csum_oc16
 *   /root/reference/lib/src/in_cksum.c:133-137  ip_cksum
 *   /root/reference/lib/src/in_cksum.c:140-167  payload_cksum
 *   /root/reference/lib/src/ip4.h:55-66,75-92   ip4_hdr layout, ip_v, ip4_hl
 *   /root/reference/lib/src/ip6.h:45-57         ip6_hdr layout
 *
 * Parity status: the reference object cannot be built here (in_cksum.c pulls
 * <warpcore/config.h>, which only CMake generates), so this restatement is
 * pinned only by the known answers SURVEY.md / BASELINE.md recorded from the
 * compiled reference (tests/golden/kat.json) and by external RFC examples.
 * Everything else is "parity unpinned" against the reference -- see DESIGN.md
 * section 3.  The standard RFC 1071 arithmetic (word sum, fold, byte order,
 * IPv4 / IPv6 pseudo-headers with next header 17) is additionally pinned by
 * checksums the Linux kernel computed on the same bytes
 * (tests/golden/linux_vectors.npz, make_kernel_vectors.py).
 */
#pragma once

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { ORACLE_KIND_IP = 0, ORACLE_KIND_PAYLOAD = 1 };

/* Exact 32-bit accumulator the reference builds before folding
 * (in_cksum.c:107-120 for ip_cksum; in_cksum.c:142-164 for payload_cksum). */
uint32_t oracle_ip_sum(const void *buf, uint16_t len);
uint32_t oracle_payload_sum(const void *buf, uint16_t len);

/* Fold + complement (in_cksum.c:74-80). */
uint16_t oracle_fold(uint32_t sum);

/* Scalar restatements of ip_cksum / payload_cksum (in_cksum.c:133-167). */
uint16_t oracle_ip_cksum(const void *buf, uint16_t len);
uint16_t oracle_payload_cksum(const void *buf, uint16_t len);

/* Batch drivers: one scalar call per packet, exactly like the reference's
 * per-packet call sites, spread over `threads` pthreads (contiguous shards). */
void oracle_cksum_strided(const uint8_t *base, uint64_t stride, uint16_t len,
                          uint64_t n, uint16_t *out, int kind, int threads);
void oracle_cksum_ragged(const uint8_t *base, const uint64_t *off,
                         const uint16_t *len, uint64_t n, uint16_t *out,
                         int kind, int threads);

/* Timed CPU baseline: repeats oracle_cksum_strided over the batch until at
 * least `min_seconds` have elapsed; returns payload bytes per second and
 * writes the number of passes made to *passes. */
double oracle_bench_strided(const uint8_t *base, uint64_t stride, uint16_t len,
                            uint64_t n, uint16_t *out, int kind, int threads,
                            double min_seconds, uint64_t *passes);

/* RX verdict of one Ethernet frame of `flen` bytes: what the reference's RX
 * path decides from checksums and header format (eth_rx eth.c:52-88 ->
 * ip4_rx ip4.c:87-138 / ip6_rx ip6.c:83-111 -> udp_rx udp.c:80-139), codes
 * as in include/warpcore_gpu/wc_cksum.h (enum wc_rx_verdict).  Reads only
 * bytes [0, flen).  Engine state (MAC / address filters, bound sockets) is
 * the caller's and not part of the verdict. */
int oracle_rx_verdict(const uint8_t *frame, uint16_t flen);
void oracle_rx_verdict_ragged(const uint8_t *base, const uint64_t *off, const uint16_t *flen,
                              uint64_t n, uint8_t *out, int threads);

/* Counter-based synthetic bytes: little-endian 8-byte word k of the stream is
 * splitmix64 output number k for state `seed` (see warpcore_amd synth kernel,
 * which must produce identical bytes). */
void oracle_synth_fill(uint8_t *buf, uint64_t nbytes, uint64_t seed);

#ifdef __cplusplus
}
#endif
