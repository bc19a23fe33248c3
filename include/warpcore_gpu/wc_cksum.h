/*
 * wc_cksum.h -- C ABI of the MI355X (gfx950) Internet / UDP checksum library
 * (libwccksum.so).  Plain C types only; every device-side pointer is a HIP
 * device (or mapped pinned host) address, every `stream` is a hipStream_t
 * passed as void* (NULL = the legacy default stream).
 *
 * Drop-in boundary.  The reference exposes exactly two checksum entry points,
 * declared at /root/reference/lib/src/in_cksum.h:32-36 and defined at
 * /root/reference/lib/src/in_cksum.c:133-167:
 *
 *     uint16_t ip_cksum(const void *buf, uint16_t len);
 *     uint16_t payload_cksum(const void *buf, uint16_t len);
 *
 * This library exports both under the same names and with the same semantics
 * (bit-identical results, no error channel, result stored raw into the
 * packet), computed on the GPU.  Around them it adds the batch entry points
 * the reference's per-packet loops would call at their natural batch points
 * (w_tx's sq_foreach, backend_netmap.c:348-358, and the RX ring drain,
 * backend_netmap.c:379-391); see INTEGRATION.md.
 *
 * Return convention of the int-returning functions: 0 on success, a negative
 * WC_E* code on a caller error, or -(int)hipError_t on a HIP runtime error.
 */
#pragma once

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Which reference function each packet is checksummed with. */
enum wc_cksum_kind {
    WC_CKSUM_IP = 0,      /* ip_cksum(buf, len)       in_cksum.c:133-137 */
    WC_CKSUM_PAYLOAD = 1, /* payload_cksum(buf, len)  in_cksum.c:140-167 */
};

/* Library error codes (HIP errors are returned as -(int)hipError_t, which
 * never collides with these). */
#define WC_OK 0
#define WC_EINVAL (-10001)   /* bad argument (NULL pointer, bad kind, ...) */
#define WC_ENODEV (-10002)   /* no usable gfx950 device */
#define WC_ENOMEM (-10003)   /* scratch / staging allocation failed */
#define WC_ECOMM (-10004)    /* RCCL unavailable or a collective failed */

/* --- drop-in scalar entry points (reference in_cksum.h:32-36) ------------ */

/* Same contract as the reference: `buf` is host memory owned by the caller
 * (a netmap slot or w_iov buffer), read only; the return value is the
 * checksum as a native uint16 whose in-memory bytes are the network-order
 * checksum.  There is no error channel -- like the reference's ensure()/die()
 * (util.h:280-340) an unusable GPU aborts the process with a message. */
uint16_t ip_cksum(const void *buf, uint16_t len);
uint16_t payload_cksum(const void *buf, uint16_t len);

/* --- device-resident batch entry points ---------------------------------- */

/* Packet i occupies [base + i*stride, base + i*stride + len).  Any alignment
 * and any stride (including stride < len, overlapping) is accepted.
 * out[i] receives the checksum of packet i (device memory, n entries). */
int wc_cksum_strided(const void *d_base, uint64_t stride, uint16_t len,
                     uint64_t n, uint16_t *d_out, int kind, void *stream);

/* Packet i occupies [base + d_off[i], base + d_off[i] + d_len[i]) (d_off and
 * d_len are device arrays of n entries).  Any alignment is accepted. */
int wc_cksum_ragged(const void *d_base, const uint64_t *d_off,
                    const uint16_t *d_len, uint64_t n, uint16_t *d_out,
                    int kind, void *stream);

/* RX-side verification (udp.c:132-139, ip4.c:110-115): like the batch calls
 * above, and additionally counts the packets whose checksum is not 0 into
 * *d_bad (a device uint64, accumulated, not reset).  d_out may be NULL. */
int wc_verify_strided(const void *d_base, uint64_t stride, uint16_t len,
                      uint64_t n, uint16_t *d_out, uint64_t *d_bad, int kind,
                      void *stream);
int wc_verify_ragged(const void *d_base, const uint64_t *d_off,
                     const uint16_t *d_len, uint64_t n, uint16_t *d_out,
                     uint64_t *d_bad, int kind, void *stream);

/* Fused IP + UDP pass over IP packets (each at its IP header, len = IP
 * header + UDP length, as payload_cksum takes them): d_out_payload[i] =
 * payload_cksum(pkt, len) and d_out_ip_hdr[i] = ip_cksum(pkt, ip4_hl(pkt[0]))
 * -- the IPv4 header checksum mk_ip4_hdr / ip4_rx compute (ip4.c:184-186,
 * 110-115) -- or 0 for an IPv6 packet, which has no header checksum
 * (ip6.c:83-113).  One read of the packet bytes for both. */
int wc_cksum_ip_udp_strided(const void *d_base, uint64_t stride, uint16_t len,
                            uint64_t n, uint16_t *d_out_ip_hdr,
                            uint16_t *d_out_payload, void *stream);
int wc_cksum_ip_udp_ragged(const void *d_base, const uint64_t *d_off,
                           const uint16_t *d_len, uint64_t n, uint16_t *d_out_ip_hdr,
                           uint16_t *d_out_payload, void *stream);

/* --- RX verdict: the reference's RX checks, decided on the device -------- */

/* What the reference's RX path decides for one Ethernet frame from its
 * checksums and header format: eth_rx (eth.c:75-86) -> ip4_rx
 * (ip4.c:95-138) / ip6_rx (ip6.c:91-111) -> udp_rx (udp.c:99-139).  The
 * checks run in the reference's order; the first that fails names the code.
 * Engine state -- MAC and IP address filters (eth.c:65-73, ip4.c:103-108,
 * ip6.c:98-103), bound sockets -- is not part of the verdict. */
enum wc_rx_verdict {
    WC_RX_OK = 0,            /* UDP, checksum verified (udp.c:134): deliver */
    WC_RX_OK_NO_CKSUM = 1,   /* UDP checksum field 0: accepted unverified (udp.c:132) */
    WC_RX_BAD_IP_CKSUM = 2,  /* ip_cksum(ip, hl) != 0 (ip4.c:110-115): drop */
    WC_RX_BAD_UDP_CKSUM = 3, /* payload_cksum(ip, udp_len + hl) != 0 (udp.c:134-139): drop */
    WC_RX_SHORT = 4,         /* IP payload shorter than a UDP header (udp.c:123-126): drop */
    WC_RX_FRAGMENT = 5,      /* IPv4 fragment offset != 0 (ip4.c:123-127): drop */
    WC_RX_BAD_VERSION = 6,   /* version nibble != the EtherType's (ip4.c:95-98, ip6.c:91-95): drop */
    WC_RX_NOT_UDP = 7,       /* IPv4 / IPv6, another protocol (ICMP, ...): the host's (ip4.c:129-137) */
    WC_RX_NOT_IP = 8,        /* EtherType neither IPv4 nor IPv6 (ARP, ...): the host's (eth.c:75-86) */
    WC_RX_TRUNCATED = 9,     /* a byte the reference reads lies past the frame: drop */
};
#define WC_RX_IS_DROP(v) \
    ((v) != WC_RX_OK && (v) != WC_RX_OK_NO_CKSUM && (v) != WC_RX_NOT_UDP && (v) != WC_RX_NOT_IP)

/* Frame i is the Ethernet frame [d_base + d_off[i], + d_frame_len[i]) -- a
 * netmap slot buffer and its slot length (backend_netmap.c:379-391), or any
 * batch of frames; no header is parsed on the host.  d_verdict[i] receives
 * its enum wc_rx_verdict code (uint8); *d_drops (device uint64, optional,
 * accumulated) counts the frames whose code is a drop (WC_RX_IS_DROP).  No
 * byte outside a frame is read: what the reference would read past the frame
 * (its neighbouring buffers) yields WC_RX_TRUNCATED. */
int wc_rx_verdict_ragged(const void *d_base, const uint64_t *d_off, const uint16_t *d_frame_len,
                         uint64_t n, uint8_t *d_verdict, uint64_t *d_drops, void *stream);

/* Host-memory frames (the netmap buffer area w->mem, ideally registered with
 * wc_host_register): synchronous; *h_drops (optional) = the drop count. */
int wc_rx_verdict_host(const void *h_base, uint64_t h_bytes, const uint64_t *h_off,
                       const uint16_t *h_frame_len, uint64_t n, uint8_t *h_verdict,
                       uint64_t *h_drops);

/* --- host-memory batch (end-to-end: pinned H2D, kernel, D2H) ------------- */

/* Same as wc_cksum_ragged, but every buffer is host memory: packet i is
 * h_len[i] bytes at h_base + h_off[i], inside [h_base, h_base + h_bytes)
 * (WC_EINVAL otherwise), in any order.  Synchronous; results land in h_out.
 *   - Registered region (wc_host_register), up to 256 packets: the resident
 *     server grid answers (no launch); up to 4096 packets and 8 MiB: one
 *     kernel reads the packets in place over PCIe -- the low-latency path for
 *     a socket or ring batch.
 *   - Registered, larger, and sparse (the packets cover < 7/8 of their byte
 *     range: netmap slots) or out of order: kernels read the packets in place,
 *     64 K packets per launch -- only the lines they touch cross the link.
 *   - Otherwise chunks are streamed over several HIP streams with
 *     hipMemcpyAsync: dense ascending offsets ship the byte range a chunk
 *     covers (DMA straight from a registered region), anything else is
 *     gathered packet by packet into the library's pinned staging first. */
int wc_cksum_host(const void *h_base, uint64_t h_bytes, const uint64_t *h_off,
                  const uint16_t *h_len, uint64_t n, uint16_t *h_out, int kind);

/* The fused TX pair over host-memory IP packets (each at its IP header, len =
 * IP header + UDP length, as udp_tx hands them to payload_cksum):
 * h_out_payload[i] = payload_cksum(pkt, len) and h_out_ip_hdr[i] =
 * ip_cksum(pkt, ip4_hl(pkt[0])) for IPv4 (0 for IPv6) -- the two checksums
 * mk_ip4_hdr and udp_tx compute per iov inside w_tx's loop (ip4.c:184-186,
 * udp.c:209-213, backend_netmap.c:348-358), for a whole w_iov_sq in one
 * call, one read of each packet's bytes.  Both fields must hold 0 in the
 * bytes (as the reference zeroes them before summing); store each result
 * raw.  Same paths and rules as wc_cksum_host: a small registered batch is
 * answered by the resident server or one zero-copy launch, anything else is
 * pipelined.  An IPv4 header (hl bytes, options included) must lie inside
 * [h_base, h_base + h_bytes) even where len is shorter: its checksum is
 * defined whatever len is, and every path reads it whole.  len < hl itself is
 * outside payload_cksum's defined inputs (the reference's len - hl wraps to
 * ~4 GiB, in_cksum.c:164): h_out_payload is then unspecified (no byte past
 * the packet's span is read).  Synchronous. */
int wc_cksum_ip_udp_host(const void *h_base, uint64_t h_bytes, const uint64_t *h_off,
                         const uint16_t *h_len, uint64_t n, uint16_t *h_out_ip_hdr,
                         uint16_t *h_out_payload);

/* The resident small-batch server's counters since the process started, over
 * every device (any pointer may be NULL): batches it answered, batches it was
 * asked for but could not answer (they took the launch path instead), and
 * grid launches. */
int wc_server_stats(uint64_t *served, uint64_t *fallbacks, uint64_t *launches);

/* Quiesce the resident server.  While its grid is resident (it stays up while
 * small registered calls keep coming, and for WC_SERVE_IDLE_US -- 20 ms --
 * after the last), a device-wide synchronisation in the same process
 * (hipDeviceSynchronize, torch.cuda.synchronize()) waits for it: under steady
 * small-batch traffic, with no end.  wc_server_pause stops the grid on every
 * device and returns once no wave of it is left; until the matching
 * wc_server_resume, small registered batches take the zero-copy launch
 * instead (the same results, ~10 us more per call).  Pauses nest: the server
 * serves again after as many resumes as pauses.  wc_server_resume without a
 * pause is WC_EINVAL.  Callable from any thread. */
int wc_server_pause(void);
int wc_server_resume(void);

/* Page-lock a host region (e.g. the netmap buffer area w->mem,
 * backend_netmap.c:149-151) so wc_cksum_host can DMA from it directly.
 * Registering the same base again drops the old registration and pins the
 * pages mapped there now, at the new size (if that fails, the old range is
 * pinned again and the error returned).  Call wc_host_unregister before
 * freeing a registered region: a batch over a freed and re-allocated range
 * that was not registered again reads the pages pinned before the free. */
int wc_host_register(void *h_ptr, uint64_t bytes);
int wc_host_unregister(void *h_ptr);

/* --- multi-GPU batches (one host thread, G devices) ----------------------- */

/* The batch shards across the GPUs of one node as an even contiguous split
 * of packet indices: shard g of G holds packets
 * [g*n/G, (g+1)*n/G).  Packets are independent, so no data moves between
 * GPUs during the checksum; RCCL over xGMI is used only to gather the 2-byte
 * results afterwards, if the caller wants them on every device.  Everything
 * below is callable from warpcore's single engine thread (README.md:24-28). */

/* Set up G shard executors, one per device: devices[g], or device g when
 * `devices` is NULL (ngpus <= 0: every visible device).  A device may be
 * listed more than once (shards then share it; rehearsal on fewer GPUs).
 * Creates each device's scratch, streams and pinned staging.  The caller's
 * current device is left unchanged. */
int wc_gpu_init_multi(int ngpus, const int *devices);
/* Number of shard executors set up by wc_gpu_init_multi (0 before). */
int wc_gpu_multi_count(void);

/* The even contiguous split: packets [*lo, *hi) of n go to shard g of G.
 * Pure arithmetic (no GPU); the split every *_multi call uses. */
int wc_shard_range(uint64_t n, int g, int ngpus, uint64_t *lo, uint64_t *hi);

/* wc_cksum_host over the G shard devices: shard g's packets are copied to
 * and checksummed on its own device (its own PCIe link and copy engines),
 * the devices' pipelines interleaved by the calling thread; results land in
 * h_out in packet order.  Synchronous.  A region registered with
 * wc_host_register is DMA'd directly by every device.  A small registered
 * batch (the zero-copy size of wc_cksum_host) runs on shard 0 alone.
 * Before wc_gpu_init_multi this is wc_cksum_host on the current device. */
int wc_cksum_host_multi(const void *h_base, uint64_t h_bytes, const uint64_t *h_off,
                        const uint16_t *h_len, uint64_t n, uint16_t *h_out, int kind);

/* Device-resident shards: shard g (g < wc_gpu_multi_count()) is the batch
 * d_base[g] (+ d_off[g] / d_len[g]) of n[g] packets on shard g's device,
 * results into d_out[g] on that device, enqueued on streams[g] (streams may
 * be NULL: each device's default stream).  Asynchronous, like the
 * single-device calls. */
int wc_cksum_strided_multi(const void *const *d_base, uint64_t stride, uint16_t len,
                           const uint64_t *n, uint16_t *const *d_out, int kind,
                           void *const *streams);
int wc_cksum_ragged_multi(const void *const *d_base, const uint64_t *const *d_off,
                          const uint16_t *const *d_len, const uint64_t *n,
                          uint16_t *const *d_out, int kind, void *const *streams);

/* After the shards: every shard device g receives all Σn results in packet
 * order in d_all[g] (shard h at offset Σ n[<h]) -- RCCL over xGMI, one
 * ncclBroadcast per shard in one group, on communicators the library creates
 * at the first call (ncclCommInitAll over the shard devices, which must be
 * distinct) and frees in wc_gpu_fini.  Enqueued on streams[g]; RCCL is
 * loaded at run time (WC_ECOMM if it is missing). */
int wc_gather_results_multi(uint16_t *const *d_shard_out, const uint64_t *n,
                            uint16_t *const *d_all, void *const *streams);

/* --- library lifetime / introspection ------------------------------------ */

/* Select the HIP device for this thread and create the library's scratch
 * (staging ring, streams).  Called implicitly by every entry point with
 * device -1 ("current device"); calling it explicitly is optional. */
int wc_gpu_init(int device);
/* Release the scratch created by wc_gpu_init / wc_gpu_init_multi and the
 * RCCL communicators.  Page-locks taken with wc_host_register are the
 * caller's and stay until wc_host_unregister.  Every other entry point may
 * be called from any thread at any time, but not while wc_gpu_fini runs:
 * the caller quiesces its engine threads first. */
int wc_gpu_fini(void);

/* The WC_* environment is read once, at the first initialisation.  This
 * (shipped) library reads only the resident server's WC_SERVE (0: off),
 * WC_SERVE_IDLE_US, WC_SERVE_WAVES and WC_SERVE_MAX, and the staging pool's
 * WC_STAGE_THREADS; its kernel shapes and path choices are a compile-time
 * table.  The tuning build (libwccksum_tune.so, -DWC_TUNING) also reads every
 * path knob.  Re-read the environment now. */
int wc_config_reload(void);

/* Counter-based synthetic packet bytes (bench / tests): little-endian 8-byte
 * word k of [d_buf, d_buf + nbytes) is splitmix64 output k for `seed`. */
int wc_synth_fill(void *d_buf, uint64_t nbytes, uint64_t seed, void *stream);

/* Shader-clock probe (bench / tools): one wave on `stream` writes n pairs
 * (100-MHz wall clock, shader clock counter) to d_samples[2 i], [2 i + 1],
 * one pair every `interval` wall-clock ticks, then ends.  Run beside a
 * timed workload on another stream; the ratio of successive deltas x 100 is
 * the shader clock in MHz while it ran. */
int wc_sclk_probe(uint64_t *d_samples, int n, uint64_t interval, void *stream);

/* Kernel-configuration introspection: fills the group width G (lanes per
 * packet), chunk loads per lane and packets per group-iteration the
 * dispatcher picks for a strided batch of `len`-byte packets. */
int wc_plan_strided(uint64_t base_addr, uint64_t stride, uint16_t len,
                    uint64_t n, int kind, int *group, int *chunks_per_lane,
                    int *unroll, int *grid);

/* Which kernel family the dispatcher picks for that strided batch: "lean"
 * (aligned, one pass per packet), "group" (group-per-packet) or "seg"
 * (segmented-prefix stream of a packed batch). */
const char *wc_plan_strided_kernel(uint64_t base_addr, uint64_t stride, uint16_t len,
                                   uint64_t n, int kind);

const char *wc_strerror(int err);
const char *wc_version(void);

#ifdef __cplusplus
}
#endif
