/*
 * wc_oracle.c -- TEST INFRASTRUCTURE ONLY (see wc_oracle.h).
 *
 * A plain-C restatement of warpcore's RFC 1071 checksum, written from the
 * behaviour documented in SURVEY.md section 8(a).  It is the parity checker for
 * the HIP kernels and the timed CPU baseline; it is never linked into the
 * product library.
 *
 * Parity: "parity unpinned" against the reference except for the known
 * answers in tests/golden/kat.json (recorded by SURVEY.md/BASELINE.md from the
 * compiled reference object) -- the reference itself is unbuildable here
 * because in_cksum.c needs the CMake-generated <warpcore/config.h>.  The
 * standard arithmetic is also pinned by Linux-kernel-computed checksums
 * (tests/golden/linux_vectors.npz).
 */
#define _GNU_SOURCE
#include "wc_oracle.h"

#include <pthread.h>
#include <string.h>
#include <time.h>

#if !defined(__BYTE_ORDER__) || __BYTE_ORDER__ != __ORDER_LITTLE_ENDIAN__
#error "the reference reads native uint16 words; this restatement assumes LE"
#endif

/* Σ of the buffer read as native (little-endian) 16-bit words, odd trailing
 * byte added as a low byte -- in_cksum.c:107-120.  For len <= 65535 the sum
 * is < 2^32 (32767 * 65535 + 255), so uint32 never wraps here. */
static inline uint32_t le16_word_sum(const uint8_t *p, uint32_t len)
{
    uint32_t acc = 0;
    const uint32_t words = len >> 1;
    for (uint32_t w = 0; w < words; w++) {
        uint16_t v;
        memcpy(&v, p + 2 * (size_t)w, sizeof v); /* unaligned-safe load */
        acc += v;
    }
    if (len & 1u)
        acc += p[len - 1];
    return acc;
}

/* End-around-carry fold, then one's complement -- in_cksum.c:74-80.
 * 0 -> 0xFFFF; any other multiple of 0xFFFF -> 0x0000 (never % 0xFFFF). */
uint16_t oracle_fold(uint32_t sum)
{
    while (sum > 0xFFFFu)
        sum = (sum >> 16) + (sum & 0xFFFFu);
    return (uint16_t)~sum;
}

uint32_t oracle_ip_sum(const void *buf, uint16_t len)
{
    return le16_word_sum((const uint8_t *)buf, len);
}

uint16_t oracle_ip_cksum(const void *buf, uint16_t len)
{
    return oracle_fold(oracle_ip_sum(buf, len)); /* in_cksum.c:133-137 */
}

/* payload_cksum accumulator -- in_cksum.c:140-164.  `buf` points at the IP
 * header; version from the high nibble of byte 0 (ip4.h:75-79).  Any version
 * other than 4 takes the IPv6 branch, as the reference does. */
uint32_t oracle_payload_sum(const void *buf, uint16_t len)
{
    const uint8_t *ip = (const uint8_t *)buf;
    uint32_t hl;
    uint32_t acc;

    if ((ip[0] >> 4) == 4) {
        hl = (uint32_t)(ip[0] & 0x0Fu) * 4u;              /* ip4.h:88-92 */
        acc = (uint32_t)ip[9] << 8;                        /* proto, byte 9 */
        acc += le16_word_sum(ip + 12, 4);                  /* src @12 */
        acc += le16_word_sum(ip + 16, 4);                  /* dst @16 */
        /* total length @2 (network order) minus header length, truncated to
         * 16 bits, put back in network order and read as a native word. */
        const uint16_t tot = (uint16_t)((ip[2] << 8) | ip[3]);
        const uint16_t plen = (uint16_t)(tot - hl);
        uint8_t be[2] = {(uint8_t)(plen >> 8), (uint8_t)plen};
        acc += le16_word_sum(be, 2);
    } else {
        hl = 40;                                           /* sizeof ip6_hdr */
        acc = (uint32_t)ip[6] << 24;                       /* next_hdr @6 */
        acc += le16_word_sum(ip + 8, 16);                  /* src @8 */
        acc += le16_word_sum(ip + 24, 16);                 /* dst @24 */
        acc += le16_word_sum(ip + 4, 2);                   /* payload len @4 */
    }
    /* (len - hl) is converted to uint32 by the reference; len < hl would read
     * ~4 GiB past the buffer there, so callers must pass len >= hl. */
    acc += le16_word_sum(ip + hl, (uint32_t)len - hl);     /* wraps mod 2^32 */
    return acc;
}

uint16_t oracle_payload_cksum(const void *buf, uint16_t len)
{
    return oracle_fold(oracle_payload_sum(buf, len));
}

/* ------------------------------------------------------------------------- */
/* Batch drivers (pthreads over contiguous packet shards).                   */

struct shard {
    const uint8_t *base;
    const uint64_t *off;
    const uint16_t *lens;
    uint64_t stride;
    uint16_t len;
    uint64_t lo, hi;
    uint16_t *out;
    int kind;
};

static void *run_shard(void *arg)
{
    const struct shard *s = arg;
    for (uint64_t i = s->lo; i < s->hi; i++) {
        const uint8_t *p = s->off ? s->base + s->off[i] : s->base + i * s->stride;
        const uint16_t l = s->lens ? s->lens[i] : s->len;
        s->out[i] = s->kind == ORACLE_KIND_PAYLOAD ? oracle_payload_cksum(p, l)
                                                   : oracle_ip_cksum(p, l);
    }
    return NULL;
}

static void run_batch(struct shard proto, uint64_t n, int threads)
{
    if (threads < 1)
        threads = 1;
    if ((uint64_t)threads > n)
        threads = n ? (int)n : 1;
    if (threads > 256)
        threads = 256;
    pthread_t tid[256];
    struct shard sh[256];
    for (int t = 0; t < threads; t++) {
        sh[t] = proto;
        sh[t].lo = n * (uint64_t)t / (uint64_t)threads;
        sh[t].hi = n * (uint64_t)(t + 1) / (uint64_t)threads;
    }
    if (threads == 1) {
        run_shard(&sh[0]);
        return;
    }
    for (int t = 0; t < threads; t++)
        pthread_create(&tid[t], NULL, run_shard, &sh[t]);
    for (int t = 0; t < threads; t++)
        pthread_join(tid[t], NULL);
}

void oracle_cksum_strided(const uint8_t *base, uint64_t stride, uint16_t len,
                          uint64_t n, uint16_t *out, int kind, int threads)
{
    struct shard p = {.base = base, .stride = stride, .len = len, .out = out,
                      .kind = kind};
    run_batch(p, n, threads);
}

void oracle_cksum_ragged(const uint8_t *base, const uint64_t *off,
                         const uint16_t *len, uint64_t n, uint16_t *out,
                         int kind, int threads)
{
    struct shard p = {.base = base, .off = off, .lens = len, .out = out,
                      .kind = kind};
    run_batch(p, n, threads);
}

/* ------------------------------------------------------------------------- */
/* RX verdict (the checksum and format decisions of the reference's RX path). */

enum {
    RX_OK = 0, RX_OK_NO_CKSUM = 1, RX_BAD_IP_CKSUM = 2, RX_BAD_UDP_CKSUM = 3,
    RX_SHORT = 4, RX_FRAGMENT = 5, RX_BAD_VERSION = 6, RX_NOT_UDP = 7, RX_NOT_IP = 8,
    RX_TRUNCATED = 9,
};

static inline uint16_t be16_at(const uint8_t *p) { return (uint16_t)((p[0] << 8) | p[1]); }

int oracle_rx_verdict(const uint8_t *f, uint16_t flen)
{
    /* eth_rx (eth.c:75-86): dispatch on the EtherType @12 (eth.h:44-53). */
    if (flen < 14)
        return RX_TRUNCATED;
    const uint16_t type = be16_at(f + 12);
    if (type != 0x0800 && type != 0x86DD)
        return RX_NOT_IP; /* ARP and the rest: the engine's business */
    const uint8_t *ip = f + 14;
    const uint32_t room = (uint32_t)flen - 14; /* IP bytes inside the frame */
    if (room < 1)
        return RX_TRUNCATED;
    const int v4 = type == 0x0800;
    /* ip4_rx / ip6_rx: version nibble (ip4.c:95-98, ip6.c:91-95, ip4.h:75-79) */
    if ((ip[0] >> 4) != (v4 ? 4 : 6))
        return RX_BAD_VERSION;
    uint32_t hl, ip_plen, proto;
    if (v4) {
        hl = (uint32_t)(ip[0] & 0x0Fu) * 4u; /* ip4_hl, ip4.h:88-92 */
        /* ip4_rx and udp_rx read the fixed header (len @2, off @6, p @9,
         * src/dst @12..19) and ip_cksum reads [0, hl). */
        if (room < (hl > 20 ? hl : 20))
            return RX_TRUNCATED;
        if (oracle_ip_cksum(ip, (uint16_t)hl) != 0) /* ip4.c:110-115 */
            return RX_BAD_IP_CKSUM;
        /* ip->off & IP4_OFFMASK (0xff1f in network order, ip4.h:49): the
         * 13-bit fragment offset; the MF flag alone passes (ip4.c:123-127). */
        if ((ip[6] & 0x1Fu) || ip[7])
            return RX_FRAGMENT;
        proto = ip[9];
        /* udp.c:104: uint16 arithmetic, wraps when len < hl */
        ip_plen = (uint16_t)(be16_at(ip + 2) - hl);
    } else {
        hl = 40; /* sizeof(struct ip6_hdr), udp.c:113 */
        if (room < 40)
            return RX_TRUNCATED;
        proto = ip[6];          /* next_hdr, ip6.c:105 */
        ip_plen = be16_at(ip + 4); /* udp.c:114 */
    }
    if (proto != 17) /* IP_P_UDP: ICMP and the rest go elsewhere */
        return RX_NOT_UDP;
    if (ip_plen < 8) /* udp.c:123-126 */
        return RX_SHORT;
    if (room < hl + 8) /* the UDP header (udp.h:41-46) at ip + hl */
        return RX_TRUNCATED;
    const uint8_t *udp = ip + hl;
    const uint32_t ulen = be16_at(udp + 4);
    const uint32_t udp_len = ulen < ip_plen ? ulen : ip_plen; /* udp.c:128 */
    if (udp[6] == 0 && udp[7] == 0) /* udp.c:132: no checksum, accepted */
        return RX_OK_NO_CKSUM;
    /* payload_cksum(ip, udp_len + hl) reads [0, max(len, 20)) -- the length
     * is passed as a uint16, and any value past 65535 would wrap below hl
     * (a ~4 GiB read in the reference): both are past the frame here. */
    const uint32_t plen = udp_len + hl;
    if (room < (plen > 20 ? plen : 20))
        return RX_TRUNCATED;
    return oracle_payload_cksum(ip, (uint16_t)plen) != 0 ? RX_BAD_UDP_CKSUM : RX_OK;
}

struct rx_shard {
    const uint8_t *base;
    const uint64_t *off;
    const uint16_t *flen;
    uint64_t lo, hi;
    uint8_t *out;
};

static void *run_rx_shard(void *arg)
{
    const struct rx_shard *s = arg;
    for (uint64_t i = s->lo; i < s->hi; i++)
        s->out[i] = (uint8_t)oracle_rx_verdict(s->base + s->off[i], s->flen[i]);
    return NULL;
}

void oracle_rx_verdict_ragged(const uint8_t *base, const uint64_t *off, const uint16_t *flen,
                              uint64_t n, uint8_t *out, int threads)
{
    if (threads < 1)
        threads = 1;
    if ((uint64_t)threads > n)
        threads = n ? (int)n : 1;
    if (threads > 256)
        threads = 256;
    pthread_t tid[256];
    struct rx_shard sh[256];
    for (int t = 0; t < threads; t++) {
        sh[t] = (struct rx_shard){base, off, flen, n * (uint64_t)t / (uint64_t)threads,
                                  n * (uint64_t)(t + 1) / (uint64_t)threads, out};
        if (threads > 1)
            pthread_create(&tid[t], NULL, run_rx_shard, &sh[t]);
    }
    if (threads == 1) {
        run_rx_shard(&sh[0]);
        return;
    }
    for (int t = 0; t < threads; t++)
        pthread_join(tid[t], NULL);
}

static double now_s(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC_RAW, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

double oracle_bench_strided(const uint8_t *base, uint64_t stride, uint16_t len,
                            uint64_t n, uint16_t *out, int kind, int threads,
                            double min_seconds, uint64_t *passes)
{
    uint64_t k = 0;
    const double t0 = now_s();
    double t1;
    do {
        oracle_cksum_strided(base, stride, len, n, out, kind, threads);
        k++;
        t1 = now_s();
    } while (t1 - t0 < min_seconds);
    if (passes)
        *passes = k;
    return (double)k * (double)n * (double)len / (t1 - t0);
}

/* ------------------------------------------------------------------------- */

static inline uint64_t splitmix64_at(uint64_t seed, uint64_t k)
{
    uint64_t z = seed + (k + 1) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

void oracle_synth_fill(uint8_t *buf, uint64_t nbytes, uint64_t seed)
{
    const uint64_t words = nbytes / 8;
    for (uint64_t k = 0; k < words; k++) {
        const uint64_t v = splitmix64_at(seed, k);
        memcpy(buf + 8 * k, &v, 8);
    }
    if (nbytes % 8) {
        const uint64_t v = splitmix64_at(seed, words);
        memcpy(buf + 8 * words, &v, nbytes % 8);
    }
}
