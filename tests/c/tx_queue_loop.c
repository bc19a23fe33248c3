/*
 * tx_queue_loop.c -- the TX batch hook of INTEGRATION.md section 3, compiled
 * and driven the way the reference sends a w_iov_sq.
 *
 * The reference's w_tx walks the queue iov by iov and calls udp_tx on each
 * (/root/reference/lib/src/backend_netmap.c:348-358): udp_tx fills the IP
 * header (mk_ip4_hdr: ip4.c:153-186, IPv4 header checksum ip_cksum(ip, 20)
 * with the field 0; mk_ip6_hdr for IPv6), the UDP header, and -- unless the
 * socket enables UDP zero checksums -- payload_cksum over IP header + UDP
 * datagram with udp->cksum 0 (udp.c:189-220); a full TX ring makes w_tx
 * call w_nic_tx and run udp_tx on the same iov again (backend_netmap.c:
 * 353-356).
 *
 * The hook here splits that loop in two:
 *   1. per queue, build every iov's headers with both checksum fields 0 (what
 *      mk_ip4_hdr / udp_tx write before summing) and gather each packet's
 *      offset in the buffer region (w->mem) and its length -- IP header + UDP
 *      length; for a zero-checksum IPv4 socket just the IP header (its
 *      payload is not summed); a zero-checksum IPv6 packet needs no checksum
 *      at all and stays out of the batch;
 *   2. ONE wc_cksum_ip_udp_host call for the queue, then each result stored
 *      raw (ip->cksum, udp->cksum; 0 stays in udp->cksum for zero-checksum
 *      sockets), then the TX-ring loop: an iov that finds the ring full
 *      forces a w_nic_tx and is placed again WITHOUT recomputing anything --
 *      its checksums are already in its bytes.
 * w_nic_tx here moves the ring's frames onto a "wire": another buffer region,
 * one 2048-B slot per frame.  At the end every wire frame goes through
 * wc_rx_verdict_host, the reference's RX checks: each must be WC_RX_OK, or
 * WC_RX_OK_NO_CKSUM for a zero-checksum socket (or a UDP checksum that came
 * out 0, which the reference also sends as "no checksum").  Every GPU result
 * is compared with the oracle's on the same bytes.
 *
 * Sockets: IPv4, IPv4 with header options (a 24..60-byte header; the
 * reference's mk_ip4_hdr always writes 20 bytes, options cover the general
 * header length), IPv6, and a zero-checksum socket of each family.  Queues of
 * 1 .. 5000 iovs: the resident server, the zero-copy launch and the pipelined
 * path; pass 1 runs on an unregistered (pageable) region.
 *
 *   tx_queue_loop [queues_per_socket] [--oracle-only]
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "warpcore_gpu/wc_cksum.h"
#include "wc_oracle.h"

#define BUF_SIZE 2048
#define RING_SLOTS 64
#define MAX_Q 5000

static uint64_t rng = 0x9E3779B97F4A7C15ull;
static uint32_t rnd(void)
{
    rng ^= rng << 13;
    rng ^= rng >> 7;
    rng ^= rng << 17;
    return (uint32_t)(rng >> 11);
}

static void put16(uint8_t *p, uint16_t v) /* network order (bswap16 stores) */
{
    p[0] = (uint8_t)(v >> 8);
    p[1] = (uint8_t)v;
}

enum { S_V4, S_V4_OPTS, S_V6, S_V4_ZERO, S_V6_ZERO, NSOCK };

struct sock { /* the w_sock fields udp_tx reads */
    int af6, opt_hl, zero_cksum;
    uint8_t laddr[16], raddr[16];
    uint16_t lport, rport;
};

struct iov { /* w_iov: buffer index in w->mem, payload length */
    uint32_t idx;
    uint16_t len;     /* payload bytes (v->len before udp_tx) */
    uint16_t ip_len;  /* IP header + UDP datagram, once the headers are built */
    int in_batch;     /* position in the queue's batch, -1 if not summed */
};

/* mk_eth_hdr + mk_ip4_hdr / mk_ip6_hdr + the UDP header (udp.c:189-207),
 * both checksum fields 0; returns the IP header length. */
static uint32_t build_headers(uint8_t *frame, const struct sock *s, struct iov *v)
{
    uint8_t *ip = frame + 14;
    uint32_t hl;
    memset(frame, 0, 12);
    frame[0] = 0x02; /* locally administered MACs */
    frame[6] = 0x02;
    frame[5] = (uint8_t)rnd();
    frame[11] = (uint8_t)rnd();
    if (s->af6) {
        put16(frame + 12, 0x86DD);
        hl = 40;
        ip[0] = 0x60;
        ip[1] = (uint8_t)(rnd() & 0x0F); /* traffic class / flow label */
        ip[2] = (uint8_t)rnd();
        ip[3] = (uint8_t)rnd();
        put16(ip + 4, (uint16_t)(8 + v->len)); /* payload length */
        ip[6] = 17;                            /* next header UDP */
        ip[7] = 0xff;                          /* hop limit */
        memcpy(ip + 8, s->laddr, 16);
        memcpy(ip + 24, s->raddr, 16);
    } else {
        put16(frame + 12, 0x0800);
        hl = 20 + (uint32_t)s->opt_hl;
        ip[0] = (uint8_t)(0x40 | (hl >> 2));
        ip[1] = (uint8_t)(rnd() & 0xFC);
        put16(ip + 2, (uint16_t)(hl + 8 + v->len));
        ip[4] = (uint8_t)rnd(); /* id: random (ip4.c:167) */
        ip[5] = (uint8_t)rnd();
        ip[6] = 0x40; /* IP4_DF */
        ip[7] = 0x00;
        ip[8] = 0xff; /* ttl */
        ip[9] = 17;
        ip[10] = ip[11] = 0; /* ip->cksum = 0 before summing (ip4.c:185) */
        memcpy(ip + 12, s->laddr, 4);
        memcpy(ip + 16, s->raddr, 4);
        for (uint32_t i = 20; i < hl; i++)
            ip[i] = i + 1 == hl ? 0x00 : 0x01; /* NOPs, then end of options */
    }
    uint8_t *udp = ip + hl;
    put16(udp, s->lport);
    put16(udp + 2, s->rport);
    put16(udp + 4, (uint16_t)(8 + v->len));
    udp[6] = udp[7] = 0; /* udp->cksum = 0 (udp.c:208) */
    v->ip_len = (uint16_t)(hl + 8 + v->len);
    return hl;
}

#define FAIL(...)                                                              \
    do {                                                                       \
        printf("tx_queue_loop: FAIL ");                                        \
        printf(__VA_ARGS__);                                                   \
        printf("\n");                                                          \
        return 1;                                                              \
    } while (0)

struct ring { /* a netmap TX ring: frames waiting for w_nic_tx */
    uint32_t idx[RING_SLOTS];
    uint16_t len[RING_SLOTS];
    uint32_t n;
};

struct wire { /* what w_nic_tx put on the link: one slot per frame */
    uint8_t *mem;
    uint64_t *off;
    uint16_t *len;
    int *sock;
    uint32_t n, cap;
};

/* w_nic_tx: the ring's frames go out (copied onto the wire), the ring empties */
static void nic_tx(struct ring *r, const uint8_t *mem, struct wire *w, int sock)
{
    for (uint32_t i = 0; i < r->n && w->n < w->cap; i++) {
        memcpy(w->mem + (uint64_t)w->n * BUF_SIZE, mem + (uint64_t)r->idx[i] * BUF_SIZE, r->len[i]);
        w->off[w->n] = (uint64_t)w->n * BUF_SIZE;
        w->len[w->n] = r->len[i];
        w->sock[w->n] = sock;
        w->n++;
    }
    r->n = 0;
}

int main(int argc, char **argv)
{
    const int queues = argc > 1 ? atoi(argv[1]) : 3;
    const int oracle_only = argc > 2 && !strcmp(argv[2], "--oracle-only");
    const uint32_t nbufs = MAX_Q + 64;
    const uint64_t mem_size = (uint64_t)nbufs * BUF_SIZE;
    uint8_t *mem = aligned_alloc(4096, mem_size); /* w->mem */
    uint32_t *free_idx = malloc(nbufs * sizeof *free_idx);
    struct iov *q = malloc(MAX_Q * sizeof *q);
    uint64_t *off = malloc(MAX_Q * sizeof *off);
    uint16_t *len = malloc(MAX_Q * sizeof *len);
    uint16_t *hdr = malloc(MAX_Q * sizeof *hdr), *pay = malloc(MAX_Q * sizeof *pay);
    const uint32_t wire_cap = 2 * NSOCK * (uint32_t)queues * MAX_Q;
    struct wire w = {aligned_alloc(4096, (uint64_t)wire_cap * BUF_SIZE),
                     malloc(wire_cap * sizeof(uint64_t)), malloc(wire_cap * sizeof(uint16_t)),
                     malloc(wire_cap * sizeof(int)), 0, wire_cap};
    uint8_t *verdict = malloc(wire_cap);
    if (!mem || !free_idx || !q || !off || !len || !hdr || !pay || !w.mem || !w.off || !w.len ||
        !w.sock || !verdict)
        FAIL("alloc");
    memset(mem, 0, mem_size);
    for (uint32_t i = 0; i < nbufs; i++)
        free_idx[i] = i;

    struct sock socks[NSOCK];
    for (int k = 0; k < NSOCK; k++) {
        struct sock *s = &socks[k];
        s->af6 = k == S_V6 || k == S_V6_ZERO;
        s->opt_hl = k == S_V4_OPTS ? 4 * (1 + (int)(rnd() % 10)) : 0;
        s->zero_cksum = k == S_V4_ZERO || k == S_V6_ZERO;
        for (int i = 0; i < 16; i++) {
            s->laddr[i] = (uint8_t)rnd();
            s->raddr[i] = (uint8_t)rnd();
        }
        s->lport = (uint16_t)rnd();
        s->rport = (uint16_t)rnd();
    }
    static const uint32_t qlen[] = {1, 7, 64, 200, 1000, 5000};
    const int nq = (int)(sizeof qlen / sizeof qlen[0]);

    uint64_t calls = 0, retries = 0, pkts = 0, summed = 0, path_pass[2] = {0, 0};
    for (int pass = 0; pass < 2; pass++) {
        /* pass 0: w->mem registered (server / zero-copy / DMA); pass 1 pageable */
        if (!oracle_only && pass == 0 && wc_host_register(mem, mem_size) != WC_OK)
            FAIL("wc_host_register");
        if (!oracle_only && pass == 1 && wc_host_unregister(mem) != WC_OK)
            FAIL("wc_host_unregister");
        for (int qi = 0; qi < queues; qi++)
            for (int k = 0; k < NSOCK; k++) {
                const struct sock *s = &socks[k];
                const uint32_t n = qlen[(qi + k + pass) % nq];
                /* w_alloc: buffers in scrambled order */
                for (uint32_t i = nbufs - 1; i > 0; i--) {
                    const uint32_t j = rnd() % (i + 1), t = free_idx[i];
                    free_idx[i] = free_idx[j];
                    free_idx[j] = t;
                }
                /* the application's payloads */
                for (uint32_t i = 0; i < n; i++) {
                    q[i].idx = free_idx[i];
                    const uint32_t room = BUF_SIZE - 14 - (s->af6 ? 40 : 20 + s->opt_hl) - 8;
                    q[i].len = (uint16_t)(rnd() % 5 == 0 ? rnd() % 16 : rnd() % (room + 1));
                    uint8_t *pl = mem + (uint64_t)q[i].idx * BUF_SIZE + 14 +
                                  (s->af6 ? 40 : 20 + s->opt_hl) + 8;
                    for (uint32_t b = 0; b < q[i].len; b++)
                        pl[b] = (uint8_t)rnd();
                }
                /* 1. headers for the whole queue, then one batch */
                uint32_t m = 0;
                for (uint32_t i = 0; i < n; i++) {
                    uint8_t *frame = mem + (uint64_t)q[i].idx * BUF_SIZE;
                    const uint32_t hl = build_headers(frame, s, &q[i]);
                    q[i].in_batch = -1;
                    if (s->zero_cksum && s->af6)
                        continue; /* no header checksum, no UDP checksum */
                    q[i].in_batch = (int)m;
                    off[m] = (uint64_t)q[i].idx * BUF_SIZE + 14;
                    len[m] = s->zero_cksum ? (uint16_t)hl : q[i].ip_len;
                    m++;
                }
                if (!oracle_only && m) {
                    const int rc = wc_cksum_ip_udp_host(mem, mem_size, off, len, m, hdr, pay);
                    if (rc != WC_OK)
                        FAIL("wc_cksum_ip_udp_host: %s (%d)", wc_strerror(rc), rc);
                    ++calls;
                }
                /* check against the oracle on the bytes as built, then store raw */
                for (uint32_t i = 0; i < n; i++) {
                    if (q[i].in_batch < 0)
                        continue;
                    uint8_t *ip = mem + (uint64_t)q[i].idx * BUF_SIZE + 14;
                    const uint32_t hl = s->af6 ? 40 : (uint32_t)(ip[0] & 15) * 4;
                    const uint32_t b = (uint32_t)q[i].in_batch;
                    const uint16_t oh = s->af6 ? 0 : oracle_ip_cksum(ip, (uint16_t)hl);
                    const uint16_t op = oracle_payload_cksum(ip, len[b]);
                    if (oracle_only) {
                        hdr[b] = oh;
                        pay[b] = op;
                    } else if (hdr[b] != oh || (!s->zero_cksum && pay[b] != op)) {
                        FAIL("sock %d queue %u iov %u: gpu %04x/%04x oracle %04x/%04x", k, n, i,
                             hdr[b], pay[b], oh, op);
                    }
                    if (!s->af6)
                        memcpy(ip + 10, &hdr[b], 2); /* ip->cksum (ip4.c:186) */
                    if (!s->zero_cksum)
                        memcpy(ip + hl + 6, &pay[b], 2); /* udp->cksum (udp.c:213) */
                    ++summed;
                }
                /* 2. w_tx: into the TX ring; a full ring forces w_nic_tx and
                 * the same iov is placed again, its checksums already stored */
                struct ring r = {.n = 0};
                for (uint32_t i = 0; i < n; i++) {
                    while (r.n == RING_SLOTS) {
                        nic_tx(&r, mem, &w, k);
                        ++retries;
                    }
                    r.idx[r.n] = q[i].idx;
                    r.len[r.n] = (uint16_t)(14 + q[i].ip_len);
                    r.n++;
                }
                nic_tx(&r, mem, &w, k);
                pkts += n;
                path_pass[pass] += m;
            }
    }
    if (w.n != pkts)
        FAIL("wire holds %u frames for %llu sent", w.n, (unsigned long long)pkts);
    /* the receiver: the reference's RX checks on every frame */
    uint64_t drops = 0;
    if (!oracle_only) {
        if (wc_host_register(w.mem, (uint64_t)w.n * BUF_SIZE) != WC_OK)
            FAIL("wc_host_register wire");
        const int rc = wc_rx_verdict_host(w.mem, (uint64_t)w.n * BUF_SIZE, w.off, w.len, w.n,
                                          verdict, &drops);
        wc_host_unregister(w.mem);
        if (rc != WC_OK)
            FAIL("wc_rx_verdict_host: %s (%d)", wc_strerror(rc), rc);
    }
    uint64_t no_cksum = 0;
    for (uint32_t i = 0; i < w.n; i++) {
        const uint8_t *fr = w.mem + w.off[i];
        const int orc = oracle_rx_verdict(fr, w.len[i]);
        const int v = oracle_only ? orc : verdict[i];
        const int zero = socks[w.sock[i]].zero_cksum;
        const uint32_t hl = socks[w.sock[i]].af6 ? 40 : (uint32_t)(fr[14] & 15) * 4;
        const int field0 = fr[14 + hl + 6] == 0 && fr[14 + hl + 7] == 0;
        const int want = zero || field0 ? WC_RX_OK_NO_CKSUM : WC_RX_OK;
        if (v != orc || v != want)
            FAIL("wire frame %u (sock %d): gpu %d oracle %d expected %d", i, w.sock[i], v, orc,
                 want);
        no_cksum += v == WC_RX_OK_NO_CKSUM;
    }
    if (!oracle_only) {
        uint64_t served = 0, fallbacks = 0, launches = 0;
        wc_server_stats(&served, &fallbacks, &launches);
        if (fallbacks)
            FAIL("the resident server fell back %llu times", (unsigned long long)fallbacks);
        if (!served)
            FAIL("no batch was answered by the resident server");
        wc_gpu_fini();
        printf("tx_queue_loop: ok (%llu iovs in %llu batch calls, %llu checksummed, %llu ring-full "
               "retries without recomputing, %u frames verified on the wire, %llu without UDP "
               "checksum, %llu drops; server answered %llu batches)\n",
               (unsigned long long)pkts, (unsigned long long)calls, (unsigned long long)summed,
               (unsigned long long)retries, w.n, (unsigned long long)no_cksum,
               (unsigned long long)drops, (unsigned long long)served);
    } else {
        printf("tx_queue_loop: oracle-only ok (%llu iovs, %u frames)\n", (unsigned long long)pkts,
               w.n);
    }
    if (drops)
        FAIL("%llu frames dropped", (unsigned long long)drops);
    return 0;
}
