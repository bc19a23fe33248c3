/*
 * rx_ring_loop.c -- the RX batch hook of INTEGRATION.md section 3, compiled
 * and driven the way the reference drains its netmap RX rings.
 *
 * The reference walks every RX ring slot by slot and calls eth_rx per frame
 * (w_nic_rx, /root/reference/lib/src/backend_netmap.c:379-391); its fuzz
 * harness stands up such a ring in memory (test/fuzz.c:46-93).  Here the same
 * shape is built from this program's own netmap-like structs: several rings
 * of slots {buf_idx, len}, buffers in one region (w->mem) in a scrambled
 * buf_idx order, cur/tail wrapping round the ring.  Per ring the hook
 * gathers each pending slot's buffer offset and length, calls
 * wc_rx_verdict_host ONCE, then walks the slots in ring order and branches
 * per slot on WC_RX_IS_DROP: a drop is counted and skipped (the reference's
 * warn + return false), anything else goes to a stand-in for eth_rx.  The
 * ring's head/cur then advance to tail, as nm_ring_next does.  Passes 0 and
 * 2 run on the registered region (zero-copy), pass 1 on pageable memory.
 *
 * Every frame is built to hit one decision of the reference's RX order
 * (eth.c:75-86 -> ip4.c:95-138 / ip6.c:91-111 -> udp.c:99-139): the code it
 * should get is known by construction, and the library's code, the oracle's
 * code (oracle_rx_verdict) and the per-slot deliver / drop branch must all
 * agree with it; the returned drop count must equal the slots dropped.
 *
 *   rx_ring_loop [rings] [slots_per_ring] [--oracle-only]
 *
 * --oracle-only (no GPU needed) checks just the construction: every frame's
 * expected code against oracle_rx_verdict.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <hip/hip_runtime_api.h>

#include "warpcore_gpu/wc_cksum.h"
#include "wc_oracle.h"

#define BUF_SIZE 2048

/* netmap_slot / netmap_ring, the fields w_nic_rx touches (netmap.h) */
struct nm_slot {
    uint32_t buf_idx;
    uint16_t len;
    uint16_t flags;
    uint64_t ptr;
};
struct nm_ring {
    uint32_t num_slots, nr_buf_size;
    uint32_t head, cur, tail;
    struct nm_slot *slot;
};

static uint32_t nm_ring_next(const struct nm_ring *r, uint32_t i)
{
    return i + 1 == r->num_slots ? 0 : i + 1;
}

static uint64_t rng = 0x1234567887654321ull;
static uint32_t rnd(void)
{
    rng ^= rng << 13;
    rng ^= rng >> 7;
    rng ^= rng << 17;
    return (uint32_t)(rng >> 11);
}

static void put16(uint8_t *p, uint16_t v)
{
    p[0] = (uint8_t)(v >> 8);
    p[1] = (uint8_t)v;
}

enum {
    C_OK4, C_OK4_OPTS, C_OK6, C_OK_NO_CKSUM, C_OK_UDPLEN_SHORT, C_OK_MF, C_BAD_UDP,
    C_BAD_UDP6, C_BAD_IP, C_FRAGMENT, C_BAD_VERSION, C_NOT_UDP, C_NOT_UDP6, C_NOT_IP,
    C_SHORT, C_TRUNC_PAYLOAD, C_TRUNC_RUNT, C_TRUNC_HDR, NCASES
};

/* Frame of case `k` at f (room for BUF_SIZE bytes); returns the slot length
 * and the code the reference's checks give it in *want. */
static uint16_t make_frame(uint8_t *f, int k, int *want)
{
    const int v6 = k == C_OK6 || k == C_BAD_UDP6 || k == C_NOT_UDP6;
    const uint32_t hl = v6 ? 40 : (k == C_OK4_OPTS ? 20 + 4 * (1 + rnd() % 10) : 20);
    const uint32_t pay = rnd() % 1400;
    uint32_t ip_len = hl + 8 + pay;
    if (ip_len > BUF_SIZE - 14)
        ip_len = BUF_SIZE - 14;
    for (uint32_t i = 0; i < 14 + ip_len; i++)
        f[i] = (uint8_t)rnd();
    put16(f + 12, v6 ? 0x86DD : 0x0800);
    uint8_t *ip = f + 14;
    uint8_t *udp = ip + hl;
    uint16_t ulen = (uint16_t)(ip_len - hl);
    if (k == C_OK_UDPLEN_SHORT)
        ulen = (uint16_t)(8 + pay / 2); /* udp->len < IP payload (udp.c:128) */
    if (v6) {
        ip[0] = 0x60;
        put16(ip + 4, (uint16_t)(ip_len - 40));
        ip[6] = k == C_NOT_UDP6 ? 58 : 17; /* ICMPv6 / UDP */
    } else {
        ip[0] = (uint8_t)(0x40 | (hl / 4));
        put16(ip + 2, (uint16_t)ip_len);
        ip[6] = k == C_OK_MF ? 0x20 : 0x40; /* MF alone passes; DF */
        ip[7] = 0;
        if (k == C_FRAGMENT) {
            ip[6] = 0x00;
            ip[7] = (uint8_t)(1 + rnd() % 200); /* offset != 0 (ip4.c:123) */
        }
        ip[9] = k == C_NOT_UDP ? 1 : 17;
        if (k == C_SHORT)
            put16(ip + 2, (uint16_t)(hl + rnd() % 8)); /* ip_plen < 8 (udp.c:123) */
        ip[10] = ip[11] = 0;
        const uint16_t hc = oracle_ip_cksum(ip, (uint16_t)hl);
        memcpy(ip + 10, &hc, 2);
    }
    put16(udp + 4, ulen);
    udp[6] = udp[7] = 0;
    if (k != C_OK_NO_CKSUM) {
        /* udp_tx (udp.c:209-213): payload_cksum over hl + udp length */
        uint16_t uc = oracle_payload_cksum(ip, (uint16_t)(hl + ulen));
        if (uc == 0)
            uc = 0xFFFF; /* same class, non-zero field: the check runs */
        memcpy(udp + 6, &uc, 2);
    } else {
        udp[8 + pay / 3] ^= 0x5A; /* not verified (udp.c:132) */
    }
    uint16_t flen = (uint16_t)(14 + ip_len);
    switch (k) {
    case C_BAD_UDP:
    case C_BAD_UDP6:
        udp[2] += 1; /* destination port: inside the summed bytes */
        *want = WC_RX_BAD_UDP_CKSUM;
        break;
    case C_BAD_IP:
        ip[8] += 1; /* TTL, not re-checksummed */
        *want = WC_RX_BAD_IP_CKSUM;
        break;
    case C_FRAGMENT:
        *want = WC_RX_FRAGMENT;
        break;
    case C_BAD_VERSION:
        ip[0] = (uint8_t)(0x60 | (ip[0] & 0x0F)); /* EtherType IPv4, version 6 */
        *want = WC_RX_BAD_VERSION;
        break;
    case C_NOT_UDP:
    case C_NOT_UDP6:
        *want = WC_RX_NOT_UDP;
        break;
    case C_NOT_IP:
        put16(f + 12, 0x0806); /* ARP */
        *want = WC_RX_NOT_IP;
        break;
    case C_SHORT:
        *want = WC_RX_SHORT;
        break;
    case C_TRUNC_PAYLOAD:
        flen = (uint16_t)(14 + hl + 8 + pay / 2); /* slot shorter than the datagram */
        *want = pay > 0 ? WC_RX_TRUNCATED : WC_RX_OK;
        break;
    case C_TRUNC_RUNT:
        flen = (uint16_t)(rnd() % 14); /* no whole Ethernet header */
        *want = WC_RX_TRUNCATED;
        break;
    case C_TRUNC_HDR:
        flen = (uint16_t)(14 + rnd() % 20); /* IPv4 header cut */
        *want = WC_RX_TRUNCATED;
        break;
    case C_OK_NO_CKSUM:
        *want = WC_RX_OK_NO_CKSUM;
        break;
    default:
        *want = WC_RX_OK;
    }
    return flen;
}

#define FAIL(...)                                                              \
    do {                                                                       \
        printf("rx_ring_loop: FAIL ");                                         \
        printf(__VA_ARGS__);                                                   \
        printf("\n");                                                          \
        return 1;                                                              \
    } while (0)

int main(int argc, char **argv)
{
    const uint32_t nrings = argc > 1 ? (uint32_t)atoi(argv[1]) : 4;
    const uint32_t nslots = argc > 2 ? (uint32_t)atoi(argv[2]) : 1024;
    const int oracle_only = argc > 3 && !strcmp(argv[3], "--oracle-only");
    const uint32_t nbufs = nrings * nslots;
    const uint64_t mem_size = (uint64_t)nbufs * BUF_SIZE;
    uint8_t *mem = aligned_alloc(4096, mem_size); /* w->mem: every netmap buffer */
    struct nm_ring *rings = calloc(nrings, sizeof *rings);
    uint32_t *bufs = malloc(nbufs * sizeof *bufs);
    int *want_of_buf = malloc(nbufs * sizeof *want_of_buf);
    uint64_t *off = malloc(nslots * sizeof *off);
    uint16_t *flen = malloc(nslots * sizeof *flen);
    uint8_t *verdict = malloc(nslots);
    if (!mem || !rings || !bufs || !want_of_buf || !off || !flen || !verdict)
        FAIL("alloc");
    /* buffers handed out in scrambled order (zero-copy swaps, netmap) */
    for (uint32_t i = 0; i < nbufs; i++)
        bufs[i] = i;
    for (uint32_t i = nbufs - 1; i > 0; i--) {
        const uint32_t j = rnd() % (i + 1), t = bufs[i];
        bufs[i] = bufs[j];
        bufs[j] = t;
    }
    if (oracle_only) {
        uint64_t seen[NCASES] = {0};
        for (uint32_t i = 0; i < 64u * NCASES * 8u; i++) {
            const int k = (int)(i % NCASES);
            int want = 0;
            const uint16_t fl = make_frame(mem, k, &want);
            const int orc = oracle_rx_verdict(mem, fl);
            if (orc != want)
                FAIL("case %d frame %u: oracle %d expected %d", k, i, orc, want);
            seen[k]++;
        }
        printf("rx_ring_loop: oracle-only ok (%d cases x %llu frames)\n", NCASES,
               (unsigned long long)seen[0]);
        return 0;
    }
    if (wc_host_register(mem, mem_size) != WC_OK)
        FAIL("wc_host_register");

    uint64_t per_case[NCASES] = {0}, slots_seen = 0, dropped_total = 0, delivered_total = 0;
    uint64_t to_udp = 0, to_host = 0;
    for (int pass = 0; pass < 3; pass++) {
        /* pass 1 with the region unregistered: the pipelined (staged) path;
         * passes 0 and 2 registered: the zero-copy path */
        if (pass == 1 && wc_host_unregister(mem) != WC_OK)
            FAIL("wc_host_unregister");
        if (pass == 2 && wc_host_register(mem, mem_size) != WC_OK)
            FAIL("wc_host_register again");
        /* (re)fill: ring r owns buffers [r*nslots, (r+1)*nslots) of bufs[];
         * the pending span [cur, tail) wraps round the ring */
        for (uint32_t r = 0; r < nrings; r++) {
            struct nm_ring *R = &rings[r];
            if (!R->slot) {
                R->slot = calloc(nslots, sizeof *R->slot);
                if (!R->slot)
                    FAIL("alloc slots");
            }
            R->num_slots = nslots;
            R->nr_buf_size = BUF_SIZE;
            R->cur = R->head = rnd() % nslots;
            const uint32_t pending = pass == 2 ? nslots - 1 : 1 + rnd() % (nslots - 1);
            R->tail = (R->cur + pending) % nslots;
            for (uint32_t s = 0; s < nslots; s++) {
                const uint32_t b = bufs[r * nslots + s];
                const int k = (int)(rnd() % NCASES);
                int want = 0;
                R->slot[s].buf_idx = b;
                R->slot[s].len = make_frame(mem + (uint64_t)b * BUF_SIZE, k, &want);
                want_of_buf[b] = want;
                per_case[k] += pass == 0;
            }
        }
        /* w_nic_rx: loop over all rx rings; one verdict batch per ring */
        for (uint32_t r = 0; r < nrings; r++) {
            struct nm_ring *R = &rings[r];
            uint32_t n = 0;
            for (uint32_t c = R->cur; c != R->tail; c = nm_ring_next(R, c), n++) {
                off[n] = (uint64_t)R->slot[c].buf_idx * R->nr_buf_size; /* NETMAP_BUF - w->mem */
                flen[n] = R->slot[c].len;
            }
            uint64_t drops = 0;
            const int rc = wc_rx_verdict_host(mem, mem_size, off, flen, n, verdict, &drops);
            if (rc != WC_OK)
                FAIL("wc_rx_verdict_host: %s (%d)", wc_strerror(rc), rc);
            uint64_t dropped = 0;
            uint32_t q = 0;
            while (R->cur != R->tail) { /* nm_ring_empty(r) is cur == tail */
                const struct nm_slot *sl = &R->slot[R->cur];
                const uint8_t *buf = mem + (uint64_t)sl->buf_idx * R->nr_buf_size;
                const int v = verdict[q];
                const int want = want_of_buf[sl->buf_idx];
                const int orc = oracle_rx_verdict(buf, sl->len);
                if (v != want || orc != want)
                    FAIL("ring %u slot %u (buf %u, len %u): gpu %d oracle %d expected %d", r,
                         R->cur, sl->buf_idx, sl->len, v, orc, want);
                if (WC_RX_IS_DROP(v)) {
                    ++dropped; /* the reference warns and drops (ip4.c:111-115, udp.c:134-139) */
                } else if (v == WC_RX_OK || v == WC_RX_OK_NO_CKSUM) {
                    ++to_udp; /* eth_rx -> ip4_rx / ip6_rx -> udp_rx, checks done */
                } else {
                    ++to_host; /* ARP / ICMP: eth_rx as today */
                }
                R->head = R->cur = nm_ring_next(R, R->cur);
                ++q;
            }
            if (q != n || drops != dropped)
                FAIL("ring %u: %u slots walked for %u verdicts, drops %llu vs %llu", r, q, n,
                     (unsigned long long)drops, (unsigned long long)dropped);
            slots_seen += n;
            dropped_total += dropped;
            delivered_total += n - dropped;
        }
    }
    for (int k = 0; k < NCASES; k++)
        if (!per_case[k])
            FAIL("case %d never generated", k);
    wc_host_unregister(mem);
    wc_gpu_fini();
    printf("rx_ring_loop: ok (%u rings x %u slots, 3 passes: %llu frames, %llu dropped, "
           "%llu to udp_rx, %llu to the host stack)\n",
           nrings, nslots, (unsigned long long)slots_seen, (unsigned long long)dropped_total,
           (unsigned long long)to_udp, (unsigned long long)to_host);
    return 0;
}
