/*
 * sock_verify.c -- SURVEY config 1 (sockping -> sockinetd echo over
 * loopback, 1472-B UDP payloads) with a GPU verification pass on the socket
 * RX path.
 *
 * The reference's socket backend never checksums: w_rx (backend_sock.c:
 * 415-531) recvmmsg()s up to RECV_SIZE = 64 datagrams per call into w_iov
 * buffers carved from one calloc'ed pool (backend_sock.c:145), and sockping
 * (bin/ping.c:217-300) times one payload's round trip through the echo
 * service.  This harness rebuilds that loop in plain C sockets and, after
 * each receive, checksums every received payload with wc_cksum_host (in
 * place, from the registered pool) and compares it with the checksum the
 * sender computed on TX -- the verify pass a libsockcore caller would add.
 * Iterations alternate between "verify off" and "verify on", so the
 * reported RTT medians share one clock and one system state.
 *
 * Test infrastructure: it links the CPU oracle (oracle/wc_oracle.c) to check
 * the GPU results bit-exact on every payload as well.
 *
 * usage: sock_verify [-s len] [-b batch] [-l loops] [-t prefix]
 * prints one JSON line.  With -t, every timed iteration is also written in
 * sockping's TSV format (bin/ping.c:215, 301-302: iface driver mbps byte pkts
 * tx rx, nanoseconds; "lo" / "lo" / UINT32_MAX for the loopback interface,
 * as plat_get_iface_driver / plat_get_mbps report it) to prefix.off.tsv
 * (verify off) and prefix.on.tsv (verify on), so the rows plot with
 * misc/plot.r next to the reference's own.
 */
#define _GNU_SOURCE
#include <arpa/inet.h>
#include <errno.h>
#include <netinet/in.h>
#include <poll.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/socket.h>
#include <time.h>
#include <unistd.h>

#include "warpcore_gpu/wc_cksum.h"
#include "wc_oracle.h"

#define RECV_SIZE 64     /* backend_sock.c:426 */
#define SLOT 2048        /* max_buf_len: MTU-capped buffer (backend_sock.c:139-145) */
#define NSLOTS (4 * RECV_SIZE)

static volatile int g_stop;

static uint64_t now_ns(void)
{
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC_RAW, &t);
    return (uint64_t)t.tv_sec * 1000000000ull + (uint64_t)t.tv_nsec;
}

static uint64_t xorshift(uint64_t *s)
{
    uint64_t x = *s;
    x ^= x << 13;
    x ^= x >> 7;
    x ^= x << 17;
    return *s = x;
}

static int udp_socket(struct sockaddr_in *bound)
{
    int fd = socket(AF_INET, SOCK_DGRAM, 0);
    if (fd < 0)
        return -1;
    int sz = 8 << 20;
    setsockopt(fd, SOL_SOCKET, SO_RCVBUF, &sz, sizeof sz);
    setsockopt(fd, SOL_SOCKET, SO_SNDBUF, &sz, sizeof sz);
    struct sockaddr_in a = {.sin_family = AF_INET, .sin_port = 0};
    a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
    socklen_t al = sizeof a;
    if (bind(fd, (struct sockaddr *)&a, sizeof a) ||
        getsockname(fd, (struct sockaddr *)&a, &al)) {
        close(fd);
        return -1;
    }
    *bound = a;
    return fd;
}

/* The echo service of sockinetd (bin/inetd.c): send every datagram back. */
static void *echo_main(void *arg)
{
    const int fd = *(int *)arg;
    static uint8_t buf[RECV_SIZE][SLOT];
    struct iovec iov[RECV_SIZE];
    struct sockaddr_in sa[RECV_SIZE];
    struct mmsghdr mv[RECV_SIZE];
    while (!g_stop) {
        struct pollfd p = {.fd = fd, .events = POLLIN};
        if (poll(&p, 1, 50) <= 0)
            continue;
        for (int j = 0; j < RECV_SIZE; j++) {
            iov[j] = (struct iovec){.iov_base = buf[j], .iov_len = SLOT};
            mv[j].msg_hdr = (struct msghdr){.msg_name = &sa[j],
                                            .msg_namelen = sizeof sa[j],
                                            .msg_iov = &iov[j],
                                            .msg_iovlen = 1};
        }
        const int n = recvmmsg(fd, mv, RECV_SIZE, MSG_DONTWAIT, 0);
        if (n <= 0)
            continue;
        for (int j = 0; j < n; j++)
            iov[j].iov_len = mv[j].msg_len;
        int sent = 0;
        while (sent < n) {
            const int k = sendmmsg(fd, mv + sent, (unsigned)(n - sent), 0);
            if (k <= 0)
                break;
            sent += k;
        }
    }
    return 0;
}

static int cmp_u64(const void *a, const void *b)
{
    const uint64_t x = *(const uint64_t *)a, y = *(const uint64_t *)b;
    return x < y ? -1 : x > y;
}

static double median(uint64_t *v, int n)
{
    if (n == 0)
        return 0;
    qsort(v, (size_t)n, sizeof *v, cmp_u64);
    return n % 2 ? (double)v[n / 2] : 0.5 * (double)(v[n / 2 - 1] + v[n / 2]);
}

int main(int argc, char **argv)
{
    int len = 1472, batch = 1, loops = 2000, opt;
    const char *tsv = NULL;
    while ((opt = getopt(argc, argv, "s:b:l:t:")) != -1) {
        if (opt == 's')
            len = atoi(optarg);
        else if (opt == 'b')
            batch = atoi(optarg);
        else if (opt == 'l')
            loops = atoi(optarg);
        else if (opt == 't')
            tsv = optarg;
    }
    FILE *tsv_f[2] = {NULL, NULL};
    if (tsv) {
        char path[4096];
        for (int v = 0; v < 2; v++) {
            snprintf(path, sizeof path, "%s.%s.tsv", tsv, v ? "on" : "off");
            tsv_f[v] = fopen(path, "w");
            if (!tsv_f[v]) {
                fprintf(stderr, "sock_verify: cannot write %s\n", path);
                return 2;
            }
            fputs("iface\tdriver\tmbps\tbyte\tpkts\ttx\trx\n", tsv_f[v]); /* ping.c:215 */
        }
    }
    if (len < 0 || len > SLOT - 16 || batch < 1 || batch > RECV_SIZE || loops < 2) {
        fprintf(stderr, "sock_verify: bad arguments\n");
        return 2;
    }

    /* One pool for all w_iov buffers, registered once at engine start. */
    uint8_t *pool = calloc(NSLOTS, SLOT);
    if (!pool || wc_host_register(pool, (uint64_t)NSLOTS * SLOT) != WC_OK) {
        fprintf(stderr, "sock_verify: pool setup failed\n");
        return 1;
    }

    struct sockaddr_in srv_a, cli_a;
    int srv = udp_socket(&srv_a), cli = udp_socket(&cli_a);
    if (srv < 0 || cli < 0 || connect(cli, (struct sockaddr *)&srv_a, sizeof srv_a)) {
        fprintf(stderr, "sock_verify: socket setup failed: %s\n", strerror(errno));
        return 1;
    }
    pthread_t th;
    pthread_create(&th, 0, echo_main, &srv);

    uint64_t *rtt_off = calloc((size_t)loops, 8), *rtt_on = calloc((size_t)loops, 8);
    uint64_t *ver_ns = calloc((size_t)loops, 8);
    int n_off = 0, n_on = 0;
    uint64_t rng = 0x5EEDull, pkts_verified = 0, gpu_mismatch = 0, oracle_mismatch = 0;
    uint64_t lost = 0;
    uint64_t tx_off[RECV_SIZE], rx_off[RECV_SIZE];
    uint16_t tx_len[RECV_SIZE], rx_len[RECV_SIZE], tx_ck[RECV_SIZE], rx_ck[RECV_SIZE];
    int rc = 0;

    for (int it = 0; it < loops; it++) {
        const int verify = it & 1;
        /* TX: fresh payloads in pool slots, checksummed like udp.c:213. */
        for (int j = 0; j < batch; j++) {
            const int s = (it * batch + j) % (NSLOTS / 2); /* TX: lower half */
            tx_off[j] = (uint64_t)s * SLOT;
            tx_len[j] = (uint16_t)len;
            uint8_t *p = pool + tx_off[j];
            for (int k = 0; k < len; k += 8) {
                const uint64_t r = xorshift(&rng);
                memcpy(p + k, &r, (size_t)(len - k < 8 ? len - k : 8));
            }
        }
        if (wc_cksum_host(pool, (uint64_t)NSLOTS * SLOT, tx_off, tx_len,
                          (uint64_t)batch, tx_ck, WC_CKSUM_IP) != WC_OK) {
            rc = 1;
            break;
        }

        struct iovec iov[RECV_SIZE];
        struct mmsghdr mv[RECV_SIZE];
        for (int j = 0; j < batch; j++) {
            iov[j] = (struct iovec){.iov_base = pool + tx_off[j], .iov_len = tx_len[j]};
            mv[j].msg_hdr = (struct msghdr){.msg_iov = &iov[j], .msg_iovlen = 1};
        }
        const uint64_t t0 = now_ns();
        int sent = 0;
        while (sent < batch) {
            const int k = sendmmsg(cli, mv + sent, (unsigned)(batch - sent), 0);
            if (k <= 0)
                break;
            sent += k;
        }
        const uint64_t t_tx = now_ns();

        /* RX: w_rx-style recvmmsg into free slots of the upper half (in
         * reverse pool order, as a free list returns them), until the batch
         * is back or 1 s passes. */
        int got = 0;
        const uint64_t deadline = t0 + 1000000000ull;
        while (got < batch && now_ns() < deadline) {
            for (int j = got; j < batch; j++) {
                const int s = NSLOTS - 1 - ((it * batch + j) % (NSLOTS / 2));
                rx_off[j] = (uint64_t)s * SLOT;
                iov[j] = (struct iovec){.iov_base = pool + rx_off[j], .iov_len = SLOT};
                mv[j].msg_hdr = (struct msghdr){.msg_iov = &iov[j], .msg_iovlen = 1};
            }
            const int k = recvmmsg(cli, mv + got, (unsigned)(batch - got), MSG_DONTWAIT, 0);
            if (k > 0) {
                for (int j = got; j < got + k; j++)
                    rx_len[j] = (uint16_t)mv[j].msg_len;
                got += k;
            }
        }
        if (got < batch)
            lost += (uint64_t)(batch - got);

        /* The verify pass: every received payload, one batch, in place. */
        uint64_t t_v = 0;
        if (verify && got) {
            const uint64_t v0 = now_ns();
            if (wc_cksum_host(pool, (uint64_t)NSLOTS * SLOT, rx_off, rx_len,
                              (uint64_t)got, rx_ck, WC_CKSUM_IP) != WC_OK) {
                rc = 1;
                break;
            }
            t_v = now_ns() - v0;
        }
        const uint64_t t1 = now_ns();
        if (tsv_f[verify]) /* ping.c:301-302: rx is "NA" for a lost round trip */
            fprintf(tsv_f[verify], "lo\tlo\t%u\t%u\t%d\t%llu\t", 0xFFFFFFFFu,
                    got ? (unsigned)rx_len[0] : 0u, got, (unsigned long long)(t_tx - t0));
        if (tsv_f[verify]) {
            if (got == batch)
                fprintf(tsv_f[verify], "%llu\n", (unsigned long long)(t1 - t0));
            else
                fputs("NA\n", tsv_f[verify]);
        }
        if (got < batch)
            continue;
        if (verify) {
            rtt_on[n_on++] = t1 - t0;
            ver_ns[n_on - 1] = t_v;
            /* Loopback keeps order, so the j-th echo is the j-th payload. */
            for (int j = 0; j < got; j++) {
                pkts_verified++;
                gpu_mismatch += rx_len[j] != tx_len[j] || rx_ck[j] != tx_ck[j];
                oracle_mismatch +=
                    rx_ck[j] != oracle_ip_cksum(pool + rx_off[j], rx_len[j]) ||
                    tx_ck[j] != oracle_ip_cksum(pool + tx_off[j], tx_len[j]);
            }
        } else {
            rtt_off[n_off++] = t1 - t0;
        }
    }

    g_stop = 1;
    pthread_join(th, 0);
    close(cli);
    close(srv);
    wc_host_unregister(pool);
    for (int v = 0; v < 2; v++)
        if (tsv_f[v])
            fclose(tsv_f[v]);

    printf("{\"config\": \"sockping->echo loopback\", \"len\": %d, \"batch\": %d, "
           "\"loops\": %d, \"rtt_ns_median_verify_off\": %.0f, "
           "\"rtt_ns_median_verify_on\": %.0f, \"verify_ns_median\": %.0f, "
           "\"packets_verified\": %llu, \"gpu_mismatch\": %llu, "
           "\"oracle_mismatch\": %llu, \"lost\": %llu, \"rc\": %d}\n",
           len, batch, loops, median(rtt_off, n_off), median(rtt_on, n_on),
           median(ver_ns, n_on), (unsigned long long)pkts_verified,
           (unsigned long long)gpu_mismatch, (unsigned long long)oracle_mismatch,
           (unsigned long long)lost, rc);
    return rc || gpu_mismatch || oracle_mismatch || !pkts_verified;
}
