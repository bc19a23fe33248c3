/*
 * host_latency.c -- per-call latency of the host-memory entry points from a
 * C caller (the shape of the reference's batch points: one netmap ring or one
 * w_iov_sq per call, backend_netmap.c:348-358 TX, 379-391 RX), beside the CPU
 * restatement on the same batch (1 core = the reference's own engine thread,
 * and N threads).
 *
 * Packets of L bytes in a pool of 2048-B slots (netmap buffers / the socket
 * backend's pool, backend_sock.c:145), slots picked at random; well-formed
 * Ethernet + IPv4 + UDP frames with valid checksums for the RX verdict.  For
 * n packets and L bytes, one JSON line with the median (and p90) per call of:
 *   srv_us       wc_cksum_host, pool registered, batch answered by the
 *                resident server (no launch, no sync: WC_SERVE=1, n <= 256)
 *   zc_us        wc_cksum_host, pool registered, one zero-copy kernel launch
 *                per call reading the packets in place (WC_SERVE=0)
 *   pipe_us      wc_cksum_host, pool not registered (pinned staging + copies)
 *   rx_srv_us / rx_zc_us   wc_rx_verdict_host, pool registered, server /
 *                launch
 *   floor_us     wc_cksum_strided on 1 device-resident packet + stream sync:
 *                the launch + completion floor, no PCIe data
 *   cpu1_us      oracle_cksum_ragged on the calling thread (the reference's
 *                one engine thread)
 *   cpuN_us      the same batch split over N threads of a PERSISTENT pool
 *                (N - 1 workers spinning on a generation counter, plus the
 *                caller; no thread is created per call): the box's all-core
 *                share as a polling engine would use it
 *   cpu1_rx_us / cpuN_rx_us   oracle_rx_verdict_ragged, 1 thread / the pool
 * Every GPU result is checked against the oracle.
 *
 *   host_latency [threads] [seconds_per_point]
 */
#include <pthread.h>
#include <stdatomic.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include <hip/hip_runtime_api.h>

#include "warpcore_gpu/wc_cksum.h"
#include "wc_oracle.h"

#define SLOT 2048
#define NSLOTS 8192

static double now_us(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec * 1e6 + ts.tv_nsec * 1e-3;
}

static int cmp_d(const void *a, const void *b)
{
    const double x = *(const double *)a, y = *(const double *)b;
    return x < y ? -1 : x > y;
}

static uint64_t rng_state = 0x9E3779B97F4A7C15ull;
static uint64_t rnd(void)
{
    uint64_t z = (rng_state += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

/* Well-formed Ethernet / IPv4 (IHL 5) / UDP frame of ip_len IP bytes at p
 * (eth.h:44-53, ip4.h:55-66, udp.h:41-46), checksums as mk_ip4_hdr / udp_tx
 * compute them (ip4.c:184-186, udp.c:209-213). */
static void make_frame(uint8_t *p, uint16_t ip_len)
{
    for (int i = 0; i < 14 + ip_len; i++)
        p[i] = (uint8_t)rnd();
    p[12] = 0x08;
    p[13] = 0x00;
    uint8_t *ip = p + 14;
    ip[0] = 0x45;
    ip[2] = (uint8_t)(ip_len >> 8);
    ip[3] = (uint8_t)ip_len;
    ip[6] = 0x40; /* DF, offset 0 */
    ip[7] = 0;
    ip[9] = 17;
    ip[10] = ip[11] = 0;
    const uint16_t hc = oracle_ip_cksum(ip, 20);
    memcpy(ip + 10, &hc, 2);
    uint8_t *udp = ip + 20;
    const uint16_t ulen = (uint16_t)(ip_len - 20);
    udp[4] = (uint8_t)(ulen >> 8);
    udp[5] = (uint8_t)ulen;
    udp[6] = udp[7] = 0;
    uint16_t uc = oracle_payload_cksum(ip, ip_len);
    if (uc == 0)
        uc = 0xffff;
    memcpy(udp + 6, &uc, 2);
}

typedef int (*call_fn)(void *ctx);

/* median / p90 microseconds per call over ~`secs` seconds (>= 20 calls) */
static void time_calls(call_fn f, void *ctx, double secs, double *med, double *p90)
{
    enum { MAXS = 200000 };
    static double s[MAXS];
    int k = 0;
    for (int w = 0; w < 5; w++)
        f(ctx);
    const double t_end = now_us() + secs * 1e6;
    while (k < MAXS && (k < 20 || now_us() < t_end)) {
        const double t0 = now_us();
        if (f(ctx) != 0) {
            fprintf(stderr, "call failed\n");
            exit(1);
        }
        s[k++] = now_us() - t0;
    }
    qsort(s, k, sizeof s[0], cmp_d);
    *med = s[k / 2];
    *p90 = s[(k * 9) / 10];
}

struct ctx {
    uint8_t *pool;
    uint64_t *off;
    uint16_t *len, *out;
    uint16_t *flen;
    uint8_t *verdict;
    uint64_t n;
    int threads;
    void *d_pkt;
    uint16_t *d_out;
    hipStream_t st;
};

static int c_host(void *v)
{
    struct ctx *c = v;
    return wc_cksum_host(c->pool, (uint64_t)NSLOTS * SLOT, c->off, c->len, c->n, c->out,
                         WC_CKSUM_IP);
}

static int c_rx(void *v)
{
    struct ctx *c = v;
    uint64_t drops = 0;
    return wc_rx_verdict_host(c->pool, (uint64_t)NSLOTS * SLOT, c->off, c->flen, c->n,
                              c->verdict, &drops);
}

static int c_floor(void *v)
{
    struct ctx *c = v;
    int rc = wc_cksum_strided(c->d_pkt, 64, 64, 1, c->d_out, WC_CKSUM_IP, c->st);
    if (rc == WC_OK)
        rc = hipStreamSynchronize(c->st) == hipSuccess ? WC_OK : -1;
    return rc;
}

static int c_cpu(void *v)
{
    struct ctx *c = v;
    oracle_cksum_ragged(c->pool, c->off, c->len, c->n, c->out, ORACLE_KIND_IP, 1);
    return 0;
}

/* Persistent CPU pool: `parts` - 1 workers spin on `gen` (no sleep, no
 * thread creation per call); a call publishes its batch, bumps gen, takes
 * shard 0 itself and waits for the workers' `done` count. */
static struct {
    int parts;
    pthread_t th[256];
    _Atomic uint64_t gen;
    _Atomic int done, quit;
    struct ctx *job;
    int rx;
} P;

static void pool_shard(int part)
{
    struct ctx *c = P.job;
    const uint64_t lo = c->n * (uint64_t)part / (uint64_t)P.parts;
    const uint64_t hi = c->n * (uint64_t)(part + 1) / (uint64_t)P.parts;
    if (hi <= lo)
        return;
    if (P.rx)
        oracle_rx_verdict_ragged(c->pool, c->off + lo, c->flen + lo, hi - lo, c->verdict + lo, 1);
    else
        oracle_cksum_ragged(c->pool, c->off + lo, c->len + lo, hi - lo, c->out + lo,
                            ORACLE_KIND_IP, 1);
}

static void *pool_worker(void *arg)
{
    const int part = (int)(intptr_t)arg;
    uint64_t seen = 0;
    for (;;) {
        uint64_t g;
        while ((g = atomic_load_explicit(&P.gen, memory_order_acquire)) == seen)
            if (atomic_load_explicit(&P.quit, memory_order_relaxed))
                return NULL;
        seen = g;
        pool_shard(part);
        atomic_fetch_add_explicit(&P.done, 1, memory_order_acq_rel);
    }
}

static void pool_start(int parts)
{
    P.parts = parts < 1 ? 1 : parts > 256 ? 256 : parts;
    atomic_store(&P.quit, 0);
    atomic_store(&P.gen, 0);
    for (int t = 1; t < P.parts; t++)
        pthread_create(&P.th[t], NULL, pool_worker, (void *)(intptr_t)t);
}

static void pool_stop(void)
{
    atomic_store(&P.quit, 1);
    for (int t = 1; t < P.parts; t++)
        pthread_join(P.th[t], NULL);
}

static int pool_call(struct ctx *c, int rx)
{
    P.job = c;
    P.rx = rx;
    atomic_store_explicit(&P.done, 0, memory_order_relaxed);
    atomic_fetch_add_explicit(&P.gen, 1, memory_order_release);
    pool_shard(0);
    while (atomic_load_explicit(&P.done, memory_order_acquire) != P.parts - 1)
        ;
    return 0;
}

static int c_cpu_pool(void *v) { return pool_call(v, 0); }
static int c_cpu_pool_rx(void *v) { return pool_call(v, 1); }

static int c_cpu_rx(void *v)
{
    struct ctx *c = v;
    oracle_rx_verdict_ragged(c->pool, c->off, c->flen, c->n, c->verdict, 1);
    return 0;
}

int main(int argc, char **argv)
{
    const int threads = argc > 1 ? atoi(argv[1]) : 16;
    const double secs = argc > 2 ? atof(argv[2]) : 0.4;
    uint8_t *pool = aligned_alloc(4096, (size_t)NSLOTS * SLOT);
    uint8_t *pool2 = aligned_alloc(4096, (size_t)NSLOTS * SLOT);
    static uint64_t off[NSLOTS];
    static uint16_t len[NSLOTS], flen[NSLOTS], out[NSLOTS], want[NSLOTS];
    static uint8_t verdict[NSLOTS], vwant[NSLOTS];
    static uint32_t perm[NSLOTS];
    if (!pool || !pool2)
        return 1;
    for (uint32_t i = 0; i < NSLOTS; i++)
        perm[i] = i;
    for (uint32_t i = NSLOTS - 1; i > 0; i--) {
        const uint32_t j = (uint32_t)(rnd() % (i + 1));
        const uint32_t t = perm[i];
        perm[i] = perm[j];
        perm[j] = t;
    }
    struct ctx c = {0};
    c.threads = threads;
    if (hipMalloc(&c.d_pkt, 128) != hipSuccess || hipMalloc((void **)&c.d_out, 64) != hipSuccess ||
        hipStreamCreateWithFlags(&c.st, hipStreamNonBlocking) != hipSuccess)
        return 1;
    if (wc_host_register(pool, (uint64_t)NSLOTS * SLOT) != WC_OK) {
        fprintf(stderr, "register failed\n");
        return 1;
    }
    const int Ls[] = {64, 1472};
    const uint64_t ns[] = {1, 8, 64, 256, 1024, 4096};
    for (int li = 0; li < 2; li++) {
        const uint16_t L = (uint16_t)Ls[li];
        /* frame = 14 + L (L = IP bytes incl. headers, >= 28) */
        for (uint32_t i = 0; i < NSLOTS; i++)
            make_frame(pool + (size_t)i * SLOT, L);
        memcpy(pool2, pool, (size_t)NSLOTS * SLOT);
        for (size_t q = 0; q < sizeof ns / sizeof ns[0]; q++) {
            const uint64_t n = ns[q];
            for (uint64_t i = 0; i < n; i++) {
                off[i] = (uint64_t)perm[i] * SLOT;
                flen[i] = (uint16_t)(L + 14);
                len[i] = L; /* ip_cksum over the frame's first L bytes */
            }
            c.off = off;
            c.len = len;
            c.flen = flen;
            c.out = out;
            c.verdict = verdict;
            c.n = n;
            double zc, zc9, pp, pp9, rx, rx9, fl, fl9, c1, c19, cn, cn9, r1, r19;
            double sv = -1, sv9 = -1, rs = -1, rs9 = -1;
            c.pool = pool;
            if (n <= 256) {
                setenv("WC_SERVE", "1", 1);
                wc_config_reload();
                memset(out, 0, n * 2);
                time_calls(c_host, &c, secs, &sv, &sv9);
                oracle_cksum_ragged(pool, off, len, n, want, ORACLE_KIND_IP, 1);
                if (memcmp(out, want, n * 2)) {
                    printf("host_latency: FAIL server n=%llu L=%u\n", (unsigned long long)n, L);
                    return 1;
                }
                memset(verdict, 0xEE, n);
                time_calls(c_rx, &c, secs, &rs, &rs9);
                oracle_rx_verdict_ragged(pool, off, flen, n, vwant, 1);
                if (memcmp(verdict, vwant, n)) {
                    printf("host_latency: FAIL server rx n=%llu L=%u\n", (unsigned long long)n, L);
                    return 1;
                }
            }
            setenv("WC_SERVE", "0", 1);
            wc_config_reload();
            time_calls(c_host, &c, secs, &zc, &zc9);
            oracle_cksum_ragged(pool, off, len, n, want, ORACLE_KIND_IP, 1);
            if (memcmp(out, want, n * 2)) {
                printf("host_latency: FAIL zero-copy n=%llu L=%u\n", (unsigned long long)n, L);
                return 1;
            }
            time_calls(c_rx, &c, secs, &rx, &rx9);
            oracle_rx_verdict_ragged(pool, off, flen, n, vwant, 1);
            if (memcmp(verdict, vwant, n)) {
                printf("host_latency: FAIL rx n=%llu L=%u\n", (unsigned long long)n, L);
                return 1;
            }
            for (uint64_t i = 0; i < n; i++)
                if (vwant[i] != WC_RX_OK) {
                    printf("host_latency: FAIL frame %llu verdict %u\n", (unsigned long long)i,
                           vwant[i]);
                    return 1;
                }
            c.pool = pool2;
            memset(out, 0, n * 2);
            time_calls(c_host, &c, secs, &pp, &pp9);
            if (memcmp(out, want, n * 2)) {
                printf("host_latency: FAIL pipelined n=%llu L=%u\n", (unsigned long long)n, L);
                return 1;
            }
            time_calls(c_floor, &c, secs / 2, &fl, &fl9);
            c.pool = pool;
            time_calls(c_cpu, &c, secs / 2, &c1, &c19);
            time_calls(c_cpu_rx, &c, secs / 2, &r1, &r19);
            double rn, rn9;
            pool_start(threads); /* the workers spin only while this point runs */
            memset(out, 0, n * 2);
            time_calls(c_cpu_pool, &c, secs / 2, &cn, &cn9);
            if (memcmp(out, want, n * 2)) {
                printf("host_latency: FAIL cpu pool n=%llu L=%u\n", (unsigned long long)n, L);
                return 1;
            }
            memset(verdict, 0xEE, n);
            time_calls(c_cpu_pool_rx, &c, secs / 2, &rn, &rn9);
            pool_stop();
            if (memcmp(verdict, vwant, n)) {
                printf("host_latency: FAIL cpu pool rx n=%llu L=%u\n", (unsigned long long)n, L);
                return 1;
            }
            printf("{\"n\": %llu, \"L\": %u, \"srv_us\": %.2f, \"srv_p90_us\": %.2f, "
                   "\"zc_us\": %.2f, \"zc_p90_us\": %.2f, "
                   "\"pipe_us\": %.2f, \"rx_srv_us\": %.2f, \"rx_srv_p90_us\": %.2f, "
                   "\"rx_zc_us\": %.2f, \"rx_zc_p90_us\": %.2f, "
                   "\"floor_us\": %.2f, \"cpu1_us\": %.3f, \"cpu%d_us\": %.3f, "
                   "\"cpu1_rx_us\": %.3f, \"cpu%d_rx_us\": %.3f}\n",
                   (unsigned long long)n, L, sv, sv9, zc, zc9, pp, rs, rs9, rx, rx9, fl, c1,
                   threads, cn, r1, threads, rn);
            fflush(stdout);
        }
    }
    uint64_t served = 0, fallbacks = 0, launches = 0;
    wc_server_stats(&served, &fallbacks, &launches);
    if (!served || fallbacks) {
        /* the srv_* columns must be the server's own answers, not a fallback */
        printf("host_latency: FAIL server answered %llu batches, %llu fell back\n",
               (unsigned long long)served, (unsigned long long)fallbacks);
        return 1;
    }
    wc_host_unregister(pool);
    wc_gpu_fini();
    printf("host_latency: ok (%s; server answered %llu batches, 0 fallbacks, %llu grid "
           "launches)\n", wc_version(), (unsigned long long)served, (unsigned long long)launches);
    return 0;
}
