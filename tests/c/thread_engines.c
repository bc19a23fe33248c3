/*
 * thread_engines.c -- several warpcore engines, each on its own thread,
 * calling the library at the same time.
 *
 * warpcore runs one engine per interface (w_init, /root/reference/lib/src/
 * warpcore.c), and an application may drive several from different threads;
 * each engine's TX / RX batch points (backend_netmap.c:348-358, 379-391) then
 * call the drop-in concurrently.  This program runs, for a few seconds:
 *   - host engines: own netmap-like buffer region (2048-B buffers), registered
 *     or pageable, batches of 1 .. 3000 packets at random buffers through
 *     wc_cksum_host (ip / payload), wc_cksum_ip_udp_host and
 *     wc_rx_verdict_host -- so the resident server, the zero-copy launch and
 *     the pipelined path are all hit from several threads;
 *   - device engines: own HIP stream and device buffer, strided / ragged /
 *     fused / RX-verdict batches enqueued on that stream, synchronised on
 *     that stream only;
 *   - a scalar caller: the drop-in ip_cksum / payload_cksum;
 *   - a churn thread: registers and unregisters a scratch region over and
 *     over (each stops the resident server grid) and reads the server stats;
 *   - a pauser: wc_server_pause, then a device-wide hipDeviceSynchronize
 *     while the host engines keep calling (it must return within 0.5 s:
 *     no grid left to wait for), then wc_server_resume, every ~40 ms.
 * Every result is compared with the oracle (oracle/wc_oracle.c) on the same
 * bytes.  At the end the server must have answered and never failed
 * (wc_server_stats: served > 0, fallbacks 0).
 *
 *   thread_engines [seconds] [host_engines] [device_engines]
 */
#include <execinfo.h>
#include <pthread.h>
#include <signal.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <unistd.h>

#include <hip/hip_runtime_api.h>

#include "warpcore_gpu/wc_cksum.h"
#include "wc_oracle.h"

#define BUF 2048
#define NBUF 4096 /* 8 MiB region per host engine */
#define MAXN 3000

static double g_seconds = 4.0;
static volatile int g_stop = 0;
static pthread_mutex_t g_print = PTHREAD_MUTEX_INITIALIZER;

static uint64_t xs(uint64_t *s)
{
    *s ^= *s << 13;
    *s ^= *s >> 7;
    *s ^= *s << 17;
    return *s;
}

static double now_s(void)
{
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec + t.tv_nsec * 1e-9;
}

static void fill(uint8_t *p, uint64_t n, uint64_t *s)
{
    for (uint64_t i = 0; i < n; i += 8) {
        const uint64_t v = xs(s);
        memcpy(p + i, &v, n - i < 8 ? n - i : 8);
    }
}

/* Make buffer b look like an Ethernet frame of IPv4 or IPv6 (random rest:
 * the verdicts spread over the RX codes) or leave it random (NOT_IP). */
static void frame_hdr(uint8_t *f, uint64_t r)
{
    switch (r % 3) {
    case 0:
        f[12] = 0x08, f[13] = 0x00, f[14] = 0x45;
        break;
    case 1:
        f[12] = 0x86, f[13] = 0xDD, f[14] = 0x60;
        break;
    default:
        break;
    }
}

/* payload_cksum is defined for len >= the header length only (the reference
 * converts len - hl to uint32: a shorter len reads ~4 GiB past the packet,
 * in_cksum.c:160-165), so payload lengths are raised to it. */
static uint16_t payload_len(const uint8_t *pk, uint16_t len)
{
    const uint16_t hl = (pk[0] >> 4) == 4 ? (uint16_t)((pk[0] & 15u) * 4u) : 40u;
    return len < hl ? hl : len;
}

struct result {
    uint64_t calls, packets, bad;
};

static void report(const char *who, int id, const char *what, uint64_t i, unsigned got,
                   unsigned want)
{
    pthread_mutex_lock(&g_print);
    fprintf(stderr, "%s %d: %s packet %llu: got %#x, oracle %#x\n", who, id, what,
            (unsigned long long)i, got, want);
    pthread_mutex_unlock(&g_print);
}

/* ---- host engines ------------------------------------------------------- */

struct host_arg {
    int id, registered;
    struct result r;
};

static void *host_engine(void *p)
{
    struct host_arg *a = p;
    uint64_t s = 0x1234567ull + 7919ull * (uint64_t)a->id;
    wc_gpu_init(0);
    uint8_t *mem = aligned_alloc(4096, (uint64_t)NBUF * BUF);
    uint64_t *off = malloc(MAXN * sizeof *off);
    uint16_t *len = malloc(MAXN * sizeof *len);
    uint16_t *out = malloc(MAXN * sizeof *out), *out2 = malloc(MAXN * sizeof *out2);
    uint8_t *verdict = malloc(MAXN);
    fill(mem, (uint64_t)NBUF * BUF, &s);
    if (a->registered && wc_host_register(mem, (uint64_t)NBUF * BUF) != WC_OK) {
        fprintf(stderr, "host %d: wc_host_register failed\n", a->id);
        a->r.bad++;
        g_stop = 1;
    }
    static const uint64_t sizes[] = {1, 3, 17, 64, 256, 700, 3000};
    const double t_end = now_s() + g_seconds;
    for (uint64_t it = 0; !g_stop && now_s() < t_end; ++it) {
        const uint64_t n = sizes[xs(&s) % (sizeof sizes / sizeof *sizes)];
        const int op = (int)(it % 4);
        for (uint64_t i = 0; i < n; ++i) {
            const uint64_t b = xs(&s) % NBUF;
            off[i] = b * BUF;
            len[i] = (uint16_t)(xs(&s) % 1515);
            if (op == 1 || op == 2)
                len[i] = payload_len(mem + off[i], len[i]);
            if (op == 3) /* a fresh frame header for this buffer */
                frame_hdr(mem + off[i], xs(&s));
        }
        int rc;
        uint64_t drops = 0;
        switch (op) {
        case 0:
        case 1:
            rc = wc_cksum_host(mem, (uint64_t)NBUF * BUF, off, len, n, out,
                               op == 0 ? WC_CKSUM_IP : WC_CKSUM_PAYLOAD);
            break;
        case 2:
            rc = wc_cksum_ip_udp_host(mem, (uint64_t)NBUF * BUF, off, len, n, out2, out);
            break;
        default:
            rc = wc_rx_verdict_host(mem, (uint64_t)NBUF * BUF, off, len, n, verdict, &drops);
            break;
        }
        if (rc != WC_OK) {
            fprintf(stderr, "host %d: op %d n %llu: %s\n", a->id, op, (unsigned long long)n,
                    wc_strerror(rc));
            a->r.bad++;
            break;
        }
        uint64_t odrops = 0;
        for (uint64_t i = 0; i < n; ++i) {
            const uint8_t *pk = mem + off[i];
            if (op <= 1) {
                const uint16_t w = op == 0 ? oracle_ip_cksum(pk, len[i])
                                           : oracle_payload_cksum(pk, len[i]);
                if (out[i] != w && a->r.bad++ < 5)
                    report("host", a->id, op == 0 ? "ip_cksum" : "payload_cksum", i, out[i], w);
            } else if (op == 2) {
                const int v4 = (pk[0] >> 4) == 4;
                const uint16_t wh = v4 ? oracle_ip_cksum(pk, (uint16_t)((pk[0] & 15u) * 4u)) : 0;
                const uint16_t wp = oracle_payload_cksum(pk, len[i]);
                if ((out2[i] != wh || out[i] != wp) && a->r.bad++ < 5)
                    report("host", a->id, "fused", i, (unsigned)out2[i] << 16 | out[i],
                           (unsigned)wh << 16 | wp);
            } else {
                const int w = oracle_rx_verdict(pk, len[i]);
                odrops += WC_RX_IS_DROP(w);
                if (verdict[i] != w && a->r.bad++ < 5)
                    report("host", a->id, "rx verdict", i, verdict[i], (unsigned)w);
            }
        }
        if (op == 3 && drops != odrops && a->r.bad++ < 5)
            report("host", a->id, "rx drops", n, (unsigned)drops, (unsigned)odrops);
        a->r.calls++;
        a->r.packets += n;
    }
    if (a->registered && wc_host_unregister(mem) != WC_OK)
        a->r.bad++;
    free(mem), free(off), free(len), free(out), free(out2), free(verdict);
    return NULL;
}

/* ---- device engines ----------------------------------------------------- */

#define DBYTES (16u << 20)
#define DMAXN 20000

struct dev_arg {
    int id;
    struct result r;
};

static int hip_ok(hipError_t e, int id, const char *what)
{
    if (e == hipSuccess)
        return 1;
    fprintf(stderr, "device %d: %s: %s\n", id, what, hipGetErrorString(e));
    return 0;
}

static void *device_engine(void *p)
{
    struct dev_arg *a = p;
    uint64_t s = 0xabcdefull + 104729ull * (uint64_t)a->id;
    wc_gpu_init(0);
    hipStream_t st = NULL;
    uint8_t *d_buf = NULL, *h_buf = malloc(DBYTES);
    uint64_t *d_off = NULL, *h_off = malloc(DMAXN * sizeof *h_off);
    uint16_t *d_len = NULL, *h_len = malloc(DMAXN * sizeof *h_len);
    uint16_t *d_out = NULL, *h_out = malloc(DMAXN * 2);
    uint16_t *d_out2 = NULL, *h_out2 = malloc(DMAXN * 2);
    uint64_t *d_drops = NULL;
    int ok = hip_ok(hipStreamCreateWithFlags(&st, hipStreamNonBlocking), a->id, "stream") &&
             hip_ok(hipMalloc((void **)&d_buf, DBYTES), a->id, "hipMalloc") &&
             hip_ok(hipMalloc((void **)&d_off, DMAXN * sizeof *d_off), a->id, "hipMalloc") &&
             hip_ok(hipMalloc((void **)&d_len, DMAXN * sizeof *d_len), a->id, "hipMalloc") &&
             hip_ok(hipMalloc((void **)&d_out, DMAXN * 2), a->id, "hipMalloc") &&
             hip_ok(hipMalloc((void **)&d_out2, DMAXN * 2), a->id, "hipMalloc") &&
             hip_ok(hipMalloc((void **)&d_drops, 8), a->id, "hipMalloc");
    if (ok) {
        fill(h_buf, DBYTES, &s);
        for (uint64_t b = 0; b + BUF <= DBYTES; b += BUF)
            frame_hdr(h_buf + b, xs(&s));
        ok = hip_ok(hipMemcpyAsync(d_buf, h_buf, DBYTES, hipMemcpyHostToDevice, st), a->id,
                    "H2D") &&
             hip_ok(hipStreamSynchronize(st), a->id, "sync");
    }
    if (!ok) {
        a->r.bad++;
        g_stop = 1;
    }
    const double t_end = now_s() + g_seconds;
    for (uint64_t it = 0; ok && !g_stop && now_s() < t_end; ++it) {
        const int op = (int)(it % 4);
        uint64_t n;
        uint16_t L = (uint16_t)(1 + xs(&s) % 1500);
        if (op == 0 && (it / 4) % 2 && L < 60) /* payload: L >= any header length */
            L = 60;
        const uint64_t stride = L + xs(&s) % 64;
        int rc;
        if (op == 0) { /* strided, packed or sparse */
            n = 1 + xs(&s) % (DBYTES / stride - 1);
            if (n > DMAXN)
                n = DMAXN;
            rc = wc_cksum_strided(d_buf, stride, L, n, d_out,
                                  (it / 4) % 2 ? WC_CKSUM_PAYLOAD : WC_CKSUM_IP, st);
        } else {
            n = 1 + xs(&s) % (DMAXN - 1);
            for (uint64_t i = 0; i < n; ++i) {
                h_off[i] = (xs(&s) % (DBYTES / BUF)) * BUF + (op == 3 ? 0 : xs(&s) % 64);
                h_len[i] = (uint16_t)(xs(&s) % 1515);
                if (op == 2 || (op == 1 && (it / 4) % 2))
                    h_len[i] = payload_len(h_buf + h_off[i], h_len[i]);
            }
            ok = hip_ok(hipMemcpyAsync(d_off, h_off, n * 8, hipMemcpyHostToDevice, st), a->id,
                        "H2D") &&
                 hip_ok(hipMemcpyAsync(d_len, h_len, n * 2, hipMemcpyHostToDevice, st), a->id,
                        "H2D") &&
                 hip_ok(hipMemsetAsync(d_drops, 0, 8, st), a->id, "memset");
            if (!ok)
                break;
            if (op == 1)
                rc = wc_cksum_ragged(d_buf, d_off, d_len, n, d_out,
                                     (it / 4) % 2 ? WC_CKSUM_PAYLOAD : WC_CKSUM_IP, st);
            else if (op == 2)
                rc = wc_cksum_ip_udp_ragged(d_buf, d_off, d_len, n, d_out2, d_out, st);
            else
                rc = wc_rx_verdict_ragged(d_buf, d_off, d_len, n, (uint8_t *)d_out, d_drops, st);
        }
        if (rc != WC_OK) {
            fprintf(stderr, "device %d: op %d: %s\n", a->id, op, wc_strerror(rc));
            a->r.bad++;
            break;
        }
        uint64_t drops = 0;
        ok = hip_ok(hipMemcpyAsync(h_out, d_out, n * 2, hipMemcpyDeviceToHost, st), a->id,
                    "D2H") &&
             hip_ok(hipMemcpyAsync(h_out2, d_out2, n * 2, hipMemcpyDeviceToHost, st), a->id,
                    "D2H") &&
             hip_ok(hipMemcpyAsync(&drops, d_drops, 8, hipMemcpyDeviceToHost, st), a->id,
                    "D2H") &&
             hip_ok(hipStreamSynchronize(st), a->id, "sync");
        if (!ok)
            break;
        const int kind = (it / 4) % 2 ? ORACLE_KIND_PAYLOAD : ORACLE_KIND_IP;
        uint64_t odrops = 0;
        for (uint64_t i = 0; i < n; ++i) {
            const uint8_t *pk = h_buf + (op == 0 ? i * stride : h_off[i]);
            const uint16_t l = op == 0 ? L : h_len[i];
            if (op <= 1) {
                const uint16_t w = kind == ORACLE_KIND_IP ? oracle_ip_cksum(pk, l)
                                                          : oracle_payload_cksum(pk, l);
                if (h_out[i] != w && a->r.bad++ < 5)
                    report("device", a->id, op == 0 ? "strided" : "ragged", i, h_out[i], w);
            } else if (op == 2) {
                const int v4 = (pk[0] >> 4) == 4;
                const uint16_t wh = v4 ? oracle_ip_cksum(pk, (uint16_t)((pk[0] & 15u) * 4u)) : 0;
                const uint16_t wp = oracle_payload_cksum(pk, l);
                if ((h_out2[i] != wh || h_out[i] != wp) && a->r.bad++ < 5)
                    report("device", a->id, "fused", i, (unsigned)h_out2[i] << 16 | h_out[i],
                           (unsigned)wh << 16 | wp);
            } else {
                const int w = oracle_rx_verdict(pk, l);
                odrops += WC_RX_IS_DROP(w);
                if (((const uint8_t *)h_out)[i] != w && a->r.bad++ < 5)
                    report("device", a->id, "rx verdict", i, ((const uint8_t *)h_out)[i],
                           (unsigned)w);
            }
        }
        if (op == 3 && drops != odrops && a->r.bad++ < 5)
            report("device", a->id, "rx drops", n, (unsigned)drops, (unsigned)odrops);
        a->r.calls++;
        a->r.packets += n;
    }
    if (!ok)
        a->r.bad++;
    if (st)
        (void)hipStreamSynchronize(st), (void)hipStreamDestroy(st);
    (void)hipFree(d_buf), (void)hipFree(d_off), (void)hipFree(d_len), (void)hipFree(d_out);
    (void)hipFree(d_out2), (void)hipFree(d_drops);
    free(h_buf), free(h_off), free(h_len), free(h_out), free(h_out2);
    return NULL;
}

/* ---- scalar caller and registration churn -------------------------------- */

static void *scalar_caller(void *p)
{
    struct result *r = p;
    uint64_t s = 0x5151ull;
    uint8_t buf[2048];
    const double t_end = now_s() + g_seconds;
    while (!g_stop && now_s() < t_end) {
        uint16_t l = (uint16_t)(xs(&s) % 1515);
        fill(buf, sizeof buf, &s);
        const int pay = (int)(r->calls & 1);
        if (pay)
            l = payload_len(buf, l);
        const uint16_t got = pay ? payload_cksum(buf, l) : ip_cksum(buf, l);
        const uint16_t w = pay ? oracle_payload_cksum(buf, l) : oracle_ip_cksum(buf, l);
        if (got != w && r->bad++ < 5)
            report("scalar", 0, pay ? "payload_cksum" : "ip_cksum", r->calls, got, w);
        r->calls++;
        r->packets++;
    }
    return NULL;
}

static void *churn(void *p)
{
    struct result *r = p;
    const uint64_t bytes = 1u << 20;
    uint8_t *scratch = aligned_alloc(4096, bytes);
    memset(scratch, 0, bytes);
    const double t_end = now_s() + g_seconds;
    while (!g_stop && now_s() < t_end) {
        if (wc_host_register(scratch, bytes) != WC_OK || wc_host_unregister(scratch) != WC_OK) {
            fprintf(stderr, "churn: register / unregister failed\n");
            r->bad++;
            break;
        }
        uint64_t served = 0, fallbacks = 0;
        wc_server_stats(&served, &fallbacks, NULL);
        r->calls++;
        struct timespec ts = {0, 20 * 1000 * 1000}; /* 20 ms */
        nanosleep(&ts, NULL);
    }
    free(scratch);
    return NULL;
}

/* The quiesce API under traffic: after wc_server_pause no grid is resident,
 * so a device-wide synchronisation waits only for the engines' own short
 * kernels -- never for the next idle period of the host engines. */
static double g_max_sync_s = 0;

static void *pauser(void *p)
{
    struct result *r = p;
    const double t_end = now_s() + g_seconds;
    while (!g_stop && now_s() < t_end) {
        if (wc_server_pause() != WC_OK) {
            fprintf(stderr, "pauser: wc_server_pause failed\n");
            r->bad++;
            break;
        }
        const double t0 = now_s();
        const hipError_t e = hipDeviceSynchronize();
        const double dt = now_s() - t0;
        if (dt > g_max_sync_s)
            g_max_sync_s = dt;
        if (e != hipSuccess || dt > 0.5) {
            fprintf(stderr, "pauser: device sync after a pause took %.3f s (%s)\n", dt,
                    hipGetErrorString(e));
            r->bad++;
        }
        struct timespec ts = {0, 10 * 1000 * 1000}; /* 10 ms paused */
        nanosleep(&ts, NULL);
        if (wc_server_resume() != WC_OK) {
            fprintf(stderr, "pauser: wc_server_resume failed\n");
            r->bad++;
            break;
        }
        r->calls++;
        ts.tv_nsec = 30 * 1000 * 1000; /* 30 ms serving */
        nanosleep(&ts, NULL);
    }
    return NULL;
}

/* Every engine must have been served in turn: the library's lock is first
 * come, first served, and device-resident calls do not wait for it. */
static int starved(const char *who, int id, uint64_t calls, uint64_t min_calls)
{
    if (calls >= min_calls)
        return 0;
    fprintf(stderr, "%s %d: only %llu calls in %.1f s (starved)\n", who, id,
            (unsigned long long)calls, g_seconds);
    return 1;
}

/* A crash names its place: the backtrace (library frames as lib(+offset)
 * for addr2line) on stderr, then the signal's exit status. */
static void on_fault(int sig)
{
    void *bt[64];
    const int n = backtrace(bt, 64);
    static const char msg[] = "thread_engines: fatal signal, backtrace:\n";
    (void)!write(2, msg, sizeof msg - 1);
    backtrace_symbols_fd(bt, n, 2);
    _exit(128 + sig);
}

int main(int argc, char **argv)
{
    setvbuf(stdout, NULL, _IOLBF, 0);
    signal(SIGSEGV, on_fault);
    signal(SIGBUS, on_fault);
    signal(SIGABRT, on_fault);
    if (argc > 1)
        g_seconds = atof(argv[1]);
    const int nh = argc > 2 ? atoi(argv[2]) : 4, nd = argc > 3 ? atoi(argv[3]) : 2;
    if (nh < 0 || nh > 16 || nd < 0 || nd > 8) {
        fprintf(stderr, "usage: thread_engines [seconds] [host 0..16] [device 0..8]\n");
        return 2;
    }
    if (wc_gpu_init(0) != WC_OK) {
        fprintf(stderr, "thread_engines: no gfx950 device\n");
        return 1;
    }
    uint64_t served0 = 0, fb0 = 0, l0 = 0;
    wc_server_stats(&served0, &fb0, &l0);
    pthread_t th[32];
    struct host_arg ha[16];
    struct dev_arg da[8];
    struct result sc = {0}, ch = {0}, pz = {0};
    int k = 0;
    for (int i = 0; i < nh; ++i) {
        ha[i] = (struct host_arg){i, i % 4 != 3, {0}}; /* every 4th region pageable */
        pthread_create(&th[k++], NULL, host_engine, &ha[i]);
    }
    for (int i = 0; i < nd; ++i) {
        da[i] = (struct dev_arg){i, {0}};
        pthread_create(&th[k++], NULL, device_engine, &da[i]);
    }
    pthread_create(&th[k++], NULL, scalar_caller, &sc);
    pthread_create(&th[k++], NULL, churn, &ch);
    pthread_create(&th[k++], NULL, pauser, &pz);
    for (int i = 0; i < k; ++i)
        pthread_join(th[i], NULL);

    uint64_t bad = sc.bad + ch.bad + pz.bad;
    printf("thread_engines: %.1f s, %d host engines, %d device engines\n", g_seconds, nh, nd);
    for (int i = 0; i < nh; ++i) {
        printf("  host %d (%s): %llu calls, %llu packets, %llu mismatches\n", i,
               ha[i].registered ? "registered" : "pageable", (unsigned long long)ha[i].r.calls,
               (unsigned long long)ha[i].r.packets, (unsigned long long)ha[i].r.bad);
        bad += ha[i].r.bad + starved("host", i, ha[i].r.calls, 20);
    }
    for (int i = 0; i < nd; ++i) {
        printf("  device %d: %llu calls, %llu packets, %llu mismatches\n", i,
               (unsigned long long)da[i].r.calls, (unsigned long long)da[i].r.packets,
               (unsigned long long)da[i].r.bad);
        bad += da[i].r.bad + starved("device", i, da[i].r.calls, 20);
    }
    printf("  scalar: %llu calls, %llu mismatches; churn: %llu register cycles\n",
           (unsigned long long)sc.calls, (unsigned long long)sc.bad,
           (unsigned long long)ch.calls);
    printf("  pauser: %llu pause / sync / resume cycles, longest device sync %.1f ms\n",
           (unsigned long long)pz.calls, g_max_sync_s * 1e3);
    bad += starved("scalar", 0, sc.calls, 20) + starved("churn", 0, ch.calls, 5) +
           starved("pauser", 0, pz.calls, 5);
    uint64_t served = 0, fb = 0, l = 0;
    wc_server_stats(&served, &fb, &l);
    printf("  server: %llu batches served, %llu fallbacks, %llu grid launches\n",
           (unsigned long long)(served - served0), (unsigned long long)(fb - fb0),
           (unsigned long long)(l - l0));
    if (nh > 0 && (served == served0 || fb != fb0)) {
        fprintf(stderr, "thread_engines: the resident server did not answer every batch\n");
        bad++;
    }
    wc_gpu_fini();
    if (bad) {
        printf("thread_engines: FAILED (%llu)\n", (unsigned long long)bad);
        return 1;
    }
    printf("thread_engines: ok\n");
    return 0;
}
