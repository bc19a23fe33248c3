/*
 * multi_test.c -- a single-threaded C host (like warpcore's engine thread,
 * README.md:24-28) driving the multi-GPU entry points of libwccksum.so:
 *
 *   1. wc_cksum_host_multi over every visible GPU, then over 4 shards that
 *      share device 0 (the split and the interleaved pipelines rehearsed on
 *      fewer GPUs), pageable and registered, both kinds;
 *   2. device-resident shards (wc_cksum_ragged_multi), one per GPU, and the
 *      RCCL result gather (wc_gather_results_multi) back into packet order
 *      on every device.
 *
 * Every result is compared with the CPU oracle (oracle/wc_oracle.c, test
 * infrastructure) on the same bytes.  Prints "multi: ok ..." on success.
 *
 *     multi_test [packets]
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <hip/hip_runtime_api.h>

#include "warpcore_gpu/wc_cksum.h"
#include "wc_oracle.h"

#define CHECK(c)                                                               \
    do {                                                                       \
        if (!(c)) {                                                            \
            printf("multi: FAIL %s (line %d)\n", #c, __LINE__);                \
            return 1;                                                          \
        }                                                                      \
    } while (0)

static uint64_t rng_state = 0x9E3779B97F4A7C15ull;

static uint64_t rnd(void)
{
    uint64_t z = (rng_state += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

/* Ragged batch in host memory: lengths 64..1500 (a few jumbo), gaps 0..40,
 * arbitrary alignment -- an RX ring drained into one buffer.  Random bytes
 * read as IP headers for payload_cksum: every len >= 64 >= the largest
 * header length (the reference reads ~4 GiB when len < hl). */
static int make_batch(uint64_t n, uint8_t **buf, uint64_t *bytes, uint64_t **off,
                      uint16_t **len)
{
    *off = malloc(n * 8);
    *len = malloc(n * 2);
    if (!*off || !*len)
        return 1;
    uint64_t at = 3;
    for (uint64_t i = 0; i < n; i++) {
        const uint64_t r = rnd();
        (*len)[i] = (r & 1023) == 0 ? (uint16_t)(9000 + (r >> 20) % 100)
                                    : (uint16_t)(64 + (r >> 10) % 1437);
        (*off)[i] = at;
        at += (*len)[i] + (r >> 40) % 41;
    }
    *bytes = at + 64;
    *buf = malloc(*bytes);
    if (!*buf)
        return 1;
    for (uint64_t k = 0; k < *bytes; k++)
        (*buf)[k] = (uint8_t)rnd();
    return 0;
}

static int host_multi_case(const char *what, const uint8_t *buf, uint64_t bytes,
                           const uint64_t *off, const uint16_t *len, uint64_t n,
                           const uint16_t *want_ip, const uint16_t *want_pl, uint16_t *got)
{
    for (int kind = 0; kind < 2; kind++) {
        memset(got, 0xA5, n * 2);
        const int rc = wc_cksum_host_multi(buf, bytes, off, len, n, got, kind);
        if (rc != WC_OK) {
            printf("multi: FAIL %s kind %d: %s\n", what, kind, wc_strerror(rc));
            return 1;
        }
        const uint16_t *want = kind ? want_pl : want_ip;
        for (uint64_t i = 0; i < n; i++)
            if (got[i] != want[i]) {
                printf("multi: FAIL %s kind %d packet %llu: %04x != %04x\n", what, kind,
                       (unsigned long long)i, got[i], want[i]);
                return 1;
            }
    }
    return 0;
}

int main(int argc, char **argv)
{
    const uint64_t n = argc > 1 ? strtoull(argv[1], NULL, 0) : 200000;
    int ndev = 0;
    CHECK(hipGetDeviceCount(&ndev) == hipSuccess && ndev > 0);

    /* The split every *_multi call uses. */
    uint64_t lo, hi, prev = 0;
    for (int g = 0; g < 8; g++) {
        CHECK(wc_shard_range(n, g, 8, &lo, &hi) == WC_OK);
        CHECK(lo == prev && hi >= lo && hi - lo <= n / 8 + 1);
        prev = hi;
    }
    CHECK(prev == n);
    CHECK(wc_shard_range(n, 8, 8, &lo, &hi) == WC_EINVAL);

    uint8_t *buf;
    uint64_t bytes, *off;
    uint16_t *len;
    CHECK(make_batch(n, &buf, &bytes, &off, &len) == 0);
    uint16_t *want_ip = malloc(n * 2), *want_pl = malloc(n * 2), *got = malloc(n * 2);
    CHECK(want_ip && want_pl && got);
    /* payload_cksum reads 20 header bytes whatever len is: every packet here
     * has them inside the buffer (gaps + the 64-byte tail). */
    oracle_cksum_ragged(buf, off, len, n, want_ip, 0, 8);
    oracle_cksum_ragged(buf, off, len, n, want_pl, 1, 8);

    /* Before wc_gpu_init_multi: the single-device host path. */
    CHECK(wc_gpu_multi_count() == 0);
    CHECK(host_multi_case("uninitialised", buf, bytes, off, len, n, want_ip, want_pl, got) == 0);

    /* 1a. every visible GPU, pageable then registered */
    CHECK(wc_gpu_init_multi(ndev, NULL) == WC_OK);
    CHECK(wc_gpu_multi_count() == ndev);
    CHECK(host_multi_case("all GPUs", buf, bytes, off, len, n, want_ip, want_pl, got) == 0);
    CHECK(wc_host_register(buf, bytes) == WC_OK);
    CHECK(host_multi_case("all GPUs registered", buf, bytes, off, len, n, want_ip, want_pl,
                          got) == 0);
    /* small registered batch: the zero-copy path on shard 0 */
    CHECK(host_multi_case("zero-copy", buf, bytes, off, len, 1000, want_ip, want_pl, got) == 0);

    /* 1b. 4 shards sharing device 0 */
    const int same[4] = {0, 0, 0, 0};
    CHECK(wc_gpu_init_multi(4, same) == WC_OK);
    CHECK(wc_gpu_multi_count() == 4);
    CHECK(host_multi_case("4 shards on GPU 0 registered", buf, bytes, off, len, n, want_ip,
                          want_pl, got) == 0);
    CHECK(wc_host_unregister(buf) == WC_OK);
    CHECK(host_multi_case("4 shards on GPU 0", buf, bytes, off, len, n, want_ip, want_pl,
                          got) == 0);
    /* an invalid device list is refused before the shard set changes, and
     * the old set keeps working (no half-built executors) */
    {
        const int bad[2] = {0, 4096};
        CHECK(wc_gpu_init_multi(2, bad) == WC_EINVAL);
        CHECK(wc_gpu_multi_count() == 4);
        CHECK(host_multi_case("after a refused init", buf, bytes, off, len, n, want_ip, want_pl,
                              got) == 0);
        const int neg[1] = {-1};
        CHECK(wc_gpu_init_multi(1, neg) == WC_EINVAL);
        CHECK(wc_gpu_multi_count() == 4);
    }
    /* a shard device listed twice cannot join an RCCL communicator twice */
    {
        uint16_t *dummy[4] = {0};
        uint64_t cnt[4] = {0};
        CHECK(wc_gather_results_multi(dummy, cnt, dummy, NULL) == WC_EINVAL);
    }

    /* 2. device-resident shards, one per GPU, then the RCCL gather */
    CHECK(wc_gpu_init_multi(ndev, NULL) == WC_OK);
    enum { kMax = 64 };
    void *d_base[kMax];
    uint64_t *d_off[kMax];
    uint16_t *d_len[kMax], *d_out[kMax], *d_all[kMax];
    uint64_t cnt[kMax];
    hipStream_t st[kMax];
    uint64_t *h_roff = malloc(n * 8);
    CHECK(h_roff);
    for (int g = 0; g < ndev; g++) {
        CHECK(wc_shard_range(n, g, ndev, &lo, &hi) == WC_OK);
        cnt[g] = hi - lo;
        const uint64_t b0 = off[lo];
        const uint64_t b1 = hi > lo ? off[hi - 1] + (len[hi - 1] > 20 ? len[hi - 1] : 20) : b0;
        for (uint64_t i = lo; i < hi; i++)
            h_roff[i] = off[i] - b0;
        CHECK(hipSetDevice(g) == hipSuccess);
        CHECK(hipStreamCreate(&st[g]) == hipSuccess);
        CHECK(hipMalloc(&d_base[g], b1 - b0 + 64) == hipSuccess);
        CHECK(hipMalloc((void **)&d_off[g], cnt[g] * 8 + 8) == hipSuccess);
        CHECK(hipMalloc((void **)&d_len[g], cnt[g] * 2 + 2) == hipSuccess);
        CHECK(hipMalloc((void **)&d_out[g], cnt[g] * 2 + 2) == hipSuccess);
        CHECK(hipMalloc((void **)&d_all[g], n * 2) == hipSuccess);
        CHECK(hipMemcpy(d_base[g], buf + b0, b1 - b0, hipMemcpyHostToDevice) == hipSuccess);
        CHECK(hipMemcpy(d_off[g], h_roff + lo, cnt[g] * 8, hipMemcpyHostToDevice) == hipSuccess);
        CHECK(hipMemcpy(d_len[g], len + lo, cnt[g] * 2, hipMemcpyHostToDevice) == hipSuccess);
    }
    CHECK(hipSetDevice(0) == hipSuccess);
    CHECK(wc_cksum_ragged_multi((const void *const *)d_base, (const uint64_t *const *)d_off,
                                (const uint16_t *const *)d_len, cnt, d_out, WC_CKSUM_IP,
                                (void *const *)st) == WC_OK);
    const int grc = wc_gather_results_multi(d_out, cnt, d_all, (void *const *)st);
    if (grc != WC_OK) {
        printf("multi: FAIL gather: %s\n", wc_strerror(grc));
        return 1;
    }
    for (int g = 0; g < ndev; g++) {
        CHECK(hipSetDevice(g) == hipSuccess);
        CHECK(hipStreamSynchronize(st[g]) == hipSuccess);
        CHECK(hipMemcpy(got, d_all[g], n * 2, hipMemcpyDeviceToHost) == hipSuccess);
        for (uint64_t i = 0; i < n; i++)
            if (got[i] != want_ip[i]) {
                printf("multi: FAIL gathered on device %d, packet %llu: %04x != %04x\n", g,
                       (unsigned long long)i, got[i], want_ip[i]);
                return 1;
            }
        hipFree(d_base[g]);
        hipFree(d_off[g]);
        hipFree(d_len[g]);
        hipFree(d_out[g]);
        hipFree(d_all[g]);
        hipStreamDestroy(st[g]);
    }
    CHECK(wc_gpu_fini() == WC_OK);
    CHECK(wc_gpu_multi_count() == 0);
    printf("multi: ok %d GPU(s), %llu packets (%s)\n", ndev, (unsigned long long)n,
           wc_version());
    free(buf);
    free(off);
    free(len);
    free(want_ip);
    free(want_pl);
    free(got);
    free(h_roff);
    return 0;
}
