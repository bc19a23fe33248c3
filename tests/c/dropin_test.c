/*
 * dropin_test.c -- a C caller using libwccksum.so exactly where warpcore's
 * stack calls in_cksum.c: compute on TX (udp.c:209-213, ip4.c:184-186),
 * verify on RX (udp.c:132-139, ip4.c:110-115), then one batch call at the
 * w_tx batch point (backend_netmap.c:348-358).  Expected values are the
 * known answers of tests/golden/kat.json.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <hip/hip_runtime_api.h>

#include "warpcore_gpu/wc_cksum.h"

#define CHECK(c)                                                               \
    do {                                                                       \
        if (!(c)) {                                                            \
            printf("dropin: FAIL %s (line %d)\n", #c, __LINE__);               \
            return 1;                                                          \
        }                                                                      \
    } while (0)

int main(void)
{
    /* RFC 1071 sec. 3 bytes -> 0x0d22 (memory 22 0d). */
    const uint8_t rfc[8] = {0x00, 0x01, 0xf2, 0x03, 0xf4, 0xf5, 0xf6, 0xf7};
    CHECK(ip_cksum(rfc, sizeof rfc) == 0x0d22);

    /* IPv4 header: compute like mk_ip4_hdr, then verify like ip4_rx. */
    uint8_t ip[20] = {0x45, 0x00, 0x00, 0x73, 0x00, 0x00, 0x40, 0x00, 0x40, 0x11,
                      0x00, 0x00, 0xc0, 0xa8, 0x00, 0x01, 0xc0, 0xa8, 0x00, 0xc7};
    const uint16_t c = ip_cksum(ip, sizeof ip);
    CHECK(c == 0x61b8);
    memcpy(ip + 10, &c, 2);
    CHECK(ip_cksum(ip, sizeof ip) == 0);

    /* UDP over IPv4: udp_tx computes with cksum = 0, udp_rx verifies to 0. */
    uint8_t pkt[20 + 8 + 100];
    memset(pkt, 0, sizeof pkt);
    memcpy(pkt, ip, 20);
    pkt[2] = 0;
    pkt[3] = sizeof pkt; /* total length */
    pkt[20 + 5] = 8 + 100; /* udp->len (network order, < 256) */
    for (int i = 0; i < 100; i++)
        pkt[28 + i] = (uint8_t)(i * 7 + 3);
    const uint16_t u = payload_cksum(pkt, sizeof pkt);
    memcpy(pkt + 26, &u, 2);
    CHECK(payload_cksum(pkt, sizeof pkt) == 0);

    /* Batch entry at the TX batch point: 64 copies of the RFC bytes. */
    enum { N = 64 };
    uint8_t *d_buf = NULL;
    uint16_t *d_out = NULL, h_out[N];
    CHECK(hipMalloc((void **)&d_buf, N * 8) == hipSuccess);
    CHECK(hipMalloc((void **)&d_out, N * 2) == hipSuccess);
    uint8_t h_buf[N * 8];
    for (int i = 0; i < N; i++)
        memcpy(h_buf + 8 * i, rfc, 8);
    CHECK(hipMemcpy(d_buf, h_buf, sizeof h_buf, hipMemcpyHostToDevice) == hipSuccess);
    CHECK(wc_cksum_strided(d_buf, 8, 8, N, d_out, WC_CKSUM_IP, NULL) == WC_OK);
    CHECK(hipMemcpy(h_out, d_out, sizeof h_out, hipMemcpyDeviceToHost) == hipSuccess);
    for (int i = 0; i < N; i++)
        CHECK(h_out[i] == 0x0d22);
    CHECK(wc_cksum_strided(d_buf, 8, 8, N, NULL, WC_CKSUM_IP, NULL) == WC_EINVAL);
    CHECK(wc_cksum_strided(d_buf, 8, 8, N, d_out, 7, NULL) == WC_EINVAL);
    hipFree(d_buf);
    hipFree(d_out);
    CHECK(wc_gpu_fini() == WC_OK);
    printf("dropin: ok (%s)\n", wc_version());
    return 0;
}
