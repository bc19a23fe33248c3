// wc_rccl.h -- internal interface of wc_rccl.cpp (RCCL result gather).
#pragma once

#include <stdint.h>

namespace wc {

// Every device g receives shard h's n[h] results (send[h], on device h) at
// recv[g] + Σ n[<h], for all h: an all-gather with unequal shard sizes, as
// one ncclBroadcast per root in a single group, enqueued on streams[g].
// devs[] must be distinct (one communicator rank per GPU).  Caller holds the
// library lock.  Returns WC_OK, WC_EINVAL or WC_ECOMM.
int rccl_allgatherv_u16(int ndev, const int *devs, const uint16_t *const *send,
                        const uint64_t *n, uint16_t *const *recv, void *const *streams);

// Destroy the cached communicators (wc_gpu_fini).
void rccl_fini();

} // namespace wc
