// wc_rccl.cpp -- RCCL (over xGMI) for the multi-GPU result gather of
// libwccksum (wc_gather_results_multi, include/warpcore_gpu/wc_cksum.h).
//
// The checksum itself has no exchange step: a batch shards into independent
// packet ranges.  The only collective is the gather of the
// 2-byte results after the shards are done -- an all-gather with unequal
// shard sizes, expressed as one ncclBroadcast per root inside a single
// ncclGroupStart/End (every device receives shard h at its packet offset,
// straight into the caller's buffer: no padding, no re-pack).  The library
// owns the communicators: ncclCommInitAll over the shard devices, created on
// the first gather and kept until wc_gpu_fini.
//
// RCCL is resolved at run time (dlopen of librccl.so.1): a caller that never
// gathers does not need it, and inside a Python process the copy torch has
// already loaded (same SONAME) is the one used.
#include "wc_rccl.h"

#include "warpcore_gpu/wc_cksum.h"

#include <rccl/rccl.h> // types only; the functions come from dlsym

#include <dlfcn.h>

#include <algorithm>
#include <cstdio>
#include <vector>

namespace wc {
namespace {

struct Rccl {
    void *h = nullptr;
    decltype(&ncclCommInitAll) comm_init_all = nullptr;
    decltype(&ncclCommDestroy) comm_destroy = nullptr;
    decltype(&ncclBroadcast) broadcast = nullptr;
    decltype(&ncclGroupStart) group_start = nullptr;
    decltype(&ncclGroupEnd) group_end = nullptr;
    decltype(&ncclGetErrorString) error_string = nullptr;
};

Rccl g_rccl;
std::vector<int> g_comm_devs;       // device list of the cached communicators
std::vector<ncclComm_t> g_comms;

int load_rccl()
{
    if (g_rccl.h)
        return WC_OK;
    void *h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h)
        h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) {
        fprintf(stderr, "wccksum: RCCL not loadable: %s\n", dlerror());
        return WC_ECOMM;
    }
    Rccl r;
    r.h = h;
    r.comm_init_all = (decltype(r.comm_init_all))dlsym(h, "ncclCommInitAll");
    r.comm_destroy = (decltype(r.comm_destroy))dlsym(h, "ncclCommDestroy");
    r.broadcast = (decltype(r.broadcast))dlsym(h, "ncclBroadcast");
    r.group_start = (decltype(r.group_start))dlsym(h, "ncclGroupStart");
    r.group_end = (decltype(r.group_end))dlsym(h, "ncclGroupEnd");
    r.error_string = (decltype(r.error_string))dlsym(h, "ncclGetErrorString");
    if (!r.comm_init_all || !r.comm_destroy || !r.broadcast || !r.group_start ||
        !r.group_end || !r.error_string) {
        fprintf(stderr, "wccksum: librccl.so.1 lacks a required symbol\n");
        return WC_ECOMM;
    }
    g_rccl = r;
    return WC_OK;
}

int nccl_err(ncclResult_t r, const char *what)
{
    if (r == ncclSuccess)
        return WC_OK;
    fprintf(stderr, "wccksum: %s: %s\n", what, g_rccl.error_string(r));
    return WC_ECOMM;
}

int ensure_comms(int ndev, const int *devs)
{
    int rc = load_rccl();
    if (rc)
        return rc;
    if ((int)g_comm_devs.size() == ndev &&
        std::equal(g_comm_devs.begin(), g_comm_devs.end(), devs))
        return WC_OK;
    rccl_fini();
    std::vector<ncclComm_t> comms(ndev);
    rc = nccl_err(g_rccl.comm_init_all(comms.data(), ndev, devs), "ncclCommInitAll");
    if (rc)
        return rc;
    g_comms = comms;
    g_comm_devs.assign(devs, devs + ndev);
    return WC_OK;
}

} // namespace

int rccl_allgatherv_u16(int ndev, const int *devs, const uint16_t *const *send,
                        const uint64_t *n, uint16_t *const *recv, void *const *streams)
{
    for (int a = 0; a < ndev; ++a)
        for (int b = a + 1; b < ndev; ++b)
            if (devs[a] == devs[b])
                return WC_EINVAL; // one communicator rank per GPU
    int rc = ensure_comms(ndev, devs);
    if (rc)
        return rc;
    std::vector<uint64_t> off(ndev + 1, 0);
    for (int h = 0; h < ndev; ++h)
        off[h + 1] = off[h] + n[h];
    rc = nccl_err(g_rccl.group_start(), "ncclGroupStart");
    if (rc)
        return rc;
    for (int h = 0; h < ndev; ++h) {
        if (n[h] == 0)
            continue;
        for (int g = 0; g < ndev; ++g) {
            const ncclResult_t r = g_rccl.broadcast(
                send[h], recv[g] + off[h], (size_t)n[h] * 2, ncclUint8, h, g_comms[g],
                streams ? (hipStream_t)streams[g] : (hipStream_t)0);
            if (r != ncclSuccess) {
                (void)g_rccl.group_end();
                return nccl_err(r, "ncclBroadcast");
            }
        }
    }
    return nccl_err(g_rccl.group_end(), "ncclGroupEnd");
}

void rccl_fini()
{
    if (!g_rccl.h)
        return;
    for (ncclComm_t c : g_comms)
        (void)g_rccl.comm_destroy(c);
    g_comms.clear();
    g_comm_devs.clear();
}

} // namespace wc
