// wc_rt.h -- internal interface of the host runtime behind the C ABI of
// libwccksum.so (include/warpcore_gpu/wc_cksum.h).  The runtime is split by
// responsibility:
//   wc_rt_config.cpp   configuration (the WC_* table), device state, lifetime
//   wc_rt_plan.cpp     launch planner, device-resident batch calls, scalar drop-ins
//   wc_rt_rx.cpp       RX verdict launches (ADAPT: EARLY or HT per launch)
//   wc_rt_server.cpp   host side of the resident small-batch server
//   wc_rt_host.cpp     host-memory batches: zero-copy launch, staging, pipeline
//   wc_rt_multi.cpp    the batch split over the GPUs of one node
// Nothing here is exported from the library (hidden visibility).
#pragma once

#include "warpcore_gpu/wc_cksum.h"

#include "wc_cksum_kernels.h"

#include <hip/hip_runtime.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <map>
#include <mutex>

namespace wc {
namespace rt __attribute__((visibility("hidden"))) {

constexpr int kMaxDevices = 64;
constexpr int kPipe = 3;                          // host-path pipeline depth
constexpr uint64_t kChunkBytes = 64ull << 20;     // host-path bytes per chunk
constexpr uint64_t kChunkPkts = 1ull << 20;       // host-path packets per chunk
constexpr uint64_t kScalarStage = 65536 + 64;     // one max-size packet
constexpr uint64_t kZcPkts = 4096;                // zero-copy path: max packets
constexpr int kFlatMinDefault = 0;                // ragged: flat kernel from n >= this
// Internal batch kinds of the host paths beside WC_CKSUM_IP / WC_CKSUM_PAYLOAD:
// RX verdicts of Ethernet frames (lengths = frame lengths, 1-byte results),
// and the fused TX pair (payload_cksum into the main results, the IPv4
// header's ip_cksum into a second array; wc_cksum_ip_udp_host).
constexpr int kKindRx = 2;
constexpr int kKindFused = 3;

// Small batches over registered memory skip the copy engines: the kernel
// reads the packets straight out of the page-locked region over PCIe, and
// the offsets, lengths and results sit in mapped pinned memory.  Batches up
// to this many payload bytes take it (WC_ZC_BYTES overrides; 0 disables).
constexpr int kZcBytesDefault = 8 << 20;
// Zero-copy batches up to this many packets use the ragged group kernel
// (every packet's loads cross PCIe at once); larger ones the flat kernel.
// Measured on MI355X, tools/host_latency.py.
constexpr uint64_t kZcGroupMax = 1024;

struct HostPipe {
    hipStream_t st[kPipe] = {};
    hipEvent_t done[kPipe] = {};
    uint8_t *d_bytes[kPipe] = {};
    uint64_t *d_off[kPipe] = {};
    uint16_t *d_len[kPipe] = {};
    uint16_t *d_out[kPipe] = {};
    uint16_t *d_out2[kPipe] = {};  // fused pass: the IPv4 header checksums
    uint8_t *h_bytes[kPipe] = {};  // pinned staging for unregistered input
    uint64_t *h_off[kPipe] = {};   // pinned, rebased offsets
    uint16_t *h_len[kPipe] = {};
    uint16_t *h_out[kPipe] = {};
    uint16_t *h_out2[kPipe] = {};
    bool ready = false;
};

struct ZeroCopy {
    hipStream_t st = nullptr;
    uint64_t *h_off = nullptr, *d_off = nullptr; // mapped pinned
    uint16_t *h_len = nullptr, *d_len = nullptr;
    uint16_t *h_out = nullptr, *d_out = nullptr;
    uint16_t *h_out2 = nullptr, *d_out2 = nullptr; // fused pass: header checksums
    bool ready = false;
};

// Large batches in a registered region, read by the kernels in place over
// PCIe (host_zc_stream): chunks of up to kZsPkts packets, one launch each,
// their offsets / lengths / results double-buffered in mapped pinned memory.
// Only the lines the packets touch cross the link -- not the gaps between
// netmap slots the pipeline's range copy ships -- and nothing is staged.
constexpr uint64_t kZsPkts = 1ull << 16;
struct ZcStream {
    hipStream_t st = nullptr;
    hipEvent_t done[2] = {};
    uint64_t *h_off[2] = {}, *d_off[2] = {}; // mapped pinned
    uint16_t *h_len[2] = {}, *d_len[2] = {};
    uint16_t *h_out[2] = {}, *d_out[2] = {};
    uint16_t *h_out2[2] = {}, *d_out2[2] = {}; // fused pass: header checksums
    bool ready = false;
};

// The resident small-batch server of one device (wc_k_serve.hip): its
// stream, the mapped pinned request records and result slots, the request
// counter, and whether its grid is running.
struct Server {
    hipStream_t st = nullptr;
    wc::SrvRec *h_rec = nullptr, *d_rec = nullptr;
    wc::SrvRes *h_res = nullptr, *d_res = nullptr;
    uint32_t *h_hb = nullptr, *d_hb = nullptr; // heartbeat: the latest request number
    uint32_t seq = 0;
    int waves = 0;
    bool ready = false, running = false, broken = false;
    // last: the last answered call (the idle watcher's clock); posted: the
    // grid's launch or its last request (the drain-safety clock)
    std::chrono::steady_clock::time_point last{}, posted{};
};

// wc_server_stats, over every device and the whole process (under g_mu):
// batches the grid answered, batches it was asked for but could not answer
// (the launch path took them), grid launches.
struct ServerStats {
    uint64_t served = 0, fallbacks = 0, launches = 0;
};
extern ServerStats g_srv_stats;

struct Device {
    bool ok = false;
    int cus = 0;
    uint64_t clock_khz = 100000; // wall_clock64 rate (hipDeviceAttributeWallClockRate)
    hipStream_t scalar_st = nullptr;
    uint8_t *h_stage = nullptr;  // pinned + mapped scalar staging
    uint8_t *d_stage = nullptr;
    uint16_t *h_res = nullptr;
    uint16_t *d_res = nullptr;
    HostPipe pipe;
    ZeroCopy zc;
    ZcStream zs;
    Server srv;
    // RX verdict ADAPT mode: kRxSets tally arrays in mapped pinned memory,
    // one per recent launch (launch g writes set g % kRxSets), and the mode
    // the newest tally chose (rx_launch).
    uint32_t *h_rx_tally[4] = {}, *d_rx_tally[4] = {};
    uint32_t rx_words[4] = {}; // tally words launch g % kRxSets may write
    uint32_t rx_gen = 0;
    bool rx_early = false;
    uint32_t rx_nlaunch[2] = {}, rx_ndecided = 0; // WC_RX_TRACE=2 counts
};
constexpr int kRxSets = 4;
extern std::mutex g_rx_mu; // rx_launch's tally bookkeeping (batch calls run outside g_mu)

struct Registration {
    uint64_t bytes;
    // Device address of the region's first byte, looked up per device on
    // first use (hipHostGetDevicePointer with that device current).
    const uint8_t *dptr[kMaxDevices] = {};
};

// Tuning knobs (the WC_* environment), read once when the library first
// initialises and again only on wc_config_reload(); the defaults are the
// values tuned on MI355X (DESIGN.md sections 4-5).  Batch calls take a copy
// under g_cfg_mu (written with g_mu and g_cfg_mu held), so a reload never
// races a launch.
struct Config {
    int blocks_per_cu = 0;         // WC_BLOCKS_PER_CU: cap the one-shot grid
    int grid = 0;                  // WC_GRID: fixed grid (grid-stride)
    int variant = 0;               // WC_VARIANT: experimental kernel variants (tuning build)
    bool have_shape = false;       // WC_SHAPE=G,CPL,U: force the strided shape
    wc::Shape shape{};
    bool have_rshape = false;      // WC_RAGGED_SHAPE: small ragged group shape
    wc::Shape rshape{};
    int strided_seg = 1;           // WC_STRIDED_SEG: 0 never, 1 by the table, 2 always
    int flat_un = 2;               // WC_FLAT_UN: flat kernel rows per group
    int flat_tpw = 1;              // WC_FLAT_TPW: flat kernel tiles per wave
    int seg = 1;                   // WC_SEG: 0 = flat kernel for ragged batches
    int seg_rows = 4;              // WC_SEG_ROWS (ragged; packed strided: set = forced)
    bool seg_rows_set = false;
    int zc_seg = 0;                // WC_ZC_SEG: seg kernel on zero-copy batches
    int zc_group_max = (int)kZcGroupMax; // WC_ZC_GROUP_MAX
    int zc_bytes = kZcBytesDefault;      // WC_ZC_BYTES
    int zc_stream = 1;             // WC_ZC_STREAM: large registered batches read in place (0: pipeline)
    uint64_t zs_pkts = kZsPkts;    // WC_ZS_PKTS: packets per zero-copy stream launch (<= kZsPkts)
    uint64_t flat_min = kFlatMinDefault; // WC_FLAT_MIN: ragged group kernel below this n
    int diag_noload = 0;           // WC_DIAG_NOLOAD: timing-only kernel (tuning build)
    int nt = 1;                    // WC_NT: nontemporal loads
    int grp_dense = 65;            // WC_GRP_DENSE (64ths; 65 = never)
    int grp_sparse = 40;           // WC_GRP_SPARSE
    int grp_rows = 4;              // WC_GRP_ROWS
    int flat_pk = 1;               // WC_FLAT_PK: flat kernel chunks per lane slot
    int gather = 1;                // WC_GATHER: seg kernel's gathered-stream path (0 off, 2 forced)
    int lean_max = 48;             // WC_LEAN_MAX: lean kernel for aligned packets up to this many chunks
    // Large batches as back-to-back launches (one launch of millions of
    // one-shot workgroups lets the XCDs drift apart in the address space;
    // DESIGN.md section 5.3): strided batches in pieces of WC_SPLIT_BYTES of
    // stride (default 3 GiB: the 49-GB C5 window 0.907 -> 0.944 of peak,
    // profiles/ab_r05_split.log), and, if set, any batch in pieces of
    // WC_SPLIT_PKTS packets (ragged batches: off by default, C4 measured
    // slower split).
    uint64_t split_bytes = 3ull << 30; // WC_SPLIT_BYTES (0 = off)
    uint64_t split_pkts = 0;           // WC_SPLIT_PKTS (0 = off; overrides WC_SPLIT_BYTES)
    int lean_phase = 1;            // WC_LEAN_PHASE: lean kernel for sparse packets at an even phase too
    int serve = 1;                 // WC_SERVE: resident server for small registered host batches
    int serve_waves = 64;          // WC_SERVE_WAVES: its waves (one 64-lane workgroup each)
    int serve_max = 256;           // WC_SERVE_MAX: largest batch (packets) it takes
    int serve_idle_us = 20000;     // WC_SERVE_IDLE_US: stopped after this long without a call
    int serve_prio = 1;            // WC_SERVE_PRIO=0: its stream at normal priority (the A/B of
                                   // server_stream_create; other streams then queue behind it)
    // RX verdict kernel modes (profiles/ab_r04_rx_*.log): transposed header
    // loads win everywhere (mixed ring 127.5 -> 111.4 us); parsing first
    // (EARLY) wins when many frames need no UDP check (a third ARP: 111.8 ->
    // 96.6 us) and loses 3 us on an all-UDP ring; SKIP loses on all-UDP rings.
    int rx_early = 0;              // WC_RX_EARLY: RX verdict parses before streaming
    int rx_hdrt = 1;               // WC_RX_HDRT: RX verdict header chunks loaded transposed
    int rx_skip = 0;               // WC_RX_SKIP: frames the parse rules out leave the stream
    int rx_adapt = 1;              // WC_RX_ADAPT: EARLY or HT per launch, by the ring's mix
    int rx_trace = 0;              // WC_RX_TRACE: log each ADAPT decision to stderr (tools;
                                   // 2: one summary line per 512 launches)
    int rx_force = 0;              // WC_RX_FORCE: ADAPT's decision fixed, 1 HT / 2 EARLY (tools)
    int rx_grid = 0;               // WC_RX_GRID: cap the RX grid at this many blocks (tools)
    int rx_mode() const
    {
        // The default: ADAPT (EARLY or the HT stream per tile, by the share
        // of frames the launch's earlier tiles ruled out).  A fixed mode set
        // by WC_RX_EARLY / WC_RX_SKIP / WC_RX_HDRT=0 / WC_RX_ADAPT=0 wins.
        if (rx_adapt && !rx_early && !rx_skip && rx_hdrt)
            return wc::kRxAdapt | wc::kRxHdrT;
        // EARLY streams only the frames that need the check already, so
        // SKIP has nothing to take out: it is dropped rather than sending
        // EARLY | SKIP to a variant that ignores the HDRT / NT settings.
        return (rx_early ? wc::kRxEarly : 0) | (rx_hdrt ? wc::kRxHdrT : 0) |
               (rx_skip && !rx_early ? wc::kRxSkip : 0);
    }
};

// The library lock: first come, first served.  Host-memory batch calls hold
// it for a whole call (the server, zero-copy and pipeline resources are the
// device's), and several engine threads may call back to back; a plain
// std::mutex let the thread that had just released it take it again, and one
// engine starved the others for seconds (tests/c/thread_engines.c: 123,710
// calls on one thread, 2-4 on each of seven others).  A ticket order, with a
// short spin before sleeping (the server answers in ~5 us).
class FairMutex {
public:
    void lock()
    {
        const uint64_t t = next_.fetch_add(1, std::memory_order_relaxed);
        for (int spin = 0; spin < 4096; ++spin) {
            if (serving_.load(std::memory_order_acquire) == t)
                return;
            __builtin_ia32_pause();
        }
        std::unique_lock<std::mutex> l(m_);
        cv_.wait(l, [&] { return serving_.load(std::memory_order_acquire) == t; });
    }
    void unlock()
    {
        {
            std::lock_guard<std::mutex> l(m_); // (no lost wake-up between test and wait)
            serving_.fetch_add(1, std::memory_order_release);
        }
        cv_.notify_all();
    }

private:
    std::atomic<uint64_t> next_{0}, serving_{0};
    std::mutex m_;
    std::condition_variable cv_;
};


extern FairMutex g_mu;
extern Device g_dev[kMaxDevices];
// Device d's state is built (set under g_mu once init_locked has finished it,
// cleared by wc_gpu_fini): device-resident batch calls then only copy the
// configuration (g_cfg_mu) and enqueue on the caller's stream, without
// queueing behind a host-memory call that holds g_mu.
extern std::atomic<bool> g_dev_ready[kMaxDevices];
extern std::mutex g_cfg_mu; // g_cfg is written with g_mu AND g_cfg_mu held
extern std::map<uintptr_t, Registration> g_registered; // host base -> region
extern Config g_cfg;
extern bool g_cfg_loaded;

// Multi-GPU shard executors (wc_gpu_init_multi): shard g runs on device
// g_shard[g].dev with its own host pipeline, so two shards may share a GPU.
struct ShardExec {
    int dev = -1;
    HostPipe pipe;
};
extern ShardExec g_shard[kMaxDevices];
extern int g_multi_n;

// --- wc_rt_config.cpp ---------------------------------------------------------
int hip_err(hipError_t e);
int current_device(int *dev);
void load_config_locked();
// Create per-device state (caller holds g_mu).
int init_locked(int device, Device **out);
// The device-resident batch calls' entry (see wc_rt_config.cpp).
int ensure_device(Device **out, Config *cfg);

// --- wc_rt_plan.cpp -----------------------------------------------------------
struct Plan {
    wc::Shape shape;
    bool full;
    int grid;
    int seg_rows = 0; // ragged: k_cksum_seg row-group size, 0 = flat kernel
    bool lean = false; // aligned strided, one pass per packet: k_cksum_lean
};
Plan plan_strided(const Device &D, const Config &C, uint64_t base, uint64_t stride,
                  uint32_t len, uint64_t n, int kind, bool hdr = false);
Plan plan_ragged(const Device &D, const Config &C, uint64_t n, int kind,
                 bool zero_copy = false, bool hdr = false);
int run(const Device &D, const Config &C, const wc::LaunchArgs &args, const Plan &p,
        hipStream_t st);

// --- wc_rt_rx.cpp -------------------------------------------------------------
hipError_t rx_launch(Device &D, const Config &C, const void *base, const uint64_t *offs,
                     const uint16_t *flens, uint64_t n, uint8_t *verdict, uint64_t *drops,
                     hipStream_t st);

// --- wc_rt_server.cpp ---------------------------------------------------------
constexpr int kSrvFallback = 1; // serve_batch: not served, take the launch path
// One small registered batch through the server (caller holds g_mu, the
// device is current).  Returns kSrvFallback when the server can't take it.
int serve_batch(Device &D, int dev, const uint8_t *dbase, const uint64_t *h_off,
                const uint16_t *h_len, uint64_t n, uint8_t *h_out, int kind,
                uint16_t *h_out2 = nullptr);
void server_stop_all_locked();
// Whether small registered batches may go to the server (not paused).
bool server_enabled_locked();

// --- wc_rt_host.cpp -----------------------------------------------------------
void pipe_free(HostPipe &P);
void zs_free(ZcStream &S);
int pipe_init_locked(HostPipe &P);
const uint8_t *registered_dptr_locked(const void *p, uint64_t bytes);
uint64_t span_of(uint16_t len, int kind);
int out_size(int kind);
int host_zero_copy(Device &D, const uint8_t *dbase, const uint64_t *h_off,
                   const uint16_t *h_len, uint64_t n, uint8_t *h_out, int kind,
                   uint16_t *h_out2 = nullptr);
// Every packet of a host batch inside [0, h_bytes); whether the offsets
// ascend, the bytes the packets' checks read, and (optional) the byte range
// they span.
bool host_batch_ok(const uint8_t *hb, uint64_t h_bytes, const uint64_t *h_off,
                   const uint16_t *h_len, uint64_t n, int kind, bool *ascending, uint64_t *total,
                   uint64_t *range = nullptr);
void shard_range(uint64_t n, int g, int G, uint64_t *lo, uint64_t *hi);

// Pipelined path over one HostPipe on one device (wc_rt_host.cpp): one chunk
// per step(), so a single host thread can interleave the runs of several
// devices (wc_cksum_host_multi).
struct PipeRun {
    Device *D = nullptr;
    HostPipe *P = nullptr;
    int dev = 0;
    const uint8_t *hb = nullptr;
    bool registered = false, ascending = true;
    const uint64_t *h_off = nullptr;
    const uint16_t *h_len = nullptr;
    uint8_t *h_out = nullptr; // out_size(kind) bytes per packet
    uint16_t *h_out2 = nullptr; // fused pair: the header checksums
    int kind = WC_CKSUM_IP;
    uint64_t i = 0, hi = 0;
    uint64_t pend_lo[kPipe] = {}, pend_n[kPipe] = {};
    bool pend[kPipe] = {};
    int slot = 0;

    bool done() const { return i >= hi; }
    uint64_t span(uint64_t j) const;
    int drain(int s);
    int fail(int rc);
    int step();
    int finish();
};

} // namespace rt
} // namespace wc
