// wc_cksum_api.cpp -- the C ABI of libwccksum.so (include/warpcore_gpu/wc_cksum.h).
//
// Host-side runtime around the gfx950 kernels: device selection and
// per-device scratch, the launch planner (group shape + grid), the scalar
// drop-ins for the reference's ip_cksum / payload_cksum
// (/root/reference/lib/src/in_cksum.h:32-36), the device-resident batch calls
// and the pipelined host-memory path.  There is no CPU checksum anywhere in
// this library: if no gfx950 device is usable, batch calls return WC_ENODEV
// and the scalar drop-ins abort (the reference's die(), util.h:280-340).

#include "warpcore_gpu/wc_cksum.h"

#include "wc_cksum_kernels.h"
#include "wc_rccl.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <condition_variable>
#include <functional>
#include <string>
#include <thread>
#include <vector>

namespace {

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
} g_srv_stats;

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
std::mutex g_rx_mu; // rx_launch's tally bookkeeping (batch calls run outside g_mu)

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

FairMutex g_mu;
Device g_dev[kMaxDevices];
// Device d's state is built (set under g_mu once init_locked has finished it,
// cleared by wc_gpu_fini): device-resident batch calls then only copy the
// configuration (g_cfg_mu) and enqueue on the caller's stream, without
// queueing behind a host-memory call that holds g_mu.
std::atomic<bool> g_dev_ready[kMaxDevices];
std::mutex g_cfg_mu; // g_cfg is written with g_mu AND g_cfg_mu held
std::map<uintptr_t, Registration> g_registered; // host base -> region
Config g_cfg;
bool g_cfg_loaded = false;

// Multi-GPU shard executors (wc_gpu_init_multi): shard g runs on device
// g_shard[g].dev with its own host pipeline, so two shards may share a GPU.
struct ShardExec {
    int dev = -1;
    HostPipe pipe;
};
ShardExec g_shard[kMaxDevices];
int g_multi_n = 0;

int hip_err(hipError_t e) { return e == hipSuccess ? WC_OK : -(int)e; }

int env_int(const char *name, int dflt)
{
    const char *v = getenv(name);
    return (v && *v) ? atoi(v) : dflt;
}

uint64_t env_u64(const char *name, uint64_t dflt)
{
    const char *v = getenv(name);
    return (v && *v) ? strtoull(v, nullptr, 0) : dflt;
}

bool parse_shape(const char *v, wc::Shape *sh)
{
    int g = 0, c = 0, u = 0;
    if (!v || !*v || sscanf(v, "%d,%d,%d", &g, &c, &u) != 3)
        return false;
    *sh = {g, c, u};
    return true;
}

void load_config_locked()
{
    Config c;
    // Every knob below only chooses among exact paths (shapes, grids, tile
    // paths, load flavour): results stay bit-identical whatever they say.
    // The two that do not -- WC_VARIANT (experimental kernel branches, one of
    // which drops the result store) and WC_DIAG_NOLOAD (a timing-only build
    // that reads no packet bytes) -- exist only in the tuning build
    // (-DWC_TUNING, libwccksum_tune.so for tools/); the shipped library
    // ignores them.
    c.blocks_per_cu = env_int("WC_BLOCKS_PER_CU", c.blocks_per_cu);
    c.grid = env_int("WC_GRID", c.grid);
#ifdef WC_TUNING
    c.variant = env_int("WC_VARIANT", c.variant);
    c.diag_noload = env_int("WC_DIAG_NOLOAD", c.diag_noload);
#endif
    c.have_shape = parse_shape(getenv("WC_SHAPE"), &c.shape);
    c.have_rshape = parse_shape(getenv("WC_RAGGED_SHAPE"), &c.rshape);
    c.strided_seg = env_int("WC_STRIDED_SEG", c.strided_seg);
    c.flat_un = env_int("WC_FLAT_UN", c.flat_un);
    c.flat_tpw = env_int("WC_FLAT_TPW", c.flat_tpw);
    c.seg = env_int("WC_SEG", c.seg);
    c.seg_rows = env_int("WC_SEG_ROWS", c.seg_rows);
    c.seg_rows_set = getenv("WC_SEG_ROWS") && *getenv("WC_SEG_ROWS");
    c.zc_seg = env_int("WC_ZC_SEG", c.zc_seg);
    c.zc_group_max = env_int("WC_ZC_GROUP_MAX", c.zc_group_max);
    c.zc_bytes = env_int("WC_ZC_BYTES", c.zc_bytes);
    c.flat_min = env_u64("WC_FLAT_MIN", c.flat_min);
    c.nt = env_int("WC_NT", c.nt);
    c.grp_dense = env_int("WC_GRP_DENSE", c.grp_dense);
    c.grp_sparse = env_int("WC_GRP_SPARSE", c.grp_sparse);
    c.grp_rows = env_int("WC_GRP_ROWS", c.grp_rows);
    c.flat_pk = env_int("WC_FLAT_PK", c.flat_pk);
    c.gather = env_int("WC_GATHER", c.gather);
    c.lean_max = env_int("WC_LEAN_MAX", c.lean_max);
    c.split_bytes = env_u64("WC_SPLIT_BYTES", c.split_bytes);
    c.split_pkts = env_u64("WC_SPLIT_PKTS", c.split_pkts);
    c.lean_phase = env_int("WC_LEAN_PHASE", c.lean_phase);
    c.serve = env_int("WC_SERVE", c.serve);
    c.serve_waves = std::max(1, std::min(env_int("WC_SERVE_WAVES", c.serve_waves), 1024));
    c.serve_max = std::max(0, std::min(env_int("WC_SERVE_MAX", c.serve_max), (int)wc::kSrvMaxPkts));
    c.serve_idle_us = std::max(100, env_int("WC_SERVE_IDLE_US", c.serve_idle_us));
    c.serve_prio = env_int("WC_SERVE_PRIO", c.serve_prio) != 0;
    c.rx_early = env_int("WC_RX_EARLY", c.rx_early);
    c.rx_hdrt = env_int("WC_RX_HDRT", c.rx_hdrt);
    c.rx_skip = env_int("WC_RX_SKIP", c.rx_skip);
    c.rx_adapt = env_int("WC_RX_ADAPT", c.rx_adapt);
    c.rx_trace = env_int("WC_RX_TRACE", c.rx_trace);
    c.rx_force = env_int("WC_RX_FORCE", c.rx_force);
    c.rx_grid = std::max(0, env_int("WC_RX_GRID", c.rx_grid));
    {
        std::lock_guard<std::mutex> lk(g_cfg_mu);
        g_cfg = c;
    }
    g_cfg_loaded = true;
}

int current_device(int *dev)
{
    int d = 0;
    hipError_t e = hipGetDevice(&d);
    if (e != hipSuccess)
        return hip_err(e);
    if (d < 0 || d >= kMaxDevices)
        return WC_ENODEV;
    *dev = d;
    return WC_OK;
}

// Create per-device state (caller holds g_mu).
int init_locked(int device, Device **out)
{
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0)
        return WC_ENODEV;
    if (device >= 0) {
        if (device >= ndev || device >= kMaxDevices)
            return WC_EINVAL;
        hipError_t e = hipSetDevice(device);
        if (e != hipSuccess)
            return hip_err(e);
    } else {
        int rc = current_device(&device);
        if (rc)
            return rc;
    }
    if (!g_cfg_loaded)
        load_config_locked();
    Device &D = g_dev[device];
    if (!D.ok) {
        hipDeviceProp_t prop;
        hipError_t e = hipGetDeviceProperties(&prop, device);
        if (e != hipSuccess)
            return hip_err(e);
        if (strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
            fprintf(stderr, "wccksum: device %d is %s, this build targets gfx950\n",
                    device, prop.gcnArchName);
            return WC_ENODEV;
        }
        D.cus = prop.multiProcessorCount;
        int khz = 0;
        if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, device) == hipSuccess &&
            khz > 0)
            D.clock_khz = (uint64_t)khz;
        e = hipStreamCreateWithFlags(&D.scalar_st, hipStreamNonBlocking);
        if (e != hipSuccess)
            return hip_err(e);
        e = hipHostMalloc((void **)&D.h_stage, kScalarStage,
                          hipHostMallocMapped | hipHostMallocCoherent);
        if (e != hipSuccess)
            return WC_ENOMEM;
        e = hipHostMalloc((void **)&D.h_res, 64,
                          hipHostMallocMapped | hipHostMallocCoherent);
        if (e != hipSuccess)
            return WC_ENOMEM;
        if (hipHostGetDevicePointer((void **)&D.d_stage, D.h_stage, 0) != hipSuccess ||
            hipHostGetDevicePointer((void **)&D.d_res, D.h_res, 0) != hipSuccess)
            return WC_ENOMEM;
        for (int k = 0; k < kRxSets; ++k) {
            if (hipHostMalloc((void **)&D.h_rx_tally[k], wc::kRxTallyWords * 4,
                              hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess ||
                hipHostGetDevicePointer((void **)&D.d_rx_tally[k], D.h_rx_tally[k], 0) !=
                    hipSuccess)
                return WC_ENOMEM;
            memset(D.h_rx_tally[k], 0, wc::kRxTallyWords * 4);
        }
        D.ok = true;
        g_dev_ready[device].store(true, std::memory_order_release);
    }
    *out = &D;
    return WC_OK;
}

// The device-resident batch calls' entry: the current device's state and a
// copy of the configuration.  Once the device is set up this takes only the
// configuration lock (held for the copy), never g_mu.
int ensure_device(Device **out, Config *cfg)
{
    int dev = 0;
    if (current_device(&dev) == WC_OK && g_dev_ready[dev].load(std::memory_order_acquire)) {
        *out = &g_dev[dev];
        std::lock_guard<std::mutex> lk(g_cfg_mu);
        *cfg = g_cfg;
        return WC_OK;
    }
    std::lock_guard<FairMutex> lk(g_mu);
    const int rc = init_locked(-1, out);
    if (rc == WC_OK) {
        std::lock_guard<std::mutex> lc(g_cfg_mu);
        *cfg = g_cfg;
    }
    return rc;
}

// ---------------------------------------------------------------------------
// Planner.

wc::Shape shape_for_chunks(uint32_t nch, bool full, bool payload, bool aligned,
                           bool sparse = false)
{
    // Smallest group covering the packet in one pass, with U packets per
    // group so every lane keeps ~4-18 16-byte loads in flight (tuned on
    // MI355X: DESIGN.md section 5, profiles/tune_r01_*.log).
    if (nch <= 4)
        return {4, 1, 4};
    // Sparse batches (stride >= twice the packet's chunk span: netmap slots)
    // run at the rate of the cache lines they touch, one or two per packet;
    // shapes with more lanes per packet reach it (2048-B slots at +14,
    // profiles/ab_r03_slot_shapes.log): ip_cksum 5-6 chunks on 8 x 1 x 4
    // (64 / 72 / 80 B: 36 -> 41, 41 -> 47, 46 -> 52 %).  payload_cksum keeps
    // 4 x 2 x 2 there (8 x 1 x 4: 36 -> 28 %: its header hand-off between
    // lanes costs more the wider the group), and takes it for sparse packets
    // of up to 16 chunks too, even where that is two passes: read from HBM
    // (rotating buffers, round 4) it beats the (8,1,4) / (8,2,4) round 3
    // picked on Infinity-Cache-resident reruns -- 96 B 35.6 -> 27.2 us, 128 B
    // 49.2 -> 44.4, 160 B 49.6 -> 44.3, 200 B 50.0 -> 46.2, 240 B 48.4 ->
    // 45.9 (profiles/ab_r04_payload_small.log).
    if (nch <= 6 || (sparse && payload && nch <= 16))
        return sparse && !payload ? wc::Shape{8, 1, 4} : wc::Shape{4, 2, 2};
    if (nch <= 8)
        return {8, 1, 4};
    // 9..24 chunks: 8 lanes x 3 chunks, two packets per group -- fewer dead
    // lane slots than 16 x 2 (profiles/sweep_r01_mid_shapes.log: 256 B 78.7 -> 84.1 %,
    // 200 B 55 -> 67.5 %, 256 B at +14 50 -> 60 % of HBM peak)
    if (nch <= 16 || (nch <= 24 && !full))
        return {8, 3, 2};
    // aligned unmasked 17..30 chunks: 16 x 2 x 4 (320 B 80.8 -> 85.4 %,
    // profiles/sweep_r02_small_shapes.log)
    if (nch <= 30)
        return {16, 2, 4};
    // ~512 B: 8 lanes x 6 chunks, one packet per group (85 -> 90.8 % packed,
    // 81 -> 87 % in 2048-B slots); 576 B: (16,3,2) (85 -> 86.6 %)
    // (profiles/sweep_r01_mid_shapes.log)
    if (nch <= 34)
        return {8, 6, 1};
    // 35..48 chunks: one packet per 16-lane group when aligned unmasked
    // (704 B 90.5 -> 93.6 %, 576 B 90.7 -> 91.2 %)
    if (nch <= 48)
        return full ? wc::Shape{16, 3, 1} : wc::Shape{16, 3, 2};
    // 49..96 chunks (784..1536 B): 32-lane groups with 2-4 loads per lane
    // beat 16 x 6 for ip_cksum (profiles/sweep_r02_wide_shapes.log: C2
    // 1472 B 88.6-91 -> 93.3-95 %, 1024 B 82 -> 94 %, 2048-B slots at +14
    // +2..5 points).  Aligned unmasked (FULL) batches and masked ones differ
    // below 88 chunks.  payload_cksum (more registers per lane) keeps 16-lane
    // groups, fewer packets per group when aligned
    // (profiles/sweep_r02_payload_shapes.log: C2 payload 84 -> 92.5 %).
    if (payload && nch <= 96) {
        if (aligned)
            return {16, 6, 2};
        return nch <= 80 ? wc::Shape{16, 5, 4} : wc::Shape{32, 3, 2};
    }
    if (nch <= 56)
        return full ? wc::Shape{32, 2, 4} : wc::Shape{16, 5, 4};
    if (nch <= 63)
        return full ? wc::Shape{32, 2, 2} : wc::Shape{16, 5, 4};
    if (nch <= 77)
        return full ? wc::Shape{32, 4, 2} : wc::Shape{32, 3, 2};
    if (nch <= 87)
        return full ? wc::Shape{32, 4, 1} : wc::Shape{32, 4, 2};
    if (nch <= 128)
        return {32, 4, 1};
    if (nch <= 256)
        return {64, 4, 1};
    if (nch <= 576)
        return {32, 18, 1};
    return {64, 9, 1};
}

// Lean-kernel shape: a group whose one pass the packet fills exactly (G *
// CPL == chunks, no dead slots -- a pass the packet does not fill costs the
// masked path: 576 B in (16,3,1) ran at 70 vs 91 %), groups of >= 8 lanes
// (a 4-lane group reads 64-B half lines per load, 128 B in (4,2,2) ran at
// 75 vs 89 % in (8,1,4)) except for 64-B packets, which 4-lane groups read
// as one contiguous kilobyte per load; ~4 loads in flight per lane
// (profiles/ab_r03_lean*.log).  {0,0,0}: no such shape, not lean.  Packets
// under 4 chunks take the masked path of (4, 1, 4).
// Lean-kernel shape for packets at a start phase (PH): one pass covering the
// window, dead slots allowed (they read nothing new and are masked).
wc::Shape lean_ph_shape(uint32_t nch)
{
    if (nch <= 4)
        return {4, 1, 4};
    if (nch <= 8)
        return {8, 1, 4};
    if (nch <= 16)
        return {8, 2, 4};
    if (nch <= 24)
        return {8, 3, 2};
    if (nch <= 32)
        return {16, 2, 2};
    if (nch <= 48)
        return {16, 3, 1};
    return {0, 0, 0};
}

wc::Shape lean_shape_for(uint32_t nch)
{
    if (nch <= 4)
        return {4, 1, 4};
    for (int g = 8; g <= 64; g *= 2) {
        if (nch % (uint32_t)g)
            continue;
        const int cpl = (int)(nch / (uint32_t)g);
        if (cpl > 3)
            continue;
        return {g, cpl, cpl == 1 ? 4 : cpl == 2 ? 2 : (g <= 8 ? 2 : 1)};
    }
    return {0, 0, 0};
}

int grid_for(const Device &D, const Config &C, const wc::Shape &sh, uint64_t n)
{
    const uint64_t ppw = (uint64_t)(64 / sh.group) * sh.unroll;
    const uint64_t waves = (n + ppw - 1) / ppw;
    const uint64_t blocks = (waves + 3) / 4;
    // One-shot grid by default: every block handles one wave-iteration per
    // wave and retires (measured faster than a resident grid-stride loop on
    // MI355X: DESIGN.md section 5).  WC_BLOCKS_PER_CU / WC_GRID cap it into a
    // grid-stride launch for experiments.
    // The kernel grid-strides, so capping at wc::kMaxGridBlocks (gridDim.x *
    // 256 must fit in a uint32) stays correct for any n.
    uint64_t cap = wc::kMaxGridBlocks;
    if (C.blocks_per_cu > 0)
        cap = std::min(cap, (uint64_t)D.cus * (uint64_t)C.blocks_per_cu);
    if (C.grid > 0)
        cap = std::min(cap, (uint64_t)C.grid);
    return (int)std::max<uint64_t>(1, std::min(blocks, cap));
}

struct Plan {
    wc::Shape shape;
    bool full;
    int grid;
    int seg_rows = 0; // ragged: k_cksum_seg row-group size, 0 = flat kernel
    bool lean = false; // aligned strided, one pass per packet: k_cksum_lean
};

bool lean_shape_ok(const wc::Shape &sh)
{
#define WC_SHAPE(G_, C_, U_)                                                   \
    if (sh.group == G_ && sh.cpl == C_ && sh.unroll == U_)                     \
        return true;
    WC_LEAN_SHAPE_LIST
#undef WC_SHAPE
    return false;
}

Plan plan_strided(const Device &D, const Config &C, uint64_t base, uint64_t stride,
                  uint32_t len, uint64_t n, int kind, bool hdr = false)
{
    Plan p;
    const uint32_t span = kind == WC_CKSUM_PAYLOAD ? std::max(len, 20u) : len;
    // Worst-case start phase within a 16-byte chunk over the batch.
    const uint32_t phase = (stride % 16 == 0) ? (uint32_t)(base % 16) : 15u;
    const uint32_t nch = (phase + span + 15u) / 16u;
    p.full = kind == WC_CKSUM_IP && base % 16 == 0 && stride % 16 == 0 &&
             len % 16 == 0 && !(C.variant & 2);
    p.shape = C.have_shape ? C.shape
                           : shape_for_chunks(nch, p.full, kind == WC_CKSUM_PAYLOAD, phase == 0,
                                              stride >= 32ull * nch);
    p.grid = grid_for(D, C, p.shape, n);
    // Packed (or nearly packed) packets that the group kernel would have to
    // mask: the seg kernel streams their byte range instead (k_cksum_seg<STR>)
    // where it measured faster -- a 60-length x 2-offset sweep on MI355X
    // (profiles/sweep_r02_planner.log):
    //   stride % 64 == 0   group kernel (every packet at the same offset in
    //                      its cache lines: 256 B at +14 85 % vs seg 70-73 %)
    //   <= 5 chunks        group kernel
    //   6..14 chunks       seg, 2-row groups (120 B: 74 % vs group 51-56 %)
    //   36..48 chunks      group kernel (550-700 B: 84-89 % vs seg 83-84 %)
    //   >= 90 chunks       group kernel
    //   otherwise          seg, 4-row groups (300 B: 84 % vs group 69 %)
    // Aligned unmasked (FULL) packets of 5..16 chunks at a stride that is not
    // a multiple of 64 take the seg kernel too: the group kernel leaves most
    // of its lane slots dead there (80..240 B packed: 64-77 % vs seg 71-85 %;
    // 64 / 128 / 256 B, whose packets share cache-line phases, keep the
    // group kernel: profiles/sweep_r02_small_aligned.log), 2-row groups up to
    // 9 chunks, 4-row groups above.
    // payload_cksum: packed packets below 64 chunks take the seg kernel at any
    // stride -- it reads the header bytes from its own stream, where the group
    // kernel exchanges them between lanes (64 B 46 -> 56 %, 192 B 54 -> 82 %,
    // 576 B 74-77 -> 83-84 %, 900 B 78 -> 84 %; from 64 chunks on the group
    // kernel's 87-92 % wins: profiles/sweep_r02_payload_seg.log).
    // WC_STRIDED_SEG = 0 never, 2 always (no fused header), 1 = the table;
    // WC_SEG_ROWS forces the row-group size.
    const int sseg = C.strided_seg;
    const bool payload = kind == WC_CKSUM_PAYLOAD;
    const bool packed = len != 0 && stride >= len && stride <= len + len / 8u;
    const bool seg_table =
        payload ? nch < 64
                : stride % 64 != 0 && (p.full ? nch >= 5 && nch <= 16
                                              : nch > 5 && !(nch >= 36 && nch <= 48) && nch < 90);
    if (!hdr && n >= 64 && packed && (sseg == 2 || (sseg == 1 && seg_table))) {
        p.shape = {0, 1, C.flat_un};
        const uint32_t rows2 = payload ? 5u : (p.full ? 9u : 14u);
        p.seg_rows = C.seg_rows_set ? C.seg_rows : (nch <= rows2 ? 2 : 4);
        p.grid = 0;
    }
    // Aligned packets (base, stride and len multiples of 16) that one pass of
    // a group covers take the lean kernel (wc_k_lean.hip): scalar wave
    // addresses, word sums, payload_cksum's header terms from the group's
    // first lane.  payload_cksum needs len >= 48 there (the whole IPv4 /
    // IPv6 header inside the packet); up to WC_LEAN_MAX chunks.
    const bool aligned16 = base % 16 == 0 && stride % 16 == 0 && len % 16 == 0 && len != 0;
    // Sparse payload_cksum packets at one even start phase (netmap slots: IP
    // packets at +14) of up to 18 window chunks take it too, with per-slot
    // byte masks (PH, wc_k_lean.hip): in 2048-B slots at +14, from HBM,
    // payload 64 B 24.2 -> 22.5 us, 128 B 41.3 -> 39.8, 256 B 58.2 -> 56.1
    // against the group kernel, within 1 us of ip_cksum; ip_cksum gains
    // nothing (128 B 39.2 -> 41.2 us) and 576 B loses on both kinds (96.9 ->
    // 112.7 us), so they keep the group kernel (profiles/ab_r05_lean_phase.log).
    const bool phased = !aligned16 && C.lean_phase && C.nt && stride % 16 == 0 &&
                        base % 2 == 0 && len != 0 && !packed && sseg != 2 && payload &&
                        nch <= 18;
    if (!hdr && C.lean_max > 0 && (aligned16 || phased) && (!payload || len >= 48) &&
        nch <= (uint32_t)C.lean_max && (sseg != 2 || !packed)) {
        const wc::Shape sh = C.have_shape ? C.shape : aligned16 ? lean_shape_for(nch)
                                                                 : lean_ph_shape(nch);
        const uint64_t ppw = (uint64_t)(64 / std::max(sh.group, 1)) * sh.unroll;
        if (lean_shape_ok(sh) && nch <= (uint32_t)(sh.group * sh.cpl) && ppw <= 64 &&
            ppw * stride < (1ull << 32)) {
            p.shape = sh;
            p.lean = true;
            p.seg_rows = 0;
            p.grid = grid_for(D, C, sh, n);
        }
    }
    return p;
}

// Ragged batches take the segmented-prefix kernel k_cksum_seg (both kinds):
// dense tiles stream their byte range, sparse ones take its flat path
// (DESIGN.md section 4.4), the fused header pass (out_hdr) included (group =
// 0 marks both the seg and the flat kernel; unroll = 64-chunk rows per
// ping-pong group of the flat path, WC_FLAT_UN).  WC_SEG = 0 forces the flat
// kernel; WC_SEG_ROWS = 2 / 4 / 8 rows per seg row group.  A host zero-copy batch of
// at most kZcGroupMax packets takes the ragged group kernel instead: a flat
// wave walks its 64-packet tile's rows one PCIe latency at a time, the group
// kernel issues every packet's loads at once.  (Device-resident batches
// measured no better on the group kernel at any size -- launch cost
// dominates small ones -- so WC_FLAT_MIN defaults to 0.)
Plan plan_ragged(const Device &D, const Config &C, uint64_t n, int kind,
                 bool zero_copy = false, bool hdr = false)
{
    (void)D;
    Plan p;
    p.full = false;
    const bool small = (zero_copy && n <= (uint64_t)C.zc_group_max) ||
                       n < C.flat_min;
    if (small && !hdr) {
        p.shape = C.have_rshape ? C.rshape : wc::Shape{64, 2, 1};
        const uint64_t ppw = (uint64_t)(64 / p.shape.group) * p.shape.unroll;
        p.grid = (int)std::min<uint64_t>(
            wc::kMaxGridBlocks, std::max<uint64_t>(1, ((n + ppw - 1) / ppw + 3) / 4));
        return p;
    }
    p.shape = {0, 1, C.flat_un};
    p.grid = 0;
    if ((!zero_copy || C.zc_seg) && C.diag_noload == 0 && C.seg != 0 &&
        (!hdr || kind == WC_CKSUM_PAYLOAD))
        p.seg_rows = C.seg_rows;
    return p;
}

int run(const Device &D, const Config &C, const wc::LaunchArgs &args, const Plan &p,
        hipStream_t st)
{
    (void)D;
    wc::LaunchArgs a = args;
    a.seg_rows = p.seg_rows;
    a.grp_thr = C.grp_dense | (C.grp_sparse << 8);
    a.grp_rows = C.grp_rows;
    a.flat_pk = C.flat_pk;
    a.gather = C.gather;
    hipError_t e = p.lean              ? wc::launch_lean(a, p.shape, p.grid, st)
                   : p.shape.group == 0 ? wc::launch_flat(a, p.shape.unroll, st)
                                        : wc::launch_cksum(a, p.shape, p.grid, st);
    return hip_err(e);
}

int batch_strided(const void *d_base, uint64_t stride, uint16_t len, uint64_t n,
                  uint16_t *d_out, uint64_t *d_bad, int kind, void *stream,
                  uint16_t *d_out_hdr = nullptr)
{
    if (kind != WC_CKSUM_IP && kind != WC_CKSUM_PAYLOAD)
        return WC_EINVAL;
    if (n == 0)
        return WC_OK;
    if (!d_base || (!d_out && !d_bad))
        return WC_EINVAL;
    Device *D = nullptr;
    Config C;
    int rc = ensure_device(&D, &C);
    if (rc)
        return rc;
    // A batch larger than the piece runs as back-to-back launches of it on
    // the same stream, each planned on its own (Config::split_bytes).
    uint64_t piece = n;
    if (C.split_pkts)
        piece = std::min(n, C.split_pkts);
    else if (C.split_bytes && stride)
        piece = std::min(n, std::max<uint64_t>(1, C.split_bytes / stride));
    for (uint64_t p0 = 0; p0 < n; p0 += piece) {
        const uint64_t cnt = std::min(piece, n - p0);
        const uint8_t *b = (const uint8_t *)d_base + p0 * stride;
        const Plan p = plan_strided(*D, C, (uint64_t)b, stride, len, cnt, kind, d_out_hdr != nullptr);
        wc::LaunchArgs a{b,      stride, len,  nullptr,  nullptr, cnt,
                         d_out ? d_out + p0 : nullptr,  d_bad,  kind, false,    p.full,  C.nt != 0,
                         0,      d_out_hdr ? d_out_hdr + p0 : nullptr};
        a.variant = C.variant;
        rc = run(*D, C, a, p, (hipStream_t)stream);
        if (rc)
            return rc;
    }
    return WC_OK;
}

int batch_ragged(const void *d_base, const uint64_t *d_off, const uint16_t *d_len,
                 uint64_t n, uint16_t *d_out, uint64_t *d_bad, int kind,
                 void *stream, uint16_t *d_out_hdr = nullptr)
{
    if (kind != WC_CKSUM_IP && kind != WC_CKSUM_PAYLOAD)
        return WC_EINVAL;
    if (n == 0)
        return WC_OK;
    if (!d_base || !d_off || !d_len || (!d_out && !d_bad))
        return WC_EINVAL;
    Device *D = nullptr;
    Config C;
    int rc = ensure_device(&D, &C);
    if (rc)
        return rc;
    const uint64_t piece = C.split_pkts && n > C.split_pkts ? C.split_pkts : n;
    for (uint64_t p0 = 0; p0 < n; p0 += piece) {
        const uint64_t cnt = std::min(piece, n - p0);
        const Plan p = plan_ragged(*D, C, cnt, kind, false, d_out_hdr != nullptr);
        wc::LaunchArgs a{d_base, 0,     0,    d_off + p0, d_len + p0, cnt,
                         d_out ? d_out + p0 : nullptr,  d_bad, kind, true,  false, C.nt != 0,
                         C.flat_tpw, d_out_hdr ? d_out_hdr + p0 : nullptr, C.diag_noload != 0};
        a.variant = C.variant;
        rc = run(*D, C, a, p, (hipStream_t)stream);
        if (rc)
            return rc;
    }
    return WC_OK;
}

[[noreturn]] void die(const char *what, int rc)
{
    fprintf(stderr, "wccksum: %s failed: %s (%d)\n", what, wc_strerror(rc), rc);
    abort();
}

uint16_t scalar_cksum(const void *buf, uint16_t len, int kind, const char *who)
{
    std::lock_guard<FairMutex> lk(g_mu);
    Device *D = nullptr;
    int rc = init_locked(-1, &D);
    if (rc)
        die(who, rc);
    // payload_cksum reads the IPv4 header fields up to byte 19 whatever len is
    // (in_cksum.c:149-151); stage the same bytes the reference reads.
    const size_t span =
        kind == WC_CKSUM_PAYLOAD ? std::max<size_t>(len, 20) : (size_t)len;
    memcpy(D->h_stage, buf, span);
    // (the load flavour the planner assumed: the lean kernel's phase path,
    // which a 1-packet batch at an even staging phase may take, exists with
    // nontemporal loads only)
    Plan p = plan_strided(*D, g_cfg, (uint64_t)D->d_stage, 0, len, 1, kind);
    wc::LaunchArgs a{D->d_stage, 0,   len,  nullptr, nullptr, 1,
                     D->d_res,   nullptr, kind, false,   p.full,  g_cfg.nt != 0};
    rc = run(*D, g_cfg, a, p, D->scalar_st);
    if (rc)
        die(who, rc);
    hipError_t e = hipStreamSynchronize(D->scalar_st);
    if (e != hipSuccess)
        die(who, hip_err(e));
    return *(volatile uint16_t *)D->h_res;
}

// ---------------------------------------------------------------------------
// Host-memory pipeline.

// Frees whatever a (possibly partly built) pipeline holds.
void pipe_free(HostPipe &P)
{
    for (int s = 0; s < kPipe; ++s) {
        if (P.st[s])
            (void)hipStreamSynchronize(P.st[s]);
        (void)hipFree(P.d_bytes[s]);
        (void)hipFree(P.d_off[s]);
        (void)hipFree(P.d_len[s]);
        (void)hipFree(P.d_out[s]);
        (void)hipFree(P.d_out2[s]);
        (void)hipHostFree(P.h_bytes[s]);
        (void)hipHostFree(P.h_off[s]);
        (void)hipHostFree(P.h_len[s]);
        (void)hipHostFree(P.h_out[s]);
        (void)hipHostFree(P.h_out2[s]);
        if (P.done[s])
            (void)hipEventDestroy(P.done[s]);
        if (P.st[s])
            (void)hipStreamDestroy(P.st[s]);
    }
    P = HostPipe{};
}

// Streams, events and staging of one host pipeline, created on the current
// device.
int pipe_init_locked(HostPipe &P)
{
    if (P.ready)
        return WC_OK;
    for (int s = 0; s < kPipe; ++s) {
        if (hipStreamCreateWithFlags(&P.st[s], hipStreamNonBlocking) != hipSuccess ||
            hipEventCreateWithFlags(&P.done[s], hipEventDisableTiming) != hipSuccess ||
            hipMalloc((void **)&P.d_bytes[s], kChunkBytes + 64) != hipSuccess ||
            hipMalloc((void **)&P.d_off[s], kChunkPkts * 8) != hipSuccess ||
            hipMalloc((void **)&P.d_len[s], kChunkPkts * 2) != hipSuccess ||
            hipMalloc((void **)&P.d_out[s], kChunkPkts * 2) != hipSuccess ||
            hipMalloc((void **)&P.d_out2[s], kChunkPkts * 2) != hipSuccess ||
            hipHostMalloc((void **)&P.h_bytes[s], kChunkBytes + 64, 0) != hipSuccess ||
            hipHostMalloc((void **)&P.h_off[s], kChunkPkts * 8, 0) != hipSuccess ||
            hipHostMalloc((void **)&P.h_len[s], kChunkPkts * 2, 0) != hipSuccess ||
            hipHostMalloc((void **)&P.h_out[s], kChunkPkts * 2, 0) != hipSuccess ||
            hipHostMalloc((void **)&P.h_out2[s], kChunkPkts * 2, 0) != hipSuccess) {
            pipe_free(P);
            return WC_ENOMEM;
        }
    }
    P.ready = true;
    return WC_OK;
}

int zc_init_locked(Device &D)
{
    ZeroCopy &Z = D.zc;
    if (Z.ready)
        return WC_OK;
    const unsigned fl = hipHostMallocMapped | hipHostMallocCoherent;
    if (hipStreamCreateWithFlags(&Z.st, hipStreamNonBlocking) != hipSuccess ||
        hipHostMalloc((void **)&Z.h_off, kZcPkts * 8, fl) != hipSuccess ||
        hipHostMalloc((void **)&Z.h_len, kZcPkts * 2, fl) != hipSuccess ||
        hipHostMalloc((void **)&Z.h_out, kZcPkts * 2, fl) != hipSuccess ||
        hipHostMalloc((void **)&Z.h_out2, kZcPkts * 2, fl) != hipSuccess ||
        hipHostGetDevicePointer((void **)&Z.d_off, Z.h_off, 0) != hipSuccess ||
        hipHostGetDevicePointer((void **)&Z.d_len, Z.h_len, 0) != hipSuccess ||
        hipHostGetDevicePointer((void **)&Z.d_out, Z.h_out, 0) != hipSuccess ||
        hipHostGetDevicePointer((void **)&Z.d_out2, Z.h_out2, 0) != hipSuccess)
        return WC_ENOMEM;
    Z.ready = true;
    return WC_OK;
}

// Address on the CURRENT device of host range [p, p + bytes) if it lies
// inside one registered region, else nullptr.  The region was registered
// portable and mapped; its device address is looked up for this device the
// first time (a batch may run on a shard device other than the one current
// at wc_host_register).
const uint8_t *registered_dptr_locked(const void *p, uint64_t bytes)
{
    const uintptr_t a = (uintptr_t)p;
    auto it = g_registered.upper_bound(a);
    if (it == g_registered.begin())
        return nullptr;
    --it;
    if (a < it->first || a + bytes > it->first + it->second.bytes)
        return nullptr;
    int dev = 0;
    if (current_device(&dev) != WC_OK)
        return nullptr;
    const uint8_t *&d = it->second.dptr[dev];
    if (!d) {
        void *dp = nullptr;
        if (hipHostGetDevicePointer(&dp, (void *)it->first, 0) != hipSuccess)
            return nullptr;
        d = (const uint8_t *)dp;
    }
    return d + (a - it->first);
}

// Bytes the reference reads for one packet (payload_cksum reads the IPv4
// header fields up to byte 19 whatever len is, in_cksum.c:149-151).
uint64_t span_of(uint16_t len, int kind)
{
    return kind == WC_CKSUM_PAYLOAD || kind == kKindFused ? std::max<uint64_t>(len, 20) : len;
}

// Bytes the fused TX pair reads of the packet at p (whose first
// span_of(len, kKindFused) bytes are known to be readable): payload_cksum's,
// and the IPv4 header's hl bytes ip_cksum sums (ip4.c:184-186) when they run
// past them (options behind a short len).
uint64_t fused_span(const uint8_t *p, uint16_t len)
{
    const uint64_t s = span_of(len, kKindFused);
    return (p[0] >> 4) == 4 ? std::max<uint64_t>(s, (uint64_t)(p[0] & 15u) * 4u) : s;
}

// Result bytes per packet in the main result array: a uint16 checksum, or a
// uint8 RX verdict.
int out_size(int kind) { return kind == kKindRx ? 1 : 2; }

// One RX verdict launch.  ADAPT (the default): EARLY or HT by the newest
// earlier launch on this device whose tally has arrived (>= 8 sampled tiles,
// or all it will write): EARLY when more than 1 in 8 of its sampled frames
// needed no UDP check (ARP / ICMP / TCP / zero checksums / drops), else HT;
// the previous choice stands until a tally arrives.  The kernel's tally is a
// store per 64 tiles into mapped host memory -- nothing to wait for here,
// and launches stay asynchronous (a tally read while its launch still runs
// is a partial sample).
hipError_t rx_launch(Device &D, const Config &C, const void *base, const uint64_t *offs,
                     const uint16_t *flens, uint64_t n, uint8_t *verdict, uint64_t *drops,
                     hipStream_t st)
{
    const int mode = C.rx_mode();
    if (!(mode & wc::kRxAdapt) || !D.h_rx_tally[0])
        return wc::launch_rx_verdict(base, offs, flens, n, verdict, drops, C.nt != 0, st, mode,
                                     nullptr, 0u, C.rx_grid);
    std::lock_guard<std::mutex> lk(g_rx_mu);
    const auto t0 = std::chrono::steady_clock::now();
    uint32_t from = 0, from_words = 0, from_seen = 0, from_out = 0;
    for (uint32_t back = 1; back < (uint32_t)kRxSets && back <= D.rx_gen; ++back) {
        const uint32_t g = D.rx_gen - back;
        const int set = (int)(g % kRxSets);
        const volatile uint32_t *t = D.h_rx_tally[set];
        uint32_t words = 0, seen = 0, out = 0;
        for (uint32_t i = 0; i < D.rx_words[set]; ++i) {
            const uint32_t w = t[i];
            if ((w >> 16) != (g & 0xFFFFu))
                continue;
            ++words;
            seen += w & 0xFFu;
            out += (w >> 8) & 0xFFu;
        }
        if (words >= 8 || (words && words == D.rx_words[set])) {
            D.rx_early = out * 8u > seen;
            from = g;
            from_words = words;
            from_seen = seen;
            from_out = out;
            break;
        }
    }
    const uint32_t g = ++D.rx_gen;
    const int set = (int)(g % kRxSets);
    const uint64_t tiles = (n + 63) / 64;
    const uint32_t words = (uint32_t)std::min<uint64_t>((tiles + 63) / 64, wc::kRxTallyWords);
    // cleared first: a word older launches left there could carry this
    // launch's 16-bit tag once the tags come round (a late store of launch
    // g - 4 after the clear carries g - 4's tag and is not counted)
    memset(D.h_rx_tally[set], 0, words * 4u);
    D.rx_words[set] = words;
    if (C.rx_force) // (tools: the tallying kernel with the decision fixed)
        D.rx_early = C.rx_force == 2;
    const int m = wc::kRxHdrT | (D.rx_early ? wc::kRxEarly : 0);
    if (C.rx_trace == 2) { // one summary line per 512 launches
        ++D.rx_nlaunch[D.rx_early ? 1 : 0];
        D.rx_ndecided += from_words != 0;
        if ((g & 511u) == 0) {
            fprintf(stderr, "wccksum rx gen %u: last 512 launches %u HT / %u EARLY, %u decided "
                            "from an arrived tally\n",
                    g, D.rx_nlaunch[0], D.rx_nlaunch[1], D.rx_ndecided);
            D.rx_nlaunch[0] = D.rx_nlaunch[1] = D.rx_ndecided = 0;
        }
    } else if (C.rx_trace)
        fprintf(stderr, "wccksum rx gen %u: %s (tally of gen %u: %u words, %u of %u frames ruled "
                        "out; %.1f us on the host)\n",
                g, D.rx_early ? "EARLY" : "HT", from, from_words, from_out, from_seen,
                std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0)
                    .count());
    return wc::launch_rx_verdict(base, offs, flens, n, verdict, drops, C.nt != 0, st, m,
                                 D.d_rx_tally[set], g & 0xFFFFu, C.rx_grid);
}

// One device launch over a ragged batch of `kind` (a checksum kind, RX
// verdicts -- lengths are frame lengths --, or the fused pair, whose header
// checksums go to d_out_hdr).
int run_ragged_any(Device &D, const Config &C, const uint8_t *d_base, const uint64_t *d_off,
                   const uint16_t *d_len, uint64_t n, void *d_out, int kind, bool zero_copy,
                   hipStream_t st, uint16_t *d_out_hdr = nullptr)
{
    if (kind == kKindRx)
        return hip_err(rx_launch(D, C, d_base, d_off, d_len, n, (uint8_t *)d_out, nullptr, st));
    const bool fused = kind == kKindFused;
    const int k = fused ? WC_CKSUM_PAYLOAD : kind;
    const Plan p = plan_ragged(D, C, n, k, zero_copy, fused);
    wc::LaunchArgs a{d_base, 0,       0,    d_off, d_len, n,
                     (uint16_t *)d_out, nullptr, k, true,  false, C.nt != 0,
                     C.flat_tpw, fused ? d_out_hdr : nullptr};
    return run(D, C, a, p, st);
}

// ---------------------------------------------------------------------------
// The resident small-batch server (wc_k_serve.hip).  A small batch in a
// registered region is answered by a persistent grid that polls request
// records in mapped pinned memory: no launch, no stream synchronisation, no
// copy per call.  The grid is started by the first such call, kept while
// calls keep coming, and stopped (stop flag in every record, then the stream
// drained) by the idle watcher after WC_SERVE_IDLE_US without a call, by
// wc_gpu_fini, or at process exit -- so it never outlives its process.  If it
// ever fails to answer, the call falls back to the zero-copy launch and the
// server stays off for the process.

constexpr int kSrvFallback = 1; // serve_batch: not served, take the launch path
constexpr uint64_t kSrvSafetyMs = 4000; // the grid drains itself after this idle time

std::atomic<bool> g_srv_quit{false};
std::thread g_srv_watcher;
bool g_srv_hooks = false; // watcher started, atexit registered

// The grid's stream must not share a hardware queue with other work.  HIP
// maps a process's streams onto a few shared hardware queues per priority
// level (GPU_MAX_HW_QUEUES, 4 here), and a queue runs its commands in order:
// every kernel or copy of another stream that lands on the grid's queue waits
// until the grid leaves -- and the idle watcher that stops it needs g_mu,
// which a host call waiting for such a kernel holds, so the wait lasted until
// the grid's own 4-s drain (tests/c/thread_engines.c: 2-3 host calls per
// engine in 8 s).  The grid's stream takes the highest priority, whose queues
// are not shared with normal-priority streams (the library's own and, by
// default, the caller's); it stays non-blocking, so work on the null stream
// (torch's default) never waits for the grid either.  (A CU-masked stream
// would get a queue of its own too, but HIP creates those as blocking
// streams.)
hipError_t server_stream_create(hipStream_t *st)
{
    int least = 0, greatest = 0;
    if (g_cfg.serve_prio && hipDeviceGetStreamPriorityRange(&least, &greatest) == hipSuccess &&
        greatest != least)
        return hipStreamCreateWithPriority(st, hipStreamNonBlocking, greatest);
    return hipStreamCreateWithFlags(st, hipStreamNonBlocking);
}

int server_init_locked(Device &D)
{
    Server &S = D.srv;
    if (S.ready)
        return WC_OK;
    const unsigned fl = hipHostMallocMapped | hipHostMallocCoherent;
    if (server_stream_create(&S.st) != hipSuccess ||
        hipHostMalloc((void **)&S.h_rec, wc::kSrvMaxPkts * sizeof(wc::SrvRec), fl) != hipSuccess ||
        hipHostMalloc((void **)&S.h_res, wc::kSrvMaxPkts * sizeof(wc::SrvRes), fl) != hipSuccess ||
        hipHostMalloc((void **)&S.h_hb, 64, fl) != hipSuccess ||
        hipHostGetDevicePointer((void **)&S.d_rec, S.h_rec, 0) != hipSuccess ||
        hipHostGetDevicePointer((void **)&S.d_res, S.h_res, 0) != hipSuccess ||
        hipHostGetDevicePointer((void **)&S.d_hb, S.h_hb, 0) != hipSuccess)
        return WC_ENOMEM;
    memset(S.h_rec, 0, wc::kSrvMaxPkts * sizeof(wc::SrvRec));
    memset((void *)S.h_res, 0, wc::kSrvMaxPkts * sizeof(wc::SrvRes));
    memset(S.h_hb, 0, 64);
    S.ready = true;
    return WC_OK;
}

// Launch the grid with every record rewritten to {S.seq, no stop} first:
// nothing pending, stop flags cleared, the heartbeat at S.seq.
int server_launch_locked(Device &D)
{
    Server &S = D.srv;
    for (uint32_t k = 0; k < wc::kSrvMaxPkts; ++k) {
        S.h_rec[k].addr = 0;
        S.h_rec[k].info = 0;
        __atomic_store_n(&S.h_rec[k].seq, S.seq, __ATOMIC_RELEASE);
    }
    __atomic_store_n(S.h_hb, S.seq, __ATOMIC_RELEASE);
    const uint64_t idle_ticks = kSrvSafetyMs * D.clock_khz;
    const hipError_t e =
        wc::launch_serve(S.d_rec, S.d_res, S.d_hb, S.seq, S.waves, idle_ticks, S.st);
    if (e != hipSuccess)
        return hip_err(e);
    S.running = true;
    S.posted = std::chrono::steady_clock::now();
    ++g_srv_stats.launches;
    return WC_OK;
}

// Stop flag in every polled record, then wait for the grid to drain.
void server_stop_locked(Device &D, int dev)
{
    Server &S = D.srv;
    if (!S.running)
        return;
    for (int k = 0; k < S.waves && k < (int)wc::kSrvMaxPkts; ++k)
        __atomic_store_n(&S.h_rec[k].info, 1u << 24, __ATOMIC_RELEASE);
    int cur = -1;
    (void)hipGetDevice(&cur);
    (void)hipSetDevice(dev);
    (void)hipStreamSynchronize(S.st);
    if (cur >= 0)
        (void)hipSetDevice(cur);
    S.running = false;
}

void server_stop_all_locked()
{
    for (int d = 0; d < kMaxDevices; ++d)
        if (g_dev[d].ok && g_dev[d].srv.running)
            server_stop_locked(g_dev[d], d);
}

void server_watch()
{
    while (!g_srv_quit.load()) {
        std::this_thread::sleep_for(std::chrono::milliseconds(2));
        std::lock_guard<FairMutex> lk(g_mu);
        const auto now = std::chrono::steady_clock::now();
        for (int d = 0; d < kMaxDevices; ++d) {
            Device &D = g_dev[d];
            if (D.ok && D.srv.running &&
                now - D.srv.last > std::chrono::microseconds(g_cfg.serve_idle_us))
                server_stop_locked(D, d);
        }
    }
}

void server_atexit()
{
    g_srv_quit.store(true);
    if (g_srv_watcher.joinable())
        g_srv_watcher.join();
    std::lock_guard<FairMutex> lk(g_mu);
    server_stop_all_locked();
}

// The next request number (0 is the records' initial value: never used).
uint32_t server_next_seq(Server &S)
{
    S.seq = S.seq + 1 == 0 ? 1 : S.seq + 1;
    return S.seq;
}

// Post request `seq`: the heartbeat first, then one record per packet, last
// packet first -- a wave that sees its first record current finds every
// later one of the request current too (stores become visible in program
// order).
void server_post(Server &S, uint32_t seq, const uint8_t *dbase, const uint64_t *h_off,
                 const uint16_t *h_len, uint64_t n, uint32_t rkind)
{
    __atomic_store_n(S.h_hb, seq, __ATOMIC_RELEASE);
    for (uint64_t k = n; k-- > 0;) {
        wc::SrvRec &r = S.h_rec[k];
        r.addr = (uint64_t)(dbase + h_off[k]) | (n << wc::kSrvAddrBits);
        r.info = (uint32_t)h_len[k] | (rkind << 16);
        __atomic_store_n(&r.seq, seq, __ATOMIC_RELEASE);
    }
    S.posted = std::chrono::steady_clock::now();
}

// One small registered batch through the server (caller holds g_mu, the
// device is current).  Returns kSrvFallback when the server can't take it.
// h_out2: the fused pair's header checksums (kind kKindFused).
int serve_batch(Device &D, int dev, const uint8_t *dbase, const uint64_t *h_off,
                const uint16_t *h_len, uint64_t n, uint8_t *h_out, int kind,
                uint16_t *h_out2 = nullptr)
{
    Server &S = D.srv;
    if (S.broken) {
        ++g_srv_stats.fallbacks;
        return kSrvFallback;
    }
    // The record packs the count above a 48-bit address: every packet's
    // (offsets come in any order).
    for (uint64_t k = 0; k < n; ++k)
        if ((uint64_t)dbase + h_off[k] >= (1ull << wc::kSrvAddrBits)) {
            ++g_srv_stats.fallbacks;
            return kSrvFallback;
        }
    int rc = server_init_locked(D);
    if (rc)
        return rc;
    if (!g_srv_hooks) {
        g_srv_hooks = true;
        g_srv_watcher = std::thread(server_watch);
        std::atexit(server_atexit);
    }
    // A grid left without a request for half its own drain time is stopped
    // and started afresh: it may be about to leave (each wave leaves once
    // kSrvSafetyMs passed without a request it or the heartbeat showed), and
    // a request posted to a grid that is half gone would not be answered in
    // full.  (The idle watcher normally stops it within WC_SERVE_IDLE_US.)
    if (S.running && std::chrono::steady_clock::now() - S.posted >
                         std::chrono::milliseconds(kSrvSafetyMs / 2))
        server_stop_locked(D, dev);
    if (!S.running) {
        S.waves = g_cfg.serve_waves;
        rc = server_launch_locked(D);
        if (rc)
            return rc;
    }
    const uint32_t rkind = kind == kKindRx      ? wc::kSrvKindRx
                           : kind == kKindFused ? wc::kSrvKindFused
                                                : (uint32_t)kind;
    uint32_t seq = server_next_seq(S);
    server_post(S, seq, dbase, h_off, h_len, n, rkind);
    auto t0 = std::chrono::steady_clock::now();
    bool relaunched = false;
    for (uint64_t k = 0; k < n; ++k) {
        for (uint32_t spin = 1;; ++spin) {
            if (__atomic_load_n(&S.h_res[k].seq, __ATOMIC_ACQUIRE) == seq)
                break;
            __builtin_ia32_pause();
            if (spin % 4096)
                continue;
            const auto dt = std::chrono::steady_clock::now() - t0;
            if (dt > std::chrono::milliseconds(50) && !relaunched &&
                hipStreamQuery(S.st) == hipSuccess) {
                // The grid is gone (it cannot leave part-way: see above):
                // start it afresh -- every record reset, so no wave takes a
                // stale record for a request -- and post the batch again.
                relaunched = true;
                S.running = false;
                rc = server_launch_locked(D);
                if (rc)
                    return rc;
                seq = server_next_seq(S);
                server_post(S, seq, dbase, h_off, h_len, n, rkind);
                t0 = std::chrono::steady_clock::now();
                k = 0;
                spin = 0;
                continue;
            }
            if (dt > std::chrono::milliseconds(2000)) {
                fprintf(stderr, "wccksum: resident server did not answer; using launches\n");
                server_stop_locked(D, dev);
                S.broken = true;
                ++g_srv_stats.fallbacks;
                return kSrvFallback;
            }
        }
    }
    if (kind == kKindRx) {
        for (uint64_t k = 0; k < n; ++k)
            h_out[k] = (uint8_t)S.h_res[k].value;
    } else {
        uint16_t *o = (uint16_t *)h_out;
        for (uint64_t k = 0; k < n; ++k)
            o[k] = (uint16_t)S.h_res[k].value;
        if (kind == kKindFused)
            for (uint64_t k = 0; k < n; ++k)
                h_out2[k] = (uint16_t)(S.h_res[k].value >> 16);
    }
    S.last = std::chrono::steady_clock::now();
    ++g_srv_stats.served;
    return WC_OK;
}

// Small registered batch: one launch reading host memory in place.
int host_zero_copy(Device &D, const uint8_t *dbase, const uint64_t *h_off,
                   const uint16_t *h_len, uint64_t n, uint8_t *h_out, int kind,
                   uint16_t *h_out2 = nullptr)
{
    int rc = zc_init_locked(D);
    if (rc)
        return rc;
    ZeroCopy &Z = D.zc;
    memcpy(Z.h_off, h_off, n * 8);
    memcpy(Z.h_len, h_len, n * 2);
    rc = run_ragged_any(D, g_cfg, dbase, Z.d_off, Z.d_len, n, Z.d_out, kind, true, Z.st,
                        Z.d_out2);
    if (rc)
        return rc;
    hipError_t e = hipStreamSynchronize(Z.st);
    if (e != hipSuccess)
        return hip_err(e);
    memcpy(h_out, (const void *)Z.h_out, n * out_size(kind));
    if (kind == kKindFused)
        memcpy(h_out2, (const void *)Z.h_out2, n * 2);
    return WC_OK;
}

// Library-owned staging workers.  Pageable input reaches the GPU through
// the pinned staging ring, and copying it there was the end-to-end path's
// limit on one thread (24.6-28.9 GB/s against ~55 GB/s for DMA from
// registered memory) -- for every shard of
// wc_cksum_host_multi alike, since the engine thread stages them all.  The
// copy of each chunk is split over W workers plus the calling thread
// (WC_STAGE_THREADS, default min(8, cores - 1); 0 = the calling thread
// alone).  Created at the first pageable chunk, joined at exit.
class StagePool {
public:
    explicit StagePool(int workers)
    {
        for (int i = 0; i < workers; ++i)
            th_.emplace_back([this] { loop(); });
    }
    ~StagePool()
    {
        {
            std::lock_guard<std::mutex> lk(mu_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto &t : th_)
            t.join();
    }
    int width() const { return (int)th_.size() + 1; }
    // fn(0) .. fn(parts - 1), the calling thread taking its share; returns
    // when all are done.
    void run(int parts, const std::function<void(int)> &fn)
    {
        if (parts <= 1 || th_.empty()) {
            for (int i = 0; i < parts; ++i)
                fn(i);
            return;
        }
        std::unique_lock<std::mutex> lk(mu_);
        job_ = &fn;
        parts_ = parts;
        next_ = 0;
        pending_ = parts;
        ++gen_;
        cv_.notify_all();
        while (next_ < parts_) {
            const int i = next_++;
            lk.unlock();
            fn(i);
            lk.lock();
            --pending_;
        }
        done_.wait(lk, [this] { return pending_ == 0; });
        job_ = nullptr;
    }

private:
    void loop()
    {
        uint64_t seen = 0;
        std::unique_lock<std::mutex> lk(mu_);
        for (;;) {
            cv_.wait(lk, [&] { return stop_ || (gen_ != seen && job_ && next_ < parts_); });
            if (stop_)
                return;
            seen = gen_;
            while (job_ && next_ < parts_) {
                const int i = next_++;
                const std::function<void(int)> *fn = job_;
                lk.unlock();
                (*fn)(i);
                lk.lock();
                if (--pending_ == 0)
                    done_.notify_all();
            }
        }
    }
    std::vector<std::thread> th_;
    std::mutex mu_;
    std::condition_variable cv_, done_;
    const std::function<void(int)> *job_ = nullptr;
    int parts_ = 0, next_ = 0, pending_ = 0;
    uint64_t gen_ = 0;
    bool stop_ = false;
};

StagePool &stage_pool()
{
    static StagePool pool([] {
        const char *v = getenv("WC_STAGE_THREADS");
        if (v && *v)
            return std::max(0, atoi(v));
        const int hw = (int)std::thread::hardware_concurrency();
        return std::max(0, std::min(8, hw - 1));
    }());
    return pool;
}

// memcpy of `bytes` split over the staging pool (pieces of >= 2 MiB).
void stage_copy(void *dst, const void *src, uint64_t bytes)
{
    StagePool &P = stage_pool();
    constexpr uint64_t kPiece = 2ull << 20;
    const int parts = (int)std::min<uint64_t>((uint64_t)P.width(), (bytes + kPiece - 1) / kPiece);
    if (parts <= 1) {
        memcpy(dst, src, bytes);
        return;
    }
    const uint64_t step = ((bytes + parts - 1) / parts + 63) & ~63ull;
    P.run(parts, [&](int i) {
        const uint64_t lo = std::min(bytes, (uint64_t)i * step);
        const uint64_t hi = std::min(bytes, lo + step);
        memcpy((uint8_t *)dst + lo, (const uint8_t *)src + lo, hi - lo);
    });
}

// Pipelined path: chunks of packets go through kPipe streams, each chunk
// H2D -> kernel -> D2H.  An ascending batch ships the byte range its chunk
// covers (straight from registered memory, else via pinned staging); any
// other order is gathered packet by packet into pinned staging first.
//
// A PipeRun walks packets [i, hi) of a batch through one HostPipe on one
// device, one chunk per step(), so a single host thread can interleave the
// runs of several devices (wc_cksum_host_multi): while it stages device g's
// next chunk, the other devices' copies and kernels are in flight.
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

    // Bytes packet j's check reads (the fused pair: also its IPv4 header).
    uint64_t span(uint64_t j) const
    {
        return kind == kKindFused ? fused_span(hb + h_off[j], h_len[j]) : span_of(h_len[j], kind);
    }

    // Wait for a slot's chunk and copy its results out.
    int drain(int s)
    {
        if (!pend[s])
            return WC_OK;
        hipError_t e = hipEventSynchronize(P->done[s]);
        if (e != hipSuccess)
            return hip_err(e);
        const int osz = out_size(kind);
        memcpy(h_out + pend_lo[s] * osz, P->h_out[s], pend_n[s] * osz);
        if (kind == kKindFused)
            memcpy(h_out2 + pend_lo[s], P->h_out2[s], pend_n[s] * 2);
        pend[s] = false;
        return WC_OK;
    }

    // On any error, wait for every slot's in-flight copies and kernel before
    // returning: they use the library's pinned staging, which the next call
    // rewrites with plain memcpy.
    int fail(int rc)
    {
        for (int s = 0; s < kPipe; ++s) {
            (void)hipStreamSynchronize(P->st[s]);
            pend[s] = false;
        }
        return rc;
    }

    // Stage and enqueue the next chunk (caller: current device = dev).
    int step()
    {
        int rc = drain(slot);
        if (rc)
            return rc;
        const uint64_t i0 = i;
        uint64_t j = i, bytes = 0;
        const uint8_t *src = nullptr;
        if (ascending) {
            const uint64_t lo = h_off[i];
            uint64_t top = lo;
            while (j < hi && j - i0 < kChunkPkts) {
                const uint64_t e = h_off[j] + span(j);
                if (std::max(top, e) - lo > kChunkBytes && j > i0)
                    break;
                top = std::max(top, e);
                P->h_off[slot][j - i0] = h_off[j] - lo;
                P->h_len[slot][j - i0] = h_len[j];
                ++j;
            }
            bytes = top - lo;
            src = hb + lo;
            if (!registered) {
                stage_copy(P->h_bytes[slot], src, bytes);
                src = P->h_bytes[slot];
            }
        } else {
            // Rebased offsets first (a prefix sum), then the packet copies
            // in parallel ranges of the staging pool.
            while (j < hi && j - i0 < kChunkPkts) {
                const uint64_t sp = span(j);
                if (bytes + sp > kChunkBytes && j > i0)
                    break;
                P->h_off[slot][j - i0] = bytes;
                P->h_len[slot][j - i0] = h_len[j];
                bytes += sp;
                ++j;
            }
            const uint64_t cnt = j - i0;
            StagePool &pool = stage_pool();
            const int parts = (int)std::min<uint64_t>((uint64_t)pool.width(), (cnt + 4095) / 4096);
            uint8_t *dst = P->h_bytes[slot];
            const uint64_t *roff = P->h_off[slot];
            auto gather = [&](int t) {
                const uint64_t a = cnt * (uint64_t)t / (uint64_t)parts;
                const uint64_t b = cnt * (uint64_t)(t + 1) / (uint64_t)parts;
                for (uint64_t q = a; q < b; ++q)
                    memcpy(dst + roff[q], hb + h_off[i0 + q], span(i0 + q));
            };
            pool.run(std::max(parts, 1), gather);
            src = P->h_bytes[slot];
        }
        const uint64_t cnt = j - i0;
        hipStream_t st = P->st[slot];
        hipError_t e = hipMemcpyAsync(P->d_bytes[slot], src, bytes, hipMemcpyHostToDevice, st);
        if (e == hipSuccess)
            e = hipMemcpyAsync(P->d_off[slot], P->h_off[slot], cnt * 8, hipMemcpyHostToDevice,
                               st);
        if (e == hipSuccess)
            e = hipMemcpyAsync(P->d_len[slot], P->h_len[slot], cnt * 2, hipMemcpyHostToDevice,
                               st);
        if (e != hipSuccess)
            return hip_err(e);
        rc = run_ragged_any(*D, g_cfg, P->d_bytes[slot], P->d_off[slot], P->d_len[slot], cnt,
                            P->d_out[slot], kind, false, st, P->d_out2[slot]);
        if (rc)
            return rc;
        e = hipMemcpyAsync(P->h_out[slot], P->d_out[slot], cnt * out_size(kind),
                           hipMemcpyDeviceToHost, st);
        if (e == hipSuccess && kind == kKindFused)
            e = hipMemcpyAsync(P->h_out2[slot], P->d_out2[slot], cnt * 2, hipMemcpyDeviceToHost,
                               st);
        if (e == hipSuccess)
            e = hipEventRecord(P->done[slot], st);
        if (e != hipSuccess)
            return hip_err(e);
        pend[slot] = true;
        pend_lo[slot] = i0;
        pend_n[slot] = cnt;
        i = j;
        slot = (slot + 1) % kPipe;
        return WC_OK;
    }

    int finish()
    {
        for (int s = 0; s < kPipe; ++s) {
            int rc = drain((slot + s) % kPipe);
            if (rc)
                return rc;
        }
        return WC_OK;
    }
};

// Every packet of a host batch inside [0, h_bytes); its order and bytes.
bool host_batch_ok(const uint8_t *hb, uint64_t h_bytes, const uint64_t *h_off,
                   const uint16_t *h_len, uint64_t n, int kind, bool *ascending, uint64_t *total)
{
    bool asc = true;
    uint64_t tot = 0;
    for (uint64_t i = 0; i < n; ++i) {
        const uint64_t o = h_off[i];
        uint64_t sp = span_of(h_len[i], kind);
        if (o > h_bytes || sp > h_bytes - o)
            return false;
        if (kind == kKindFused) { // (its first sp >= 20 bytes are in range)
            sp = fused_span(hb + o, h_len[i]);
            if (sp > h_bytes - o)
                return false;
        }
        asc &= i == 0 || o >= h_off[i - 1];
        tot += sp;
    }
    *ascending = asc;
    *total = tot;
    return true;
}

void shard_range(uint64_t n, int g, int G, uint64_t *lo, uint64_t *hi)
{
    // n * g / G without overflow for any uint64 n
    *lo = (uint64_t)((unsigned __int128)n * (unsigned)g / (unsigned)G);
    *hi = (uint64_t)((unsigned __int128)n * (unsigned)(g + 1) / (unsigned)G);
}

int host_pipeline(Device &D, const uint8_t *hb, bool registered, bool ascending,
                  const uint64_t *h_off, const uint16_t *h_len, uint64_t n,
                  uint8_t *h_out, int kind, uint16_t *h_out2)
{
    PipeRun r;
    r.D = &D;
    r.P = &D.pipe;
    r.hb = hb;
    r.registered = registered;
    r.ascending = ascending;
    r.h_off = h_off;
    r.h_len = h_len;
    r.h_out = h_out;
    r.h_out2 = h_out2;
    r.kind = kind;
    r.hi = n;
    while (!r.done()) {
        const int rc = r.step();
        if (rc)
            return r.fail(rc);
    }
    const int rc = r.finish();
    return rc ? r.fail(rc) : WC_OK;
}


// Run fn(g) for every shard with its device current; the caller's device is
// restored.  Snapshot of the shard devices taken under the lock (the batch
// calls take it themselves).
template <class F>
int for_each_shard(F &&fn)
{
    int devs[kMaxDevices];
    int G = 0;
    {
        std::lock_guard<FairMutex> lk(g_mu);
        G = g_multi_n;
        for (int g = 0; g < G; ++g)
            devs[g] = g_shard[g].dev;
    }
    if (G == 0)
        return WC_EINVAL; // wc_gpu_init_multi first
    int cur = 0;
    if (hipGetDevice(&cur) != hipSuccess)
        return WC_ENODEV;
    int rc = WC_OK;
    for (int g = 0; g < G && rc == WC_OK; ++g) {
        rc = hip_err(hipSetDevice(devs[g]));
        if (rc == WC_OK)
            rc = fn(g);
    }
    (void)hipSetDevice(cur);
    return rc;
}

// wc_cksum_host / wc_rx_verdict_host / wc_cksum_ip_udp_host: a host-memory
// batch on the current device -- the resident server or one zero-copy launch
// for a small registered batch, else the pipeline.  h_out2: the fused pair's
// header checksums.
int host_batch(const void *h_base, uint64_t h_bytes, const uint64_t *h_off,
               const uint16_t *h_len, uint64_t n, uint8_t *h_out, int kind,
               uint16_t *h_out2 = nullptr)
{
    if (n == 0)
        return WC_OK;
    if (!h_base || !h_off || !h_len || !h_out || (kind == kKindFused && !h_out2))
        return WC_EINVAL;
    bool ascending = true;
    uint64_t total = 0;
    if (!host_batch_ok((const uint8_t *)h_base, h_bytes, h_off, h_len, n, kind, &ascending,
                       &total))
        return WC_EINVAL;

    std::lock_guard<FairMutex> lk(g_mu);
    Device *D = nullptr;
    int rc = init_locked(-1, &D);
    if (rc)
        return rc;
    const uint8_t *dbase = registered_dptr_locked(h_base, h_bytes);
    if (dbase && g_cfg.serve && n <= (uint64_t)g_cfg.serve_max) {
        bool fits = true; // (a fused header adds at most 40 bytes to the span)
        for (uint64_t i = 0; i < n && fits; ++i)
            fits = span_of(h_len[i], kind) + (kind == kKindFused ? 40u : 0u) <= wc::kSrvMaxBytes;
        int dev = 0;
        if (fits && current_device(&dev) == WC_OK) {
            rc = serve_batch(*D, dev, dbase, h_off, h_len, n, h_out, kind, h_out2);
            if (rc != kSrvFallback)
                return rc;
        }
    }
    if (dbase && n <= kZcPkts && total <= (uint64_t)g_cfg.zc_bytes)
        return host_zero_copy(*D, dbase, h_off, h_len, n, h_out, kind, h_out2);
    rc = pipe_init_locked(D->pipe);
    if (rc)
        return rc;
    return host_pipeline(*D, (const uint8_t *)h_base, dbase != nullptr, ascending,
                         h_off, h_len, n, h_out, kind, h_out2);
}

} // namespace

// ===========================================================================
// Exported C ABI.

extern "C" {

uint16_t ip_cksum(const void *buf, uint16_t len)
{
    return scalar_cksum(buf, len, WC_CKSUM_IP, "ip_cksum");
}

uint16_t payload_cksum(const void *buf, uint16_t len)
{
    return scalar_cksum(buf, len, WC_CKSUM_PAYLOAD, "payload_cksum");
}

int wc_cksum_strided(const void *d_base, uint64_t stride, uint16_t len,
                     uint64_t n, uint16_t *d_out, int kind, void *stream)
{
    if (!d_out && n)
        return WC_EINVAL;
    return batch_strided(d_base, stride, len, n, d_out, nullptr, kind, stream);
}

int wc_cksum_ragged(const void *d_base, const uint64_t *d_off,
                    const uint16_t *d_len, uint64_t n, uint16_t *d_out,
                    int kind, void *stream)
{
    if (!d_out && n)
        return WC_EINVAL;
    return batch_ragged(d_base, d_off, d_len, n, d_out, nullptr, kind, stream);
}

int wc_verify_strided(const void *d_base, uint64_t stride, uint16_t len,
                      uint64_t n, uint16_t *d_out, uint64_t *d_bad, int kind,
                      void *stream)
{
    if (!d_bad && n)
        return WC_EINVAL;
    return batch_strided(d_base, stride, len, n, d_out, d_bad, kind, stream);
}

int wc_verify_ragged(const void *d_base, const uint64_t *d_off,
                     const uint16_t *d_len, uint64_t n, uint16_t *d_out,
                     uint64_t *d_bad, int kind, void *stream)
{
    if (!d_bad && n)
        return WC_EINVAL;
    return batch_ragged(d_base, d_off, d_len, n, d_out, d_bad, kind, stream);
}

int wc_cksum_ip_udp_strided(const void *d_base, uint64_t stride, uint16_t len,
                            uint64_t n, uint16_t *d_out_ip_hdr,
                            uint16_t *d_out_payload, void *stream)
{
    if (n && (!d_out_ip_hdr || !d_out_payload))
        return WC_EINVAL;
    return batch_strided(d_base, stride, len, n, d_out_payload, nullptr,
                         WC_CKSUM_PAYLOAD, stream, d_out_ip_hdr);
}

int wc_cksum_ip_udp_ragged(const void *d_base, const uint64_t *d_off,
                           const uint16_t *d_len, uint64_t n, uint16_t *d_out_ip_hdr,
                           uint16_t *d_out_payload, void *stream)
{
    if (n && (!d_out_ip_hdr || !d_out_payload))
        return WC_EINVAL;
    return batch_ragged(d_base, d_off, d_len, n, d_out_payload, nullptr,
                        WC_CKSUM_PAYLOAD, stream, d_out_ip_hdr);
}

int wc_host_register(void *h_ptr, uint64_t bytes)
{
    if (!h_ptr || !bytes)
        return WC_EINVAL;
    std::lock_guard<FairMutex> lk(g_mu);
    Device *D = nullptr;
    int rc = init_locked(-1, &D);
    if (rc)
        return rc;
    // The resident server grid would hold up a device-wide synchronisation
    // that (un)registering may do until the idle watcher stopped it -- and
    // the watcher waits for g_mu, held here.  Stop it first; the next small
    // call starts it again.
    server_stop_all_locked();
    // Registering a base address again always pins the pages mapped there
    // NOW: the caller may have freed the old region without
    // wc_host_unregister and got a new buffer at the same address, whose
    // pages the old registration (and its cached device addresses) do not
    // cover.  So the old registration is dropped and the range registered
    // afresh; if that fails, the old range is registered again so a live
    // region keeps working, and the error is returned.
    uint64_t old_bytes = 0;
    auto it = g_registered.find((uintptr_t)h_ptr);
    if (it != g_registered.end()) {
        old_bytes = it->second.bytes;
        g_registered.erase(it);
        (void)hipHostUnregister(h_ptr);
    }
    const unsigned flags = hipHostRegisterMapped | hipHostRegisterPortable;
    auto pin = [&](uint64_t nb) -> hipError_t {
        // Portable: every device (wc_cksum_host_multi's shards) may DMA from it.
        hipError_t e = hipHostRegister(h_ptr, nb, flags);
        if (e != hipSuccess)
            return e;
        void *dptr = nullptr;
        e = hipHostGetDevicePointer(&dptr, h_ptr, 0);
        if (e != hipSuccess) {
            (void)hipHostUnregister(h_ptr);
            return e;
        }
        Registration reg;
        reg.bytes = nb;
        int dev = 0;
        if (current_device(&dev) == WC_OK)
            reg.dptr[dev] = (const uint8_t *)dptr;
        g_registered[(uintptr_t)h_ptr] = reg;
        return hipSuccess;
    };
    const hipError_t e = pin(bytes);
    if (e != hipSuccess && old_bytes)
        (void)pin(old_bytes);
    return hip_err(e);
}

int wc_host_unregister(void *h_ptr)
{
    if (!h_ptr)
        return WC_EINVAL;
    std::lock_guard<FairMutex> lk(g_mu);
    auto it = g_registered.find((uintptr_t)h_ptr);
    if (it == g_registered.end())
        return WC_EINVAL;
    g_registered.erase(it);
    server_stop_all_locked(); // (see wc_host_register)
    return hip_err(hipHostUnregister(h_ptr));
}

int wc_cksum_host(const void *h_base, uint64_t h_bytes, const uint64_t *h_off,
                  const uint16_t *h_len, uint64_t n, uint16_t *h_out, int kind)
{
    if (kind != WC_CKSUM_IP && kind != WC_CKSUM_PAYLOAD)
        return WC_EINVAL;
    return host_batch(h_base, h_bytes, h_off, h_len, n, (uint8_t *)h_out, kind);
}

int wc_cksum_ip_udp_host(const void *h_base, uint64_t h_bytes, const uint64_t *h_off,
                         const uint16_t *h_len, uint64_t n, uint16_t *h_out_ip_hdr,
                         uint16_t *h_out_payload)
{
    if (n && (!h_out_ip_hdr || !h_out_payload))
        return WC_EINVAL;
    return host_batch(h_base, h_bytes, h_off, h_len, n, (uint8_t *)h_out_payload, kKindFused,
                      h_out_ip_hdr);
}

int wc_server_stats(uint64_t *served, uint64_t *fallbacks, uint64_t *launches)
{
    std::lock_guard<FairMutex> lk(g_mu);
    if (served)
        *served = g_srv_stats.served;
    if (fallbacks)
        *fallbacks = g_srv_stats.fallbacks;
    if (launches)
        *launches = g_srv_stats.launches;
    return WC_OK;
}

int wc_rx_verdict_ragged(const void *d_base, const uint64_t *d_off, const uint16_t *d_frame_len,
                         uint64_t n, uint8_t *d_verdict, uint64_t *d_drops, void *stream)
{
    if (n == 0)
        return WC_OK;
    if (!d_base || !d_off || !d_frame_len || !d_verdict)
        return WC_EINVAL;
    Device *D = nullptr;
    Config C;
    int rc = ensure_device(&D, &C);
    if (rc)
        return rc;
    return hip_err(rx_launch(*D, C, d_base, d_off, d_frame_len, n, d_verdict, d_drops,
                             (hipStream_t)stream));
}

int wc_rx_verdict_host(const void *h_base, uint64_t h_bytes, const uint64_t *h_off,
                       const uint16_t *h_frame_len, uint64_t n, uint8_t *h_verdict,
                       uint64_t *h_drops)
{
    if (n && !h_verdict)
        return WC_EINVAL;
    const int rc = host_batch(h_base, h_bytes, h_off, h_frame_len, n, h_verdict, kKindRx);
    if (rc == WC_OK && h_drops) {
        uint64_t d = 0;
        for (uint64_t i = 0; i < n; ++i)
            d += WC_RX_IS_DROP(h_verdict[i]);
        *h_drops = d;
    }
    return rc;
}

// ---------------------------------------------------------------------------
// Multi-GPU: an even contiguous packet split over the shard
// executors, no data-path collective; RCCL only for the optional result
// gather.

int wc_shard_range(uint64_t n, int g, int ngpus, uint64_t *lo, uint64_t *hi)
{
    if (ngpus < 1 || g < 0 || g >= ngpus || !lo || !hi)
        return WC_EINVAL;
    shard_range(n, g, ngpus, lo, hi);
    return WC_OK;
}

int wc_gpu_init_multi(int ngpus, const int *devices)
{
    std::lock_guard<FairMutex> lk(g_mu);
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0)
        return WC_ENODEV;
    if (ngpus <= 0) {
        if (devices)
            return WC_EINVAL;
        ngpus = ndev;
    }
    if (ngpus > kMaxDevices)
        return WC_EINVAL;
    int devs[kMaxDevices];
    for (int g = 0; g < ngpus; ++g) {
        devs[g] = devices ? devices[g] : g;
        if (devs[g] < 0 || devs[g] >= ndev || devs[g] >= kMaxDevices)
            return WC_EINVAL;
    }
    int cur = 0;
    if (hipGetDevice(&cur) != hipSuccess)
        return WC_ENODEV;
    // A new shard set replaces the old one (its pipelines and communicators).
    wc::rccl_fini();
    for (int g = 0; g < g_multi_n; ++g) {
        (void)hipSetDevice(g_shard[g].dev);
        pipe_free(g_shard[g].pipe);
        g_shard[g] = ShardExec{};
    }
    g_multi_n = 0;
    // All or nothing: a shard that fails to come up (its device's scratch or
    // its pipeline) tears down the ones built before it, so a later
    // wc_cksum_host_multi never runs on a half-built executor -- it falls
    // back to the current device, as before any wc_gpu_init_multi.
    int rc = WC_OK;
    int built = 0;
    for (int g = 0; g < ngpus && rc == WC_OK; ++g) {
        Device *D = nullptr;
        rc = init_locked(devs[g], &D); // sets device devs[g]
        g_shard[g].dev = devs[g];
        if (rc == WC_OK)
            rc = pipe_init_locked(g_shard[g].pipe);
        built = g + 1; // pipe_free below also frees a partly built pipe
    }
    if (rc != WC_OK) {
        for (int g = 0; g < built; ++g) {
            (void)hipSetDevice(g_shard[g].dev);
            pipe_free(g_shard[g].pipe);
            g_shard[g] = ShardExec{};
        }
    } else {
        g_multi_n = ngpus;
    }
    (void)hipSetDevice(cur);
    return rc;
}

int wc_gpu_multi_count(void)
{
    std::lock_guard<FairMutex> lk(g_mu);
    return g_multi_n;
}

int wc_cksum_host_multi(const void *h_base, uint64_t h_bytes, const uint64_t *h_off,
                        const uint16_t *h_len, uint64_t n, uint16_t *h_out, int kind)
{
    if (kind != WC_CKSUM_IP && kind != WC_CKSUM_PAYLOAD)
        return WC_EINVAL;
    if (n == 0)
        return WC_OK;
    if (!h_base || !h_off || !h_len || !h_out)
        return WC_EINVAL;
    int G = 0;
    {
        std::lock_guard<FairMutex> lk(g_mu);
        G = g_multi_n;
    }
    if (G == 0)
        return wc_cksum_host(h_base, h_bytes, h_off, h_len, n, h_out, kind);
    bool ascending = true;
    uint64_t total = 0;
    if (!host_batch_ok((const uint8_t *)h_base, h_bytes, h_off, h_len, n, kind, &ascending,
                       &total))
        return WC_EINVAL;
    {
        std::lock_guard<FairMutex> lk(g_mu);
        G = g_multi_n;
        int cur = 0;
        if (hipGetDevice(&cur) != hipSuccess)
            return WC_ENODEV;
        const bool registered = registered_dptr_locked(h_base, h_bytes) != nullptr;
        if (registered && n <= kZcPkts && total <= (uint64_t)g_cfg.zc_bytes) {
            // Small registered batch: one zero-copy launch on shard 0, with
            // the region's address as shard 0's device sees it.
            Device *D = nullptr;
            int rc = init_locked(g_shard[0].dev, &D); // sets shard 0's device
            const uint8_t *dbase = rc == WC_OK ? registered_dptr_locked(h_base, h_bytes) : nullptr;
            if (rc == WC_OK && !dbase)
                rc = WC_EINVAL;
            if (rc == WC_OK)
                rc = host_zero_copy(*D, dbase, h_off, h_len, n, (uint8_t *)h_out, kind);
            (void)hipSetDevice(cur);
            return rc;
        }
        PipeRun runs[kMaxDevices];
        for (int g = 0; g < G; ++g) {
            PipeRun &r = runs[g];
            r.D = &g_dev[g_shard[g].dev];
            r.P = &g_shard[g].pipe;
            r.dev = g_shard[g].dev;
            r.hb = (const uint8_t *)h_base;
            r.registered = registered;
            r.ascending = ascending;
            r.h_off = h_off;
            r.h_len = h_len;
            r.h_out = (uint8_t *)h_out;
            r.kind = kind;
            shard_range(n, g, G, &r.i, &r.hi);
        }
        // One thread, G pipelines: each pass stages one chunk per unfinished
        // shard, so every device's copies and kernels overlap the staging of
        // the others.
        int rc = WC_OK;
        for (bool more = true; more && rc == WC_OK;) {
            more = false;
            for (int g = 0; g < G && rc == WC_OK; ++g) {
                if (runs[g].done())
                    continue;
                more = true;
                rc = hip_err(hipSetDevice(runs[g].dev));
                if (rc == WC_OK)
                    rc = runs[g].step();
            }
        }
        for (int g = 0; g < G; ++g) {
            (void)hipSetDevice(runs[g].dev);
            if (rc == WC_OK)
                rc = runs[g].finish();
        }
        if (rc != WC_OK)
            for (int g = 0; g < G; ++g) {
                (void)hipSetDevice(runs[g].dev);
                (void)runs[g].fail(rc);
            }
        (void)hipSetDevice(cur);
        return rc;
    }
}

int wc_cksum_strided_multi(const void *const *d_base, uint64_t stride, uint16_t len,
                           const uint64_t *n, uint16_t *const *d_out, int kind,
                           void *const *streams)
{
    if (!d_base || !n || !d_out)
        return WC_EINVAL;
    return for_each_shard([&](int g) {
        return wc_cksum_strided(d_base[g], stride, len, n[g], d_out[g], kind,
                                streams ? streams[g] : nullptr);
    });
}

int wc_cksum_ragged_multi(const void *const *d_base, const uint64_t *const *d_off,
                          const uint16_t *const *d_len, const uint64_t *n,
                          uint16_t *const *d_out, int kind, void *const *streams)
{
    if (!d_base || !d_off || !d_len || !n || !d_out)
        return WC_EINVAL;
    return for_each_shard([&](int g) {
        return wc_cksum_ragged(d_base[g], d_off[g], d_len[g], n[g], d_out[g], kind,
                               streams ? streams[g] : nullptr);
    });
}

int wc_gather_results_multi(uint16_t *const *d_shard_out, const uint64_t *n,
                            uint16_t *const *d_all, void *const *streams)
{
    if (!d_shard_out || !n || !d_all)
        return WC_EINVAL;
    std::lock_guard<FairMutex> lk(g_mu);
    if (g_multi_n == 0)
        return WC_EINVAL;
    int devs[kMaxDevices];
    for (int g = 0; g < g_multi_n; ++g)
        devs[g] = g_shard[g].dev;
    int cur = 0;
    if (hipGetDevice(&cur) != hipSuccess)
        return WC_ENODEV;
    const int rc = wc::rccl_allgatherv_u16(g_multi_n, devs, d_shard_out, n, d_all, streams);
    (void)hipSetDevice(cur);
    return rc;
}

int wc_gpu_init(int device)
{
    std::lock_guard<FairMutex> lk(g_mu);
    Device *D = nullptr;
    return init_locked(device, &D);
}

int wc_gpu_fini(void)
{
    std::lock_guard<FairMutex> lk(g_mu);
    int cur = 0;
    const bool have_cur = hipGetDevice(&cur) == hipSuccess;
    for (int d = 0; d < kMaxDevices; ++d) // (device calls take the locked path again)
        g_dev_ready[d].store(false, std::memory_order_release);
    server_stop_all_locked();
    wc::rccl_fini();
    for (int g = 0; g < g_multi_n; ++g) {
        (void)hipSetDevice(g_shard[g].dev);
        pipe_free(g_shard[g].pipe);
        g_shard[g] = ShardExec{};
    }
    g_multi_n = 0;
    for (int d = 0; d < kMaxDevices; ++d) {
        Device &D = g_dev[d];
        if (!D.ok)
            continue;
        (void)hipSetDevice(d);
        pipe_free(D.pipe);
        if (D.zc.ready) {
            (void)hipStreamSynchronize(D.zc.st);
            (void)hipStreamDestroy(D.zc.st);
            (void)hipHostFree(D.zc.h_off);
            (void)hipHostFree(D.zc.h_len);
            (void)hipHostFree(D.zc.h_out);
            (void)hipHostFree(D.zc.h_out2);
        }
        if (D.srv.ready) {
            (void)hipStreamDestroy(D.srv.st);
            (void)hipHostFree(D.srv.h_rec);
            (void)hipHostFree(D.srv.h_res);
            (void)hipHostFree(D.srv.h_hb);
        }
        (void)hipStreamSynchronize(D.scalar_st);
        (void)hipDeviceSynchronize(); // (an RX launch may still write its tally)
        for (int k = 0; k < kRxSets; ++k)
            (void)hipHostFree(D.h_rx_tally[k]);
        (void)hipStreamDestroy(D.scalar_st);
        (void)hipHostFree(D.h_stage);
        (void)hipHostFree(D.h_res);
        D = Device{};
    }
    // Page-locks taken with wc_host_register belong to the caller and stay
    // until wc_host_unregister (a ring registered once keeps its zero-copy
    // path across fini / init).  The WC_* configuration is re-read at the
    // next initialisation.
    g_cfg_loaded = false;
    if (have_cur)
        (void)hipSetDevice(cur);
    return WC_OK;
}

int wc_config_reload(void)
{
    std::lock_guard<FairMutex> lk(g_mu);
    load_config_locked();
    return WC_OK;
}

int wc_sclk_probe(uint64_t *d_samples, int n, uint64_t interval, void *stream)
{
    if (n <= 0)
        return WC_OK;
    if (!d_samples || !interval || ((uintptr_t)d_samples & 7u))
        return WC_EINVAL;
    Device *D = nullptr;
    Config C;
    int rc = ensure_device(&D, &C);
    if (rc)
        return rc;
    return hip_err(wc::launch_sclk_probe(d_samples, n, interval, (hipStream_t)stream));
}

int wc_synth_fill(void *d_buf, uint64_t nbytes, uint64_t seed, void *stream)
{
    if (!nbytes)
        return WC_OK;
    if (!d_buf || ((uintptr_t)d_buf & 15u))
        return WC_EINVAL;
    Device *D = nullptr;
    Config C;
    int rc = ensure_device(&D, &C);
    if (rc)
        return rc;
    const uint64_t threads = (nbytes / 16) + 1;
    const int grid = (int)std::min<uint64_t>((threads + 255) / 256,
                                             (uint64_t)D->cus * 8);
    return hip_err(wc::launch_synth(d_buf, nbytes, seed, grid, (hipStream_t)stream));
}

int wc_plan_strided(uint64_t base_addr, uint64_t stride, uint16_t len,
                    uint64_t n, int kind, int *group, int *chunks_per_lane,
                    int *unroll, int *grid)
{
    if (kind != WC_CKSUM_IP && kind != WC_CKSUM_PAYLOAD)
        return WC_EINVAL;
    Device *D = nullptr;
    Config C;
    int rc = ensure_device(&D, &C);
    if (rc)
        return rc;
    const Plan p = plan_strided(*D, C, base_addr, stride, len, n, kind);
    if (group)
        *group = p.shape.group;
    if (chunks_per_lane)
        *chunks_per_lane = p.shape.cpl;
    if (unroll)
        *unroll = p.shape.unroll;
    if (grid)
        *grid = p.grid;
    return WC_OK;
}

const char *wc_plan_strided_kernel(uint64_t base_addr, uint64_t stride, uint16_t len, uint64_t n,
                                   int kind)
{
    if (kind != WC_CKSUM_IP && kind != WC_CKSUM_PAYLOAD)
        return "invalid";
    Device *D = nullptr;
    Config C;
    if (ensure_device(&D, &C))
        return "invalid";
    const Plan p = plan_strided(*D, C, base_addr, stride, len, n, kind);
    return p.lean ? "lean" : p.shape.group == 0 ? "seg" : "group";
}

const char *wc_strerror(int err)
{
    switch (err) {
    case WC_OK:
        return "success";
    case WC_EINVAL:
        return "invalid argument";
    case WC_ENODEV:
        return "no usable gfx950 device";
    case WC_ENOMEM:
        return "out of memory";
    case WC_ECOMM:
        return "RCCL unavailable or collective failed";
    default:
        if (err < 0 && err > -10000)
            return hipGetErrorString((hipError_t)(-err));
        return "unknown error";
    }
}

#ifdef WC_TUNING
const char *wc_version(void) { return "wccksum 0.3.0 (gfx950, TUNING build: WC_VARIANT/WC_DIAG_NOLOAD live)"; }
#else
const char *wc_version(void) { return "wccksum 0.3.0 (gfx950)"; }
#endif

} // extern "C"
