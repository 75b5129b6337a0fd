// bm_api.hip -- C ABI of libbtcminer.so (include/btcminer.h): device
// contexts, launch sizing, the per-device reduction and the multi-GPU
// RCCL allgather of 16-byte partials (one process over N devices, or one
// process per device joined into an RCCL communicator).
//
// Drop-in for the reference miner's job loop body: miner.go:58-65 calls
// bitcoin.Hash (hash.go:11-15) once per nonce and keeps a strict-'<' minimum;
// bm_search_gpu returns the same (hash, nonce) for the same (msg, range).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <chrono>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <condition_variable>
#include <functional>
#include <memory>
#include <mutex>
#include <new>
#include <system_error>
#include <thread>
#include <vector>

#include "bm_aux_kernels.hpp"
#include "bm_plan.hpp"
#include "btcminer.h"

namespace bm {

// search kernel table [nbv-1][P], filled by bm_inst.hip at load time; rows
// 2 + K hold the padding-block layouts (P >= 55) with their constants folded
// after K whole prefix blocks: search_kernel_padc<P> (K = 0, a one-block
// message) and search_kernel_padk<P, K> (K = 1..kMaxPadPrefixBlocks = 15)
constexpr int kSearchRows = 3 + kMaxPadPrefixBlocks;
static const void* g_search[kSearchRows][64];

constexpr int kMaxInnerDigits = 2;  // S <= 100 nonces per task: small dequeue chunks, short tail
constexpr uint32_t kNoncesPerLaneChunk = 100;  // default nonces per lane per dequeue (BTCMINER_CHUNK)
constexpr int kEventPairs = BM_MAX_LAUNCH_STATS;
// Launch streams per device.  Every search launch is a persistent grid that
// drains a work counter, so its last tasks leave CUs idle (about half a
// 100-nonce task, ~0.5 ms).  With more than one stream the launches of one
// call go out biggest first over the streams, and the next launch's
// workgroups fill the CUs the previous one frees.
constexpr int kMaxStreams = 4;
constexpr uint64_t kMaxTailNonces = 1ull << 40;
constexpr size_t kCtrStride = 32;  // u64 words per launch: counter [0], clock stamps [16..19] (kClockSlot)
// Balance (bm_ctx_set_balance): a device's rate is measured only when its
// piece held at least this many nonces (about 20 ms of one MI355X), and the
// shares are the rates scaled so the fastest device gets kShareScale.
constexpr uint64_t kBalanceMinNonces = 1ull << 30;
constexpr double kShareScale = 65536.0;
// A device's start offset (bm_stats_t.dev_start_ms) enters its rate only
// above host jitter: at least 1 ms and 1% of its span.
constexpr double kBalanceStartMinMs = 1.0;
constexpr double kBalanceStartMinFrac = 0.01;

// What each device / rank contributes to the combine: its partial and a
// status word (a rank that failed the call before the combine still takes
// part in the allgather, with its status here).  32 bytes = 4 u64.
struct Slot {
    Partial p;
    uint64_t status;
    uint64_t pad;
};
static_assert(sizeof(Slot) == 32, "slot layout");
constexpr size_t kSlotWords = sizeof(Slot) / sizeof(uint64_t);

struct DeviceCtx {
    int id = -1;
    int cus = 0;
    hipStream_t stream = nullptr;
    Partial* d_part = nullptr;
    size_t part_cap = 0;
    unsigned long long* d_ctr = nullptr;  // per launch a strip of kCtrStride words: [0] dequeue
                                          // counter, [16..19] clock stamps (bm_kernels.hpp)
    unsigned long long* h_ctr = nullptr;  // pinned copy of the strips (timing on)
    size_t ctr_cap = 0;
    Slot* d_slot = nullptr;    // this device's slot (reduce_partials writes its partial)
    Slot* d_gather = nullptr;  // nslots slots (allgather target)
    Slot* h_slots = nullptr;   // pinned: nslots slots, + 1 staging slot (a failed rank's status)
    int nslots = 1;
    Partial* d_test = nullptr;    // bm_reduce_gpu's staging buffer
    size_t test_cap = 0;
    uint64_t* d_hash_io = nullptr;
    size_t hash_cap = 0;
    hipEvent_t ev[2 * kEventPairs] = {};
    hipStream_t aux[kMaxStreams - 1] = {};  // extra launch streams (ctx->streams > 1)
    hipEvent_t fork = nullptr, join[kMaxStreams - 1] = {};
    hipEvent_t bal[2] = {};     // the device's first op and the end of its reduction (balance, timing)
    hipEvent_t ag[2] = {};      // around the device's allgather (timing): its wait for the peers + transfer
    hipEvent_t own_done = nullptr;  // rank contexts: this rank's reduction done (before the allgather)
    uint64_t piece_nonces = 0;  // nonces of the device's piece in the last call
    std::chrono::steady_clock::time_point submitted{};  // host time of the call's first op on this device
    int test_delay_us = 0;      // test hook: hold back this device's submission (bm_ctx_set_test_start_delay)
    ncclComm_t comm = nullptr;  // multi-device ctx: ncclCommInitAll; joined rank ctx: the process group's
    std::vector<std::pair<const void*, int>> occ;  // kernel -> blocks per CU
    double wall_clock_hz = 100e6;                  // s_memrealtime rate
};

struct Launch {
    const void* fn;
    SearchArgs args;
    uint32_t grid;
    bm_launch_stat_t stat;
};

// bm_ctx_join_rank's worker: one communicator set-up, shared with the caller
// (who may give up on it: then the worker aborts what it made).  A join the
// caller gave up on stays on the context as its pending join, so a context
// never has more than one worker inside RCCL.
struct JoinJob {
    std::mutex m;
    std::condition_variable cv;
    bool done = false, abandoned = false;
    ncclComm_t comm = nullptr;
    int rc = BM_ERCCL;
    double init_ms = 0.0;  // the init's host time, until it settled
};

namespace {
int hip_status(hipError_t e) { return e == hipSuccess ? BM_OK : BM_EHIP; }

// BTCMINER_TRACE=1: one stderr line per step of the group set-up and combine
// (diagnostics of multi-process runs; off by default)
void trace(const char* fmt, ...) {
    static const bool on = std::getenv("BTCMINER_TRACE") != nullptr;
    if (!on) return;
    va_list ap;
    va_start(ap, fmt);
    std::fprintf(stderr, "[btcminer] ");
    std::vfprintf(stderr, fmt, ap);
    std::fprintf(stderr, "\n");
    va_end(ap);
}

#define BM_HIP(call)                                 \
    do {                                             \
        hipError_t e_ = (call);                      \
        if (e_ != hipSuccess) return hip_status(e_); \
    } while (0)

// The submission threads of a multi-device context: created once,
// at the context's first search over several devices, and kept until the
// context is destroyed, so a search does not create and join N - 1 threads
// (about 0.2 ms at N = 8, most of a small job's fixed cost).
// run(n, f) runs f(1) .. f(n - 1) on the pool's threads and f(0) on the
// caller, and returns when all of them have.  f must not throw (the search
// wraps it in guarded()).  A context is not re-entrant, so one run at a time.
class SubmitPool {
   public:
    SubmitPool() = default;
    SubmitPool(const SubmitPool&) = delete;
    SubmitPool& operator=(const SubmitPool&) = delete;
    ~SubmitPool() { stop(); }

    // false when the threads could not be started: the caller submits serially
    bool run(int n, const std::function<void(int)>& f) {
        if (!ensure(n - 1)) return false;
        {
            std::lock_guard<std::mutex> g(m_);
            job_ = &f;
            pending_ = n - 1;
            ++gen_;
        }
        work_.notify_all();
        f(0);
        std::unique_lock<std::mutex> l(m_);
        done_.wait(l, [&] { return pending_ == 0; });
        job_ = nullptr;
        return true;
    }
    int threads() const { return (int)th_.size(); }

   private:
    bool ensure(int k) {
        if ((int)th_.size() == k) return true;
        stop();  // (a context's device count never changes; this is only the first call)
        try {
            for (int i = 0; i < k; ++i) th_.emplace_back([this, i] { loop(i + 1); });
        } catch (const std::system_error&) {
            stop();
            return false;
        }
        return true;
    }
    void loop(int di) {
        uint64_t seen = 0;
        for (;;) {
            const std::function<void(int)>* job;
            {
                std::unique_lock<std::mutex> l(m_);
                work_.wait(l, [&] { return quit_ || gen_ != seen; });
                if (quit_) return;
                seen = gen_;
                job = job_;
            }
            (*job)(di);
            std::lock_guard<std::mutex> g(m_);
            if (--pending_ == 0) done_.notify_one();
        }
    }
    void stop() {
        {
            std::lock_guard<std::mutex> g(m_);
            quit_ = true;
        }
        work_.notify_all();
        for (auto& t : th_) t.join();
        th_.clear();
        quit_ = false;
    }
    std::mutex m_;
    std::condition_variable work_, done_;
    std::vector<std::thread> th_;
    const std::function<void(int)>* job_ = nullptr;
    uint64_t gen_ = 0;
    int pending_ = 0;
    bool quit_ = false;
};

// Restores the caller's current device on scope exit.
struct DeviceGuard {
    int prev = -1;
    DeviceGuard() {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    }
    ~DeviceGuard() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};

}  // namespace
}  // namespace bm

struct bm_ctx {
    std::vector<bm::DeviceCtx> devs;
    bool timing = false;
    int blocks_per_cu = 0;
    int max_windows = bm::kDefaultMaxWindows;
    int combine = BM_COMBINE_AUTO;
    int task_digits = 0;  // 0: per launch (size_launch); 1 or 2: forced
    uint64_t tail_nonces = 1ull << 24;  // split off the biggest launch's last nonces (BTCMINER_TAIL; 0: off; profiles/r01/ab_tail.log)
    int streams = 2;      // launch streams per device (1..kMaxStreams; BTCMINER_STREAMS; profiles/r01/ab_streams.log)
    bool nccl_ready = false;
    int rccl_status = 0;      // multi-device ctx: the RCCL failure it fell back from (then: host copies)
    int rank = 0, world = 1;  // rank contexts: this process's place in the group
    bool rank_ctx = false;    // made by bm_ctx_create_rank_local (one device, one slot of `world`)
    bool joined = false;      // rank ctx: member of an RCCL group (devs[0].comm)
    int group_status = 0;     // joined rank ctx whose communicator failed (BM_ERCCL / BM_ETIMEDOUT)
    int peer_timeout_ms = BM_DEFAULT_PEER_TIMEOUT_MS;  // joined rank ctx: wait at most this long for
                                                       // the group (0: no limit)
    double rccl_init_ms = 0.0;  // host time the current communicator(s) took to form
    int fault_after = -1;     // test hook: fail after enqueueing this many launches (-1: off)
    int test_rccl_fault = 0;  // test hook: 1 communicator set-up fails, 2 every allgather fails,
                              // 3 the gathered slots report a failed peer (rank groups)
    uint64_t lane_chunk = bm::kNoncesPerLaneChunk;  // nonces per lane per dequeue, at most (BTCMINER_CHUNK)
    std::vector<uint32_t> shares;  // the partitioner's shares per slot (empty: near-equal pieces)
    bool balance = false;          // multi-device: shares follow each device's measured rate
    bool padc = true;              // use search_kernel_padc / _padk where they apply (BTCMINER_PADC=0: never; A/B knob)
    // rank ctx: a join whose caller timed out while its worker was still
    // inside RCCL (the worker aborts the communicator if it ever gets one)
    std::shared_ptr<bm::JoinJob> pending_join;
    std::thread pending_worker;
    bm_stats_t stats;
    bm::SubmitPool submit;  // multi-device: one submission thread per device but the first (last member:
                            // stopped first, when every device is idle)
};

extern "C" void bm_register_search_kernel(int p, int nbv, const void* fn) {
    if (p >= 0 && p < 64 && nbv >= 1 && nbv <= bm::kSearchRows) bm::g_search[nbv - 1][p] = fn;
}

namespace bm {
namespace {

int blocks_per_cu(bm_ctx* ctx, DeviceCtx& d, const void* fn) {
    if (ctx->blocks_per_cu > 0) return ctx->blocks_per_cu;
    for (auto& e : d.occ)
        if (e.first == fn) return e.second;
    int nb = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, fn, kBlock, 0) != hipSuccess || nb < 1) nb = 1;
    d.occ.emplace_back(fn, nb);
    return nb;
}

// Size one launch: S = 10^ms nonces per task (ms <= digits of word LW),
// chunks of 64*m tasks dequeued per wave, and at most one resident grid of
// workgroups (any surplus workgroup simply finds the counter exhausted).
// A folded padding-block kernel applies when the segment's padding block is
// the one of a message of K whole blocks plus the varying block ending at
// byte P (bm_sha256.hpp pad_kw_const(P, K), K <= kMaxPadPrefixBlocks), and for
// K = 0 its entering state is the IV: the constants the kernel folds.
// Returns K, or -1 when the generic kernel must run.
int pad_fold_k(const bm_segment_t& s) {
    if (!s.pad_block || s.nbv != 1 || s.p < 55) return -1;
    // the only K this padding block can be: its bit length 8 * (64K + P + 1)
    const uint32_t bits = s.pad_w[15];
    if (bits % 8 != 0 || bits / 8 < (uint32_t)s.p + 1 || (bits / 8 - s.p - 1) % 64 != 0) return -1;
    const uint32_t k = (bits / 8 - s.p - 1) / 64;
    if (k > (uint32_t)kMaxPadPrefixBlocks) return -1;
    uint32_t w[64];
    for (int i = 0; i < 16; ++i) w[i] = s.pad_w[i];
    host::expand(w);
    const KW64 kw = pad_kw_const(s.p, (int)k);
    for (int t = 0; t < 64; ++t)
        if (kK256[t] + w[t] != kw.v[t]) return -1;
    if (k == 0)
        for (int q = 0; q < 8; ++q)
            if (s.mid[q] != kIV256[q]) return -1;
    return (int)k;
}

int size_launch(bm_ctx* ctx, DeviceCtx& d, const bm_segment_t& s, uint32_t part_off, Launch& L) {
    // the folded kernel where it applies and this build registered it (an
    // A/B build may instantiate only some layouts): else the generic one,
    // which gives the same answer
    const int fk = ctx->padc ? pad_fold_k(s) : -1;
    const void* fn = fk >= 0 ? g_search[2 + fk][s.p] : nullptr;
    const bool padc = fn != nullptr;
    if (!fn) fn = g_search[s.nbv - 1][s.p];
    if (!fn) return BM_EINTERNAL;
    int ms = std::max(1, std::min(s.max_inner, kMaxInnerDigits));
    // word LW holds one digit: the kernel steps the next one in word LW-1
    // (bm_kernels.hpp TWOW), so a task can still be 100 nonces
    if (s.p % 4 == 0 && s.p / 4 >= 1 && s.nd >= 2) ms = 2;
    const uint64_t resident = (uint64_t)blocks_per_cu(ctx, d, fn) * (uint64_t)d.cus;
    if (ctx->task_digits > 0) {
        ms = std::min(ms, ctx->task_digits);
    } else if (ms > 1) {
        // A launch with fewer 100-nonce tasks than twice its resident lanes
        // (the 1..8-digit segments of a search from 0) leaves SIMDs half
        // empty while each lane runs its one 100-nonce task: use 10-nonce
        // tasks instead, so every lane has work and the launch ends sooner.
        const uint64_t lanes = resident * (uint64_t)kBlock;
        const uint64_t tasks100 = (s.vhi - s.vlo) / 100 + 1;
        if (tasks100 < 2 * lanes) ms = 1;
    }
    const uint64_t S = kPow10[ms];
    const uint64_t t0 = s.vlo / S, t_end = s.vhi / S + 1;
    const uint64_t T = t_end - t0;
    // Tasks per lane per dequeue: about 100 nonces, but at least ~8 dequeues
    // per resident lane so the launch drains evenly (small launches: 1).
    const uint64_t m_max = std::max<uint64_t>(1, ctx->lane_chunk / S);
    const uint32_t m = (uint32_t)std::max<uint64_t>(
        1, std::min<uint64_t>(m_max, T / (8 * resident * (uint64_t)kBlock)));
    const uint64_t chunks = (T + 64ull * m - 1) / (64ull * m);
    const uint64_t grid = std::max<uint64_t>(1, std::min<uint64_t>((chunks + 3) / 4, resident));
    const uint64_t k = (chunks + grid * 4 - 1) / (grid * 4);  // chunks per wave (approx.)

    SearchArgs& A = L.args;
    std::memset(&A, 0, sizeof A);
    std::memcpy(A.mid, s.mid, sizeof A.mid);
    std::memcpy(A.tmpl, s.tmpl, sizeof A.tmpl);
    if (s.pad_block) {
        uint32_t w[64];
        for (int i = 0; i < 16; ++i) w[i] = s.pad_w[i];
        host::expand(w);
        for (int i = 0; i < 64; ++i) A.padkw[i] = kK256[i] + w[i];
    }
    A.vlo = s.vlo;
    A.vhi = s.vhi;
    A.nonce_base = s.nonce_base;
    A.t0 = t0;
    A.t_end = t_end;
    A.chunk_m = m;
    A.S = (uint32_t)S;
    A.ms = (uint32_t)ms;
    A.nd = (uint32_t)s.nd;
    A.part_off = part_off;
    L.fn = fn;
    L.grid = (uint32_t)grid;
    std::memset(&L.stat, 0, sizeof L.stat);
    L.stat.p = s.p;
    L.stat.nbv = s.nbv;
    L.stat.pad_block = padc ? 2 + fk : s.pad_block;
    L.stat.digits = s.digits;
    L.stat.inner_digits = ms;
    L.stat.nonces = s.vhi - s.vlo + 1;
    L.stat.grid = (uint32_t)grid;
    L.stat.tasks_per_thread = (uint32_t)(k * m);
    return BM_OK;
}

int ensure_counters(DeviceCtx& d, size_t n) {
    if (n <= d.ctr_cap) return BM_OK;
    if (d.d_ctr) BM_HIP(hipFree(d.d_ctr));
    if (d.h_ctr) BM_HIP(hipHostFree(d.h_ctr));
    d.d_ctr = nullptr;
    d.h_ctr = nullptr;
    d.ctr_cap = 0;
    size_t cap = std::max<size_t>(n, 256);
    BM_HIP(hipMalloc(&d.d_ctr, cap * kCtrStride * sizeof(unsigned long long)));
    BM_HIP(hipHostMalloc(&d.h_ctr, cap * kCtrStride * sizeof(unsigned long long), hipHostMallocDefault));
    d.ctr_cap = cap;
    return BM_OK;
}

int ensure_partials(DeviceCtx& d, size_t n) {
    if (n <= d.part_cap) return BM_OK;
    if (d.d_part) BM_HIP(hipFree(d.d_part));
    d.d_part = nullptr;
    d.part_cap = 0;
    size_t cap = std::max<size_t>(n, 4096);
    BM_HIP(hipMalloc(&d.d_part, cap * sizeof(Partial)));
    d.part_cap = cap;
    return BM_OK;
}

// nslots: partials the combine gathers (devices of the ctx, or ranks of its
// process group).
int init_device(DeviceCtx& d, int id, int nslots) {
    d.id = id;
    BM_HIP(hipSetDevice(id));
    hipDeviceProp_t prop;
    BM_HIP(hipGetDeviceProperties(&prop, id));
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) return BM_ENODEV;  // kernels are gfx950 code objects
    d.cus = prop.multiProcessorCount;
    int wall_khz = 0;
    if (hipDeviceGetAttribute(&wall_khz, hipDeviceAttributeWallClockRate, id) == hipSuccess && wall_khz > 0)
        d.wall_clock_hz = 1e3 * wall_khz;
    BM_HIP(hipStreamCreateWithFlags(&d.stream, hipStreamNonBlocking));
    d.nslots = nslots;
    BM_HIP(hipMalloc(&d.d_slot, sizeof(Slot)));
    BM_HIP(hipMalloc(&d.d_gather, sizeof(Slot) * (size_t)nslots));
    BM_HIP(hipHostMalloc(&d.h_slots, sizeof(Slot) * (size_t)(nslots + 1), hipHostMallocDefault));
    for (auto& e : d.ev) BM_HIP(hipEventCreate(&e));
    for (auto& s : d.aux) BM_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    BM_HIP(hipEventCreateWithFlags(&d.fork, hipEventDisableTiming));
    for (auto& e : d.join) BM_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    for (auto& e : d.bal) BM_HIP(hipEventCreate(&e));
    for (auto& e : d.ag) BM_HIP(hipEventCreate(&e));
    BM_HIP(hipEventCreateWithFlags(&d.own_done, hipEventDisableTiming));
    int rc = ensure_counters(d, 256);
    if (rc != BM_OK) return rc;
    return ensure_partials(d, 4096);
}

void destroy_device(DeviceCtx& d) {
    if (d.id < 0) return;
    (void)hipSetDevice(d.id);
    if (d.stream) (void)hipStreamSynchronize(d.stream);
    for (auto& s : d.aux)
        if (s) (void)hipStreamSynchronize(s);
    // abort, not destroy: the streams are drained, so nothing of ours is in
    // flight, and an abort never waits on a peer (a joined rank whose group
    // lost a member would otherwise block in teardown)
    if (d.comm) (void)ncclCommAbort(d.comm);
    d.comm = nullptr;
    for (auto& e : d.ev)
        if (e) (void)hipEventDestroy(e);
    if (d.d_part) (void)hipFree(d.d_part);
    if (d.d_ctr) (void)hipFree(d.d_ctr);
    if (d.h_ctr) (void)hipHostFree(d.h_ctr);
    if (d.d_slot) (void)hipFree(d.d_slot);
    if (d.d_gather) (void)hipFree(d.d_gather);
    if (d.d_hash_io) (void)hipFree(d.d_hash_io);
    if (d.d_test) (void)hipFree(d.d_test);
    if (d.h_slots) (void)hipHostFree(d.h_slots);
    if (d.own_done) (void)hipEventDestroy(d.own_done);
    for (auto& e : d.join)
        if (e) (void)hipEventDestroy(e);
    for (auto& e : d.bal)
        if (e) (void)hipEventDestroy(e);
    for (auto& e : d.ag)
        if (e) (void)hipEventDestroy(e);
    if (d.fork) (void)hipEventDestroy(d.fork);
    for (auto& s : d.aux)
        if (s) (void)hipStreamDestroy(s);
    if (d.stream) (void)hipStreamDestroy(d.stream);
}

bool distinct_devices(const bm_ctx* ctx) {
    for (size_t i = 0; i < ctx->devs.size(); ++i)
        for (size_t j = 0; j < i; ++j)
            if (ctx->devs[i].id == ctx->devs[j].id) return false;
    return true;
}

int ensure_nccl(bm_ctx* ctx) {
    if (ctx->nccl_ready) return BM_OK;
    // an RCCL communicator holds one rank per GPU: a device listed twice
    // (a one-GPU rehearsal of the N-device split) combines on the host
    if (!distinct_devices(ctx)) return BM_EINVAL;
    if (ctx->test_rccl_fault == 1) return BM_ERCCL;  // test hook
    const int n = (int)ctx->devs.size();
    std::vector<ncclComm_t> comms(n);
    std::vector<int> ids(n);
    for (int i = 0; i < n; ++i) ids[i] = ctx->devs[i].id;
    const auto t0 = std::chrono::steady_clock::now();
    if (ncclCommInitAll(comms.data(), n, ids.data()) != ncclSuccess) return BM_ERCCL;
    ctx->rccl_init_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    for (int i = 0; i < n; ++i) ctx->devs[i].comm = comms[i];
    ctx->nccl_ready = true;
    return BM_OK;
}

// Drops every communicator of the context after a failure (ncclCommAbort:
// also ends any collective of it still queued on a stream).
void abort_nccl(bm_ctx* ctx) {
    for (auto& d : ctx->devs) {
        if (!d.comm) continue;
        (void)hipSetDevice(d.id);
        (void)ncclCommAbort(d.comm);
        d.comm = nullptr;
    }
    ctx->nccl_ready = false;
    ctx->rccl_init_ms = 0.0;
}

// A non-blocking communicator's last operation: wait until it leaves
// ncclInProgress (or the deadline passes: BM_ETIMEDOUT).
int comm_settle(ncclComm_t comm, ncclResult_t r, std::chrono::steady_clock::time_point deadline, bool limited) {
    while (r == ncclInProgress) {
        if (limited && std::chrono::steady_clock::now() > deadline) return BM_ETIMEDOUT;
        std::this_thread::sleep_for(std::chrono::microseconds(50));
        if (ncclCommGetAsyncError(comm, &r) != ncclSuccess) return BM_ERCCL;
    }
    return r == ncclSuccess ? BM_OK : BM_ERCCL;
}

void join_worker(std::shared_ptr<JoinJob> job, int dev, int world, int rank, ncclUniqueId u) {
    ncclComm_t comm = nullptr;
    int rc = BM_ERCCL;
    const auto t0 = std::chrono::steady_clock::now();
    if (hipSetDevice(dev) == hipSuccess) {
        ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
        cfg.blocking = 0;
        ncclResult_t r = ncclCommInitRankConfig(&comm, world, u, rank, &cfg);
        trace("rank %d: init returned %d", rank, (int)r);
        while (r == ncclInProgress) {
            {
                std::lock_guard<std::mutex> g(job->m);
                if (job->abandoned) break;
            }
            std::this_thread::sleep_for(std::chrono::microseconds(200));
            if (ncclCommGetAsyncError(comm, &r) != ncclSuccess) r = ncclInternalError;
        }
        rc = r == ncclSuccess ? BM_OK : BM_ERCCL;
    }
    // publish; a communicator nobody will use (a failed set-up, or a caller
    // that gave up) is aborted first, outside the lock: an abort may block,
    // and the caller's timed wait must still be able to take the lock
    for (;;) {
        {
            std::lock_guard<std::mutex> g(job->m);
            if (!comm || (rc == BM_OK && !job->abandoned)) {
                job->comm = comm;
                job->rc = rc;
                job->init_ms =
                    std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
                job->done = true;
                job->cv.notify_all();
                return;
            }
        }
        (void)ncclCommAbort(comm);
        comm = nullptr;
        trace("rank %d: communicator aborted", rank);
    }
}

// Waits for everything a call may have queued on any stream of the context.
// Used when a call fails part-way: launches already on the aux streams keep
// running against d_ctr / d_part, so the next call (whose counter memset is
// ordered only on the main stream) must not start before they end.
void drain(bm_ctx* ctx) {
    for (auto& d : ctx->devs) {
        if (hipSetDevice(d.id) != hipSuccess) continue;
        (void)hipStreamSynchronize(d.stream);
        for (auto& s : d.aux)
            if (s) (void)hipStreamSynchronize(s);
    }
    (void)hipGetLastError();
}

// Stage 2 of a search, one device: enqueue its launches and its second-pass
// reduction (its partial lands in d_slot).  `enqueued` counts launches over
// every device (the test fault).  On failure the caller drains.
int enqueue_device(bm_ctx* ctx, int di, std::vector<Launch>& launches, uint32_t& first,
                   std::atomic<int>& enqueued) {
    DeviceCtx& d = ctx->devs[di];
    const bool mark = ctx->balance || ctx->timing;  // per-device span events
    BM_HIP(hipSetDevice(d.id));
    if (d.test_delay_us > 0) std::this_thread::sleep_for(std::chrono::microseconds(d.test_delay_us));
    // the call's first op on this device: its stream is idle, so it starts
    // about when it is submitted (the common start of bm_stats_t.dev_start_ms)
    if (mark) BM_HIP(hipEventRecord(d.bal[0], d.stream));
    d.submitted = std::chrono::steady_clock::now();
    uint32_t nparts = 0, li = 0;
    if (!launches.empty())
        BM_HIP(hipMemsetAsync(d.d_ctr, 0, launches.size() * kCtrStride * sizeof(unsigned long long), d.stream));
    // stream of each launch: biggest first, round-robin over the streams
    const int ns = std::max(1, std::min<int>(ctx->streams, (int)launches.size()));
    std::vector<uint32_t> order(launches.size());
    for (uint32_t i = 0; i < order.size(); ++i) order[i] = i;
    if (ns > 1) {
        std::stable_sort(order.begin(), order.end(),
                         [&](uint32_t x, uint32_t y) { return launches[x].stat.nonces > launches[y].stat.nonces; });
        BM_HIP(hipEventRecord(d.fork, d.stream));
        for (int k = 0; k + 1 < ns; ++k) BM_HIP(hipStreamWaitEvent(d.aux[k], d.fork, 0));
    }
    if (!order.empty()) first = order[0];
    for (uint32_t r = 0; r < order.size(); ++r) {
        li = order[r];
        Launch& L = launches[li];
        hipStream_t s = (r % ns) == 0 ? d.stream : d.aux[r % ns - 1];
        if (ctx->fault_after >= 0 && enqueued.fetch_add(1) >= ctx->fault_after) return BM_EINTERNAL;  // test hook
        const bool timed = ctx->timing && li < (uint32_t)kEventPairs;
        if (timed) BM_HIP(hipEventRecord(d.ev[2 * li], s));
        unsigned long long* ctr = d.d_ctr + kCtrStride * li;
        void* kargs[] = {&L.args, &d.d_part, &ctr};
        BM_HIP(hipLaunchKernel(L.fn, dim3(L.grid), dim3(kBlock), kargs, 0, s));
        if (timed) BM_HIP(hipEventRecord(d.ev[2 * li + 1], s));
        nparts += L.grid;
    }
    for (int k = 0; k + 1 < ns; ++k) {
        BM_HIP(hipEventRecord(d.join[k], d.aux[k]));
        BM_HIP(hipStreamWaitEvent(d.stream, d.join[k], 0));
    }
    // nparts = 0 (a device or rank with nothing to scan) writes (2^64-1, 2^64-1)
    reduce_partials<<<1, kReduceThreads, 0, d.stream>>>(d.d_part, nparts, &d.d_slot->p);
    BM_HIP(hipGetLastError());
    if (mark) BM_HIP(hipEventRecord(d.bal[1], d.stream));
    if (BM_CLOCK_PROBE && ctx->timing && !launches.empty())  // clock stamps, for the launch stats
        BM_HIP(hipMemcpyAsync(d.h_ctr, d.d_ctr, launches.size() * kCtrStride * sizeof(unsigned long long),
                              hipMemcpyDeviceToHost, d.stream));
    return BM_OK;
}

// f() as a status: an exception (std::bad_alloc from a plan or order vector,
// anything else a bug) becomes BM_ENOMEM / BM_EINTERNAL instead of leaving
// the C ABI -- or, on a submission thread, calling std::terminate and taking
// the host process down.
template <class F>
int guarded(F&& f) noexcept {
    try {
        return f();
    } catch (const std::bad_alloc&) {
        return BM_ENOMEM;
    } catch (...) {
        return BM_EINTERNAL;
    }
}

// Stage 2 of a search: every device's work.  A context of several devices
// submits each device's work from a host thread of its own (the context's
// SubmitPool, kept across searches since round 6), so device N-1 does not
// wait for the other devices' ~15 API calls each before it starts (the start
// skew of a serial submission; bm_stats_t.dev_start_ms reports what is left
// of it).
int enqueue(bm_ctx* ctx, std::vector<std::vector<Launch>>& launches, std::vector<uint32_t>& first) {
    const int ndev = (int)ctx->devs.size();
    if (ctx->fault_after == 0) return BM_EINTERNAL;  // test hook (also for a rank with nothing to scan)
    std::atomic<int> enqueued{0};
    ctx->stats.start_threads = 1;
    auto one = [&](int di) { return guarded([&] { return enqueue_device(ctx, di, launches[di], first[di], enqueued); }); };
    if (ndev == 1) return one(0);
    std::vector<int> rc(ndev, BM_OK);
    const std::function<void(int)> job = [&](int di) { rc[di] = one(di); };
    bool pooled = false;
    try {
        pooled = ctx->submit.run(ndev, job);
    } catch (...) {  // std::function or the pool's own bookkeeping: submit serially
        pooled = false;
    }
    if (!pooled)  // no threads: this one submits every device's work itself
        for (int di = 0; di < ndev; ++di) rc[di] = one(di);
    ctx->stats.start_threads = pooled ? 1 + ctx->submit.threads() : 1;
    for (int r : rc)
        if (r != BM_OK) return r;
    return BM_OK;
}

// What RCCL reports about the communicator(s) a combine just ran over, into
// the stats: its rank count, and each device's rank and the HIP device RCCL
// placed it on (bm_stats_t.rccl_*).  used = false (no RCCL combine), or a
// device without a communicator: 0 ranks, -1 elsewhere.
void record_rccl(bm_ctx* ctx, bool used) {
    bm_stats_t& st = ctx->stats;
    for (int i = 0; i < BM_MAX_STAT_DEVICES; ++i) st.dev_rccl_rank[i] = st.dev_rccl_device[i] = -1;
    st.rccl_nranks = 0;
    st.rccl_rank = -1;
    for (size_t di = 0; used && di < ctx->devs.size(); ++di) {
        ncclComm_t c = ctx->devs[di].comm;
        int n = 0, r = -1, dev = -1;
        if (!c || ncclCommCount(c, &n) != ncclSuccess) continue;
        if (ncclCommUserRank(c, &r) != ncclSuccess) r = -1;
        if (ncclCommCuDevice(c, &dev) != ncclSuccess) dev = -1;
        if (di == 0) {
            st.rccl_nranks = n;
            st.rccl_rank = r;
        }
        if (di < (size_t)BM_MAX_STAT_DEVICES) {
            st.dev_rccl_rank[di] = r;
            st.dev_rccl_device[di] = dev;
        }
    }
}

// The allgather's event pair on each device (timing on; the streams have
// been synchronised): bm_stats_t.dev_allgather_ms and their max.
void record_allgather(bm_ctx* ctx) {
    bm_stats_t& st = ctx->stats;
    for (size_t di = 0; di < ctx->devs.size() && di < (size_t)BM_MAX_STAT_DEVICES; ++di) {
        DeviceCtx& d = ctx->devs[di];
        float ms = 0.f;
        if (hipSetDevice(d.id) != hipSuccess || hipEventElapsedTime(&ms, d.ag[0], d.ag[1]) != hipSuccess) continue;
        st.dev_allgather_ms[di] = ms;
        st.rccl_allgather_ms = std::max(st.rccl_allgather_ms, (double)ms);
    }
}

Partial lex_min_slots(const Slot* s, int n) {
    Partial best{UINT64_MAX, UINT64_MAX};
    for (int i = 0; i < n; ++i) {
        const Partial& p = s[i].p;
        if (p.hash < best.hash || (p.hash == best.hash && p.nonce < best.nonce)) best = p;
    }
    return best;
}

// Stage 3 of a search, one process: combine the devices' partials with one
// RCCL allgather, or by host copies (BM_COMBINE_HOST, a device listed twice,
// or RCCL failing at run time: the context then aborts its communicators and
// stays on host copies, reported in the stats).  A rank context outside a
// group copies its own partial.
int combine_local(bm_ctx* ctx, Partial* best_out) {
    bm_stats_t& st = ctx->stats;
    const int ndev = (int)ctx->devs.size();
    int nslots = ndev;
    bool via_rccl = false;
    if (!ctx->rank_ctx) {
        const bool distinct = distinct_devices(ctx);
        if (ctx->combine == BM_COMBINE_RCCL && !distinct) return BM_EINVAL;
        const bool want = ctx->combine == BM_COMBINE_RCCL || (ctx->combine == BM_COMBINE_AUTO && ndev > 1 && distinct);
        if (want && ctx->rccl_status == 0) {
            int rc = ensure_nccl(ctx);
            if (rc == BM_OK) {
                for (int di = 0; di < ndev && rc == BM_OK; ++di) {
                    DeviceCtx& d = ctx->devs[di];
                    if (hipSetDevice(d.id) != hipSuccess ||
                        hipMemsetAsync(&d.d_slot->status, 0, 2 * sizeof(uint64_t), d.stream) != hipSuccess ||
                        (ctx->timing && hipEventRecord(d.ag[0], d.stream) != hipSuccess))
                        return BM_EHIP;
                }
                if (ctx->test_rccl_fault == 2) {
                    rc = BM_ERCCL;  // test hook: as if the grouped allgather failed
                } else if (ncclGroupStart() != ncclSuccess) {
                    rc = BM_ERCCL;
                } else {
                    for (int di = 0; di < ndev && rc == BM_OK; ++di) {
                        DeviceCtx& d = ctx->devs[di];
                        if (ncclAllGather(d.d_slot, d.d_gather, kSlotWords, ncclUint64, d.comm, d.stream) !=
                            ncclSuccess)
                            rc = BM_ERCCL;
                    }
                    if (ncclGroupEnd() != ncclSuccess) rc = BM_ERCCL;
                }
                // the allgather's span on each device: from the end of its own
                // reduction (recorded before the collective was enqueued) to the
                // collective's end, so it includes the wait for the slowest device
                for (int di = 0; di < ndev && rc == BM_OK && ctx->timing; ++di) {
                    DeviceCtx& d = ctx->devs[di];
                    if (hipSetDevice(d.id) != hipSuccess || hipEventRecord(d.ag[1], d.stream) != hipSuccess)
                        return BM_EHIP;
                }
            }
            if (rc == BM_OK) {
                DeviceCtx& d0 = ctx->devs[0];
                BM_HIP(hipSetDevice(d0.id));
                BM_HIP(hipMemcpyAsync(d0.h_slots, d0.d_gather, sizeof(Slot) * ndev, hipMemcpyDeviceToHost,
                                      d0.stream));
                via_rccl = true;
            } else if (rc == BM_ERCCL) {
                ctx->rccl_status = rc;  // fall back to host copies, now and for every later call
                abort_nccl(ctx);
            } else {
                return rc;
            }
        }
    } else {
        nslots = 1;  // a rank outside a group: its own partial
    }
    if (!via_rccl) {
        for (int di = 0; di < ndev; ++di) {
            DeviceCtx& d = ctx->devs[di];
            BM_HIP(hipSetDevice(d.id));
            BM_HIP(hipMemcpyAsync(ctx->devs[0].h_slots + di, d.d_slot, sizeof(Partial), hipMemcpyDeviceToHost,
                                  d.stream));
        }
    }
    // the end of every device's own work (its reduction, bal[1]) seen on the
    // host: from there on the wait is the combine's (bm_stats_t.combine_ms)
    if (ctx->balance || ctx->timing)
        for (int di = 0; di < ndev; ++di) {
            BM_HIP(hipSetDevice(ctx->devs[di].id));
            BM_HIP(hipEventSynchronize(ctx->devs[di].bal[1]));
        }
    const auto t_own = std::chrono::steady_clock::now();
    for (int di = 0; di < ndev; ++di) {
        BM_HIP(hipSetDevice(ctx->devs[di].id));
        BM_HIP(hipStreamSynchronize(ctx->devs[di].stream));
    }
    st.combine_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_own).count();
    st.combine_used = ctx->rank_ctx ? BM_COMBINED_LOCAL : via_rccl ? BM_COMBINED_RCCL : BM_COMBINED_HOST;
    st.rccl_status = ctx->rccl_status;
    record_rccl(ctx, via_rccl);
    if (via_rccl && ctx->timing) record_allgather(ctx);
    *best_out = lex_min_slots(ctx->devs[0].h_slots, nslots);
    return BM_OK;
}

// Stage 3 of a search, a rank of a group: one allgather of every rank's
// slot.  A rank whose call failed before this point (own_rc) still takes
// part, with its status in the slot, so the group fails the call together
// instead of waiting for it.  The wait for the group after this rank's own
// work is bounded by peer_timeout_ms (then the communicator is aborted).
int combine_group(bm_ctx* ctx, int own_rc, Partial* best_out) {
    bm_stats_t& st = ctx->stats;
    DeviceCtx& d = ctx->devs[0];
    const int world = ctx->world;
    // Post this rank's slot.  A HIP failure while staging it becomes this
    // rank's status (it still takes part, so the group fails the call
    // together instead of waiting for it); only a slot that cannot be posted
    // at all leaves the group (abort below).
    bool posted = hipSetDevice(d.id) == hipSuccess;
    if (posted && own_rc == BM_OK &&
        hipMemsetAsync(&d.d_slot->status, 0, 2 * sizeof(uint64_t), d.stream) != hipSuccess)
        own_rc = BM_EHIP;
    if (posted && own_rc != BM_OK) {
        Slot& out = d.h_slots[d.nslots];  // pinned staging slot
        out = Slot{Partial{UINT64_MAX, UINT64_MAX}, (uint64_t)(int64_t)own_rc, 0};
        posted = hipMemcpyAsync(d.d_slot, &out, sizeof(Slot), hipMemcpyHostToDevice, d.stream) == hipSuccess;
    }
    // the end of this rank's own work, from which the peer timeout counts
    // (without the event: from the moment the allgather is enqueued)
    const bool own_mark = posted && hipEventRecord(d.own_done, d.stream) == hipSuccess;
    auto t_own = std::chrono::steady_clock::now();
    const bool limited = ctx->peer_timeout_ms > 0;
    int rc = BM_OK;
    bool copied = false;
    if (!posted) {
        rc = own_rc != BM_OK ? own_rc : BM_EHIP;
    } else if (ctx->test_rccl_fault == 2) {
        rc = BM_ERCCL;  // test hook: as if the allgather failed (world 1 only: no peer is left waiting)
    } else {
        // the allgather goes on the stream behind this rank's own work (a
        // non-blocking communicator may first report ncclInProgress: then it
        // is enqueued once the communicator settles)
        const auto timeout = std::chrono::milliseconds(ctx->peer_timeout_ms);
        const bool ag_timed = ctx->timing && hipEventRecord(d.ag[0], d.stream) == hipSuccess;
        rc = comm_settle(d.comm, ncclAllGather(d.d_slot, d.d_gather, kSlotWords, ncclUint64, d.comm, d.stream),
                         std::chrono::steady_clock::now() + timeout, limited);
        // the allgather's span on this rank's stream: from the end of its own
        // work to the end of the collective (the wait for the slowest rank included)
        if (rc == BM_OK && ag_timed) (void)hipEventRecord(d.ag[1], d.stream);
        // a failed copy of the gathered slots is this rank's own error: the
        // collective itself still runs, so the communicator stays good
        copied = rc == BM_OK && hipMemcpyAsync(d.h_slots, d.d_gather, sizeof(Slot) * world,
                                               hipMemcpyDeviceToHost, d.stream) == hipSuccess;
        // only the wait for the other ranks is bounded
        if (own_mark) (void)hipEventSynchronize(d.own_done);
        t_own = std::chrono::steady_clock::now();  // this rank's own work is done: the rest is the group's
        const auto deadline = t_own + timeout;
        if (rc == BM_OK && !limited && hipStreamSynchronize(d.stream) != hipSuccess) rc = BM_EHIP;
        for (auto pause = std::chrono::microseconds(10); rc == BM_OK && limited;) {
            const hipError_t q = hipStreamQuery(d.stream);
            if (q == hipSuccess) break;
            if (q != hipErrorNotReady) {
                rc = BM_EHIP;  // the stream itself failed: the allgather's fate is unknown
                break;
            }
            if (std::chrono::steady_clock::now() > deadline) {
                rc = BM_ETIMEDOUT;
                break;
            }
            std::this_thread::sleep_for(pause);
            pause = std::min(pause * 2, std::chrono::microseconds(100));
        }
    }
    if (rc != BM_OK) {
        // the communicator cannot be trusted any more: abort it (this also
        // ends an allgather still waiting on the stream); later searches
        // return the same status until bm_ctx_leave_rank
        if (d.comm) (void)ncclCommAbort(d.comm);
        d.comm = nullptr;
        ctx->group_status = rc;
        (void)hipStreamSynchronize(d.stream);
        (void)hipGetLastError();
        st.rccl_status = rc;
        return own_rc != BM_OK ? own_rc : rc;  // this rank's own failure stays the one it reports
    }
    st.combine_used = BM_COMBINED_RCCL;
    st.combine_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_own).count();
    record_rccl(ctx, true);
    if (ctx->timing) record_allgather(ctx);
    if (!copied) return own_rc != BM_OK ? own_rc : BM_EHIP;
    // test hook: the last slot arrives carrying a peer's failure status, as
    // a real peer's would (at world 1 that slot is this rank's own)
    if (ctx->test_rccl_fault == 3) d.h_slots[world - 1].status = (uint64_t)(int64_t)BM_EHIP;
    for (int r = 0; r < world; ++r)
        if (d.h_slots[r].status != 0) return own_rc != BM_OK ? own_rc : BM_EPEER;
    if (own_rc != BM_OK) return own_rc;
    *best_out = lex_min_slots(d.h_slots, world);
    return BM_OK;
}

// Stage 1 of a search: this process's piece (rank contexts: every rank
// passes the same range and scans its contiguous share of it), split over
// the devices (the partitioner: slot_pieces over ctx->shares; an empty piece
// has lo > hi); plan and size every launch.
int plan_launches(bm_ctx* ctx, const uint8_t* msg, size_t len, uint64_t lower, uint64_t upper,
                  std::vector<std::vector<Launch>>& launches) {
    bm_stats_t& st = ctx->stats;
    const int ndev = (int)ctx->devs.size();
    uint64_t lo = lower, hi = upper;
    bool have = true;
    if (ctx->rank_ctx) {
        const Piece mine = slot_pieces(lower, upper, ctx->world, ctx->shares)[(size_t)ctx->rank];
        lo = mine.lo;
        hi = mine.hi;
        have = lo <= hi;  // else a range shorter than the group (or a tiny share): nothing here
    }
    if (have) st.nonces = hi - lo + 1;  // wraps to 0 only for the full 2^64 range
    const std::vector<Piece> pieces =
        slot_pieces(have ? lo : 1, have ? hi : 0, ndev, ctx->rank_ctx ? std::vector<uint32_t>() : ctx->shares);
    for (int di = 0; di < ndev; ++di) {
        ctx->devs[di].piece_nonces = pieces[di].lo <= pieces[di].hi ? pieces[di].hi - pieces[di].lo + 1 : 0;
        if (pieces[di].lo > pieces[di].hi) continue;
        std::vector<bm_segment_t> segs;
        int rc = plan_segments(msg, len, pieces[di].lo, pieces[di].hi, segs, ctx->max_windows);
        if (rc != BM_OK) return rc;
        // With streams to overlap on, the biggest segment's last tail_nonces
        // become a launch of their own: it is small enough for 10-nonce tasks
        // (size_launch), so the call ends on a short drain instead of half a
        // 100-nonce task.
        if (ctx->streams > 1 && ctx->tail_nonces > 0 && !segs.empty()) {
            size_t big = 0;
            for (size_t i = 1; i < segs.size(); ++i)
                if (segs[i].vhi - segs[i].vlo > segs[big].vhi - segs[big].vlo) big = i;
            bm_segment_t& b = segs[big];
            if ((b.vhi - b.vlo) / 8 >= ctx->tail_nonces) {
                bm_segment_t t = b;
                t.vlo = b.vhi - ctx->tail_nonces + 1;
                b.vhi = t.vlo - 1;
                segs.push_back(t);
            }
        }
        uint32_t off = 0;
        for (const auto& s : segs) {
            Launch L;
            rc = size_launch(ctx, ctx->devs[di], s, off, L);
            if (rc != BM_OK) return rc;
            L.stat.device = di;
            off += L.grid;
            launches[di].push_back(L);
        }
        BM_HIP(hipSetDevice(ctx->devs[di].id));
        rc = ensure_partials(ctx->devs[di], off);
        if (rc != BM_OK) return rc;
        rc = ensure_counters(ctx->devs[di], launches[di].size());
        if (rc != BM_OK) return rc;
    }
    return BM_OK;
}

// The RCCL figures every call reports, whatever its outcome: the library's
// RCCL version and, while the context holds a communicator, the time it took
// to form.
int rccl_version() {
    static const int v = [] {
        int x = 0;
        return ncclGetVersion(&x) == ncclSuccess ? x : 0;
    }();
    return v;
}

void stamp_common(bm_ctx* ctx) {
    bm_stats_t& st = ctx->stats;
    st.rccl_version = rccl_version();
    const bool have = ctx->rank_ctx ? ctx->joined && ctx->devs[0].comm != nullptr : ctx->nccl_ready;
    st.rccl_init_ms = have ? ctx->rccl_init_ms : 0.0;
    if (st.start_threads == 0) st.start_threads = 1;
}

int search_impl(bm_ctx* ctx, const uint8_t* msg, size_t len, uint64_t lower, uint64_t upper, bm_result_t* out) {
    const auto t_start = std::chrono::steady_clock::now();
    bm_stats_t& st = ctx->stats;
    std::memset(&st, 0, sizeof st);
    record_rccl(ctx, false);
    const int ndev = (int)ctx->devs.size();
    const bool group = ctx->rank_ctx && ctx->joined;
    if (group && ctx->group_status != BM_OK) {  // the communicator failed earlier: leave the group first
        st.rccl_status = ctx->group_status;
        stamp_common(ctx);
        return ctx->group_status;
    }
    if (lower > upper) {  // miner.go:45-46 with zero iterations (every rank sees the same range)
        stamp_common(ctx);
        out->hash = UINT64_MAX;
        out->nonce = UINT64_MAX;
        return BM_OK;
    }

    // 1-2. plan and size every launch; enqueue them and each device's
    // second-pass reduction.  A failure part-way drains every stream first,
    // so the context stays usable.
    std::vector<std::vector<Launch>> launches(ndev);
    std::vector<uint32_t> first(ndev, 0);
    int rc = guarded([&] { return plan_launches(ctx, msg, len, lower, upper, launches); });
    if (rc == BM_OK) rc = enqueue(ctx, launches, first);
    if (rc != BM_OK) drain(ctx);

    // 3. combine (a rank of a group takes part even after a failure)
    Partial best{UINT64_MAX, UINT64_MAX};
    if (group) {
        const int grc = combine_group(ctx, rc, &best);
        if (grc != BM_OK) {
            drain(ctx);
            const int keep = st.rccl_status;
            std::memset(&st, 0, sizeof st);
            record_rccl(ctx, false);
            st.rccl_status = keep;
            stamp_common(ctx);
            return grc;
        }
    } else {
        if (rc == BM_OK) rc = combine_local(ctx, &best);
        if (rc != BM_OK) {
            drain(ctx);
            std::memset(&st, 0, sizeof st);
            record_rccl(ctx, false);
            stamp_common(ctx);
            return rc;
        }
    }

    // each device's start against the earliest device's (host submission times)
    std::vector<double> start_ms(ndev, 0.0);
    {
        auto t0 = ctx->devs[0].submitted;
        for (const auto& d : ctx->devs) t0 = std::min(t0, d.submitted);
        for (int di = 0; di < ndev; ++di)
            start_ms[di] = std::chrono::duration<double, std::milli>(ctx->devs[di].submitted - t0).count();
    }

    // 4. balance: the next call's shares follow each device's measured rate,
    // its nonces over the time from the call's common start to its reduction,
    // so a device that starts late gets a smaller piece
    if (ctx->balance && ndev > 1) {
        std::vector<double> rate(ndev, 0.0);
        bool ok = true;
        for (int di = 0; di < ndev && ok; ++di) {
            DeviceCtx& d = ctx->devs[di];
            float ms = 0.f;
            ok = d.piece_nonces >= kBalanceMinNonces && hipSetDevice(d.id) == hipSuccess &&
                 hipEventElapsedTime(&ms, d.bal[0], d.bal[1]) == hipSuccess && ms > 0.f;
            // a start offset counts only when it is more than host jitter
            // (thread scheduling: sub-ms to ms on a loaded host), so shares
            // move only for a persistent late start
            const double late = start_ms[di] >= std::max(kBalanceStartMinMs, kBalanceStartMinFrac * ms) ? start_ms[di]
                                                                                                          : 0.0;
            if (ok) rate[di] = (double)d.piece_nonces / (late + ms);
        }
        if (ok) {
            const double top = *std::max_element(rate.begin(), rate.end());
            ctx->shares.assign(ndev, 1);
            for (int di = 0; di < ndev; ++di)
                ctx->shares[di] = (uint32_t)std::max(1.0, std::floor(rate[di] / top * kShareScale + 0.5));
        }
    }

    // 5. statistics
    st.devices = (uint32_t)std::min(ndev, BM_MAX_STAT_DEVICES);
    for (int di = 0; di < ndev; ++di) {
        DeviceCtx& d = ctx->devs[di];
        if (di < BM_MAX_STAT_DEVICES) {
            st.dev_nonces[di] = d.piece_nonces;
            if (ctx->timing || ctx->balance) st.dev_start_ms[di] = start_ms[di];
            float ms = 0.f;
            if ((ctx->timing || ctx->balance) && hipSetDevice(d.id) == hipSuccess &&
                hipEventElapsedTime(&ms, d.bal[0], d.bal[1]) == hipSuccess)
                st.dev_span_ms[di] = ms;
        }
        uint32_t li = 0;
        const bool span_ok = ctx->timing && !launches[di].empty() && first[di] < (uint32_t)kEventPairs;
        for (Launch& L : launches[di]) {
            ++st.launches;
            if (ctx->timing && li < (uint32_t)kEventPairs) {
                float ms = 0.f;
                BM_HIP(hipEventElapsedTime(&ms, d.ev[2 * li], d.ev[2 * li + 1]));
                L.stat.ms = ms;
                st.kernel_ms += ms;
                const unsigned long long* c = d.h_ctr + kCtrStride * li + kClockSlot - 1;
                if (BM_CLOCK_PROBE && c[4] > c[2] && c[3] > c[1])  // shader cycles over constant-rate ticks
                    L.stat.clock_ghz = (double)(c[3] - c[1]) / ((double)(c[4] - c[2]) / d.wall_clock_hz) / 1e9;
                if (span_ok) {  // the first launch's start to this launch's end
                    float sp = 0.f;
                    BM_HIP(hipEventElapsedTime(&sp, d.ev[2 * first[di]], d.ev[2 * li + 1]));
                    st.span_ms = std::max(st.span_ms, (double)sp);
                }
            }
            if (st.recorded < BM_MAX_LAUNCH_STATS) st.launch[st.recorded++] = L.stat;
            ++li;
        }
    }
    stamp_common(ctx);
    st.wall_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_start).count();
    out->hash = best.hash;
    out->nonce = best.nonce;
    return BM_OK;
}

// bm_reduce_gpu: n partials, one per lane, through block_min (ds_swizzle
// butterflies, readlane, LDS) and then reduce_partials -- the reductions the
// search uses above its per-lane scans.
int reduce_impl(bm_ctx* ctx, const bm_result_t* in, size_t n, bm_result_t* out) {
    DeviceCtx& d = ctx->devs[0];
    BM_HIP(hipSetDevice(d.id));
    const size_t blocks = (n + kBlock - 1) / kBlock;
    const size_t need = n + blocks + 1;
    if (need > d.test_cap) {
        if (d.d_test) BM_HIP(hipFree(d.d_test));
        d.d_test = nullptr;
        d.test_cap = 0;
        BM_HIP(hipMalloc(&d.d_test, need * sizeof(Partial)));
        d.test_cap = need;
    }
    Partial* d_in = d.d_test;
    Partial* d_blk = d.d_test + n;
    Partial* d_out = d_blk + blocks;
    if (n) BM_HIP(hipMemcpyAsync(d_in, in, n * sizeof(Partial), hipMemcpyHostToDevice, d.stream));
    if (blocks) {
        lane_partials_min<<<dim3((uint32_t)blocks), kBlock, 0, d.stream>>>(d_in, (uint32_t)n, d_blk);
        BM_HIP(hipGetLastError());
    }
    reduce_partials<<<1, kReduceThreads, 0, d.stream>>>(d_blk, (uint32_t)blocks, d_out);
    BM_HIP(hipGetLastError());
    Partial r;
    BM_HIP(hipMemcpyAsync(&r, d_out, sizeof r, hipMemcpyDeviceToHost, d.stream));
    BM_HIP(hipStreamSynchronize(d.stream));
    out->hash = r.hash;
    out->nonce = r.nonce;
    return BM_OK;
}

int hash_impl(bm_ctx* ctx, const uint8_t* msg, size_t len, const uint64_t* nonces, size_t n, uint64_t* out) {
    if (n == 0) return BM_OK;
    DeviceCtx& d = ctx->devs[0];
    BM_HIP(hipSetDevice(d.id));
    HashArgs A;
    std::memset(&A, 0, sizeof A);
    // midstate over the whole 64-byte blocks of "msg "
    const uint64_t pre = (uint64_t)len + 1;
    const uint64_t full = pre / 64;
    uint32_t st[8];
    for (int i = 0; i < 8; ++i) st[i] = kIV256[i];
    uint8_t blk[64];
    for (uint64_t b = 0; b < full; ++b) {
        for (int i = 0; i < 64; ++i) {
            const uint64_t pos = b * 64 + (uint64_t)i;
            blk[i] = pos < len ? msg[pos] : (uint8_t)' ';
        }
        host::compress_bytes(st, blk);
    }
    std::memcpy(A.mid, st, sizeof st);
    A.tail_len = (uint32_t)(pre - full * 64);
    for (uint32_t i = 0; i < A.tail_len; ++i) {
        const uint64_t pos = full * 64 + i;
        A.tail[i] = pos < len ? msg[pos] : (uint8_t)' ';
    }
    A.total_prefix = pre;
    A.n = n;
    if (n > d.hash_cap) {
        if (d.d_hash_io) BM_HIP(hipFree(d.d_hash_io));
        d.d_hash_io = nullptr;
        d.hash_cap = 0;
        BM_HIP(hipMalloc(&d.d_hash_io, 2 * n * sizeof(uint64_t)));
        d.hash_cap = n;
    }
    BM_HIP(hipMemcpyAsync(d.d_hash_io, nonces, n * sizeof(uint64_t), hipMemcpyHostToDevice, d.stream));
    const uint64_t grid = (n + kHashThreads - 1) / kHashThreads;
    hash_kernel<<<dim3((uint32_t)grid), kHashThreads, 0, d.stream>>>(A, d.d_hash_io, d.d_hash_io + n);
    BM_HIP(hipGetLastError());
    BM_HIP(hipMemcpyAsync(out, d.d_hash_io + n, n * sizeof(uint64_t), hipMemcpyDeviceToHost, d.stream));
    BM_HIP(hipStreamSynchronize(d.stream));
    return BM_OK;
}

}  // namespace
}  // namespace bm

// ------------------------------------------------------------------ C ABI --

extern "C" {

int bm_abi_version(void) { return BM_ABI_VERSION; }

const char* bm_strerror(int status) {
    switch (status) {
        case BM_OK: return "ok";
        case BM_EINVAL: return "invalid argument";
        case BM_ENODEV: return "no usable gfx950 device";
        case BM_EHIP: return "HIP runtime error";
        case BM_ERCCL: return "RCCL error";
        case BM_ENOMEM: return "out of memory";
        case BM_EINTERNAL: return "internal error";
        case BM_EPEER: return "another rank of the group failed";
        case BM_ETIMEDOUT: return "the group did not answer within the peer timeout";
        default: return "unknown status";
    }
}

int bm_device_count(int* out) {
    if (!out) return BM_EINVAL;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
    *out = n;
    return BM_OK;
}

int bm_device_pci_bus_id(int device, char* buf, int len) {
    if (!buf || len < 13) return BM_EINVAL;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || device < 0 || device >= n) return BM_ENODEV;
    return hipDeviceGetPCIBusId(buf, len, device) == hipSuccess ? BM_OK : BM_EHIP;
}

}  // extern "C"

namespace bm {
namespace {
// Environment knobs read at context creation.  Malformed or out-of-range
// values keep the default (results never depend on them).
void read_env(bm_ctx* ctx) {
    if (const char* e = std::getenv("BTCMINER_STREAMS")) {
        const int v = std::atoi(e);
        if (v >= 1 && v <= kMaxStreams) ctx->streams = v;
    }
    if (const char* e = std::getenv("BTCMINER_TAIL")) {
        char* end = nullptr;
        errno = 0;
        const unsigned long long v = std::strtoull(e, &end, 10);
        if (end != e && *end == '\0' && errno == 0 && v <= kMaxTailNonces) ctx->tail_nonces = v;
    }
    if (const char* e = std::getenv("BTCMINER_PADC")) ctx->padc = std::strcmp(e, "0") != 0;
    if (const char* e = std::getenv("BTCMINER_CHUNK")) {
        char* end = nullptr;
        errno = 0;
        const unsigned long long v = std::strtoull(e, &end, 10);
        if (end != e && *end == '\0' && errno == 0 && v >= 10 && v <= 100000) ctx->lane_chunk = v;
    }

}

int create_ctx(const int* devices, int n, int nslots, bm_ctx** out) {
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count < 1) return BM_ENODEV;
    for (int i = 0; i < n; ++i)
        if (devices[i] < 0 || devices[i] >= count) return BM_ENODEV;
    bm_ctx* ctx = new (std::nothrow) bm_ctx();
    if (!ctx) return BM_ENOMEM;
    std::memset(&ctx->stats, 0, sizeof ctx->stats);
    record_rccl(ctx, false);
    read_env(ctx);
    DeviceGuard guard;
    ctx->devs.resize(n);
    for (int i = 0; i < n; ++i) {
        int rc = init_device(ctx->devs[i], devices[i], nslots);
        if (rc != BM_OK) {
            for (auto& d : ctx->devs) destroy_device(d);
            delete ctx;
            return rc;
        }
    }
    *out = ctx;
    return BM_OK;
}
}  // namespace
}  // namespace bm

extern "C" {

int bm_ctx_create_devices(const int* devices, int n, bm_ctx_t** out) {
    if (!out || !devices || n < 1) return BM_EINVAL;
    return bm::create_ctx(devices, n, n, out);
}

int bm_rccl_unique_id(uint8_t* id) {
    if (!id) return BM_EINVAL;
    static_assert(sizeof(ncclUniqueId) == BM_RCCL_ID_BYTES, "RCCL unique id size");
    ncclUniqueId u;
    if (ncclGetUniqueId(&u) != ncclSuccess) return BM_ERCCL;
    std::memcpy(id, &u, sizeof u);
    return BM_OK;
}

int bm_ctx_create_rank_local(int device, int rank, int world, bm_ctx_t** out) {
    if (!out || world < 1 || world > BM_MAX_SLOTS || rank < 0 || rank >= world) return BM_EINVAL;
    bm_ctx* ctx = nullptr;
    int rc = bm::create_ctx(&device, 1, world, &ctx);
    if (rc != BM_OK) return rc;
    ctx->rank = rank;
    ctx->world = world;
    ctx->rank_ctx = true;
    *out = ctx;
    return BM_OK;
}

int bm_ctx_join_rank(bm_ctx_t* ctx, const uint8_t* id, int timeout_ms) {
    if (!ctx || !id || !ctx->rank_ctx || ctx->joined || timeout_ms < 0) return BM_EINVAL;
    if (ctx->test_rccl_fault == 1) return BM_ERCCL;  // test hook
    bm::DeviceGuard guard;
    bm::DeviceCtx& d = ctx->devs[0];
    if (hipSetDevice(d.id) != hipSuccess) return BM_EHIP;
    ncclUniqueId u;
    std::memcpy(&u, id, sizeof u);
    const int dev = d.id, world = ctx->world, rank = ctx->rank;
    // one deadline for the whole call: the wait for a pending join and the
    // new join share timeout_ms
    const auto deadline = std::chrono::steady_clock::now() + std::chrono::milliseconds(timeout_ms);
    // An earlier join this context gave up on may still be inside RCCL: wait
    // for it (within this call's timeout) rather than put a second worker
    // there; it has abandoned = true, so it aborts whatever it ends with.
    if (ctx->pending_join) {
        auto& pj = ctx->pending_join;
        std::unique_lock<std::mutex> lk(pj->m);
        const bool ended = timeout_ms == 0 ? (pj->cv.wait(lk, [&] { return pj->done; }), true)
                                           : pj->cv.wait_until(lk, deadline, [&] { return pj->done; });
        lk.unlock();
        if (!ended) {
            bm::trace("rank %d: the previous join is still inside RCCL; not starting another", rank);
            return BM_ETIMEDOUT;
        }
        ctx->pending_worker.join();
        ctx->pending_join.reset();
        if (timeout_ms > 0 && std::chrono::steady_clock::now() >= deadline) {
            bm::trace("rank %d: the previous join ended, but no time is left for a new one", rank);
            return BM_ETIMEDOUT;
        }
    }
    // The join runs on a worker thread: a non-blocking ncclCommInitRankConfig
    // polled until it settles.  With a timeout the caller waits at most that
    // long; past it the worker becomes the context's pending join (neither
    // the init of a group whose peer never comes nor its abort is guaranteed
    // to return promptly), and the call returns BM_ETIMEDOUT.
    auto job = std::make_shared<bm::JoinJob>();
    bm::trace("rank %d/%d: joining (timeout %d ms)", rank, world, timeout_ms);
    std::thread worker([job, dev, world, rank, u]() { bm::join_worker(job, dev, world, rank, u); });
    std::unique_lock<std::mutex> lk(job->m);
    if (timeout_ms == 0) {
        job->cv.wait(lk, [&] { return job->done; });
    } else if (!job->cv.wait_until(lk, deadline, [&] { return job->done; })) {
        job->abandoned = true;
        lk.unlock();
        ctx->pending_join = job;
        ctx->pending_worker = std::move(worker);
        bm::trace("rank %d: join timed out; the worker aborts the communicator if it ever gets one", rank);
        return BM_ETIMEDOUT;
    }
    lk.unlock();
    worker.join();
    bm::trace("rank %d: join status %d", rank, job->rc);
    if (job->rc != BM_OK) return job->rc;
    d.comm = job->comm;
    ctx->rccl_init_ms = job->init_ms;
    ctx->joined = true;
    ctx->group_status = BM_OK;
    return BM_OK;
}

int bm_ctx_leave_rank(bm_ctx_t* ctx) {
    if (!ctx || !ctx->rank_ctx) return BM_EINVAL;
    bm::DeviceGuard guard;
    bm::DeviceCtx& d = ctx->devs[0];
    if (d.comm) {
        // leaving is what a rank does when the group cannot be trusted (a
        // peer failed to join, or the caller falls back): abort, which frees
        // this rank's side without waiting for any peer
        (void)hipSetDevice(d.id);
        (void)hipStreamSynchronize(d.stream);
        (void)ncclCommAbort(d.comm);
        d.comm = nullptr;
    }
    ctx->joined = false;
    ctx->group_status = BM_OK;
    return BM_OK;
}

int bm_ctx_rank_joined(const bm_ctx_t* ctx, int* joined) {
    if (!ctx || !joined) return BM_EINVAL;
    *joined = ctx->joined ? 1 : 0;
    return BM_OK;
}

int bm_ctx_set_peer_timeout(bm_ctx_t* ctx, int timeout_ms) {
    if (!ctx || timeout_ms < 0) return BM_EINVAL;
    ctx->peer_timeout_ms = timeout_ms;
    return BM_OK;
}

int bm_ctx_create_rank(int device, int rank, int world, const uint8_t* id, bm_ctx_t** out) {
    if (!out || !id) return BM_EINVAL;
    bm_ctx* ctx = nullptr;
    int rc = bm_ctx_create_rank_local(device, rank, world, &ctx);
    if (rc != BM_OK) return rc;
    rc = bm_ctx_join_rank(ctx, id, 0);  // blocks until every rank of the group has joined
    if (rc != BM_OK) {
        bm_ctx_destroy(ctx);
        return rc;
    }
    *out = ctx;
    return BM_OK;
}

int bm_ctx_rank(const bm_ctx_t* ctx, int* rank, int* world) {
    if (!ctx || !rank || !world) return BM_EINVAL;
    *rank = ctx->rank;
    *world = ctx->world;
    return BM_OK;
}

int bm_ctx_create(int num_gpus, bm_ctx_t** out) {
    if (!out || num_gpus < 0) return BM_EINVAL;
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count < 1) return BM_ENODEV;
    if (num_gpus == 0) num_gpus = count;
    if (num_gpus > count) return BM_ENODEV;
    std::vector<int> ids(num_gpus);
    for (int i = 0; i < num_gpus; ++i) ids[i] = i;
    return bm_ctx_create_devices(ids.data(), num_gpus, out);
}

int bm_ctx_destroy(bm_ctx_t* ctx) {
    if (!ctx) return BM_EINVAL;
    if (ctx->pending_join) {
        // a join worker that has ended is joined; one still blocked inside
        // RCCL holds only its JoinJob, so it is left to end with the process
        bool ended;
        {
            std::lock_guard<std::mutex> g(ctx->pending_join->m);
            ended = ctx->pending_join->done;
        }
        if (ended)
            ctx->pending_worker.join();
        else
            ctx->pending_worker.detach();
    }
    bm::DeviceGuard guard;
    for (auto& d : ctx->devs) bm::destroy_device(d);
    delete ctx;
    return BM_OK;
}

int bm_ctx_num_devices(const bm_ctx_t* ctx, int* out) {
    if (!ctx || !out) return BM_EINVAL;
    *out = (int)ctx->devs.size();
    return BM_OK;
}

int bm_search_gpu(bm_ctx_t* ctx, const uint8_t* msg, size_t len, uint64_t lower, uint64_t upper, bm_result_t* out) {
    if (!ctx || !out || (len && !msg) || len > BM_MAX_MSG_LEN) return BM_EINVAL;
    bm::DeviceGuard guard;
    bm_result_t r;
    int rc = bm::guarded([&] { return bm::search_impl(ctx, msg, len, lower, upper, &r); });
    if (rc == BM_OK) *out = r;
    return rc;
}

int bm_reduce_gpu(bm_ctx_t* ctx, const bm_result_t* parts, size_t n, bm_result_t* out) {
    if (!ctx || !out || (n && !parts) || n > BM_MAX_REDUCE) return BM_EINVAL;
    bm::DeviceGuard guard;
    bm_result_t r;
    int rc = bm::reduce_impl(ctx, parts, n, &r);
    if (rc == BM_OK) *out = r;
    return rc;
}

int bm_ctx_set_test_fault(bm_ctx_t* ctx, int launches) {
    if (!ctx || launches < -1) return BM_EINVAL;
    ctx->fault_after = launches;
    return BM_OK;
}

int bm_ctx_set_test_start_delay(bm_ctx_t* ctx, int device, int delay_us) {
    if (!ctx || device < 0 || device >= (int)ctx->devs.size() || delay_us < 0) return BM_EINVAL;
    ctx->devs[(size_t)device].test_delay_us = delay_us;
    return BM_OK;
}

int bm_ctx_set_test_rccl_fault(bm_ctx_t* ctx, int where) {
    if (!ctx || where < 0 || where > 3) return BM_EINVAL;
    ctx->test_rccl_fault = where;
    return BM_OK;
}

int bm_hash_gpu(bm_ctx_t* ctx, const uint8_t* msg, size_t len, const uint64_t* nonces, size_t n, uint64_t* out) {
    if (!ctx || (n && (!nonces || !out)) || (len && !msg) || len > BM_MAX_MSG_LEN) return BM_EINVAL;
    bm::DeviceGuard guard;
    return bm::hash_impl(ctx, msg, len, nonces, n, out);
}

int bm_ctx_set_timing(bm_ctx_t* ctx, int enable) {
    if (!ctx) return BM_EINVAL;
    ctx->timing = enable != 0;
    return BM_OK;
}

int bm_ctx_last_stats(const bm_ctx_t* ctx, bm_stats_t* out) {
    if (!ctx || !out) return BM_EINVAL;
    *out = ctx->stats;
    return BM_OK;
}

int bm_ctx_set_blocks_per_cu(bm_ctx_t* ctx, int blocks_per_cu) {
    if (!ctx || blocks_per_cu < 0 || blocks_per_cu > 32) return BM_EINVAL;
    ctx->blocks_per_cu = blocks_per_cu;
    return BM_OK;
}

int bm_ctx_set_combine(bm_ctx_t* ctx, int mode) {
    if (!ctx || mode < BM_COMBINE_AUTO || mode > BM_COMBINE_HOST) return BM_EINVAL;
    if (ctx->rank_ctx && mode != BM_COMBINE_AUTO) return BM_EINVAL;  // a rank combines through its group
    ctx->combine = mode;
    return BM_OK;
}

int bm_ctx_set_task_digits(bm_ctx_t* ctx, int digits) {
    if (!ctx || digits < 0 || digits > bm::kMaxInnerDigits) return BM_EINVAL;
    ctx->task_digits = digits;
    return BM_OK;
}

int bm_ctx_set_max_windows(bm_ctx_t* ctx, int max_windows) {
    if (!ctx || max_windows < 0) return BM_EINVAL;
    ctx->max_windows = max_windows;
    return BM_OK;
}

int bm_ctx_set_split(bm_ctx_t* ctx, const uint32_t* shares, int n) {
    if (!ctx || n < 0 || (n > 0 && !shares)) return BM_EINVAL;
    if (n == 0) {
        ctx->shares.clear();
        return BM_OK;
    }
    const int slots = ctx->rank_ctx ? ctx->world : (int)ctx->devs.size();
    if (n != slots) return BM_EINVAL;
    for (int i = 0; i < n; ++i)
        if (shares[i] == 0) return BM_EINVAL;
    ctx->shares.assign(shares, shares + n);
    return BM_OK;
}

int bm_ctx_get_split(const bm_ctx_t* ctx, uint32_t* shares, int cap, int* n) {
    if (!ctx || !n || cap < 0 || (cap > 0 && !shares)) return BM_EINVAL;
    *n = (int)ctx->shares.size();
    for (int i = 0; i < cap && i < *n; ++i) shares[i] = ctx->shares[(size_t)i];
    return BM_OK;
}

int bm_ctx_set_balance(bm_ctx_t* ctx, int enable) {
    // a rank sees only its own device: a group's shares need an exchange,
    // which is the caller's (the same bm_ctx_set_split on every rank)
    if (!ctx || (ctx->rank_ctx && ctx->world > 1 && enable)) return BM_EINVAL;
    ctx->balance = enable != 0;
    return BM_OK;
}

int bm_split_range(uint64_t lower, uint64_t upper, const uint32_t* shares, int n, uint64_t* lo, uint64_t* hi) {
    if (n < 1 || n > BM_MAX_SLOTS || !lo || !hi) return BM_EINVAL;
    std::vector<uint32_t> sh;
    if (shares) {
        for (int i = 0; i < n; ++i)
            if (shares[i] == 0) return BM_EINVAL;
        sh.assign(shares, shares + n);
    }
    const std::vector<bm::Piece> p = bm::slot_pieces(lower, upper, n, sh);
    for (int i = 0; i < n; ++i) {
        lo[i] = p[(size_t)i].lo;
        hi[i] = p[(size_t)i].hi;
    }
    return BM_OK;
}

int bm_plan_segments(const uint8_t* msg, size_t len, uint64_t lower, uint64_t upper, bm_segment_t* segs, int cap,
                     int* nseg) {
    return bm_plan_segments_ex(msg, len, lower, upper, bm::kDefaultMaxWindows, segs, cap, nseg);
}

int bm_plan_segments_ex(const uint8_t* msg, size_t len, uint64_t lower, uint64_t upper, int max_windows,
                        bm_segment_t* segs, int cap, int* nseg) {
    if (!nseg || cap < 0 || (cap > 0 && !segs)) return BM_EINVAL;
    std::vector<bm_segment_t> v;
    int rc = bm::plan_segments(msg, len, lower, upper, v, max_windows);
    if (rc != BM_OK) return rc;
    *nseg = (int)v.size();
    for (int i = 0; i < cap && i < (int)v.size(); ++i) segs[i] = v[i];
    return BM_OK;
}

}  // extern "C"
