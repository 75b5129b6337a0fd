/*
 * btcminer.h -- C ABI of libbtcminer.so, the MI355X (gfx950) nonce-search
 * backend for the distributed bitcoin miner.
 *
 * What it replaces in the reference (/root/reference/project2):
 *   bitcoin.Hash(msg string, nonce uint64) uint64          bitcoin/hash.go:11-15
 *   the miner's min-scan over a job's nonce range          bitcoin/miner/miner.go:43-74
 *                                                           (init :45-46, hot loop :58-65)
 * The Go miner would bind these with cgo; everything
 * else in the reference (LSP transport, JSON Join/Request/Result messages,
 * the server's scheduler) is unchanged by this library.
 *
 * Conventions
 *   - Every function returns an int status: BM_OK (0) or a negative BM_E*
 *     code; bm_strerror() names it.  Nothing aborts.  On failure the output
 *     arguments are left untouched.
 *   - msg is a raw byte string (Go's "%s" of a string: no escaping, may hold
 *     any byte).  The library copies what it needs before returning and keeps
 *     no caller pointer.
 *   - Ranges are INCLUSIVE [lower, upper] (project2/README.md:329,
 *     "0 <= n <= N").  upper = 2^64-1 is legal.  lower > upper is an empty
 *     range and yields {2^64-1, 2^64-1}, which is what miner.go:45-46 returns
 *     when its loop runs zero times.  (miner.go:59 itself loops i < Upper; a
 *     caller that wants that literal behaviour passes upper-1.)
 *   - Results are bit-exact with the reference scan: the minimum hash, and on
 *     ties the smallest nonce (strict '<' over ascending nonces, miner.go:61).
 *   - A context is not re-entrant: use one per OS thread or serialise calls.
 *     Calls are synchronous.  The caller's current HIP device is restored
 *     before each call returns.
 *   - The compute path is the gfx950 HIP kernels only.  There is no CPU
 *     fallback: without a usable GPU, bm_ctx_create() fails with BM_ENODEV.
 */
#ifndef BTCMINER_H
#define BTCMINER_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define BM_ABI_VERSION 7

/* status codes */
#define BM_OK 0
#define BM_EINVAL (-1)   /* bad argument (NULL pointer, msg too long, ...) */
#define BM_ENODEV (-2)   /* no usable gfx950 device / device id out of range */
#define BM_EHIP (-3)     /* a HIP runtime call failed */
#define BM_ERCCL (-4)    /* an RCCL call failed (multi-GPU contexts) */
#define BM_ENOMEM (-5)   /* host or device allocation failed */
#define BM_EINTERNAL (-6)/* planner invariant violated (a bug) */
#define BM_EPEER (-7)    /* rank contexts: another rank of the group failed this call */
#define BM_ETIMEDOUT (-8)/* rank contexts: the group did not answer within the peer timeout */

#define BM_MAX_MSG_LEN (1u << 20) /* bytes; LSP payloads are ~1 KB (README:61) */

/* The 16-byte result of a search: {Hash, Nonce} of bitcoin.NewResult
 * (bitcoin/message.go:36-42).  Ordered lexicographically (hash, nonce). */
typedef struct bm_result {
    uint64_t hash;
    uint64_t nonce;
} bm_result_t;

typedef struct bm_ctx bm_ctx_t;

int bm_abi_version(void);
const char* bm_strerror(int status);

/* Number of visible HIP devices (0 when there is none). */
int bm_device_count(int* out);
/* PCI bus id of a visible device ("0000:05:00.0"; len >= 13), e.g. to find
 * its driver clock in sysfs (bench.py samples it while it times). */
int bm_device_pci_bus_id(int device, char* buf, int len);

/* Context over devices 0..num_gpus-1 (num_gpus = 0: all visible devices).
 * A context with several devices splits every search across them and
 * combines the per-device partials with one RCCL allgather (host copies if
 * RCCL fails at run time; see bm_ctx_set_combine).
 * Launch-overlap tuning is read from the environment at creation (results
 * never depend on it): BTCMINER_STREAMS = launch streams per device (1..4,
 * default 2); BTCMINER_TAIL = nonces split off the biggest launch into a
 * short-task launch of their own (default 16777216, 0 = off); BTCMINER_CHUNK =
 * nonces per lane per work-counter dequeue, at most (10..100000, default 100);
 * BTCMINER_PADC=0 = never use the padding-block kernels with folded constants
 * (search_kernel_padc / search_kernel_padk; default: wherever they apply). */
int bm_ctx_create(int num_gpus, bm_ctx_t** out);
/* Context over an explicit device list (e.g. {LOCAL_RANK} for one process
 * per GPU).  A device listed twice is allowed (a one-GPU rehearsal of the
 * N-device split); such a context combines on the host. */
int bm_ctx_create_devices(const int* devices, int n, bm_ctx_t** out);

/* ---- one process per GPU: a context that is one rank of an RCCL group ----
 * Every rank calls bm_search_gpu() with the SAME (msg, lower, upper): rank r
 * scans the r-th of `world` contiguous pieces of the range (near-equal, or
 * per bm_ctx_set_split).  The reference's equivalent is the server handing
 * each miner a piece of the request (bitcoin/server/server.go:153-169).
 *
 * Two steps, so that no rank waits in RCCL for a peer that failed earlier:
 *   1. bm_ctx_create_rank_local() on the rank's own device: every resource,
 *      no communicator.  Such a context is usable on its own: a search
 *      returns THIS rank's partial (its piece's min), which the caller
 *      combines over any side channel (bench.py's rendezvous gather).
 *   2. once every rank has created its context (exchange the statuses over
 *      the side channel), rank 0 calls bm_rccl_unique_id() and hands the
 *      bytes to every rank, and each calls bm_ctx_join_rank(): a
 *      non-blocking ncclCommInitRankConfig on a worker thread; the call
 *      waits for it at most timeout_ms (0: no limit) and then returns
 *      BM_ETIMEDOUT.  RCCL's bootstrap can block inside that init until
 *      every rank has connected (RCCL 2.27 does), so the worker may stay
 *      there: the context keeps it as its pending join, aborts whatever
 *      communicator it ends up with, and starts no second one -- a later
 *      bm_ctx_join_rank() first waits up to its own timeout_ms for the
 *      pending one to end and returns BM_ETIMEDOUT if it has not.
 *      bm_ctx_destroy() leaves a still-blocked worker detached (it holds no
 *      reference to the context); it ends with the process.  The context
 *      itself stays usable for searches of its own piece throughout.
 *      From then on a search ends with
 *      one RCCL allgather of 32-byte slots {hash, nonce, status, 0}, so
 *      every rank returns the whole range's answer -- or, when any rank
 *      failed the call before the combine (it still takes part, with its
 *      status in the slot -- a HIP error while staging that slot included),
 *      every rank fails it together: the failing rank with its own status,
 *      the others with BM_EPEER.  Only a rank that cannot post its slot at
 *      all aborts its communicator instead; its peers then see that as a
 *      communicator error or wait for their peer timeout.
 * bm_ctx_create_rank() is both steps in one call (blocking join).
 * bm_ctx_set_peer_timeout(): a joined rank waits at most this long for the
 *   group's allgather after its own work ends (default BM_DEFAULT_PEER_TIMEOUT_MS,
 *   10 minutes, so a peer that never posts its slot is a bounded failure;
 *   0: no limit); past it the communicator is aborted and the call returns
 *   BM_ETIMEDOUT, as does every later search until bm_ctx_leave_rank().
 *   Callers whose pieces take longer than that per call raise it.
 * bm_ctx_join_rank(): timeout_ms bounds the WHOLE call, including the wait
 *   for a pending join; 0 waits without limit.
 * bm_ctx_leave_rank(): drop the communicator; searches return the rank's
 *   own partial again.  bm_ctx_rank_joined(): 1 inside a group, else 0.
 * bm_ctx_destroy() (any context) waits for its own streams, then drops every
 *   communicator it holds with ncclCommAbort: teardown never waits on a peer,
 *   even one that has died. */
#define BM_RCCL_ID_BYTES 128
#define BM_DEFAULT_PEER_TIMEOUT_MS 600000
int bm_rccl_unique_id(uint8_t* id /* BM_RCCL_ID_BYTES */);
int bm_ctx_create_rank_local(int device, int rank, int world, bm_ctx_t** out);
int bm_ctx_join_rank(bm_ctx_t* ctx, const uint8_t* id, int timeout_ms);
int bm_ctx_leave_rank(bm_ctx_t* ctx);
int bm_ctx_rank_joined(const bm_ctx_t* ctx, int* joined);
int bm_ctx_set_peer_timeout(bm_ctx_t* ctx, int timeout_ms);
int bm_ctx_create_rank(int device, int rank, int world, const uint8_t* id, bm_ctx_t** out);
int bm_ctx_rank(const bm_ctx_t* ctx, int* rank, int* world);
int bm_ctx_destroy(bm_ctx_t* ctx);
int bm_ctx_num_devices(const bm_ctx_t* ctx, int* out);

/* The hot path: min over n in [lower, upper] of (Hash(msg, n), n).
 * Replaces miner.go:58-65 (+ hash.go:11-15 per nonce). */
int bm_search_gpu(bm_ctx_t* ctx, const uint8_t* msg, size_t len, uint64_t lower, uint64_t upper,
                  bm_result_t* out);

/* Batched bitcoin.Hash (hash.go:11-15) on the first device of ctx:
 * out[i] = Hash(msg, nonces[i]) for i < n. */
int bm_hash_gpu(bm_ctx_t* ctx, const uint8_t* msg, size_t len, const uint64_t* nonces, size_t n,
                uint64_t* out);

/* ---- measurement (used by bench.py; does not change results) ---------- */

#define BM_MAX_LAUNCH_STATS 64

typedef struct bm_launch_stat {
    int32_t device;       /* index into the context's device list */
    int32_t p;            /* byte position of the last digit in its SHA block */
    int32_t nbv;          /* varying blocks per task (1 or 2) */
    int32_t pad_block;    /* 1 when a constant padding block follows (the generic kernel: its
                             K + W from kernargs); 2 + K: the same, run by a kernel with that
                             block's constants folded in, after K whole prefix blocks (2: a
                             one-block message, search_kernel_padc; 3..17: K = 1..15,
                             search_kernel_padk, whose entering state is the midstate) */
    int32_t digits;       /* decimal digits of every nonce in the launch */
    int32_t inner_digits; /* digits iterated by each thread's inner loop */
    uint64_t nonces;      /* nonces the launch is responsible for */
    uint32_t grid;        /* workgroups launched (256 threads each) */
    uint32_t tasks_per_thread; /* approx. tasks per lane (dynamic dequeue) */
    double ms;            /* launch duration from HIP events on its stream (0 if timing off) */
    double clock_ghz;     /* average shader clock over the launch: s_memtime cycles over
                             s_memrealtime ticks stamped by workgroup 0 (timing on, and a
                             library built with BM_CLOCK_PROBE=1; 0 otherwise) */
} bm_launch_stat_t;

/* How the last search combined its partials (bm_stats_t.combine_used). */
#define BM_COMBINED_NONE 0  /* nothing to combine (empty range) */
#define BM_COMBINED_RCCL 1  /* one RCCL allgather (the devices of the context, or the ranks of its group) */
#define BM_COMBINED_HOST 2  /* device-to-host copies of every device's partial */
#define BM_COMBINED_LOCAL 3 /* a rank context outside a group: this rank's own partial */
#define BM_MAX_STAT_DEVICES 16

typedef struct bm_stats {
    uint32_t launches;     /* search-kernel launches of the last call */
    uint32_t recorded;     /* entries filled in launch[] (<= BM_MAX_LAUNCH_STATS) */
    double wall_ms;        /* host wall time of the last bm_search_gpu call */
    double kernel_ms;      /* SUM of launch durations (timing on); launches on
                              different streams overlap, so this can exceed span_ms */
    double span_ms;        /* first launch's start to the last launch's end on
                              one device (timing on; max over devices) */
    uint64_t nonces;       /* nonces this process scanned in the last call */
    int32_t combine_used;  /* BM_COMBINED_*: how the partials were combined */
    int32_t rccl_status;   /* the RCCL failure this context fell back from or
                              stopped on (BM_ERCCL / BM_ETIMEDOUT), 0 if none */
    uint32_t devices;      /* entries of dev_nonces / dev_span_ms / dev_rccl_* */
    uint32_t reserved;
    uint64_t dev_nonces[BM_MAX_STAT_DEVICES];  /* nonces each device of the context scanned */
    double dev_span_ms[BM_MAX_STAT_DEVICES];   /* each device's first operation to the end of
                                                  its reduction (timing on) */
    /* What RCCL itself reports about the communicator the last call's
     * combine ran over (combine_used = BM_COMBINED_RCCL; otherwise 0 / -1),
     * so a multi-GPU measurement can show that the collective really spanned
     * N ranks on N devices: */
    int32_t rccl_nranks;   /* ncclCommCount: ranks in the communicator */
    int32_t rccl_rank;     /* ncclCommUserRank of this process's (first) device */
    int32_t dev_rccl_rank[BM_MAX_STAT_DEVICES];   /* ncclCommUserRank of each device of the context */
    int32_t dev_rccl_device[BM_MAX_STAT_DEVICES]; /* ncclCommCuDevice: the HIP device RCCL runs that
                                                     rank on */
    /* ABI 7: what the combine and the start of a call cost, so a multi-GPU
     * line can be read without a rerun. */
    int32_t rccl_version;      /* ncclGetVersion of the RCCL the library runs on (e.g. 22703); 0 if
                                  it cannot say.  Filled on every call. */
    int32_t start_threads;     /* host threads that submitted the devices' work (1, or one per
                                  device of a multi-device context) */
    double rccl_init_ms;       /* host time the current communicator took to form: ncclCommInitAll
                                  (one process), or bm_ctx_join_rank's init, which includes waiting
                                  for every rank to arrive; 0 without a communicator */
    double rccl_allgather_ms;  /* the last call's allgather, from HIP events around it on the
                                  (first) device's stream (timing on): it starts when this
                                  device's own work is done, so it includes the wait for the
                                  slowest peer; max over the devices of a context; 0 otherwise */
    double combine_ms;         /* host time from the end of this process's own work (its devices'
                                  reductions, seen on the host) to the end of the combine: the wait
                                  for the peers, the allgather or host copies, the result copy.
                                  Without timing or balance in a one-process context, from the
                                  enqueue of the combine instead */
    double dev_allgather_ms[BM_MAX_STAT_DEVICES]; /* each device's allgather event pair (timing on) */
    double dev_start_ms[BM_MAX_STAT_DEVICES];     /* host time at which each device's first
                                  operation of the call was submitted, relative to the earliest
                                  device's (its stream is idle then, so this is when it starts);
                                  set_balance measures rates from that common start (timing or
                                  balance on) */
    bm_launch_stat_t launch[BM_MAX_LAUNCH_STATS];
} bm_stats_t;

/* Enable per-launch HIP event timing (default off). */
int bm_ctx_set_timing(bm_ctx_t* ctx, int enable);
int bm_ctx_last_stats(const bm_ctx_t* ctx, bm_stats_t* out);

/* Occupancy override for the search kernels: workgroups of 256 threads kept
 * resident per CU (0 = ask the runtime).  Exposed for tuning. */
int bm_ctx_set_blocks_per_cu(bm_ctx_t* ctx, int blocks_per_cu);

/* Planner knob: a digit-count segment whose high digits take more than
 * max_windows distinct values is run as ONE launch whose tasks re-compress
 * the block holding them (nbv = 2) instead of one launch per value
 * (default 64; 0 forces nbv = 2 wherever the digits straddle a block).
 * Results do not depend on it. */
int bm_ctx_set_max_windows(bm_ctx_t* ctx, int max_windows);

/* Nonces per kernel task = 10^digits, the digits a lane steps in its inner
 * loop.  0 (default): per launch, 100-nonce tasks, or 10-nonce tasks for a
 * launch too small to give every resident lane two 100-nonce tasks; 1 or 2:
 * forced (tests use it to cover both loop shapes at small sizes).  Results do
 * not depend on it. */
int bm_ctx_set_task_digits(bm_ctx_t* ctx, int digits);

/* How a context combines its per-device 16-byte partials:
 * BM_COMBINE_AUTO (default): RCCL allgather when the context has > 1
 * distinct device, a plain device-to-host copy otherwise; BM_COMBINE_RCCL:
 * always RCCL (also for one device: exercises the collective path on a
 * single GPU; BM_EINVAL on a context that lists a device twice);
 * BM_COMBINE_HOST: device-to-host copies of every partial, no RCCL.
 * When RCCL fails at run time (ncclCommInitAll or the allgather), the
 * context aborts its communicators, combines that call and every later one
 * by host copies, and reports it: combine_used = BM_COMBINED_HOST,
 * rccl_status = BM_ERCCL.  The answer is the same either way. */
#define BM_COMBINE_AUTO 0
#define BM_COMBINE_RCCL 1
#define BM_COMBINE_HOST 2
int bm_ctx_set_combine(bm_ctx_t* ctx, int mode);

/* ---- the multi-GPU range partitioner (results never depend on it) -----
 * A search's range is cut into one contiguous piece per slot: the devices of
 * a context, or the ranks of an RCCL group.  Default: near-equal pieces.
 * GPUs run this kernel at different clocks (PMC put it at 2.09-2.23 GHz on
 * the MI355Xs measured), and a search ends when its slowest slot does;
 * pieces in proportion to each slot's speed end together.
 *
 * bm_ctx_set_split: n integer shares, one per slot (n = devices of the
 *   context, or world of a rank context), each >= 1; slot i gets the nonces
 *   [lower + B_i, lower + B_{i+1} - 1] with B_i = floor(count * (s_0 + ... +
 *   s_{i-1}) / S), S = sum of the shares (exact integer arithmetic, so every
 *   rank of a group derives the same pieces from the same shares).  Every
 *   rank of a group must set the same shares.  n = 0: back to near-equal.
 * bm_ctx_set_balance: a multi-device context sets its own shares after each
 *   search in which every device's piece held >= 2^30 nonces: each device's
 *   nonces over the time from the call's common start (the earliest device's
 *   first operation; bm_stats_t.dev_start_ms) to its reduction, scaled so the
 *   fastest device has 65536 -- a device that starts late gets a smaller
 *   piece.  Each device's work is submitted from a host thread of its own, so
 *   the starts are close anyway.  BM_EINVAL on a rank context of more than
 *   one rank: a rank sees only its own device, so a group exchanges its rates
 *   itself and calls bm_ctx_set_split (bench.py does, over its rendezvous).
 * bm_ctx_get_split: the shares the next search will use (*n = 0: near-equal).
 * bm_split_range: the pieces themselves, pure CPU: lo[i] > hi[i] marks an
 *   empty piece; shares = NULL gives the near-equal pieces. */
#define BM_MAX_SLOTS 1024
int bm_ctx_set_split(bm_ctx_t* ctx, const uint32_t* shares, int n);
int bm_ctx_get_split(const bm_ctx_t* ctx, uint32_t* shares, int cap, int* n);
int bm_ctx_set_balance(bm_ctx_t* ctx, int enable);
int bm_split_range(uint64_t lower, uint64_t upper, const uint32_t* shares, int n, uint64_t* lo, uint64_t* hi);

/* ---- test entries (do not change search results) ---------------------- */

/* Lexicographic (hash, nonce) min of n partials on the first device of ctx,
 * computed by the reductions the search runs above its per-lane scans
 * (ds_swizzle/readlane wave min, LDS workgroup min, second-pass kernel).
 * Pins the tie rule (equal hashes -> smallest nonce, miner.go:61) on inputs
 * the search itself cannot produce.  n <= BM_MAX_REDUCE. */
#define BM_MAX_REDUCE (1u << 24)
int bm_reduce_gpu(bm_ctx_t* ctx, const bm_result_t* parts, size_t n, bm_result_t* out);

/* Make every later bm_search_gpu fail with BM_EINTERNAL after enqueueing
 * `launches` search launches (-1: off).  Exercises the failure path: the
 * call drains what it queued and the context stays usable.  On a joined
 * rank context the failure reaches the whole group through the status word
 * of the allgather (the others return BM_EPEER). */
int bm_ctx_set_test_fault(bm_ctx_t* ctx, int launches);

/* Make RCCL fail on purpose (0: off): 1 = the next communicator set-up
 * (ncclCommInitAll, or bm_ctx_join_rank), 2 = every allgather, before it is
 * enqueued.  A multi-device context then falls back to host copies; a
 * joined rank context fails the call (at world 1 only: a real group's peers
 * would wait for it until their peer timeout).  3 = a joined rank context's
 * allgather succeeds but its last slot carries a failure status, as a failed
 * peer's slot does: the call returns BM_EPEER and the group stays joined. */
int bm_ctx_set_test_rccl_fault(bm_ctx_t* ctx, int where);

/* Hold back the submission of device `device`'s work (an index into the
 * context's device list) by delay_us microseconds at the start of every later
 * search (0: off): a late-starting GPU, on demand, for the balance test. */
int bm_ctx_set_test_start_delay(bm_ctx_t* ctx, int device, int delay_us);

/* ---- host-side plan introspection (pure CPU; used by the CPU tests) ---- */

/* One kernel launch of a search: every nonce n = nonce_base + v with v in
 * [vlo, vhi] has exactly `digits` decimal digits and a message whose bytes
 * before the varying SHA-256 block(s) are constant (folded into mid[]). */
typedef struct bm_segment {
    int32_t p;            /* byte index of the last digit inside the last varying block */
    int32_t nbv;          /* varying blocks (1, or 2 when a task also re-compresses the block before) */
    int32_t pad_block;    /* 1: a constant padding block follows the varying block */
    int32_t digits;       /* decimal digits of every nonce */
    int32_t nd;           /* digits of v that live in the varying block(s) */
    int32_t max_inner;    /* max digits the inner loop may iterate (all in one word) */
    uint64_t vlo, vhi;    /* inclusive range of v */
    uint64_t nonce_base;  /* nonce = nonce_base + v */
    uint32_t mid[8];      /* SHA-256 state before the varying block(s) */
    uint32_t tmpl[32];    /* varying block words, big-endian, digit bytes = '0' */
    uint32_t pad_w[16];   /* words of the constant padding block (pad_block) */
} bm_segment_t;

/* Fill up to cap segments for (msg, [lower, upper]); *nseg gets the count
 * needed (call with cap = 0 to size). */
int bm_plan_segments(const uint8_t* msg, size_t len, uint64_t lower, uint64_t upper,
                     bm_segment_t* segs, int cap, int* nseg);
/* Same with an explicit max_windows (see bm_ctx_set_max_windows). */
int bm_plan_segments_ex(const uint8_t* msg, size_t len, uint64_t lower, uint64_t upper, int max_windows,
                        bm_segment_t* segs, int cap, int* nseg);

#ifdef __cplusplus
}
#endif
#endif /* BTCMINER_H */
