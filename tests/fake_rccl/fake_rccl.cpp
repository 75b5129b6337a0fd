// fake_rccl.cpp -- TEST INFRASTRUCTURE ONLY: a stand-in for the RCCL calls
// libbtcminer.so makes (csrc/bm_api.hip), so that two or more rank processes
// on ONE GPU can form a group.  Real RCCL refuses two ranks on one GPU, and
// every box of this pool has one GPU, so without this the library's world > 1
// group paths (the status-carrying allgather, BM_EPEER between live ranks,
// the peer timeout and its abort) never run anywhere but on an 8-GPU node.
//
// It is linked into a test variant of the library only
// (tests/fake_rccl/libbtcminer_fakerccl.so, `make -C csrc fakerccl`), which
// the tests load in their own subprocesses through BTCMINER_LIB.  The product
// library links the real librccl.
//
// The collective runs on the host, ordered on the caller's stream like a
// real one:
//   ncclAllGather = D2H copy of this rank's bytes -> a host function that
//   posts them into a shared-memory slot and waits for every rank's post of
//   the same call -> H2D copy of all ranks' bytes.
// So a rank that never posts keeps its peers' streams busy, exactly what the
// library's peer timeout polls for; ncclCommAbort releases the wait.
// ncclCommInitRankConfig waits (without limit, like RCCL's bootstrap) until
// every rank has mapped the shared segment named by the unique id.
// ncclCommInitAll (the one-process multi-device path) is not emulated: it
// returns ncclInvalidUsage, and such a context combines by host copies.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <fcntl.h>
#include <sys/mman.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <random>
#include <string>
#include <thread>

namespace {
constexpr int kMaxRanks = 64;
constexpr size_t kMaxBytes = 256;  // per rank per allgather (the library sends 32)
constexpr char kMagic[] = "FAKERCCL";

struct Slot {
    std::atomic<uint64_t> seq[2];   // the call whose bytes buffer b holds (seq parity b)
    uint8_t data[2][kMaxBytes];
};
struct Shared {
    std::atomic<int> joined;
    Slot slot[kMaxRanks];
};
static_assert(std::atomic<uint64_t>::is_always_lock_free, "cross-process atomics");

std::string shm_path(const ncclUniqueId& id) {
    return std::string("/dev/shm/fakerccl-") + std::string(id.internal + sizeof kMagic, 16);
}

size_t type_bytes(ncclDataType_t t) {
    switch (t) {
        case ncclInt8: case ncclUint8: return 1;
        case ncclFloat16: case ncclBfloat16: return 2;
        case ncclInt32: case ncclUint32: case ncclFloat32: return 4;
        case ncclInt64: case ncclUint64: case ncclFloat64: return 8;
        default: return 0;
    }
}
}  // namespace

struct ncclComm {
    int rank = 0, nranks = 1, dev = 0;
    Shared* sh = nullptr;
    std::atomic<bool> aborted{false};
    uint64_t seq = 0;       // allgathers enqueued so far
    // pinned staging buffers: reused call after call, which is safe because
    // one communicator's calls run in the order of its one stream
    uint8_t* h_send = nullptr;
    uint8_t* h_recv = nullptr;
};

namespace {
// What one allgather's host function needs, fixed when the call is enqueued
// (held on the communicator, a second call enqueued before the
// first's host function ran would have made both use the second's seq).
struct Call {
    ncclComm* c;
    uint64_t seq;
    size_t bytes;
};

// The host function of one allgather (runs in stream order, after the D2H
// copy of this rank's bytes).  No HIP calls in here.  Frees its Call.
void exchange(void* p) {
    Call* call = static_cast<Call*>(p);
    ncclComm* c = call->c;
    const uint64_t s = call->seq;
    const size_t bytes = call->bytes;
    delete call;
    const int b = (int)(s & 1);
    Slot& mine = c->sh->slot[c->rank];
    std::memcpy(mine.data[b], c->h_send, bytes);
    mine.seq[b].store(s, std::memory_order_release);
    for (int r = 0; r < c->nranks; ++r) {
        Slot& o = c->sh->slot[r];
        while (o.seq[b].load(std::memory_order_acquire) < s) {
            if (c->aborted.load()) {
                std::memset(c->h_recv, 0xFF, bytes * (size_t)c->nranks);
                return;
            }
            std::this_thread::sleep_for(std::chrono::microseconds(20));
        }
        std::memcpy(c->h_recv + (size_t)r * bytes, o.data[b], bytes);
    }
}
}  // namespace

extern "C" {

ncclResult_t ncclGetVersion(int* version) {
    if (!version) return ncclInvalidArgument;
    *version = 1;  // not a real RCCL version: the stats show which library ran
    return ncclSuccess;
}

ncclResult_t ncclGetUniqueId(ncclUniqueId* id) {
    if (!id) return ncclInvalidArgument;
    std::memset(id->internal, 0, sizeof id->internal);
    std::memcpy(id->internal, kMagic, sizeof kMagic);
    std::random_device rd;
    static const char hex[] = "0123456789abcdef";
    for (int i = 0; i < 16; ++i) id->internal[sizeof kMagic + i] = hex[rd() & 15];
    return ncclSuccess;
}

ncclResult_t ncclCommInitRankConfig(ncclComm_t* out, int nranks, ncclUniqueId id, int rank, ncclConfig_t*) {
    if (!out || nranks < 1 || nranks > kMaxRanks || rank < 0 || rank >= nranks ||
        std::memcmp(id.internal, kMagic, sizeof kMagic) != 0)
        return ncclInvalidArgument;
    const std::string path = shm_path(id);
    const int fd = open(path.c_str(), O_RDWR | O_CREAT, 0600);
    if (fd < 0) return ncclSystemError;
    if (ftruncate(fd, sizeof(Shared)) != 0) {
        close(fd);
        return ncclSystemError;
    }
    void* m = mmap(nullptr, sizeof(Shared), PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    close(fd);
    if (m == MAP_FAILED) return ncclSystemError;
    ncclComm* c = new ncclComm();
    c->rank = rank;
    c->nranks = nranks;
    c->sh = static_cast<Shared*>(m);  // a fresh file is zeros: no posts, nobody joined
    if (hipGetDevice(&c->dev) != hipSuccess ||
        hipHostMalloc(&c->h_send, kMaxBytes, hipHostMallocDefault) != hipSuccess ||
        hipHostMalloc(&c->h_recv, kMaxBytes * kMaxRanks, hipHostMallocDefault) != hipSuccess) {
        if (c->h_send) (void)hipHostFree(c->h_send);
        munmap(m, sizeof(Shared));
        delete c;
        return ncclUnhandledCudaError;
    }
    c->sh->joined.fetch_add(1);
    while (c->sh->joined.load() < nranks) std::this_thread::sleep_for(std::chrono::milliseconds(1));
    if (rank == 0) unlink(path.c_str());  // every rank has it mapped by now
    *out = c;
    return ncclSuccess;
}

ncclResult_t ncclCommInitAll(ncclComm_t*, int, const int*) { return ncclInvalidUsage; }

ncclResult_t ncclCommGetAsyncError(ncclComm_t c, ncclResult_t* err) {
    if (!c || !err) return ncclInvalidArgument;
    *err = ncclSuccess;
    return ncclSuccess;
}

// Releases any allgather still waiting for a peer.  The communicator itself
// is left allocated: a host function of it may still be queued on a stream.
ncclResult_t ncclCommAbort(ncclComm_t c) {
    if (!c) return ncclInvalidArgument;
    c->aborted.store(true);
    return ncclSuccess;
}

ncclResult_t ncclCommCount(const ncclComm_t c, int* n) {
    if (!c || !n) return ncclInvalidArgument;
    *n = c->nranks;
    return ncclSuccess;
}

ncclResult_t ncclCommUserRank(const ncclComm_t c, int* r) {
    if (!c || !r) return ncclInvalidArgument;
    *r = c->rank;
    return ncclSuccess;
}

ncclResult_t ncclCommCuDevice(const ncclComm_t c, int* d) {
    if (!c || !d) return ncclInvalidArgument;
    *d = c->dev;
    return ncclSuccess;
}

ncclResult_t ncclGroupStart() { return ncclSuccess; }
ncclResult_t ncclGroupEnd() { return ncclSuccess; }

ncclResult_t ncclAllGather(const void* send, void* recv, size_t count, ncclDataType_t type, ncclComm_t c,
                           hipStream_t stream) {
    if (!c || !send || !recv) return ncclInvalidArgument;
    const size_t bytes = count * type_bytes(type);
    if (bytes == 0 || bytes > kMaxBytes) return ncclInvalidArgument;
    if (c->aborted.load()) return ncclInvalidUsage;
    Call* call = new Call{c, ++c->seq, bytes};
    if (hipMemcpyAsync(c->h_send, send, bytes, hipMemcpyDeviceToHost, stream) != hipSuccess) {
        delete call;
        return ncclUnhandledCudaError;
    }
    if (hipLaunchHostFunc(stream, exchange, call) != hipSuccess) {
        delete call;  // never queued: nobody else frees it
        return ncclUnhandledCudaError;
    }
    if (hipMemcpyAsync(recv, c->h_recv, bytes * (size_t)c->nranks, hipMemcpyHostToDevice, stream) != hipSuccess)
        return ncclUnhandledCudaError;
    return ncclSuccess;
}

}  // extern "C"
