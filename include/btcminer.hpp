// btcminer.hpp -- C++17 host side above the C ABI (btcminer.h).
//
// The reference is Go (compiled code) and its toolchain is absent here, so
// the host side of the path is C++ (the Python package mirrors it for tests
// and the system programs).  Two parts:
//
//   btcminer::Context   RAII owner of a bm_ctx (one process over N GPUs, or
//                       one rank of an RCCL group); errors are exceptions.
//   bitcoin::           the reference's `bitcoin` package for this path:
//                       Hash (hash.go:11-15), MsgType / Message / NewRequest /
//                       NewResult / NewJoin / String (message.go:5-60), with
//                       Message::Marshal producing the bytes Go's
//                       encoding/json produces for the Go struct, and
//                       Message::Unmarshal accepting what the Python mirror
//                       (distributed_bitcoin_minter_amd/bitcoin.py) accepts.
//
// Header-only; link with -lbtcminer.
#pragma once

#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>
#include <string_view>
#include <utility>
#include <vector>

#include "bm_json.hpp"
#include "btcminer.h"

namespace btcminer {

class Error : public std::runtime_error {
   public:
    Error(int status, const std::string& what)
        : std::runtime_error(what + ": " + bm_strerror(status) + " (" + std::to_string(status) + ")"),
          status_(status) {}
    int status() const { return status_; }

   private:
    int status_;
};

inline void check(int status, const char* what) {
    if (status != BM_OK) throw Error(status, what);
}

struct Result {
    uint64_t hash = UINT64_MAX;
    uint64_t nonce = UINT64_MAX;
};

// Owns a bm_ctx.  Not thread-safe, like the C context (one per OS thread).
class Context {
   public:
    // num_gpus = 0: every visible GPU
    explicit Context(int num_gpus = 1) { check(bm_ctx_create(num_gpus, &ctx_), "bm_ctx_create"); }
    explicit Context(const std::vector<int>& devices) {
        check(bm_ctx_create_devices(devices.data(), (int)devices.size(), &ctx_), "bm_ctx_create_devices");
    }
    // rank `rank` of an RCCL group of `world` processes (blocks until all join)
    static Context rank(int device, int rank, int world, const uint8_t (&id)[BM_RCCL_ID_BYTES]) {
        Context c{Empty{}};
        check(bm_ctx_create_rank(device, rank, world, id, &c.ctx_), "bm_ctx_create_rank");
        return c;
    }
    // rank `rank` of `world` outside a group: search() returns this rank's
    // partial; join() then makes it a member of the RCCL group
    static Context rank_local(int device, int rank, int world) {
        Context c{Empty{}};
        check(bm_ctx_create_rank_local(device, rank, world, &c.ctx_), "bm_ctx_create_rank_local");
        return c;
    }
    void join(const uint8_t (&id)[BM_RCCL_ID_BYTES], int timeout_ms = 0) {
        check(bm_ctx_join_rank(ctx_, id, timeout_ms), "bm_ctx_join_rank");
    }
    void leave() { check(bm_ctx_leave_rank(ctx_), "bm_ctx_leave_rank"); }
    // a joined rank's wait for its peers, at most (default BM_DEFAULT_PEER_TIMEOUT_MS; 0: no limit)
    void set_peer_timeout(int timeout_ms) {
        check(bm_ctx_set_peer_timeout(ctx_, timeout_ms), "bm_ctx_set_peer_timeout");
    }
    // per-launch HIP event timing, and what the last search reported (bm_stats_t)
    void set_timing(bool on) { check(bm_ctx_set_timing(ctx_, on ? 1 : 0), "bm_ctx_set_timing"); }
    bm_stats_t last_stats() const {
        bm_stats_t s;
        check(bm_ctx_last_stats(ctx_, &s), "bm_ctx_last_stats");
        return s;
    }
    Context(Context&& o) noexcept : ctx_(std::exchange(o.ctx_, nullptr)) {}
    Context& operator=(Context&& o) noexcept {
        if (this != &o) {
            reset();
            ctx_ = std::exchange(o.ctx_, nullptr);
        }
        return *this;
    }
    Context(const Context&) = delete;
    Context& operator=(const Context&) = delete;
    ~Context() { reset(); }

    // min over n in [lower, upper] of (Hash(msg, n), n): miner.go:58-65
    Result search(std::string_view msg, uint64_t lower, uint64_t upper) {
        bm_result_t r;
        check(bm_search_gpu(ctx_, reinterpret_cast<const uint8_t*>(msg.data()), msg.size(), lower, upper, &r),
              "bm_search_gpu");
        return Result{r.hash, r.nonce};
    }
    // bitcoin.Hash for each nonce (hash.go:11-15), on the first device
    std::vector<uint64_t> hash(std::string_view msg, const std::vector<uint64_t>& nonces) {
        std::vector<uint64_t> out(nonces.size());
        check(bm_hash_gpu(ctx_, reinterpret_cast<const uint8_t*>(msg.data()), msg.size(), nonces.data(),
                          nonces.size(), out.data()),
              "bm_hash_gpu");
        return out;
    }
    int num_devices() const {
        int n = 0;
        check(bm_ctx_num_devices(ctx_, &n), "bm_ctx_num_devices");
        return n;
    }
    // the range partitioner: shares per slot (empty: near-equal), or shares
    // that follow each device's measured rate (multi-device contexts)
    void set_split(const std::vector<uint32_t>& shares) {
        check(bm_ctx_set_split(ctx_, shares.data(), (int)shares.size()), "bm_ctx_set_split");
    }
    void set_balance(bool on) { check(bm_ctx_set_balance(ctx_, on ? 1 : 0), "bm_ctx_set_balance"); }
    bm_ctx_t* get() const { return ctx_; }

   private:
    struct Empty {};
    explicit Context(Empty) {}
    void reset() {
        if (ctx_) bm_ctx_destroy(ctx_);
        ctx_ = nullptr;
    }
    bm_ctx_t* ctx_ = nullptr;
};

}  // namespace btcminer

namespace bitcoin {

// message.go:5-11
enum class MsgType : int64_t { Join = 0, Request = 1, Result = 2 };

using DecodeError = bmjson::DecodeError;
namespace detail = ::bmjson;

// message.go:16-21
struct Message {
    MsgType Type = MsgType::Join;
    std::string Data;
    uint64_t Lower = 0, Upper = 0, Hash = 0, Nonce = 0;

    // json.Marshal of the Go struct: fields in declaration order, integers
    // as JSON numbers, Data with encoding/json's escaping.
    std::string Marshal() const {
        return "{\"Type\":" + std::to_string((int64_t)Type) + ",\"Data\":" + detail::go_json_string(Data) +
               ",\"Lower\":" + std::to_string(Lower) + ",\"Upper\":" + std::to_string(Upper) +
               ",\"Hash\":" + std::to_string(Hash) + ",\"Nonce\":" + std::to_string(Nonce) + "}";
    }

    // json.Unmarshal into a Message: absent or null fields keep zero values;
    // a field of the wrong JSON type, a number out of range, a Type outside
    // Join/Request/Result, or anything but one object throws DecodeError.
    static Message Unmarshal(std::string_view raw) {
        detail::Reader rd(raw, "bitcoin message");
        Message m;
        rd.expect('{');
        if (!rd.eat('}')) {
            do {
                const std::string key = rd.string();
                rd.expect(':');
                __int128 v = 0;
                if (key == "Type") {
                    if (rd.integer(INT64_MIN, INT64_MAX, &v)) {
                        if (v < 0 || v > 2) rd.fail("unknown message type");
                        m.Type = (MsgType)(int64_t)v;
                    } else {
                        m.Type = MsgType::Join;
                    }
                } else if (key == "Data") {
                    if (rd.literal("null")) m.Data.clear();
                    else if (rd.peek() == '"') m.Data = rd.string();
                    else rd.fail("Data is not a string");
                } else if (key == "Lower" || key == "Upper" || key == "Hash" || key == "Nonce") {
                    uint64_t& f = key == "Lower" ? m.Lower : key == "Upper" ? m.Upper : key == "Hash" ? m.Hash : m.Nonce;
                    f = rd.integer(0, (__int128)UINT64_MAX, &v) ? (uint64_t)v : 0;
                } else {
                    rd.skip_value();
                }
            } while (rd.eat(','));
            rd.expect('}');
        }
        if (!rd.at_end()) rd.fail("trailing bytes");
        return m;
    }

    // message.go:49-60
    std::string String() const {
        switch (Type) {
            case MsgType::Request:
                return "[Request " + Data + " " + std::to_string(Lower) + " " + std::to_string(Upper) + "]";
            case MsgType::Result: return "[Result " + std::to_string(Hash) + " " + std::to_string(Nonce) + "]";
            case MsgType::Join: return "[Join]";
        }
        return "";
    }
    bool operator==(const Message& o) const {
        return Type == o.Type && Data == o.Data && Lower == o.Lower && Upper == o.Upper && Hash == o.Hash &&
               Nonce == o.Nonce;
    }
};

// message.go:25-47
inline Message NewRequest(std::string data, uint64_t lower, uint64_t upper) {
    Message m;
    m.Type = MsgType::Request;
    m.Data = std::move(data);
    m.Lower = lower;
    m.Upper = upper;
    return m;
}
inline Message NewResult(uint64_t hash, uint64_t nonce) {
    Message m;
    m.Type = MsgType::Result;
    m.Hash = hash;
    m.Nonce = nonce;
    return m;
}
inline Message NewJoin() { return Message{}; }

// hash.go:11-15 -- "Only miners should ever need to call this method"; on
// the context's first GPU.
inline uint64_t Hash(btcminer::Context& ctx, std::string_view msg, uint64_t nonce) {
    return ctx.hash(msg, {nonce})[0];
}

}  // namespace bitcoin
