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

class DecodeError : public std::runtime_error {
    using std::runtime_error::runtime_error;
};

namespace detail {

// One rune of s at i, as Go's utf8.DecodeRuneInString: (rune, size), with
// (0xFFFD, 1) for any invalid or overlong sequence, surrogate or > U+10FFFF.
inline std::pair<uint32_t, size_t> decode_rune(std::string_view s, size_t i) {
    const auto b = [&](size_t k) { return (uint8_t)s[i + k]; };
    const size_t n = s.size() - i;
    const uint8_t c0 = b(0);
    if (c0 < 0x80) return {c0, 1};
    const auto cont = [&](size_t k) { return k < n && (b(k) & 0xC0) == 0x80; };
    if (c0 >= 0xC2 && c0 <= 0xDF && cont(1)) return {((c0 & 0x1Fu) << 6) | (b(1) & 0x3Fu), 2};
    if (c0 >= 0xE0 && c0 <= 0xEF && cont(1) && cont(2)) {
        const uint32_t r = ((c0 & 0x0Fu) << 12) | ((b(1) & 0x3Fu) << 6) | (b(2) & 0x3Fu);
        if (r >= 0x800 && !(r >= 0xD800 && r <= 0xDFFF)) return {r, 3};
    }
    if (c0 >= 0xF0 && c0 <= 0xF4 && cont(1) && cont(2) && cont(3)) {
        const uint32_t r =
            ((c0 & 0x07u) << 18) | ((b(1) & 0x3Fu) << 12) | ((b(2) & 0x3Fu) << 6) | (b(3) & 0x3Fu);
        if (r >= 0x10000 && r <= 0x10FFFF) return {r, 4};
    }
    return {0xFFFD, 1};
}

inline void put_utf8(std::string& out, uint32_t r) {
    if (r < 0x80) {
        out += (char)r;
    } else if (r < 0x800) {
        out += (char)(0xC0 | (r >> 6));
        out += (char)(0x80 | (r & 0x3F));
    } else if (r < 0x10000) {
        out += (char)(0xE0 | (r >> 12));
        out += (char)(0x80 | ((r >> 6) & 0x3F));
        out += (char)(0x80 | (r & 0x3F));
    } else {
        out += (char)(0xF0 | (r >> 18));
        out += (char)(0x80 | ((r >> 12) & 0x3F));
        out += (char)(0x80 | ((r >> 6) & 0x3F));
        out += (char)(0x80 | (r & 0x3F));
    }
}

// encoding/json's string encoder with HTML escaping (json.Marshal's default).
inline std::string go_json_string(std::string_view s) {
    static const char* hex = "0123456789abcdef";
    std::string out = "\"";
    for (size_t i = 0; i < s.size();) {
        const auto [r, size] = decode_rune(s, i);
        if (r == 0xFFFD && size == 1) {
            out += "\\ufffd";  // an invalid byte: Go writes this escape (encoding/json)
        } else if (r == '"' || r == '\\') {
            out += '\\';
            out += (char)r;
        } else if (r == '\n') {
            out += "\\n";
        } else if (r == '\r') {
            out += "\\r";
        } else if (r == '\t') {
            out += "\\t";
        } else if (r < 0x20 || r == '<' || r == '>' || r == '&') {
            out += "\\u00";
            out += hex[r >> 4];
            out += hex[r & 15];
        } else if (r == 0x2028 || r == 0x2029) {
            out += r == 0x2028 ? "\\u2028" : "\\u2029";
        } else {
            out.append(s.substr(i, size));
        }
        i += size;
    }
    out += '"';
    return out;
}

// A strict reader of one flat JSON object (the Message's shape).
class Reader {
   public:
    explicit Reader(std::string_view s) : s_(s) {}

    void ws() {
        while (i_ < s_.size() && (s_[i_] == ' ' || s_[i_] == '\t' || s_[i_] == '\n' || s_[i_] == '\r')) ++i_;
    }
    bool eat(char c) {
        ws();
        if (i_ < s_.size() && s_[i_] == c) {
            ++i_;
            return true;
        }
        return false;
    }
    void expect(char c) {
        if (!eat(c)) fail(std::string("expected '") + c + "'");
    }
    bool at_end() {
        ws();
        return i_ == s_.size();
    }
    [[noreturn]] void fail(const std::string& why) const {
        throw DecodeError("bitcoin message: " + why + " at byte " + std::to_string(i_));
    }
    char peek() {
        ws();
        if (i_ >= s_.size()) fail("unexpected end");
        return s_[i_];
    }
    bool literal(std::string_view w) {
        ws();
        if (s_.substr(i_, w.size()) == w) {
            i_ += w.size();
            return true;
        }
        return false;
    }

    std::string string() {
        expect('"');
        std::string out;
        while (true) {
            if (i_ >= s_.size()) fail("unterminated string");
            const uint8_t c = (uint8_t)s_[i_];
            if (c == '"') {
                ++i_;
                return out;
            }
            if (c < 0x20) fail("control character in string");
            if (c == '\\') {
                if (++i_ >= s_.size()) fail("bad escape");
                const char e = s_[i_++];
                switch (e) {
                    case '"': out += '"'; break;
                    case '\\': out += '\\'; break;
                    case '/': out += '/'; break;
                    case 'b': out += '\b'; break;
                    case 'f': out += '\f'; break;
                    case 'n': out += '\n'; break;
                    case 'r': out += '\r'; break;
                    case 't': out += '\t'; break;
                    case 'u': {
                        uint32_t r = hex4();
                        if (r >= 0xD800 && r <= 0xDBFF && s_.substr(i_, 2) == "\\u") {
                            const size_t save = i_;
                            i_ += 2;
                            const uint32_t lo = hex4();
                            if (lo >= 0xDC00 && lo <= 0xDFFF)
                                r = 0x10000 + ((r - 0xD800) << 10) + (lo - 0xDC00);
                            else
                                i_ = save;
                        }
                        if (r >= 0xD800 && r <= 0xDFFF) r = 0xFFFD;  // a lone surrogate
                        put_utf8(out, r);
                        break;
                    }
                    default: fail("bad escape");
                }
                continue;
            }
            // raw bytes must be valid UTF-8 (as the Python mirror requires)
            const auto [r, size] = decode_rune(s_, i_);
            if (r == 0xFFFD && size == 1) fail("invalid UTF-8");
            out.append(s_.substr(i_, size));
            i_ += size;
        }
    }

    // An integer literal (no fraction, no exponent) in [lo, hi]; returns
    // false for null.  Booleans, strings, floats and objects are errors.
    bool integer(__int128 lo, __int128 hi, __int128* v) {
        if (literal("null")) return false;
        ws();
        const size_t start = i_;
        bool neg = false;
        if (i_ < s_.size() && s_[i_] == '-') {
            neg = true;
            ++i_;
        }
        if (i_ >= s_.size() || s_[i_] < '0' || s_[i_] > '9') fail("expected an integer");
        if (s_[i_] == '0' && i_ + 1 < s_.size() && s_[i_ + 1] >= '0' && s_[i_ + 1] <= '9') fail("leading zero");
        __int128 x = 0;
        while (i_ < s_.size() && s_[i_] >= '0' && s_[i_] <= '9') {
            x = x * 10 + (s_[i_++] - '0');
            if (x > ((__int128)1 << 65)) fail("integer out of range");
        }
        if (i_ < s_.size() && (s_[i_] == '.' || s_[i_] == 'e' || s_[i_] == 'E')) {
            i_ = start;
            fail("not an integer");
        }
        if (neg) x = -x;
        if (x < lo || x > hi) fail("integer out of range");
        *v = x;
        return true;
    }

    void skip_value() {  // an unknown field's value (Go ignores unknown fields)
        const char c = peek();
        if (c == '"') {
            string();
        } else if (c == '{' || c == '[') {
            const char open = c, close = c == '{' ? '}' : ']';
            expect(open);
            if (eat(close)) return;
            do {
                if (open == '{') {
                    string();
                    expect(':');
                }
                skip_value();
            } while (eat(','));
            expect(close);
        } else if (literal("true") || literal("false") || literal("null")) {
        } else {
            ws();
            const size_t start = i_;
            while (i_ < s_.size() && std::strchr("+-0123456789.eE", s_[i_])) ++i_;
            if (i_ == start) fail("bad value");
        }
    }

   private:
    uint32_t hex4() {
        if (i_ + 4 > s_.size()) fail("bad \\u escape");
        uint32_t r = 0;
        for (int k = 0; k < 4; ++k) {
            const char h = s_[i_++];
            r <<= 4;
            if (h >= '0' && h <= '9') r |= (uint32_t)(h - '0');
            else if (h >= 'a' && h <= 'f') r |= (uint32_t)(h - 'a' + 10);
            else if (h >= 'A' && h <= 'F') r |= (uint32_t)(h - 'A' + 10);
            else fail("bad \\u escape");
        }
        return r;
    }
    std::string_view s_;
    size_t i_ = 0;
};

}  // namespace detail

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
        detail::Reader rd(raw);
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
