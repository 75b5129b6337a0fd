// lsp.hpp -- C++17 client side of the Live Sequence Protocol, the transport the
// reference's miner and request client speak (project2/README.md:67-239).
//
// It is the C++ twin of distributed_bitcoin_minter_amd/lsp.py's client and
// talks to that server (or to any conforming one) over UDP:
//
//   lsp::Params           params.go:8-35 (EpochLimit 5, EpochMillis 2000, WindowSize 1)
//   lsp::Message          message.go:10-66, marshalled as Go's encoding/json does
//                         ({"Type":..,"ConnID":..,"SeqNum":..,"Payload":base64|null})
//   lsp::Client           client_api.go:6-30: NewClient / ConnID / Read / Write / Close
//   lspnet::Set...DropPercent   staff.go:31-43, the client-side drop injection
//
// Protocol rules (README:67-138), as in lsp.py:
//   * connect: (Connect,0,0) every epoch until (Ack,id,0); K epochs -> error;
//   * data seqnums start at 1; at most WindowSize unacked; receive window of
//     WindowSize, in-order delivery, every data message at or below the window
//     acknowledged (duplicates too);
//   * each epoch: Ack 0 while no data has arrived, resend unacked data, re-ack
//     the last WindowSize distinct data seqnums; K silent epochs -> lost;
//   * Close blocks until everything written is acknowledged or the
//     connection is lost.
// One background thread per client reads the socket and runs the epoch timer;
// all state sits behind one mutex.
#pragma once

#include <netdb.h>
#include <poll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <optional>
#include <random>
#include <set>
#include <stdexcept>
#include <string>
#include <string_view>
#include <thread>

#include "bm_json.hpp"

namespace lspnet {

// staff.go:15-63: package-global drop percentages (0..100) of this process's
// client reads and writes.
namespace detail {
inline std::atomic<int>& read_drop() {
    static std::atomic<int> v{0};
    return v;
}
inline std::atomic<int>& write_drop() {
    static std::atomic<int> v{0};
    return v;
}
inline bool drop(int pct) {
    if (pct <= 0) return false;
    static std::mutex mu;
    static std::mt19937 rng{std::random_device{}()};
    std::lock_guard<std::mutex> g(mu);
    return (int)(rng() % 100) < pct;
}
}  // namespace detail

inline void SetClientReadDropPercent(int p) {
    if (p >= 0 && p <= 100) detail::read_drop() = p;
}
inline void SetClientWriteDropPercent(int p) {
    if (p >= 0 && p <= 100) detail::write_drop() = p;
}
inline void ResetDropPercent() {
    SetClientReadDropPercent(0);
    SetClientWriteDropPercent(0);
}

constexpr size_t kMaxPacket = 2000;  // conn.go:35

}  // namespace lspnet

namespace lsp {

enum class MsgType : int64_t { Connect = 0, Data = 1, Ack = 2 };  // message.go:8-13

// params.go:8-35
struct Params {
    int EpochLimit = 5;
    int EpochMillis = 2000;
    int WindowSize = 1;
    std::string String() const {
        return "[EpochLimit: " + std::to_string(EpochLimit) + ", EpochMillis: " + std::to_string(EpochMillis) +
               ", WindowSize: " + std::to_string(WindowSize) + "]";
    }
};

class LSPError : public std::runtime_error {
    using std::runtime_error::runtime_error;
};

namespace detail {

inline std::string b64encode(std::string_view in) {
    static const char* tab = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/";
    std::string out;
    out.reserve((in.size() + 2) / 3 * 4);
    size_t i = 0;
    for (; i + 3 <= in.size(); i += 3) {
        const uint32_t v = ((uint8_t)in[i] << 16) | ((uint8_t)in[i + 1] << 8) | (uint8_t)in[i + 2];
        out += tab[v >> 18];
        out += tab[(v >> 12) & 63];
        out += tab[(v >> 6) & 63];
        out += tab[v & 63];
    }
    if (in.size() - i == 1) {
        const uint32_t v = (uint8_t)in[i] << 16;
        out += tab[v >> 18];
        out += tab[(v >> 12) & 63];
        out += "==";
    } else if (in.size() - i == 2) {
        const uint32_t v = ((uint8_t)in[i] << 16) | ((uint8_t)in[i + 1] << 8);
        out += tab[v >> 18];
        out += tab[(v >> 12) & 63];
        out += tab[(v >> 6) & 63];
        out += '=';
    }
    return out;
}

// Standard alphabet, padded; anything else is a DecodeError (as
// base64.b64decode(validate=True) in the Python mirror).
inline std::string b64decode(std::string_view in) {
    const auto val = [](char c) -> int {
        if (c >= 'A' && c <= 'Z') return c - 'A';
        if (c >= 'a' && c <= 'z') return c - 'a' + 26;
        if (c >= '0' && c <= '9') return c - '0' + 52;
        if (c == '+') return 62;
        if (c == '/') return 63;
        return -1;
    };
    if (in.size() % 4) throw bmjson::DecodeError("lsp message: Payload is not base64");
    std::string out;
    for (size_t i = 0; i < in.size(); i += 4) {
        const bool last = i + 4 == in.size();
        const int pad = last ? (in[i + 3] == '=') + (in[i + 2] == '=' && in[i + 3] == '=') : 0;
        uint32_t v = 0;
        for (int k = 0; k < 4 - pad; ++k) {
            const int x = val(in[i + k]);
            if (x < 0) throw bmjson::DecodeError("lsp message: Payload is not base64");
            v |= (uint32_t)x << (18 - 6 * k);
        }
        out += (char)(v >> 16);
        if (pad < 2) out += (char)(v >> 8);
        if (pad < 1) out += (char)v;
    }
    return out;
}

}  // namespace detail

// message.go:16-22
struct Message {
    MsgType Type = MsgType::Connect;
    int64_t ConnID = 0;
    int64_t SeqNum = 0;
    std::optional<std::string> Payload;  // nullopt = Go's nil []byte

    std::string Marshal() const {
        return "{\"Type\":" + std::to_string((int64_t)Type) + ",\"ConnID\":" + std::to_string(ConnID) +
               ",\"SeqNum\":" + std::to_string(SeqNum) +
               ",\"Payload\":" + (Payload ? "\"" + detail::b64encode(*Payload) + "\"" : std::string("null")) + "}";
    }

    // json.Unmarshal into a Message; throws bmjson::DecodeError on anything but
    // one object with integer (or null) Type/ConnID/SeqNum and a base64 (or
    // null) Payload, so a stray datagram never stops a reader.
    static Message Unmarshal(std::string_view raw) {
        bmjson::Reader rd(raw, "lsp message");
        Message m;
        rd.expect('{');
        if (!rd.eat('}')) {
            do {
                const std::string key = rd.string();
                rd.expect(':');
                __int128 v = 0;
                if (key == "Type" || key == "ConnID" || key == "SeqNum") {
                    const int64_t x = rd.integer(INT64_MIN, INT64_MAX, &v) ? (int64_t)v : 0;
                    if (key == "Type") m.Type = (MsgType)x;
                    else if (key == "ConnID") m.ConnID = x;
                    else m.SeqNum = x;
                } else if (key == "Payload") {
                    if (rd.literal("null")) m.Payload.reset();
                    else if (rd.peek() == '"') m.Payload = detail::b64decode(rd.string());
                    else rd.fail("Payload is not a base64 string");
                } else {
                    rd.skip_value();
                }
            } while (rd.eat(','));
            rd.expect('}');
        }
        if (!rd.at_end()) rd.fail("trailing bytes");
        return m;
    }

    // message.go:53-66
    std::string String() const {
        std::string name, payload;
        switch (Type) {
            case MsgType::Connect: name = "Connect"; break;
            case MsgType::Data: name = "Data"; payload = " " + Payload.value_or(""); break;
            case MsgType::Ack: name = "Ack"; break;
        }
        return "[" + name + " " + std::to_string(ConnID) + " " + std::to_string(SeqNum) + payload + "]";
    }
};

inline Message NewConnect() { return Message{}; }
inline Message NewData(int64_t connID, int64_t seqNum, std::string payload) {
    return Message{MsgType::Data, connID, seqNum, std::move(payload)};
}
inline Message NewAck(int64_t connID, int64_t seqNum) { return Message{MsgType::Ack, connID, seqNum, std::nullopt}; }

namespace detail {

// A UDP socket connected to host:port (lspnet.Dial); drops per lspnet.
class Conn {
   public:
    explicit Conn(const std::string& hostport) {
        const size_t colon = hostport.rfind(':');
        if (colon == std::string::npos) throw LSPError("bad address " + hostport);
        const std::string host = hostport.substr(0, colon), port = hostport.substr(colon + 1);
        addrinfo hints{}, *res = nullptr;
        hints.ai_family = AF_UNSPEC;
        hints.ai_socktype = SOCK_DGRAM;
        if (getaddrinfo(host.c_str(), port.c_str(), &hints, &res) != 0 || !res)
            throw LSPError("cannot resolve " + hostport);
        for (addrinfo* a = res; a; a = a->ai_next) {
            fd_ = ::socket(a->ai_family, a->ai_socktype, a->ai_protocol);
            if (fd_ < 0) continue;
            if (::connect(fd_, a->ai_addr, a->ai_addrlen) == 0) break;
            ::close(fd_);
            fd_ = -1;
        }
        freeaddrinfo(res);
        if (fd_ < 0) throw LSPError("cannot reach " + hostport);
    }
    ~Conn() {
        if (fd_ >= 0) ::close(fd_);
    }
    Conn(const Conn&) = delete;
    Conn& operator=(const Conn&) = delete;

    void write(const std::string& b) {
        if (lspnet::detail::drop(lspnet::detail::write_drop())) return;
        (void)::send(fd_, b.data(), b.size(), 0);  // UDP: a failed send is a lost packet
    }
    // One datagram, or nullopt after timeout_ms (or a dropped read).
    std::optional<std::string> read(int timeout_ms) {
        pollfd p{fd_, POLLIN, 0};
        if (::poll(&p, 1, timeout_ms) <= 0) return std::nullopt;
        char buf[lspnet::kMaxPacket];
        const ssize_t n = ::recv(fd_, buf, sizeof buf, 0);
        if (n < 0) return std::nullopt;
        if (lspnet::detail::drop(lspnet::detail::read_drop())) return std::nullopt;
        return std::string(buf, (size_t)n);
    }

   private:
    int fd_ = -1;
};

}  // namespace detail

// client_api.go:6-30.  Create with NewClient.
class Client {
   public:
    Client(std::unique_ptr<detail::Conn> conn, int64_t id, const Params& p)
        : conn_(std::move(conn)), p_(p), id_(id), w_(std::max(1, p.WindowSize)), k_(std::max(1, p.EpochLimit)) {
        thread_ = std::thread([this] { loop(); });
    }
    Client(const Client&) = delete;
    Client& operator=(const Client&) = delete;
    ~Client() {
        {
            std::lock_guard<std::mutex> g(mu_);
            stop_ = true;
        }
        cv_.notify_all();
        if (thread_.joinable()) thread_.join();
    }

    int64_t ConnID() const { return id_; }

    // Blocks for the next payload; LSPError once closed or lost with nothing left.
    std::string Read() {
        std::unique_lock<std::mutex> g(mu_);
        cv_.wait(g, [&] { return !reads_.empty() || lost_ || closing_; });
        if (!reads_.empty()) {
            std::string r = std::move(reads_.front());
            reads_.pop_front();
            return r;
        }
        throw LSPError(lost_ ? "connection lost" : "connection closed");
    }

    // Non-blocking; LSPError only if the connection has been lost.
    void Write(std::string payload) {
        std::lock_guard<std::mutex> g(mu_);
        if (lost_) throw LSPError("connection lost");
        pending_.push_back(std::move(payload));
        pump();
    }

    // Blocks until every written message is acknowledged (or the connection
    // is lost), then stops the background thread.
    void Close() {
        bool lost_pending;
        {
            std::unique_lock<std::mutex> g(mu_);
            closing_ = true;
            cv_.notify_all();
            cv_.wait(g, [&] { return drained() || lost_; });
            lost_pending = lost_ && !drained();
            stop_ = true;
        }
        cv_.notify_all();
        if (thread_.joinable()) thread_.join();
        if (lost_pending) throw LSPError("connection lost before pending messages were acknowledged");
    }

   private:
    using clock = std::chrono::steady_clock;

    void send(const Message& m) { conn_->write(m.Marshal()); }
    bool drained() const { return pending_.empty() && unacked_.empty(); }
    bool window_open() const {
        const int64_t base = unacked_.empty() ? next_seq_ : unacked_.begin()->first;
        return next_seq_ < base + w_;
    }
    void pump() {  // caller holds mu_
        while (!pending_.empty() && window_open()) {
            Message m = NewData(id_, next_seq_, std::move(pending_.front()));
            pending_.pop_front();
            unacked_.emplace(next_seq_++, m);
            send(m);
        }
    }
    void on_message(const Message& m) {  // caller holds mu_
        idle_ = 0;
        if (m.Type == MsgType::Ack) {
            if (unacked_.erase(m.SeqNum)) pump();
            return;
        }
        if (m.Type != MsgType::Data || m.SeqNum < 1) return;
        const int64_t s = m.SeqNum;
        if (s >= expect_ + w_) return;  // beyond the receive window: discard
        send(NewAck(id_, s));
        if (std::find(recent_.begin(), recent_.end(), s) == recent_.end()) {
            recent_.push_back(s);
            if ((int)recent_.size() > w_) recent_.pop_front();
        }
        got_data_ = true;
        if (s >= expect_) ooo_.emplace(s, m.Payload.value_or(""));
        bool any = false;
        for (auto it = ooo_.find(expect_); it != ooo_.end(); it = ooo_.find(expect_)) {
            reads_.push_back(std::move(it->second));
            ooo_.erase(it);
            ++expect_;
            any = true;
        }
        if (any) cv_.notify_all();
    }
    void on_epoch() {  // caller holds mu_
        if (lost_) return;
        if (++idle_ >= k_) {
            lost_ = true;
            cv_.notify_all();
            return;
        }
        if (!got_data_) send(NewAck(id_, 0));
        for (const auto& kv : unacked_) send(kv.second);
        for (int64_t s : recent_) send(NewAck(id_, s));
    }
    void loop() {
        const auto period = std::chrono::milliseconds(p_.EpochMillis);
        auto next = clock::now() + period;
        for (;;) {
            {
                std::lock_guard<std::mutex> g(mu_);
                if (stop_) return;
                if (clock::now() >= next) {
                    next += period;
                    on_epoch();
                }
            }
            const auto left = std::chrono::duration_cast<std::chrono::milliseconds>(next - clock::now()).count();
            const auto got = conn_->read((int)std::clamp<long long>(left, 0, 50));
            if (!got) continue;
            Message m;
            try {
                m = Message::Unmarshal(*got);
            } catch (const bmjson::DecodeError&) {
                continue;
            }
            std::lock_guard<std::mutex> g(mu_);
            if (m.ConnID != id_ || lost_) continue;
            on_message(m);
        }
    }

    std::unique_ptr<detail::Conn> conn_;
    const Params p_;
    const int64_t id_;
    const int w_, k_;
    std::mutex mu_;
    std::condition_variable cv_;
    std::thread thread_;
    int64_t next_seq_ = 1, expect_ = 1;
    std::deque<std::string> pending_, reads_;
    std::map<int64_t, Message> unacked_;
    std::map<int64_t, std::string> ooo_;
    std::deque<int64_t> recent_;
    bool got_data_ = false, lost_ = false, closing_ = false, stop_ = false;
    int idle_ = 0;
};

// client_impl.go:52 / README:111-138: blocks until the server acknowledges
// the connection; LSPError after EpochLimit epochs without an Ack.
inline std::unique_ptr<Client> NewClient(const std::string& hostport, const Params& p = Params{}) {
    auto conn = std::make_unique<detail::Conn>(hostport);
    const std::string connect = NewConnect().Marshal();
    for (int e = 0; e < std::max(1, p.EpochLimit); ++e) {
        conn->write(connect);
        const auto deadline = std::chrono::steady_clock::now() + std::chrono::milliseconds(p.EpochMillis);
        for (;;) {
            const auto left = std::chrono::duration_cast<std::chrono::milliseconds>(
                                  deadline - std::chrono::steady_clock::now())
                                  .count();
            if (left <= 0) break;
            const auto got = conn->read((int)left);
            if (!got) continue;
            try {
                const Message m = Message::Unmarshal(*got);
                if (m.Type == MsgType::Ack && m.SeqNum == 0 && m.ConnID > 0)
                    return std::make_unique<Client>(std::move(conn), m.ConnID, p);
            } catch (const bmjson::DecodeError&) {
            }
        }
    }
    throw LSPError("could not connect to " + hostport);
}

}  // namespace lsp
