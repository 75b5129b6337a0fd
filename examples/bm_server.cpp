// bm_server.cpp -- the bitcoin server (range scheduler) in C++ on lsp.hpp.
//
//   bm_server port [--chunk N] [--depth D] [--target-ms T] [--max-mult M] [--epoch-limit K]
//             [--epoch-millis MS] [--window-size W] [--host ADDR] [--drop-read P] [--drop-write P] [-v]
//
// The C++ twin of distributed_bitcoin_minter_amd/server.py (whose docstring
// states the design) for bitcoin/server/server.go and README:341-417:
//   * a miner connects and sends Join; a client sends Request(Data, Lower, Upper);
//   * the inclusive range is cut into chunks of --chunk nonces (default 2^32,
//     retuned from server.go:18's minerLoad = 24 for GPU miners), handed to
//     miners with free job slots (each holds up to --depth jobs, default 2);
//   * each miner's chunks are a multiple of --chunk sized from its measured
//     rate (server.py chunk_for): about --target-ms of its work (default 300;
//     0 = fixed chunks), at most --max-mult bases (64), at most twice its
//     previous multiple, at most its rate share of the request's remainder;
//   * fair share: the next chunk goes to the active request with the fewest
//     chunks in flight (oldest on ties), to the miner with the fewest queued
//     jobs (longest-free on ties);
//   * merge: the lexicographic (hash, nonce) minimum, equal to the sequential
//     strict-< scan of the whole range in any arrival order;
//   * a lost miner's chunks go back to the front of their request's queue; a
//     lost client's requests are dropped; a client's results go out in the
//     order it sent its requests.
// With port 0 the chosen port is printed first ("port <n>").  No GPU needed.
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <deque>
#include <vector>
#include <map>
#include <memory>
#include <string>
#include <tuple>

#include "btcminer.hpp"
#include "lsp.hpp"

namespace {

using Range = std::pair<uint64_t, uint64_t>;  // inclusive [lo, hi]

struct Request {
    uint64_t rid;
    int64_t client;
    std::string data;
    uint64_t upper, next_lower;
    bool done;                  // every chunk issued
    std::deque<Range> retry;    // chunks of lost miners, issued first
    long inflight = 0;
    std::pair<uint64_t, uint64_t> best{UINT64_MAX, UINT64_MAX};  // miner.go:45-46
    bool answered = false;

    Request(uint64_t id, int64_t c, const bitcoin::Message& m)
        : rid(id), client(c), data(m.Data), upper(m.Upper), next_lower(m.Lower), done(m.Lower > m.Upper) {}
    bool has_work() const { return !retry.empty() || !done; }
    bool finished() const { return !has_work() && inflight == 0; }
    // At most `chunk` nonces; a lost miner's chunk first, cut to the taker's
    // size (server.py _Request.take), its rest left at the front.
    Range take(uint64_t chunk) {
        if (!retry.empty()) {
            Range r = retry.front();
            retry.pop_front();
            if (r.second - r.first >= chunk) {
                retry.push_front({r.first + chunk, r.second});
                r.second = r.first + chunk - 1;
            }
            return r;
        }
        const uint64_t lo = next_lower;
        const uint64_t hi = upper - lo >= chunk ? lo + chunk - 1 : upper;
        if (hi == upper) done = true;
        else next_lower = hi + 1;
        return {lo, hi};
    }
};

using Clock = std::chrono::steady_clock;

struct Job {
    uint64_t rid;
    Range r;
    Clock::time_point sent;
};

// A miner's measured rate: its last jobs' nonces per second (server.py RATE_SAMPLES).
struct MinerRate {
    std::deque<double> samples;
    uint64_t mult = 0;  // multiple of its last fresh chunk
    bool have_done = false;
    Clock::time_point last_done;
    double rate() const {  // median, 0 before the first result
        if (samples.empty()) return 0.0;
        std::vector<double> v(samples.begin(), samples.end());
        std::sort(v.begin(), v.end());
        const size_t m = v.size() / 2;
        return v.size() % 2 ? v[m] : (v[m - 1] + v[m]) / 2;
    }
};
constexpr size_t kRateSamples = 5;

// server.py chunk_for: the multiple k >= 1 of `base` for a miner's next job.
uint64_t chunk_for(uint64_t base, double target_s, uint64_t max_mult, double rate, uint64_t prev_mult,
                   double remaining, double share) {
    if (target_s <= 0 || rate <= 0) return 1;
    const double want = std::floor(rate * target_s / (double)base + 0.5);
    uint64_t k = want >= (double)max_mult ? max_mult : (uint64_t)std::max(1.0, want);
    k = std::max<uint64_t>(1, std::min({k, max_mult, 2 * std::max<uint64_t>(1, prev_mult)}));
    if (share > 0 && share < 1) {
        const double mine = std::floor(remaining * share);
        const uint64_t cap = (uint64_t)std::ceil(mine / (double)base);
        k = std::min(k, std::max<uint64_t>(1, cap));
    }
    return k;
}

class BitcoinServer {
   public:
    BitcoinServer(lsp::Server& srv, uint64_t chunk, size_t depth, double target_s, uint64_t max_mult, bool verbose)
        : srv_(srv), chunk_(chunk), depth_(depth), target_s_(target_s), max_mult_(max_mult), verbose_(verbose) {}

    void serve() {
        for (;;) {
            int64_t cid;
            std::string payload;
            try {
                std::tie(cid, payload) = srv_.Read();
            } catch (const lsp::ServerError& e) {
                if (e.conn_id() == 0) return;  // server closed
                on_lost(e.conn_id());
                continue;
            }
            try {
                on_message(cid, bitcoin::Message::Unmarshal(payload));
            } catch (const bitcoin::DecodeError& e) {
                if (verbose_) std::fprintf(stderr, "conn %lld: bad message: %s\n", (long long)cid, e.what());
            }
        }
    }

   private:
    void on_message(int64_t cid, const bitcoin::Message& m) {
        switch (m.Type) {
            case bitcoin::MsgType::Join:
                if (!miners_.count(cid)) {
                    miners_[cid];
                    rates_[cid];
                    free_since_[cid] = tick_++;
                    if (verbose_) std::fprintf(stderr, "miner %lld joined\n", (long long)cid);
                }
                break;
            case bitcoin::MsgType::Request: {
                if (miners_.count(cid)) return;  // a miner does not make requests
                const uint64_t rid = next_rid_++;
                auto& r = requests_.emplace(rid, Request(rid, cid, m)).first->second;
                client_reqs_[cid].push_back(rid);
                maybe_finish(r);
                break;
            }
            case bitcoin::MsgType::Result: {
                auto mi = miners_.find(cid);
                if (mi == miners_.end() || mi->second.empty()) return;  // stray
                const Job j = mi->second.front();  // a miner answers in the order it got its jobs
                mi->second.pop_front();
                free_since_[cid] = tick_++;
                // its rate on this job: from when it could start it (sent, or its
                // previous result if that came later) to this result
                MinerRate& mr = rates_[cid];
                const auto now = Clock::now();
                const auto start = mr.have_done ? std::max(j.sent, mr.last_done) : j.sent;
                mr.last_done = now;
                mr.have_done = true;
                const double secs = std::chrono::duration<double>(now - start).count();
                if (secs > 0) {
                    mr.samples.push_back((double)(j.r.second - j.r.first + 1) / secs);
                    if (mr.samples.size() > kRateSamples) mr.samples.pop_front();
                }
                auto ri = requests_.find(j.rid);
                if (ri != requests_.end()) {  // else its client is gone (README:414)
                    Request& r = ri->second;
                    --r.inflight;
                    r.best = std::min(r.best, std::make_pair(m.Hash, m.Nonce));
                    maybe_finish(r);
                }
                break;
            }
        }
        schedule();
    }

    void on_lost(int64_t cid) {
        auto mi = miners_.find(cid);
        if (mi != miners_.end()) {
            for (auto it = mi->second.rbegin(); it != mi->second.rend(); ++it) {  // README:413, lowest first
                auto ri = requests_.find(it->rid);
                if (ri != requests_.end()) {
                    --ri->second.inflight;
                    ri->second.retry.push_front(it->r);
                }
            }
            miners_.erase(mi);
            free_since_.erase(cid);
            rates_.erase(cid);
            if (verbose_) std::fprintf(stderr, "miner %lld lost\n", (long long)cid);
        } else {
            auto ci = client_reqs_.find(cid);
            if (ci != client_reqs_.end()) {
                for (uint64_t rid : ci->second) requests_.erase(rid);  // README:414
                client_reqs_.erase(ci);
            }
        }
        schedule();
    }

    Request* pick() {  // fewest chunks in flight, oldest on ties (requests_ is ordered by rid)
        Request* best = nullptr;
        for (auto& kv : requests_)
            if (kv.second.has_work() && (!best || kv.second.inflight < best->inflight)) best = &kv.second;
        return best;
    }

    int64_t free_miner() const {  // fewest queued jobs, then longest since its count dropped
        int64_t best = 0;
        std::pair<size_t, uint64_t> key{SIZE_MAX, UINT64_MAX};
        for (const auto& kv : miners_)
            if (kv.second.size() < depth_) {
                const auto k = std::make_pair(kv.second.size(), free_since_.at(kv.first));
                if (k < key) {
                    key = k;
                    best = kv.first;
                }
            }
        return best;
    }

    // Nonces of miner mid's next fresh chunk of r (chunk_for).
    uint64_t chunk_size(int64_t mid, const Request& r) {
        MinerRate& mr = rates_[mid];
        const double rate = mr.rate();
        uint64_t k = 1;
        if (target_s_ > 0 && rate > 0) {
            double known = 0, total = 0;
            size_t nk = 0;
            for (const auto& kv : rates_)
                if (kv.second.rate() > 0) {
                    known += kv.second.rate();
                    ++nk;
                }
            for (const auto& kv : rates_) total += kv.second.rate() > 0 ? kv.second.rate() : known / (double)nk;
            // as a double: the whole 2^64 range does not fit a u64 count
            const double remaining = r.done ? 0.0 : (double)(r.upper - r.next_lower) + 1.0;
            k = chunk_for(chunk_, target_s_, max_mult_, rate, mr.mult, remaining, total > 0 ? rate / total : 1.0);
        }
        mr.mult = k;
        return k > UINT64_MAX / chunk_ ? UINT64_MAX : k * chunk_;
    }

    void schedule() {
        for (;;) {
            const int64_t mid = free_miner();
            if (!mid) return;
            Request* r = pick();
            if (!r) return;
            const Range c = r->take(chunk_size(mid, *r));
            try {
                srv_.Write(mid, bitcoin::NewRequest(r->data, c.first, c.second).Marshal());
            } catch (const lsp::LSPError&) {  // miner already gone (server.go:177-179)
                r->retry.push_front(c);
                on_lost(mid);
                return;
            }
            miners_[mid].push_back(Job{r->rid, c, Clock::now()});
            ++r->inflight;
        }
    }

    void maybe_finish(Request& r) {
        if (!r.finished()) return;
        r.answered = true;
        auto ci = client_reqs_.find(r.client);
        if (ci == client_reqs_.end()) return;
        auto& q = ci->second;
        while (!q.empty() && requests_.at(q.front()).answered) {  // in the order the client sent them
            auto done = requests_.find(q.front());
            q.pop_front();
            try {
                srv_.Write(done->second.client, bitcoin::NewResult(done->second.best.first, done->second.best.second)
                                                    .Marshal());
            } catch (const lsp::LSPError&) {  // client gone; Read reports its loss
            }
            requests_.erase(done);
        }
        if (q.empty()) client_reqs_.erase(ci);
    }

    lsp::Server& srv_;
    const uint64_t chunk_;
    const size_t depth_;
    const double target_s_;
    const uint64_t max_mult_;
    const bool verbose_;
    std::map<int64_t, MinerRate> rates_;
    std::map<int64_t, std::deque<Job>> miners_;  // conn id -> jobs sent, oldest first
    std::map<int64_t, uint64_t> free_since_;
    uint64_t tick_ = 0, next_rid_ = 1;
    std::map<uint64_t, Request> requests_;  // by rid = arrival order
    std::map<int64_t, std::deque<uint64_t>> client_reqs_;
};

[[noreturn]] void usage(const char* argv0) {
    std::fprintf(stderr,
                 "usage: %s port [--chunk N] [--depth D] [--target-ms T] [--max-mult M] [--epoch-limit K]\n"
                 "          [--epoch-millis MS] [--window-size W]\n"
                 "          [--host ADDR] [--drop-read P] [--drop-write P] [-v]\n",
                 argv0);
    std::exit(1);
}

}  // namespace

int main(int argc, char** argv) {
    lsp::Params p;
    uint64_t chunk = 1ull << 32;
    long long depth = 2, target_ms = 300, max_mult = 64;
    int port = -1;
    std::string host = "127.0.0.1";
    bool verbose = false;
    for (int i = 1; i < argc; ++i) {
        const std::string a = argv[i];
        const auto val = [&]() -> const char* {
            if (i + 1 >= argc) usage(argv[0]);
            return argv[++i];
        };
        if (a == "--chunk") chunk = std::strtoull(val(), nullptr, 10);
        else if (a == "--depth") depth = std::atoll(val());
        else if (a == "--target-ms") target_ms = std::atoll(val());
        else if (a == "--max-mult") max_mult = std::atoll(val());
        else if (a == "--epoch-limit") p.EpochLimit = std::atoi(val());
        else if (a == "--epoch-millis") p.EpochMillis = std::atoi(val());
        else if (a == "--window-size") p.WindowSize = std::atoi(val());
        else if (a == "--host") host = val();
        else if (a == "--drop-read") lspnet::SetServerReadDropPercent(std::atoi(val()));
        else if (a == "--drop-write") lspnet::SetServerWriteDropPercent(std::atoi(val()));
        else if (a == "-v") verbose = true;
        else if (port < 0 && !a.empty() && a[0] != '-') port = std::atoi(a.c_str());
        else usage(argv[0]);
    }
    if (port < 0 || chunk < 1 || depth < 1 || target_ms < 0 || max_mult < 1) usage(argv[0]);
    std::unique_ptr<lsp::Server> srv;
    try {
        srv = lsp::NewServer(port, p, host);
    } catch (const lsp::LSPError& e) {
        std::fprintf(stderr, "Failed to start server: %s\n", e.what());
        return 1;
    }
    if (port == 0) {
        std::printf("port %d\n", srv->port());
        std::fflush(stdout);
    }
    BitcoinServer(*srv, chunk, (size_t)depth, (double)target_ms / 1e3, (uint64_t)max_mult, verbose).serve();
    return 0;
}
