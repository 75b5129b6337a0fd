// bm_miner.cpp -- the reference miner process in C++ over the C ABI.
//
//   bm_miner host:port [--gpus N | --device D] [--exclusive-upper]
//            [--epoch-limit K] [--epoch-millis MS] [--window-size W]
//            [--drop-read P] [--drop-write P] [-v]
//       bitcoin/miner/miner.go:20-74: open the GPU context first (no GPU ->
//       "error -2 ..." and exit 2, before joining: there is no CPU fallback),
//       connect over LSP (lsp.hpp), send Join (:34-38), then answer every
//       Request with the Result of one bm_search_gpu call (:49-72) until the
//       server is lost, which shuts the miner down (README:412).
//   bm_miner --stdin [--gpus N] [--exclusive-upper]
//       the same job loop over JSON lines on stdin/stdout (Join first).
//   bm_miner --json-selftest
//       no GPU: re-marshal each stdin line, "error <why>" when it does not decode.
//
// Bounds are inclusive (README:329); --exclusive-upper reproduces
// miner.go:59's literal `i < Upper`.  Undecodable jobs go to stderr as
// "bad job" and the loop goes on.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <iostream>
#include <memory>
#include <string>

#include "btcminer.hpp"
#include "lsp.hpp"

namespace {

struct Options {
    std::string hostport;
    int gpus = 1, device = -1;
    bool exclusive = false, stdin_mode = false, selftest = false, verbose = false;
    lsp::Params params;
    int drop_read = 0, drop_write = 0;
};

// Request -> Result (miner.go:54-72); nullopt for other message types.
std::optional<bitcoin::Message> answer(btcminer::Context& ctx, const bitcoin::Message& job, bool exclusive) {
    if (job.Type != bitcoin::MsgType::Request) return std::nullopt;
    uint64_t upper = job.Upper;
    if (exclusive) {
        if (upper <= job.Lower) return bitcoin::NewResult(UINT64_MAX, UINT64_MAX);  // zero iterations (:45-46)
        --upper;
    }
    const btcminer::Result r = ctx.search(job.Data, job.Lower, upper);
    return bitcoin::NewResult(r.hash, r.nonce);
}

btcminer::Context open_context(const Options& o) {
    btcminer::Context ctx = o.device >= 0 ? btcminer::Context(std::vector<int>{o.device}) : btcminer::Context(o.gpus);
    if (ctx.num_devices() > 1) ctx.set_balance(true);  // pieces follow each GPU's measured rate
    return ctx;
}

int run_stdin(const Options& o) {
    btcminer::Context ctx = open_context(o);
    std::cout << bitcoin::NewJoin().Marshal() << std::endl;
    std::string line;
    while (std::getline(std::cin, line)) {
        try {
            if (auto r = answer(ctx, bitcoin::Message::Unmarshal(line), o.exclusive))
                std::cout << r->Marshal() << std::endl;
        } catch (const bitcoin::DecodeError& e) {
            std::cerr << "bad job: " << e.what() << "\n";
        }
    }
    return 0;
}

int run_lsp(const Options& o) {
    btcminer::Context ctx = open_context(o);
    lspnet::SetClientReadDropPercent(o.drop_read);
    lspnet::SetClientWriteDropPercent(o.drop_write);
    std::unique_ptr<lsp::Client> c;
    try {
        c = lsp::NewClient(o.hostport, o.params);  // miner.go:29-31
    } catch (const lsp::LSPError& e) {
        std::fprintf(stderr, "Failed to connect to %s: %s\n", o.hostport.c_str(), e.what());
        return 1;
    }
    long jobs = 0;
    try {
        c->Write(bitcoin::NewJoin().Marshal());  // miner.go:34-38
        for (;;) {
            const std::string payload = c->Read();  // miner.go:49
            std::optional<bitcoin::Message> r;
            try {
                r = answer(ctx, bitcoin::Message::Unmarshal(payload), o.exclusive);
            } catch (const bitcoin::DecodeError& e) {
                std::cerr << "bad job: " << e.what() << "\n";
                continue;
            }
            if (!r) continue;
            c->Write(r->Marshal());  // miner.go:68-72
            ++jobs;
        }
    } catch (const lsp::LSPError& e) {
        if (o.verbose) std::fprintf(stderr, "lost contact with the server after %ld jobs: shutting down\n", jobs);
    }
    try {
        c->Close();
    } catch (const lsp::LSPError&) {
    }
    return 0;
}

[[noreturn]] void usage(const char* argv0) {
    std::fprintf(stderr,
                 "usage: %s host:port [--gpus N | --device D] [--exclusive-upper] [--epoch-limit K]\n"
                 "          [--epoch-millis MS] [--window-size W] [--drop-read P] [--drop-write P] [-v]\n"
                 "       %s --stdin [--gpus N | --device D] [--exclusive-upper]\n"
                 "       %s --json-selftest\n",
                 argv0, argv0, argv0);
    std::exit(1);
}

}  // namespace

int main(int argc, char** argv) {
    Options o;
    for (int i = 1; i < argc; ++i) {
        const std::string a = argv[i];
        const auto num = [&]() -> int {
            if (i + 1 >= argc) usage(argv[0]);
            return std::atoi(argv[++i]);
        };
        if (a == "--gpus") o.gpus = num();
        else if (a == "--device") o.device = num();
        else if (a == "--exclusive-upper") o.exclusive = true;
        else if (a == "--stdin") o.stdin_mode = true;
        else if (a == "--json-selftest") o.selftest = true;
        else if (a == "--epoch-limit") o.params.EpochLimit = num();
        else if (a == "--epoch-millis") o.params.EpochMillis = num();
        else if (a == "--window-size") o.params.WindowSize = num();
        else if (a == "--drop-read") o.drop_read = num();
        else if (a == "--drop-write") o.drop_write = num();
        else if (a == "-v") o.verbose = true;
        else if (a.size() && a[0] != '-' && o.hostport.empty()) o.hostport = a;
        else usage(argv[0]);
    }
    if (o.selftest) {
        std::string line;
        while (std::getline(std::cin, line)) {
            try {
                std::cout << bitcoin::Message::Unmarshal(line).Marshal() << "\n";
            } catch (const bitcoin::DecodeError& e) {
                std::cout << "error " << e.what() << "\n";
            }
        }
        return 0;
    }
    if (o.stdin_mode == !o.hostport.empty()) usage(argv[0]);
    try {
        return o.stdin_mode ? run_stdin(o) : run_lsp(o);
    } catch (const btcminer::Error& e) {
        std::cout << "error " << e.status() << " " << e.what() << std::endl;
        return 2;
    }
}
