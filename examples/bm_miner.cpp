// bm_miner.cpp -- the reference miner's job loop in C++ over the C ABI.
//
// Mirrors bitcoin/miner/miner.go:20-74 for everything but the transport:
// it first emits the Join message (miner.go:34-38), then reads one JSON
// bitcoin.Message per input line (what miner.Read() would deliver, :49-55),
// answers every Request with the JSON Result of the GPU search
// (:58-72, through btcminer::Context::search = bm_search_gpu), ignores other
// message types, and reports undecodable lines on stderr and goes on.
// Bounds are inclusive (README:329); --exclusive-upper reproduces
// miner.go:59's literal `i < Upper`.
//
//   bm_miner [--gpus N] [--exclusive-upper] < requests.jsonl > results.jsonl
//   bm_miner --json-selftest < messages.jsonl   (no GPU: re-marshal each line,
//                                                 "error <why>" when it does not decode)
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <iostream>
#include <string>

#include "btcminer.hpp"

int main(int argc, char** argv) {
    int gpus = 1;
    bool exclusive = false, selftest = false;
    for (int i = 1; i < argc; ++i) {
        if (!std::strcmp(argv[i], "--gpus") && i + 1 < argc) gpus = std::atoi(argv[++i]);
        else if (!std::strcmp(argv[i], "--exclusive-upper")) exclusive = true;
        else if (!std::strcmp(argv[i], "--json-selftest")) selftest = true;
        else {
            std::fprintf(stderr, "usage: %s [--gpus N] [--exclusive-upper] | --json-selftest\n", argv[0]);
            return 1;
        }
    }
    std::string line;
    if (selftest) {
        while (std::getline(std::cin, line)) {
            try {
                std::cout << bitcoin::Message::Unmarshal(line).Marshal() << "\n";
            } catch (const bitcoin::DecodeError& e) {
                std::cout << "error " << e.what() << "\n";
            }
        }
        return 0;
    }
    try {
        btcminer::Context ctx(gpus);  // no GPU: BM_ENODEV, before joining (no CPU fallback)
        std::cout << bitcoin::NewJoin().Marshal() << std::endl;
        while (std::getline(std::cin, line)) {
            bitcoin::Message job;
            try {
                job = bitcoin::Message::Unmarshal(line);
            } catch (const bitcoin::DecodeError& e) {
                std::cerr << "bad job: " << e.what() << "\n";
                continue;
            }
            if (job.Type != bitcoin::MsgType::Request) continue;
            uint64_t upper = job.Upper;
            if (exclusive) {
                if (upper <= job.Lower) {  // the loop runs zero times (miner.go:45-46)
                    std::cout << bitcoin::NewResult(UINT64_MAX, UINT64_MAX).Marshal() << std::endl;
                    continue;
                }
                --upper;
            }
            const btcminer::Result r = ctx.search(job.Data, job.Lower, upper);
            std::cout << bitcoin::NewResult(r.hash, r.nonce).Marshal() << std::endl;
        }
    } catch (const btcminer::Error& e) {
        std::cout << "error " << e.status() << " " << e.what() << std::endl;
        return 2;
    }
    return 0;
}
