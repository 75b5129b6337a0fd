// bm_client.cpp -- the reference's request client in C++ (no GPU needed).
//
//   bm_client host:port message maxNonce [--epoch-limit K] [--epoch-millis MS]
//             [--window-size W] [--drop-read P] [--drop-write P]
//
// bitcoin/client/client.go:14-83 and README:378-406: connect over LSP, send
// Request(message, 0, maxNonce) (:33-36), wait for the server's Result
// (:42-50) and print "Result <minHash> <nonce>" (printResult, :76-78), or
// "Disconnected" (printDisconnected, :81-83) when the connection is lost or
// cannot be made.  maxNonce is an unsigned 64-bit decimal.
#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <memory>
#include <string>

#include "btcminer.hpp"
#include "lsp.hpp"

int main(int argc, char** argv) {
    std::string pos[3];
    int npos = 0, drop_read = 0, drop_write = 0;
    lsp::Params p;
    for (int i = 1; i < argc; ++i) {
        const std::string a = argv[i];
        const bool has = i + 1 < argc;
        if (a == "--epoch-limit" && has) p.EpochLimit = std::atoi(argv[++i]);
        else if (a == "--epoch-millis" && has) p.EpochMillis = std::atoi(argv[++i]);
        else if (a == "--window-size" && has) p.WindowSize = std::atoi(argv[++i]);
        else if (a == "--drop-read" && has) drop_read = std::atoi(argv[++i]);
        else if (a == "--drop-write" && has) drop_write = std::atoi(argv[++i]);
        else if (npos < 3 && a.rfind("--", 0) != 0) pos[npos++] = a;  // "-1" is a (bad) maxNonce, not a flag
        else npos = 4;
    }
    if (npos != 3) {
        std::fprintf(stderr, "usage: %s host:port message maxNonce [--epoch-limit K] [--epoch-millis MS] ...\n",
                     argv[0]);
        return 1;
    }
    errno = 0;
    char* end = nullptr;
    const unsigned long long max_nonce = std::strtoull(pos[2].c_str(), &end, 10);
    // strconv.ParseUint(s, 10, 64): digits only (strtoull alone would take
    // leading spaces and a sign)
    const bool digits = !pos[2].empty() && pos[2].find_first_not_of("0123456789") == std::string::npos;
    if (!digits || *end || errno == ERANGE) {
        std::fprintf(stderr, "maxNonce must be an unsigned 64-bit integer, got '%s'\n", pos[2].c_str());
        return 2;
    }
    lspnet::SetClientReadDropPercent(drop_read);
    lspnet::SetClientWriteDropPercent(drop_write);
    try {
        auto c = lsp::NewClient(pos[0], p);
        try {
            c->Write(bitcoin::NewRequest(pos[1], 0, max_nonce).Marshal());
            for (;;) {
                bitcoin::Message m;
                try {
                    m = bitcoin::Message::Unmarshal(c->Read());
                } catch (const bitcoin::DecodeError&) {
                    continue;
                }
                if (m.Type == bitcoin::MsgType::Result) {
                    std::printf("Result %llu %llu\n", (unsigned long long)m.Hash, (unsigned long long)m.Nonce);
                    try {
                        c->Close();
                    } catch (const lsp::LSPError&) {
                    }
                    return 0;
                }
            }
        } catch (const lsp::LSPError&) {
            try {
                c->Close();
            } catch (const lsp::LSPError&) {
            }
        }
    } catch (const lsp::LSPError&) {
    }
    std::printf("Disconnected\n");
    return 0;
}
