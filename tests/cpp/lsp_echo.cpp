// lsp_echo.cpp -- test driver for lsp::Server (include/lsp.hpp): echoes every
// payload back to the connection it came from.  Prints "port <n>" first; on
// stdin EOF it calls Close() and prints "closed ok" or "closed lost".  Lost
// connections are reported as "lost <id>".  A stdin line "drain" waits (at
// most 60 s) until every echo written so far is acknowledged and prints
// "drained" (or "not drained").  Built and run by
// tests/test_cpp_server.py (the Python LSP clients are the other side).
//
//   lsp_echo [--epoch-limit K] [--epoch-millis MS] [--window-size W]
//            [--drop-read P] [--drop-write P]
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <iostream>
#include <string>
#include <thread>

#include "lsp.hpp"

int main(int argc, char** argv) {
    lsp::Params p;
    for (int i = 1; i + 1 < argc; i += 2) {
        const std::string a = argv[i];
        const int v = std::atoi(argv[i + 1]);
        if (a == "--epoch-limit") p.EpochLimit = v;
        else if (a == "--epoch-millis") p.EpochMillis = v;
        else if (a == "--window-size") p.WindowSize = v;
        else if (a == "--drop-read") lspnet::SetServerReadDropPercent(v);
        else if (a == "--drop-write") lspnet::SetServerWriteDropPercent(v);
        else return 1;
    }
    auto srv = lsp::NewServer(0, p);
    std::printf("port %d\n", srv->port());
    std::fflush(stdout);
    std::thread echo([&] {
        for (;;) {
            try {
                auto [cid, payload] = srv->Read();
                try {
                    srv->Write(cid, payload);
                } catch (const lsp::LSPError&) {
                }
            } catch (const lsp::ServerError& e) {
                if (e.conn_id() == 0) return;
                std::printf("lost %lld\n", (long long)e.conn_id());
                std::fflush(stdout);
            }
        }
    });
    std::string line;
    while (std::getline(std::cin, line)) {
        if (line != "drain") continue;
        bool ok = false;
        for (int i = 0; i < 12000 && !(ok = srv->Drained()); ++i)
            std::this_thread::sleep_for(std::chrono::milliseconds(5));
        std::printf(ok ? "drained\n" : "not drained\n");
        std::fflush(stdout);
    }
    bool lost = false;
    try {
        srv->Close();
    } catch (const lsp::LSPError&) {
        lost = true;
    }
    echo.join();
    std::printf("closed %s\n", lost ? "lost" : "ok");
    return 0;
}
