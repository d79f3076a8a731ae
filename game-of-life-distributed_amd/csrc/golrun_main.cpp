// golrun — the reference's command line (main.go:13-66) over the C++ mirror
// of gol.Run (gol_host.h) and libgolhip.so.
//
//   golrun [-t threads] [-w width] [-h height] [-turns n] [-noVis] [-root dir] [-device n]
//
// Same flags, defaults and output as main.go: "Threads: / Width: / Height:"
// lines, then gol.Run on images/<w>x<h>.pgm with an events channel of
// capacity 1000 and a keyPresses channel of capacity 10.  There is no SDL
// window in this build (sdl/ is out of scope): without -noVis
// the run is headless too, and single-character lines on stdin (s, q, p, k)
// are forwarded as key presses, the keys the SDL loop forwards (sdl/loop.go).
// The headless drain loop ends at FinalTurnComplete (main.go:59-66) or when
// the events channel closes.
#include <climits>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <iostream>
#include <string>
#include <thread>

#include "gol_host.h"

namespace {

[[noreturn]] void usage(const char *msg) {
    std::fprintf(stderr, "golrun: %s\nusage: golrun [-t threads] [-w width] [-h height] [-turns n] [-noVis] "
                         "[-root dir] [-device n]\n", msg);
    std::exit(2);
}

long long parse_int(const std::string &s, const char *flag) {
    char *end = nullptr;
    const long long v = std::strtoll(s.c_str(), &end, 10);
    if (s.empty() || *end) usage((std::string("invalid value \"") + s + "\" for flag -" + flag).c_str());
    return v;
}

}  // namespace

int main(int argc, char **argv) {
    gol::Params params;
    params.Threads = 8;
    params.ImageWidth = 512;
    params.ImageHeight = 512;
    long long turns = 10000000000LL;  // main.go:37-41
    bool no_vis = false;
    gol::RunOptions opt;
    for (int i = 1; i < argc; ++i) {
        std::string a = argv[i];
        if (a.rfind("--", 0) == 0) a = a.substr(1);  // Go's flag package accepts -flag and --flag
        std::string key = a, val;
        const size_t eq = a.find('=');
        if (eq != std::string::npos) {
            key = a.substr(0, eq);
            val = a.substr(eq + 1);
        }
        auto value = [&]() -> std::string {
            if (eq != std::string::npos) return val;
            if (i + 1 >= argc) usage(("flag needs an argument: " + key).c_str());
            return argv[++i];
        };
        if (key == "-t") {
            params.Threads = parse_int(value(), "t");
        } else if (key == "-w") {
            params.ImageWidth = parse_int(value(), "w");
        } else if (key == "-h") {
            params.ImageHeight = parse_int(value(), "h");
        } else if (key == "-turns") {
            turns = parse_int(value(), "turns");
        } else if (key == "-noVis") {
            no_vis = eq == std::string::npos || val == "true" || val == "1";
        } else if (key == "-root") {
            opt.root = value();
        } else if (key == "-device") {
            opt.device = (int)parse_int(value(), "device");
        } else {
            usage(("flag provided but not defined: " + key).c_str());
        }
    }
    params.Turns = turns;  // a Go int (64-bit): the reference's 10^10 default passes through

    std::printf("Threads: %lld\nWidth: %lld\nHeight: %lld\n", (long long)params.Threads, (long long)params.ImageWidth,
                (long long)params.ImageHeight);
    std::fflush(stdout);
    if (!no_vis) std::fprintf(stderr, "golrun: no SDL window in this build; running headless (keys s/q/p/k on stdin)\n");

    gol::Chan<char32_t> keys(10);
    gol::Chan<gol::Event> events(1000);
    std::string error;
    std::thread engine([&] {
        try {
            gol::Run(params, &events, &keys, opt);
        } catch (const std::exception &e) {
            error = e.what();
            events.close();
        }
    });
    if (!no_vis) {
        std::thread([&keys] {  // detached: blocks on stdin until the process ends
            std::string line;
            while (std::getline(std::cin, line))
                if (line.size() == 1 && std::strchr("sqpk", line[0])) keys.send((char32_t)line[0]);
        }).detach();
    }
    gol::Event ev;
    while (events.recv(ev)) {  // main.go:59-66
        if (ev.kind == gol::EventKind::FinalTurnComplete) break;
    }
    while (events.recv(ev)) {  // let Run finish (StateChange Quitting, close)
    }
    engine.join();
    if (!error.empty()) {
        std::fprintf(stderr, "golrun: %s\n", error.c_str());
        return 1;
    }
    return 0;
}
