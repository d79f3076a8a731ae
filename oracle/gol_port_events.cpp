// gol_port_events.cpp — TEST INFRASTRUCTURE ONLY (CPU baseline of bench.py).
//
// The worker-pool port of gol_oracle.c run the way the reference's gol.Run
// runs it end to end, with every event delivered: distributor.go:72-80 (a
// CellFlipped for every cell alive at load), per turn :116-173 (the pool's
// turn, then initializeAliveCells :212-220 sending one CellFlipped per
// changed cell, then TurnComplete), and the end :180-206 (ImageOutputComplete,
// FinalTurnComplete with calculateAliveCells :420-432, StateChange Quitting,
// close).  The events go through the same channel type and the same send
// pattern as the GPU line's host mirror (gol::Chan<gol::Event> from
// csrc/gol_host.h; initial cells one send each, a turn's flips in chunks of
// 4096 through send_batch, TurnComplete one send), and a consumer thread runs
// the same drain loop as golrun_drain (main.go:59-66: recv_batch of up to
// 1024, counting by kind).  So bench.py's configs[0] CPU number "with events"
// is the same workload as its GPU line; oracle_run_workerpool stays the
// "engine only" number.  Nothing in the product links this file.
#include <pthread.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include "gol_host.h"  // gol::Chan / gol::Event: header-only parts, no HIP

extern "C" uint8_t *oracle_pool_turn(const uint8_t *world, int W, int H, int threads, pthread_t *tid);

namespace {
constexpr uint8_t kAlive = 255;

gol::Event flip_event(int64_t turn, int64_t x, int64_t y) {
    gol::Event e;
    e.kind = gol::EventKind::CellFlipped;
    e.CompletedTurns = turn;
    e.Cell.X = x;  // {X: col, Y: row}: the mirror's default orientation
    e.Cell.Y = y;
    return e;
}
}  // namespace

// Runs `turns` turns of the port on `board` (H x W bytes, 0/255) in place
// with every event through a channel of capacity `events_cap` (0: the
// unbuffered channel of gol_test.go; 1000: main.go:53).  counts[6] gets the
// events received by kind (gol::EventKind order), *last_turn the last
// TurnComplete, *final_alive len(FinalTurnComplete.Alive).  When out_pgm is
// not null the final board is written there as io.go:42-87's PGM (the GPU
// line writes out/<W>x<H>x<T>.pgm too).  Returns 0, or -1 on failure.
extern "C" int oracle_run_workerpool_events(uint8_t *board, int W, int H, long turns, int threads, int events_cap,
                                            uint64_t counts[6], int64_t *last_turn, int64_t *final_alive,
                                            const char *out_pgm) {
    if (!board || W <= 0 || H <= 0 || turns < 0 || threads < 1 || events_cap < 0 || !counts) return -1;
    const size_t n = (size_t)W * H;
    gol::Chan<gol::Event> events((size_t)events_cap);
    for (int k = 0; k < 6; ++k) counts[k] = 0;
    int64_t last = 0, fin = 0;
    std::thread drain([&] {  // main.go:59-66 (golrun_drain's loop)
        std::vector<gol::Event> batch;
        batch.reserve(1024);
        while (events.recv_batch(batch, 1024))
            for (const gol::Event &e : batch) {
                const int k = (int)e.kind;
                if (k >= 0 && k < 6) counts[k]++;
                if (e.kind == gol::EventKind::TurnComplete) last = e.CompletedTurns;
                if (e.kind == gol::EventKind::FinalTurnComplete) fin = (int64_t)e.Alive.size();
            }
    });
    // :72-80: every cell alive at load, turn 0, one send each
    for (int r = 0; r < H; ++r)
        for (int c = 0; c < W; ++c)
            if (board[(size_t)r * W + c] == kAlive) events.send(flip_event(0, c, r));
    std::vector<pthread_t> tid((size_t)threads + 1);
    uint8_t *world = (uint8_t *)malloc(n);
    if (!world) {
        events.close();
        drain.join();
        return -1;
    }
    memcpy(world, board, n);
    constexpr size_t kChunk = 4096;
    std::vector<gol::Event> chunk;
    chunk.reserve(kChunk);
    for (long t = 0; t < turns; ++t) {
        uint8_t *nw = oracle_pool_turn(world, W, H, threads, tid.data());
        // initializeAliveCells (:212-220): the changed cells in row-major order
        for (int r = 0; r < H; ++r)
            for (int c = 0; c < W; ++c) {
                const size_t i = (size_t)r * W + c;
                if (nw[i] == world[i]) continue;
                chunk.push_back(flip_event(t + 1, c, r));
                if (chunk.size() == kChunk) {
                    events.send_batch(chunk.data(), chunk.size());
                    chunk.clear();
                }
            }
        if (!chunk.empty()) {
            events.send_batch(chunk.data(), chunk.size());
            chunk.clear();
        }
        gol::Event tc;
        tc.kind = gol::EventKind::TurnComplete;
        tc.CompletedTurns = t + 1;
        events.send(tc);
        free(world);
        world = nw;
    }
    // :180-206
    std::vector<util::Cell> alive;
    for (int r = 0; r < H; ++r)
        for (int c = 0; c < W; ++c)
            if (world[(size_t)r * W + c] == kAlive) alive.push_back(util::Cell{c, r});
    int rc = 0;
    if (out_pgm) {
        FILE *f = fopen(out_pgm, "wb");
        if (!f || fprintf(f, "P5\n%d %d\n255\n", W, H) < 0 || fwrite(world, 1, n, f) != n) rc = -1;
        if (f) fclose(f);
    }
    gol::Event io;
    io.kind = gol::EventKind::ImageOutputComplete;
    io.CompletedTurns = turns;
    events.send(io);
    gol::Event ft;
    ft.kind = gol::EventKind::FinalTurnComplete;
    ft.CompletedTurns = turns;
    ft.Alive = std::move(alive);
    events.send(ft);
    gol::Event q;
    q.kind = gol::EventKind::StateChange;
    q.CompletedTurns = turns;
    q.NewState = gol::State::Quitting;
    events.send(q);
    events.close();
    drain.join();
    memcpy(board, world, n);
    free(world);
    if (last_turn) *last_turn = last;
    if (final_alive) *final_alive = fin;
    return rc;
}
