// gol_host.cpp — the reference's gol.Run host flow over libgolhip.so.
//
// Mirrors gol/distributor.go:30-209 (distributor), :223-280 (keyPress),
// :283-302 (ticker) and gol/io.go:42-126 (PGM io).  The turn loop itself is
// golhip_step; everything here is event sequencing and file I/O.
#include "gol_host.h"

#include <sys/stat.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>
#include <thread>

#include "../../include/golhip.h"
#include "../../include/golrun.h"

namespace gol {

std::string StateString(State s) {
    switch (s) {
        case State::Paused: return "Paused";
        case State::Executing: return "Executing";
        case State::Quitting: return "Quitting";
    }
    return "Incorrect State";
}

std::string Event::String() const {
    switch (kind) {
        case EventKind::AliveCellsCount: return "Alive Cells " + std::to_string(CellsCount);
        case EventKind::ImageOutputComplete: return "File " + Filename + " output complete";
        case EventKind::StateChange: return StateString(NewState);
        default: return "";  // CellFlipped, TurnComplete, FinalTurnComplete (event.go:107-129)
    }
}

// ---------------------------------------------------------------- PGM io
// readPgmImage (io.go:90-126): whitespace-separated fields P5, W, H, 255;
// the raster follows the single whitespace byte after maxval.
std::vector<uint8_t> ReadPgm(const std::string &path, int64_t width, int64_t height) {
    std::ifstream f(path, std::ios::binary);
    if (!f) throw std::runtime_error("open " + path + ": no such file or directory");
    std::vector<uint8_t> data((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
    size_t pos = 0;
    auto ws = [](uint8_t c) { return c == ' ' || c == '\t' || c == '\n' || c == '\r' || c == '\v' || c == '\f'; };
    std::string fields[4];
    for (auto &fld : fields) {
        while (pos < data.size() && ws(data[pos])) ++pos;
        while (pos < data.size() && !ws(data[pos])) fld.push_back((char)data[pos++]);
    }
    ++pos;
    if (fields[0] != "P5") throw std::runtime_error("Not a pgm file");
    if (std::atoll(fields[1].c_str()) != width) throw std::runtime_error("Incorrect width");
    if (std::atoll(fields[2].c_str()) != height) throw std::runtime_error("Incorrect height");
    if (std::atoll(fields[3].c_str()) != 255) throw std::runtime_error("Incorrect maxval/bit depth");
    const size_t n = (size_t)width * height;
    if (data.size() < pos + n) throw std::runtime_error("short raster in " + path);
    return std::vector<uint8_t>(data.begin() + pos, data.begin() + pos + n);
}

// writePgmImage (io.go:42-87): "P5\n" W " " H "\n" "255\n" + raster, one bulk write.
void WritePgm(const std::string &path, int64_t width, int64_t height, const uint8_t *raster) {
    std::ofstream f(path, std::ios::binary | std::ios::trunc);
    if (!f) throw std::runtime_error("create " + path + " failed");
    f << "P5\n" << width << " " << height << "\n" << 255 << "\n";
    f.write(reinterpret_cast<const char *>(raster), (std::streamsize)width * height);
    f.flush();
    if (!f) throw std::runtime_error("write " + path + " failed");
}

namespace {

void check(int rc) {
    if (rc != GOLHIP_OK) throw std::runtime_error(std::string("golhip: ") + golhip_last_error());
}

int env_int(const char *name, int dflt) {
    const char *v = std::getenv(name);
    return (v && *v) ? std::atoi(v) : dflt;
}

// The board behind Run: one whole-torus handle, or row strips (GOL_NGPU /
// GOL_STRIPS) stepped together by golhip_group_step_ex.  Every side channel
// of the strips is gathered in strip order, which is the board's row-major
// order: alive lists and flip lists concatenate, counts add up.
// Page-locked flip-list buffer the engine's flip kernel writes directly
// (golhip_host_alloc): 4-byte cell indices y * W + x.
struct FlipBuffer {
    uint32_t *p = nullptr;
    uint64_t cap = 0;  // entries
    void grow(uint64_t n) { grow_keep(n, 0); }
    // at least n entries (doubling), the first `keep` entries preserved
    void grow_keep(uint64_t n, uint64_t keep) {
        if (n <= cap) return;
        if (keep) n = std::max<uint64_t>(n, 2 * cap);
        void *q = nullptr;
        check(golhip_host_alloc(n * sizeof(uint32_t), &q));
        if (keep) memcpy(q, p, keep * sizeof(uint32_t));
        if (p) golhip_host_free(p);
        p = static_cast<uint32_t *>(q);
        cap = n;
    }
    ~FlipBuffer() {
        if (p) golhip_host_free(p);
    }
};

struct Engine {
    std::vector<golhip_t> hs;
    std::vector<int64_t> row0;
    int64_t W = 0, H = 0;
    Engine(int64_t w, int64_t hgt, const RunOptions &opt) : W(w), H(hgt) {
        const int ngpu = opt.ngpu >= 0 ? opt.ngpu : env_int("GOL_NGPU", 1);
        const int strips = opt.strips >= 0 ? opt.strips : env_int("GOL_STRIPS", 0);
        int n = strips > 0 ? strips : std::max(1, ngpu);
        n = (int)std::min<int64_t>(n, hgt);
        if (n <= 1) {
            hs.push_back(nullptr);
            row0.push_back(0);
            check(golhip_create((int32_t)w, (int32_t)hgt, opt.device, 0, &hs[0]));
            return;
        }
        int32_t ndev = 0;
        check(golhip_device_count(&ndev));
        const int devs = std::max(1, std::min(ngpu > 0 ? ngpu : 1, (int)ndev));
        for (int i = 0; i < n; ++i) {
            const int64_t r0 = hgt * i / n, r1 = hgt * (i + 1) / n;
            golhip_t h = nullptr;
            const int dev = devs > 1 ? i % devs : opt.device;
            const int rc = golhip_create_strip((int32_t)w, (int32_t)hgt, (int32_t)r0, (int32_t)(r1 - r0), dev, 0, &h);
            if (rc != GOLHIP_OK) {
                for (golhip_t x : hs) golhip_destroy(x);
                hs.clear();
                check(rc);
            }
            hs.push_back(h);
            row0.push_back(r0);
        }
    }
    ~Engine() {
        for (golhip_t h : hs) golhip_destroy(h);
    }
    bool one() const { return hs.size() == 1; }
    int64_t rows(size_t i) const { return (i + 1 < row0.size() ? row0[i + 1] : H) - row0[i]; }
    void load(const uint8_t *raster) {
        for (size_t i = 0; i < hs.size(); ++i) check(golhip_load_bytes(hs[i], raster + row0[i] * W));
    }
    void snapshot(uint8_t *out) {
        for (size_t i = 0; i < hs.size(); ++i) check(golhip_snapshot_bytes(hs[i], out + row0[i] * W));
    }
    void alive_count(uint64_t *n, int64_t *at) {
        *n = 0;
        for (golhip_t h : hs) {
            uint64_t c = 0;
            check(golhip_alive_count(h, &c, at));
            *n += c;
        }
    }
    // calculateAliveCells (distributor.go:420-432) / the flips of the last turn
    std::vector<util::Cell> cells(int (*fn)(golhip_t, int32_t *, uint64_t, uint64_t *), bool transpose) {
        std::vector<util::Cell> out;
        for (golhip_t h : hs) {
            uint64_t n = 0;
            int rc = fn(h, nullptr, 0, &n);
            if (rc != GOLHIP_OK && rc != GOLHIP_ERANGE) check(rc);
            std::vector<int32_t> xy(2 * std::max<uint64_t>(n, 1));
            check(fn(h, xy.data(), n, &n));
            for (uint64_t i = 0; i < n; ++i) {
                util::Cell c;
                c.X = transpose ? xy[2 * i + 1] : xy[2 * i];
                c.Y = transpose ? xy[2 * i] : xy[2 * i + 1];
                out.push_back(c);
            }
        }
        return out;
    }
    void step(int64_t turns) {
        if (one()) {
            check(golhip_step(hs[0], turns, 0));
            check(golhip_sync(hs[0]));
        } else {
            check(golhip_group_step_ex(hs.data(), (int32_t)hs.size(), turns, 0));
        }
    }
    // Up to `want` turns with every turn's flip list as cell indices y * W + x
    // (golhip_flip_stream's contract: stops before a turn that does not fit;
    // GOLHIP_ERANGE with *n = what the first turn needs).  Strips: one turn a
    // group step; each strip's list of that turn is sized after the step
    // (golhip_flips with cap 0) and the buffer grown to fit before the copy,
    // so every turn runs and the buffer holds only what the lists need.
    int flip_stream(int64_t want, FlipBuffer &fb, uint64_t *counts, int64_t *done, uint64_t *n) {
        if (one()) return golhip_flip_stream(hs[0], want, GOLHIP_FLIPS_INDEX, fb.p, fb.cap, counts, done, n);
        *done = 0;
        *n = 0;
        std::vector<int32_t> xy;
        for (int64_t t = 0; t < want; ++t) {
            check(golhip_group_step_ex(hs.data(), (int32_t)hs.size(), 1, 1));
            uint64_t turn_n = 0;
            for (golhip_t h : hs) {
                uint64_t k = 0;
                int rc = golhip_flips(h, nullptr, 0, &k);
                if (rc != GOLHIP_OK && rc != GOLHIP_ERANGE) check(rc);
                if (k == 0) continue;
                xy.resize(2 * k);
                check(golhip_flips(h, xy.data(), k, &k));
                fb.grow_keep(*n + turn_n + k, *n + turn_n);
                for (uint64_t e = 0; e < k; ++e)
                    fb.p[*n + turn_n + e] = (uint32_t)((uint64_t)xy[2 * e + 1] * (uint64_t)W + (uint64_t)xy[2 * e]);
                turn_n += k;
            }
            counts[t] = turn_n;
            *n += turn_n;
            *done = t + 1;
        }
        return GOLHIP_OK;
    }
};

}  // namespace

void Run(Params p, Chan<Event> *events, Chan<char32_t> *keyPresses, const RunOptions &opt) {
    const int64_t W = p.ImageWidth, H = p.ImageHeight;
    if (W <= 0 || H <= 0 || W > INT32_MAX || H > INT32_MAX || p.Turns < 0) throw std::runtime_error("bad Params");
    const std::string name = std::to_string(W) + "x" + std::to_string(H);
    const bool quirks = opt.ref_quirks;

    // distributor.go:39-41 -> io.readPgmImage
    std::vector<uint8_t> raster = ReadPgm(opt.root + "/images/" + name + ".pgm", W, H);
    std::printf("File %s input done!\n", name.c_str());
    std::fflush(stdout);

    Engine board(W, H, opt);
    board.load(raster.data());

    auto send = [&](Event e) {
        if (events) events->send(std::move(e));
    };
    auto write_snapshot = [&](int64_t turn, bool transposed) -> std::string {
        std::vector<uint8_t> snap((size_t)W * H);
        board.snapshot(snap.data());
        if (transposed) {  // the reference streams (*world)[x][y] for s/q (distributor.go:234-238)
            std::vector<uint8_t> t((size_t)W * H);
            for (int64_t y = 0; y < H; ++y)
                for (int64_t x = 0; x < W; ++x) t[(size_t)x * H + y] = snap[(size_t)y * W + x];
            snap.swap(t);
        }
        const std::string fname = name + "x" + std::to_string(turn);
        mkdir((opt.root + "/out").c_str(), 0777);  // io.go:43 os.Mkdir("out")
        WritePgm(opt.root + "/out/" + fname + ".pgm", W, H, snap.data());
        std::printf("File %s output done!\n", fname.c_str());
        std::fflush(stdout);
        return fname;
    };

    // distributor.go:72-80: CellFlipped for every cell alive at load, turn 0.
    if (opt.cell_events && events)
        for (const util::Cell &c : board.cells(golhip_alive_cells, quirks)) {
            Event e;
            e.kind = EventKind::CellFlipped;
            e.CompletedTurns = 0;
            e.Cell = c;
            send(e);
        }

    std::mutex mu;                 // the reference's `mu`: held by the turn loop and by pause
    std::atomic<int> waiters{0};   // helpers queued for `mu` (std::mutex is not fair)
    std::atomic<int64_t> turn{0};  // completed turns
    // helpers take `mu` through this, so the turn loop can step aside for them
    auto lock_mu = [&]() {
        ++waiters;
        std::unique_lock<std::mutex> g(mu);
        --waiters;
        return g;
    };
    std::atomic<bool> finished{false}, quit{false};
    std::mutex tick_mu;
    std::condition_variable tick_cv;

    // ticker (distributor.go:283-302): (turn, count) read as one pair from the engine.
    std::exception_ptr helper_err;  // first exception raised on a helper thread
    std::mutex err_mu;
    auto guarded = [&](auto body) {
        return [&, body] {
            try {
                body();
            } catch (...) {
                std::lock_guard<std::mutex> g(err_mu);
                if (!helper_err) helper_err = std::current_exception();
                quit = true;
            }
        };
    };
    std::thread ticker(guarded([&] {
        const auto period = std::chrono::duration<double>(opt.ticker_seconds);
        for (;;) {
            {
                std::unique_lock<std::mutex> lk(tick_mu);
                if (tick_cv.wait_for(lk, period, [&] { return finished.load(); })) break;
            }
            uint64_t n = 0;
            int64_t at = 0;
            {
                auto g = lock_mu();  // blocked while paused, like the reference
                board.alive_count(&n, &at);
            }
            Event e;
            e.kind = EventKind::AliveCellsCount;
            e.CompletedTurns = at;
            e.CellsCount = (int64_t)n;
            send(e);
        }
    }));

    // keyPress (distributor.go:223-280); a nil channel simply never delivers.
    std::thread keys;
    if (keyPresses) keys = std::thread(guarded([&] {
        char32_t k;
        while (!finished.load()) {
            int r = keyPresses->try_recv(k);
            if (r < 0) break;
            if (r == 0) {
                std::this_thread::sleep_for(std::chrono::milliseconds(2));
                continue;
            }
            if (k == U's' || k == U'q') {
                std::string fname;
                int64_t t;
                {
                    auto g = lock_mu();  // snapshot at a turn boundary
                    t = turn.load();
                    fname = write_snapshot(t, quirks);
                }
                Event e;
                e.kind = EventKind::ImageOutputComplete;
                e.CompletedTurns = t;
                e.Filename = fname;
                send(e);
                if (k == U'q') {
                    quit = true;
                    break;
                }
            } else if (k == U'p') {
                auto g = lock_mu();
                std::printf("%lld\n", (long long)turn.load());
                std::fflush(stdout);
                if (!quirks) {
                    Event e;
                    e.kind = EventKind::StateChange;
                    e.CompletedTurns = turn.load();
                    e.NewState = State::Paused;
                    send(e);
                }
                char32_t k2 = 0;
                while (!finished.load()) {
                    int r2 = keyPresses->try_recv(k2);
                    if (r2 < 0) break;
                    if (r2 == 1 && k2 == U'p') break;
                    std::this_thread::sleep_for(std::chrono::milliseconds(2));
                }
                std::printf("Continuing\n");
                std::fflush(stdout);
                if (!quirks) {
                    Event e;
                    e.kind = EventKind::StateChange;
                    e.CompletedTurns = turn.load();
                    e.NewState = State::Executing;
                    send(e);
                }
            }
        }
    }));

    auto stop_helpers = [&] {
        {
            std::lock_guard<std::mutex> lk(tick_mu);
            finished = true;
        }
        tick_cv.notify_all();
        if (ticker.joinable()) ticker.join();
        if (keys.joinable()) keys.join();
        if (helper_err) std::rethrow_exception(helper_err);
    };

    try {
        // The turn loop in batches (distributor.go:93-173): each engine call
        // runs up to `batch` turns; with cell events it is the fused flip
        // stream (golhip_flip_stream: every turn's CellFlipped list, written
        // by the device straight into a page-locked buffer as cell indices),
        // otherwise fused step launches.  `mu` is held only for the call, so
        // the ticker, s/q snapshots and p (which takes `mu`, as the
        // reference's pause does) act between batches, at a turn boundary.
        const int64_t batch = opt.batch_turns > 0 ? opt.batch_turns : (opt.cell_events ? 64 : 256);
        FlipBuffer fb;
        if (opt.cell_events) fb.grow((uint64_t)std::min<int64_t>(W * H * std::min<int64_t>(batch, 4), 64ll << 20));
        std::vector<uint64_t> counts((size_t)batch);
        constexpr uint64_t kFlipChunk = 4096;
        std::vector<Event> flip_evs;
        int64_t t = 0;
        while (t < p.Turns && !quit.load()) {
            const int64_t want = std::min<int64_t>(batch, p.Turns - t);
            int64_t done = want;
            uint64_t n = 0;
            {
                std::lock_guard<std::mutex> g(mu);
                if (opt.cell_events) {
                    int rc = board.flip_stream(want, fb, counts.data(), &done, &n);
                    if (rc == GOLHIP_ERANGE) {  // one turn needs more than the buffer: grow, nothing advanced
                        fb.grow(n);
                        rc = board.flip_stream(want, fb, counts.data(), &done, &n);
                    }
                    check(rc);
                } else {
                    board.step(want);
                }
                t += done;
                turn = t;
            }
            // let a queued ticker / key handler take `mu` before the next batch
            while (waiters.load() > 0) std::this_thread::sleep_for(std::chrono::microseconds(20));
            const int64_t t0 = t - done;
            uint64_t off = 0;
            for (int64_t i = 0; i < done; ++i) {
                const int64_t completed = t0 + i + 1;  // quirks: the reference's 0-based turn (:113, :171, :216)
                if (opt.cell_events) {
                    // initializeAliveCells (:212-220): the turn's list, in order, sent in
                    // chunks (Chan::send_batch: one lock a chunk on a buffered channel)
                    const uint64_t n = counts[(size_t)i];
                    for (uint64_t e0 = off; e0 < off + n && events; e0 += kFlipChunk) {
                        const uint64_t m = std::min<uint64_t>(kFlipChunk, off + n - e0);
                        flip_evs.resize(m);
                        for (uint64_t j = 0; j < m; ++j) {
                            const uint64_t idx = fb.p[e0 + j];
                            Event &ev = flip_evs[j];
                            ev.kind = EventKind::CellFlipped;
                            ev.CompletedTurns = quirks ? completed - 1 : completed;
                            ev.Cell.X = quirks ? (int64_t)(idx / W) : (int64_t)(idx % W);
                            ev.Cell.Y = quirks ? (int64_t)(idx % W) : (int64_t)(idx / W);
                        }
                        events->send_batch(flip_evs.data(), m);
                    }
                    off += n;
                }
                if (opt.turn_events) {
                    Event ev;
                    ev.kind = EventKind::TurnComplete;
                    ev.CompletedTurns = quirks ? completed - 1 : completed;
                    send(ev);
                }
            }
        }
        stop_helpers();
        if (quit.load()) {
            // `q` (:244-261): snapshot already written; the reference os.Exit(0)s
            // without FinalTurnComplete.  The mirror ends the run instead.
            Event e;
            e.kind = EventKind::StateChange;
            e.CompletedTurns = turn.load();
            e.NewState = State::Quitting;
            send(e);
            if (events) events->close();
            return;
        }
        // distributor.go:180-206
        std::vector<util::Cell> alive = board.cells(golhip_alive_cells, false);
        const std::string fname = write_snapshot(p.Turns, false);
        Event io;
        io.kind = EventKind::ImageOutputComplete;
        io.CompletedTurns = p.Turns;
        io.Filename = fname;
        send(io);
        Event fin;
        fin.kind = EventKind::FinalTurnComplete;
        fin.CompletedTurns = p.Turns;
        fin.Alive = std::move(alive);
        send(fin);
        Event q;
        q.kind = EventKind::StateChange;
        q.CompletedTurns = p.Turns;
        q.NewState = State::Quitting;
        send(q);
        if (events) events->close();
    } catch (...) {
        stop_helpers();
        if (events) events->close();
        throw;
    }
}

}  // namespace gol

// ---------------------------------------------------------------------------
// C-ABI of the host mirror (include/golrun.h): lets non-C++ callers (the
// Python parity tests) drive gol::Run the way gol_test.go drives gol.Run.
// ---------------------------------------------------------------------------
struct golrun {
    gol::Chan<gol::Event> events;
    gol::Chan<char32_t> keys;
    bool use_keys;
    std::thread th;
    std::string err;
    std::atomic<bool> done{false};
    gol::Event current;
    golrun(size_t cap, bool k) : events(cap), keys(16), use_keys(k) {}
};

namespace {
thread_local std::string g_run_err;
int run_fail(const std::string &m) {
    g_run_err = m;
    return GOLHIP_EINVAL;
}
}  // namespace

extern "C" {

const char *golrun_last_error(void) { return g_run_err.c_str(); }

int golrun_start(int64_t turns, int64_t threads, int64_t width, int64_t height, const char *root, int32_t device,
                 uint32_t flags, int32_t events_cap, int32_t ticker_ms, golrun_t *out) {
    if (!out || !root || events_cap < 0) return run_fail("bad arguments");
    gol::Params p;
    p.Turns = turns;
    p.Threads = threads;
    p.ImageWidth = width;
    p.ImageHeight = height;
    gol::RunOptions o;
    o.root = root;
    o.device = device;
    o.ref_quirks = (flags & GOLRUN_FLAG_REF_QUIRKS) != 0;
    o.cell_events = (flags & GOLRUN_FLAG_NO_CELL_EVENTS) == 0;
    o.turn_events = (flags & GOLRUN_FLAG_NO_TURN_EVENTS) == 0;
    if (ticker_ms > 0) o.ticker_seconds = ticker_ms / 1000.0;
    golrun *r = new golrun((size_t)events_cap, (flags & GOLRUN_FLAG_KEYS) != 0);
    r->th = std::thread([r, p, o] {
        try {
            gol::Run(p, &r->events, r->use_keys ? &r->keys : nullptr, o);
        } catch (const std::exception &e) {
            r->err = e.what();
            r->events.close();
        }
        r->done = true;
    });
    *out = r;
    return GOLHIP_OK;
}

int golrun_next_event(golrun_t r, golrun_event_t *ev, int32_t timeout_ms) {
    if (!r || !ev) return run_fail("bad arguments");
    const auto t_end = std::chrono::steady_clock::now() + std::chrono::milliseconds(timeout_ms < 0 ? 0 : timeout_ms);
    for (;;) {
        int got = r->events.try_recv(r->current);
        if (got == 1) break;
        if (got < 0) return 0;  // closed and drained: the `range events` loop ends
        if (timeout_ms >= 0 && std::chrono::steady_clock::now() >= t_end) return 2;
        std::this_thread::sleep_for(std::chrono::microseconds(50));
    }
    const gol::Event &e = r->current;
    memset(ev, 0, sizeof *ev);
    ev->kind = (int32_t)e.kind;
    ev->completed_turns = e.CompletedTurns;
    ev->cells_count = e.CellsCount;
    ev->new_state = (int32_t)e.NewState;
    ev->cell_x = e.Cell.X;
    ev->cell_y = e.Cell.Y;
    ev->alive_len = (int64_t)e.Alive.size();
    std::snprintf(ev->filename, sizeof ev->filename, "%s", e.Filename.c_str());
    std::snprintf(ev->text, sizeof ev->text, "%s", e.String().c_str());
    return 1;
}

int golrun_event_string(const golrun_event_t *ev, char *out, uint64_t cap) {
    if (!ev || !out || cap == 0) return run_fail("bad arguments");
    gol::Event e;
    e.kind = (gol::EventKind)ev->kind;
    e.CompletedTurns = ev->completed_turns;
    e.CellsCount = ev->cells_count;
    e.NewState = (gol::State)ev->new_state;
    e.Filename = std::string(ev->filename, strnlen(ev->filename, sizeof ev->filename));
    std::snprintf(out, cap, "%s", e.String().c_str());
    return GOLHIP_OK;
}

int golrun_event_cells(golrun_t r, int64_t *xy, uint64_t cap) {
    if (!r) return run_fail("bad arguments");
    const auto &a = r->current.Alive;
    if (cap < a.size() || (!xy && !a.empty())) return run_fail("buffer too small");
    for (size_t i = 0; i < a.size(); ++i) {
        xy[2 * i] = a[i].X;
        xy[2 * i + 1] = a[i].Y;
    }
    return GOLHIP_OK;
}

int golrun_drain(golrun_t r, golrun_drain_stats_t *st, uint64_t *flips, uint64_t *digests, int64_t turns_cap,
                 int64_t width) {
    if (!r || !st || turns_cap < 0 || ((flips || digests) && width <= 0)) return run_fail("bad arguments");
    memset(st, 0, sizeof *st);
    for (int64_t t = 0; t < turns_cap; ++t) {
        if (flips) flips[t] = 0;
        if (digests) digests[t] = 0;
    }
    auto mix = [](uint64_t x) {
        uint64_t z = x + 0x9E3779B97F4A7C15ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        return z ^ (z >> 31);
    };
    std::vector<gol::Event> batch;
    batch.reserve(1024);
    while (r->events.recv_batch(batch, 1024)) {  // main.go:59-66, until close (every event, in order)
        for (const gol::Event &e : batch) {
            const int k = (int)e.kind;
            if (k >= 0 && k < 6) st->count[k]++;
            if (e.kind == gol::EventKind::TurnComplete) st->last_turn = e.CompletedTurns;
            if (e.kind == gol::EventKind::FinalTurnComplete) st->final_alive = (int64_t)e.Alive.size();
            if (e.kind != gol::EventKind::CellFlipped || e.CompletedTurns < 1 || e.CompletedTurns > turns_cap)
                continue;
            const int64_t t = e.CompletedTurns - 1;
            const uint64_t i = flips ? ++flips[t] : 0;
            if (digests) digests[t] += mix(i) * ((uint64_t)e.Cell.Y * (uint64_t)width + (uint64_t)e.Cell.X + 1);
        }
    }
    return GOLHIP_OK;
}

int golrun_send_key(golrun_t r, uint32_t key) {
    if (!r || !r->use_keys) return run_fail("run has no key channel");
    return r->keys.send((char32_t)key) ? GOLHIP_OK : run_fail("key channel closed");
}

int golrun_wait(golrun_t r, char *err, uint64_t err_cap) {
    if (!r) return run_fail("bad arguments");
    // drain whatever the caller left unread so the run can finish
    gol::Event tmp;
    while (!r->done.load()) {
        if (r->events.try_recv(tmp) == 0) std::this_thread::sleep_for(std::chrono::microseconds(200));
    }
    if (r->th.joinable()) r->th.join();
    if (err && err_cap) std::snprintf(err, err_cap, "%s", r->err.c_str());
    return r->err.empty() ? GOLHIP_OK : GOLHIP_EINVAL;
}

int golrun_destroy(golrun_t r) {
    if (!r) return GOLHIP_OK;
    golrun_wait(r, nullptr, 0);
    delete r;
    return GOLHIP_OK;
}

}  // extern "C"
