// gol_host.h — C++ mirror of the reference's host API, package gol
// (gol/gol.go, gol/event.go, gol/io.go, util/cell.go), running the turn loop
// on libgolhip.so instead of the goroutine worker pool.
//
// Same names and argument meaning as the Go API:
//   gol::Params{Turns, Threads, ImageWidth, ImageHeight}      gol.go:4-9
//   gol::Run(Params, events, keyPresses)                       gol.go:12
//   gol::Event (AliveCellsCount, ImageOutputComplete, StateChange,
//              CellFlipped, TurnComplete, FinalTurnComplete)  event.go:19-68
//   String() / GetCompletedTurns()                             event.go:72-131
//   util::Cell{X, Y}                                           util/cell.go:4-6
// Channels follow Go semantics (capacity 0 = rendezvous, close + drain).
// Input:  <root>/images/<W>x<H>.pgm   Output: <root>/out/<W>x<H>x<T>.pgm (io.go:48, :95)
#pragma once

#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <vector>

// Go's int is 64-bit (gol.go:4-9, event.go:19-68, util/cell.go:4-6): every
// integer of the mirror's API is int64_t, so a 262144^2 board's ~6.5e9 alive
// cells and the CLI's 10^10 default turns (main.go:37-41) pass through intact.
namespace util {
struct Cell {
    int64_t X = 0, Y = 0;
    bool operator==(const Cell &o) const { return X == o.X && Y == o.Y; }
};
}  // namespace util

namespace gol {

struct Params {
    int64_t Turns = 0;
    int64_t Threads = 1;  // accepted for API parity; the GPU engine ignores it
    int64_t ImageWidth = 0;
    int64_t ImageHeight = 0;
};

enum class State { Paused = 0, Executing = 1, Quitting = 2 };
std::string StateString(State s);

enum class EventKind {
    AliveCellsCount = 0,
    ImageOutputComplete = 1,
    StateChange = 2,
    CellFlipped = 3,
    TurnComplete = 4,
    FinalTurnComplete = 5,
};

// One tagged struct for the six event types; unused fields stay default.
struct Event {
    EventKind kind = EventKind::TurnComplete;
    int64_t CompletedTurns = 0;
    int64_t CellsCount = 0;           // AliveCellsCount
    std::string Filename;             // ImageOutputComplete
    State NewState = State::Executing;  // StateChange
    util::Cell Cell;                  // CellFlipped
    std::vector<util::Cell> Alive;    // FinalTurnComplete
    std::string String() const;       // event.go:72-131 text
    int64_t GetCompletedTurns() const { return CompletedTurns; }
};

// Go channel: capacity 0 is a rendezvous (send returns once received).
template <typename T>
class Chan {
   public:
    explicit Chan(size_t cap = 0) : cap_(cap) {}
    // Returns false if the channel is closed (Go would panic).
    bool send(T v) {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return closed_ || q_.size() < std::max<size_t>(cap_, 1); });
        if (closed_) return false;
        q_.push_back(std::move(v));
        const uint64_t ticket = ++sent_;
        cv_.notify_all();
        if (cap_ == 0) cv_.wait(lk, [&] { return received_ >= ticket || closed_; });
        return true;
    }
    // Blocks; false once closed and drained (a `range` loop ends).
    bool recv(T &out) {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return closed_ || !q_.empty(); });
        if (q_.empty()) return false;
        out = std::move(q_.front());
        q_.pop_front();
        ++received_;
        cv_.notify_all();
        return true;
    }
    // Non-blocking receive: 1 = got one, 0 = empty, -1 = closed and drained.
    int try_recv(T &out) {
        std::lock_guard<std::mutex> lk(mu_);
        if (q_.empty()) return closed_ ? -1 : 0;
        out = std::move(q_.front());
        q_.pop_front();
        ++received_;
        cv_.notify_all();
        return 1;
    }
    void close() {
        std::lock_guard<std::mutex> lk(mu_);
        closed_ = true;
        cv_.notify_all();
    }
    bool closed() {
        std::lock_guard<std::mutex> lk(mu_);
        return closed_;
    }

   private:
    size_t cap_;
    std::mutex mu_;
    std::condition_variable cv_;
    std::deque<T> q_;
    bool closed_ = false;
    uint64_t sent_ = 0, received_ = 0;
};

// Host-mirror options beyond the Go API (all default to the reference's
// documented contract; see DESIGN.md "Quirks").
struct RunOptions {
    std::string root = ".";       // directory holding images/ and out/
    int device = 0;               // HIP device
    bool ref_quirks = false;      // reproduce the reference's quirks (0-based TurnComplete,
                                  // transposed CellFlipped, transposed s/q snapshots, no Final on q)
    bool cell_events = true;      // per-cell CellFlipped events (the SDL feed)
    bool turn_events = true;      // TurnComplete every turn
    double ticker_seconds = 2.0;  // AliveCellsCount period (distributor.go:285)
    int64_t batch_turns = 0;      // turns per engine call (0: 64 with cell events, 256 without);
                                  // keys, pause and the ticker are served between calls
    // Row-strip decomposition (README halo extension):
    // ngpu > 1 splits the board into row strips on devices 0..ngpu-1, stepped
    // together with peer-copied halos (golhip_group_step_ex); strips > 1 sets
    // the strip count (round-robin over the devices; tests run 2 or 3 strips
    // on device 0).  -1: from the environment, GOL_NGPU / GOL_STRIPS (unset: 1).
    int ngpu = -1;
    int strips = -1;
};

// The PGM goroutine's file formats (io.go:42-126).
std::vector<uint8_t> ReadPgm(const std::string &path, int64_t width, int64_t height);
void WritePgm(const std::string &path, int64_t width, int64_t height, const uint8_t *raster);

// gol.Run: blocks until the run finishes (events closed) or `q` stops it.
// Throws std::runtime_error where the reference panics / log.Fatal-s.
void Run(Params p, Chan<Event> *events, Chan<char32_t> *keyPresses, const RunOptions &opt = RunOptions());

}  // namespace gol
