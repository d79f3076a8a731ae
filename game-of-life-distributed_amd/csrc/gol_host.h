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

#include <algorithm>
#include <atomic>
#include <chrono>
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
// Go hands a value between goroutines in ~100-200 ns; a mutex + condition
// variable per event costs two thread wake-ups (~5 us), which made a 512^2
// x 100 run's 380k CellFlipped events take ~1 s.  So both sides spin briefly
// on atomics (a waiting receiver is usually on another core) before they
// sleep, and a side notifies the other only when it is asleep.
template <typename T>
class Chan {
   public:
    explicit Chan(size_t cap = 0) : cap_(cap) {}
    // Returns false if the channel is closed (Go would panic).
    bool send(T v) {
        if (cap_ == 0) return send0(std::move(v));
        std::unique_lock<std::mutex> lk(mu_);
        const size_t room = std::max<size_t>(cap_, 1);
        if (!closed_ && q_.size() >= room) {
            lk.unlock();
            spin([&] { return closed_a_.load(std::memory_order_acquire) ||
                              sent_a_.load(std::memory_order_acquire) -
                                      received_a_.load(std::memory_order_acquire) < room; });
            lk.lock();
            ++send_sleepers_;
            send_cv_.wait(lk, [&] { return closed_ || q_.size() < room; });
            --send_sleepers_;
        }
        if (closed_) return false;
        q_.push_back(std::move(v));
        ++sent_;
        sent_a_.store(sent_, std::memory_order_release);
        if (recv_sleepers_) recv_cv_.notify_one();
        return true;
    }
    // Sends v[0..n) in order, as n sends would (false if the channel closed on
    // the way).  A buffered channel takes them in chunks of its free room
    // under one lock and one wake-up each, so a turn's CellFlipped list
    // does not pay a lock round trip per event; an unbuffered one keeps
    // the rendezvous per value.  Other senders may interleave between
    // chunks, as between any two Go sends.
    bool send_batch(T *v, size_t n) {
        if (cap_ == 0) {
            for (size_t i = 0; i < n; ++i)
                if (!send(std::move(v[i]))) return false;
            return true;
        }
        size_t i = 0;
        while (i < n) {
            std::unique_lock<std::mutex> lk(mu_);
            if (!closed_ && q_.size() >= cap_) {
                lk.unlock();
                spin([&] { return closed_a_.load(std::memory_order_acquire) ||
                                  sent_a_.load(std::memory_order_acquire) -
                                          received_a_.load(std::memory_order_acquire) < cap_; });
                lk.lock();
                ++send_sleepers_;
                send_cv_.wait(lk, [&] { return closed_ || q_.size() < cap_; });
                --send_sleepers_;
            }
            if (closed_) return false;
            const size_t k = std::min(n - i, cap_ - q_.size());
            for (size_t j = 0; j < k; ++j) q_.push_back(std::move(v[i + j]));
            i += k;
            sent_ += k;
            sent_a_.store(sent_, std::memory_order_release);
            // k values queued: wake every sleeping receiver when more than one
            // can take something (Go channels allow several consumers)
            if (recv_sleepers_) {
                if (k > 1) recv_cv_.notify_all();
                else recv_cv_.notify_one();
            }
        }
        return true;
    }
    // Blocks; false once closed and drained (a `range` loop ends).
    bool recv(T &out) {
        if (cap_ == 0) return recv0(out);
        spin([&] { return closed_a_.load(std::memory_order_acquire) ||
                          sent_a_.load(std::memory_order_acquire) != received_a_.load(std::memory_order_acquire); });
        std::unique_lock<std::mutex> lk(mu_);
        if (!closed_ && q_.empty()) {
            ++recv_sleepers_;
            recv_cv_.wait(lk, [&] { return closed_ || !q_.empty(); });
            --recv_sleepers_;
        }
        if (q_.empty()) return false;
        take(out);
        return true;
    }
    // Blocks for the first value like recv, then takes every value already
    // queued too (at most `max`), in order: one lock per batch for a
    // consumer of a buffered channel (main.go's capacity-1000 events
    // channel).  Returns the count; 0 once closed and drained.
    size_t recv_batch(std::vector<T> &out, size_t max) {
        out.clear();
        if (cap_ == 0) {  // at most the one value a sender offers
            T v;
            if (max == 0 || !recv0(v)) return 0;
            out.push_back(std::move(v));
            return 1;
        }
        spin([&] { return closed_a_.load(std::memory_order_acquire) ||
                          sent_a_.load(std::memory_order_acquire) != received_a_.load(std::memory_order_acquire); });
        std::unique_lock<std::mutex> lk(mu_);
        if (!closed_ && q_.empty()) {
            ++recv_sleepers_;
            recv_cv_.wait(lk, [&] { return closed_ || !q_.empty(); });
            --recv_sleepers_;
        }
        while (!q_.empty() && out.size() < max) {
            out.push_back(std::move(q_.front()));
            q_.pop_front();
        }
        received_ += out.size();
        received_a_.store(received_, std::memory_order_release);
        if (send_sleepers_ && !out.empty()) send_cv_.notify_all();
        return out.size();
    }
    // Non-blocking receive: 1 = got one, 0 = empty, -1 = closed and drained.
    int try_recv(T &out) {
        if (cap_ == 0) {
            // a receiver blocked in recv0 holds recv_mu_ for its whole wait: then
            // the offer (if any) is that receiver's, and this call must not
            // block.  Any other holder (a concurrent try_recv) holds it for a
            // few instructions: retry rather than report "empty" while a sender
            // may be parked with a value (Go's select-with-default fails only
            // when no sender is ready).
            std::unique_lock<std::mutex> rg(recv_mu_, std::defer_lock);
            for (int i = 0; !rg.try_lock(); ++i) {
                if (recv_waiting_.load(std::memory_order_acquire) > 0 || i == 4096)
                    return closed_a_.load(std::memory_order_acquire) ? -1 : 0;
                __builtin_ia32_pause();
            }
            const uint64_t q = box_.seq.load(std::memory_order_acquire);
            if (q & 1) {
                out = std::move(box_.value);
                box_.seq.store(q + 1, std::memory_order_release);
                wake(send_sleepers0_, send_cv_);
                return 1;
            }
            return closed_a_.load(std::memory_order_acquire) ? -1 : 0;
        }
        std::lock_guard<std::mutex> lk(mu_);
        if (q_.empty()) return closed_ ? -1 : 0;
        take(out);
        return 1;
    }
    void close() {
        std::lock_guard<std::mutex> lk(mu_);
        closed_ = true;
        closed_a_.store(true, std::memory_order_release);
        send_cv_.notify_all();
        recv_cv_.notify_all();
    }
    bool closed() {
        std::lock_guard<std::mutex> lk(mu_);
        return closed_;
    }

   private:
    // ---- capacity 0: the rendezvous.  One slot and a sequence word (odd =
    // a value waits in the slot); senders queue on send_mu_, receivers on
    // recv_mu_, so a hand-off between one sender and one receiver moves only
    // the slot's and the sequence word's cache lines (~1.5 us a value with a
    // shared mutex and counters before).  A side that waits past the spin
    // sleeps on mu_'s condition variables (wait0 / wake).
    bool send0(T v) {
        std::lock_guard<std::mutex> sg(send_mu_);
        if (closed_a_.load(std::memory_order_acquire)) return false;
        const uint64_t q = box_.seq.load(std::memory_order_relaxed);  // even: the previous value was taken
        box_.value = std::move(v);
        box_.seq.store(q + 1, std::memory_order_release);
        wake(recv_sleepers0_, recv_cv_);
        // Go: the send completes when a receiver has the value
        wait0([&] { return box_.seq.load(std::memory_order_acquire) != q + 1 || closed_a_.load(std::memory_order_acquire); },
              send_sleepers0_, send_cv_);
        return true;
    }
    bool recv0(T &out) {
        std::lock_guard<std::mutex> rg(recv_mu_);
        recv_waiting_.fetch_add(1, std::memory_order_release);  // (try_recv: this receiver owns the next offer)
        wait0([&] { return (box_.seq.load(std::memory_order_acquire) & 1) || closed_a_.load(std::memory_order_acquire); },
              recv_sleepers0_, recv_cv_);
        recv_waiting_.fetch_sub(1, std::memory_order_release);
        const uint64_t q = box_.seq.load(std::memory_order_acquire);
        if (!(q & 1)) return false;  // closed, nothing offered
        out = std::move(box_.value);
        box_.seq.store(q + 1, std::memory_order_release);
        wake(send_sleepers0_, send_cv_);
        return true;
    }
    // Sleep until `ready` (after the spin).  With wake(): the sleeper counts
    // itself, then re-checks; the waker publishes, then reads the count (both
    // behind seq_cst fences), so one of them sees the other's write, and a
    // waker that sees a sleeper takes mu_ first, so the notify cannot fall
    // between the sleeper's check and its wait.
    template <typename F>
    void wait0(F &&ready, std::atomic<int> &sleepers, std::condition_variable &cv) {
        if (spin(ready)) return;
        std::unique_lock<std::mutex> lk(mu_);
        sleepers.fetch_add(1, std::memory_order_relaxed);
        std::atomic_thread_fence(std::memory_order_seq_cst);
        while (!ready()) cv.wait(lk);
        sleepers.fetch_sub(1, std::memory_order_relaxed);
    }
    void wake(std::atomic<int> &sleepers, std::condition_variable &cv) {
        std::atomic_thread_fence(std::memory_order_seq_cst);
        if (sleepers.load(std::memory_order_relaxed) > 0) {
            { std::lock_guard<std::mutex> lk(mu_); }
            cv.notify_all();
        }
    }
    // Spin up to ~100 us for `ready` (a partner thread that is running answers
    // well within that; sleeping and being woken costs ~10 us a side); true
    // if it became true meanwhile.
    template <typename F>
    static bool spin(F &&ready) {
        const auto t0 = std::chrono::steady_clock::now();
        for (int i = 0;; ++i) {
            if (ready()) return true;
            __builtin_ia32_pause();
            if ((i & 255) == 255 && std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(100))
                return ready();
        }
    }
    void take(T &out) {  // mu_ held, q_ not empty
        out = std::move(q_.front());
        q_.pop_front();
        ++received_;
        received_a_.store(received_, std::memory_order_release);
        if (send_sleepers_) send_cv_.notify_all();  // senders wait on different tickets
    }
    size_t cap_;
    std::mutex mu_;
    std::condition_variable send_cv_, recv_cv_;
    std::deque<T> q_;
    bool closed_ = false;
    uint64_t sent_ = 0, received_ = 0;
    int send_sleepers_ = 0, recv_sleepers_ = 0;
    // Each spun-on word on a line of its own: the sender writes sent_a_, the
    // receiver received_a_, and neither should bounce the mutex's line.
    alignas(64) std::atomic<uint64_t> sent_a_{0};
    alignas(64) std::atomic<uint64_t> received_a_{0};
    alignas(64) std::atomic<bool> closed_a_{false};
    // capacity 0 (send0 / recv0): the sequence word shares a cache line with
    // the start of the slot, so a hand-off moves the slot's lines and no other
    alignas(64) std::mutex send_mu_;
    alignas(64) std::mutex recv_mu_;
    struct alignas(64) Slot {
        std::atomic<uint64_t> seq{0};
        T value{};
    } box_;
    alignas(64) std::atomic<int> send_sleepers0_{0};
    alignas(64) std::atomic<int> recv_sleepers0_{0};
    std::atomic<int> recv_waiting_{0};     // receivers inside recv0 (they own the next offer)
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
