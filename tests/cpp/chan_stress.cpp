// Stress test of gol::Chan (gol_host.h): Go channel semantics under
// contention -- every value delivered exactly once and in per-sender order,
// an unbuffered send returns only after its value was received, close ends
// a range loop once drained.  Built and run by tests/test_chan_cpu.py.
#include <chrono>
#include <cstdio>
#include <thread>
#include <algorithm>
#include <atomic>
#include <vector>

#include "gol_host.h"

static int run(size_t cap, int senders, int per_sender) {
    gol::Chan<int64_t> ch(cap);
    std::atomic<int64_t> received_count{0};
    std::vector<std::thread> ts;
    std::atomic<int> order_errors{0};
    for (int s = 0; s < senders; ++s)
        ts.emplace_back([&, s] {
            std::vector<int64_t> buf;
            for (int i = 0; i < per_sender;) {
                if ((i / 16) % 2 == 0) {  // single sends and send_batch runs of 1..13 alternate
                    if (!ch.send((int64_t)s << 32 | i)) order_errors++;
                    // rendezvous: the receiver has taken this value before send returned
                    if (cap == 0 && received_count.load() < 0) order_errors++;
                    ++i;
                } else {
                    const int k = std::min(per_sender - i, 1 + (i * 7 + s) % 13);
                    buf.clear();
                    for (int j = 0; j < k; ++j) buf.push_back((int64_t)s << 32 | (i + j));
                    if (!ch.send_batch(buf.data(), buf.size())) order_errors++;
                    i += k;
                }
            }
        });
    std::vector<int> next(senders, 0);
    std::thread closer([&] {
        for (auto &t : ts) t.join();
        ch.close();
    });
    int64_t v, n = 0;
    std::vector<int64_t> batch;
    auto take = [&](int64_t v) {
        const int s = (int)(v >> 32), i = (int)(v & 0xffffffff);
        if (s < 0 || s >= senders || next[s] != i) order_errors++;
        else next[s]++;
        received_count++;
        n++;
    };
    for (bool more = true; more;) {  // alternate single and batched receives
        if (n % 2 == 0) {
            more = ch.recv(v);
            if (more) take(v);
        } else {
            more = ch.recv_batch(batch, 5) > 0;
            for (int64_t x : batch) take(x);
        }
    }
    closer.join();
    if (n != (int64_t)senders * per_sender || order_errors.load()) {
        std::printf("FAIL cap=%zu senders=%d got %lld errors %d\n", cap, senders, (long long)n, order_errors.load());
        return 1;
    }
    if (ch.send(1)) {
        std::printf("FAIL send after close succeeded\n");
        return 1;
    }
    return 0;
}

int main() {
    int rc = 0;
    for (size_t cap : {0, 1, 7, 1000})
        for (int senders : {1, 3})
            rc |= run(cap, senders, 20000);
    // unbuffered rendezvous: send blocks until the (late) receiver takes the value
    gol::Chan<int> ch(0);
    std::thread r([&] {
        std::this_thread::sleep_for(std::chrono::milliseconds(50));
        int v;
        ch.recv(v);
    });
    const auto t0 = std::chrono::steady_clock::now();
    ch.send(7);
    const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    r.join();
    if (ms < 40) {
        std::printf("FAIL unbuffered send returned after %.1f ms, before the receiver\n", ms);
        rc = 1;
    }
    // try_recv never blocks, even beside a receiver blocked in recv on an
    // unbuffered channel (golrun_next_event's timeout and golrun_wait rely on it)
    {
        gol::Chan<int> c0(0);
        std::atomic<int> got{0};
        std::thread blocked([&] {
            int v;
            if (c0.recv(v)) got++;
        });
        std::this_thread::sleep_for(std::chrono::milliseconds(20));  // past the spin: asleep in recv0
        const auto t1 = std::chrono::steady_clock::now();
        int v, tries = 0;
        for (; tries < 1000; ++tries)
            if (c0.try_recv(v) == 1) got++;
        const double tms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t1).count();
        std::thread s2([&] { c0.send(1); c0.send(2); });
        while (got.load() < 2) {
            if (c0.try_recv(v) == 1) got++;
            std::this_thread::yield();
        }
        s2.join();
        blocked.join();
        if (tms > 500) {
            std::printf("FAIL 1000 try_recv beside a blocked recv took %.1f ms\n", tms);
            rc = 1;
        }
    }
    // send_batch of k > 1 values wakes every sleeping receiver that can take one
    {
        gol::Chan<int> cb(8);
        std::atomic<int> got{0};
        std::vector<std::thread> rs;
        for (int i = 0; i < 2; ++i)
            rs.emplace_back([&] {
                int v;
                if (cb.recv(v)) got++;
            });
        std::this_thread::sleep_for(std::chrono::milliseconds(20));  // both asleep on the condition variable
        int two[2] = {1, 2};
        cb.send_batch(two, 2);
        const auto t2 = std::chrono::steady_clock::now();
        while (got.load() < 2 && std::chrono::steady_clock::now() - t2 < std::chrono::seconds(1))
            std::this_thread::sleep_for(std::chrono::milliseconds(1));
        if (got.load() < 2) {
            std::printf("FAIL a batch of 2 woke %d of 2 sleeping receivers\n", got.load());
            rc = 1;
            cb.close();
        }
        for (auto &t : rs) t.join();
    }
    // try_recv pollers contending on an unbuffered channel (no blocked recv):
    // a poller that finds recv_mu_ held by the other poller retries instead of
    // reporting "empty" (ADVICE r5), every value arrives exactly once
    {
        gol::Chan<int64_t> cp(0);
        const int N = 20000;
        std::atomic<int64_t> sum{0}, cnt{0};
        std::thread snd([&] {
            for (int i = 1; i <= N; ++i) cp.send(i);
        });
        std::vector<std::thread> polls;
        for (int k = 0; k < 2; ++k)
            polls.emplace_back([&] {
                int64_t v;
                while (cnt.load() < N)
                    if (cp.try_recv(v) == 1) {
                        sum += v;
                        cnt++;
                    }
            });
        snd.join();
        for (auto &t : polls) t.join();
        if (cnt.load() != N || sum.load() != (int64_t)N * (N + 1) / 2) {
            std::printf("FAIL two try_recv pollers got %lld values, sum %lld\n", (long long)cnt.load(),
                        (long long)sum.load());
            rc = 1;
        }
    }
    std::printf(rc ? "chan stress FAILED\n" : "chan stress ok\n");
    return rc;
}
