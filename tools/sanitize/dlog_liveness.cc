// tools/sanitize/dlog_liveness.cc -- deterministic liveness test of the
// durable log's segment-switch protocol (consus_amd/csrc/durable_log.cc).
//
// An appender whose reservation fails (the active segment is sealed or full)
// waits for the flush thread to switch segments.  Round 3 waited for
// "m_active != seg", which two switches (seg -> other -> seg) satisfy and then
// undo before the appender looks: the appender then waits for a switch that
// never comes, because the flush thread sleeps on the empty active segment
// (Weak 1: the driver's dlog bench hung 60 s in append()).
//
// This program parks one appender P at the log's test hook points and drives
// the flush thread through both interleavings:
//
//   sealed: P reads segment A, parks (point 0); X is appended to A, which is
//           sealed and flushed (switch A -> B); P resumes, finds A sealed and
//           parks again (point 1); Y is appended to B and flushed
//           (switch B -> A); P resumes: it must append into A.
//   full:   the flush thread is held inside its batch CRC for segment A while
//           two frames fill B exactly; P (parked at point 0 on B) resumes and
//           finds B full (point 1); the flush thread is released, seals and
//           switches B -> A; Y goes to A and is flushed (A -> B); P resumes:
//           it must append into B.
//
// P must return within 10 s.  If it does not, the program prints the log's
// debug_state, rescues P with one more append (which forces a switch) and
// exits 1 -- so the test never hangs.  Every other wait is bounded too (exit 3).
// Reference: txman/durable_log.cc:195-213 (append never waits for a switch).
#include <errno.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <memory>
#include <mutex>
#include <string>
#include <thread>

#include "txman/durable_log.h"

namespace {

using clk = std::chrono::steady_clock;

uint32_t bitwise_crc(const unsigned char* p, size_t n)
{
    uint32_t s = ~0u;
    for (size_t i = 0; i < n; ++i)
    {
        s ^= p[i];
        for (int k = 0; k < 8; ++k) s = (s >> 1) ^ (0x82F63B78u & (0u - (s & 1u)));
    }
    return ~s;
}

// A batch engine the test can hold shut (the flush thread then stays inside
// its checksum of the sealed segment).
struct Gate
{
    std::mutex mu;
    std::condition_variable cv;
    bool open = true;
    int inside = 0;  // flush calls waiting at the gate
};

int gated_crc(void* ctx, const void* base, const uint64_t* off, const uint32_t* len, size_t n,
              uint64_t, uint32_t* out)
{
    auto* g = static_cast<Gate*>(ctx);
    {
        std::unique_lock<std::mutex> hold(g->mu);
        ++g->inside;
        g->cv.notify_all();
        g->cv.wait(hold, [&] { return g->open; });
        --g->inside;
    }
    for (size_t i = 0; i < n; ++i)
        out[i] = bitwise_crc(static_cast<const unsigned char*>(base) + off[i], len[i]);
    return 0;
}

// Parks the thread `who` at hook point 0 and/or 1, once each.
struct Park
{
    std::mutex mu;
    std::condition_variable cv;
    std::thread::id who;
    bool armed[2] = {true, true};
    bool parked[2] = {false, false};
    bool release[2] = {false, false};
};

void hook(void* ctx, int point)
{
    auto* p = static_cast<Park*>(ctx);
    std::unique_lock<std::mutex> hold(p->mu);
    if (std::this_thread::get_id() != p->who || point < 0 || point > 1 || !p->armed[point]) return;
    p->armed[point] = false;
    p->parked[point] = true;
    p->cv.notify_all();
    p->cv.wait(hold, [&] { return p->release[point]; });
}

// Bounded waits poll instead of condition_variable::wait_until: libstdc++
// implements that with pthread_cond_clockwait, which this image's
// ThreadSanitizer does not intercept (it then reports the waiter's mutex as
// locked twice).
template <typename Pred>
bool poll_until(std::unique_lock<std::mutex>& hold, Pred pred)
{
    const auto until = clk::now() + std::chrono::seconds(10);
    while (!pred())
    {
        if (clk::now() > until) return false;
        hold.unlock();
        usleep(500);
        hold.lock();
    }
    return true;
}

template <typename Pred>
void must(std::unique_lock<std::mutex>& hold, std::condition_variable&, Pred pred,
          consus::durable_log& log, const char* what)
{
    if (!poll_until(hold, pred))
    {
        char st[512];
        log.debug_state(st, sizeof st);
        fprintf(stderr, "liveness: timed out waiting for %s\n  state: %s\n", what, st);
        fflush(stderr);
        _exit(3);
    }
}

void wait_durable(consus::durable_log& log, int64_t recno, const char* what)
{
    const auto until = clk::now() + std::chrono::seconds(10);
    while (log.durable() <= recno)
    {
        if (log.error() != 0 || clk::now() > until)
        {
            char st[512];
            log.debug_state(st, sizeof st);
            fprintf(stderr, "liveness: %s not durable (error %d)\n  state: %s\n", what,
                    log.error(), st);
            fflush(stderr);
            _exit(3);
        }
        usleep(200);
    }
}

// One scenario's state (on the heap, so each scenario's mutexes are fresh
// objects to ThreadSanitizer).
struct State
{
    explicit State(size_t cap) : log(cap) {}
    consus::durable_log log;
    Gate gate;
    Park park;
};

// Runs one scenario; returns 0 if P's append returned in time.
int scenario(const std::string& dir, bool full)
{
    const size_t cap = 4096;
    std::unique_ptr<State> state(new State(cap));
    consus::durable_log& log = state->log;
    Gate& gate = state->gate;
    Park& park = state->park;
    log.set_batch_crc_for_testing(gated_crc, &gate);
    log.set_append_hook_for_testing(hook, &park);
    if (!log.open(dir))
    {
        fprintf(stderr, "liveness: open %s: %s\n", dir.c_str(), strerror(errno));
        return 2;
    }
    const std::string small(40, 'x');
    const std::string half(cap / 2 - 20, 'h');  // a frame of exactly cap / 2 bytes
    std::atomic<int64_t> p_rec{0};
    std::atomic<bool> p_done{false};
    std::mutex done_mu;
    int64_t last = 0;

    if (full)
    {
        std::unique_lock<std::mutex> g(gate.mu);
        gate.open = false;
    }
    if (full)
    {
        // segment A: one frame; the flush thread seals it, switches to B and
        // stops inside the batch CRC of A
        last = log.append(small.data(), small.size());
        std::unique_lock<std::mutex> g(gate.mu);
        must(g, gate.cv, [&] { return gate.inside == 1; }, log, "flush thread at the gate");
    }
    std::thread p([&] {
        {
            std::lock_guard<std::mutex> hold(park.mu);
            park.who = std::this_thread::get_id();
        }
        const int64_t r = log.append("parked appender", 15);
        p_rec.store(r);
        std::lock_guard<std::mutex> hold(done_mu);
        p_done.store(true);
    });
    {
        std::unique_lock<std::mutex> hold(park.mu);
        must(hold, park.cv, [&] { return park.parked[0]; }, log, "P at point 0");
    }
    if (!full)
    {
        // P holds segment A.  X into A: sealed, flushed, switch A -> B.
        last = log.append(small.data(), small.size());
        wait_durable(log, last, "X");
    }
    else
    {
        // P holds segment B.  Fill B exactly with two cap/2 frames.
        log.append(half.data(), half.size());
        last = log.append(half.data(), half.size());
    }
    {
        std::unique_lock<std::mutex> hold(park.mu);
        park.release[0] = true;
        park.cv.notify_all();
        must(hold, park.cv, [&] { return park.parked[1]; }, log, "P at point 1 (reservation failed)");
    }
    if (full)
    {
        {
            std::lock_guard<std::mutex> g(gate.mu);
            gate.open = true;
            gate.cv.notify_all();
        }
        // the flush thread finishes A, seals the full B and switches B -> A
        wait_durable(log, last, "the frames of the full segment");
    }
    // Y into the other segment; its flush switches back to P's segment, which
    // is then active again, empty and unsealed
    const int64_t y = log.append(small.data(), small.size());
    wait_durable(log, y, "Y");
    {
        std::lock_guard<std::mutex> hold(park.mu);
        park.release[1] = true;
        park.cv.notify_all();
    }
    int rc = 0;
    {
        std::unique_lock<std::mutex> hold(done_mu);
        if (!poll_until(hold, [&] { return p_done.load(); }))
        {
            char st[512];
            log.debug_state(st, sizeof st);
            fprintf(stderr, "liveness (%s): parked append did not return after two segment "
                            "switches\n  state: %s\n",
                    full ? "full" : "sealed", st);
            rc = 1;
        }
    }
    if (rc)
    {
        // rescue P: a frame in the active segment makes the flush thread switch
        log.append(small.data(), small.size());
    }
    p.join();
    if (!rc && p_rec.load() != y + 1)
    {
        fprintf(stderr, "liveness (%s): parked append got record %lld, want %lld\n",
                full ? "full" : "sealed", (long long)p_rec.load(), (long long)(y + 1));
        rc = 1;
    }
    if (!rc) wait_durable(log, p_rec.load(), "P's record");
    log.close();
    return rc;
}

}  // namespace

int main(int argc, char** argv)
{
    char tmpl[] = "/tmp/dlog_liveness_XXXXXX";
    const char* root = argc > 1 ? argv[1] : mkdtemp(tmpl);
    if (!root)
    {
        perror("mkdtemp");
        return 2;
    }
    const std::string r(root);
    std::string mk = "mkdir -p '" + r + "'";
    if (system(mk.c_str()) != 0) return 2;
    int rc = 0;
    const int sealed = scenario(r + "/sealed", false);
    const int full = scenario(r + "/full", true);
    std::string cmd = "rm -rf '" + r + "'";
    if (system(cmd.c_str()) != 0) fprintf(stderr, "cleanup of %s failed\n", root);
    rc = sealed ? sealed : full;
    printf("liveness sealed=%s full=%s\n", sealed ? "HUNG" : "ok", full ? "HUNG" : "ok");
    if (!rc) printf("liveness ok\n");
    return rc;
}
