// mppi_prewarm.cpp -- the opt-in prewarm thread (mppi_set_prewarm, ABI 8).  It reads only the
// engine's atomics (call_t, call_n, pw_*) and, once a native control call has stored pw_native
// (release, after e->aql was set), the engine's native queue, into which it writes touch packets
// under the queue's mutex (mppi_aql.cpp step_touch; a batch holds the queue through step_guard).
#include <sys/prctl.h>
#include <emmintrin.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdlib>
#include <string>
#include <thread>

#include "mppi_engine.h"

// ---------------------------------------------------------------- prewarm (the node's idle gaps)
// At the node's cadence (rospy.Rate(100), kinova.py:101) the engine's queue sits empty ~10 ms
// between calls, and a call on a queue idle for more than ~50-100 us runs ~6-7 us longer than
// back to back; a pair of one-wave packets on the same queue 20-50 us before the call removes
// that, a touch 100 us or more before it does not, nor does a touch on another queue or the
// doorbell alone (profiles/r05/prewarm/).  So the thread predicts the next call from the median
// interval of the last calls and, from pw_us before the prediction until the call starts (or
// pw_us after it), touches the queue every kTouchNs.  Calls back to back or slower than 1 s get
// no touches; nothing the engine computes changes (the touch writes a scratch word only).
namespace mppi_host {
constexpr int64_t kTouchNs = 25000;

int64_t steady_ns() {
    return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch())
        .count();
}

void note_call(mppi_engine* e) {   // mppi_step entry (the caller's thread)
    if (!e->pw_us.load(std::memory_order_relaxed)) return;
    const int64_t n = e->call_n.load(std::memory_order_relaxed);
    e->call_t[n % 8].store(steady_ns(), std::memory_order_relaxed);
    e->call_n.store(n + 1, std::memory_order_release);
}

// The next window from the last m (<= 8) call starts t[] (oldest first): the median interval P
// predicts the call at t[m-1] + P, the window is [that - win, that + win].  0: no window (fewer
// than 4 calls, P < 4 windows -- back to back -- or P > 1 s); 1: *start / *end set.
int prewarm_plan(const int64_t* t, int m, int64_t win, int64_t* start, int64_t* end) {
    if (m < 4) return 0;
    int64_t d[8];
    for (int i = 1; i < m; ++i) d[i - 1] = t[i] - t[i - 1];
    std::nth_element(d, d + (m - 1) / 2, d + (m - 1));
    const int64_t P = d[(m - 1) / 2];
    if (P < 4 * win || P > 1000000000) return 0;
    *start = t[m - 1] + P - win;
    *end = t[m - 1] + P + win;
    return 1;
}

void prewarm_loop(mppi_engine* e) {
    prctl(PR_SET_TIMERSLACK, 1000UL, 0UL, 0UL, 0UL);   // this thread's sleeps end ~1 us after their deadline
    std::unique_lock<std::mutex> lk(e->pw_mu);
    auto nap = [&](int64_t ns) { e->pw_cv.wait_for(lk, std::chrono::nanoseconds(ns), [&] { return e->pw_stop.load(); }); };
    while (!e->pw_stop.load()) {
        const int64_t win = (int64_t)e->pw_us.load() * 1000;
        const int64_t n = e->call_n.load(std::memory_order_acquire);
        // pw_native (acquire) first: a native call stored it (release) after e->aql was set, so the
        // pointer is read only once its write is visible here.  HIP-launched calls: nothing to warm.
        if (n < 4 || !e->pw_native.load(std::memory_order_acquire) || !e->aql) { nap(2000000); continue; }
        const int m = (int)std::min<int64_t>(n, 8);
        int64_t t[8], start = 0, end = 0;
        for (int i = 0; i < m; ++i) t[i] = e->call_t[(n - m + i) % 8].load(std::memory_order_relaxed);
        const int64_t now = steady_ns();
        if (!prewarm_plan(t, m, win, &start, &end) || now > end) { nap(2000000); continue; }   // no cadence, or the call is late
        if (now < start - 200000) { nap(start - 100000 - now); continue; }           // (then look again)
        lk.unlock();   // through the window: a touch, then sleep to the next (the host keeps its core)
        int64_t next = start;
        while (!e->pw_stop.load(std::memory_order_relaxed) && e->call_n.load(std::memory_order_acquire) == n) {
            const int64_t tn = steady_ns();
            if (tn > end) break;
            if (tn >= next) {
                std::string err;
                if (mppi_aql::step_touch(e->aql, true, &err) == 0) e->pw_touches.fetch_add(1, std::memory_order_relaxed);
                next = tn + kTouchNs;
            }
            if (e->pw_spin) _mm_pause();
            else std::this_thread::sleep_for(std::chrono::nanoseconds(std::max<int64_t>(1000, next - steady_ns())));
        }
        lk.lock();
        if (e->call_n.load(std::memory_order_acquire) == n) nap(1000000);   // the window passed without the call
    }
}

void prewarm_stop(mppi_engine* e) {
    if (!e->pw_thr.joinable()) return;
    {
        std::lock_guard<std::mutex> lk(e->pw_mu);
        e->pw_stop.store(true);
    }
    e->pw_cv.notify_all();
    e->pw_thr.join();
    e->pw_stop.store(false);
}
}  // namespace mppi_host

using namespace mppi_host;

extern "C" {

mppi_status mppi_set_prewarm(mppi_engine* e, int32_t window_us) {
    if (!e) return fail(MPPI_ERR_INVALID_ARG, "null engine");
    if (window_us != 0 && (window_us < 50 || window_us > 5000))
        return fail(MPPI_ERR_INVALID_ARG, "prewarm window %d us: 0 (off) or 50 .. 5000", window_us);
    prewarm_stop(e);
    e->pw_us.store(window_us);
    e->call_n.store(0);
    const char* spin = getenv("MPPI_PREWARM_SPIN");
    e->pw_spin = spin && spin[0] == '1';
    if (window_us) e->pw_thr = std::thread(prewarm_loop, e);
    return MPPI_OK;
}

mppi_status mppi_get_prewarm(mppi_engine* e, int32_t* window_us, int64_t* touches) {
    if (!e || !window_us || !touches) return fail(MPPI_ERR_INVALID_ARG, "null argument");
    *window_us = e->pw_us.load();
    *touches = e->pw_touches.load();
    return MPPI_OK;
}

// Diagnostic (host only, tests/test_prewarm_cpu.py): the prewarm thread's window for call starts
// t[0..m) in ns and a window of window_us: 1 and [*start, *end], or 0 (no window).
int32_t mppi_debug_prewarm_plan(const int64_t* t, int32_t m, int32_t window_us, int64_t* start, int64_t* end) {
    if (!t || !start || !end || m < 0 || m > 8) return MPPI_ERR_INVALID_ARG;
    return prewarm_plan(t, m, (int64_t)window_us * 1000, start, end);
}

}  // extern "C"
