// mw_inflight.h — which C-ABI call, and which step of it, every thread is in
// (a GPU test run went silent inside one call and left no
// trace of where).  Host-only C++; shared by the product library
// (mw_kernels.hip) and the CPU test that exercises it (tests/native/inflight_check.cpp).
//
// * A call opens a CallMark and names its steps as it goes ("lock",
//   "pool_get", "hipHostMalloc", "sync", ...).  The record lives in a fixed
//   table of per-thread slots written with relaxed atomics: no lock, no
//   allocation, so reading it can never block behind the call it reports.
// * mw::inflight_report formats the calls in flight (call, step, ms in each)
//   for a watchdog on another thread (tests/conftest.py calls
//   mg_debug_inflight through ctypes while the stuck call holds no GIL).
// * A step that took longer than MYTHRIL_AMD_SLOW_STEP_MS (default 2000)
//   prints one line on stderr when it ends, so a slow but finished step
//   names itself too.
#pragma once
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <map>
#include <mutex>
#include <string>
#include <thread>

namespace mw {

struct InflightSlot {
  std::atomic<uint64_t> tid{0};
  std::atomic<const char*> call{nullptr};   // nullptr: no call in flight on this thread
  std::atomic<const char*> step{nullptr};
  std::atomic<double> t_call{0.0}, t_step{0.0};
  std::atomic<uint64_t> arg{0};             // a step's size or count (bytes, programs), 0 if none
};

constexpr int kInflightSlots = 128;

inline InflightSlot* inflight_table() {
  static InflightSlot t[kInflightSlots];
  return t;
}

inline double inflight_now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

inline double slow_step_ms() {
  static const double v = [] {
    const char* e = std::getenv("MYTHRIL_AMD_SLOW_STEP_MS");
    const double x = e ? std::atof(e) : 2000.0;
    return x > 0 ? x : 2000.0;
  }();
  return v;
}

// this thread's slot: claimed once (threads beyond the table are not tracked)
inline InflightSlot* inflight_slot() {
  static std::atomic<int> next{0};
  thread_local int k = -1;
  if (k < 0) {
    k = next.fetch_add(1, std::memory_order_relaxed);
    if (k < kInflightSlots)
      inflight_table()[k].tid.store((uint64_t)std::hash<std::thread::id>()(std::this_thread::get_id()),
                                    std::memory_order_relaxed);
  }
  return k < kInflightSlots ? &inflight_table()[k] : nullptr;
}

// Step-time accounting (MYTHRIL_AMD_STEP_TIMES=1; tools/dropin_profile.py):
// wall time and count per "call/step", summed over the process until read
// (mw::step_times_report, mg_debug_step_times).  Off by default: one getenv.
inline bool step_times_on() {
  static const bool on = [] {
    const char* e = std::getenv("MYTHRIL_AMD_STEP_TIMES");
    return e && e[0] == '1';
  }();
  return on;
}
struct StepTimes {
  std::mutex mu;
  std::map<std::string, std::pair<double, uint64_t>> t;   // "call/step" -> (ms, count)
};
inline StepTimes& step_times() {
  static StepTimes st;
  return st;
}
inline void step_times_add(const char* call, const char* step, double ms) {
  StepTimes& st = step_times();
  std::lock_guard<std::mutex> lk(st.mu);
  auto& e = st.t[std::string(call) + "/" + step];
  e.first += ms;
  e.second += 1;
}

class CallMark;
inline CallMark*& current_mark() {
  thread_local CallMark* m = nullptr;
  return m;
}

class CallMark {
 public:
  explicit CallMark(const char* call) : call_(call), t_step_(inflight_now_ms()) {
    if (current_mark()) return;   // a call made by another call (mg_keccak256): the outer one reports
    current_mark() = this;
    outer_ = true;
    step_ = "enter";
    t_call_ = t_step_;
    s_ = inflight_slot();
    if (s_) {
      s_->t_call.store(t_step_, std::memory_order_relaxed);
      s_->t_step.store(t_step_, std::memory_order_relaxed);
      s_->step.store("enter", std::memory_order_relaxed);
      s_->arg.store(0, std::memory_order_relaxed);
      s_->call.store(call, std::memory_order_release);
    }
  }
  CallMark(const CallMark&) = delete;
  CallMark& operator=(const CallMark&) = delete;
  // the call moves on to step `name` (arg: its size, for the report)
  void step(const char* name, uint64_t arg = 0) {
    if (!outer_) {
      if (CallMark* m = current_mark()) m->step(name, arg);
      return;
    }
    finish_step();
    step_ = name;
    arg_ = arg;
    t_step_ = inflight_now_ms();
    if (s_) {
      s_->t_step.store(t_step_, std::memory_order_relaxed);
      s_->arg.store(arg, std::memory_order_relaxed);
      s_->step.store(name, std::memory_order_release);
    }
  }
  ~CallMark() {
    if (!outer_) return;
    finish_step();
    if (step_times_on()) step_times_add(call_, "(call)", inflight_now_ms() - t_call_);
    if (s_) s_->call.store(nullptr, std::memory_order_release);
    current_mark() = nullptr;
  }

 private:
  void finish_step() {
    if (!step_) return;
    const double d = inflight_now_ms() - t_step_;
    if (step_times_on()) step_times_add(call_, step_, d);
    if (d > slow_step_ms())
      std::fprintf(stderr, "[mythril_amd] slow step: %s/%s (%llu) took %.0f ms\n", call_, step_,
                   (unsigned long long)arg_, d);
  }
  InflightSlot* s_ = nullptr;
  bool outer_ = false;
  const char* call_;
  const char* step_ = nullptr;
  uint64_t arg_ = 0;
  double t_step_, t_call_ = 0.0;
};

// Name the current step of this thread's call from inside a helper
// (pool_get, ensure_launch, ...); nothing when no call is open.
inline void inflight_step(const char* name, uint64_t arg = 0) {
  if (CallMark* m = current_mark()) m->step(name, arg);
}

// One line per call in flight: "tid call/step arg call_ms step_ms".  Returns
// the number of calls; writes at most n bytes (NUL-terminated) into buf.
inline int inflight_report(char* buf, size_t n) {
  const double now = inflight_now_ms();
  size_t used = 0;
  int calls = 0;
  if (buf && n) buf[0] = 0;
  for (int i = 0; i < kInflightSlots; ++i) {
    InflightSlot& s = inflight_table()[i];
    const char* c = s.call.load(std::memory_order_acquire);
    if (!c) continue;
    const char* st = s.step.load(std::memory_order_acquire);
    ++calls;
    if (buf && used + 1 < n) {
      const int w = std::snprintf(buf + used, n - used, "tid=%016llx %s/%s arg=%llu call_ms=%.0f step_ms=%.0f\n",
                                  (unsigned long long)s.tid.load(std::memory_order_relaxed), c, st ? st : "?",
                                  (unsigned long long)s.arg.load(std::memory_order_relaxed),
                                  now - s.t_call.load(std::memory_order_relaxed),
                                  now - s.t_step.load(std::memory_order_relaxed));
      if (w > 0) used = std::min(n - 1, used + (size_t)w);
    }
  }
  return calls;
}

// "call/step ms count" per line, then the table is cleared; returns the
// number of lines (0 when MYTHRIL_AMD_STEP_TIMES is off).
inline int step_times_report(char* buf, size_t n) {
  StepTimes& st = step_times();
  std::lock_guard<std::mutex> lk(st.mu);
  size_t used = 0;
  int lines = 0;
  if (buf && n) buf[0] = 0;
  for (auto& kv : st.t) {
    if (buf && used + 1 < n) {
      const int w = std::snprintf(buf + used, n - used, "%s %.6f %llu\n", kv.first.c_str(), kv.second.first,
                                  (unsigned long long)kv.second.second);
      if (w > 0) used = std::min(n - 1, used + (size_t)w);
    }
    ++lines;
  }
  st.t.clear();
  return lines;
}

}  // namespace mw
