// CPU check of mw_inflight.h (tests/test_inflight.py): a call blocked in a
// step is reported by another thread, with its call and step names; a
// nested call's steps are the outer call's; a slow step prints its line
// when it ends; finished calls leave the report.
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <thread>

#include "../../mythril_amd/csrc/mw_inflight.h"

static std::mutex mu;
static std::condition_variable cv;
static bool entered = false, release = false;

static void helper() { mw::inflight_step("helper_step", 42); }

static void blocked_call() {
  mw::CallMark m("mg_test_call");
  m.step("first");
  {
    mw::CallMark inner("mg_inner");   // nested: reports through the outer call
    inner.step("inner_step", 7);
  }
  helper();
  m.step("blocked", 4096);
  std::unique_lock<std::mutex> lk(mu);
  entered = true;
  cv.notify_all();
  cv.wait(lk, [] { return release; });
}

int main() {
  char buf[4096];
  if (mw::inflight_report(buf, sizeof buf) != 0 || buf[0] != 0) return std::puts("FAIL idle report"), 1;
  std::thread t(blocked_call);
  {
    std::unique_lock<std::mutex> lk(mu);
    cv.wait(lk, [] { return entered; });
  }
  std::this_thread::sleep_for(std::chrono::milliseconds(120));   // > MYTHRIL_AMD_SLOW_STEP_MS in the test
  const int n = mw::inflight_report(buf, sizeof buf);
  std::printf("%s", buf);
  if (n != 1 || !std::strstr(buf, "mg_test_call/blocked arg=4096")) return std::puts("FAIL blocked report"), 1;
  if (std::strstr(buf, "mg_inner")) return std::puts("FAIL nested call reported on its own"), 1;
  {
    std::lock_guard<std::mutex> lk(mu);
    release = true;
  }
  cv.notify_all();
  t.join();
  if (mw::inflight_report(buf, sizeof buf) != 0) return std::puts("FAIL finished call still reported"), 1;
  // a tiny buffer is truncated, never overrun
  std::thread t2([] { mw::CallMark m("mg_again"); m.step("x"); std::this_thread::sleep_for(std::chrono::milliseconds(50)); });
  std::this_thread::sleep_for(std::chrono::milliseconds(20));
  char small[8];
  std::memset(small, 'Z', sizeof small);
  mw::inflight_report(small, 4);
  t2.join();
  if (small[3] != 0 || small[4] != 'Z') return std::puts("FAIL truncation"), 1;
  std::puts("OK");
  return 0;
}
