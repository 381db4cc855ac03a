// handles_stress.cpp — the C-ABI's handle lifetime protocol (mythril_amd/csrc/
// mw_handles.h, the code mw_kernels.hip runs) under ThreadSanitizer and
// AddressSanitizer on the host.  Contexts and programs own heap buffers in
// place of device memory; threads load programs, search, free programs and
// free contexts concurrently, with stale and double frees mixed in.  A use
// after free or a data race makes the sanitizer fail the run; the protocol's
// answers (refused stale handles, no leaked program) are checked here.
#include <atomic>
#include <cstdio>
#include <cstring>
#include <random>
#include <thread>
#include <vector>

#include "../../mythril_amd/csrc/mw_handles.h"

struct Ctx {
  std::mutex mu;
  bool dead = false;
  std::vector<unsigned>* scratch = new std::vector<unsigned>(64, 1u);   // "device" buffers
};
struct Prog {
  std::shared_ptr<Ctx> ctx;
  bool dead = false;
  unsigned* buf = new unsigned[32]();
};

static mw::Registry<Ctx, Prog> reg;
static std::atomic<long> searches{0}, refused{0}, bad_frees{0};
static std::atomic<long> released_progs{0}, loaded_progs{0};

static void release_prog(Prog& p) {
  delete[] p.buf;
  p.buf = nullptr;
  released_progs++;
}
static void release_ctx(Ctx& c) {
  delete c.scratch;
  c.scratch = nullptr;
}

static uint64_t load(uint64_t ch) {   // mg_prog_load
  auto c = reg.ctx(ch);
  if (!c) return 0;
  std::lock_guard<std::mutex> lk(c->mu);
  if (c->dead) return 0;
  auto p = std::make_shared<Prog>();
  p->ctx = c;
  loaded_progs++;
  return reg.add_prog(std::move(p));
}

static bool search(uint64_t ch, const std::vector<uint64_t>& ps) {   // mg_search
  mw::Call<Ctx, Prog> call;
  if (mw::enter(reg, ch, ps.data(), ps.size(), call)) {
    refused++;
    return false;
  }
  unsigned acc = 0;
  for (auto& p : call.ps)
    for (int k = 0; k < 32; ++k) acc += p->buf[k]++;   // touches every program's buffer
  (*call.c->scratch)[acc & 63] += acc;
  searches++;
  return true;
}

int main(int argc, char** argv) {
  const int rounds = argc > 1 ? std::atoi(argv[1]) : 300;
  std::mt19937_64 rng(12345);
  for (int r = 0; r < rounds; ++r) {
    auto c = std::make_shared<Ctx>();
    const uint64_t ch = reg.add_ctx(c);
    c.reset();
    std::vector<uint64_t> ps;
    for (int i = 0; i < 8; ++i) ps.push_back(load(ch));
    std::atomic<bool> go{false};
    const unsigned seed = (unsigned)rng();
    std::thread searcher([&] {
      while (!go) {}
      for (int i = 0; i < 50; ++i)   // single programs and the whole batch
        search(ch, i % 5 == 4 ? ps : std::vector<uint64_t>{ps[i % ps.size()]});
    });
    std::thread loader([&] {
      while (!go) {}
      for (int i = 0; i < 20; ++i) {
        const uint64_t p = load(ch);
        if (p && (i & 1)) mw::free_prog(reg, p, release_prog);
      }
    });
    std::thread prog_freer([&, seed] {
      while (!go) {}
      std::mt19937 g(seed);
      for (int i = 0; i < 12; ++i) {
        const uint64_t p = ps[g() % ps.size()];
        if (!mw::free_prog(reg, p, release_prog)) bad_frees++;   // twice, or after its context: refused
      }
    });
    std::thread ctx_freer([&] {
      while (!go) {}
      std::this_thread::yield();
      if (!mw::free_ctx(reg, ch, release_prog, release_ctx)) bad_frees++;
    });
    go = true;
    searcher.join();
    loader.join();
    prog_freer.join();
    ctx_freer.join();
    // everything of this context is gone; stale handles stay refused even
    // after the allocator reuses the records' memory
    if (mw::free_ctx(reg, ch, release_prog, release_ctx)) { std::puts("FAIL: double mg_free accepted"); return 1; }
    for (uint64_t p : ps)
      if (mw::free_prog(reg, p, release_prog)) { std::puts("FAIL: stale program freed"); return 1; }
    if (search(ch, ps)) { std::puts("FAIL: search on a freed context"); return 1; }
  }
  if (reg.live_progs() != 0) { std::puts("FAIL: programs left in the registry"); return 1; }
  if (released_progs.load() != loaded_progs.load()) {
    std::printf("FAIL: %ld programs loaded, %ld released\n", loaded_progs.load(), released_progs.load());
    return 1;
  }
  std::printf("OK rounds=%d searches=%ld refused=%ld refused_frees=%ld programs=%ld\n", rounds, searches.load(),
              refused.load(), bad_frees.load(), loaded_progs.load());
  return 0;
}
