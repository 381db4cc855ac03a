// mw_handles.h — lifetimes of the C-ABI's context and program handles
// (include/mythril_witness.h, "Lifetimes").  Host-only C++; shared by the
// product library (mw_kernels.hip) and the CPU stress test that runs this
// protocol under ThreadSanitizer (tests/native/handles_stress.cpp).
//
// * A handle is an id, never an address, and ids are never reused: a stale
//   handle (freed, freed with its context, or made up) resolves to nothing, so
//   it is an MG_E_ARG even after the allocator hands its memory to a new object.
// * Objects are reference counted.  A call resolves its handles to shared
//   references first, so a concurrent free cannot delete what the call is using.
// * Every context has a mutex (`mu`) that serialises the calls on it and guards
//   the `dead` flags of the context and its programs.  A call locks it and then
//   re-checks that nothing it resolved was freed in between; a free marks the
//   object dead and releases its resources under the same lock, so it waits for
//   the call in flight.
// * Lock order: a context's mu, then the registry's own mutex (never the other
//   way round).
#pragma once
#include <cstdint>
#include <memory>
#include <mutex>
#include <unordered_map>
#include <vector>

namespace mw {

// C needs `std::mutex mu; bool dead;`, P needs `std::shared_ptr<C> ctx; bool dead;`.
template <class C, class P>
class Registry {
 public:
  using CtxRef = std::shared_ptr<C>;
  using ProgRef = std::shared_ptr<P>;

  uint64_t add_ctx(CtxRef c) {
    std::lock_guard<std::mutex> lk(mu_);
    const uint64_t h = fresh();
    ctxs_.emplace(h, std::move(c));
    return h;
  }
  // The caller holds p->ctx->mu and has checked that the context is not dead.
  uint64_t add_prog(ProgRef p) {
    std::lock_guard<std::mutex> lk(mu_);
    const uint64_t h = fresh();
    progs_.emplace(h, std::move(p));
    return h;
  }
  CtxRef ctx(uint64_t h) {
    std::lock_guard<std::mutex> lk(mu_);
    auto it = ctxs_.find(h);
    return it == ctxs_.end() ? nullptr : it->second;
  }
  ProgRef prog(uint64_t h) {
    std::lock_guard<std::mutex> lk(mu_);
    auto it = progs_.find(h);
    return it == progs_.end() ? nullptr : it->second;
  }
  CtxRef take_ctx(uint64_t h) {
    std::lock_guard<std::mutex> lk(mu_);
    auto it = ctxs_.find(h);
    if (it == ctxs_.end()) return nullptr;
    CtxRef c = std::move(it->second);
    ctxs_.erase(it);
    return c;
  }
  ProgRef take_prog(uint64_t h) {
    std::lock_guard<std::mutex> lk(mu_);
    auto it = progs_.find(h);
    if (it == progs_.end()) return nullptr;
    ProgRef p = std::move(it->second);
    progs_.erase(it);
    return p;
  }
  std::vector<ProgRef> take_progs_of(const C* c) {
    std::lock_guard<std::mutex> lk(mu_);
    std::vector<ProgRef> out;
    for (auto it = progs_.begin(); it != progs_.end();) {
      if (it->second->ctx.get() == c) {
        out.push_back(std::move(it->second));
        it = progs_.erase(it);
      } else {
        ++it;
      }
    }
    return out;
  }
  size_t live_progs() {
    std::lock_guard<std::mutex> lk(mu_);
    return progs_.size();
  }

 private:
  // 16-aligned, far from small integers, never 0, never reused (2^60 ids)
  uint64_t fresh() { return next_ += 0x10; }
  std::mutex mu_;
  uint64_t next_ = 0x7e5000000000ull;
  std::unordered_map<uint64_t, CtxRef> ctxs_;
  std::unordered_map<uint64_t, ProgRef> progs_;
};

// A call on one context and some of its programs, with the context's mu held
// for the call's lifetime.
template <class C, class P>
struct Call {
  std::shared_ptr<C> c;
  std::vector<std::shared_ptr<P>> ps;
  std::unique_lock<std::mutex> lk;
};

// Resolve and lock.  Returns nullptr, or why the call is refused.
template <class C, class P>
const char* enter(Registry<C, P>& r, uint64_t ch, const uint64_t* ph, size_t n, Call<C, P>& out) {
  out.c = r.ctx(ch);
  if (!out.c) return "not a live context";
  out.ps.resize(n);
  for (size_t i = 0; i < n; ++i) {
    out.ps[i] = r.prog(ph[i]);
    if (!out.ps[i]) return "a program handle is not live (already freed, or freed with its context)";
    if (out.ps[i]->ctx != out.c) return "program from another context";
  }
  out.lk = std::unique_lock<std::mutex>(out.c->mu);
  if (out.c->dead) return "the context was freed during the call";
  for (auto& p : out.ps)
    if (p->dead) return "a program was freed during the call";
  return nullptr;
}

// A call on one program (its context's mu held).
template <class C, class P>
const char* enter_prog(Registry<C, P>& r, uint64_t ph, Call<C, P>& out) {
  std::shared_ptr<P> p = r.prog(ph);
  if (!p) return "not a live program (already freed, or freed with its context)";
  out.c = p->ctx;
  out.ps.assign(1, p);
  out.lk = std::unique_lock<std::mutex>(out.c->mu);
  if (out.c->dead || p->dead) return "the program was freed during the call";
  return nullptr;
}

// mg_free: the context leaves the registry (no new call resolves it), waits
// for the call in flight, is marked dead, and its programs and then itself
// release their resources.  Returns false for a handle that is not live.
template <class C, class P, class FreeProg, class FreeCtx>
bool free_ctx(Registry<C, P>& r, uint64_t h, FreeProg free_prog, FreeCtx free_c) {
  std::shared_ptr<C> c = r.take_ctx(h);
  if (!c) return false;
  std::lock_guard<std::mutex> lk(c->mu);
  c->dead = true;
  // no program can join any more: mg_prog_load publishes under this mu after checking dead
  for (auto& p : r.take_progs_of(c.get()))
    if (!p->dead) {
      free_prog(*p);
      p->dead = true;
    }
  free_c(*c);
  return true;
}

// mg_prog_free.  Returns false for a handle that is not live.
template <class C, class P, class FreeProg>
bool free_prog(Registry<C, P>& r, uint64_t h, FreeProg free_p) {
  std::shared_ptr<P> p = r.take_prog(h);
  if (!p) return false;
  std::lock_guard<std::mutex> lk(p->ctx->mu);
  if (!p->dead) {   // its context may already be gone: its own resources are freed all the same
    free_p(*p);
    p->dead = true;
  }
  return true;
}

}  // namespace mw
