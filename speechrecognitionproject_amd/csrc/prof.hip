// Opt-in per-kernel timing with HIP events on the launch stream (bench.py's live roofline).
// When enabled, every instrumented launch site records an event before and after its kernel on
// the SAME stream; srk_prof_read() waits for the recorded events and sums the elapsed times by
// kernel name.  Disabled (the default), a ProfScope costs one relaxed atomic load.
#include <atomic>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "srk_internal.h"

namespace srk {
namespace {

struct Rec {
  std::string name;
  hipEvent_t a, b;
  double work;
};

std::atomic<bool> g_on{false};
std::mutex g_mu;
std::vector<Rec> g_recs;
std::vector<hipEvent_t> g_pool;

hipEvent_t take_event() {
  if (!g_pool.empty()) {
    hipEvent_t e = g_pool.back();
    g_pool.pop_back();
    return e;
  }
  hipEvent_t e = nullptr;
  if (hipEventCreate(&e) != hipSuccess) return nullptr;
  return e;
}

void recycle_all() {
  for (auto& r : g_recs) {
    g_pool.push_back(r.a);
    g_pool.push_back(r.b);
  }
  g_recs.clear();
}

}  // namespace

ProfScope::ProfScope(const char* name, hipStream_t s, double work) : name_(name), s_(s), a_(nullptr), work_(work) {
  if (!g_on.load(std::memory_order_relaxed)) return;
  std::lock_guard<std::mutex> lk(g_mu);
  a_ = take_event();
  if (a_) (void)hipEventRecord(static_cast<hipEvent_t>(a_), s_);
}

ProfScope::~ProfScope() {
  if (!a_) return;
  std::lock_guard<std::mutex> lk(g_mu);
  hipEvent_t b = take_event();
  if (!b) return;
  (void)hipEventRecord(b, s_);
  g_recs.push_back(Rec{name_, static_cast<hipEvent_t>(a_), b, work_});
}

}  // namespace srk

extern "C" {

int srk_prof_enable(int on) {
  SRK_API_BEGIN
  std::lock_guard<std::mutex> lk(srk::g_mu);
  SRK_CHECK_HIP(hipDeviceSynchronize());
  srk::recycle_all();
  srk::g_on.store(on != 0);
  return SRK_OK;
  SRK_API_END
}

int srk_prof_read(const char* name, int64_t* count, double* total_ms, double* total_work) {
  SRK_API_BEGIN
  SRK_REQUIRE(name && count && total_ms && total_work, SRK_ERR_INVALID, "prof_read: null pointer");
  std::lock_guard<std::mutex> lk(srk::g_mu);
  int64_t n = 0;
  double tot = 0.0, work = 0.0;
  for (auto& r : srk::g_recs) {
    if (r.name != name) continue;
    SRK_CHECK_HIP(hipEventSynchronize(r.b));
    float ms = 0.f;
    SRK_CHECK_HIP(hipEventElapsedTime(&ms, r.a, r.b));
    tot += ms;
    work += r.work;
    ++n;
  }
  *count = n;
  *total_ms = tot;
  *total_work = work;
  return SRK_OK;
  SRK_API_END
}

}  // extern "C"
