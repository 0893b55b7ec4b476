// Opt-in per-kernel timing with HIP events on the launch stream (bench.py's live roofline).
// When enabled, every instrumented launch site records an event before and after its kernel on
// the SAME stream; srk_prof_read() waits for the recorded events and sums the elapsed times by
// kernel name.  Disabled (the default), a ProfScope costs one relaxed atomic load.
#include <atomic>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "srk_internal.h"

namespace srk {
namespace {

struct Rec {
  std::string name, detail;
  hipEvent_t a, b;
  double work, bytes;
};

std::atomic<bool> g_on{false};
std::mutex g_mu;
std::vector<Rec> g_recs;
std::vector<hipEvent_t> g_pool;
// scope nesting on this host thread: only the innermost scope records — a conv run as a plain GEMM is timed once,
// under the GEMM's name (the kernel that ran: rocprofv3 and the PMC files group it the same way), not again under
// the conv's
thread_local unsigned long long t_opened = 0;

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
  detail_[0] = 0;
  opened_ = ++t_opened;
  if (!g_on.load(std::memory_order_relaxed)) return;
  std::lock_guard<std::mutex> lk(g_mu);
  a_ = take_event();
  if (a_) (void)hipEventRecord(static_cast<hipEvent_t>(a_), s_);
}

ProfScope::~ProfScope() {
  if (!a_) return;
  std::lock_guard<std::mutex> lk(g_mu);
  if (t_opened != opened_) {   // a scope opened inside this one recorded the launches: drop this one
    g_pool.push_back(static_cast<hipEvent_t>(a_));
    return;
  }
  hipEvent_t b = take_event();
  if (!b) return;
  (void)hipEventRecord(b, s_);
  g_recs.push_back(Rec{name_, detail_, static_cast<hipEvent_t>(a_), b, work_, bytes_});
}

void ProfScope::detail(const char* fmt, ...) {
  if (!a_) return;
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(detail_, sizeof(detail_), fmt, ap);
  va_end(ap);
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

// Every record grouped by (name, detail), as JSON lines "name\tdetail\tcount\tms\twork\n" into buf
// (NUL-terminated, truncated at cap); *needed = the full length + 1.
int srk_prof_kernels(char* buf, int64_t cap, int64_t* needed) {
  SRK_API_BEGIN
  SRK_REQUIRE(needed && (buf || cap == 0), SRK_ERR_INVALID, "prof_kernels: null pointer");
  std::lock_guard<std::mutex> lk(srk::g_mu);
  struct Agg { int64_t n = 0; double ms = 0.0, work = 0.0, bytes = 0.0; };
  std::map<std::pair<std::string, std::string>, Agg> agg;
  for (auto& r : srk::g_recs) {
    SRK_CHECK_HIP(hipEventSynchronize(r.b));
    float ms = 0.f;
    SRK_CHECK_HIP(hipEventElapsedTime(&ms, r.a, r.b));
    Agg& g = agg[{r.name, r.detail}];
    g.n += 1;
    g.ms += ms;
    g.work += r.work;
    g.bytes += r.bytes;
  }
  std::string out;
  char line[360];
  for (auto& kv : agg) {
    snprintf(line, sizeof(line), "%s\t%s\t%lld\t%.6f\t%.6e\t%.6e\n", kv.first.first.c_str(),
             kv.first.second.c_str(), (long long)kv.second.n, kv.second.ms, kv.second.work, kv.second.bytes);
    out += line;
  }
  *needed = (int64_t)out.size() + 1;
  if (cap > 0) {
    const size_t n = std::min<size_t>(out.size(), (size_t)cap - 1);
    memcpy(buf, out.data(), n);
    buf[n] = 0;
  }
  return SRK_OK;
  SRK_API_END
}

}  // extern "C"
