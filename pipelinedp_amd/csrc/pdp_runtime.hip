// pdp_runtime.hip — error reporting, kernel profiler and small C ABI utilities.
#include <cstring>
#include <map>
#include <mutex>
#include <vector>

#include "pdp_internal.h"

namespace pdp {

namespace {
thread_local std::string g_last_error;
}

int set_error(int code, const char* msg) {
  g_last_error = msg;
  return code;
}

const char* last_error() { return g_last_error.c_str(); }

// profiler: (name, start, stop) event triples, resolved by pdp_profiler_report
namespace {
struct ProfRecord {
  std::string name;
  hipEvent_t start, stop;
};
std::mutex g_prof_mu;
bool g_prof_on = false;
std::vector<ProfRecord> g_prof;
std::vector<hipEvent_t> g_free_events;
std::string g_open_name;
hipEvent_t g_open_start = nullptr;

hipEvent_t take_event() {
  if (!g_free_events.empty()) {
    hipEvent_t e = g_free_events.back();
    g_free_events.pop_back();
    return e;
  }
  hipEvent_t e = nullptr;
  if (hipEventCreate(&e) != hipSuccess) return nullptr;
  return e;
}
}  // namespace

bool profiler_enabled() { return g_prof_on; }

void profiler_begin(const char* name, hipStream_t stream) {
  std::lock_guard<std::mutex> lock(g_prof_mu);
  g_open_start = take_event();
  g_open_name = name;
  if (g_open_start) (void)hipEventRecord(g_open_start, stream);
}

void profiler_end(hipStream_t stream) {
  std::lock_guard<std::mutex> lock(g_prof_mu);
  if (!g_open_start) return;
  hipEvent_t stop = take_event();
  if (!stop) return;
  (void)hipEventRecord(stop, stream);
  g_prof.push_back(ProfRecord{g_open_name, g_open_start, stop});
  g_open_start = nullptr;
}

}  // namespace pdp

extern "C" {

int pdp_abi_version(void) { return PDP_ABI_VERSION; }

const char* pdp_last_error(void) { return pdp::last_error(); }

int pdp_bound_error_flags(const void* workspace, uint32_t* flags, void* stream) {
  if (workspace == nullptr || flags == nullptr) return pdp::set_error(PDP_E_INVALID, "NULL argument");
  hipStream_t st = (hipStream_t)stream;
  PDP_HIP_CHECK(hipMemcpyAsync(flags, workspace, 4, hipMemcpyDeviceToHost, st));
  PDP_HIP_CHECK(hipStreamSynchronize(st));
  return PDP_OK;
}

int pdp_profiler_enable(int enable) {
  std::lock_guard<std::mutex> lock(pdp::g_prof_mu);
  for (auto& r : pdp::g_prof) {
    pdp::g_free_events.push_back(r.start);
    pdp::g_free_events.push_back(r.stop);
  }
  pdp::g_prof.clear();
  pdp::g_prof_on = enable != 0;
  return PDP_OK;
}

int pdp_profiler_report(int32_t max_entries, char* names, double* total_ms, int64_t* calls,
                        int32_t* n_entries) {
  if (n_entries == nullptr || max_entries < 0 || (max_entries > 0 && (!names || !total_ms || !calls)))
    return pdp::set_error(PDP_E_INVALID, "bad argument");
  std::lock_guard<std::mutex> lock(pdp::g_prof_mu);
  std::map<std::string, std::pair<double, int64_t>> agg;
  std::vector<std::string> order;
  for (auto& r : pdp::g_prof) {
    PDP_HIP_CHECK(hipEventSynchronize(r.stop));
    float ms = 0.f;
    PDP_HIP_CHECK(hipEventElapsedTime(&ms, r.start, r.stop));
    if (!agg.count(r.name)) order.push_back(r.name);
    agg[r.name].first += ms;
    agg[r.name].second += 1;
  }
  int k = 0;
  for (auto& name : order) {
    if (k >= max_entries) break;
    std::strncpy(names + (size_t)k * PDP_PROF_NAME_LEN, name.c_str(), PDP_PROF_NAME_LEN - 1);
    names[(size_t)k * PDP_PROF_NAME_LEN + PDP_PROF_NAME_LEN - 1] = 0;
    total_ms[k] = agg[name].first;
    calls[k] = agg[name].second;
    ++k;
  }
  *n_entries = k;
  return PDP_OK;
}

}  // extern "C"
