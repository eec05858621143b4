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

namespace {
// parallel.owner_of: the rank that owns a privacy-id identity
__device__ __forceinline__ int owner_of(int64_t z, int world) {
  z = (int64_t)((uint64_t)(z ^ (z >> 31)) * 0x9E3779B97F4A7C15ULL);
  z ^= z >> 29;
  int64_t r = z % world;
  return (int)(r < 0 ? r + world : r);
}

// grid-stride, 16-byte loads where aligned; one saturating atomic per wave with a mismatch
__global__ void __launch_bounds__(kBlock) k_owner_mismatches(const int64_t* __restrict__ ids, int64_t n, int world,
                                                             int rank, unsigned* out) {
  unsigned bad = 0;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const bool vec = ((uintptr_t)ids & 15) == 0;
  const int64_t n2 = vec ? n / 2 : 0;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n2; i += stride) {
    const longlong2 v = reinterpret_cast<const longlong2*>(ids)[i];
    bad += (owner_of(v.x, world) != rank) + (owner_of(v.y, world) != rank);
  }
  for (int64_t i = 2 * n2 + blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += stride)
    bad += owner_of(ids[i], world) != rank;
  for (int off = 32; off > 0; off >>= 1) bad += __shfl_down(bad, off, 64);
  if ((threadIdx.x & 63) == 0 && bad) {  // saturating add: a count that wrapped to 0 would read as "owned"
    unsigned old = __hip_atomic_load(out, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT), assumed;
    do {
      assumed = old;
      const unsigned sum = assumed + bad < assumed ? 0xFFFFFFFFu : assumed + bad;
      old = atomicCAS(out, assumed, sum);
    } while (old != assumed);
  }
}
}  // namespace

}  // namespace pdp

extern "C" {

int pdp_owner_mismatches(const int64_t* ids, int64_t n, int32_t world, int32_t rank, uint32_t* mismatches,
                         void* stream) {
  if (mismatches == nullptr || n < 0 || (n > 0 && ids == nullptr) || world < 1 || rank < 0 || rank >= world)
    return pdp::set_error(PDP_E_INVALID, "pdp_owner_mismatches: bad argument");
  hipStream_t st = (hipStream_t)stream;
  PDP_HIP_CHECK(hipMemsetAsync(mismatches, 0, 4, st));
  if (n == 0) return PDP_OK;
  const int64_t want = (n + 2 * pdp::kBlock - 1) / (2 * pdp::kBlock);
  const unsigned grid = (unsigned)(want < 4096 ? want : 4096);
  hipLaunchKernelGGL(pdp::k_owner_mismatches, dim3(grid), dim3(pdp::kBlock), 0, st, ids, n, (int)world, (int)rank,
                     mismatches);
  PDP_HIP_CHECK(hipGetLastError());
  return PDP_OK;
}


int pdp_abi_version(void) { return PDP_ABI_VERSION; }

const char* pdp_last_error(void) { return pdp::last_error(); }

int pdp_bound_error_flags(const void* workspace, uint32_t* flags, void* stream) {
  if (workspace == nullptr || flags == nullptr) return pdp::set_error(PDP_E_INVALID, "NULL argument");
  hipStream_t st = (hipStream_t)stream;
  PDP_HIP_CHECK(hipMemcpyAsync(flags, workspace, 4, hipMemcpyDeviceToHost, st));
  PDP_HIP_CHECK(hipStreamSynchronize(st));
  return PDP_OK;
}

int pdp_bound_error_flags_async(const void* workspace, uint32_t* flags, void* stream) {
  if (workspace == nullptr || flags == nullptr) return pdp::set_error(PDP_E_INVALID, "NULL argument");
  PDP_HIP_CHECK(hipMemcpyAsync(flags, workspace, 4, hipMemcpyDeviceToHost, (hipStream_t)stream));
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
