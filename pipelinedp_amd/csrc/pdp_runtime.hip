// pdp_runtime.hip — error reporting and small C ABI utilities.
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

}  // extern "C"
