// omf_runtime.cpp — error reporting and version of the C ABI (host only).
#include <hip/hip_runtime.h>

#include <string>

#include "../../include/omf_codec.h"
#include "omf_common.h"

namespace omf {

static thread_local std::string g_last_error;

void set_error(const std::string& msg) { g_last_error = msg; }

int fail(int code, const std::string& msg) {
  g_last_error = msg;
  return code;
}

int hip_fail(hipError_t e, const char* what) {
  g_last_error = std::string(what) + ": " + hipGetErrorString(e);
  return OMF_EHIP;
}

}  // namespace omf

extern "C" {

int omf_abi_version(void) { return OMF_ABI_VERSION; }

const char* omf_last_error(void) { return omf::g_last_error.c_str(); }

}  // extern "C"
