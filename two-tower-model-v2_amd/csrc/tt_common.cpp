// tt_common.cpp -- error plumbing for the C ABI (thread-local last error).
#include "tt_common.hpp"

namespace tt {

static thread_local std::string g_last_error;

void set_error(const std::string& msg) { g_last_error = msg; }

int fail(int code, const std::string& msg) {
  g_last_error = msg;
  return code;
}

int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    return fail(TT_ERR_LAUNCH, std::string(what) + ": " + hipGetErrorString(e));
  }
  return TT_OK;
}

}  // namespace tt

extern "C" int tt_version(void) { return 100; /* 0.1.0 */ }

extern "C" const char* tt_last_error(void) { return tt::g_last_error.c_str(); }
