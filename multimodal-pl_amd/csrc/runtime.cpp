// Error plumbing and small shared host code for libu3d.
#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdio>
#include <string>

#include "common.h"

namespace u3d {

static thread_local std::string g_last_error;

void set_error(const std::string& msg) { g_last_error = msg; }

int fail(int code, const char* fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_last_error = buf;
  return code;
}

int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(U3D_EHIP, "%s launch: %s", what, hipGetErrorString(e));
  return U3D_OK;
}

}  // namespace u3d

extern "C" const char* u3d_last_error(void) { return u3d::g_last_error.c_str(); }
extern "C" int u3d_abi_version(void) { return 1; }
