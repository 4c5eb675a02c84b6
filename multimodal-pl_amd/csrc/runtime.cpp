// Error plumbing and small shared host code for libu3d.
#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
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

namespace {
struct OptDef {
  const char* name;
  int dflt;
};
constexpr OptDef kOpts[OPT_COUNT] = {
    {"IGEMM_BN", 0},       {"IGEMM_NS", 0},     {"IGEMM_TARGET", 512}, {"IGEMM_AUTO", 1}, {"CONVG_CO32", -1},
    {"CONVG_PERSIST", 1},  {"CONVG_BW8", -1},   {"RING_KR", -1},       {"RING_WGS", 256}, {"RING_SC", 0},
    {"SMALL_WGS", 256},    {"GN_MAXBLK", 256},  {"HEAD_TR", 1},        {"STEM1", 1},      {"UP_BWD_BLK", -1},
    {"WGRAD_BD", 3},       {"WB_WGS", 256},     {"WR_TILE16", 0},      {"WR_WGS", 256},     {"WB_S2CO64", 1},
    {"IGEMM_BM", 128}, {"WSTD_ROW", 1}, {"UP_QUAD", 1}, {"LOSS_PAIR", 1},
    {"HEAD_NB", 768},  {"HEAD_GN_NB", 512}, {"STEM_MFMA", 1}, {"WB_S2BD", 3},
};
std::atomic<int> g_opt[OPT_COUNT];
std::once_flag g_opt_once;

void opt_init() {
  std::call_once(g_opt_once, [] {
    for (int i = 0; i < OPT_COUNT; ++i) {
      const std::string env = std::string("U3D_") + kOpts[i].name;
      const char* e = getenv(env.c_str());
      g_opt[i].store(e ? atoi(e) : kOpts[i].dflt);
    }
  });
}
}  // namespace

int opt(Opt o) {
  opt_init();
  return g_opt[o].load(std::memory_order_relaxed);
}

}  // namespace u3d

extern "C" int u3d_set_option(const char* name, int value) {
  u3d::opt_init();
  for (int i = 0; i < u3d::OPT_COUNT; ++i)
    if (name && strcmp(name, u3d::kOpts[i].name) == 0) {
      u3d::g_opt[i].store(value);
      return U3D_OK;
    }
  return u3d::fail(U3D_EINVAL, "u3d_set_option: unknown option '%s'", name ? name : "(null)");
}

extern "C" int u3d_get_option(const char* name, int* value) {
  u3d::opt_init();
  for (int i = 0; i < u3d::OPT_COUNT; ++i)
    if (name && value && strcmp(name, u3d::kOpts[i].name) == 0) {
      *value = u3d::g_opt[i].load();
      return U3D_OK;
    }
  return u3d::fail(U3D_EINVAL, "u3d_get_option: unknown option '%s'", name ? name : "(null)");
}

extern "C" const char* u3d_last_error(void) { return u3d::g_last_error.c_str(); }
extern "C" int u3d_abi_version(void) { return 1; }

