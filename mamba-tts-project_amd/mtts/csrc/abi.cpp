// ABI version, thread-local error string and the kernel-path override table
// of libmtts.so.
#include <stdarg.h>
#include <stdio.h>

#include "common.h"

namespace mtts {
static thread_local char g_err[512] = "";
// every key starts at MTTS_OVR_AUTO (-1), whatever MTTS_OVR_COUNT is
struct OvrTable {
  int v[MTTS_OVR_COUNT];
  OvrTable() { for (int& x : v) x = -1; }
};
static OvrTable g_ovr_tab;
static int* const g_ovr = g_ovr_tab.v;
int override_of(int key) { return (key >= 0 && key < MTTS_OVR_COUNT) ? __atomic_load_n(&g_ovr[key], __ATOMIC_RELAXED) : -1; }
void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}
}  // namespace mtts

extern "C" int mtts_abi_version(void) { return MTTS_ABI_VERSION; }
extern "C" const char* mtts_last_error(void) { return mtts::g_err; }
extern "C" int mtts_set_override(int key, int value) {
  if (key < 0 || key >= MTTS_OVR_COUNT) {
    mtts::set_error("set_override: unknown key %d", key);
    return MTTS_EINVAL;
  }
  return __atomic_exchange_n(&mtts::g_ovr[key], value < 0 ? -1 : value, __ATOMIC_RELAXED);
}
extern "C" int mtts_get_override(int key) { return mtts::override_of(key); }
