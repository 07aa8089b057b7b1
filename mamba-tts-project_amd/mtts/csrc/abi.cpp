// ABI version + thread-local error string for libmtts.so.
#include <stdarg.h>
#include <stdio.h>

#include "common.h"

namespace mtts {
static thread_local char g_err[512] = "";
void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}
}  // namespace mtts

extern "C" int mtts_abi_version(void) { return MTTS_ABI_VERSION; }
extern "C" const char* mtts_last_error(void) { return mtts::g_err; }
