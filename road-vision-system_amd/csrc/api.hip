// ABI housekeeping: version and thread-local last-error text.
#include <stdarg.h>
#include "common.h"

namespace rv {
static thread_local char g_err[512] = "";

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}
}  // namespace rv

extern "C" int rv_abi_version(void) { return 2; }
extern "C" const char* rv_last_error(void) { return rv::g_err; }
