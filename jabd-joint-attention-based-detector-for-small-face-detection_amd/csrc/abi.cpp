// Library identity and thread-local error reporting for the C-ABI.
#include <string.h>

#include "common.h"

namespace jabd {
static thread_local char g_err[512] = {0};

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}
}  // namespace jabd

extern "C" const char* jabd_version(void) { return "jabd-mi355x 0.1.0 (gfx950)"; }

extern "C" int jabd_last_error(char* buf, size_t len) {
  if (!buf || len == 0) return JABD_EINVAL;
  strncpy(buf, jabd::g_err, len - 1);
  buf[len - 1] = 0;
  return JABD_OK;
}
