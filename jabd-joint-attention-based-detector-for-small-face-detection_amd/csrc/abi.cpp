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

// Sizes of the argument structs, so bindings can check their mirrors.
extern "C" int64_t jabd_abi_struct_size(int32_t which) {
  switch (which) {
    case 0: return (int64_t)sizeof(jabd_conv_args);
    case 1: return (int64_t)sizeof(jabd_dw_args);
    case 2: return (int64_t)sizeof(jabd_expdw_args);
    case 3: return (int64_t)sizeof(jabd_window_copy);
    default: return -1;
  }
}
