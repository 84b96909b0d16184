// capi.cpp -- library-wide C ABI pieces: thread-local error text and version.
#include <stdarg.h>
#include <stdio.h>

#include <string>

#include "mc_common.h"

namespace mc {
static thread_local std::string g_last_error;

void set_error(const char* fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_last_error = buf;
}

const char* last_error() { return g_last_error.c_str(); }
}  // namespace mc

extern "C" const char* mc_last_error(void) { return mc::last_error(); }
extern "C" const char* mc_version(void) { return "mamba_clip_amd 0.1.0 (gfx950)"; }
