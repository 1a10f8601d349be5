// fail() / krcn_last_error_string for the host-only sanitizer builds (the
// library's own are in krcn_plan.hip, next to the HIP code).
#include <cstdarg>
#include <cstdio>
#include <string>

#include "krcn_host.hpp"

static thread_local std::string g_err;

krcn_status fail(krcn_status s, const char* fmt, ...) {
  char buf[2048];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_err = buf;
  return s;
}

extern "C" const char* krcn_last_error_string(void) { return g_err.c_str(); }
