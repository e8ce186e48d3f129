// errors.cpp -- per-thread last-error text, the version string and the source hash of the C-ABI.
#include <cstdarg>
#include <cstdio>
#include <string>

#include "common.h"

namespace gcg {
namespace {
thread_local std::string g_last_error;
}

gcg_status fail(gcg_status st, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_last_error = buf;
  return st;
}

const char* last_error() { return g_last_error.c_str(); }
}  // namespace gcg

#ifndef GCG_SOURCE_HASH
#define GCG_SOURCE_HASH "unknown"
#endif

extern "C" {
const char* gcg_version(void) { return "0.2.0"; }
const char* gcg_source_hash(void) { return GCG_SOURCE_HASH; }
const char* gcg_last_error(void) { return gcg::last_error(); }
}
