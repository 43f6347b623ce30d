// ABI bookkeeping: last-error buffer, version and arch queries.
#include "common.hpp"

#include <cstring>

namespace s3 {

static thread_local char g_err[1024] = {0};

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

void clear_error() { g_err[0] = 0; }

}  // namespace s3

extern "C" const char* s3_last_error(void) { return s3::g_err; }
extern "C" int s3_abi_version(void) { return 1; }
extern "C" const char* s3_arch(void) { return "gfx950"; }
