// C-ABI housekeeping: thread-local error string and version (SURVEY.md §8(b) error contract:
// negative return code + lnr_last_error(), which the Python layer raises as RuntimeError as
// tcnn's CHECK_THROW does).
#include "common.hpp"

#include <string>

namespace lnr {
static thread_local std::string g_err;
void set_error(const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_err = buf;
}
}  // namespace lnr

extern "C" const char* lnr_last_error(void) { return lnr::g_err.c_str(); }
extern "C" int lnr_version(void) { return 1; }

