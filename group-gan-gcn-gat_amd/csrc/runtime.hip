// Error reporting / version of libsgg.so.
#include "sgg_common.h"
#include <string.h>

namespace sgg {
static thread_local char g_err[512] = "";
void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}
}  // namespace sgg

extern "C" int sgg_version(void) { return 1; }
extern "C" const char* sgg_last_error(void) { return sgg::g_err; }
