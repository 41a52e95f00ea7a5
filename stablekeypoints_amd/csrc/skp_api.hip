// libskp error plumbing and version (C ABI in include/skp.h).
#include "skp_common.h"

namespace skp {
static thread_local std::string g_last_error;
void set_error(const std::string& msg) { g_last_error = msg; }
}  // namespace skp

extern "C" const char* skp_last_error(void) { return skp::g_last_error.c_str(); }
extern "C" int skp_version(void) { return 1; }
