// Thread-local error reporting for the C ABI (mopo_last_error).
#include <string>

#include "../../include/mopo_hip.h"

namespace mopo {
static thread_local std::string g_err;
void set_error(const std::string& msg) { g_err = msg; }
int fail(const std::string& msg) {
  g_err = msg;
  return -1;
}
}  // namespace mopo

extern "C" const char* mopo_last_error(void) { return mopo::g_err.c_str(); }
extern "C" int mopo_version(void) { return 1; }
