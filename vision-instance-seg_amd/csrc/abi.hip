// Error plumbing and version query of the visionseg C ABI (include/visionseg.h).
#include "common.h"

namespace vs {
namespace {
thread_local std::string g_last_error;
}
void set_error(const std::string& msg) { g_last_error = msg; }
}  // namespace vs

extern "C" int vs_abi_version(void) { return VS_ABI_VERSION; }
extern "C" const char* vs_last_error(void) { return vs::g_last_error.c_str(); }
