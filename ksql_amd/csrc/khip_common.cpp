// khip_common.cpp — error reporting and version entry points of the C ABI.
#include <string>

#include "khip_util.hpp"

namespace khip {
static thread_local std::string g_last_error;
void set_error(const std::string& msg) { g_last_error = msg; }
void clear_error() { g_last_error.clear(); }
}  // namespace khip

extern "C" {

const char* khip_last_error(void) { return khip::g_last_error.c_str(); }

int32_t khip_abi_version(void) { return KHIP_ABI_VERSION; }

const char* khip_build_target(void) { return "gfx950"; }

}  // extern "C"
