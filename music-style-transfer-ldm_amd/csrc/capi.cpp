// Error state and introspection entry points of the C ABI (include/ldm_capi.h).
#include <hip/hip_runtime.h>

#include <string>

#include "common.h"

namespace ldm {

static thread_local std::string g_last_error;

void set_error(const std::string& msg) { g_last_error = msg; }

int fail(int code, const std::string& msg) {
    g_last_error = msg;
    return code;
}

}  // namespace ldm

extern "C" const char* ldm_last_error(void) { return ldm::g_last_error.c_str(); }

extern "C" int ldm_capi_version(void) { return LDM_CAPI_VERSION; }

extern "C" int ldm_device_count(int* count) {
    LDM_REQUIRE(count, "device_count: null argument");
    int n = 0;
    LDM_HIP_TRY(hipGetDeviceCount(&n));
    *count = n;
    return 0;
}
