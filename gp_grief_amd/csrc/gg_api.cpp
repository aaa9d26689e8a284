// Runtime entry points of the C ABI (include/gp_grief_amd.h): version, errors,
// device selection.  Compute entry points live next to their kernels.
#include <cstring>
#include <string>

#include "gg_internal.h"

namespace gg {
static thread_local std::string g_last_error;
void set_last_error(const std::string& msg) { g_last_error = msg; }
}  // namespace gg

extern "C" {

int gg_abi_version(void) { return GG_ABI_VERSION; }

int gg_last_error(char* buf, size_t len) {
  if (!buf || len == 0) return GG_ERR_VALUE;
  const std::string& s = gg::g_last_error;
  const size_t n = s.size() < len - 1 ? s.size() : len - 1;
  std::memcpy(buf, s.data(), n);
  buf[n] = '\0';
  return GG_OK;
}

int gg_set_device(int device) {
  return gg::guard([&] { GG_HIP(hipSetDevice(device)); });
}

int gg_device_synchronize(void) {
  return gg::guard([&] { GG_HIP(hipDeviceSynchronize()); });
}

}  // extern "C"
