// api_common.cpp -- see api_common.h.
#include "api_common.h"

#include "srsran_amd/ldpc.h"
#include <cstdarg>
#include <cstdio>
#include <string>

namespace srs_amd {

namespace {
thread_local std::string g_last_error;
} // namespace

int fail(int code, const char* fmt, ...)
{
  char    buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_last_error = buf;
  return code;
}

int hip_fail(hipError_t e, const char* what)
{
  return fail(SRS_AMD_EHIP, "%s: %s", what, hipGetErrorString(e));
}

const char* last_error()
{
  return g_last_error.c_str();
}

int select_device(int& device)
{
  int        ndev = 0;
  hipError_t e    = hipGetDeviceCount(&ndev);
  if (e != hipSuccess || ndev == 0) {
    return fail(SRS_AMD_EHIP, "no HIP device available (%s)", hipGetErrorString(e));
  }
  if (device < 0) {
    e = hipGetDevice(&device);
    if (e != hipSuccess) {
      return hip_fail(e, "hipGetDevice");
    }
  }
  e = hipSetDevice(device);
  if (e != hipSuccess) {
    return hip_fail(e, "hipSetDevice");
  }
  return SRS_AMD_OK;
}

} // namespace srs_amd
