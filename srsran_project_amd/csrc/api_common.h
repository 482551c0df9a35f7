// api_common.h -- error reporting shared by the C-ABI entry points.
//
// The reference aborts through srsran_assert on invalid arguments; the C-ABI
// instead returns SRS_AMD_EINVAL (or SRS_AMD_EHIP for runtime failures) and
// keeps the reference's message in a thread-local string.
#pragma once

#include <hip/hip_runtime.h>

namespace srs_amd {

// Records the formatted message and returns `code`.
int fail(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));

// fail(SRS_AMD_EHIP, "<what>: <hip error string>").
int hip_fail(hipError_t e, const char* what);

const char* last_error();

// Checks that a HIP device exists and makes `device` (current if < 0) current;
// returns the device actually used through `device`.
int select_device(int& device);

} // namespace srs_amd
