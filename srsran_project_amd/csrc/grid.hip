// grid.hip -- resource-grid row merge (include/srsran_amd/grid.h): the host's changes of a device-resident grid
// applied RE by RE (XOR with the last agreed state), one thread per RE of the changed rows.  HBM-bound: 4 B read per RE
// of delta, 8 B more per changed RE.
#include <hip/hip_runtime.h>

#include "srsran_amd/grid.h"
#include "srsran_amd/ldpc.h"

#include "api_common.h"

namespace srs_amd {
namespace {

constexpr int MERGE_THREADS = 256;

__global__ __launch_bounds__(MERGE_THREADS) void grid_merge_rows_kernel(uint32_t* grid, const uint32_t* delta,
                                                                         const uint32_t* rows, uint32_t row_len)
{
  const uint32_t k = blockIdx.x * MERGE_THREADS + threadIdx.x;
  if (k >= row_len) {
    return;
  }
  const uint32_t v = delta[static_cast<size_t>(blockIdx.y) * row_len + k];
  if (v != 0) {
    uint32_t* p = grid + static_cast<size_t>(rows[blockIdx.y]) * row_len + k;
    *p ^= v;
  }
}

} // namespace
} // namespace srs_amd

extern "C" int srs_amd_grid_merge_rows(uint32_t* d_grid, const uint32_t* d_delta, const uint32_t* d_rows,
                                       uint32_t nof_rows, uint32_t row_len, void* stream)
{
  if (nof_rows == 0 || row_len == 0) {
    return SRS_AMD_OK;
  }
  if (d_grid == nullptr || d_delta == nullptr || d_rows == nullptr) {
    return srs_amd::fail(SRS_AMD_EINVAL, "null device buffer");
  }
  if (nof_rows > 65535) {
    return srs_amd::fail(SRS_AMD_EINVAL, "at most 65535 rows per merge");
  }
  hipLaunchKernelGGL(srs_amd::grid_merge_rows_kernel,
                     dim3((row_len + srs_amd::MERGE_THREADS - 1) / srs_amd::MERGE_THREADS, nof_rows),
                     dim3(srs_amd::MERGE_THREADS), 0, static_cast<hipStream_t>(stream), d_grid, d_delta, d_rows,
                     row_len);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? SRS_AMD_OK : srs_amd::hip_fail(e, "grid_merge_rows_kernel launch");
}
