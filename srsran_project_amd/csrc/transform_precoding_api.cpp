// transform_precoding_api.cpp -- C-ABI of the MI355X transform deprecoder (include/srsran_amd/transform_precoding.h),
// transform_precoder_dft_impl (lib/phy/generic_functions/transform_precoding/transform_precoder_dft_impl.cpp).
#include "srsran_amd/transform_precoding.h"
#include "srsran_amd/ldpc.h"

#include <hip/hip_runtime.h>

#include "api_common.h"
#include "device_buffer.h"
#include "transform_precoding_args.h"
#include <cmath>
#include <mutex>

using namespace srs_amd;

struct srs_amd_transform_precoder {
  int           device = 0;
  hipStream_t   stream = nullptr;
  device_buffer host_io;
  std::mutex    mtx;
  ~srs_amd_transform_precoder()
  {
    (void)hipSetDevice(device);
    if (stream) {
      (void)hipStreamSynchronize(stream);
      (void)hipStreamDestroy(stream);
    }
  }
};

namespace {

constexpr uint32_t MAX_NOF_PRBS = 275; // include/srsran/ran/resource_block.h

// M1: the divisor of M closest to sqrt(M) from below (the first pass sums M1 terms, the second M / M1).
uint32_t factor_of(uint32_t M)
{
  uint32_t best = 1;
  for (uint32_t d = 1; d * d <= M; ++d) {
    if (M % d == 0) {
      best = d;
    }
  }
  return best;
}

int check_size(uint32_t nof_subc)
{
  if (nof_subc == 0 || nof_subc % 12 != 0) {
    return fail(SRS_AMD_EINVAL, "The number of subcarriers (i.e., %u) must be muliple of 12.", nof_subc);
  }
  if (!srs_amd_transform_precoding_nof_prbs_valid(nof_subc / 12)) {
    return fail(SRS_AMD_EINVAL, "The number of PRB (i.e., %u) is not valid.", nof_subc / 12);
  }
  return SRS_AMD_OK;
}

} // namespace

extern "C" {

int srs_amd_transform_precoding_nof_prbs_valid(uint32_t nof_prb)
{
  if (nof_prb == 0 || nof_prb > MAX_NOF_PRBS) {
    return 0;
  }
  for (uint32_t f : {2u, 3u, 5u}) {
    while (nof_prb % f == 0) {
      nof_prb /= f;
    }
  }
  return nof_prb == 1 ? 1 : 0;
}

int srs_amd_transform_precoder_create(srs_amd_transform_precoder** tp, int device)
{
  if (tp == nullptr) {
    return fail(SRS_AMD_EINVAL, "null handle pointer");
  }
  *tp    = nullptr;
  int rc = select_device(device);
  if (rc != SRS_AMD_OK) {
    return rc;
  }
  auto* t      = new srs_amd_transform_precoder();
  t->device    = device;
  hipError_t e = hipStreamCreateWithFlags(&t->stream, hipStreamNonBlocking);
  if (e != hipSuccess) {
    delete t;
    return hip_fail(e, "transform precoder stream");
  }
  *tp = t;
  return SRS_AMD_OK;
}

void srs_amd_transform_precoder_destroy(srs_amd_transform_precoder* tp)
{
  delete tp;
}

int srs_amd_transform_deprecode_batch(srs_amd_transform_precoder* tp,
                                      float*                      d_symbols,
                                      uint64_t                    sym_stride,
                                      float*                      d_noise_vars,
                                      uint64_t                    nv_stride,
                                      uint32_t                    nof_subc,
                                      uint32_t                    nof_rows,
                                      void*                       stream)
{
  if (tp == nullptr) {
    return fail(SRS_AMD_EINVAL, "null transform precoder");
  }
  int rc = check_size(nof_subc);
  if (rc != SRS_AMD_OK) {
    return rc;
  }
  if (nof_rows == 0) {
    return SRS_AMD_OK;
  }
  if (d_symbols == nullptr) {
    return fail(SRS_AMD_EINVAL, "null device buffer");
  }
  if (nof_rows > 1 && (sym_stride < nof_subc || (d_noise_vars != nullptr && nv_stride < nof_subc))) {
    return fail(SRS_AMD_EINVAL, "row stride shorter than the symbol (%u subcarriers)", nof_subc);
  }
  tp_args a{};
  a.symbols    = reinterpret_cast<float2*>(d_symbols);
  a.sym_stride = sym_stride;
  a.noise      = d_noise_vars;
  a.nv_stride  = nv_stride;
  a.M          = nof_subc;
  a.M1         = factor_of(nof_subc);
  a.M2         = nof_subc / a.M1;
  a.nof_rows   = nof_rows;
  a.scale      = 1.0f / std::sqrt(static_cast<float>(nof_subc)); // transform_precoder_dft_impl.cpp:45
  std::lock_guard<std::mutex> lock(tp->mtx);
  hipError_t                  e = hipSetDevice(tp->device);
  if (e == hipSuccess) {
    e = launch_transform_deprecode(a, static_cast<hipStream_t>(stream));
  }
  return e == hipSuccess ? SRS_AMD_OK : hip_fail(e, "transform_deprecode_kernel launch");
}

// Host forms: one symbol through the device path (input uploaded, output downloaded, synchronous).
static int deprecode_host(srs_amd_transform_precoder* tp, float* out, const float* in, uint32_t nof_subc, bool noise)
{
  if (tp == nullptr || out == nullptr || in == nullptr) {
    return fail(SRS_AMD_EINVAL, "null argument");
  }
  int rc = check_size(nof_subc);
  if (rc != SRS_AMD_OK) {
    return rc;
  }
  const size_t bytes = (noise ? 1 : 2) * sizeof(float) * nof_subc;
  hipError_t   e     = hipSuccess;
  {
    std::lock_guard<std::mutex> lock(tp->mtx);
    e = hipSetDevice(tp->device);
    if (e == hipSuccess) {
      // noise form: a zero symbol in front, the variances after it
      e = tp->host_io.ensure(2 * sizeof(float) * nof_subc + bytes);
    }
    if (e == hipSuccess && noise) {
      e = hipMemsetAsync(tp->host_io.ptr, 0, 2 * sizeof(float) * nof_subc, tp->stream);
    }
    if (e == hipSuccess) {
      e = hipMemcpyAsync(tp->host_io.as<uint8_t>() + (noise ? 2 * sizeof(float) * nof_subc : 0), in, bytes,
                         hipMemcpyHostToDevice, tp->stream);
    }
  }
  if (e != hipSuccess) {
    return hip_fail(e, "transform deprecoder upload");
  }
  float* base = tp->host_io.as<float>();
  rc          = srs_amd_transform_deprecode_batch(tp, base, nof_subc, noise ? base + 2 * nof_subc : nullptr, nof_subc,
                                                  nof_subc, 1, tp->stream);
  if (rc != SRS_AMD_OK) {
    return rc;
  }
  e = hipMemcpyAsync(out, noise ? base + 2 * nof_subc : base, bytes, hipMemcpyDeviceToHost, tp->stream);
  if (e == hipSuccess) {
    e = hipStreamSynchronize(tp->stream);
  }
  return e == hipSuccess ? SRS_AMD_OK : hip_fail(e, "transform deprecoder download");
}

int srs_amd_transform_deprecode(srs_amd_transform_precoder* tp, float* out, const float* in, uint32_t nof_subc)
{
  return deprecode_host(tp, out, in, nof_subc, false);
}

int srs_amd_transform_deprecode_noise(srs_amd_transform_precoder* tp, float* out, const float* in, uint32_t nof_subc)
{
  return deprecode_host(tp, out, in, nof_subc, true);
}

} // extern "C"

int srs_amd::make_tp_args(float2* symbols, uint64_t sym_stride, float* noise, uint64_t nv_stride, uint32_t nof_subc,
                          uint32_t nof_rows, tp_args& a, size_t& lds)
{
  int rc = check_size(nof_subc);
  if (rc != SRS_AMD_OK) {
    return rc;
  }
  a            = tp_args{};
  a.symbols    = symbols;
  a.sym_stride = sym_stride;
  a.noise      = noise;
  a.nv_stride  = nv_stride;
  a.M          = nof_subc;
  a.M1         = factor_of(nof_subc);
  a.M2         = nof_subc / a.M1;
  a.nof_rows   = nof_rows;
  a.scale      = 1.0f / std::sqrt(static_cast<float>(nof_subc)); // transform_precoder_dft_impl.cpp:45
  lds          = (2 * a.M + a.M1 + a.M2) * sizeof(float2);
  return SRS_AMD_OK;
}
