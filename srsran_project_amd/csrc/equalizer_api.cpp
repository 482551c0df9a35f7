// equalizer_api.cpp -- C-ABI of the MI355X channel equalizer (include/srsran_amd/equalizer.h).
//
// Host-side logic follows channel_equalizer_generic_impl.cpp: is_supported
// (:240-270), the assertions of assert_sizes (:36-100) and tx_scaling > 0
// (:296), the per-port validity of the 1-layer path (:131) and the
// most-pessimistic noise variance of the 2-layer path (:304).
#include "srsran_amd/equalizer.h"

#include <hip/hip_runtime.h>

#include "api_common.h"
#include "equalizer_args.h"
#include <algorithm>
#include <cmath>
#include <mutex>

using namespace srs_amd;

struct srs_amd_channel_equalizer {
  int         algorithm = SRS_AMD_EQ_ZF;
  int         device    = 0;
  hipStream_t stream    = nullptr;
  void*       scratch   = nullptr;
  size_t      scratch_size = 0;
  std::mutex  mtx;
  ~srs_amd_channel_equalizer()
  {
    (void)hipSetDevice(device);
    if (stream) {
      (void)hipStreamSynchronize(stream);
      (void)hipStreamDestroy(stream);
    }
    (void)hipFree(scratch);
  }
};

namespace {

bool supported(int algorithm, uint32_t nof_ports, uint32_t nof_layers)
{
  if (nof_ports != 1 && nof_ports != 2 && nof_ports != 4) {
    return false;
  }
  if (nof_ports < nof_layers) {
    return false;
  }
  // channel_equalizer_generic_impl.cpp:240-270 allows ZF for 1-2 layers and MMSE for 1; the L-layer
  // solves of equalizer_device.h add ZF 3 x 4 / 4 x 4 and MMSE 2 x N / 3 x 4 / 4 x 4 (parity unpinned:
  // the open reference asserts for them, channel_equalizer_generic_impl.cpp:197-247).
  return nof_layers >= 1 && nof_layers <= 4 && (algorithm == SRS_AMD_EQ_ZF || algorithm == SRS_AMD_EQ_MMSE);
}

int make_args(equalizer_args& a, const srs_amd_channel_equalizer* eq, const float* nvars, uint32_t nof_re,
              uint32_t nof_ports, uint32_t nof_layers, float tx_scaling)
{
  if (eq == nullptr || nvars == nullptr) {
    return fail(SRS_AMD_EINVAL, "null argument");
  }
  if (!supported(eq->algorithm, nof_ports, nof_layers)) {
    return fail(SRS_AMD_EINVAL,
                "Invalid combination of channel spatial topology (i.e., %u Rx ports, %u Tx layers) and algorithm "
                "(i.e., %s).",
                nof_ports, nof_layers, eq->algorithm == SRS_AMD_EQ_ZF ? "ZF" : "MMSE");
  }
  if (!(tx_scaling > 0)) {
    return fail(SRS_AMD_EINVAL, "Tx scaling factor must be positive.");
  }
  a            = equalizer_args{};
  a.nof_re     = nof_re;
  a.tx_scaling = tx_scaling;
  for (uint32_t p = 0; p < nof_ports; ++p) {
    a.port_noise_var[p] = nvars[p];
    if (std::isnormal(nvars[p]) && nvars[p] > 0) {
      a.valid_ports |= 1u << p;
    }
  }
  a.noise_var = *std::max_element(nvars, nvars + nof_ports);
  a.noise_ok  = (std::isnormal(a.noise_var) && a.noise_var >= 0.0F) ? 1 : 0;
  a.mmse      = eq->algorithm == SRS_AMD_EQ_MMSE ? 1 : 0;
  return SRS_AMD_OK;
}

} // namespace

extern "C" {

int srs_amd_channel_equalizer_create(srs_amd_channel_equalizer** eq, int algorithm, int device)
{
  if (eq == nullptr) {
    return fail(SRS_AMD_EINVAL, "null handle pointer");
  }
  *eq = nullptr;
  if (algorithm != SRS_AMD_EQ_ZF && algorithm != SRS_AMD_EQ_MMSE) {
    return fail(SRS_AMD_EINVAL, "invalid equalizer algorithm %d", algorithm);
  }
  int rc = select_device(device);
  if (rc != SRS_AMD_OK) {
    return rc;
  }
  auto* h      = new srs_amd_channel_equalizer();
  h->algorithm = algorithm;
  h->device    = device;
  hipError_t e = hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking);
  if (e != hipSuccess) {
    delete h;
    return hip_fail(e, "hipStreamCreate");
  }
  *eq = h;
  return SRS_AMD_OK;
}

void srs_amd_channel_equalizer_destroy(srs_amd_channel_equalizer* eq)
{
  delete eq;
}

int srs_amd_channel_equalizer_is_supported(const srs_amd_channel_equalizer* eq, uint32_t nof_ports, uint32_t nof_layers)
{
  return (eq != nullptr && supported(eq->algorithm, nof_ports, nof_layers)) ? 1 : 0;
}

int srs_amd_channel_equalize_batch(srs_amd_channel_equalizer* eq,
                                   float*                     d_eq_symbols,
                                   float*                     d_eq_noise_vars,
                                   const uint16_t*            d_ch_symbols,
                                   const uint16_t*            d_ch_estimates,
                                   const float*               noise_var_estimates,
                                   uint32_t                   nof_re,
                                   uint32_t                   nof_ports,
                                   uint32_t                   nof_layers,
                                   float                      tx_scaling,
                                   void*                      stream)
{
  equalizer_args a;
  int rc = make_args(a, eq, noise_var_estimates, nof_re, nof_ports, nof_layers, tx_scaling);
  if (rc != SRS_AMD_OK) {
    return rc;
  }
  if (nof_re == 0) {
    return SRS_AMD_OK;
  }
  if (d_eq_symbols == nullptr || d_eq_noise_vars == nullptr || d_ch_symbols == nullptr || d_ch_estimates == nullptr) {
    return fail(SRS_AMD_EINVAL, "null device buffer");
  }
  a.symbols       = d_ch_symbols;
  a.estimates     = d_ch_estimates;
  a.eq_symbols    = d_eq_symbols;
  a.eq_noise_vars = d_eq_noise_vars;
  std::lock_guard<std::mutex> lock(eq->mtx);
  hipError_t                  e = hipSetDevice(eq->device);
  if (e == hipSuccess) {
    e = launch_equalizer(a, nof_ports, nof_layers, static_cast<hipStream_t>(stream));
  }
  return e == hipSuccess ? SRS_AMD_OK : hip_fail(e, "equalizer kernel launch");
}

int srs_amd_channel_equalize(srs_amd_channel_equalizer* eq,
                             float*                     eq_symbols,
                             float*                     eq_noise_vars,
                             const uint16_t*            ch_symbols,
                             const uint16_t*            ch_estimates,
                             const float*               noise_var_estimates,
                             uint32_t                   nof_re,
                             uint32_t                   nof_ports,
                             uint32_t                   nof_layers,
                             float                      tx_scaling)
{
  equalizer_args a;
  int rc = make_args(a, eq, noise_var_estimates, nof_re, nof_ports, nof_layers, tx_scaling);
  if (rc != SRS_AMD_OK) {
    return rc;
  }
  if (nof_re == 0) {
    return SRS_AMD_OK;
  }
  if (eq_symbols == nullptr || eq_noise_vars == nullptr || ch_symbols == nullptr || ch_estimates == nullptr) {
    return fail(SRS_AMD_EINVAL, "null argument");
  }
  const size_t sym_b = static_cast<size_t>(nof_ports) * nof_re * 4;
  const size_t est_b = static_cast<size_t>(nof_layers) * sym_b;
  const size_t eq_b  = static_cast<size_t>(nof_re) * nof_layers * 8;
  const size_t nv_b  = static_cast<size_t>(nof_re) * nof_layers * 4;
  uint8_t*     base  = nullptr;
  {
    std::lock_guard<std::mutex> lock(eq->mtx);
    hipError_t                  e = hipSetDevice(eq->device);
    const size_t                need = sym_b + est_b + eq_b + nv_b + 64;
    if (e == hipSuccess && need > eq->scratch_size) {
      (void)hipFree(eq->scratch);
      eq->scratch      = nullptr;
      eq->scratch_size = 0;
      e                = hipMalloc(&eq->scratch, need);
      if (e == hipSuccess) {
        eq->scratch_size = need;
      }
    }
    base = static_cast<uint8_t*>(eq->scratch);
    if (e == hipSuccess) {
      e = hipMemcpyAsync(base, ch_symbols, sym_b, hipMemcpyHostToDevice, eq->stream);
    }
    if (e == hipSuccess) {
      e = hipMemcpyAsync(base + sym_b, ch_estimates, est_b, hipMemcpyHostToDevice, eq->stream);
    }
    if (e != hipSuccess) {
      return hip_fail(e, "staging equalizer inputs");
    }
  }
  // eq symbols need 16 B alignment for two layers
  const size_t eq_off = (sym_b + est_b + 15) / 16 * 16;
  rc = srs_amd_channel_equalize_batch(eq, reinterpret_cast<float*>(base + eq_off),
                                      reinterpret_cast<float*>(base + eq_off + eq_b),
                                      reinterpret_cast<const uint16_t*>(base),
                                      reinterpret_cast<const uint16_t*>(base + sym_b), noise_var_estimates, nof_re,
                                      nof_ports, nof_layers, tx_scaling, eq->stream);
  if (rc != SRS_AMD_OK) {
    return rc;
  }
  hipError_t e = hipMemcpyAsync(eq_symbols, base + eq_off, eq_b, hipMemcpyDeviceToHost, eq->stream);
  if (e == hipSuccess) {
    e = hipMemcpyAsync(eq_noise_vars, base + eq_off + eq_b, nv_b, hipMemcpyDeviceToHost, eq->stream);
  }
  if (e == hipSuccess) {
    e = hipStreamSynchronize(eq->stream);
  }
  return e == hipSuccess ? SRS_AMD_OK : hip_fail(e, "channel equalize");
}

} // extern "C"
