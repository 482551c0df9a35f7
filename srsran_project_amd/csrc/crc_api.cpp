// crc_api.cpp -- C-ABI of the MI355X CRC calculator (include/srsran_amd/crc.h).
// Replaces crc_calculator::calculate (crc_calculator.h:81) of
// crc_calculator_generic_impl.cpp and the codeblock CRC attachment of the
// LDPC segmenter (ldpc_segmenter_impl.cpp, TS 38.212 5.2.2).
#include "srsran_amd/crc.h"

#include <hip/hip_runtime.h>

#include "api_common.h"
#include "crc_args.h"
#include "crc_internal.h"
#include "ldpc_common.h"
#include <mutex>
#include <vector>

using namespace srs_amd;

struct srs_amd_crc_calculator {
  int         device   = 0;
  int         poly     = 0;
  uint32_t    polynom  = 0;
  int         order    = 0;
  uint32_t    max_bits = 0;
  uint32_t*   d_table  = nullptr;
  hipStream_t stream   = nullptr;
  void*       scratch  = nullptr;
  size_t      scratch_size = 0;
  uint32_t*   d_acc        = nullptr; // per-row accumulators of the long-row path
  uint32_t    acc_rows     = 0;
  std::mutex  mtx;
  ~srs_amd_crc_calculator()
  {
    (void)hipSetDevice(device);
    if (stream) {
      (void)hipStreamSynchronize(stream);
      (void)hipStreamDestroy(stream);
    }
    (void)hipFree(d_table);
    (void)hipFree(scratch);
    (void)hipFree(d_acc);
  }
};

namespace {

int check_rows(srs_amd_crc_calculator* crc, uint32_t stride, uint32_t nof_bits, uint32_t extra)
{
  if (crc == nullptr) {
    return fail(SRS_AMD_EINVAL, "null CRC calculator");
  }
  if (nof_bits > crc->max_bits) {
    return fail(SRS_AMD_EINVAL, "message of %u bits exceeds the calculator's %u", nof_bits, crc->max_bits);
  }
  if (static_cast<uint64_t>(stride) * 8 < static_cast<uint64_t>(nof_bits) + extra) {
    return fail(SRS_AMD_EINVAL, "row stride %u bytes too small for %u bits", stride, nof_bits + extra);
  }
  return SRS_AMD_OK;
}

int launch(srs_amd_crc_calculator* crc, uint32_t* d_out, uint8_t* d_bits, uint32_t stride, uint32_t nof_bits,
           uint32_t nof_rows, bool attach, hipStream_t stream)
{
  crc_args a{};
  a.bits      = d_bits;
  a.checksums = d_out;
  a.table     = crc->d_table;
  a.stride    = stride;
  a.nof_bits  = nof_bits;
  a.polynom   = crc->polynom;
  a.order     = static_cast<uint32_t>(crc->order);
  a.attach    = attach ? 1 : 0;
  hipError_t e = hipSetDevice(crc->device);
  if (e == hipSuccess && crc_needs_accumulator(nof_bits)) {
    // One accumulator per row (the caller holds crc->mtx); grown only (hipFree waits for
    // the device), calls on one calculator are serialised by the caller's stream order.
    if (crc->acc_rows < nof_rows) {
      (void)hipFree(crc->d_acc);
      crc->d_acc    = nullptr;
      crc->acc_rows = 0;
      e             = hipMalloc(&crc->d_acc, sizeof(uint32_t) * nof_rows);
      if (e == hipSuccess) {
        crc->acc_rows = nof_rows;
      }
    }
    a.acc = crc->d_acc;
  }
  if (e == hipSuccess) {
    e = launch_crc(a, nof_rows, stream);
  }
  return e == hipSuccess ? SRS_AMD_OK : hip_fail(e, "crc_kernel launch");
}

} // namespace

extern "C" {

int srs_amd_crc_calculator_create(srs_amd_crc_calculator** out, int poly, uint32_t max_bits, int device)
{
  if (out == nullptr) {
    return fail(SRS_AMD_EINVAL, "null handle pointer");
  }
  *out             = nullptr;
  uint32_t polynom = 0;
  int      order   = 0;
  if (!crc_params(poly, polynom, order)) {
    return fail(SRS_AMD_EINVAL, "Invalid CRC polynomial %d.", poly);
  }
  if (max_bits == 0 || max_bits > (1u << 26)) {
    return fail(SRS_AMD_EINVAL, "max_bits %u out of range", max_bits);
  }
  int rc = select_device(device);
  if (rc != SRS_AMD_OK) {
    return rc;
  }
  auto* c     = new srs_amd_crc_calculator();
  c->device   = device;
  c->poly     = poly;
  c->polynom  = polynom;
  c->order    = order;
  c->max_bits = max_bits;
  std::vector<uint32_t> t = crc_linear_table(poly, static_cast<int>(max_bits) + 32);
  hipError_t            e = hipMalloc(&c->d_table, t.size() * sizeof(uint32_t));
  if (e == hipSuccess) {
    e = hipMemcpy(c->d_table, t.data(), t.size() * sizeof(uint32_t), hipMemcpyHostToDevice);
  }
  if (e == hipSuccess) {
    e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
  }
  if (e != hipSuccess) {
    delete c;
    return hip_fail(e, "CRC table");
  }
  *out = c;
  return SRS_AMD_OK;
}

void srs_amd_crc_calculator_destroy(srs_amd_crc_calculator* crc)
{
  delete crc;
}

uint32_t srs_amd_crc_order(const srs_amd_crc_calculator* crc)
{
  return crc ? static_cast<uint32_t>(crc->order) : 0;
}

int srs_amd_crc_calculate_batch(srs_amd_crc_calculator* crc,
                                uint32_t*               d_checksums,
                                const uint8_t*          d_bits,
                                uint32_t                stride,
                                uint32_t                nof_bits,
                                uint32_t                nof_rows,
                                void*                   stream)
{
  int rc = check_rows(crc, stride, nof_bits, 0);
  if (rc != SRS_AMD_OK) {
    return rc;
  }
  if (nof_rows == 0) {
    return SRS_AMD_OK;
  }
  if (d_checksums == nullptr || (d_bits == nullptr && nof_bits > 0)) {
    return fail(SRS_AMD_EINVAL, "null device buffer");
  }
  std::lock_guard<std::mutex> lock(crc->mtx);
  return launch(crc, d_checksums, const_cast<uint8_t*>(d_bits), stride, nof_bits, nof_rows, false,
                static_cast<hipStream_t>(stream));
}

int srs_amd_crc_attach_batch(srs_amd_crc_calculator* crc,
                             uint8_t*                d_bits,
                             uint32_t                stride,
                             uint32_t                nof_bits,
                             uint32_t                nof_rows,
                             void*                   stream)
{
  int rc = check_rows(crc, stride, nof_bits, crc ? static_cast<uint32_t>(crc->order) : 0);
  if (rc != SRS_AMD_OK) {
    return rc;
  }
  if (nof_rows == 0) {
    return SRS_AMD_OK;
  }
  if (d_bits == nullptr) {
    return fail(SRS_AMD_EINVAL, "null device buffer");
  }
  std::lock_guard<std::mutex> lock(crc->mtx);
  return launch(crc, nullptr, d_bits, stride, nof_bits, nof_rows, true, static_cast<hipStream_t>(stream));
}

int srs_amd_crc_calculate(srs_amd_crc_calculator* crc, uint32_t* checksum, const uint8_t* bits, uint32_t nof_bits)
{
  const uint32_t nbytes = (nof_bits + 7) / 8;
  int            rc     = check_rows(crc, nbytes, nof_bits, 0);
  if (rc != SRS_AMD_OK) {
    return rc;
  }
  if (checksum == nullptr || (bits == nullptr && nof_bits > 0)) {
    return fail(SRS_AMD_EINVAL, "null argument");
  }
  std::lock_guard<std::mutex> lock(crc->mtx);
  hipError_t                  e = hipSetDevice(crc->device);
  const size_t                need = 64 + nbytes;
  if (e == hipSuccess && need > crc->scratch_size) {
    (void)hipFree(crc->scratch);
    crc->scratch      = nullptr;
    crc->scratch_size = 0;
    e                 = hipMalloc(&crc->scratch, need);
    if (e == hipSuccess) {
      crc->scratch_size = need;
    }
  }
  if (e != hipSuccess) {
    return hip_fail(e, "CRC scratch");
  }
  auto* d_crc  = static_cast<uint32_t*>(crc->scratch);
  auto* d_bits = static_cast<uint8_t*>(crc->scratch) + 64;
  if (nbytes > 0) {
    e = hipMemcpyAsync(d_bits, bits, nbytes, hipMemcpyHostToDevice, crc->stream);
  }
  if (e != hipSuccess) {
    return hip_fail(e, "CRC upload");
  }
  rc = launch(crc, d_crc, d_bits, nbytes, nof_bits, 1, false, crc->stream);
  if (rc != SRS_AMD_OK) {
    return rc;
  }
  e = hipMemcpyAsync(checksum, d_crc, sizeof(uint32_t), hipMemcpyDeviceToHost, crc->stream);
  if (e == hipSuccess) {
    e = hipStreamSynchronize(crc->stream);
  }
  return e == hipSuccess ? SRS_AMD_OK : hip_fail(e, "CRC download");
}

} // extern "C"

const uint32_t* srs_amd::crc_device_table(const srs_amd_crc_calculator* crc)
{
  return crc ? crc->d_table : nullptr;
}

uint32_t srs_amd::crc_polynom(const srs_amd_crc_calculator* crc)
{
  return crc ? crc->polynom : 0;
}

uint32_t srs_amd::crc_order(const srs_amd_crc_calculator* crc)
{
  return crc ? static_cast<uint32_t>(crc->order) : 0;
}
