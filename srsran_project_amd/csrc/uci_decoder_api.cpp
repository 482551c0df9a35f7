// uci_decoder_api.cpp -- C-ABI of the MI355X UCI decoder (include/srsran_amd/uci_decoder.h): the short-block
// detector kernel for 1-11 bits; for 12-1706 bits the codeblock segmentation of uci_decoder_impl.cpp:47-76
// (get_nof_uci_codeblocks, get_uci_crc_size), one polar chain launch per codeblock (polar.h, codes cached per
// (K', E')) and the CRC / filler kernel.
#include "srsran_amd/uci_decoder.h"
#include "srsran_amd/polar.h"

#include <hip/hip_runtime.h>

#include "api_common.h"
#include "device_buffer.h"
#include "uci_args.h"
#include <algorithm>
#include <map>
#include <mutex>
#include <utility>

using namespace srs_amd;

struct srs_amd_uci_decoder {
  int                                                  device = 0;
  hipStream_t                                          stream = nullptr;
  std::map<std::pair<uint32_t, uint32_t>, srs_amd_polar_code*> codes;
  device_buffer                                        cbs;     // decoded polar codeblocks
  device_buffer                                        host_io; // host single-call staging
  std::mutex                                           mtx;
  ~srs_amd_uci_decoder()
  {
    (void)hipSetDevice(device);
    if (stream) {
      (void)hipStreamSynchronize(stream);
      (void)hipStreamDestroy(stream);
    }
    for (auto& c : codes) {
      srs_amd_polar_code_destroy(c.second);
    }
  }
  // polar_code::set(K, E, 10, polar_code_ibil::present) (uci_decoder_impl.cpp:87)
  srs_amd_polar_code* code(uint32_t K, uint32_t E)
  {
    auto it = codes.find({K, E});
    if (it != codes.end()) {
      return it->second;
    }
    srs_amd_polar_code* c = nullptr;
    if (srs_amd_polar_code_create(&c, K, E, 10, 1, device) != SRS_AMD_OK) {
      return nullptr;
    }
    codes.emplace(std::make_pair(K, E), c);
    return c;
  }
};

namespace {

uint32_t crc_size(uint32_t A) // get_uci_crc_size (uci_info.h:54-65)
{
  return A < 12 ? 0u : (A < 20 ? 6u : 11u);
}

uint32_t nof_codeblocks(uint32_t A, uint32_t E) // get_nof_uci_codeblocks (uci_info.h:40-46)
{
  return ((A >= 360 && E >= 1088) || A >= 1013) ? 2u : 1u;
}

} // namespace

int srs_amd::uci_slot_build(srs_amd_uci_decoder* dec, const uci_slot_message* msgs, uint32_t n, uint8_t* d_cbs,
                            uci_slot_plan& out)
{
  out = uci_slot_plan{};
  std::lock_guard<std::mutex> lock(dec->mtx);
  for (uint32_t i = 0; i != n; ++i) {
    const uci_slot_message& m  = msgs[i];
    const uint32_t          qm = m.modulation < 2 ? 1u : static_cast<uint32_t>(m.modulation);
    if (m.K == 0 || m.K > 1706) {
      return fail(SRS_AMD_EINVAL, "Invalid UCI payload size %u.", m.K);
    }
    if (m.K <= 11) {
      out.shorts.push_back(uci_short_args{m.llrs, 0, m.msg, 0, m.status, 0, m.E, m.K, qm, m.pred, m.pred_val});
      continue;
    }
    // polar codeblocks (uci_decoder_impl.cpp:47-76), as srs_amd_uci_decode_batch
    const uint32_t C  = nof_codeblocks(m.K, m.E);
    const uint32_t L  = crc_size(m.K);
    const uint32_t A0 = m.K / C, E0 = m.E / C, F0 = m.K % C;
    const uint32_t A1 = (m.K + C - 1) / C, E1 = m.E / C;
    const uint32_t K0 = A0 + L + F0, K1 = A1 + L;
    if (E0 == 0) {
      return fail(SRS_AMD_EINVAL, "UCI codeword of %u bits too short.", m.E);
    }
    const uint64_t cb_stride = (std::max(K0, K1) + 63) / 64 * 64;
    uint8_t*       cbs       = d_cbs + out.cb_bytes;
    for (uint32_t r = 0; r != C; ++r) {
      srs_amd_polar_code* c = dec->code(r == 0 ? K0 : K1, r == 0 ? E0 : E1);
      if (c == nullptr) {
        return SRS_AMD_EINVAL; // the polar code reported why
      }
      polar_args a = polar_code_base(c);
      a.llrs       = m.llrs + r * E0;
      a.msgs_out   = cbs + r * cb_stride;
      a.llr_stride = r == 0 ? E0 : E1;
      a.msg_stride = static_cast<uint32_t>(cb_stride);
      a.nof        = 1;
      a.pred       = m.pred;
      a.pred_val   = m.pred_val;
      out.polars.push_back(a);
    }
    out.finishes.push_back(uci_polar_args{cbs, cb_stride, m.msg, 0, m.status, 0, C, A0, F0, A1, L, m.pred, m.pred_val});
    out.cb_bytes += C * cb_stride;
  }
  return SRS_AMD_OK;
}

extern "C" {

int srs_amd_uci_decoder_create(srs_amd_uci_decoder** dec, int device)
{
  if (dec == nullptr) {
    return fail(SRS_AMD_EINVAL, "null handle pointer");
  }
  *dec   = nullptr;
  int rc = select_device(device);
  if (rc != SRS_AMD_OK) {
    return rc;
  }
  auto* d      = new srs_amd_uci_decoder();
  d->device    = device;
  hipError_t e = hipStreamCreateWithFlags(&d->stream, hipStreamNonBlocking);
  if (e != hipSuccess) {
    delete d;
    return hip_fail(e, "UCI decoder stream");
  }
  *dec = d;
  return SRS_AMD_OK;
}

void srs_amd_uci_decoder_destroy(srs_amd_uci_decoder* dec)
{
  delete dec;
}

int srs_amd_uci_decode_batch(srs_amd_uci_decoder* dec,
                             const int8_t*        d_llrs,
                             uint64_t             llr_stride,
                             uint32_t             E,
                             uint32_t             K,
                             int32_t              modulation,
                             uint8_t*             d_messages,
                             uint64_t             msg_stride,
                             int32_t*             d_status,
                             uint64_t             status_stride,
                             uint32_t             nof,
                             void*                stream)
{
  if (dec == nullptr) {
    return fail(SRS_AMD_EINVAL, "null decoder");
  }
  if (K == 0 || K > 1706) {
    return fail(SRS_AMD_EINVAL, "Invalid UCI payload size %u.", K);
  }
  if (!(modulation == 0 || modulation == 1 || modulation == 2 || modulation == 4 || modulation == 6 ||
        modulation == 8)) {
    return fail(SRS_AMD_EINVAL, "Invalid modulation %d.", modulation);
  }
  if (nof == 0) {
    return SRS_AMD_OK;
  }
  if (d_llrs == nullptr || d_messages == nullptr || d_status == nullptr || (nof > 1 && (llr_stride < E ||
                                                                                        msg_stride < K))) {
    return fail(SRS_AMD_EINVAL, "invalid device buffers or strides");
  }
  auto           s  = static_cast<hipStream_t>(stream);
  const uint32_t qm = modulation < 2 ? 1u : static_cast<uint32_t>(modulation);
  std::lock_guard<std::mutex> lock(dec->mtx);
  hipError_t                  e = hipSetDevice(dec->device);
  if (e != hipSuccess) {
    return hip_fail(e, "UCI decoder device");
  }
  if (K <= 11) {
    uci_short_args a{d_llrs, llr_stride, d_messages, msg_stride, d_status, status_stride, E, K, qm};
    e = launch_uci_short(a, nof, s);
    return e == hipSuccess ? SRS_AMD_OK : hip_fail(e, "uci_short_kernel launch");
  }
  // polar codeblocks (uci_decoder_impl.cpp:47-76)
  const uint32_t C  = nof_codeblocks(K, E);
  const uint32_t L  = crc_size(K);
  const uint32_t A0 = K / C, E0 = E / C, F0 = K % C;
  const uint32_t A1 = (K + C - 1) / C, E1 = E / C;
  const uint32_t K0 = A0 + L + F0, K1 = A1 + L;
  if (E0 == 0) {
    return fail(SRS_AMD_EINVAL, "UCI codeword of %u bits too short.", E);
  }
  srs_amd_polar_code* c0 = dec->code(K0, E0);
  srs_amd_polar_code* c1 = C > 1 ? dec->code(K1, E1) : nullptr;
  if (c0 == nullptr || (C > 1 && c1 == nullptr)) {
    return SRS_AMD_EINVAL; // the polar code reported why
  }
  const uint64_t cb_stride = (std::max(K0, K1) + 63) / 64 * 64;
  e                        = dec->cbs.ensure(static_cast<size_t>(nof) * C * cb_stride);
  if (e != hipSuccess) {
    return hip_fail(e, "UCI decoder scratch");
  }
  auto* cbs = dec->cbs.as<uint8_t>();
  // codeblock r of message i at row i * C + r
  int rc = srs_amd_polar_decode_batch(c0, d_llrs, static_cast<uint32_t>(nof > 1 ? llr_stride : E), cbs,
                                      static_cast<uint32_t>(C * cb_stride), nof, stream);
  if (rc == SRS_AMD_OK && C > 1) {
    rc = srs_amd_polar_decode_batch(c1, d_llrs + E0, static_cast<uint32_t>(nof > 1 ? llr_stride : E), cbs + cb_stride,
                                    static_cast<uint32_t>(C * cb_stride), nof, stream);
  }
  if (rc != SRS_AMD_OK) {
    return rc;
  }
  uci_polar_args a{cbs, cb_stride, d_messages, msg_stride, d_status, status_stride, C, A0, F0, A1, L};
  e = launch_uci_polar_finish(a, nof, s);
  return e == hipSuccess ? SRS_AMD_OK : hip_fail(e, "uci_polar_finish_kernel launch");
}

int srs_amd_uci_decode(srs_amd_uci_decoder* dec, uint8_t* message, uint32_t K, const int8_t* llrs, uint32_t E,
                       int32_t modulation)
{
  if (dec == nullptr || message == nullptr || (llrs == nullptr && E != 0)) {
    return fail(SRS_AMD_EINVAL, "null argument");
  }
  const size_t o_msg = align_up(std::max<size_t>(E, 1), 256), o_st = o_msg + align_up(std::max<size_t>(K, 1), 256);
  hipError_t   e;
  {
    std::lock_guard<std::mutex> lock(dec->mtx);
    e = hipSetDevice(dec->device);
    if (e == hipSuccess) {
      e = dec->host_io.ensure(o_st + 256);
    }
  }
  if (e != hipSuccess) {
    return hip_fail(e, "UCI decoder buffers");
  }
  auto* b = dec->host_io.as<uint8_t>();
  if (E != 0) {
    e = hipMemcpyAsync(b, llrs, E, hipMemcpyHostToDevice, dec->stream);
  }
  if (e != hipSuccess) {
    return hip_fail(e, "UCI decoder upload");
  }
  int rc = srs_amd_uci_decode_batch(dec, reinterpret_cast<int8_t*>(b), E, E, K, modulation, b + o_msg, K,
                                    reinterpret_cast<int32_t*>(b + o_st), 4, 1, dec->stream);
  if (rc != SRS_AMD_OK) {
    (void)hipStreamSynchronize(dec->stream);
    return rc;
  }
  int32_t status = 0;
  e              = hipMemcpyAsync(message, b + o_msg, K, hipMemcpyDeviceToHost, dec->stream);
  if (e == hipSuccess) {
    e = hipMemcpyAsync(&status, b + o_st, 4, hipMemcpyDeviceToHost, dec->stream);
  }
  if (e == hipSuccess) {
    e = hipStreamSynchronize(dec->stream);
  }
  return e == hipSuccess ? status : hip_fail(e, "UCI decoder download");
}

int32_t srs_amd_uci_part2_get_size(const uint8_t*                            part1,
                                   uint32_t                                  nof_part1_bits,
                                   const srs_amd_uci_part2_size_description* descr)
{
  if (descr == nullptr || descr->nof_entries > 2 || (nof_part1_bits != 0 && part1 == nullptr)) {
    return -1;
  }
  uint32_t result = 0;
  for (uint32_t e = 0; e < descr->nof_entries; ++e) {
    const srs_amd_uci_part2_entry& en = descr->entries[e];
    if (en.nof_parameters > 2) {
      return -1;
    }
    uint32_t index = 0, bits = 0;
    for (uint32_t q = 0; q < en.nof_parameters; ++q) {
      const srs_amd_uci_part2_parameter& prm = en.parameters[q];
      if (static_cast<uint32_t>(prm.offset) + prm.width > nof_part1_bits) {
        return -1;
      }
      uint32_t value = 0; // the field's first bit is its most significant (extract_parameter, :28-51)
      for (uint32_t b = 0; b < prm.width; ++b) {
        value = (value << 1) | (part1[prm.offset + b] & 1u);
      }
      index = (index << prm.width) | value;
      bits += prm.width;
    }
    if (bits > 4 || en.map_size != (1u << bits) || index >= en.map_size) {
      return -1;
    }
    result += en.map[index];
  }
  return static_cast<int32_t>(result);
}

} // extern "C"
