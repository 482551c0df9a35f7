// pdsch_api.cpp -- C-ABI of the MI355X PDSCH encoder (include/srsran_amd/sch.h),
// pdsch_encoder_impl::encode (lib/phy/upper/channel_processors/pdsch/pdsch_encoder_impl.cpp:28-80)
// for a batch of transport blocks:
//   1. TB CRC (CRC16 / CRC24A)            crc kernel over the TB rows
//   2. segmentation                       segment_kernel (sch.hip)
//   3. CB CRC24B attachment (C > 1)       crc kernel, in place
//   4. LDPC encoding                      srs_amd_ldpc_encode_batch
//   5. rate matching + concatenation      srs_amd_ldpc_rate_match_batch into the codeword rows
#include "srsran_amd/crc.h"
#include "srsran_amd/ldpc_encoder.h"
#include "srsran_amd/ldpc_rate_matching.h"
#include "srsran_amd/sch.h"

#include <hip/hip_runtime.h>

#include "api_common.h"
#include "crc_internal.h"
#include "device_buffer.h"
#include "ldpc_codec_internal.h"
#include "rate_matching_common.h"
#include "sch_args.h"
#include <algorithm>
#include <cstring>
#include <mutex>
#include <vector>

using namespace srs_amd;

struct srs_amd_pdsch_encoder {
  int                        device = 0;
  hipStream_t                stream = nullptr;
  srs_amd_crc_calculator*    crc16  = nullptr;
  srs_amd_crc_calculator*    crc24a = nullptr;
  srs_amd_crc_calculator*    crc24b = nullptr;
  srs_amd_ldpc_encoder*      enc    = nullptr;
  srs_amd_ldpc_rate_matcher* rm     = nullptr;
  device_buffer              tb_crcs, msgs, coded, rm_arrays, host_io;
  stream_order               order; // scratch reuse across the callers' streams
  std::mutex                 mtx;
  ~srs_amd_pdsch_encoder()
  {
    (void)hipSetDevice(device);
    if (stream) {
      (void)hipStreamSynchronize(stream);
      (void)hipStreamDestroy(stream);
    }
    srs_amd_crc_calculator_destroy(crc16);
    srs_amd_crc_calculator_destroy(crc24a);
    srs_amd_crc_calculator_destroy(crc24b);
    srs_amd_ldpc_encoder_destroy(enc);
    srs_amd_ldpc_rate_matcher_destroy(rm);
  }
};

namespace {

int check_plan(const srs_amd_sch_plan* p)
{
  if (p == nullptr || p->nof_segments == 0 || p->lifting_size == 0) {
    return fail(SRS_AMD_EINVAL, "plan not computed (srs_amd_sch_plan_compute)");
  }
  return SRS_AMD_OK;
}

int encode_locked(srs_amd_pdsch_encoder* e,
                  const srs_amd_sch_plan* p,
                  uint8_t*                d_cw,
                  uint32_t                cw_stride,
                  const uint8_t*          d_tbs,
                  uint32_t                tb_stride,
                  uint32_t                nof_tbs,
                  hipStream_t             stream)
{
  const uint32_t C          = p->nof_segments;
  const uint32_t rows       = nof_tbs * C;
  const uint32_t K          = p->segment_length;
  const uint32_t msg_stride = static_cast<uint32_t>(align_up((K + 7) / 8, 64));
  const uint32_t N          = srs_amd_ldpc_codeblock_length(p->base_graph, p->lifting_size);
  const uint32_t cb_stride  = static_cast<uint32_t>(align_up((N + 7) / 8, 64));
  hipError_t     he         = hipSetDevice(e->device);
  if (he == hipSuccess) {
    he = e->tb_crcs.ensure(sizeof(uint32_t) * nof_tbs);
  }
  if (he == hipSuccess) {
    he = e->msgs.ensure(static_cast<size_t>(rows) * msg_stride);
  }
  if (he == hipSuccess) {
    he = e->coded.ensure(static_cast<size_t>(rows) * cb_stride);
  }
  if (he == hipSuccess) {
    he = e->rm_arrays.ensure(sizeof(uint32_t) * 2 * rows);
  }
  if (he != hipSuccess) {
    return hip_fail(he, "PDSCH encoder scratch");
  }
  // Rate-matching lengths and codeword offsets, uploaded when the geometry changes.
  he = e->order.begin(stream);
  if (he == hipSuccess) {
    he = launch_rm_arrays(e->rm_arrays.as<uint32_t>(), nof_tbs, C, p->nof_short_segments, p->rm_length_short,
                          p->rm_length_long, cw_stride * 8, stream);
  }
  if (he != hipSuccess) {
    return hip_fail(he, "PDSCH encoder rate-matching arrays");
  }
  // 1. TB CRC.
  srs_amd_crc_calculator* tbcrc = p->nof_tb_crc_bits == 16 ? e->crc16 : e->crc24a;
  int rc = srs_amd_crc_calculate_batch(tbcrc, e->tb_crcs.as<uint32_t>(), d_tbs, tb_stride, p->tbs, nof_tbs, stream);
  if (rc != SRS_AMD_OK) {
    return rc;
  }
  // 2. Segmentation.
  segment_args sa{};
  sa.tbs            = d_tbs;
  sa.tb_crcs        = e->tb_crcs.as<uint32_t>();
  sa.msgs           = e->msgs.as<uint8_t>();
  sa.tb_stride      = tb_stride;
  sa.msg_stride     = msg_stride;
  sa.msg_bytes      = (K + 7) / 8;
  sa.nof_segments   = C;
  sa.cb_info_bits   = p->cb_info_bits;
  sa.last_data_bits = p->cb_info_bits - p->nof_tb_crc_bits - p->zero_pad;
  sa.tb_crc_bits    = p->nof_tb_crc_bits;
  sa.nof_rows       = rows;
  he                = launch_segment(sa, stream);
  if (he != hipSuccess) {
    return hip_fail(he, "segment_kernel launch");
  }
  // 3. Codeblock CRC.
  if (C > 1) {
    rc = srs_amd_crc_attach_batch(e->crc24b, e->msgs.as<uint8_t>(), msg_stride, p->cb_info_bits, rows, stream);
    if (rc != SRS_AMD_OK) {
      return rc;
    }
  }
  // 4. LDPC encoding.
  // Only the circular-buffer window the rate matcher reads, [0, k0 + E + F) capped at Ncb
  // (ldpc_rate_matcher_impl.cpp:95-130), is encoded.
  srs_amd_ldpc_encoder_config ec{p->base_graph, p->lifting_size, p->Nref};
  rm_geometry                 rg{};
  uint32_t                    max_bits = 0xffffffffu;
  if (make_rm_geometry(rg, p->base_graph, p->lifting_size, p->rv, p->modulation_order, p->Nref,
                       p->nof_filler_bits) == nullptr) {
    const uint64_t window = static_cast<uint64_t>(rg.k0) + std::max(p->rm_length_long, p->rm_length_short) + rg.F;
    max_bits              = window >= rg.Ncb ? rg.Ncb : static_cast<uint32_t>(window);
  }
  rc = ldpc_encode_batch_ex(e->enc, &ec, e->msgs.as<uint8_t>(), msg_stride, e->coded.as<uint8_t>(), cb_stride, rows,
                            stream, max_bits);
  if (rc != SRS_AMD_OK) {
    return rc;
  }
  // 5. Rate matching into the codeword rows.
  srs_amd_codeblock_metadata md{p->base_graph, p->lifting_size, p->rv, p->modulation_order, p->Nref,
                                p->nof_filler_bits};
  rc = srs_amd_ldpc_rate_match_batch(e->rm, &md, e->coded.as<uint8_t>(), cb_stride, e->rm_arrays.as<uint32_t>(),
                                     e->rm_arrays.as<uint32_t>() + rows, p->rm_length_long, d_cw, rows, stream);
  if (rc != SRS_AMD_OK) {
    return rc;
  }
  he = e->order.end(stream);
  return he == hipSuccess ? SRS_AMD_OK : hip_fail(he, "PDSCH encoder completion event");
}

} // namespace

extern "C" {

int srs_amd_pdsch_encoder_create(srs_amd_pdsch_encoder** out, int device)
{
  if (out == nullptr) {
    return fail(SRS_AMD_EINVAL, "null handle pointer");
  }
  *out   = nullptr;
  int rc = select_device(device);
  if (rc != SRS_AMD_OK) {
    return rc;
  }
  auto* e   = new srs_amd_pdsch_encoder();
  e->device = device;
  rc        = srs_amd_crc_calculator_create(&e->crc16, 3, 3824, device);
  if (rc == SRS_AMD_OK) {
    rc = srs_amd_crc_calculator_create(&e->crc24a, 0, 1277992, device);
  }
  if (rc == SRS_AMD_OK) {
    rc = srs_amd_crc_calculator_create(&e->crc24b, 1, 8448, device);
  }
  if (rc == SRS_AMD_OK) {
    rc = srs_amd_ldpc_encoder_create(&e->enc, device);
  }
  if (rc == SRS_AMD_OK) {
    rc = srs_amd_ldpc_rate_matcher_create(&e->rm, device);
  }
  if (rc == SRS_AMD_OK) {
    hipError_t he = hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking);
    if (he != hipSuccess) {
      rc = hip_fail(he, "PDSCH encoder stream");
    }
  }
  if (rc != SRS_AMD_OK) {
    delete e;
    return rc;
  }
  *out = e;
  return SRS_AMD_OK;
}

void srs_amd_pdsch_encoder_destroy(srs_amd_pdsch_encoder* enc)
{
  delete enc;
}

int srs_amd_pdsch_encode_batch(srs_amd_pdsch_encoder*  enc,
                               const srs_amd_sch_plan* plan,
                               uint8_t*                d_codewords,
                               uint32_t                cw_stride,
                               const uint8_t*          d_tbs,
                               uint32_t                tb_stride,
                               uint32_t                nof_tbs,
                               void*                   stream)
{
  if (enc == nullptr) {
    return fail(SRS_AMD_EINVAL, "null PDSCH encoder");
  }
  int rc = check_plan(plan);
  if (rc != SRS_AMD_OK) {
    return rc;
  }
  if (nof_tbs == 0) {
    return SRS_AMD_OK;
  }
  if (d_codewords == nullptr || d_tbs == nullptr) {
    return fail(SRS_AMD_EINVAL, "null device buffer");
  }
  if (static_cast<uint64_t>(cw_stride) * 8 < plan->cw_length || static_cast<uint64_t>(tb_stride) * 8 < plan->tbs) {
    return fail(SRS_AMD_EINVAL, "row strides too small (codeword %u bits, TB %u bits)", plan->cw_length, plan->tbs);
  }
  if (static_cast<uint64_t>(nof_tbs) * cw_stride * 8 >= (1ull << 32)) {
    return fail(SRS_AMD_EINVAL, "batch of %u codewords exceeds 2^32 bits", nof_tbs);
  }
  std::lock_guard<std::mutex> lock(enc->mtx);
  return encode_locked(enc, plan, d_codewords, cw_stride, d_tbs, tb_stride, nof_tbs, static_cast<hipStream_t>(stream));
}

int srs_amd_pdsch_encode(srs_amd_pdsch_encoder* enc, uint8_t* codeword, const uint8_t* transport_block,
                         const srs_amd_sch_plan* plan)
{
  if (enc == nullptr || codeword == nullptr || transport_block == nullptr) {
    return fail(SRS_AMD_EINVAL, "null argument");
  }
  int rc = check_plan(plan);
  if (rc != SRS_AMD_OK) {
    return rc;
  }
  const uint32_t tb_bytes = plan->tbs / 8;
  const uint32_t cw_bytes = (plan->cw_length + 7) / 8;
  const size_t   tb_off   = align_up(cw_bytes, 256);
  std::lock_guard<std::mutex> lock(enc->mtx);
  hipError_t                  he = hipSetDevice(enc->device);
  if (he == hipSuccess) {
    he = enc->host_io.ensure(tb_off + tb_bytes);
  }
  uint8_t* d_cw = enc->host_io.as<uint8_t>();
  uint8_t* d_tb = d_cw + tb_off;
  if (he == hipSuccess) {
    he = hipMemcpyAsync(d_tb, transport_block, tb_bytes, hipMemcpyHostToDevice, enc->stream);
  }
  if (he != hipSuccess) {
    return hip_fail(he, "PDSCH encoder upload");
  }
  rc = encode_locked(enc, plan, d_cw, cw_bytes, d_tb, tb_bytes, 1, enc->stream);
  if (rc != SRS_AMD_OK) {
    return rc;
  }
  std::vector<uint8_t> packed(cw_bytes);
  he = hipMemcpyAsync(packed.data(), d_cw, cw_bytes, hipMemcpyDeviceToHost, enc->stream);
  if (he == hipSuccess) {
    he = hipStreamSynchronize(enc->stream);
  }
  if (he != hipSuccess) {
    return hip_fail(he, "PDSCH encoder download");
  }
  for (uint32_t i = 0; i < plan->cw_length; ++i) {
    codeword[i] = (packed[i >> 3] >> (7 - (i & 7))) & 1u;
  }
  return SRS_AMD_OK;
}

} // extern "C"
