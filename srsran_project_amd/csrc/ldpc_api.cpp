// ldpc_api.cpp -- C-ABI entry points of the MI355X LDPC path (include/srsran_amd/ldpc.h).
//
// Error behaviour mirrors the reference's srsran_assert checks in
// lib/phy/upper/channel_coding/ldpc/ldpc_decoder_impl.cpp:30-75 (invalid
// lifting size, iterations == 0, CRC length, input length bounds); instead of
// aborting, the call returns SRS_AMD_EINVAL with the reference's message.
#include "srsran_amd/ldpc.h"

#include <hip/hip_runtime.h>

#include "api_common.h"
#include "ldpc_codec_internal.h"
#include "ldpc_common.h"
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <algorithm>
#include <vector>

namespace srs_amd {


hipError_t launch_ldpc_decode(const decode_args& args, const lifted_graph& g, int arith, int grid, hipStream_t stream);
size_t     ldpc_decode_lds_bytes(const lifted_graph& g);

namespace {

constexpr int      MAX_CRC_BITS_LEN = 22 * MAX_LIFTING_SIZE;
constexpr uint32_t DEFAULT_SLOTS    = 1u << 20;

} // namespace


} // namespace srs_amd

using namespace srs_amd;

struct srs_amd_ldpc_decoder {
  int                     arith          = ARITH_SIMD;
  int                     force_decoding = 0;
  int                     device         = 0;
  uint32_t                max_slots      = DEFAULT_SLOTS;
  uint32_t*               crc_tables     = nullptr; // 6 x MAX_CRC_BITS_LEN
  uint32_t*               edges          = nullptr; // [2][51][MAX_EDGES] lifted edge descriptors
  int8_t*                 h_in           = nullptr; // staging for the single-CB host call
  uint8_t*                h_out          = nullptr;
  int32_t*                h_it           = nullptr;
  hipStream_t             stream         = nullptr;
  lifted_graph            graph{};
  int                     graph_bg = 0, graph_Z = 0;
  std::mutex              mtx;
};

namespace {

int validate(const srs_amd_ldpc_decoder_config* cfg, int crc_poly)
{
  if (cfg == nullptr) {
    return fail(SRS_AMD_EINVAL, "null configuration");
  }
  if (cfg->base_graph != 1 && cfg->base_graph != 2) {
    return fail(SRS_AMD_EINVAL, "Invalid base graph %u", cfg->base_graph);
  }
  if (lifting_index(static_cast<int>(cfg->lifting_size)) < 0) {
    return fail(SRS_AMD_EINVAL, "Invalid lifting size %u", cfg->lifting_size);
  }
  if (cfg->max_iterations == 0) {
    return fail(SRS_AMD_EINVAL, "Max iterations must be different to 0");
  }
  if (cfg->nof_crc_bits != 16 && cfg->nof_crc_bits != 24) {
    return fail(SRS_AMD_EINVAL, "Invalid number of CRC bits.");
  }
  uint32_t K = (cfg->base_graph == 1 ? 22 : 10) * cfg->lifting_size;
  if (cfg->nof_filler_bits >= K) {
    return fail(SRS_AMD_EINVAL, "Invalid number of filler bits %u", cfg->nof_filler_bits);
  }
  if (crc_poly != SRS_AMD_NO_CRC && (crc_poly < 0 || crc_poly > 5)) {
    return fail(SRS_AMD_EINVAL, "Invalid CRC polynomial %d", crc_poly);
  }
  return SRS_AMD_OK;
}

const lifted_graph& get_graph(srs_amd_ldpc_decoder* d, int bg, int Z)
{
  if (d->graph_bg != bg || d->graph_Z != Z) {
    build_lifted_graph(d->graph, bg, Z);
    d->graph_bg = bg;
    d->graph_Z  = Z;
  }
  return d->graph;
}

} // namespace

extern "C" {

const char* srs_amd_last_error(void)
{
  return srs_amd::last_error();
}

const char* srs_amd_version(void)
{
  return "srsran_amd 0.1.0 (gfx950)";
}

uint32_t srs_amd_ldpc_message_length(uint32_t base_graph, uint32_t lifting_size)
{
  if ((base_graph != 1 && base_graph != 2) || lifting_index(static_cast<int>(lifting_size)) < 0) {
    return 0;
  }
  return (base_graph == 1 ? 22u : 10u) * lifting_size;
}

uint32_t srs_amd_ldpc_codeblock_length(uint32_t base_graph, uint32_t lifting_size)
{
  if ((base_graph != 1 && base_graph != 2) || lifting_index(static_cast<int>(lifting_size)) < 0) {
    return 0;
  }
  return (base_graph == 1 ? 66u : 50u) * lifting_size;
}

int srs_amd_ldpc_decoder_create(srs_amd_ldpc_decoder** decoder, int arith, int force_decoding, int device)
{
  if (decoder == nullptr) {
    return fail(SRS_AMD_EINVAL, "null decoder pointer");
  }
  if (arith != ARITH_SIMD && arith != ARITH_GENERIC) {
    return fail(SRS_AMD_EINVAL, "Invalid arithmetic flavour %d", arith);
  }
  *decoder = nullptr;
  int rc    = select_device(device);
  if (rc != SRS_AMD_OK) {
    return rc;
  }
  hipError_t e = hipSuccess;
  auto* d           = new srs_amd_ldpc_decoder();
  d->arith          = arith;
  d->force_decoding = force_decoding ? 1 : 0;
  d->device         = device;
  std::vector<uint32_t> tables;
  tables.reserve(6 * MAX_CRC_BITS_LEN);
  for (int p = 0; p < 6; ++p) {
    auto t = crc_linear_table(p, MAX_CRC_BITS_LEN);
    tables.insert(tables.end(), t.begin(), t.end());
  }
  e = hipMalloc(&d->crc_tables, tables.size() * sizeof(uint32_t));
  if (e == hipSuccess) {
    e = hipMemcpy(d->crc_tables, tables.data(), tables.size() * sizeof(uint32_t), hipMemcpyHostToDevice);
  }
  // Every lifted graph (2 base graphs x 51 lifting sizes, 129 KiB), uploaded once.
  std::vector<uint32_t> edges = all_lifted_edges();
  if (e == hipSuccess) {
    e = hipMalloc(&d->edges, edges.size() * sizeof(uint32_t));
  }
  if (e == hipSuccess) {
    e = hipMemcpy(d->edges, edges.data(), edges.size() * sizeof(uint32_t), hipMemcpyHostToDevice);
  }
  if (e == hipSuccess) {
    e = hipStreamCreateWithFlags(&d->stream, hipStreamNonBlocking);
  }
  if (e != hipSuccess) {
    srs_amd_ldpc_decoder_destroy(d);
    return hip_fail(e, "decoder setup");
  }
  *decoder = d;
  return SRS_AMD_OK;
}

void srs_amd_ldpc_decoder_destroy(srs_amd_ldpc_decoder* d)
{
  if (d == nullptr) {
    return;
  }
  (void)hipSetDevice(d->device);
  if (d->stream) {
    (void)hipStreamSynchronize(d->stream);
    (void)hipStreamDestroy(d->stream);
  }
  (void)hipFree(d->crc_tables);
  (void)hipFree(d->edges);
  (void)hipFree(d->h_in);
  (void)hipFree(d->h_out);
  (void)hipFree(d->h_it);
  delete d;
}

int srs_amd_ldpc_decoder_set_max_slots(srs_amd_ldpc_decoder* d, uint32_t max_slots)
{
  if (d == nullptr || max_slots == 0) {
    return fail(SRS_AMD_EINVAL, "invalid decoder or slot count");
  }
  std::lock_guard<std::mutex> lock(d->mtx);
  d->max_slots = max_slots;
  return SRS_AMD_OK;
}

int srs_amd_ldpc_decode_batch(srs_amd_ldpc_decoder*              d,
                              const srs_amd_ldpc_decoder_config* cfg,
                              int                                crc_poly,
                              const int8_t*                      d_llrs,
                              uint32_t                           llr_stride,
                              const uint32_t*                    d_llr_lens,
                              uint32_t                           llr_len,
                              uint8_t*                           d_output,
                              uint32_t                           out_stride,
                              int32_t*                           d_nof_iters,
                              int8_t*                            d_soft_out,
                              uint32_t                           nof_cbs,
                              void*                              stream)
{
  return srs_amd::ldpc_decode_batch_ex(d, cfg, crc_poly, d_llrs, llr_stride, d_llr_lens, llr_len, d_output,
                                       out_stride, d_nof_iters, d_soft_out, nof_cbs, stream, nullptr, 0);
}

} // extern "C"

int srs_amd::ldpc_decode_batch_ex(srs_amd_ldpc_decoder*              d,
                                  const srs_amd_ldpc_decoder_config* cfg,
                                  int                                crc_poly,
                                  const int8_t*                      d_llrs,
                                  uint32_t                           llr_stride,
                                  const uint32_t*                    d_llr_lens,
                                  uint32_t                           llr_len,
                                  uint8_t*                           d_output,
                                  uint32_t                           out_stride,
                                  int32_t*                           d_nof_iters,
                                  int8_t*                            d_soft_out,
                                  uint32_t                           nof_cbs,
                                  void*                              stream,
                                  const uint8_t*                     d_skip_flags,
                                  uint32_t                           skip_stride,
                                  const int32_t*                     d_fillers,
                                  const ldpc_cw_rows*                cw)
{
  if (d == nullptr) {
    return fail(SRS_AMD_EINVAL, "null decoder");
  }
  int rc = validate(cfg, crc_poly);
  if (rc != SRS_AMD_OK) {
    return rc;
  }
  const uint32_t Z       = cfg->lifting_size;
  const uint32_t K       = (cfg->base_graph == 1 ? 22 : 10) * Z;
  const uint32_t N_short = (cfg->base_graph == 1 ? 66 : 50) * Z;
  if (nof_cbs == 0) {
    return SRS_AMD_OK;
  }
  if ((d_llrs == nullptr && cw == nullptr) || d_output == nullptr || d_nof_iters == nullptr ||
      (cw != nullptr && (cw->llrs == nullptr || cw->offsets == nullptr || cw->lengths == nullptr))) {
    return fail(SRS_AMD_EINVAL, "null device buffer");
  }
  if (cw != nullptr && (d_llr_lens != nullptr || d_soft_out != nullptr || d_skip_flags != nullptr || cw->qm == 0 ||
                        !ldpc_hr_takes(static_cast<int>(cfg->base_graph), static_cast<int>(cfg->lifting_size), llr_len))) {
    return fail(SRS_AMD_EINVAL, "codeword-fed rows need the high-rate decoder's configuration");
  }
  if (out_stride < (K + 7) / 8) {
    return fail(SRS_AMD_EINVAL, "The output size %u is not equal to the message length %u.", out_stride * 8, K);
  }
  if (d_llr_lens == nullptr) {
    // ldpc_decoder_impl.cpp:62-75 input length bounds (per-row lengths are the caller's contract).
    if (llr_len > N_short) {
      return fail(SRS_AMD_EINVAL, "The input size %u exceeds the maximum message length %u.", llr_len, N_short);
    }
    if (llr_len < K + 2 * Z) {
      return fail(SRS_AMD_EINVAL, "The input length %u does not reach minimum %u", llr_len, K + 2 * Z);
    }
    if (llr_stride < llr_len) {
      return fail(SRS_AMD_EINVAL, "llr_stride %u smaller than llr_len %u", llr_stride, llr_len);
    }
  }
  std::lock_guard<std::mutex> lock(d->mtx);
  hipError_t                  e = hipSetDevice(d->device);
  if (e != hipSuccess) {
    return hip_fail(e, "hipSetDevice");
  }
  const lifted_graph& g = get_graph(d, static_cast<int>(cfg->base_graph), static_cast<int>(Z));

  decode_args a{};
  a.llrs            = d_llrs;
  a.llr_lens        = d_llr_lens;
  a.out             = d_output;
  a.nof_iters       = d_nof_iters;
  a.soft_out        = d_soft_out;
  a.crc_table       = crc_poly == SRS_AMD_NO_CRC ? nullptr : d->crc_tables + static_cast<size_t>(crc_poly) * MAX_CRC_BITS_LEN;
  a.edges = d->edges + ((cfg->base_graph - 1) * NOF_LIFTING_SIZES + lifting_size_position(static_cast<int>(Z))) *
                             static_cast<size_t>(MAX_EDGES);
  a.llr_stride      = llr_stride;
  a.aligned4        = ((reinterpret_cast<uintptr_t>(d_llrs) | llr_stride) & 3u) == 0 ? 1 : 0;
  a.llr_len         = llr_len;
  a.out_stride      = out_stride;
  a.nof_cbs         = nof_cbs;
  a.nof_filler_bits = static_cast<int32_t>(cfg->nof_filler_bits);
  a.max_iterations  = static_cast<int32_t>(cfg->max_iterations);
  a.force_decoding  = d->force_decoding;
  a.skip_flags      = d_skip_flags;
  a.skip_stride     = skip_stride;
  a.fillers         = d_fillers;
  if (cw != nullptr) {
    a.llrs        = cw->llrs;
    a.aligned4    = 1; // rows are built in LDS
    a.cw_llrs     = cw->llrs;
    a.cw_offsets  = cw->offsets;
    a.cw_lengths  = cw->lengths;
    a.cw_qm       = cw->qm;
    a.cw_nof_info = cw->nof_info;
    a.cw_filler   = cw->filler;
  }
  const int grid    = static_cast<int>(nof_cbs < d->max_slots ? nof_cbs : d->max_slots);
  e = launch_ldpc_decode(a, g, d->arith, grid, static_cast<hipStream_t>(stream));
  if (e != hipSuccess) {
    return hip_fail(e, "ldpc_decode_kernel launch");
  }
  return SRS_AMD_OK;
}

void srs_amd::ldpc_mixed_row(void* row, uint32_t bg, uint32_t Z, int crc_poly)
{
  ldpc_row_desc r{};
  r.Z        = Z;
  r.edge_off = static_cast<uint32_t>(lifted_edges_offset(static_cast<int>(bg), static_cast<int>(Z)));
  r.crc_off  = crc_poly == SRS_AMD_NO_CRC ? NO_CRC_ROW : static_cast<uint32_t>(crc_poly) * MAX_CRC_BITS_LEN;
  r.zmagic   = ldpc_z_magic(Z);
  std::memcpy(row, &r, sizeof(r));
}

int srs_amd::ldpc_decode_mixed(srs_amd_ldpc_decoder* d,
                               uint32_t              bg,
                               uint32_t              max_z,
                               uint32_t              max_iterations,
                               const int8_t*         d_llrs,
                               uint32_t              llr_stride,
                               const uint32_t*       d_llr_lens,
                               uint8_t*              d_output,
                               uint32_t              out_stride,
                               int32_t*              d_nof_iters,
                               uint32_t              nof_cbs,
                               void*                 stream,
                               const int32_t*        d_fillers,
                               const void*           d_rows)
{
  if (d == nullptr) {
    return fail(SRS_AMD_EINVAL, "null decoder");
  }
  if ((bg != 1 && bg != 2) || lifting_index(static_cast<int>(max_z)) < 0 || max_z >= 384 || max_iterations == 0) {
    return fail(SRS_AMD_EINVAL, "invalid mixed-Z decoding (bg %u, max Z %u)", bg, max_z);
  }
  if (nof_cbs == 0) {
    return SRS_AMD_OK;
  }
  if (d_llrs == nullptr || d_llr_lens == nullptr || d_output == nullptr || d_nof_iters == nullptr ||
      d_fillers == nullptr || d_rows == nullptr) {
    return fail(SRS_AMD_EINVAL, "null device buffer");
  }
  std::lock_guard<std::mutex> lock(d->mtx);
  hipError_t                  e = hipSetDevice(d->device);
  if (e != hipSuccess) {
    return hip_fail(e, "hipSetDevice");
  }
  // the launch shape (threads, LDS) of the largest lifting size; each codeblock reads its own graph
  const lifted_graph& g = get_graph(d, static_cast<int>(bg), static_cast<int>(max_z));
  decode_args         a{};
  a.llrs           = d_llrs;
  a.llr_lens       = d_llr_lens;
  a.out            = d_output;
  a.nof_iters      = d_nof_iters;
  a.crc_table      = d->crc_tables;
  a.edges          = d->edges;
  a.llr_stride     = llr_stride;
  a.aligned4       = ((reinterpret_cast<uintptr_t>(d_llrs) | llr_stride) & 3u) == 0 ? 1 : 0;
  a.out_stride     = out_stride;
  a.nof_cbs        = nof_cbs;
  a.max_iterations = static_cast<int32_t>(max_iterations);
  a.force_decoding = d->force_decoding;
  a.fillers        = d_fillers;
  a.rows           = static_cast<const ldpc_row_desc*>(d_rows);
  const int grid   = static_cast<int>(nof_cbs < d->max_slots ? nof_cbs : d->max_slots);
  e                = launch_ldpc_decode(a, g, d->arith, grid, static_cast<hipStream_t>(stream));
  return e == hipSuccess ? SRS_AMD_OK : hip_fail(e, "ldpc_decode_kernel launch");
}

extern "C" {

int srs_amd_ldpc_decode(srs_amd_ldpc_decoder*              d,
                        uint8_t*                           output_packed,
                        const int8_t*                      input,
                        uint32_t                           input_len,
                        int                                crc_poly,
                        const srs_amd_ldpc_decoder_config* cfg,
                        int32_t*                           nof_iterations)
{
  if (d == nullptr || output_packed == nullptr || input == nullptr) {
    return fail(SRS_AMD_EINVAL, "null argument");
  }
  int rc = validate(cfg, crc_poly);
  if (rc != SRS_AMD_OK) {
    return rc;
  }
  const uint32_t K      = (cfg->base_graph == 1 ? 22 : 10) * cfg->lifting_size;
  const uint32_t obytes = (K + 7) / 8;
  {
    std::lock_guard<std::mutex> lock(d->mtx);
    hipError_t                  e = hipSetDevice(d->device);
    if (e == hipSuccess && d->h_in == nullptr) {
      e = hipMalloc(&d->h_in, 66 * MAX_LIFTING_SIZE);
      if (e == hipSuccess) {
        e = hipMalloc(&d->h_out, (22 * MAX_LIFTING_SIZE + 7) / 8);
      }
      if (e == hipSuccess) {
        e = hipMalloc(&d->h_it, sizeof(int32_t));
      }
    }
    if (e == hipSuccess && input_len <= 66 * MAX_LIFTING_SIZE) {
      e = hipMemcpyAsync(d->h_in, input, input_len, hipMemcpyHostToDevice, d->stream);
    }
    if (e == hipSuccess) {
      // the reference leaves the output untouched on the forced / CRC path: preload it.
      e = hipMemcpyAsync(d->h_out, output_packed, obytes, hipMemcpyHostToDevice, d->stream);
    }
    if (e != hipSuccess) {
      return hip_fail(e, "staging input");
    }
  }
  rc = srs_amd_ldpc_decode_batch(
      d, cfg, crc_poly, d->h_in, input_len, nullptr, input_len, d->h_out, obytes, d->h_it, nullptr, 1, d->stream);
  if (rc != SRS_AMD_OK) {
    return rc;
  }
  int32_t    it = -1;
  hipError_t e  = hipMemcpyAsync(output_packed, d->h_out, obytes, hipMemcpyDeviceToHost, d->stream);
  if (e == hipSuccess) {
    e = hipMemcpyAsync(&it, d->h_it, sizeof(int32_t), hipMemcpyDeviceToHost, d->stream);
  }
  if (e == hipSuccess) {
    e = hipStreamSynchronize(d->stream);
  }
  if (e != hipSuccess) {
    return hip_fail(e, "ldpc decode");
  }
  if (nof_iterations) {
    *nof_iterations = it;
  }
  return SRS_AMD_OK;
}

} // extern "C"
