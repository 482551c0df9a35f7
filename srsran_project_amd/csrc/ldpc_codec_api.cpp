// ldpc_codec_api.cpp -- C-ABI of the MI355X LDPC encoder, rate matcher and
// rate dematcher (include/srsran_amd/ldpc_encoder.h, ldpc_rate_matching.h).
//
// Argument checks mirror the reference's srsran_assert conditions:
//   ldpc_encoder_impl.cpp:48-52 (message length), ldpc_rate_matcher_impl.cpp:36-91
//   (rv, Nref, filler, E multiple of Qm), ldpc_rate_dematcher_impl.cpp:45-118
//   (Nref, input length, multiple of Qm, base graph from the output length).
#include "srsran_amd/ldpc_encoder.h"
#include "srsran_amd/ldpc_rate_matching.h"

#include <hip/hip_runtime.h>

#include "api_common.h"
#include "ldpc_common.h"
#include "ldpc_codec_args.h"
#include "ldpc_codec_internal.h"
#include <algorithm>
#include <cstring>
#include <mutex>
#include <vector>

namespace srs_amd {

namespace {

constexpr uint32_t MAX_MSG_BITS   = 22 * MAX_LIFTING_SIZE;  // MAX_MESSAGE_SIZE
constexpr uint32_t MAX_RM_LLRS    = MAX_MSG_BITS * 35;      // MAX_CODEBLOCK_RM_SIZE (ldpc.h:122)
constexpr uint32_t ENCODE_GRID_CAP = 1u << 16;

// Builds the encoder launch parameters and checks the base-graph structure the
// kernel relies on (see ldpc_encoder.hip header).
bool build_encode_params(encode_args& a, const lifted_graph& g)
{
  a.bg      = g.bg;
  a.Z       = g.Z;
  a.K       = g.K;
  a.M       = g.M;
  a.N_short = g.N_short;
  std::copy(g.row_start, g.row_start + MAX_BG_M + 1, a.row_start);
  const uint32_t Z = static_cast<uint32_t>(g.Z);
  int            shifts[4];
  int            nshift = 0;
  for (int r = 0; r < g.M; ++r) {
    for (int e = g.row_start[r]; e < g.row_start[r + 1]; ++e) {
      const uint32_t col   = (g.edge[e] & 0xffffu) / Z;
      const uint32_t shift = g.edge[e] >> 16;
      if (e > g.row_start[r] && (g.edge[e - 1] & 0xffffu) / Z >= col) {
        return false; // not sorted by column
      }
      if (r < 4) {
        if (col == static_cast<uint32_t>(g.K)) {
          a.core_a[r]      = static_cast<int>(shift);
          shifts[nshift++] = static_cast<int>(shift);
        } else if (col > static_cast<uint32_t>(g.K) && shift != 0) {
          return false;
        }
        if (col >= static_cast<uint32_t>(g.K) + 4) {
          return false;
        }
      } else if (col >= static_cast<uint32_t>(g.K) + 4) {
        // only the row's own extension column, identity
        if (col != static_cast<uint32_t>(g.K + r) || shift != 0 || e != g.row_start[r + 1] - 1) {
          return false;
        }
      }
    }
  }
  if (nshift != 3) {
    return false;
  }
  if (shifts[0] == shifts[1]) {
    a.p0_shift = shifts[2];
  } else if (shifts[0] == shifts[2]) {
    a.p0_shift = shifts[1];
  } else if (shifts[1] == shifts[2]) {
    a.p0_shift = shifts[0];
  } else {
    return false;
  }
  // rows of column K: BG1 {0, 1, 3}, BG2 {0, 2, 3} (the kernel's row-by-row solve)
  const bool ok = g.bg == 1 ? (a.core_a[2] == 0) : (a.core_a[1] == 0);
  return ok;
}

int check_encoder_cfg(const srs_amd_ldpc_encoder_config* cfg)
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
  return SRS_AMD_OK;
}

int check_rm_cfg(const srs_amd_codeblock_metadata* cfg, rm_geometry& g)
{
  if (cfg == nullptr) {
    return fail(SRS_AMD_EINVAL, "null configuration");
  }
  const char* msg = make_rm_geometry(
      g, cfg->base_graph, cfg->lifting_size, cfg->rv, cfg->modulation_order, cfg->Nref, cfg->nof_filler_bits);
  if (msg != nullptr) {
    return fail(SRS_AMD_EINVAL, "%s", msg);
  }
  return SRS_AMD_OK;
}

// Device scratch for the synchronous single-codeblock calls.
struct staging {
  void*  ptr  = nullptr;
  size_t size = 0;
  hipError_t ensure(size_t n)
  {
    if (n <= size) {
      return hipSuccess;
    }
    (void)hipFree(ptr);
    ptr        = nullptr;
    size       = 0;
    hipError_t e = hipMalloc(&ptr, n);
    if (e == hipSuccess) {
      size = n;
    }
    return e;
  }
  ~staging() { (void)hipFree(ptr); }
};

} // namespace

} // namespace srs_amd

using namespace srs_amd;

struct srs_amd_ldpc_encoder {
  int         device = 0;
  uint32_t*   edges  = nullptr;
  hipStream_t stream = nullptr;
  staging     scratch;
  std::mutex  mtx;
};

struct srs_amd_ldpc_rate_matcher {
  int         device = 0;
  hipStream_t stream = nullptr;
  staging     scratch;
  std::mutex  mtx;
};

struct srs_amd_ldpc_rate_dematcher {
  int         device = 0;
  hipStream_t stream = nullptr;
  staging     scratch;
  std::mutex  mtx;
};

namespace {

template <typename T>
int create_with_stream(T** out, int device)
{
  if (out == nullptr) {
    return fail(SRS_AMD_EINVAL, "null handle pointer");
  }
  *out   = nullptr;
  int rc = select_device(device);
  if (rc != SRS_AMD_OK) {
    return rc;
  }
  auto* h      = new T();
  h->device    = device;
  hipError_t e = hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking);
  if (e != hipSuccess) {
    delete h;
    return hip_fail(e, "hipStreamCreate");
  }
  *out = h;
  return SRS_AMD_OK;
}

template <typename T>
void destroy_with_stream(T* h)
{
  if (h == nullptr) {
    return;
  }
  (void)hipSetDevice(h->device);
  if (h->stream) {
    (void)hipStreamSynchronize(h->stream);
    (void)hipStreamDestroy(h->stream);
  }
  delete h;
}

} // namespace

extern "C" {

/* ---------------------------------------------------------------- encoder */

int srs_amd_ldpc_encoder_create(srs_amd_ldpc_encoder** encoder, int device)
{
  int rc = create_with_stream(encoder, device);
  if (rc != SRS_AMD_OK) {
    return rc;
  }
  std::vector<uint32_t> edges = all_lifted_edges();
  hipError_t            e     = hipMalloc(&(*encoder)->edges, edges.size() * sizeof(uint32_t));
  if (e == hipSuccess) {
    e = hipMemcpy((*encoder)->edges, edges.data(), edges.size() * sizeof(uint32_t), hipMemcpyHostToDevice);
  }
  if (e != hipSuccess) {
    srs_amd_ldpc_encoder_destroy(*encoder);
    *encoder = nullptr;
    return hip_fail(e, "encoder tables");
  }
  return SRS_AMD_OK;
}

void srs_amd_ldpc_encoder_destroy(srs_amd_ldpc_encoder* encoder)
{
  if (encoder != nullptr) {
    (void)hipSetDevice(encoder->device);
    if (encoder->stream) {
      (void)hipStreamSynchronize(encoder->stream);
    }
    (void)hipFree(encoder->edges);
    encoder->edges = nullptr;
  }
  destroy_with_stream(encoder);
}

} // extern "C"

int srs_amd::ldpc_encode_batch_ex(srs_amd_ldpc_encoder*              enc,
                              const srs_amd_ldpc_encoder_config* cfg,
                              const uint8_t*                     d_messages,
                              uint32_t                           msg_stride,
                              uint8_t*                           d_codeblocks,
                              uint32_t                           cb_stride,
                              uint32_t                           nof_cbs,
                              void*                              stream,
                              uint32_t                           max_bits)
{
  if (enc == nullptr) {
    return fail(SRS_AMD_EINVAL, "null encoder");
  }
  int rc = check_encoder_cfg(cfg);
  if (rc != SRS_AMD_OK) {
    return rc;
  }
  if (nof_cbs == 0) {
    return SRS_AMD_OK;
  }
  const int      bg = static_cast<int>(cfg->base_graph);
  const int      Z  = static_cast<int>(cfg->lifting_size);
  lifted_graph   g{};
  build_lifted_graph(g, bg, Z);
  if (d_messages == nullptr || d_codeblocks == nullptr) {
    return fail(SRS_AMD_EINVAL, "null device buffer");
  }
  if (msg_stride < static_cast<uint32_t>(g.K * Z + 7) / 8) {
    return fail(SRS_AMD_EINVAL, "msg_stride %u shorter than the message (%d bits)", msg_stride, g.K * Z);
  }
  if (cb_stride < static_cast<uint32_t>(g.N_short * Z + 7) / 8) {
    return fail(SRS_AMD_EINVAL, "cb_stride %u shorter than the codeblock (%d bits)", cb_stride, g.N_short * Z);
  }
  encode_args a{};
  if (!build_encode_params(a, g)) {
    return fail(SRS_AMD_EINVAL, "unexpected base graph structure (bg %d, Z %d)", bg, Z);
  }
  a.msgs       = d_messages;
  a.cws        = d_codeblocks;
  a.edges      = enc->edges + lifted_edges_offset(bg, Z);
  a.msg_stride = msg_stride;
  a.cw_stride  = cb_stride;
  a.nof_cbs    = nof_cbs;
  // Rows whose parity columns hold shortened-codeword positions < max_bits (column c at (c - 2) Z).
  const uint32_t full_bits = static_cast<uint32_t>(g.N_short * Z);
  max_bits                 = std::min(max_bits, full_bits);
  const int cols           = static_cast<int>((max_bits + Z - 1) / Z) + 2;
  a.M_eff                  = std::max(4, std::min(a.M, cols - a.K));
  a.pack_bits              = max_bits == full_bits ? static_cast<int32_t>(full_bits)
                                                   : static_cast<int32_t>(std::min(full_bits, (max_bits + 7) / 8 * 8));
  std::lock_guard<std::mutex> lock(enc->mtx);
  hipError_t                  e = hipSetDevice(enc->device);
  if (e == hipSuccess) {
    e = launch_ldpc_encode(a, static_cast<int>(std::min(nof_cbs, ENCODE_GRID_CAP)), static_cast<hipStream_t>(stream));
  }
  return e == hipSuccess ? SRS_AMD_OK : hip_fail(e, "ldpc_encode_kernel launch");
}

extern "C" {

int srs_amd_ldpc_encode_batch(srs_amd_ldpc_encoder*              enc,
                              const srs_amd_ldpc_encoder_config* cfg,
                              const uint8_t*                     d_messages,
                              uint32_t                           msg_stride,
                              uint8_t*                           d_codeblocks,
                              uint32_t                           cb_stride,
                              uint32_t                           nof_cbs,
                              void*                              stream)
{
  return ldpc_encode_batch_ex(enc, cfg, d_messages, msg_stride, d_codeblocks, cb_stride, nof_cbs, stream,
                              0xffffffffu);
}

int srs_amd_ldpc_encode(srs_amd_ldpc_encoder*              enc,
                        uint8_t*                           codeblock,
                        uint32_t                           codeblock_len,
                        const uint8_t*                     message_packed,
                        uint32_t                           message_len,
                        const srs_amd_ldpc_encoder_config* cfg)
{
  if (enc == nullptr || codeblock == nullptr || message_packed == nullptr) {
    return fail(SRS_AMD_EINVAL, "null argument");
  }
  int rc = check_encoder_cfg(cfg);
  if (rc != SRS_AMD_OK) {
    return rc;
  }
  const uint32_t K = (cfg->base_graph == 1 ? 22 : 10) * cfg->lifting_size;
  const uint32_t N = (cfg->base_graph == 1 ? 66 : 50) * cfg->lifting_size;
  if (message_len != K) {
    return fail(SRS_AMD_EINVAL, "Input size (%u) and message length (%u) must be equal", message_len, K);
  }
  if (codeblock_len > N) {
    return fail(SRS_AMD_EINVAL, "codeblock length %u exceeds the encoded codeblock length %u", codeblock_len, N);
  }
  const uint32_t mb = (K + 7) / 8, cbb = (N + 7) / 8;
  std::vector<uint8_t> packed(cbb);
  {
    std::lock_guard<std::mutex> lock(enc->mtx);
    hipError_t                  e = hipSetDevice(enc->device);
    if (e == hipSuccess) {
      e = enc->scratch.ensure(mb + cbb);
    }
    if (e == hipSuccess) {
      e = hipMemcpyAsync(enc->scratch.ptr, message_packed, mb, hipMemcpyHostToDevice, enc->stream);
    }
    if (e != hipSuccess) {
      return hip_fail(e, "staging message");
    }
  }
  uint8_t* d_msg = static_cast<uint8_t*>(enc->scratch.ptr);
  rc             = srs_amd_ldpc_encode_batch(enc, cfg, d_msg, mb, d_msg + mb, cbb, 1, enc->stream);
  if (rc != SRS_AMD_OK) {
    return rc;
  }
  hipError_t e = hipMemcpyAsync(packed.data(), d_msg + mb, cbb, hipMemcpyDeviceToHost, enc->stream);
  if (e == hipSuccess) {
    e = hipStreamSynchronize(enc->stream);
  }
  if (e != hipSuccess) {
    return hip_fail(e, "ldpc encode");
  }
  for (uint32_t i = 0; i < codeblock_len; ++i) {
    codeblock[i] = (packed[i >> 3] >> (7 - (i & 7))) & 1u;
  }
  return SRS_AMD_OK;
}

/* ----------------------------------------------------------- rate matcher */

int srs_amd_ldpc_rate_matcher_create(srs_amd_ldpc_rate_matcher** rm, int device)
{
  return create_with_stream(rm, device);
}

void srs_amd_ldpc_rate_matcher_destroy(srs_amd_ldpc_rate_matcher* rm)
{
  destroy_with_stream(rm);
}

int srs_amd_ldpc_rate_match_batch(srs_amd_ldpc_rate_matcher*        rm,
                                  const srs_amd_codeblock_metadata* cfg,
                                  const uint8_t*                    d_codeblocks,
                                  uint32_t                          cb_stride,
                                  const uint32_t*                   d_rm_lengths,
                                  const uint32_t*                   d_out_offsets,
                                  uint32_t                          max_rm_length,
                                  uint8_t*                          d_output,
                                  uint32_t                          nof_cbs,
                                  void*                             stream)
{
  if (rm == nullptr) {
    return fail(SRS_AMD_EINVAL, "null rate matcher");
  }
  rate_match_args a{};
  int             rc = check_rm_cfg(cfg, a.g);
  if (rc != SRS_AMD_OK) {
    return rc;
  }
  if (nof_cbs == 0) {
    return SRS_AMD_OK;
  }
  if (d_codeblocks == nullptr || d_rm_lengths == nullptr || d_out_offsets == nullptr || d_output == nullptr) {
    return fail(SRS_AMD_EINVAL, "null device buffer");
  }
  if (cb_stride < (a.g.N + 7) / 8) {
    return fail(SRS_AMD_EINVAL, "cb_stride %u shorter than the codeblock (%u bits)", cb_stride, a.g.N);
  }
  if (max_rm_length > MAX_RM_LLRS) {
    return fail(SRS_AMD_EINVAL, "rate-matched length %u exceeds %u", max_rm_length, MAX_RM_LLRS);
  }
  a.cw          = d_codeblocks;
  a.cw_stride   = cb_stride;
  a.rm_lengths  = d_rm_lengths;
  a.out_offsets = d_out_offsets;
  a.out         = d_output;
  a.nof_cbs     = nof_cbs;
  std::lock_guard<std::mutex> lock(rm->mtx);
  hipError_t                  e = hipSetDevice(rm->device);
  if (e == hipSuccess) {
    e = launch_rate_match(a, max_rm_length, static_cast<hipStream_t>(stream));
  }
  return e == hipSuccess ? SRS_AMD_OK : hip_fail(e, "ldpc_rate_match_kernel launch");
}

int srs_amd_ldpc_rate_match(srs_amd_ldpc_rate_matcher*        rm,
                            uint8_t*                          output_packed,
                            uint32_t                          output_len,
                            const uint8_t*                    codeblock,
                            uint32_t                          codeblock_len,
                            const srs_amd_codeblock_metadata* cfg)
{
  if (rm == nullptr || output_packed == nullptr || codeblock == nullptr) {
    return fail(SRS_AMD_EINVAL, "null argument");
  }
  rm_geometry g{};
  int         rc = check_rm_cfg(cfg, g);
  if (rc != SRS_AMD_OK) {
    return rc;
  }
  if (codeblock_len != g.N) {
    return fail(SRS_AMD_EINVAL, "codeblock length %u does not match the configuration (%u)", codeblock_len, g.N);
  }
  if (output_len % g.Qm != 0) {
    return fail(SRS_AMD_EINVAL, "The output length should be a multiple of the modulation order.");
  }
  if (output_len > MAX_RM_LLRS) {
    return fail(SRS_AMD_EINVAL, "rate-matched length %u exceeds %u", output_len, MAX_RM_LLRS);
  }
  const uint32_t       cbb = (g.N + 7) / 8, ob = (output_len + 7) / 8;
  std::vector<uint8_t> packed(cbb, 0);
  for (uint32_t i = 0; i < codeblock_len; ++i) {
    packed[i >> 3] |= static_cast<uint8_t>((codeblock[i] & 1u) << (7 - (i & 7)));
  }
  const uint32_t meta[2] = {output_len, 0};
  uint8_t*       base    = nullptr;
  {
    std::lock_guard<std::mutex> lock(rm->mtx);
    hipError_t                  e = hipSetDevice(rm->device);
    if (e == hipSuccess) {
      e = rm->scratch.ensure(8 + cbb + ob);
    }
    base = static_cast<uint8_t*>(rm->scratch.ptr);
    if (e == hipSuccess) {
      e = hipMemcpyAsync(base, meta, 8, hipMemcpyHostToDevice, rm->stream);
    }
    if (e == hipSuccess) {
      e = hipMemcpyAsync(base + 8, packed.data(), cbb, hipMemcpyHostToDevice, rm->stream);
    }
    if (e != hipSuccess) {
      return hip_fail(e, "staging codeblock");
    }
  }
  const uint32_t* d_meta = reinterpret_cast<const uint32_t*>(base);
  rc = srs_amd_ldpc_rate_match_batch(rm, cfg, base + 8, cbb, d_meta, d_meta + 1, output_len, base + 8 + cbb, 1, rm->stream);
  if (rc != SRS_AMD_OK) {
    return rc;
  }
  hipError_t e = hipMemcpyAsync(output_packed, base + 8 + cbb, ob, hipMemcpyDeviceToHost, rm->stream);
  if (e == hipSuccess) {
    e = hipStreamSynchronize(rm->stream);
  }
  return e == hipSuccess ? SRS_AMD_OK : hip_fail(e, "ldpc rate match");
}

/* --------------------------------------------------------- rate dematcher */

int srs_amd_ldpc_rate_dematcher_create(srs_amd_ldpc_rate_dematcher** dm, int device)
{
  return create_with_stream(dm, device);
}

void srs_amd_ldpc_rate_dematcher_destroy(srs_amd_ldpc_rate_dematcher* dm)
{
  destroy_with_stream(dm);
}

int srs_amd_ldpc_rate_dematch_batch(srs_amd_ldpc_rate_dematcher*      dm,
                                    const srs_amd_codeblock_metadata* cfg,
                                    int                               new_data,
                                    const int8_t*                     d_input,
                                    const uint32_t*                   d_in_offsets,
                                    const uint32_t*                   d_rm_lengths,
                                    int8_t*                           d_soft,
                                    uint32_t                          soft_stride,
                                    uint32_t                          nof_cbs,
                                    void*                             stream)
{
  return srs_amd::rate_dematch_batch_ex(
      dm, cfg, new_data, d_input, d_in_offsets, d_rm_lengths, d_soft, soft_stride, nof_cbs, stream, false);
}

} // extern "C"

int srs_amd::rate_dematch_batch_ex(srs_amd_ldpc_rate_dematcher*      dm,
                                   const srs_amd_codeblock_metadata* cfg,
                                   int                               new_data,
                                   const int8_t*                     d_input,
                                   const uint32_t*                   d_in_offsets,
                                   const uint32_t*                   d_rm_lengths,
                                   int8_t*                           d_soft,
                                   uint32_t                          soft_stride,
                                   uint32_t                          nof_cbs,
                                   void*                             stream,
                                   bool                              fresh,
                                   uint32_t                          write_end)
{
  if (dm == nullptr) {
    return fail(SRS_AMD_EINVAL, "null rate dematcher");
  }
  dematch_args a{};
  int          rc = check_rm_cfg(cfg, a.g);
  if (rc != SRS_AMD_OK) {
    return rc;
  }
  if (nof_cbs == 0) {
    return SRS_AMD_OK;
  }
  if (d_input == nullptr || d_in_offsets == nullptr || d_rm_lengths == nullptr || d_soft == nullptr) {
    return fail(SRS_AMD_EINVAL, "null device buffer");
  }
  if (soft_stride < a.g.N) {
    return fail(SRS_AMD_EINVAL, "soft_stride %u shorter than the codeblock (%u)", soft_stride, a.g.N);
  }
  a.in          = d_input;
  a.in_offsets  = d_in_offsets;
  a.rm_lengths  = d_rm_lengths;
  a.soft        = d_soft;
  a.soft_stride = soft_stride;
  a.nof_cbs     = nof_cbs;
  a.new_data    = new_data ? 1 : 0;
  a.fresh       = (fresh && new_data) ? 1 : 0;
  a.write_end   = (write_end == 0 || write_end > a.g.N) ? a.g.N : write_end;
  std::lock_guard<std::mutex> lock(dm->mtx);
  hipError_t                  e = hipSetDevice(dm->device);
  if (e == hipSuccess) {
    e = launch_rate_dematch(a, static_cast<hipStream_t>(stream));
  }
  return e == hipSuccess ? SRS_AMD_OK : hip_fail(e, "ldpc_rate_dematch_kernel launch");
}

const uint32_t* srs_amd::ldpc_encoder_edges(const srs_amd_ldpc_encoder* enc)
{
  return enc != nullptr ? enc->edges : nullptr;
}

namespace {
// The (BG, Z) part of an encoder row descriptor: building the lifted graph and its encoding parameters takes ~1 us,
// which per UE was most of a 512-UE slot's host time (0.55 ms), so every pair is built once.
struct mixed_row_base {
  enc_row_desc r;
  int32_t      M, K, N_short;
};

const mixed_row_base& mixed_row_of(uint32_t bg, uint32_t Z)
{
  static const std::vector<mixed_row_base> table = [] {
    std::vector<mixed_row_base> t(2 * NOF_LIFTING_SIZES);
    for (int b = 1; b <= 2; ++b) {
      for (int z = 2; z <= MAX_LIFTING_SIZE; ++z) {
        const int i = lifting_size_position(z);
        if (i < 0) {
          continue;
        }
        lifted_graph g{};
        encode_args  a{};
        build_lifted_graph(g, b, z);
        (void)build_encode_params(a, g);
        mixed_row_base& m = t[(b - 1) * NOF_LIFTING_SIZES + i];
        m.r.Z             = static_cast<uint32_t>(z);
        m.r.edge_off      = static_cast<uint32_t>(lifted_edges_offset(b, z));
        m.r.p0_shift      = static_cast<uint32_t>(a.p0_shift);
        for (int c = 0; c < 3; ++c) {
          m.r.core_a[c] = static_cast<uint32_t>(a.core_a[c]);
        }
        m.M       = a.M;
        m.K       = a.K;
        m.N_short = g.N_short;
      }
    }
    return t;
  }();
  return table[(bg - 1) * NOF_LIFTING_SIZES + static_cast<uint32_t>(lifting_size_position(static_cast<int>(Z)))];
}
} // namespace

uint32_t srs_amd::ldpc_encode_mixed_row(void* row, uint32_t bg, uint32_t Z, uint32_t max_bits)
{
  // callers pass a validated plan's (bg, Z)
  const mixed_row_base& m = mixed_row_of(bg, Z);
  // as ldpc_encode_batch_ex: rows whose parity columns hold shortened-codeword positions < max_bits
  const uint32_t full_bits = static_cast<uint32_t>(m.N_short) * Z;
  max_bits                 = std::min(max_bits, full_bits);
  const int    cols        = static_cast<int>((max_bits + Z - 1) / Z) + 2;
  enc_row_desc r           = m.r;
  r.M_eff                  = static_cast<uint32_t>(std::max(4, std::min(m.M, cols - m.K)));
  r.pack_bits              = max_bits == full_bits ? full_bits : std::min(full_bits, (max_bits + 7) / 8 * 8);
  static_assert(sizeof(r) == LDPC_ENCODE_ROW_BYTES, "row descriptor size");
  std::memcpy(row, &r, sizeof(r));
  return r.M_eff;
}

int srs_amd::ldpc_encode_mixed(srs_amd_ldpc_encoder* enc,
                               uint32_t              bg,
                               uint32_t              max_z,
                               uint32_t              max_rows_eff,
                               const uint8_t*        d_messages,
                               uint32_t              msg_stride,
                               uint8_t*              d_codeblocks,
                               uint32_t              cb_stride,
                               uint32_t              nof_cbs,
                               void*                 stream,
                               const void*           d_rows)
{
  if (enc == nullptr) {
    return fail(SRS_AMD_EINVAL, "null encoder");
  }
  if (nof_cbs == 0) {
    return SRS_AMD_OK;
  }
  lifted_graph g{};
  if ((bg != 1 && bg != 2) || !build_lifted_graph(g, static_cast<int>(bg), static_cast<int>(max_z)) || max_z < 32 ||
      d_messages == nullptr || d_codeblocks == nullptr || d_rows == nullptr) {
    return fail(SRS_AMD_EINVAL, "invalid mixed-Z encoding (bg %u, max Z %u)", bg, max_z);
  }
  encode_args a{};
  (void)build_encode_params(a, g);
  a.msgs       = d_messages;
  a.cws        = d_codeblocks;
  a.edges      = enc->edges;
  a.msg_stride = msg_stride;
  a.cw_stride  = cb_stride;
  a.nof_cbs    = nof_cbs;
  a.M_eff      = static_cast<int32_t>(max_rows_eff);
  a.rows       = static_cast<const enc_row_desc*>(d_rows);
  std::lock_guard<std::mutex> lock(enc->mtx);
  hipError_t                  e = hipSetDevice(enc->device);
  if (e == hipSuccess) {
    e = launch_ldpc_encode(a, static_cast<int>(std::min(nof_cbs, ENCODE_GRID_CAP)), static_cast<hipStream_t>(stream));
  }
  return e == hipSuccess ? SRS_AMD_OK : hip_fail(e, "ldpc_encode_kernel launch");
}

int srs_amd::rate_match_ragged(srs_amd_ldpc_rate_matcher* rm,
                               const uint8_t*             d_codeblocks,
                               uint32_t                   cb_stride,
                               const uint32_t*            d_rm_lengths,
                               const uint32_t*            d_out_offsets,
                               const uint32_t*            d_row_geo,
                               const void*                d_geos,
                               uint8_t*                   d_output,
                               uint32_t                   nof_cbs,
                               void*                      stream)
{
  if (rm == nullptr) {
    return fail(SRS_AMD_EINVAL, "null rate matcher");
  }
  if (nof_cbs == 0) {
    return SRS_AMD_OK;
  }
  if (d_codeblocks == nullptr || d_rm_lengths == nullptr || d_out_offsets == nullptr || d_row_geo == nullptr ||
      d_geos == nullptr || d_output == nullptr) {
    return fail(SRS_AMD_EINVAL, "null device buffer");
  }
  // the caller (srs_amd_pdsch_encode_slot) checked every geometry and cb_stride
  rate_match_args a{};
  a.cw          = d_codeblocks;
  a.cw_stride   = cb_stride;
  a.rm_lengths  = d_rm_lengths;
  a.out_offsets = d_out_offsets;
  a.out         = d_output;
  a.nof_cbs     = nof_cbs;
  a.row_geo     = d_row_geo;
  a.geos        = static_cast<const rm_geometry*>(d_geos);
  std::lock_guard<std::mutex> lock(rm->mtx);
  hipError_t                  e = hipSetDevice(rm->device);
  if (e == hipSuccess) {
    e = launch_rate_match(a, 0, static_cast<hipStream_t>(stream));
  }
  return e == hipSuccess ? SRS_AMD_OK : hip_fail(e, "ldpc_rate_match_kernel launch");
}

int srs_amd::rate_dematch_ragged(srs_amd_ldpc_rate_dematcher* dm,
                                 const int8_t*                d_input,
                                 const uint32_t*              d_in_offsets,
                                 const uint32_t*              d_rm_lengths,
                                 const uint32_t*              d_row_geo,
                                 const void*                  d_geos,
                                 const uint32_t*              d_geo_write_end,
                                 int8_t*                      d_soft,
                                 uint32_t                     soft_stride,
                                 uint32_t                     nof_cbs,
                                 void*                        stream,
                                 const uint8_t*               d_row_flags)
{
  if (dm == nullptr) {
    return fail(SRS_AMD_EINVAL, "null rate dematcher");
  }
  if (nof_cbs == 0) {
    return SRS_AMD_OK;
  }
  if (d_input == nullptr || d_in_offsets == nullptr || d_rm_lengths == nullptr || d_row_geo == nullptr ||
      d_geos == nullptr || d_geo_write_end == nullptr || d_soft == nullptr) {
    return fail(SRS_AMD_EINVAL, "null device buffer");
  }
  // the caller (srs_amd_pusch_decode_slot) checked every geometry and soft_stride >= every N
  dematch_args a{};
  a.in            = d_input;
  a.in_offsets    = d_in_offsets;
  a.rm_lengths    = d_rm_lengths;
  a.soft          = d_soft;
  a.soft_stride   = soft_stride;
  a.nof_cbs       = nof_cbs;
  a.new_data      = 1;
  a.fresh         = 1;
  a.row_geo       = d_row_geo;
  a.geos          = static_cast<const rm_geometry*>(d_geos);
  a.geo_write_end = d_geo_write_end;
  a.row_flags     = d_row_flags;
  std::lock_guard<std::mutex> lock(dm->mtx);
  hipError_t                  e = hipSetDevice(dm->device);
  if (e == hipSuccess) {
    e = launch_rate_dematch(a, static_cast<hipStream_t>(stream));
  }
  return e == hipSuccess ? SRS_AMD_OK : hip_fail(e, "ldpc_rate_dematch_kernel launch");
}

extern "C" {

int srs_amd_ldpc_rate_dematch(srs_amd_ldpc_rate_dematcher*      dm,
                              int8_t*                           output,
                              uint32_t                          output_len,
                              const int8_t*                     input,
                              uint32_t                          input_len,
                              int                               new_data,
                              const srs_amd_codeblock_metadata* cfg)
{
  if (dm == nullptr || output == nullptr || (input == nullptr && input_len > 0) || cfg == nullptr) {
    return fail(SRS_AMD_EINVAL, "null argument");
  }
  // ldpc_rate_dematcher_impl.cpp:80-97: the base graph and lifting size follow from the output length.
  srs_amd_codeblock_metadata c = *cfg;
  if (output_len % 66 == 0 && lifting_index(static_cast<int>(output_len / 66)) >= 0) {
    c.base_graph   = 1;
    c.lifting_size = output_len / 66;
  } else if (output_len % 50 == 0 && lifting_index(static_cast<int>(output_len / 50)) >= 0) {
    c.base_graph   = 2;
    c.lifting_size = output_len / 50;
  } else {
    return fail(SRS_AMD_EINVAL, "LDPC rate dematching: invalid input length.");
  }
  if (input_len > MAX_RM_LLRS) {
    return fail(SRS_AMD_EINVAL, "The length of the rate-matched codeblock is %u but it shouldn't be more than %u.",
                input_len, MAX_RM_LLRS);
  }
  if (c.modulation_order == 0 || input_len % c.modulation_order != 0) {
    return fail(SRS_AMD_EINVAL, "The input length should be a multiple of the modulation order.");
  }
  rm_geometry g{};
  int         rc = check_rm_cfg(&c, g);
  if (rc != SRS_AMD_OK) {
    return rc;
  }
  const uint32_t meta[2] = {0, input_len};
  int8_t*        base    = nullptr;
  {
    std::lock_guard<std::mutex> lock(dm->mtx);
    hipError_t                  e = hipSetDevice(dm->device);
    if (e == hipSuccess) {
      e = dm->scratch.ensure(8 + output_len + input_len);
    }
    base = static_cast<int8_t*>(dm->scratch.ptr);
    if (e == hipSuccess) {
      e = hipMemcpyAsync(base, meta, 8, hipMemcpyHostToDevice, dm->stream);
    }
    if (e == hipSuccess) {
      e = hipMemcpyAsync(base + 8, output, output_len, hipMemcpyHostToDevice, dm->stream);
    }
    if (e == hipSuccess && input_len > 0) {
      e = hipMemcpyAsync(base + 8 + output_len, input, input_len, hipMemcpyHostToDevice, dm->stream);
    }
    if (e != hipSuccess) {
      return hip_fail(e, "staging soft buffer");
    }
  }
  const uint32_t* d_meta = reinterpret_cast<const uint32_t*>(base);
  rc = srs_amd_ldpc_rate_dematch_batch(
      dm, &c, new_data, base + 8 + output_len, d_meta, d_meta + 1, base + 8, output_len, 1, dm->stream);
  if (rc != SRS_AMD_OK) {
    return rc;
  }
  hipError_t e = hipMemcpyAsync(output, base + 8, output_len, hipMemcpyDeviceToHost, dm->stream);
  if (e == hipSuccess) {
    e = hipStreamSynchronize(dm->stream);
  }
  return e == hipSuccess ? SRS_AMD_OK : hip_fail(e, "ldpc rate dematch");
}

} // extern "C"
