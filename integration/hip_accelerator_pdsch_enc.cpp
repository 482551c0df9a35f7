// hip_accelerator_pdsch_enc.cpp -- hal::hw_accelerator_pdsch_enc over the srsran_amd C-ABI (see the header).
#include "hip_accelerator_pdsch_enc.h"

#include "srsran/ran/sch/modulation_scheme.h"
#include "srsran_amd/ldpc_encoder.h"
#include "srsran_amd/ldpc_rate_matching.h"
#include "srsran_amd/sch.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

using namespace srsran;
using namespace srsran::hip;

namespace {

constexpr unsigned MAX_CBS = 512; // codeblocks of one transport block

void log_error(const char* what, const char* detail)
{
  std::fprintf(stderr, "hip_accelerator_pdsch_enc: %s: %s\n", what, detail);
}

void require_amd(int rc, const char* what)
{
  if (rc != SRS_AMD_OK) {
    log_error(what, srs_amd_last_error());
    throw std::runtime_error(std::string("hip_accelerator_pdsch_enc: ") + what);
  }
}

unsigned message_length(ldpc_base_graph_type bg, unsigned Z)
{
  return (bg == ldpc_base_graph_type::BG1 ? 22 : 10) * Z;
}

/// The segmentation geometry pdsch_encoder_hw_impl::set_hw_enc_tb_configuration hands over
/// (pdsch_encoder_hw_impl.cpp:217-276), as the srs_amd_sch_plan the C-ABI encoder runs on.
srs_amd_sch_plan plan_of(const hal::hw_pdsch_encoder_configuration& c)
{
  srs_amd_sch_plan p{};
  const unsigned   C   = c.nof_segments;
  const unsigned   L   = C > 1 ? 24 : 0;
  p.tbs                = c.nof_tb_bits;
  p.base_graph         = c.base_graph_index == ldpc_base_graph_type::BG1 ? 1 : 2;
  p.rv                 = c.rv;
  p.modulation_order   = get_bits_per_symbol(c.modulation);
  p.Nref               = c.Nref;
  p.lifting_size       = c.lifting_size;
  p.segment_length     = message_length(c.base_graph_index, c.lifting_size);
  p.nof_segments       = C;
  p.nof_tb_crc_bits    = c.nof_tb_crc_bits;
  p.nof_crc_bits       = L;
  p.cb_info_bits       = c.nof_segment_bits;
  p.zero_pad           = (c.nof_segment_bits + L) * C - (c.nof_tb_bits + c.nof_tb_crc_bits + L * C);
  p.nof_filler_bits    = c.nof_filler_bits;
  p.nof_short_segments = c.nof_short_segments;
  p.rm_length_short    = c.cw_length_a;
  p.rm_length_long     = c.cw_length_b;
  p.cw_length          = c.nof_short_segments * c.cw_length_a + (C - c.nof_short_segments) * c.cw_length_b;
  // informational only (the encoder reads the rate-matching lengths above)
  p.nof_layers     = 1;
  p.nof_ch_symbols = p.modulation_order ? p.cw_length / p.modulation_order : 0;
  return p;
}

class hip_accelerator_pdsch_enc : public hal::hw_accelerator_pdsch_enc
{
public:
  explicit hip_accelerator_pdsch_enc(const pdsch_enc_accelerator_config& c) : cfg(c)
  {
    int dev = c.device;
    if (dev < 0 && hipGetDevice(&dev) != hipSuccess) {
      throw std::runtime_error("hip_accelerator_pdsch_enc: hipGetDevice");
    }
    require_amd(srs_amd_pdsch_encoder_create(&tb_enc, dev), "PDSCH encoder");
    require_amd(srs_amd_ldpc_encoder_create(&cb_enc, dev), "LDPC encoder");
    require_amd(srs_amd_ldpc_rate_matcher_create(&rm, dev), "rate matcher");
  }
  ~hip_accelerator_pdsch_enc() override
  {
    srs_amd_pdsch_encoder_destroy(tb_enc);
    srs_amd_ldpc_encoder_destroy(cb_enc);
    srs_amd_ldpc_rate_matcher_destroy(rm);
  }

  void reserve_queue() override
  {
    std::fill(std::begin(ready), std::end(ready), false);
  }
  void free_queue() override {}

  void configure_operation(const hal::hw_pdsch_encoder_configuration& config, unsigned cb_index) override
  {
    if (cb_index < MAX_CBS) {
      ops[cb_index] = config;
    }
  }

  bool is_cb_mode_supported() const override { return cfg.cb_mode; }

  unsigned get_max_supported_buff_size() const override { return cfg.max_buffer_size; }

  // The whole operation runs here (the GPU call is synchronous).  A failed operation (encoding or rate-matching
  // error, transport block size mismatch) never stalls the reference's driver, which calls dequeue_operation until
  // it returns true (pdsch_encoder_hw_impl.cpp:150-160): the error is logged and the operation dequeues the
  // configured codeword length as zeros.
  bool enqueue_operation(span<const uint8_t> data, span<const uint8_t> /*aux*/, unsigned cb_index) override
  {
    if (cb_index >= MAX_CBS) {
      log_error("enqueue_operation", "codeblock index beyond the queue");
      return true;
    }
    const hal::hw_pdsch_encoder_configuration& c = ops[cb_index];
    ready[cb_index]                              = true;
    out[cb_index].clear();
    if (!c.cb_mode) {
      // TB mode: TB CRC, segmentation, CB CRCs, LDPC encoding and rate matching in one C-ABI call
      const srs_amd_sch_plan p = plan_of(c);
      out[cb_index].assign(p.cw_length, 0);
      if (data.size() * 8 != p.tbs) {
        log_error("enqueue_operation", "transport block size differs from the configuration");
        return true;
      }
      if (srs_amd_pdsch_encode(tb_enc, out[cb_index].data(), data.data(), &p) != SRS_AMD_OK) {
        log_error("PDSCH encoding", srs_amd_last_error());
        std::fill(out[cb_index].begin(), out[cb_index].end(), 0);
      }
      return true;
    }
    // CB mode: the codeblock's K - F message bits (CRCs attached by the reference's segmenter), then F filler
    // bits (zero) -- LDPC encoding of K bits and rate matching to E = rm_length bits
    out[cb_index].assign(c.rm_length, 0);
    const unsigned K = message_length(c.base_graph_index, c.lifting_size);
    const unsigned N = (c.base_graph_index == ldpc_base_graph_type::BG1 ? 66 : 50) * c.lifting_size;
    const unsigned k = K - c.nof_filler_bits;
    if (data.size() * 8 < k) {
      log_error("enqueue_operation", "codeblock shorter than K - F bits");
      return true;
    }
    msg.assign((K + 7) / 8, 0);
    std::memcpy(msg.data(), data.data(), k / 8);
    if (k % 8) {
      msg[k / 8] = data[k / 8] & static_cast<uint8_t>(0xff00u >> (k % 8));
    }
    cb.resize(N);
    const srs_amd_ldpc_encoder_config ec{c.base_graph_index == ldpc_base_graph_type::BG1 ? 1u : 2u, c.lifting_size,
                                         c.Nref};
    if (srs_amd_ldpc_encode(cb_enc, cb.data(), N, msg.data(), K, &ec) != SRS_AMD_OK) {
      log_error("LDPC encoding", srs_amd_last_error());
      return true;
    }
    const srs_amd_codeblock_metadata md{ec.base_graph, c.lifting_size, c.rv, get_bits_per_symbol(c.modulation),
                                        c.Nref, c.nof_filler_bits};
    packed.assign((c.rm_length + 7) / 8, 0);
    if (srs_amd_ldpc_rate_match(rm, packed.data(), c.rm_length, cb.data(), N, &md) != SRS_AMD_OK) {
      log_error("rate matching", srs_amd_last_error());
      return true;
    }
    for (unsigned i = 0; i != c.rm_length; ++i) {
      out[cb_index][i] = (packed[i >> 3] >> (7 - (i & 7))) & 1u;
    }
    return true;
  }

  // data: the codeword (TB mode) or the rate-matched codeblock (CB mode), one bit per byte; aux: packed.  Returns
  // false only for an operation that was never enqueued; a length mismatch is logged and dequeues zeros.
  bool dequeue_operation(span<uint8_t> data, span<uint8_t> aux, unsigned cb_index) override
  {
    if (cb_index >= MAX_CBS) { // refused at the enqueue (logged there): zeros
      std::fill(data.begin(), data.end(), 0);
      std::fill(aux.begin(), aux.end(), 0);
      return true;
    }
    if (!ready[cb_index]) {
      return false;
    }
    if (data.size() != out[cb_index].size()) {
      log_error("dequeue_operation", "output length differs from the configured codeword");
      out[cb_index].assign(data.size(), 0);
    }
    std::memcpy(data.data(), out[cb_index].data(), data.size());
    std::fill(aux.begin(), aux.end(), 0);
    for (size_t i = 0; i != data.size() && i / 8 < aux.size(); ++i) {
      aux[i / 8] |= static_cast<uint8_t>(data[i] << (7 - (i & 7)));
    }
    ready[cb_index] = false;
    return true;
  }

private:
  pdsch_enc_accelerator_config        cfg;
  srs_amd_pdsch_encoder*              tb_enc = nullptr;
  srs_amd_ldpc_encoder*               cb_enc = nullptr;
  srs_amd_ldpc_rate_matcher*          rm     = nullptr;
  hal::hw_pdsch_encoder_configuration ops[MAX_CBS] = {};
  bool                                ready[MAX_CBS] = {};
  std::vector<uint8_t>                out[MAX_CBS];
  std::vector<uint8_t>                msg, cb, packed;
};

class hip_pdsch_enc_acc_factory : public hal::hw_accelerator_pdsch_enc_factory
{
public:
  explicit hip_pdsch_enc_acc_factory(const pdsch_enc_accelerator_config& c) : cfg(c) {}
  std::unique_ptr<hal::hw_accelerator_pdsch_enc> create() override
  {
    return std::make_unique<hip_accelerator_pdsch_enc>(cfg);
  }

private:
  pdsch_enc_accelerator_config cfg;
};

} // namespace

std::shared_ptr<hal::hw_accelerator_pdsch_enc_factory>
srsran::hip::create_hip_pdsch_enc_acc_factory(const pdsch_enc_accelerator_config& cfg)
{
  return std::make_shared<hip_pdsch_enc_acc_factory>(cfg);
}
