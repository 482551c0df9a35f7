// hw_harness.cpp -- TEST INFRASTRUCTURE: drives the REFERENCE's own hardware-accelerated PUSCH decoder
// (lib/phy/upper/channel_processors/pusch/pusch_decoder_hw_impl.cpp, compiled from /root/reference into
// oracle/_ref/libsrsran_ref.so) with the MI355X plug-in (integration/hip_accelerator_pusch_dec.cpp,
// hal::hw_accelerator_pusch_dec over the srsran_amd C-ABI), so tests/test_integration_gpu.py can compare
// it with the reference's software pusch_decoder_impl (ref_wrapper_sch.cpp) on the same LLRs.
// Built by oracle/Makefile into oracle/_ref/libsrsran_ref_hw.so.  Never loaded by the product.
#include "ref_builders.h"

#include "../integration/hip_accelerator_pusch_dec.h"
#include "phy/upper/channel_coding/ldpc/ldpc_segmenter_rx_impl.h"
#include "phy/upper/channel_processors/pusch/pusch_decoder_hw_impl.h"
#include "srsran/phy/upper/channel_processors/pusch/pusch_decoder_notifier.h"
#include "srsran/phy/upper/channel_processors/pusch/pusch_decoder_result.h"
#include "srsran/phy/upper/unique_rx_buffer.h"
#include <memory>
#include <vector>

using namespace srsran;

namespace {

/// In-memory rx_buffer of one HARQ process whose codeblocks have absolute ids base + index (the role of
/// rx_buffer_impl); with an external-HARQ accelerator only the CRC flags and decoded messages live here.
class harq_process_buffer : public unique_rx_buffer::callback
{
public:
  harq_process_buffer(unsigned nof_cbs, unsigned base_) : base(base_), soft(nof_cbs), data(nof_cbs), crcs(nof_cbs, 0)
  {
    for (unsigned i = 0; i != nof_cbs; ++i) {
      soft[i].assign(3 * 8448 + 64, log_likelihood_ratio(0));
      data[i].resize(8448 + 64);
    }
  }
  unsigned   get_nof_codeblocks() const override { return soft.size(); }
  void       reset_codeblocks_crc() override { std::fill(crcs.begin(), crcs.end(), 0); }
  span<bool> get_codeblocks_crc() override { return span<bool>(reinterpret_cast<bool*>(crcs.data()), crcs.size()); }
  unsigned   get_absolute_codeblock_id(unsigned codeblock_id) const override { return base + codeblock_id; }
  span<log_likelihood_ratio> get_codeblock_soft_bits(unsigned id, unsigned size) override
  {
    return span<log_likelihood_ratio>(soft[id]).first(size);
  }
  bit_buffer get_codeblock_data_bits(unsigned id, unsigned size) override { return data[id].first(size); }
  bool       try_lock() override { return true; }
  void       unlock() override {}
  void       release() override {}

private:
  unsigned                                       base;
  std::vector<std::vector<log_likelihood_ratio>> soft;
  std::vector<dynamic_bit_buffer>                data;
  std::vector<char>                              crcs;
};

class result_catcher : public pusch_decoder_notifier
{
public:
  void on_sch_data(const pusch_decoder_result& r) override
  {
    result = r;
    done   = true;
  }
  pusch_decoder_result result;
  bool                 done = false;
};

modulation_scheme scheme_of(unsigned qm)
{
  switch (qm) {
    case 1:
      return modulation_scheme::BPSK;
    case 2:
      return modulation_scheme::QPSK;
    case 4:
      return modulation_scheme::QAM16;
    case 6:
      return modulation_scheme::QAM64;
    default:
      return modulation_scheme::QAM256;
  }
}

struct hw_context {
  std::shared_ptr<hal::hw_accelerator_pusch_dec_factory> factory;
  std::unique_ptr<pusch_decoder_hw_impl>                 decoder;
};

} // namespace

extern "C" {

/* The reference's pusch_decoder_hw_impl (no executor: synchronous) with a pool of one MI355X accelerator,
 * as pusch_decoder_factory_hw builds it (lib/phy/upper/channel_processors/pusch/factories.cpp:120-150). */
void* srs_ref_hw_ctx_create(int device, int generic)
{
  auto*                                   ctx = new hw_context();
  srsran::hip::pusch_dec_accelerator_config c;
  c.device    = device;
  c.arith     = generic ? 1 : 0;
  ctx->factory = srsran::hip::create_hip_pusch_dec_acc_factory(c);
  std::vector<std::unique_ptr<hal::hw_accelerator_pusch_dec>> hw(1);
  hw[0]     = ctx->factory->create();
  auto pool = std::make_shared<pusch_decoder_hw_impl::hw_decoder_pool>(hw);
  const auto   choice = generic ? srs_ref::impl::generic : srs_ref::impl::automatic;
  pusch_decoder_hw_impl::sch_crc crcs;
  crcs.crc16   = srs_ref::make_crc(crc_generator_poly::CRC16, choice);
  crcs.crc24A  = srs_ref::make_crc(crc_generator_poly::CRC24A, choice);
  crcs.crc24B  = srs_ref::make_crc(crc_generator_poly::CRC24B, choice);
  ctx->decoder = std::make_unique<pusch_decoder_hw_impl>(std::make_unique<ldpc_segmenter_rx_impl>(), crcs, pool, nullptr);
  return ctx;
}

/* A second pusch_decoder_hw_impl whose accelerator comes from the SAME factory as ctx's (one shared HBM
 * HARQ pool), for concurrent transport blocks on two threads. */
void* srs_ref_hw_ctx_sibling(void* base, int generic)
{
  auto* b   = static_cast<hw_context*>(base);
  auto* ctx = new hw_context();
  ctx->factory = b->factory;
  std::vector<std::unique_ptr<hal::hw_accelerator_pusch_dec>> hw(1);
  hw[0]     = ctx->factory->create();
  auto pool = std::make_shared<pusch_decoder_hw_impl::hw_decoder_pool>(hw);
  const auto   choice = generic ? srs_ref::impl::generic : srs_ref::impl::automatic;
  pusch_decoder_hw_impl::sch_crc crcs;
  crcs.crc16   = srs_ref::make_crc(crc_generator_poly::CRC16, choice);
  crcs.crc24A  = srs_ref::make_crc(crc_generator_poly::CRC24A, choice);
  crcs.crc24B  = srs_ref::make_crc(crc_generator_poly::CRC24B, choice);
  ctx->decoder = std::make_unique<pusch_decoder_hw_impl>(std::make_unique<ldpc_segmenter_rx_impl>(), crcs, pool, nullptr);
  return ctx;
}

void srs_ref_hw_ctx_destroy(void* ctx)
{
  delete static_cast<hw_context*>(ctx);
}

void* srs_ref_hw_rx_buffer_create(unsigned nof_cbs, unsigned abs_base)
{
  return new harq_process_buffer(nof_cbs, abs_base);
}

void srs_ref_hw_rx_buffer_destroy(void* b)
{
  delete static_cast<harq_process_buffer*>(b);
}

/* pusch_decoder::new_data + on_new_softbits + on_end_softbits through pusch_decoder_hw_impl.
 * result[0..5] as srs_ref_pusch_decode: tb_crc_ok, nof_codeblocks_total, nof observations, sum, min, max. */
int srs_ref_hw_pusch_decode(void*         ctx,
                            void*         rx_buffer,
                            const int8_t* llrs,
                            unsigned      nof_llrs,
                            uint8_t*      tb,
                            unsigned      tb_bytes,
                            unsigned      bg,
                            unsigned      rv,
                            unsigned      qm,
                            unsigned      Nref,
                            unsigned      nof_layers,
                            unsigned      nof_iterations,
                            int           use_early_stop,
                            int           new_data,
                            double*       result)
{
  auto&                        dec = *static_cast<hw_context*>(ctx)->decoder;
  pusch_decoder::configuration cfg;
  cfg.base_graph          = bg == 1 ? ldpc_base_graph_type::BG1 : ldpc_base_graph_type::BG2;
  cfg.rv                  = rv;
  cfg.mod                 = scheme_of(qm);
  cfg.Nref                = Nref;
  cfg.nof_layers          = nof_layers;
  cfg.nof_ldpc_iterations = nof_iterations;
  cfg.force_decoding      = false;
  cfg.use_early_stop      = use_early_stop != 0;
  cfg.new_data            = new_data != 0;
  result_catcher        notifier;
  unique_rx_buffer      buf(*static_cast<harq_process_buffer*>(rx_buffer));
  pusch_decoder_buffer& in = dec.new_data(span<uint8_t>(tb, tb_bytes), std::move(buf), notifier, cfg);
  in.on_new_softbits(span<const log_likelihood_ratio>(reinterpret_cast<const log_likelihood_ratio*>(llrs), nof_llrs));
  in.on_end_softbits();
  if (!notifier.done) {
    return -1;
  }
  const auto& st = notifier.result.ldpc_decoder_stats;
  result[0]      = notifier.result.tb_crc_ok ? 1 : 0;
  result[1]      = notifier.result.nof_codeblocks_total;
  result[2]      = st.get_nof_observations();
  result[3]      = st.get_mean() * st.get_nof_observations();
  result[4]      = st.get_min();
  result[5]      = st.get_max();
  return 0;
}

} // extern "C"
