// phy_harness.cpp -- TEST INFRASTRUCTURE: drives the MI355X channel-processor plug-ins of integration/
// (libsrsran_amd_phy.so: pusch_processor_hip, pdsch_processor_hip) the way the reference's upper PHY does, so
// tests/test_phy_plugins_gpu.py can compare them with the reference's own pusch_processor_impl /
// pdsch_processor_impl (compiled from /root/reference into oracle/_ref/libsrsran_ref.so) on the same inputs:
//   * received grids are the reference's resource_grid_reader_impl over a tensor (as ref_wrapper_pusch.cpp);
//   * PUSCH PDUs arrive as the C-ABI's srs_amd_pusch_pdu (the Python tests' PuschPdu) and are turned into the
//     reference's pusch_processor::pdu_t here, then handed to pusch_processor::process once per PDU -- what
//     uplink_processor_impl::process_pusch does (uplink_processor_impl.cpp:270-326) -- with a result notifier per
//     PDU and the reference's rx_buffer glue (ref_builders.h ref_rx_buffer) as HARQ buffer;
//   * the slot boundary is the factory's flush(), completion its wait_idle().
// Built by oracle/Makefile into oracle/_ref/libsrsran_ref_hw.so.  Never loaded by the product.
#include "ref_builders.h"

#include "../integration/hip_resource_grid.h"
#include "../integration/pdcch_processor_hip.h"
#include "../integration/ssb_processor_hip.h"
#include "../integration/pucch_processor_hip.h"
#include "srsran_amd/pucch.h"
#include "../integration/pdsch_processor_hip.h"
#include "../integration/pusch_processor_hip.h"
#include "phy/generic_functions/precoding/channel_precoder_avx2.h"
#include "phy/generic_functions/precoding/channel_precoder_avx512.h"
#include "phy/support/resource_grid_impl.h"
#include "phy/support/resource_grid_mapper_impl.h"
#include "phy/support/resource_grid_reader_impl.h"
#include "phy/support/resource_grid_writer_impl.h"
#include "phy/upper/channel_coding/ldpc/ldpc_encoder_avx2.h"
#include "phy/upper/channel_coding/ldpc/ldpc_rate_matcher_impl.h"
#include "phy/upper/channel_coding/ldpc/ldpc_segmenter_tx_impl.h"
#include "phy/upper/channel_modulation/modulation_mapper_lut_impl.h"
#include "phy/upper/channel_processors/pdsch/pdsch_encoder_impl.h"
#include "phy/upper/channel_processors/pdsch/pdsch_modulator_impl.h"
#include "phy/upper/channel_processors/pdsch/pdsch_processor_impl.h"
#include "phy/upper/signal_processors/pdsch/dmrs_pdsch_processor_impl.h"
#include "phy/upper/signal_processors/ptrs/ptrs_pdsch_generator_impl.h"
#include "ref_pdcch_pdu.h"
#include "ref_ssb_pdu.h"
#include "srsran_amd/pdsch_modulator.h"
#include "srsran/adt/tensor.h"
#include "srsran/fapi/messages/ul_tti_request.h"
#include "srsran/fapi_adaptor/phy/messages/pusch.h"
#include "srsran/fapi_adaptor/uci_part2_correspondence_repository.h"
#include "srsran/phy/upper/channel_processors/pusch/pusch_processor_result_notifier.h"
#include "srsran_amd/pusch_processor.h"
#include <algorithm>
#include <atomic>
#include <chrono>
#include <stdexcept>
#include <cmath>
#include <cstring>
#include <deque>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

using namespace srsran;
using namespace srs_ref;

namespace {

using grid_tensor =
    dynamic_tensor<static_cast<unsigned>(resource_grid_dimensions::all), cbf16_t, resource_grid_dimensions>;

/// A grid handle of the harness: a host grid (the reference's reader / writer over a tensor) or a device-resident
/// hip_resource_grid; the process functions take either.
struct any_grid {
  virtual ~any_grid()                           = default;
  virtual const resource_grid_reader& rd()      = 0;
  virtual resource_grid_writer&       wr()      = 0;
};

/// A received slot grid: the reference's reader over a tensor [port][symbol][subcarrier].
struct host_grid : any_grid {
  const resource_grid_reader& rd() override { return reader; }
  resource_grid_writer&       wr() override { throw std::runtime_error("read-only grid"); }
  host_grid(const uint32_t* g, unsigned nports, unsigned nsubc) :
    data({nsubc, MAX_NSYMB_PER_SLOT, nports}), reader(data, empty)
  {
    for (unsigned p = 0; p != nports; ++p) {
      for (unsigned l = 0; l != MAX_NSYMB_PER_SLOT; ++l) {
        span<cbf16_t> row = data.get_view<static_cast<unsigned>(resource_grid_dimensions::symbol)>({l, p});
        std::memcpy(row.data(), g + (p * MAX_NSYMB_PER_SLOT + l) * nsubc, nsubc * sizeof(cbf16_t));
      }
    }
  }
  grid_tensor               data;
  std::atomic<unsigned>     empty{0};
  resource_grid_reader_impl reader;
};

modulation_scheme scheme_of(int qm)
{
  switch (qm) {
    case 0:
      return modulation_scheme::PI_2_BPSK;
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

// srs_amd_pusch_pdu -> the reference's pdu_t (rx ports 0 .. nof_rx_ports - 1, type-1 allocation).
pusch_processor::pdu_t to_pdu(const srs_amd_pusch_pdu& c)
{
  pusch_processor::pdu_t pdu = {};
  pdu.slot                   = slot_point(c.numerology, c.slot_index);
  pdu.rnti                   = static_cast<uint16_t>(c.rnti);
  pdu.bwp_size_rb            = c.bwp_size_rb;
  pdu.bwp_start_rb           = c.bwp_start_rb;
  pdu.cp                     = cyclic_prefix::NORMAL;
  pdu.mcs_descr              = sch_mcs_description{scheme_of(c.modulation), c.target_code_rate};
  pdu.codeword.emplace(pusch_processor::codeword_description{
      c.rv, c.base_graph == 1 ? ldpc_base_graph_type::BG1 : ldpc_base_graph_type::BG2, c.new_data != 0});
  pdu.uci.nof_harq_ack          = c.nof_harq_ack;
  pdu.uci.nof_csi_part1         = c.nof_csi_part1;
  pdu.uci.alpha_scaling         = c.alpha_scaling;
  pdu.uci.beta_offset_harq_ack  = c.beta_offset_harq_ack;
  pdu.uci.beta_offset_csi_part1 = c.beta_offset_csi_part1;
  pdu.uci.beta_offset_csi_part2 = c.beta_offset_csi_part2;
  for (unsigned e = 0; e != c.csi_part2_size.nof_entries; ++e) {
    const srs_amd_uci_part2_entry&     x  = c.csi_part2_size.entries[e];
    uci_part2_size_description::entry& en = pdu.uci.csi_part2_size.entries.emplace_back();
    for (unsigned q = 0; q != x.nof_parameters; ++q) {
      en.parameters.push_back(
          uci_part2_size_description::parameter{x.parameters[q].offset, static_cast<uint8_t>(x.parameters[q].width)});
    }
    for (unsigned m = 0; m != x.map_size; ++m) {
      en.map.push_back(x.map[m]);
    }
  }
  pdu.n_id          = c.n_id;
  pdu.nof_tx_layers = c.nof_tx_layers;
  for (unsigned p = 0; p != c.nof_rx_ports; ++p) {
    pdu.rx_ports.push_back(static_cast<uint8_t>(p));
  }
  pdu.dmrs_symbol_mask = symbol_slot_mask(MAX_NSYMB_PER_SLOT);
  for (unsigned l = 0; l != MAX_NSYMB_PER_SLOT; ++l) {
    if ((c.dmrs_symbol_mask >> l) & 1u) {
      pdu.dmrs_symbol_mask.set(l);
    }
  }
  if (c.transform_precoding) {
    pdu.dmrs = pusch_processor::dmrs_transform_precoding_configuration{.n_rs_id = c.n_rs_id};
  } else {
    pdu.dmrs = pusch_processor::dmrs_configuration{.dmrs          = c.dmrs_type == 2 ? dmrs_type::TYPE2 : dmrs_type::TYPE1,
                                                   .scrambling_id = c.scrambling_id,
                                                   .n_scid        = c.n_scid != 0,
                                                   .nof_cdm_groups_without_data = c.nof_cdm_groups_without_data};
  }
  pdu.freq_alloc         = rb_allocation::make_type1(c.rb_start, c.rb_count);
  pdu.start_symbol_index = c.start_symbol_index;
  pdu.nof_symbols        = c.nof_symbols;
  pdu.tbs_lbrm           = c.tbs_lbrm_bytes ? units::bytes(c.tbs_lbrm_bytes) : tbs_lbrm_default;
  return pdu;
}

/// The notifications of one process() call (a UCI-only PDU completes with on_uci: expect_sch = false).
class ticket : public pusch_processor_result_notifier
{
public:
  void on_uci(const pusch_processor_result_control& u) override
  {
    uci = u;
    ++nof_uci;
    if (!expect_sch) {
      done.store(true, std::memory_order_release);
    }
  }
  void on_sch(const pusch_processor_result_data& s) override
  {
    sch = s;
    done.store(true, std::memory_order_release);
  }
  pusch_processor_result_control uci;
  pusch_processor_result_data    sch;
  unsigned                       nof_uci    = 0;
  bool                           expect_sch = true;
  std::atomic<bool>              done{false};
};

/// A flat FAPI UL_TTI.request PUSCH PDU (SCF-222 v4.0 3.4.3.2, fapi::ul_pusch_pdu): the fields the reference's
/// MAC -> FAPI translator fills for a type-1 PUSCH (test glue; converted by the reference's own
/// convert_pusch_fapi_to_phy, lib/fapi_adaptor/phy/messages/pusch.cpp).
struct srs_ref_fapi_pusch {
  uint32_t rnti, bwp_start, bwp_size, numerology, sfn, slot;
  int32_t  qm;               /* modulation order code (0 pi/2-BPSK, 2, 4, 6, 8) */
  uint32_t target_code_rate; /* R x 1024 x 10 */
  uint32_t transform_precoding, nid_pusch, num_layers, ul_dmrs_symb_pos, dmrs_type, scrambling_id, dmrs_identity;
  uint32_t nscid, num_dmrs_cdm_grps_no_data, rb_start, rb_size, start_symbol_index, nr_of_symbols;
  uint32_t tx_direct_current_location; /* >= 3300: not set */
  uint32_t has_data, rv_index, harq_process_id, new_data, tb_size, ldpc_base_graph, tb_size_lbrm_bytes;
  uint32_t has_uci, harq_ack_bit_length, csi_part1_bit_length, alpha_scaling, beta_offset_harq_ack, beta_offset_csi1,
      beta_offset_csi2;
  uint32_t num_rx_ant;
};

struct fapi_pusch_handle {
  uplink_pdu_slot_repository::pusch_pdu pdu;
};

struct pusch_ctx {
  std::shared_ptr<hip::pusch_processor_factory_hip> factory;
  std::unique_ptr<pusch_processor>                  proc;
  std::deque<ticket>                                tickets;
  std::mutex                                        mtx;
};

// ---- PDSCH ----

/// A flat pdsch_processor::pdu_t (test glue): type-0 allocation of the BWP's VRBs (non-interleaved), one codeword,
/// wideband precoding, reserved RE patterns.
struct srs_ref_pdsch_pdu {
  uint32_t           numerology, slot_index, rnti, bwp_start_rb, bwp_size_rb;
  int32_t            qm;
  uint32_t           rv, n_id, ref_point; // ref_point: 0 CRB0, 1 PRB0
  uint32_t           dmrs_symbol_mask, dmrs_type, scrambling_id, n_scid, nof_cdm_groups_without_data;
  uint8_t            vrb_mask[SRS_AMD_CRB_MASK_BYTES];
  uint8_t            pad;
  uint32_t           start_symbol_index, nof_symbols, base_graph, tbs_lbrm_bytes;
  float              ratio_pdsch_dmrs_to_sss_dB, ratio_pdsch_data_to_sss_dB;
  uint32_t           nof_layers, nof_ports;
  float              weights[4][4][2];
  uint32_t           nof_reserved;
  srs_amd_re_pattern reserved[SRS_AMD_MAX_RE_PATTERNS];
  // PT-RS (has_ptrs != 0) and per-PRG precoding (nof_prg > 1: PRG g >= 1 from prg_weights[g - 1])
  uint32_t           has_ptrs, ptrs_freq_density, ptrs_time_density, ptrs_re_offset;
  float              ratio_ptrs_to_pdsch_data_dB;
  uint32_t           nof_prg, prg_size;
  float              prg_weights[7][4][4][2];
};

pdsch_processor::pdu_t to_pdsch_pdu(const srs_ref_pdsch_pdu& c)
{
  pdsch_processor::pdu_t pdu = {};
  pdu.slot                   = slot_point(c.numerology, c.slot_index);
  pdu.rnti                   = static_cast<uint16_t>(c.rnti);
  pdu.bwp_size_rb            = c.bwp_size_rb;
  pdu.bwp_start_rb           = c.bwp_start_rb;
  pdu.cp                     = cyclic_prefix::NORMAL;
  pdu.codewords.push_back(pdsch_processor::codeword_description{scheme_of(c.qm), c.rv});
  pdu.n_id             = c.n_id;
  pdu.ref_point        = c.ref_point ? pdsch_processor::pdu_t::PRB0 : pdsch_processor::pdu_t::CRB0;
  pdu.dmrs_symbol_mask = symbol_slot_mask(MAX_NSYMB_PER_SLOT);
  for (unsigned l = 0; l != MAX_NSYMB_PER_SLOT; ++l) {
    if ((c.dmrs_symbol_mask >> l) & 1u) {
      pdu.dmrs_symbol_mask.set(l);
    }
  }
  pdu.dmrs                        = c.dmrs_type == 2 ? dmrs_type::TYPE2 : dmrs_type::TYPE1;
  pdu.scrambling_id               = c.scrambling_id;
  pdu.n_scid                      = c.n_scid != 0;
  pdu.nof_cdm_groups_without_data = c.nof_cdm_groups_without_data;
  vrb_bitmap vrbs(c.bwp_size_rb);
  for (unsigned i = 0; i != c.bwp_size_rb; ++i) {
    if ((c.vrb_mask[i / 8] >> (i % 8)) & 1u) {
      vrbs.set(i);
    }
  }
  pdu.freq_alloc         = rb_allocation::make_type0(vrbs);
  pdu.start_symbol_index = c.start_symbol_index;
  pdu.nof_symbols        = c.nof_symbols;
  pdu.ldpc_base_graph    = c.base_graph == 1 ? ldpc_base_graph_type::BG1 : ldpc_base_graph_type::BG2;
  pdu.tbs_lbrm           = c.tbs_lbrm_bytes ? units::bytes(c.tbs_lbrm_bytes) : tbs_lbrm_default;
  for (unsigned r = 0; r != c.nof_reserved; ++r) {
    re_pattern pat;
    pat.crb_mask = crb_bitmap(MAX_NOF_PRBS);
    for (unsigned i = 0; i != MAX_NOF_PRBS; ++i) {
      if ((c.reserved[r].crb_mask[i / 8] >> (i % 8)) & 1u) {
        pat.crb_mask.set(i);
      }
    }
    for (unsigned k = 0; k != NRE; ++k) {
      if ((c.reserved[r].re_mask >> k) & 1u) {
        pat.re_mask.set(k);
      }
    }
    for (unsigned l = 0; l != MAX_NSYMB_PER_SLOT; ++l) {
      if ((c.reserved[r].symbols >> l) & 1u) {
        pat.symbols.set(l);
      }
    }
    pdu.reserved.merge(pat);
  }
  pdu.ratio_pdsch_dmrs_to_sss_dB = c.ratio_pdsch_dmrs_to_sss_dB;
  pdu.ratio_pdsch_data_to_sss_dB = c.ratio_pdsch_data_to_sss_dB;
  precoding_weight_matrix w(c.nof_layers, c.nof_ports);
  for (unsigned l = 0; l != c.nof_layers; ++l) {
    for (unsigned q = 0; q != c.nof_ports; ++q) {
      w.set_coefficient(cf_t(c.weights[l][q][0], c.weights[l][q][1]), l, q);
    }
  }
  if (c.nof_prg > 1) {
    pdu.precoding = precoding_configuration(c.nof_layers, c.nof_ports, c.nof_prg, c.prg_size);
    for (unsigned g = 0; g != c.nof_prg; ++g) {
      for (unsigned l = 0; l != c.nof_layers; ++l) {
        for (unsigned q = 0; q != c.nof_ports; ++q) {
          const float* v = g == 0 ? c.weights[l][q] : c.prg_weights[g - 1][l][q];
          pdu.precoding.set_coefficient(cf_t(v[0], v[1]), l, q, g);
        }
      }
    }
  } else {
    pdu.precoding = precoding_configuration::make_wideband(w);
  }
  if (c.has_ptrs) {
    pdu.ptrs = pdsch_processor::ptrs_configuration{static_cast<ptrs_frequency_density>(c.ptrs_freq_density),
                                                   static_cast<ptrs_time_density>(c.ptrs_time_density),
                                                   static_cast<ptrs_re_offset>(c.ptrs_re_offset),
                                                   c.ratio_ptrs_to_pdsch_data_dB};
  }
  return pdu;
}

/// A device-resident grid: hip_resource_grid (integration/hip_resource_grid.h) over the reference's resource_grid_impl.
struct dev_grid : any_grid {
  dev_grid(unsigned nports, unsigned nsubc, int device) :
    grid(std::make_unique<resource_grid_impl>(nports, MAX_NSYMB_PER_SLOT, nsubc), device)
  {
  }
  const resource_grid_reader& rd() override { return grid.get_reader(); }
  resource_grid_writer&       wr() override { return grid.get_writer(); }
  hip::hip_resource_grid      grid;
};

/// A slot grid written through the reference's resource_grid_writer_impl over a tensor [port][symbol][subcarrier].
struct host_wgrid : any_grid {
  const resource_grid_reader& rd() override { throw std::runtime_error("write-only grid"); }
  resource_grid_writer&       wr() override { return writer; }
  host_wgrid(const uint32_t* g, unsigned nports_, unsigned nsubc_) :
    nports(nports_), nsubc(nsubc_), data({nsubc_, MAX_NSYMB_PER_SLOT, nports_}), writer(data, empty)
  {
    store(g);
  }
  void store(const uint32_t* g)
  {
    for (unsigned p = 0; p != nports; ++p) {
      for (unsigned l = 0; l != MAX_NSYMB_PER_SLOT; ++l) {
        span<cbf16_t> row = data.get_view<static_cast<unsigned>(resource_grid_dimensions::symbol)>({l, p});
        std::memcpy(row.data(), g + (p * MAX_NSYMB_PER_SLOT + l) * nsubc, nsubc * sizeof(cbf16_t));
      }
    }
  }
  void load(uint32_t* g)
  {
    for (unsigned p = 0; p != nports; ++p) {
      for (unsigned l = 0; l != MAX_NSYMB_PER_SLOT; ++l) {
        span<cbf16_t> row = data.get_view<static_cast<unsigned>(resource_grid_dimensions::symbol)>({l, p});
        std::memcpy(g + (p * MAX_NSYMB_PER_SLOT + l) * nsubc, row.data(), nsubc * sizeof(cbf16_t));
      }
    }
  }
  unsigned                  nports, nsubc;
  grid_tensor               data;
  std::atomic<unsigned>     empty{0};
  resource_grid_writer_impl writer;
};

class pdsch_ticket : public pdsch_processor_notifier
{
public:
  void              on_finish_processing() override { done.store(true, std::memory_order_release); }
  std::atomic<bool> done{false};
};

struct pdsch_ctx {
  std::shared_ptr<hip::pdsch_processor_factory_hip> factory;
  std::unique_ptr<pdsch_processor>                  proc;
  std::deque<pdsch_ticket>                          tickets;
  std::deque<std::vector<uint8_t>>                  tbs; // the transport blocks' storage (shared_transport_block views)
  std::mutex                                        mtx;
};

// The reference's pdsch_processor_impl with the "auto" components of this host (as ref_chain.cpp).
std::unique_ptr<pdsch_processor_impl> make_ref_pdsch_processor()
{
  auto precoder = []() -> std::unique_ptr<channel_precoder> {
    if (host_has_avx512_ldpc()) {
      return std::make_unique<channel_precoder_avx512>();
    }
    return std::make_unique<channel_precoder_avx2>();
  };
  ldpc_segmenter_tx_impl::sch_crc crcs;
  crcs.crc16  = make_crc(crc_generator_poly::CRC16, impl::automatic);
  crcs.crc24A = make_crc(crc_generator_poly::CRC24A, impl::automatic);
  crcs.crc24B = make_crc(crc_generator_poly::CRC24B, impl::automatic);
  return std::make_unique<pdsch_processor_impl>(
      std::make_unique<pdsch_encoder_impl>(std::make_unique<ldpc_segmenter_tx_impl>(crcs),
                                           std::make_unique<ldpc_encoder_avx2>(),
                                           std::make_unique<ldpc_rate_matcher_impl>()),
      std::make_unique<pdsch_modulator_impl>(std::make_unique<modulation_mapper_lut_impl>(),
                                             std::make_unique<pseudo_random_generator_impl>(),
                                             std::make_unique<resource_grid_mapper_impl>(precoder())),
      std::make_unique<dmrs_pdsch_processor_impl>(std::make_unique<pseudo_random_generator_impl>(),
                                                  std::make_unique<resource_grid_mapper_impl>(precoder())),
      std::make_unique<ptrs_pdsch_generator_generic_impl>(std::make_unique<pseudo_random_generator_impl>(),
                                                          std::make_unique<resource_grid_mapper_impl>(precoder())));
}

void bits_out(const uci_payload_type& p, uint8_t* out)
{
  for (unsigned i = 0; i != p.size(); ++i) {
    out[i] = p.test(i) ? 1 : 0;
  }
}

} // namespace

extern "C" {

/* The MI355X PUSCH processor factory (pusch_processor_factory_hip) and one of its processors. eq: 0 ZF, 1 MMSE.
 * max_wait_us: the collector's timer (0: only flush / slot change / batch size).  NULL on failure. */
void* srs_ref_phy_pusch_create(int device, unsigned nof_prb, unsigned iterations, int eq, int generic,
                               unsigned max_wait_us)
{
  hip::pusch_processor_hip_config cfg;
  cfg.device             = device;
  cfg.nof_prb            = nof_prb;
  cfg.dec_nof_iterations = iterations;
  cfg.equalizer = eq ? channel_equalizer_algorithm_type::mmse : channel_equalizer_algorithm_type::zf;
  cfg.generic_ldpc = generic != 0;
  cfg.max_wait_us  = max_wait_us;
  auto f           = hip::create_pusch_processor_factory_hip(cfg);
  if (!f) {
    return nullptr;
  }
  auto* ctx    = new pusch_ctx;
  ctx->factory = f;
  ctx->proc    = f->create();
  return ctx;
}

void srs_ref_phy_pusch_destroy(void* h)
{
  auto* ctx = static_cast<pusch_ctx*>(h);
  ctx->factory->wait_idle();
  delete ctx;
}

/* A second processor of the same factory (shares the collector): another cell of the node. */
void* srs_ref_phy_pusch_sibling(void* h)
{
  auto* base   = static_cast<pusch_ctx*>(h);
  auto* ctx    = new pusch_ctx;
  ctx->factory = base->factory;
  ctx->proc    = base->factory->create();
  return ctx;
}

void* srs_ref_phy_grid_create(const uint32_t* grid, unsigned nports, unsigned nsubc)
{
  return new host_grid(grid, nports, nsubc);
}

void srs_ref_phy_grid_destroy(void* g)
{
  delete static_cast<any_grid*>(g);
}

/* pusch_processor::process of one PDU (asynchronous); rx_buffer: an srs_ref_rx_buffer_create handle or NULL (no
 * HARQ buffer, as a failed reservation).  Returns the ticket of the call. */
int srs_ref_phy_pusch_process(void* h, void* grid, const srs_amd_pusch_pdu* c, void* rx_buffer, uint8_t* tb,
                              unsigned tb_bytes)
{
  auto*   ctx = static_cast<pusch_ctx*>(h);
  ticket* t;
  int     id;
  {
    std::lock_guard<std::mutex> lock(ctx->mtx);
    id = static_cast<int>(ctx->tickets.size());
    t  = &ctx->tickets.emplace_back();
  }
  unique_rx_buffer buf = rx_buffer ? unique_rx_buffer(*static_cast<ref_rx_buffer*>(rx_buffer)) : unique_rx_buffer();
  ctx->proc->process(span<uint8_t>(tb, tb_bytes), std::move(buf), *t, static_cast<any_grid*>(grid)->rd(),
                     to_pdu(*c));
  return id;
}

void srs_ref_phy_pusch_flush(void* h)
{
  static_cast<pusch_ctx*>(h)->factory->flush();
}

void srs_ref_phy_pusch_wait(void* h)
{
  static_cast<pusch_ctx*>(h)->factory->wait_idle();
}

/* Result of a ticket: 0 not notified yet, 1 done.  result[0..5] as srs_ref_pusch_process (tb_crc_ok, nof_codeblocks,
 * LDPC observations, sum, min, max); csi[0..4] = SINR, EPRE, RSRP (dB), time alignment (s), CFO (Hz, NaN: none);
 * uci[0..4] = on_uci calls, HARQ-ACK / CSI part 1 / CSI part 2 statuses, CSI part 2 bits; payloads one bit per
 * byte into ack / csi1 / csi2 (NULL: not returned). */
int srs_ref_phy_pusch_result(void* h, int id, double* result, double* csi, int* uci, uint8_t* ack, uint8_t* csi1,
                             uint8_t* csi2)
{
  auto*   ctx = static_cast<pusch_ctx*>(h);
  ticket* t;
  {
    std::lock_guard<std::mutex> lock(ctx->mtx);
    if (id < 0 || static_cast<size_t>(id) >= ctx->tickets.size()) {
      return -1;
    }
    t = &ctx->tickets[id];
  }
  if (!t->done.load(std::memory_order_acquire)) {
    return 0;
  }
  const pusch_decoder_result& r  = t->sch.data;
  const auto&                 st = r.ldpc_decoder_stats;
  result[0]                      = r.tb_crc_ok ? 1 : 0;
  result[1]                      = r.nof_codeblocks_total;
  result[2]                      = st.get_nof_observations();
  result[3]                      = st.get_mean() * st.get_nof_observations();
  result[4]                      = st.get_min();
  result[5]                      = st.get_max();
  const channel_state_information& c = t->expect_sch ? t->sch.csi : t->uci.csi;
  csi[0]                             = c.get_sinr_dB().value_or(NAN);
  csi[1]                             = c.get_epre_dB().value_or(NAN);
  csi[2]                             = c.get_rsrp_dB().value_or(NAN);
  csi[3]                             = c.get_time_alignment().has_value() ? c.get_time_alignment()->to_seconds() : NAN;
  csi[4]                             = c.get_cfo_Hz().value_or(NAN);
  uci[0]                             = static_cast<int>(t->nof_uci);
  uci[1]                             = static_cast<int>(t->uci.harq_ack.status);
  uci[2]                             = static_cast<int>(t->uci.csi_part1.status);
  uci[3]                             = static_cast<int>(t->uci.csi_part2.status);
  uci[4]                             = static_cast<int>(t->uci.csi_part2.payload.size());
  if (ack != nullptr) {
    bits_out(t->uci.harq_ack.payload, ack);
  }
  if (csi1 != nullptr) {
    bits_out(t->uci.csi_part1.payload, csi1);
  }
  if (csi2 != nullptr) {
    bits_out(t->uci.csi_part2.payload, csi2);
  }
  return 1;
}

/* fapi::ul_pusch_pdu from the flat description, converted to the PHY's PUSCH PDU by the reference's
 * convert_pusch_fapi_to_phy (what the FAPI adaptor does for every UL_TTI.request PUSCH PDU).  Returns a handle (free
 * with srs_ref_fapi_pusch_free); dc_out: the converted pdu_t::dc_position (-1: unset); tb_bytes_out: tb_size. */
void* srs_ref_fapi_pusch_convert(const srs_ref_fapi_pusch* f, int* dc_out, unsigned* tb_bytes_out)
{
  fapi::ul_pusch_pdu fp = {};
  fp.pdu_bitmap.set(fapi::ul_pusch_pdu::PUSCH_DATA_BIT, f->has_data != 0);
  fp.pdu_bitmap.set(fapi::ul_pusch_pdu::PUSCH_UCI_BIT, f->has_uci != 0);
  fp.pdu_bitmap.set(fapi::ul_pusch_pdu::DFTS_OFDM_BIT, f->transform_precoding != 0);
  fp.rnti                      = to_rnti(f->rnti);
  fp.bwp_size                  = static_cast<uint16_t>(f->bwp_size);
  fp.bwp_start                 = static_cast<uint16_t>(f->bwp_start);
  fp.scs                       = to_subcarrier_spacing(f->numerology);
  fp.cp                        = cyclic_prefix::NORMAL;
  fp.target_code_rate          = static_cast<uint16_t>(f->target_code_rate);
  fp.qam_mod_order             = scheme_of(f->qm);
  fp.transform_precoding       = f->transform_precoding != 0;
  fp.nid_pusch                 = static_cast<uint16_t>(f->nid_pusch);
  fp.num_layers                = static_cast<uint8_t>(f->num_layers);
  fp.ul_dmrs_symb_pos          = static_cast<uint16_t>(f->ul_dmrs_symb_pos);
  fp.dmrs_type                 = f->dmrs_type == 2 ? fapi::dmrs_cfg_type::type_2 : fapi::dmrs_cfg_type::type_1;
  fp.pusch_dmrs_scrambling_id  = static_cast<uint16_t>(f->scrambling_id);
  fp.pusch_dmrs_identity       = static_cast<uint16_t>(f->dmrs_identity);
  fp.nscid                     = static_cast<uint8_t>(f->nscid);
  fp.num_dmrs_cdm_grps_no_data = static_cast<uint8_t>(f->num_dmrs_cdm_grps_no_data);
  fp.resource_alloc            = fapi::resource_allocation_type::type_1;
  fp.rb_start                  = static_cast<uint16_t>(f->rb_start);
  fp.rb_size                   = static_cast<uint16_t>(f->rb_size);
  fp.tx_direct_current_location = static_cast<uint16_t>(f->tx_direct_current_location);
  fp.start_symbol_index        = static_cast<uint8_t>(f->start_symbol_index);
  fp.nr_of_symbols             = static_cast<uint8_t>(f->nr_of_symbols);
  fp.pusch_data.rv_index        = static_cast<uint8_t>(f->rv_index);
  fp.pusch_data.harq_process_id = static_cast<uint8_t>(f->harq_process_id);
  fp.pusch_data.new_data        = f->new_data != 0;
  fp.pusch_data.tb_size         = units::bytes(f->tb_size);
  fp.pusch_maintenance_v3.ldpc_base_graph =
      f->ldpc_base_graph == 2 ? ldpc_base_graph_type::BG2 : ldpc_base_graph_type::BG1;
  fp.pusch_maintenance_v3.tb_size_lbrm_bytes = units::bytes(f->tb_size_lbrm_bytes);
  fp.pusch_uci.harq_ack_bit_length  = static_cast<uint16_t>(f->harq_ack_bit_length);
  fp.pusch_uci.csi_part1_bit_length = static_cast<uint16_t>(f->csi_part1_bit_length);
  fp.pusch_uci.flags_csi_part2      = 0;
  fp.pusch_uci.alpha_scaling        = static_cast<alpha_scaling_opt>(f->alpha_scaling);
  fp.pusch_uci.beta_offset_harq_ack = static_cast<uint8_t>(f->beta_offset_harq_ack);
  fp.pusch_uci.beta_offset_csi1     = static_cast<uint8_t>(f->beta_offset_csi1);
  fp.pusch_uci.beta_offset_csi2     = static_cast<uint8_t>(f->beta_offset_csi2);
  std::vector<static_vector<uint16_t, uci_part2_size_description::max_size_table>> part2(1);
  fapi_adaptor::uci_part2_correspondence_repository repo(std::move(part2));
  auto* h = new fapi_pusch_handle{};
  fapi_adaptor::convert_pusch_fapi_to_phy(h->pdu, fp, static_cast<uint16_t>(f->sfn), static_cast<uint16_t>(f->slot),
                                          static_cast<uint16_t>(f->num_rx_ant), repo);
  if (!fp.pdu_bitmap.test(fapi::ul_pusch_pdu::PUSCH_DATA_BIT)) {
    h->pdu.tb_size = units::bytes(0);
  }
  *dc_out       = h->pdu.pdu.dc_position.has_value() ? static_cast<int>(*h->pdu.pdu.dc_position) : -1;
  *tb_bytes_out = static_cast<unsigned>(h->pdu.tb_size.value());
  return h;
}

/* The converted PDU's floating-point fields: out[0..4] = mcs_descr.target_code_rate (R x 1024), uci.alpha_scaling,
 * uci.beta_offset_harq_ack, uci.beta_offset_csi_part1, uci.beta_offset_csi_part2. */
void srs_ref_fapi_pusch_params(void* h, float* out)
{
  const auto& pdu = static_cast<fapi_pusch_handle*>(h)->pdu.pdu;
  out[0]          = pdu.mcs_descr.target_code_rate;
  out[1]          = pdu.uci.alpha_scaling;
  out[2]          = pdu.uci.beta_offset_harq_ack;
  out[3]          = pdu.uci.beta_offset_csi_part1;
  out[4]          = pdu.uci.beta_offset_csi_part2;
}

void srs_ref_fapi_pusch_free(void* h)
{
  delete static_cast<fapi_pusch_handle*>(h);
}

/* pusch_processor::process of the plug-in with a converted FAPI PDU (asynchronous).  Returns the ticket. */
int srs_ref_phy_pusch_process_fapi(void* h, void* grid, void* fapi_pdu, void* rx_buffer, uint8_t* tb,
                                   unsigned tb_bytes)
{
  auto*       ctx = static_cast<pusch_ctx*>(h);
  const auto& pdu = static_cast<fapi_pusch_handle*>(fapi_pdu)->pdu.pdu;
  ticket*     t;
  int         id;
  {
    std::lock_guard<std::mutex> lock(ctx->mtx);
    id            = static_cast<int>(ctx->tickets.size());
    t             = &ctx->tickets.emplace_back();
    t->expect_sch = pdu.codeword.has_value();
  }
  unique_rx_buffer buf = rx_buffer ? unique_rx_buffer(*static_cast<ref_rx_buffer*>(rx_buffer)) : unique_rx_buffer();
  ctx->proc->process(span<uint8_t>(tb, tb_bytes), std::move(buf), *t, static_cast<any_grid*>(grid)->rd(), pdu);
  return id;
}

/* The REFERENCE's pusch_processor_impl (the "auto" decoder, ZF, filter FD smoothing, interpolate TD, CFO
 * compensation, as srs_ref_pusch_process) on the same converted FAPI PDU and grid.  Outputs as
 * srs_ref_phy_pusch_result (uci[0..4]); returns 0 when notified (on_sch, or on_uci for a UCI-only PDU), -1 otherwise. */
int srs_ref_pusch_process_fapi(void* grid, void* fapi_pdu, unsigned nof_prb, unsigned iterations, void* rx_buffer,
                               uint8_t* tb, unsigned tb_bytes, double* result, double* csi, int* uci, uint8_t* ack,
                               uint8_t* csi1)
{
  const auto& pdu    = static_cast<fapi_pusch_handle*>(fapi_pdu)->pdu.pdu;
  auto        bundle = make_pusch_processor(impl::automatic, nof_prb, static_cast<unsigned>(pdu.rx_ports.size()), 4,
                                            iterations, 0, 2, 0, true);
  ticket      t;
  t.expect_sch         = pdu.codeword.has_value();
  unique_rx_buffer buf = rx_buffer ? unique_rx_buffer(*static_cast<ref_rx_buffer*>(rx_buffer)) : unique_rx_buffer();
  bundle->proc->process(span<uint8_t>(tb, tb_bytes), std::move(buf), t, static_cast<any_grid*>(grid)->rd(), pdu);
  if (!t.done.load()) {
    return -1;
  }
  const pusch_decoder_result& r  = t.sch.data;
  const auto&                 st = r.ldpc_decoder_stats;
  result[0]                      = r.tb_crc_ok ? 1 : 0;
  result[1]                      = r.nof_codeblocks_total;
  result[2]                      = st.get_nof_observations();
  result[3]                      = st.get_mean() * st.get_nof_observations();
  result[4]                      = st.get_min();
  result[5]                      = st.get_max();
  const channel_state_information& c = t.expect_sch ? t.sch.csi : t.uci.csi;
  csi[0]                             = c.get_sinr_dB().value_or(NAN);
  csi[1]                             = c.get_epre_dB().value_or(NAN);
  csi[2]                             = c.get_rsrp_dB().value_or(NAN);
  csi[3]                             = c.get_time_alignment().has_value() ? c.get_time_alignment()->to_seconds() : NAN;
  csi[4]                             = c.get_cfo_Hz().value_or(NAN);
  uci[0]                             = static_cast<int>(t.nof_uci);
  uci[1]                             = static_cast<int>(t.uci.harq_ack.status);
  uci[2]                             = static_cast<int>(t.uci.csi_part1.status);
  uci[3]                             = static_cast<int>(t.uci.csi_part2.status);
  uci[4]                             = static_cast<int>(t.uci.csi_part2.payload.size());
  if (ack != nullptr) {
    bits_out(t.uci.harq_ack.payload, ack);
  }
  if (csi1 != nullptr) {
    bits_out(t.uci.csi_part1.payload, csi1);
  }
  return 0;
}

/* Plug-in statistics: PDUs, batches, errors, HARQ re-decodes, retransmissions, device grids, soft-buffer downloads,
 * host us: staging, buffer-set wait, result wait, notification. */
void srs_ref_phy_pusch_stats(void* h, uint64_t* out)
{
  const auto s = static_cast<pusch_ctx*>(h)->factory->get_statistics();
  out[0]       = s.nof_pdus;
  out[1]       = s.nof_batches;
  out[2]       = s.nof_errors;
  out[3]       = s.nof_harq_redecodes;
  out[4]       = s.nof_retransmissions;
  out[5]       = s.nof_device_grids;
  out[6]       = s.nof_harq_soft_downloads;
  out[7]       = s.stage_us;
  out[8]       = s.set_wait_us;
  out[9]       = s.wait_us;
  out[10]      = s.notify_us;
  out[11]      = s.stage_reads_us;
  out[12]      = s.stage_call_us;
  out[13]      = s.stage_download_us;
}

/* Throughput through the plug-in as the upper PHY drives it: every step, one PDU per cell grid (nof_cells grids,
 * each with its own processor of the factory, i.e. one cell each), process() per PDU, flush() at the slot boundary.
 * depth 1: every notification awaited before the next step; depth d > 1: d slots in flight, as the uplink processor
 * keeps them (a slot's PUSCH is processed while the next slots' symbols arrive): step s waits only for the
 * notifications of step s - d, and uses grids[(s % d) * nof_cells + i] (d sets of grids).  tbs: nof_cells rows of
 * tb_bytes.  Returns seconds per step over `steps` timed steps after `warmup`; ok_out: TBs with CRC OK in the timed
 * steps. */
double srs_ref_phy_pusch_bench(void* h, void* const* grids, unsigned nof_cells, unsigned depth,
                               const srs_amd_pusch_pdu* c, unsigned warmup, unsigned steps, uint8_t* tbs,
                               unsigned tb_bytes, unsigned* ok_out)
{
  auto*                                         ctx = static_cast<pusch_ctx*>(h);
  std::vector<std::unique_ptr<pusch_processor>> procs;
  for (unsigned i = 0; i != nof_cells; ++i) {
    procs.push_back(ctx->factory->create());
  }
  depth = std::max(depth, 1u);
  std::vector<ticket>     tickets(static_cast<size_t>(nof_cells) * depth);
  std::vector<char>       timed(depth, 0);
  const srs_amd_pusch_pdu pc = *c; // the grids hold one slot's DM-RS: every step is that slot again
  unsigned                ok = 0;
  auto                    collect = [&](unsigned b) {
    for (unsigned i = 0; i != nof_cells; ++i) {
      ticket& t = tickets[static_cast<size_t>(b) * nof_cells + i];
      while (!t.done.load(std::memory_order_acquire)) {
        std::this_thread::sleep_for(std::chrono::microseconds(20)); // (a sleeping poll: no spinning host thread)
      }
      ok += timed[b] && t.sch.data.tb_crc_ok ? 1 : 0;
    }
  };
  auto t0 = std::chrono::steady_clock::now();
  for (unsigned s = 0; s != warmup + steps; ++s) {
    const unsigned b = s % depth;
    if (s == warmup) {
      // the warm-up steps drained: the timed region starts empty (and ends drained)
      ctx->factory->wait_idle();
      for (unsigned q = s >= depth ? s - depth : 0; q != s; ++q) {
        collect(q % depth);
      }
      t0 = std::chrono::steady_clock::now();
    } else if (s >= depth) {
      collect(b); // the notifications of step s - depth
    }
    timed[b]                         = s >= warmup;
    const pusch_processor::pdu_t pdu = to_pdu(pc);
    for (unsigned i = 0; i != nof_cells; ++i) {
      ticket& t = tickets[static_cast<size_t>(b) * nof_cells + i];
      t.done.store(false);
      procs[i]->process(span<uint8_t>(tbs + static_cast<size_t>(i) * tb_bytes, tb_bytes), unique_rx_buffer(), t,
                        static_cast<any_grid*>(grids[static_cast<size_t>(b) * nof_cells + i])->rd(), pdu);
    }
    ctx->factory->flush();
    if (depth == 1) {
      ctx->factory->wait_idle();
    }
  }
  ctx->factory->wait_idle();
  const unsigned end = warmup + steps;
  for (unsigned q = std::max(warmup, end >= depth ? end - depth : 0u); q < end; ++q) {
    collect(q % depth);
  }
  const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  *ok_out         = ok;
  return steps ? dt / steps : 0.0;
}

/* ---- PDSCH: the reference's pdsch_processor_impl and the MI355X plug-in on writer-backed grids ---- */

void* srs_ref_phy_wgrid_create(const uint32_t* grid, unsigned nports, unsigned nsubc)
{
  return new host_wgrid(grid, nports, nsubc);
}

void srs_ref_phy_wgrid_destroy(void* g)
{
  delete static_cast<any_grid*>(g);
}

/* A device-resident grid (hip_resource_grid over resource_grid_impl) of nports x 14 x nsubc on HIP device `device`;
 * grid (optional) written through its host writer (the device copy is then stale until a plug-in uses it). */
void* srs_ref_phy_hgrid_create(const uint32_t* grid, unsigned nports, unsigned nsubc, int device)
{
  auto* g = new dev_grid(nports, nsubc, device);
  // (an all-zero grid is what the new grid holds already: no host write, so the grid has no writable view out)
  const size_t n = static_cast<size_t>(nports) * MAX_NSYMB_PER_SLOT * nsubc;
  if (grid != nullptr && std::any_of(grid, grid + n, [](uint32_t v) { return v != 0; })) {
    resource_grid_writer& w = g->grid.get_writer();
    for (unsigned p = 0; p != nports; ++p) {
      for (unsigned l = 0; l != MAX_NSYMB_PER_SLOT; ++l) {
        std::memcpy(w.get_view(p, l).data(), grid + (p * MAX_NSYMB_PER_SLOT + l) * nsubc, nsubc * sizeof(uint32_t));
      }
    }
  }
  return static_cast<any_grid*>(g);
}

/* Writes the grid's DEVICE copy from host memory, as a device producer would (the OFDM demodulator plug-in): the host
 * mirror is stale afterwards. */
int srs_ref_phy_hgrid_set_device(void* h, const uint32_t* grid)
{
  auto*       g = dynamic_cast<dev_grid*>(static_cast<any_grid*>(h));
  hipStream_t s = nullptr;
  if (g == nullptr || hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) {
    return -1;
  }
  uint32_t*    d     = g->grid.device_write(s);
  const size_t bytes = sizeof(uint32_t) * g->grid.nof_ports() * g->grid.nof_symbols() * g->grid.nof_subc();
  hipError_t   e     = hipMemcpyAsync(d, grid, bytes, hipMemcpyHostToDevice, s);
  g->grid.device_written(s);
  e = e == hipSuccess ? hipStreamSynchronize(s) : e;
  (void)hipStreamDestroy(s);
  return e == hipSuccess ? 0 : -1;
}

/* The grid's contents through its host reader (downloads when the device copy is newer), uint32 [ports][14][nsubc];
 * out_transfers[2] (optional): downloads, uploads so far. */
void srs_ref_phy_hgrid_read(void* h, uint32_t* out, uint64_t* out_transfers)
{
  auto*                       g = dynamic_cast<dev_grid*>(static_cast<any_grid*>(h));
  const resource_grid_reader& r = g->grid.get_reader();
  for (unsigned p = 0; p != g->grid.nof_ports(); ++p) {
    for (unsigned l = 0; l != g->grid.nof_symbols(); ++l) {
      span<const cbf16_t> v = r.get_view(p, l);
      std::memcpy(out + (p * g->grid.nof_symbols() + l) * g->grid.nof_subc(), v.data(), v.size() * sizeof(uint32_t));
    }
  }
  if (out_transfers != nullptr) {
    out_transfers[0] = g->grid.nof_downloads();
    out_transfers[1] = g->grid.nof_uploads();
  }
}

/* Transfers of a device-resident grid so far: [0] downloads, [1] uploads. */
void srs_ref_phy_hgrid_transfers(void* h, uint64_t* out)
{
  auto* g = dynamic_cast<dev_grid*>(static_cast<any_grid*>(h));
  out[0]  = g->grid.nof_downloads();
  out[1]  = g->grid.nof_uploads();
}

/* The grid's contents, uint32 [ports][14][nsubc]. */
void srs_ref_phy_wgrid_read(void* g, uint32_t* out)
{
  static_cast<host_wgrid*>(g)->load(out);
}

/* pdsch_processor_impl::process (pdsch_processor_impl.cpp:42-82) of one PDU into the grid. */
int srs_ref_pdsch_process(void* g, const srs_ref_pdsch_pdu* c, const uint8_t* tb, unsigned tb_bytes)
{
  static thread_local std::unique_ptr<pdsch_processor_impl> proc = make_ref_pdsch_processor();
  pdsch_ticket                                                 t;
  static_vector<shared_transport_block, pdsch_processor::MAX_NOF_TRANSPORT_BLOCKS> data;
  data.emplace_back(span<const uint8_t>(tb, tb_bytes));
  proc->process(static_cast<any_grid*>(g)->wr(), t, std::move(data), to_pdsch_pdu(*c));
  return t.done ? 0 : -1;
}

void* srs_ref_phy_pdsch_create(int device, unsigned nof_prb, unsigned max_wait_us)
{
  hip::pdsch_processor_hip_config cfg;
  cfg.device      = device;
  cfg.nof_prb     = nof_prb;
  cfg.max_wait_us = max_wait_us;
  auto f          = hip::create_pdsch_processor_factory_hip(cfg);
  if (!f) {
    return nullptr;
  }
  auto* ctx    = new pdsch_ctx;
  ctx->factory = f;
  ctx->proc    = f->create();
  return ctx;
}

void srs_ref_phy_pdsch_destroy(void* h)
{
  auto* ctx = static_cast<pdsch_ctx*>(h);
  ctx->factory->wait_idle();
  delete ctx;
}

/* pdsch_processor::process of the plug-in (asynchronous); the transport block is copied (the harness keeps it
 * alive until the context goes).  Returns the ticket. */
int srs_ref_phy_pdsch_process(void* h, void* g, const srs_ref_pdsch_pdu* c, const uint8_t* tb, unsigned tb_bytes)
{
  auto*                 ctx = static_cast<pdsch_ctx*>(h);
  pdsch_ticket*         t;
  std::vector<uint8_t>* b;
  int                   id;
  {
    std::lock_guard<std::mutex> lock(ctx->mtx);
    id = static_cast<int>(ctx->tickets.size());
    t  = &ctx->tickets.emplace_back();
    b  = &ctx->tbs.emplace_back(tb, tb + tb_bytes);
  }
  static_vector<shared_transport_block, pdsch_processor::MAX_NOF_TRANSPORT_BLOCKS> data;
  data.emplace_back(span<const uint8_t>(b->data(), b->size()));
  ctx->proc->process(static_cast<any_grid*>(g)->wr(), *t, std::move(data), to_pdsch_pdu(*c));
  return id;
}

void srs_ref_phy_pdsch_flush(void* h)
{
  static_cast<pdsch_ctx*>(h)->factory->flush();
}

void srs_ref_phy_pdsch_wait(void* h)
{
  static_cast<pdsch_ctx*>(h)->factory->wait_idle();
}

int srs_ref_phy_pdsch_done(void* h, int id)
{
  auto*                       ctx = static_cast<pdsch_ctx*>(h);
  std::lock_guard<std::mutex> lock(ctx->mtx);
  return (id >= 0 && static_cast<size_t>(id) < ctx->tickets.size() && ctx->tickets[id].done.load()) ? 1 : 0;
}

void srs_ref_phy_pdsch_stats(void* h, uint64_t* out)
{
  const auto s = static_cast<pdsch_ctx*>(h)->factory->get_statistics();
  out[0]       = s.nof_pdus;
  out[1]       = s.nof_batches;
  out[2]       = s.nof_errors;
  out[3]       = s.nof_device_grids;
}

/* Throughput through the PDSCH plug-in: every step one PDU per cell grid (a processor per cell), process() per PDU,
 * flush(), wait.  Returns seconds per step. */
double srs_ref_phy_pdsch_bench(void* h, void* const* grids, unsigned nof_cells, unsigned depth,
                               const srs_ref_pdsch_pdu* c, const uint8_t* tb, unsigned tb_bytes, unsigned warmup,
                               unsigned steps)
{
  auto*                                         ctx = static_cast<pdsch_ctx*>(h);
  std::vector<std::unique_ptr<pdsch_processor>> procs;
  for (unsigned i = 0; i != nof_cells; ++i) {
    procs.push_back(ctx->factory->create());
  }
  depth = std::max(depth, 1u);
  std::vector<pdsch_ticket>    tickets(static_cast<size_t>(nof_cells) * depth);
  const pdsch_processor::pdu_t pdu     = to_pdsch_pdu(*c);
  auto                         collect = [&](unsigned b) {
    for (unsigned i = 0; i != nof_cells; ++i) {
      while (!tickets[static_cast<size_t>(b) * nof_cells + i].done.load(std::memory_order_acquire)) {
        std::this_thread::sleep_for(std::chrono::microseconds(20));
      }
    }
  };
  auto t0 = std::chrono::steady_clock::now();
  for (unsigned s = 0; s != warmup + steps; ++s) {
    const unsigned b = s % depth;
    if (s == warmup) {
      ctx->factory->wait_idle(); // (the timed region starts empty and ends drained, as the PUSCH bench)
      t0 = std::chrono::steady_clock::now();
    } else if (s >= depth) {
      collect(b); // step s - depth's grids are written: the set is free again
    }
    for (unsigned i = 0; i != nof_cells; ++i) {
      static_vector<shared_transport_block, pdsch_processor::MAX_NOF_TRANSPORT_BLOCKS> data;
      data.emplace_back(span<const uint8_t>(tb, tb_bytes));
      pdsch_ticket& t = tickets[static_cast<size_t>(b) * nof_cells + i];
      t.done.store(false);
      procs[i]->process(static_cast<any_grid*>(grids[static_cast<size_t>(b) * nof_cells + i])->wr(), t,
                        std::move(data), pdu);
    }
    ctx->factory->flush();
    if (depth == 1) {
      ctx->factory->wait_idle();
    }
  }
  ctx->factory->wait_idle();
  const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  return steps ? dt / steps : 0.0;
}

} // extern "C"

/* ---- PDCCH: the MI355X plug-in (integration/pdcch_processor_hip) driven through the reference interface ---- */

namespace {
struct pdcch_ctx {
  std::shared_ptr<hip::pdcch_processor_factory_hip> factory;
  std::unique_ptr<pdcch_processor>                  proc;
  std::unique_ptr<pdcch_pdu_validator>              validator;
};
} // namespace

extern "C" {

void* srs_ref_phy_pdcch_create(int device)
{
  hip::pdcch_processor_hip_config cfg;
  cfg.device = device;
  auto ctx   = std::make_unique<pdcch_ctx>();
  ctx->factory = hip::create_pdcch_processor_factory_hip(cfg);
  if (!ctx->factory) {
    return nullptr;
  }
  ctx->proc      = ctx->factory->create();
  ctx->validator = ctx->factory->create_validator();
  return ctx.release();
}

void srs_ref_phy_pdcch_destroy(void* h)
{
  delete static_cast<pdcch_ctx*>(h);
}

/* pdcch_processor::process of each PDU, in order, into grid g (a host writer grid or a device-resident grid). */
void srs_ref_phy_pdcch_process(void* h, void* g, const srs_amd_pdcch_pdu* pdus, unsigned n)
{
  auto* ctx = static_cast<pdcch_ctx*>(h);
  for (unsigned i = 0; i != n; ++i) {
    ctx->proc->process(static_cast<any_grid*>(g)->wr(), srs_ref::pdcch_pdu_from_amd(pdus[i]));
  }
}

/* The plug-in factory's validator: 1 valid, 0 invalid (msg filled). */
int srs_ref_phy_pdcch_validate(void* h, const srs_amd_pdcch_pdu* pdu, char* msg, unsigned msg_size)
{
  error_type<std::string> r = static_cast<pdcch_ctx*>(h)->validator->is_valid(srs_ref::pdcch_pdu_from_amd(*pdu));
  if (r.has_value()) {
    return 1;
  }
  std::snprintf(msg, msg_size, "%s", r.error().c_str());
  return 0;
}

/* [0] PDUs, [1] errors, [2] device-resident grids. */
void srs_ref_phy_pdcch_stats(void* h, uint64_t* out)
{
  const auto s = static_cast<pdcch_ctx*>(h)->factory->get_statistics();
  out[0]       = s.nof_pdus;
  out[1]       = s.nof_errors;
  out[2]       = s.nof_device_grids;
}

} // extern "C"

/* ---- SSB: the MI355X plug-in (integration/ssb_processor_hip) driven through the reference interface ---- */

namespace {
struct ssb_ctx {
  std::shared_ptr<hip::ssb_processor_factory_hip> factory;
  std::unique_ptr<ssb_processor>                  proc;
  std::unique_ptr<ssb_pdu_validator>              validator;
};
} // namespace

extern "C" {

void* srs_ref_phy_ssb_create(int device)
{
  hip::ssb_processor_hip_config cfg;
  cfg.device   = device;
  auto ctx     = std::make_unique<ssb_ctx>();
  ctx->factory = hip::create_ssb_processor_factory_hip(cfg);
  if (!ctx->factory) {
    return nullptr;
  }
  ctx->proc      = ctx->factory->create();
  ctx->validator = ctx->factory->create_validator();
  return ctx.release();
}

void srs_ref_phy_ssb_destroy(void* h)
{
  delete static_cast<ssb_ctx*>(h);
}

/* ssb_processor::process of each PDU, in order, into grid g (a host writer grid or a device-resident grid). */
void srs_ref_phy_ssb_process(void* h, void* g, const srs_amd_ssb_pdu* pdus, unsigned n)
{
  auto* ctx = static_cast<ssb_ctx*>(h);
  for (unsigned i = 0; i != n; ++i) {
    ctx->proc->process(static_cast<any_grid*>(g)->wr(), srs_ref::ssb_pdu_from_amd(pdus[i]));
  }
}

/* The plug-in factory's validator: 1 valid, 0 invalid (msg filled). */
int srs_ref_phy_ssb_validate(void* h, const srs_amd_ssb_pdu* pdu, char* msg, unsigned msg_size)
{
  error_type<std::string> r = static_cast<ssb_ctx*>(h)->validator->is_valid(srs_ref::ssb_pdu_from_amd(*pdu));
  if (r.has_value()) {
    return 1;
  }
  std::snprintf(msg, msg_size, "%s", r.error().c_str());
  return 0;
}

/* [0] PDUs, [1] errors, [2] device-resident grids. */
void srs_ref_phy_ssb_stats(void* h, uint64_t* out)
{
  const auto s = static_cast<ssb_ctx*>(h)->factory->get_statistics();
  out[0]       = s.nof_pdus;
  out[1]       = s.nof_errors;
  out[2]       = s.nof_device_grids;
}

/* ---- PUCCH: the MI355X plug-in (integration/pucch_processor_hip) driven through the reference interface ---- */
struct pucch_ctx {
  std::shared_ptr<hip::pucch_processor_factory_hip> factory;
  std::unique_ptr<pucch_processor>                  proc;
  std::unique_ptr<pucch_pdu_validator>              validator;
};

void* srs_ref_phy_pucch_create(int device)
{
  hip::pucch_processor_hip_config cfg;
  cfg.device   = device;
  auto ctx     = std::make_unique<pucch_ctx>();
  ctx->factory = hip::create_pucch_processor_factory_hip(cfg);
  if (!ctx->factory) {
    return nullptr;
  }
  ctx->proc      = ctx->factory->create();
  ctx->validator = ctx->factory->create_validator();
  return ctx->proc ? ctx.release() : nullptr;
}

void srs_ref_phy_pucch_destroy(void* h)
{
  delete static_cast<pucch_ctx*>(h);
}

static void csi_out(const channel_state_information& csi, float* sinr, float* rsrp, float* epre)
{
  *sinr = csi.get_sinr_dB().value_or(NAN);
  *rsrp = csi.get_rsrp_dB().value_or(NAN);
  *epre = csi.get_epre_dB().value_or(NAN);
}

/* pucch_processor::process(format0_configuration) of a C-ABI Format 0 PDU (BWP from PRB 0 over the grid). */
void srs_ref_phy_pucch_f0(void* h, void* g, const srs_amd_pucch_f0_pdu* p, unsigned grid_prb,
                          srs_amd_pucch_result* out)
{
  pucch_processor::format0_configuration c;
  c.slot         = slot_point(p->numerology, p->slot_index);
  c.cp           = cyclic_prefix::NORMAL;
  c.bwp_size_rb  = grid_prb;
  c.bwp_start_rb = 0;
  c.starting_prb = p->starting_prb;
  if (p->second_hop_prb >= 0) {
    c.second_hop_prb = static_cast<unsigned>(p->second_hop_prb);
  }
  c.start_symbol_index   = p->start_symbol_index;
  c.nof_symbols          = p->nof_symbols;
  c.initial_cyclic_shift = p->initial_cyclic_shift;
  c.n_id                 = p->n_id;
  c.nof_harq_ack         = p->nof_harq_ack;
  c.sr_opportunity       = p->sr_opportunity != 0;
  for (unsigned i = 0; i != p->nof_ports; ++i) {
    c.ports.push_back(p->ports[i]);
  }
  const pucch_processor_result r = static_cast<pucch_ctx*>(h)->proc->process(static_cast<any_grid*>(g)->rd(), c);
  std::memset(out, 0, sizeof(*out));
  out->status       = static_cast<uint32_t>(r.message.get_status());
  out->nof_sr       = r.message.get_sr_bits().size();
  out->nof_harq_ack = r.message.get_harq_ack_bits().size();
  if (out->nof_sr != 0) {
    out->sr = r.message.get_sr_bits()[0];
  }
  for (unsigned i = 0; i != out->nof_harq_ack && i != 2; ++i) {
    out->harq_ack[i] = r.message.get_harq_ack_bits()[i];
  }
  csi_out(r.csi, &out->sinr_dB, &out->rsrp_dB, &out->epre_dB);
  out->detection_metric = std::pow(10.0F, out->sinr_dB / 10.0F);
}

/* pucch_processor::process(format1_batch_configuration) of a C-ABI batch (BWP from PRB 0 over the grid); out[e] for
 * entry e. */
void srs_ref_phy_pucch_f1(void* h, void* g, const srs_amd_pucch_f1_batch* b, unsigned grid_prb,
                          srs_amd_pucch_result* out)
{
  pucch_processor::format1_batch_configuration c;
  c.common_config.slot         = slot_point(b->numerology, b->slot_index);
  c.common_config.bwp_size_rb  = grid_prb;
  c.common_config.bwp_start_rb = 0;
  c.common_config.cp           = cyclic_prefix::NORMAL;
  c.common_config.starting_prb = b->starting_prb;
  if (b->second_hop_prb >= 0) {
    c.common_config.second_hop_prb = static_cast<unsigned>(b->second_hop_prb);
  }
  c.common_config.n_id = b->n_id;
  for (unsigned i = 0; i != b->nof_ports; ++i) {
    c.common_config.ports.push_back(b->ports[i]);
  }
  c.common_config.nof_symbols        = b->nof_symbols;
  c.common_config.start_symbol_index = b->start_symbol_index;
  for (unsigned e = 0; e != b->nof_entries; ++e) {
    c.entries.insert(b->entries[e].initial_cyclic_shift,
                     b->entries[e].time_domain_occ,
                     {.context = std::nullopt, .nof_harq_ack = b->entries[e].nof_harq_ack});
  }
  const auto res = static_cast<pucch_ctx*>(h)->proc->process(static_cast<any_grid*>(g)->rd(), c);
  for (unsigned e = 0; e != b->nof_entries; ++e) {
    const pucch_processor_result& r = res.get(b->entries[e].initial_cyclic_shift, b->entries[e].time_domain_occ);
    std::memset(&out[e], 0, sizeof(out[e]));
    out[e].status       = static_cast<uint32_t>(r.message.get_status());
    out[e].nof_harq_ack = r.message.get_harq_ack_bits().size();
    for (unsigned i = 0; i != out[e].nof_harq_ack && i != 2; ++i) {
      out[e].harq_ack[i] = r.message.get_harq_ack_bits()[i];
    }
    csi_out(r.csi, &out[e].sinr_dB, &out[e].rsrp_dB, &out[e].epre_dB);
    out[e].detection_metric = r.detection_metric.value_or(NAN);
  }
}

/* pucch_processor::process(format2_configuration) of a C-ABI Format 2 PDU; payload[nof bits]. */
void srs_ref_phy_pucch_f2(void* h, void* g, const srs_amd_pucch_f2_pdu* p, srs_amd_pucch_uci_result* out,
                          uint8_t* payload)
{
  pucch_processor::format2_configuration c;
  c.slot         = slot_point(p->numerology, p->slot_index);
  c.bwp_size_rb  = p->bwp_size_rb;
  c.bwp_start_rb = p->bwp_start_rb;
  c.cp           = cyclic_prefix::NORMAL;
  c.starting_prb = p->starting_prb;
  if (p->second_hop_prb >= 0) {
    c.second_hop_prb = static_cast<unsigned>(p->second_hop_prb);
  }
  c.nof_prb            = p->nof_prb;
  c.start_symbol_index = p->start_symbol_index;
  c.nof_symbols        = p->nof_symbols;
  c.rnti               = static_cast<uint16_t>(p->rnti);
  c.n_id               = p->n_id;
  c.n_id_0             = p->n_id_0;
  c.nof_harq_ack       = p->nof_harq_ack;
  c.nof_sr             = p->nof_sr;
  c.nof_csi_part1      = p->nof_csi_part1;
  c.nof_csi_part2      = p->nof_csi_part2;
  for (unsigned i = 0; i != p->nof_ports; ++i) {
    c.ports.push_back(p->ports[i]);
  }
  const pucch_processor_result r = static_cast<pucch_ctx*>(h)->proc->process(static_cast<any_grid*>(g)->rd(), c);
  std::memset(out, 0, sizeof(*out));
  out->status        = static_cast<uint32_t>(r.message.get_status());
  out->nof_harq_ack  = r.message.get_harq_ack_bits().size();
  out->nof_sr        = r.message.get_sr_bits().size();
  out->nof_csi_part1 = r.message.get_csi_part1_bits().size();
  out->nof_csi_part2 = r.message.get_csi_part2_bits().size();
  const auto full    = r.message.get_full_payload();
  std::memcpy(payload, full.data(), full.size());
  csi_out(r.csi, &out->sinr_dB, &out->rsrp_dB, &out->epre_dB);
  out->time_alignment_s = r.csi.get_time_alignment().has_value() ? r.csi.get_time_alignment()->to_seconds() : NAN;
  out->cfo_Hz           = r.csi.get_cfo_Hz().value_or(NAN);
}

/* pucch_processor::process(format3 / format4_configuration) of a C-ABI Format 3 / 4 PDU; payload[nof bits]. */
void srs_ref_phy_pucch_f34(void* h, void* g, const srs_amd_pucch_f34_pdu* p, srs_amd_pucch_uci_result* out,
                           uint8_t* payload)
{
  auto fill = [p](auto& c) {
    c.slot = slot_point(p->numerology, p->slot_index);
    c.cp   = cyclic_prefix::NORMAL;
    for (unsigned i = 0; i != p->nof_ports; ++i) {
      c.ports.push_back(p->ports[i]);
    }
    c.bwp_size_rb  = p->bwp_size_rb;
    c.bwp_start_rb = p->bwp_start_rb;
    c.starting_prb = p->starting_prb;
    if (p->second_hop_prb >= 0) {
      c.second_hop_prb = static_cast<unsigned>(p->second_hop_prb);
    }
    c.start_symbol_index = p->start_symbol_index;
    c.nof_symbols        = p->nof_symbols;
    c.rnti               = static_cast<uint16_t>(p->rnti);
    c.n_id_hopping       = p->n_id_hopping;
    c.n_id_scrambling    = p->n_id_scrambling;
    c.nof_harq_ack       = p->nof_harq_ack;
    c.nof_sr             = p->nof_sr;
    c.nof_csi_part1      = p->nof_csi_part1;
    c.nof_csi_part2      = p->nof_csi_part2;
    c.additional_dmrs    = p->additional_dmrs != 0;
    c.pi2_bpsk           = p->pi2_bpsk != 0;
  };
  auto*                  ctx = static_cast<pucch_ctx*>(h);
  pucch_processor_result r;
  if (p->format == 4) {
    pucch_processor::format4_configuration c;
    fill(c);
    c.occ_index  = p->occ_index;
    c.occ_length = p->occ_length;
    r            = ctx->proc->process(static_cast<any_grid*>(g)->rd(), c);
  } else {
    pucch_processor::format3_configuration c;
    fill(c);
    c.nof_prb = p->nof_prb;
    r         = ctx->proc->process(static_cast<any_grid*>(g)->rd(), c);
  }
  std::memset(out, 0, sizeof(*out));
  out->status        = static_cast<uint32_t>(r.message.get_status());
  out->nof_harq_ack  = r.message.get_harq_ack_bits().size();
  out->nof_sr        = r.message.get_sr_bits().size();
  out->nof_csi_part1 = r.message.get_csi_part1_bits().size();
  out->nof_csi_part2 = r.message.get_csi_part2_bits().size();
  const auto full    = r.message.get_full_payload();
  std::memcpy(payload, full.data(), full.size());
  csi_out(r.csi, &out->sinr_dB, &out->rsrp_dB, &out->epre_dB);
  out->time_alignment_s = r.csi.get_time_alignment().has_value() ? r.csi.get_time_alignment()->to_seconds() : NAN;
  out->cfo_Hz           = r.csi.get_cfo_Hz().value_or(NAN);
}

/* Seconds for reps calls of pucch_processor::process on one Format 0 PDU / Format 2 PDU (grid g), for the plug-in's
 * per-call latency (the reference interface returns each result synchronously). */
double srs_ref_phy_pucch_latency(void* h, void* g, const srs_amd_pucch_f0_pdu* p0, const srs_amd_pucch_f2_pdu* p2,
                                 unsigned grid_prb, unsigned reps)
{
  srs_amd_pucch_result     r0;
  srs_amd_pucch_uci_result r2;
  uint8_t                  pay[1706];
  const auto               t0 = std::chrono::steady_clock::now();
  for (unsigned i = 0; i != reps; ++i) {
    if (p0 != nullptr) {
      srs_ref_phy_pucch_f0(h, g, p0, grid_prb, &r0);
    } else {
      srs_ref_phy_pucch_f2(h, g, p2, &r2, pay);
    }
  }
  return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
}

/* The plug-in factory's validator on a Format 2 PDU: 1 valid, 0 invalid (msg filled). */
int srs_ref_phy_pucch_f2_validate(void* h, const srs_amd_pucch_f2_pdu* p, char* msg, unsigned msg_size)
{
  pucch_processor::format2_configuration c;
  c.slot         = slot_point(p->numerology, p->slot_index);
  c.bwp_size_rb  = p->bwp_size_rb;
  c.bwp_start_rb = p->bwp_start_rb;
  c.starting_prb = p->starting_prb;
  c.nof_prb      = p->nof_prb;
  c.start_symbol_index = p->start_symbol_index;
  c.nof_symbols        = p->nof_symbols;
  c.nof_harq_ack       = p->nof_harq_ack;
  c.nof_sr             = p->nof_sr;
  c.nof_csi_part1      = p->nof_csi_part1;
  c.nof_csi_part2      = p->nof_csi_part2;
  for (unsigned i = 0; i != p->nof_ports; ++i) {
    c.ports.push_back(p->ports[i]);
  }
  error_type<std::string> r = static_cast<pucch_ctx*>(h)->validator->is_valid(c);
  if (r.has_value()) {
    return 1;
  }
  std::snprintf(msg, msg_size, "%s", r.error().c_str());
  return 0;
}

/* [0] PDUs, [1] errors, [2] device-resident grids, [3] rendezvous batches, [4] / [5] the batches' host / wait us. */
void srs_ref_phy_pucch_stats(void* h, uint64_t* out)
{
  const auto s = static_cast<pucch_ctx*>(h)->factory->get_statistics();
  out[0]       = s.nof_pdus;
  out[1]       = s.nof_errors;
  out[2]       = s.nof_device_grids;
  out[3]       = s.nof_batches;
  out[4]       = s.batch_host_us;
  out[5]       = s.batch_wait_us;
}

/* The PUCCHs of `ncells` cells through the plug-in as the reference's uplink processor drives them: every PDU of a
 * cell's slot (the same lists for every cell, grid g[c]) one synchronous pucch_processor::process call each, spread
 * over `threads` PUCCH-executor threads (each with its own processor of the factory: uplink_processor_impl posts one
 * task per PDU), `reps` times.  Returns the wall seconds.  Outputs of the first rep (optional, per cell in list
 * order): r0[ncells][n0], r1[ncells][sum of entries], r2 / r34 [ncells][n] with payloads p2 / p34 [..][64]. */
double srs_ref_phy_pucch_mt_bench(void* h, void* const* grids, unsigned ncells, const srs_amd_pucch_f0_pdu* f0,
                                  unsigned n0, const srs_amd_pucch_f1_batch* f1, unsigned n1,
                                  const srs_amd_pucch_f2_pdu* f2, unsigned n2, const srs_amd_pucch_f34_pdu* f34,
                                  unsigned n34, unsigned threads, unsigned reps, unsigned grid_prb,
                                  srs_amd_pucch_result* r0, srs_amd_pucch_result* r1, srs_amd_pucch_uci_result* r2,
                                  uint8_t* p2, srs_amd_pucch_uci_result* r34, uint8_t* p34)
{
  auto* base = static_cast<pucch_ctx*>(h);
  std::vector<std::unique_ptr<pucch_ctx>> ctxs;
  for (unsigned t = 0; t != threads; ++t) {
    auto c     = std::make_unique<pucch_ctx>();
    c->factory = base->factory;
    c->proc    = base->factory->create();
    if (!c->proc) {
      return -1;
    }
    ctxs.push_back(std::move(c));
  }
  unsigned ne = 0;
  std::vector<unsigned> e0(n1);
  for (unsigned i = 0; i != n1; ++i) {
    e0[i] = ne;
    ne += f1[i].nof_entries;
  }
  const unsigned per_cell = n0 + n1 + n2 + n34;
  const unsigned items    = per_cell * ncells;
  std::atomic<unsigned> arrived{0};
  auto worker = [&](unsigned t) {
    srs_amd_pucch_result              x0;
    std::vector<srs_amd_pucch_result> x1(std::max(ne, 1u));
    srs_amd_pucch_uci_result xu;
    uint8_t                  pay[1706];
    arrived.fetch_add(1);
    while (arrived.load() != threads + 1) {
    }
    for (unsigned r = 0; r != reps; ++r) {
      for (unsigned it = t; it < items; it += threads) {
        const unsigned c = it / per_cell, k = it % per_cell;
        void*          g = grids[c];
        const bool     keep = r == 0;
        if (k < n0) {
          srs_ref_phy_pucch_f0(ctxs[t].get(), g, &f0[k], grid_prb, keep && r0 ? &r0[c * n0 + k] : &x0);
        } else if (k < n0 + n1) {
          const unsigned b = k - n0;
          srs_ref_phy_pucch_f1(ctxs[t].get(), g, &f1[b], grid_prb, keep && r1 ? &r1[c * ne + e0[b]] : x1.data());
        } else if (k < n0 + n1 + n2) {
          const unsigned i = k - n0 - n1;
          std::memset(pay, 0, 64); // (bits past the PDU's payload are not written)
          srs_ref_phy_pucch_f2(ctxs[t].get(), g, &f2[i], keep && r2 ? &r2[c * n2 + i] : &xu, pay);
          if (keep && p2) {
            std::memcpy(p2 + (static_cast<size_t>(c) * n2 + i) * 64, pay, 64);
          }
        } else {
          const unsigned i = k - n0 - n1 - n2;
          std::memset(pay, 0, 64);
          srs_ref_phy_pucch_f34(ctxs[t].get(), g, &f34[i], keep && r34 ? &r34[c * n34 + i] : &xu, pay);
          if (keep && p34) {
            std::memcpy(p34 + (static_cast<size_t>(c) * n34 + i) * 64, pay, 64);
          }
        }
      }
    }
  };
  std::vector<std::thread> pool;
  for (unsigned t = 0; t != threads; ++t) {
    pool.emplace_back(worker, t);
  }
  while (arrived.load() != threads) {
  }
  const auto t0 = std::chrono::steady_clock::now();
  arrived.fetch_add(1);
  for (auto& th : pool) {
    th.join();
  }
  return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
}

} // extern "C"

/* ---- OFDM: the demodulator plug-ins writing a device-resident grid, as the lower PHY drives them ---- */

#include "../integration/ofdm_modulator_hip.h"

namespace {

ofdm_demodulator_configuration ul_dem_cfg(unsigned mu, unsigned bw_rb, unsigned dft_size, double fc, float scale = 1.0f)
{
  ofdm_demodulator_configuration c;
  c.numerology                = mu;
  c.bw_rb                     = bw_rb;
  c.dft_size                  = dft_size;
  c.cp                        = cyclic_prefix::NORMAL;
  c.nof_samples_window_offset = 0;
  c.scale                     = scale;
  c.center_freq_Hz            = fc;
  return c;
}

// Sample offsets of the symbols of slot `slot` within the slot (per port), and the slot size.
std::vector<unsigned> symbol_offsets(const ofdm_symbol_demodulator& d, unsigned slot, unsigned& slot_size)
{
  std::vector<unsigned> off(MAX_NSYMB_PER_SLOT);
  slot_size = 0;
  for (unsigned l = 0; l != MAX_NSYMB_PER_SLOT; ++l) {
    off[l] = slot_size;
    slot_size += d.get_symbol_size(MAX_NSYMB_PER_SLOT * slot + l);
  }
  return off;
}

ofdm_modulator_configuration dl_mod_cfg(unsigned mu, unsigned bw_rb, unsigned dft_size, double fc, float scale)
{
  ofdm_modulator_configuration c;
  c.numerology     = mu;
  c.bw_rb          = bw_rb;
  c.dft_size       = dft_size;
  c.cp             = cyclic_prefix::NORMAL;
  c.scale          = scale;
  c.center_freq_Hz = fc;
  return c;
}

} // namespace

extern "C" {

/* The downlink step pdxch_processor_impl runs per OFDM symbol: every port of every symbol of slot `slot` (of the
 * subframe) of `grid` modulated through the MI355X OFDM modulator plug-in (form 1 ofdm_symbol_modulator, symbol by
 * symbol and port by port; form 0 ofdm_slot_modulator, port by port) into out [port][slot size] complex floats.
 * 0 on success, -1 when the factory refuses the configuration. */
int srs_ref_phy_ofdm_modulate(void* grid, int device, int form, unsigned mu, unsigned bw_rb, unsigned dft_size,
                              double fc, float scale, unsigned slot, unsigned nports, float* out)
{
  auto                        f = hip::create_ofdm_modulator_factory_hip(device);
  const auto                  c = dl_mod_cfg(mu, bw_rb, dft_size, fc, scale);
  const resource_grid_reader& r = static_cast<any_grid*>(grid)->rd();
  cf_t*                       y = reinterpret_cast<cf_t*>(out);
  if (form == 0) {
    auto m = f->create_ofdm_slot_modulator(c);
    if (!m) {
      return -1;
    }
    const unsigned n = m->get_slot_size(slot);
    for (unsigned p = 0; p != nports; ++p) {
      m->modulate(span<cf_t>(y + static_cast<size_t>(p) * n, n), r, p, slot);
    }
    return 0;
  }
  auto m = f->create_ofdm_symbol_modulator(c);
  if (!m) {
    return -1;
  }
  unsigned n = 0;
  for (unsigned l = 0; l != MAX_NSYMB_PER_SLOT; ++l) {
    n += m->get_symbol_size(MAX_NSYMB_PER_SLOT * slot + l);
  }
  for (unsigned l = 0, off = 0; l != MAX_NSYMB_PER_SLOT; ++l) {
    const unsigned sz = m->get_symbol_size(MAX_NSYMB_PER_SLOT * slot + l);
    for (unsigned p = 0; p != nports; ++p) {
      m->modulate(span<cf_t>(y + static_cast<size_t>(p) * n + off, sz), r, p, MAX_NSYMB_PER_SLOT * slot + l);
    }
    off += sz;
  }
  return 0;
}

/* One ofdm_symbol_modulator plug-in over two contents of the same grid: slot `slot` modulated (every port, symbol by
 * symbol) into out0, then the grid rewritten with `next` -- on the device (next_on_host = 0, as a device producer) or
 * through the host writer's put (1, as a reference processor) -- and modulated again by the SAME modulator into
 * out1.  Checks that the plug-in's per-slot sample cache follows the grid's content.  0 on success. */
int srs_ref_phy_ofdm_modulate_twice(void* grid, int device, unsigned mu, unsigned bw_rb, unsigned dft_size, double fc,
                                    float scale, unsigned slot, unsigned nports, const uint32_t* next,
                                    int next_on_host, float* out0, float* out1)
{
  auto m = hip::create_ofdm_modulator_factory_hip(device)->create_ofdm_symbol_modulator(
      dl_mod_cfg(mu, bw_rb, dft_size, fc, scale));
  auto* g = dynamic_cast<dev_grid*>(static_cast<any_grid*>(grid));
  if (!m || g == nullptr) {
    return -1;
  }
  unsigned n = 0;
  for (unsigned l = 0; l != MAX_NSYMB_PER_SLOT; ++l) {
    n += m->get_symbol_size(MAX_NSYMB_PER_SLOT * slot + l);
  }
  auto run = [&](float* out) {
    cf_t* y = reinterpret_cast<cf_t*>(out);
    for (unsigned l = 0, off = 0; l != MAX_NSYMB_PER_SLOT; ++l) {
      const unsigned sz = m->get_symbol_size(MAX_NSYMB_PER_SLOT * slot + l);
      for (unsigned p = 0; p != nports; ++p) {
        m->modulate(span<cf_t>(y + static_cast<size_t>(p) * n + off, sz), g->grid.get_reader(), p,
                    MAX_NSYMB_PER_SLOT * slot + l);
      }
      off += sz;
    }
  };
  run(out0);
  if (next_on_host) {
    resource_grid_writer& w     = g->grid.get_writer();
    const unsigned        nsubc = g->grid.nof_subc();
    for (unsigned p = 0; p != nports; ++p) {
      for (unsigned l = 0; l != MAX_NSYMB_PER_SLOT; ++l) {
        const auto* src = reinterpret_cast<const cbf16_t*>(next + (p * MAX_NSYMB_PER_SLOT + l) * nsubc);
        w.put(p, l, 0, 1, span<const cbf16_t>(src, nsubc));
      }
    }
  } else if (srs_ref_phy_hgrid_set_device(grid, next) != 0) {
    return -1;
  }
  run(out1);
  return 0;
}

/* The uplink step puxch_processor_impl runs per OFDM symbol (puxch_processor_impl.cpp:73-82): every port of every
 * symbol of slot `slot` (of the subframe) demodulated into `grid` through the MI355X OFDM demodulator plug-in, form 1
 * the ofdm_symbol_demodulator (symbol by symbol, port by port), form 0 the ofdm_slot_demodulator (port by port).
 * samples: [port][slot size] complex floats.  A device-resident grid (srs_ref_phy_hgrid_create) is written in place on
 * the device.  0 on success, -1 when the factory refuses the configuration. */
int srs_ref_phy_ofdm_demodulate(void* grid, int device, int form, unsigned mu, unsigned bw_rb, unsigned dft_size,
                                double fc, float scale, unsigned slot, unsigned nports, const float* samples)
{
  auto                  f = hip::create_ofdm_demodulator_factory_hip(device);
  const auto            c = ul_dem_cfg(mu, bw_rb, dft_size, fc, scale);
  resource_grid_writer& w = static_cast<any_grid*>(grid)->wr();
  const cf_t*           x = reinterpret_cast<const cf_t*>(samples);
  if (form == 0) {
    auto d = f->create_ofdm_slot_demodulator(c);
    if (!d) {
      return -1;
    }
    const unsigned n = d->get_slot_size(slot);
    for (unsigned p = 0; p != nports; ++p) {
      d->demodulate(w, span<const cf_t>(x + static_cast<size_t>(p) * n, n), p, slot);
    }
    return 0;
  }
  auto d = f->create_ofdm_symbol_demodulator(c);
  if (!d) {
    return -1;
  }
  unsigned                    n   = 0;
  const std::vector<unsigned> off = symbol_offsets(*d, slot, n);
  for (unsigned l = 0; l != MAX_NSYMB_PER_SLOT; ++l) {
    const unsigned sz = d->get_symbol_size(MAX_NSYMB_PER_SLOT * slot + l);
    for (unsigned p = 0; p != nports; ++p) {
      d->demodulate(w, span<const cf_t>(x + static_cast<size_t>(p) * n + off[l], sz), p, MAX_NSYMB_PER_SLOT * slot + l);
    }
  }
  return 0;
}

/* Symbol-form OFDM demodulation throughput as the lower PHY drives it: `threads` sectors, each with its own
 * ofdm_symbol_demodulator and its own slot grid, demodulating `slots` slots of `nports` ports symbol by symbol (slot
 * 0 of the subframe each time; samples: [port][slot size]).  plugin 1: the MI355X plug-in into a device-resident grid
 * (hip_resource_grid), each sector's grid then read on the device as the PUSCH plug-in reads it (device_read + stream
 * synchronise: the timed region ends when every kernel has completed); plugin 0: the reference's
 * ofdm_symbol_demodulator_impl over the generic DFT into a resource_grid_impl.  modulate = 1: the downlink twin,
 * ofdm_symbol_modulator per port and symbol (pdxch_processor_impl) of the finished grid grid0 [port][14][nsubc] --
 * on the device for the plug-in, rewritten on the device between slots as the PDSCH plug-in writes it (a new
 * content version every slot), on the host for the reference.  Returns the wall seconds from the start barrier to
 * the last sector done (-1: configuration refused); out[0] = mean host time per call (us), out[1] = grid transfers
 * (downloads + uploads, all sectors). */
double srs_ref_phy_ofdm_symbol_bench(int device, int plugin, int modulate, unsigned threads, unsigned mu,
                                     unsigned bw_rb, unsigned dft_size, unsigned nports, unsigned slots,
                                     const float* samples, const uint32_t* grid0, double* out)
{
  const unsigned nsubc = bw_rb * NRE;
  const auto     c     = ul_dem_cfg(mu, bw_rb, dft_size, 3.5e9);
  const auto     cm    = dl_mod_cfg(mu, bw_rb, dft_size, 3.5e9, 1.0f / 64);
  auto           f     = plugin && !modulate ? hip::create_ofdm_demodulator_factory_hip(device) : nullptr;
  auto           fm    = plugin && modulate ? hip::create_ofdm_modulator_factory_hip(device) : nullptr;
  std::vector<std::unique_ptr<ofdm_symbol_demodulator>> dems;
  std::vector<std::unique_ptr<ofdm_symbol_modulator>>   mods;
  std::vector<std::unique_ptr<dev_grid>>                dgrids;
  std::vector<std::unique_ptr<resource_grid_impl>>      hgrids;
  for (unsigned t = 0; t != threads; ++t) {
    if (modulate) {
      mods.push_back(plugin ? fm->create_ofdm_symbol_modulator(cm) : srs_ref::make_ref_ofdm_symbol_modulator(cm));
      if (!mods.back()) {
        return -1;
      }
    } else {
      dems.push_back(plugin ? f->create_ofdm_symbol_demodulator(c) : srs_ref::make_ref_ofdm_symbol_demodulator(c));
      if (!dems.back()) {
        return -1;
      }
    }
    if (plugin) {
      dgrids.push_back(std::make_unique<dev_grid>(nports, nsubc, device));
    } else {
      hgrids.push_back(std::make_unique<resource_grid_impl>(nports, MAX_NSYMB_PER_SLOT, nsubc));
    }
    if (modulate) {
      // the finished downlink grid: on the device for the plug-in (as the PDSCH plug-in leaves it), on the host for
      // the reference
      if (plugin) {
        if (srs_ref_phy_hgrid_set_device(static_cast<any_grid*>(dgrids.back().get()), grid0) != 0) {
          return -1;
        }
      } else {
        resource_grid_writer& w = hgrids.back()->get_writer();
        for (unsigned p = 0; p != nports; ++p) {
          for (unsigned l = 0; l != MAX_NSYMB_PER_SLOT; ++l) {
            std::memcpy(static_cast<void*>(w.get_view(p, l).data()), grid0 + (p * MAX_NSYMB_PER_SLOT + l) * nsubc,
                        nsubc * sizeof(uint32_t));
          }
        }
      }
    }
  }
  unsigned              n = 0;
  std::vector<unsigned> off(MAX_NSYMB_PER_SLOT), sz(MAX_NSYMB_PER_SLOT);
  for (unsigned l = 0; l != MAX_NSYMB_PER_SLOT; ++l) {
    sz[l]  = modulate ? mods[0]->get_symbol_size(l) : dems[0]->get_symbol_size(l);
    off[l] = n;
    n += sz[l];
  }
  const cf_t*                 x   = reinterpret_cast<const cf_t*>(samples);
  std::atomic<unsigned>       arrived{0};
  std::vector<double>         busy(threads, 0.0);
  std::vector<int>            fail(threads, 0);
  auto                        worker = [&](unsigned t) {
    (void)hipSetDevice(device < 0 ? 0 : device);
    resource_grid_writer&       w = plugin ? dgrids[t]->grid.get_writer() : hgrids[t]->get_writer();
    const resource_grid_reader& r = plugin ? dgrids[t]->grid.get_reader() : hgrids[t]->get_reader();
    std::vector<cf_t>           y(n);
    hipStream_t                 producer = nullptr; // the PDSCH plug-in's stand-in (modulator runs)
    if (plugin && modulate && hipStreamCreateWithFlags(&producer, hipStreamNonBlocking) != hipSuccess) {
      fail[t] = 1;
    }
    arrived.fetch_add(1);
    while (arrived.load() != threads + 1) {
    }
    const auto t0 = std::chrono::steady_clock::now();
    for (unsigned s = 0; s != slots; ++s) {
      for (unsigned l = 0; l != MAX_NSYMB_PER_SLOT; ++l) {
        for (unsigned p = 0; p != nports; ++p) {
          if (modulate) {
            mods[t]->modulate(span<cf_t>(y.data() + off[l], sz[l]), r, p, l);
          } else {
            dems[t]->demodulate(w, span<const cf_t>(x + static_cast<size_t>(p) * n + off[l], sz[l]), p, l);
          }
        }
      }
      if (modulate && plugin && producer != nullptr) {
        // the next slot's grid, written on the device as the PDSCH plug-in writes it: a new content version, so
        // the modulator launches again (no cached slot reused across slots)
        (void)dgrids[t]->grid.device_write(producer);
        dgrids[t]->grid.device_written(producer);
      }
    }
    if (producer != nullptr) {
      (void)hipStreamSynchronize(producer);
      (void)hipStreamDestroy(producer);
    }
    busy[t] = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    if (plugin && !modulate) {
      hipStream_t st = nullptr;
      fail[t]        = hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess;
      if (!fail[t]) {
        (void)dgrids[t]->grid.device_read(st);
        fail[t] = hipStreamSynchronize(st) != hipSuccess;
        (void)hipStreamDestroy(st);
      }
    }
  };
  std::vector<std::thread> pool;
  for (unsigned t = 0; t != threads; ++t) {
    pool.emplace_back(worker, t);
  }
  while (arrived.load() != threads) {
  }
  const auto t0 = std::chrono::steady_clock::now();
  arrived.fetch_add(1);
  for (auto& th : pool) {
    th.join();
  }
  const double dt    = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  double       calls = static_cast<double>(threads) * slots * MAX_NSYMB_PER_SLOT * nports, host = 0;
  uint64_t     xfer  = 0;
  for (unsigned t = 0; t != threads; ++t) {
    host += busy[t];
    if (plugin) {
      xfer += dgrids[t]->grid.nof_downloads() + dgrids[t]->grid.nof_uploads();
    }
    if (fail[t]) {
      return -1;
    }
  }
  out[0] = calls > 0 ? host / calls * 1e6 : 0;
  out[1] = static_cast<double>(xfer);
  return dt;
}

} // extern "C"
