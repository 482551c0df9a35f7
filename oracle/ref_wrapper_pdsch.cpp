// ref_wrapper_pdsch.cpp -- extern "C" glue around the REFERENCE's own PDSCH
// modulator (scrambling, modulation to ci8, layer mapping, precoding, RE
// mapping) and PDSCH DM-RS processor, compiled from /root/reference by
// oracle/Makefile into oracle/_ref/libsrsran_ref.so.
//
// TEST INFRASTRUCTURE ONLY: pins oracle/pdsch_mod.py (tests/test_oracle_vs_ref.py).
//
// Wrapped reference classes:
//   lib/phy/upper/channel_processors/pdsch/pdsch_modulator_impl.cpp     pdsch_modulator_impl
//   lib/phy/upper/signal_processors/pdsch/dmrs_pdsch_processor_impl.cpp dmrs_pdsch_processor_impl
//   lib/phy/support/resource_grid_mapper_impl.cpp                       resource_grid_mapper_impl
//   lib/phy/generic_functions/precoding/channel_precoder_{generic,avx2,avx512}.cpp
//   lib/phy/support/resource_grid_writer_impl.cpp                       resource_grid_writer_impl
// The grid crosses the boundary as a dense complex-bf16 array
// [port][symbol][subcarrier] (the reference's resource_grid_impl tensor layout);
// it is copied into the reference's own tensor / writer and back.
#include "phy/generic_functions/precoding/channel_precoder_avx2.h"
#include "phy/generic_functions/precoding/channel_precoder_generic.h"
#include "phy/support/resource_grid_mapper_impl.h"
#include "phy/support/resource_grid_writer_impl.h"
#include "phy/upper/channel_modulation/modulation_mapper_lut_impl.h"
#include "phy/upper/channel_processors/pdsch/pdsch_modulator_impl.h"
#include "phy/upper/sequence_generators/pseudo_random_generator_impl.h"
#include "phy/upper/signal_processors/pdsch/dmrs_pdsch_processor_impl.h"
#include "srsran/adt/tensor.h"
#include <atomic>
#include <cstring>
#include <memory>

#ifdef SRS_REF_AVX512
#include "phy/generic_functions/precoding/channel_precoder_avx512.h"
#endif

using namespace srsran;

namespace {

using grid_tensor = dynamic_tensor<static_cast<unsigned>(resource_grid_dimensions::all), cbf16_t, resource_grid_dimensions>;

// precoder: 0 generic, 1 AVX2, 2 AVX512 (falls back to AVX2 when not compiled in).
std::unique_ptr<channel_precoder> make_precoder(int precoder)
{
#ifdef SRS_REF_AVX512
  if (precoder == 2) {
    return std::make_unique<channel_precoder_avx512>();
  }
#endif
  if (precoder == 0) {
    return std::make_unique<channel_precoder_generic>();
  }
  return std::make_unique<channel_precoder_avx2>();
}

struct grid_copy {
  grid_tensor           data;
  std::atomic<unsigned> empty{0};
  cbf16_t*              flat;
  unsigned              nports, nsymb, nsubc;
  grid_copy(cbf16_t* flat_, unsigned nports_, unsigned nsymb_, unsigned nsubc_) :
    data({nsubc_, nsymb_, nports_}), flat(flat_), nports(nports_), nsymb(nsymb_), nsubc(nsubc_)
  {
    for (unsigned p = 0; p != nports; ++p) {
      for (unsigned l = 0; l != nsymb; ++l) {
        span<cbf16_t> row = data.get_view<static_cast<unsigned>(resource_grid_dimensions::symbol)>({l, p});
        std::memcpy(row.data(), flat + (p * nsymb + l) * nsubc, nsubc * sizeof(cbf16_t));
      }
    }
  }
  void copy_back()
  {
    for (unsigned p = 0; p != nports; ++p) {
      for (unsigned l = 0; l != nsymb; ++l) {
        span<const cbf16_t> row = data.get_view<static_cast<unsigned>(resource_grid_dimensions::symbol)>({l, p});
        std::memcpy(flat + (p * nsymb + l) * nsubc, row.data(), nsubc * sizeof(cbf16_t));
      }
    }
  }
};

modulation_scheme to_scheme(int qm)
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

symbol_slot_mask to_symbols(unsigned mask)
{
  symbol_slot_mask s(MAX_NSYMB_PER_SLOT);
  for (unsigned l = 0; l != MAX_NSYMB_PER_SLOT; ++l) {
    if ((mask >> l) & 1u) {
      s.set(l);
    }
  }
  return s;
}

// weights: complex float [prg][layer][port] (re, im interleaved).
precoding_configuration
to_precoding(unsigned nof_layers, unsigned nof_ports, unsigned nof_prg, unsigned prg_size, const float* weights)
{
  precoding_configuration p(nof_layers, nof_ports, nof_prg, prg_size);
  for (unsigned g = 0; g != nof_prg; ++g) {
    for (unsigned l = 0; l != nof_layers; ++l) {
      for (unsigned a = 0; a != nof_ports; ++a) {
        const float* w = weights + 2 * ((g * nof_layers + l) * nof_ports + a);
        p.set_coefficient(cf_t(w[0], w[1]), l, a, g);
      }
    }
  }
  return p;
}

} // namespace

extern "C" {

// pdsch_modulator::modulate (pdsch_modulator_impl.cpp:94-115) on a grid
// [nof_grid_ports][14][nsubc] (modified in place). VRBs: bitmap of nof_vrb_bits
// bytes... as 0/1 bytes (vrbs[i] != 0: VRB i of the BWP allocated, type-0 mask,
// no interleaving). reserved: nof_reserved patterns, each crb mask as 0/1 bytes
// [MAX_RB], re_mask (12 bits), symbols (14 bits).
int srs_ref_pdsch_modulate(uint16_t*       grid,
                       unsigned        nof_grid_ports,
                       unsigned        nsubc,
                       const uint8_t*  codeword,
                       unsigned        nof_bits,
                       unsigned        rnti,
                       unsigned        bwp_start,
                       unsigned        bwp_size,
                       int             qm,
                       const uint8_t*  vrbs,
                       unsigned        start_symbol,
                       unsigned        nof_symbols,
                       unsigned        dmrs_symb_mask,
                       int             dmrs_type2,
                       unsigned        nof_cdm_groups_without_data,
                       unsigned        n_id,
                       float           scaling,
                       const uint8_t*  reserved_crbs,
                       const uint16_t* reserved_re,
                       const uint16_t* reserved_symbols,
                       unsigned        nof_reserved,
                       unsigned        nof_layers,
                       unsigned        nof_ports,
                       const float*    weights,
                       int             precoder)
{
  pdsch_modulator_impl mod(std::make_unique<modulation_mapper_lut_impl>(),
                           std::make_unique<pseudo_random_generator_impl>(),
                           std::make_unique<resource_grid_mapper_impl>(make_precoder(precoder)));

  pdsch_modulator::config_t cfg;
  cfg.rnti        = static_cast<uint16_t>(rnti);
  cfg.bwp         = crb_interval{bwp_start, bwp_start + bwp_size};
  cfg.modulation1 = to_scheme(qm);
  cfg.modulation2 = to_scheme(qm);
  vrb_bitmap vrb_mask(bwp_size);
  for (unsigned i = 0; i != bwp_size; ++i) {
    if (vrbs[i]) {
      vrb_mask.set(i);
    }
  }
  cfg.freq_allocation             = rb_allocation::make_type0(vrb_mask);
  cfg.time_alloc                  = ofdm_symbol_range(start_symbol, start_symbol + nof_symbols);
  cfg.dmrs_symb_pos               = to_symbols(dmrs_symb_mask);
  cfg.dmrs_config_type            = dmrs_type2 ? dmrs_type::TYPE2 : dmrs_type::TYPE1;
  cfg.nof_cdm_groups_without_data = nof_cdm_groups_without_data;
  cfg.n_id                        = n_id;
  cfg.scaling                     = scaling;
  for (unsigned r = 0; r != nof_reserved; ++r) {
    re_pattern pat;
    pat.crb_mask.resize(MAX_RB);
    for (unsigned i = 0; i != MAX_RB; ++i) {
      if (reserved_crbs[r * MAX_RB + i]) {
        pat.crb_mask.set(i);
      }
    }
    for (unsigned k = 0; k != NRE; ++k) {
      pat.re_mask.set(k, (reserved_re[r] >> k) & 1u);
    }
    pat.symbols = to_symbols(reserved_symbols[r]);
    cfg.reserved.merge(pat);
  }
  cfg.precoding = to_precoding(nof_layers, nof_ports, 1, MAX_RB, weights);

  dynamic_bit_buffer cw(nof_bits);
  std::memcpy(cw.get_buffer().data(), codeword, (nof_bits + 7) / 8);

  grid_copy                 g(reinterpret_cast<cbf16_t*>(grid), nof_grid_ports, MAX_NSYMB_PER_SLOT, nsubc);
  resource_grid_writer_impl writer(g.data, g.empty);
  bit_buffer                cws[1] = {cw};
  mod.modulate(writer, cws, cfg);
  g.copy_back();
  return 0;
}

// dmrs_pdsch_processor::map (dmrs_pdsch_processor_impl.cpp:126-234). crbs: 0/1
// bytes [MAX_RB]; weights [prg][layer][port].
int srs_ref_dmrs_pdsch_map(uint16_t*      grid,
                       unsigned       nof_grid_ports,
                       unsigned       nsubc,
                       unsigned       numerology,
                       unsigned       slot_index,
                       unsigned       reference_point_k_rb,
                       int            type2,
                       unsigned       scrambling_id,
                       int            n_scid,
                       float          amplitude,
                       unsigned       symbols_mask,
                       const uint8_t* crbs,
                       unsigned       nof_layers,
                       unsigned       nof_ports,
                       unsigned       nof_prg,
                       unsigned       prg_size,
                       const float*   weights,
                       int            precoder)
{
  dmrs_pdsch_processor_impl proc(std::make_unique<pseudo_random_generator_impl>(),
                                 std::make_unique<resource_grid_mapper_impl>(make_precoder(precoder)));
  dmrs_pdsch_processor::config_t cfg;
  cfg.slot                 = slot_point(numerology, slot_index);
  cfg.reference_point_k_rb = reference_point_k_rb;
  cfg.type                 = type2 ? dmrs_type::TYPE2 : dmrs_type::TYPE1;
  cfg.scrambling_id        = scrambling_id;
  cfg.n_scid               = n_scid != 0;
  cfg.amplitude            = amplitude;
  cfg.symbols_mask         = to_symbols(symbols_mask);
  cfg.rb_mask.resize(MAX_RB);
  for (unsigned i = 0; i != MAX_RB; ++i) {
    if (crbs[i]) {
      cfg.rb_mask.set(i);
    }
  }
  cfg.precoding = to_precoding(nof_layers, nof_ports, nof_prg, prg_size, weights);

  grid_copy                 g(reinterpret_cast<cbf16_t*>(grid), nof_grid_ports, MAX_NSYMB_PER_SLOT, nsubc);
  resource_grid_writer_impl writer(g.data, g.empty);
  proc.map(writer, cfg);
  g.copy_back();
  return 0;
}

} // extern "C"
