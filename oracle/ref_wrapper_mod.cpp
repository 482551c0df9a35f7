// ref_wrapper_mod.cpp -- extern "C" glue around the REFERENCE's modulation
// mapper, soft demodulation mapper and pseudo-random generator (compiled from
// /root/reference by oracle/Makefile).  TEST INFRASTRUCTURE ONLY: pins
// oracle/srs_oracle_mod.c.
#include "phy/upper/channel_modulation/demodulation_mapper_impl.h"
#include "phy/upper/channel_modulation/modulation_mapper_lut_impl.h"
#include "phy/upper/sequence_generators/pseudo_random_generator_impl.h"
#include "srsran/adt/bit_buffer.h"
#include <cstring>
#include <vector>

using namespace srsran;

static modulation_scheme scheme_of(int Qm)
{
  switch (Qm) {
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

extern "C" {

int srs_ref_modulate(int Qm, const uint8_t* bits, unsigned nsym, float* out)
{
  unsigned           nbits = nsym * (Qm == 0 ? 1 : Qm);
  dynamic_bit_buffer in(nbits);
  std::memcpy(in.get_buffer().data(), bits, (nbits + 7) / 8);
  modulation_mapper_lut_impl mod;
  mod.modulate(span<cf_t>(reinterpret_cast<cf_t*>(out), nsym), in, scheme_of(Qm));
  return 0;
}

int srs_ref_demodulate(int Qm, const float* sym, const float* nvar, unsigned nsym, int8_t* llr)
{
  demodulation_mapper_impl dem;
  unsigned                 nbits = nsym * (Qm == 0 ? 1 : Qm);
  dem.demodulate_soft(span<log_likelihood_ratio>(reinterpret_cast<log_likelihood_ratio*>(llr), nbits),
                      span<const cf_t>(reinterpret_cast<const cf_t*>(sym), nsym),
                      span<const float>(nvar, nsym),
                      scheme_of(Qm));
  return 0;
}

// c(n) one bit per byte: apply_xor on a zero input.
int srs_ref_prbs(uint32_t c_init, unsigned len, uint8_t* c)
{
  pseudo_random_generator_impl prg;
  prg.init(c_init);
  std::vector<uint8_t> zeros(len, 0);
  prg.apply_xor(span<uint8_t>(c, len), zeros);
  return 0;
}

// LLR descrambling: apply_xor on log-likelihood ratios.
int srs_ref_descramble_llrs(uint32_t c_init, unsigned len, const int8_t* in, int8_t* out)
{
  pseudo_random_generator_impl prg;
  prg.init(c_init);
  prg.apply_xor(span<log_likelihood_ratio>(reinterpret_cast<log_likelihood_ratio*>(out), len),
                span<const log_likelihood_ratio>(reinterpret_cast<const log_likelihood_ratio*>(in), len));
  return 0;
}

// Packed bit scrambling: apply_xor on bit buffers.
int srs_ref_scramble_bits(uint32_t c_init, unsigned nbits, const uint8_t* in, uint8_t* out)
{
  pseudo_random_generator_impl prg;
  prg.init(c_init);
  dynamic_bit_buffer a(nbits), b(nbits);
  std::memcpy(a.get_buffer().data(), in, (nbits + 7) / 8);
  prg.apply_xor(b, a);
  std::memcpy(out, b.get_buffer().data(), (nbits + 7) / 8);
  return 0;
}

} // extern "C"
