// ref_wrapper.cpp -- extern "C" glue around the REFERENCE's own LDPC / CRC
// classes, compiled from the sources where they lie under /root/reference by
// oracle/Makefile into oracle/_ref/libsrsran_ref.so (git-ignored).
//
// TEST INFRASTRUCTURE ONLY: used by tests/ to pin oracle/srs_oracle.c and by
// bench.py's cpu_baseline leg ("kind": "reference").  The product never loads it.
//
// Wrapped reference interfaces:
//   include/srsran/phy/upper/channel_coding/ldpc/ldpc_decoder.h:72  ldpc_decoder::decode
//   include/srsran/phy/upper/channel_coding/ldpc/ldpc_encoder.h     ldpc_encoder::encode
//   include/srsran/phy/upper/channel_coding/crc_calculator.h        crc_calculator::calculate_bit
//   include/srsran/phy/upper/channel_coding/ldpc/ldpc_rate_matcher.h / ldpc_rate_dematcher.h
#include "phy/upper/channel_coding/crc_calculator_generic_impl.h"
#include "phy/upper/channel_coding/ldpc/ldpc_decoder_avx2.h"
#include "phy/upper/channel_coding/ldpc/ldpc_decoder_generic.h"
#include "phy/upper/channel_coding/ldpc/ldpc_encoder_avx2.h"
#include "phy/upper/channel_coding/ldpc/ldpc_encoder_generic.h"
#include "phy/upper/channel_coding/ldpc/ldpc_rate_dematcher_avx2_impl.h"
#include "phy/upper/channel_coding/ldpc/ldpc_rate_dematcher_avx512_impl.h"
#include "phy/upper/channel_coding/ldpc/ldpc_rate_dematcher_impl.h"
#include "phy/upper/channel_coding/ldpc/ldpc_rate_matcher_impl.h"
#include "srsran/phy/upper/channel_coding/ldpc/ldpc_encoder_buffer.h"
#include "srsran/srsvec/bit.h"
#include <atomic>
#include <chrono>
#include <cstring>
#include <memory>
#include <string>
#include <thread>
#include <vector>

#ifdef SRS_REF_HAVE_AVX512
#include "phy/upper/channel_coding/ldpc/ldpc_decoder_avx512.h"
#endif

using namespace srsran;

namespace {

std::unique_ptr<ldpc_decoder> make_decoder(const char* impl, bool force)
{
  std::string t(impl);
#ifdef SRS_REF_HAVE_AVX512
  if (t == "avx512") {
    if (!__builtin_cpu_supports("avx512bw")) {
      return nullptr;
    }
    return std::make_unique<ldpc_decoder_avx512>(force);
  }
#endif
  if (t == "avx2") {
    if (!__builtin_cpu_supports("avx2")) {
      return nullptr;
    }
    return std::make_unique<ldpc_decoder_avx2>(force);
  }
  if (t == "generic") {
    return std::make_unique<ldpc_decoder_generic>(force);
  }
  return nullptr;
}

crc_calculator* get_crc(int poly)
{
  static crc_calculator_generic_impl crcs[] = {crc_calculator_generic_impl(crc_generator_poly::CRC24A),
                                               crc_calculator_generic_impl(crc_generator_poly::CRC24B),
                                               crc_calculator_generic_impl(crc_generator_poly::CRC24C),
                                               crc_calculator_generic_impl(crc_generator_poly::CRC16),
                                               crc_calculator_generic_impl(crc_generator_poly::CRC11),
                                               crc_calculator_generic_impl(crc_generator_poly::CRC6)};
  if (poly < 0 || poly > 5) {
    return nullptr;
  }
  return &crcs[poly];
}

} // namespace

extern "C" {

int srs_ref_has_impl(const char* impl)
{
  return make_decoder(impl, false) != nullptr;
}

// Decodes one codeblock through the reference decoder `impl` (fresh object per
// call, like a fresh factory product).  Returns iterations, -1 = nullopt, -2 = bad impl.
int srs_ref_ldpc_decode(const char* impl,
                        int         bg,
                        int         Z,
                        int         nof_filler_bits,
                        int         nof_crc_bits,
                        int         max_iterations,
                        int         force_decoding,
                        int         crc_poly,
                        const int8_t* llrs,
                        unsigned    n_llrs,
                        uint8_t*    out_packed)
{
  auto dec = make_decoder(impl, force_decoding != 0);
  if (!dec) {
    return -2;
  }
  ldpc_decoder::configuration cfg;
  cfg.base_graph      = static_cast<ldpc_base_graph_type>(bg);
  cfg.lifting_size    = static_cast<ldpc::lifting_size_t>(Z);
  cfg.nof_filler_bits = nof_filler_bits;
  cfg.nof_crc_bits    = nof_crc_bits;
  cfg.max_iterations  = max_iterations;
  unsigned                           K = (bg == 1 ? 22 : 10) * Z;
  dynamic_bit_buffer                 out(K);
  span<const log_likelihood_ratio>   in(reinterpret_cast<const log_likelihood_ratio*>(llrs), n_llrs);
  std::optional<unsigned>            r = dec->decode(out, in, crc_poly >= 0 ? get_crc(crc_poly) : nullptr, cfg);
  std::memcpy(out_packed, out.get_buffer().data(), (K + 7) / 8);
  return r.has_value() ? static_cast<int>(*r) : -1;
}

// Encodes one message (one bit per byte, K bits) and writes n_out <= N_short*Z bits.
int srs_ref_ldpc_encode(const char* impl, int bg, int Z, const uint8_t* msg_bits, uint8_t* cw_bits, unsigned n_out)
{
  std::unique_ptr<ldpc_encoder> enc;
  if (std::string(impl) == "avx2" && __builtin_cpu_supports("avx2")) {
    enc = std::make_unique<ldpc_encoder_avx2>();
  } else if (std::string(impl) == "generic") {
    enc = std::make_unique<ldpc_encoder_generic>();
  } else {
    return -2;
  }
  unsigned           K = (bg == 1 ? 22 : 10) * Z;
  dynamic_bit_buffer msg(K);
  srsvec::bit_pack(msg, span<const uint8_t>(msg_bits, K));
  ldpc_encoder::configuration cfg;
  cfg.base_graph                = static_cast<ldpc_base_graph_type>(bg);
  cfg.lifting_size              = static_cast<ldpc::lifting_size_t>(Z);
  const ldpc_encoder_buffer& rb = enc->encode(msg, cfg);
  rb.write_codeblock(span<uint8_t>(cw_bits, n_out), 0);
  return 0;
}

unsigned srs_ref_crc_bits(int poly, const uint8_t* bits, unsigned nbits)
{
  crc_calculator* c = get_crc(poly);
  if (!c) {
    return 0xffffffffu;
  }
  return c->calculate_bit(span<const uint8_t>(bits, nbits));
}

static modulation_scheme mod_of(unsigned Qm)
{
  switch (Qm) {
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

static codeblock_metadata make_meta(int bg, int Z, unsigned rv, unsigned Qm, unsigned Nref, unsigned F, unsigned E)
{
  codeblock_metadata m;
  m.tb_common.base_graph        = static_cast<ldpc_base_graph_type>(bg);
  m.tb_common.lifting_size      = static_cast<ldpc::lifting_size_t>(Z);
  m.tb_common.rv                = rv;
  m.tb_common.mod               = mod_of(Qm);
  m.tb_common.Nref              = Nref;
  m.tb_common.cw_length         = E;
  m.cb_specific.full_length     = (bg == 1 ? 66 : 50) * Z;
  m.cb_specific.rm_length       = E;
  m.cb_specific.nof_filler_bits = F;
  return m;
}

// Encodes msg (K bits, one per byte, filler positions 0) with the reference
// encoder and rate-matches it: E bits packed MSB-first.
int srs_ref_ldpc_encode_rate_match(int            bg,
                                   int            Z,
                                   unsigned       rv,
                                   unsigned       Qm,
                                   unsigned       Nref,
                                   unsigned       F,
                                   const uint8_t* msg_bits,
                                   unsigned       E,
                                   uint8_t*       out_packed)
{
  ldpc_encoder_generic enc;
  unsigned             K = (bg == 1 ? 22 : 10) * Z;
  dynamic_bit_buffer   msg(K);
  srsvec::bit_pack(msg, span<const uint8_t>(msg_bits, K));
  ldpc_encoder::configuration cfg;
  cfg.base_graph                = static_cast<ldpc_base_graph_type>(bg);
  cfg.lifting_size              = static_cast<ldpc::lifting_size_t>(Z);
  cfg.Nref                      = Nref;
  const ldpc_encoder_buffer& rb = enc.encode(msg, cfg);
  auto                       rm = std::make_unique<ldpc_rate_matcher_impl>();
  dynamic_bit_buffer         out(E);
  rm->rate_match(out, rb, make_meta(bg, Z, rv, Qm, Nref, F, E));
  std::memcpy(out_packed, out.get_buffer().data(), (E + 7) / 8);
  return 0;
}

// Rate-dematches E LLRs into the soft buffer buf (N = N_short*Z LLRs, in/out).
int srs_ref_ldpc_rate_dematch(const char*   impl,
                              int           bg,
                              int           Z,
                              unsigned      rv,
                              unsigned      Qm,
                              unsigned      Nref,
                              unsigned      F,
                              int           new_data,
                              const int8_t* in,
                              unsigned      E,
                              int8_t*       buf)
{
  std::unique_ptr<ldpc_rate_dematcher> dm;
  if (std::string(impl) == "generic") {
    dm = std::make_unique<ldpc_rate_dematcher_impl>();
  } else if (std::string(impl) == "avx2" && __builtin_cpu_supports("avx2")) {
    dm = std::make_unique<ldpc_rate_dematcher_avx2_impl>();
  } else if (std::string(impl) == "avx512" && __builtin_cpu_supports("avx512f") && __builtin_cpu_supports("avx512bw")) {
    dm = std::make_unique<ldpc_rate_dematcher_avx512_impl>();
  } else {
    return -2;
  }
  unsigned N = (bg == 1 ? 66 : 50) * Z;
  dm->rate_dematch(span<log_likelihood_ratio>(reinterpret_cast<log_likelihood_ratio*>(buf), N),
                   span<const log_likelihood_ratio>(reinterpret_cast<const log_likelihood_ratio*>(in), E),
                   new_data != 0,
                   make_meta(bg, Z, rv, Qm, Nref, F, E));
  return 0;
}

// CPU baseline: decodes n_cbs codeblocks (codeblock i = sample row i % n_sample,
// each n_llrs LLRs) with
// `threads` worker threads, each owning one decoder (as the PUSCH decoder pool
// does).  Returns wall seconds; iteration results written to iters (may be null).
double srs_ref_ldpc_decode_many(const char*   impl,
                                int           bg,
                                int           Z,
                                int           max_iterations,
                                int           crc_poly,
                                const int8_t* llrs,
                                unsigned      n_llrs,
                                unsigned      n_sample,
                                unsigned      n_cbs,
                                int           threads,
                                uint8_t*      out_packed,
                                int*          iters)
{
  if (threads < 1) {
    threads = 1;
  }
  unsigned              K     = (bg == 1 ? 22 : 10) * Z;
  unsigned              obyte = (K + 7) / 8;
  std::atomic<unsigned> next{0};
  std::atomic<int>      bad{0};
  auto                  t0 = std::chrono::steady_clock::now();
  std::vector<std::thread> pool;
  for (int t = 0; t < threads; ++t) {
    pool.emplace_back([&]() {
      auto dec = make_decoder(impl, false);
      if (!dec) {
        bad = 1;
        return;
      }
      ldpc_decoder::configuration cfg;
      cfg.base_graph     = static_cast<ldpc_base_graph_type>(bg);
      cfg.lifting_size   = static_cast<ldpc::lifting_size_t>(Z);
      cfg.nof_crc_bits   = 24;
      cfg.max_iterations = max_iterations;
      dynamic_bit_buffer out(K);
      for (unsigned i = next++; i < n_cbs; i = next++) {
        // codeblock i reads sample row i % n_sample (bounded memory for long CPU runs)
        span<const log_likelihood_ratio> in(
            reinterpret_cast<const log_likelihood_ratio*>(llrs) + size_t(i % n_sample) * n_llrs, n_llrs);
        std::optional<unsigned>          r = dec->decode(out, in, crc_poly >= 0 ? get_crc(crc_poly) : nullptr, cfg);
        if (out_packed) {
          std::memcpy(out_packed + size_t(i % n_sample) * obyte, out.get_buffer().data(), obyte);
        }
        if (iters) {
          iters[i % n_sample] = r.has_value() ? static_cast<int>(*r) : -1;
        }
      }
    });
  }
  for (auto& th : pool) {
    th.join();
  }
  auto t1 = std::chrono::steady_clock::now();
  if (bad) {
    return -1.0;
  }
  return std::chrono::duration<double>(t1 - t0).count();
}

} // extern "C"
