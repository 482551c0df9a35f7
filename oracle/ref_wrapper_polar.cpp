// ref_wrapper_polar.cpp -- extern "C" glue around the REFERENCE's polar classes
// (lib/phy/upper/channel_coding/polar/*, compiled from /root/reference by
// oracle/Makefile).  TEST INFRASTRUCTURE ONLY: pins oracle/srs_oracle_polar.c.
// The chains mirror the reference's users: pdcch_encoder_impl (allocate ->
// encode -> rate match) and the UCI polar decoder (rate dematch -> decode ->
// deallocate).
#include "phy/upper/channel_coding/polar/polar_allocator_impl.h"
#include "phy/upper/channel_coding/polar/polar_code_impl.h"
#include "phy/upper/channel_coding/polar/polar_deallocator_impl.h"
#include "phy/upper/channel_coding/polar/polar_decoder_impl.h"
#include "phy/upper/channel_coding/polar/polar_encoder_impl.h"
#include "phy/upper/channel_coding/polar/polar_interleaver_impl.h"
#include "phy/upper/channel_coding/polar/polar_rate_dematcher_impl.h"
#include "phy/upper/channel_coding/polar/polar_rate_matcher_impl.h"
#include <chrono>
#include <cstring>
#include <memory>
#include <thread>
#include <vector>

using namespace srsran;

extern "C" {

unsigned srs_ref_polar_code(unsigned K, unsigned E, unsigned nMax, uint8_t* kmask, uint16_t* pc, unsigned* nPC)
{
  polar_code_impl code;
  code.set(K, E, nMax, polar_code_ibil::not_present);
  unsigned N = code.get_N();
  for (unsigned i = 0; i < N; ++i) {
    kmask[i] = code.get_K_set().test(i) ? 1 : 0;
  }
  *nPC = code.get_nPC();
  for (unsigned i = 0; i < code.get_nPC(); ++i) {
    pc[i] = code.get_PC_set()[i];
  }
  return N;
}

int srs_ref_polar_encode_chain(unsigned K, unsigned E, unsigned nMax, int ibil, const uint8_t* msg, uint8_t* out)
{
  polar_code_impl code;
  code.set(K, E, nMax, ibil ? polar_code_ibil::present : polar_code_ibil::not_present);
  unsigned             N = code.get_N();
  std::vector<uint8_t> u(N), x(N);
  polar_allocator_impl alloc;
  alloc.allocate(u, span<const uint8_t>(msg, K), code);
  polar_encoder_impl enc;
  enc.encode(x, u, code.get_n());
  polar_rate_matcher_impl rm;
  rm.rate_match(span<uint8_t>(out, E), x, code);
  return 0;
}

int srs_ref_polar_decode_chain(unsigned K, unsigned E, unsigned nMax, int ibil, const int8_t* llr, uint8_t* msg)
{
  polar_code_impl code;
  code.set(K, E, nMax, ibil ? polar_code_ibil::present : polar_code_ibil::not_present);
  unsigned                          N = code.get_N();
  std::vector<log_likelihood_ratio> y(N);
  std::vector<uint8_t>              d(N);
  polar_rate_dematcher_impl         dm;
  dm.rate_dematch(y, span<const log_likelihood_ratio>(reinterpret_cast<const log_likelihood_ratio*>(llr), E), code);
  polar_decoder_impl dec(std::make_unique<polar_encoder_impl>(), polar_code::NMAX_LOG);
  dec.decode(d, y, code);
  polar_deallocator_impl dealloc;
  dealloc.deallocate(span<uint8_t>(msg, K), d, code);
  return 0;
}

int srs_ref_polar_interleave(const uint8_t* in, uint8_t* out, unsigned K, int dir)
{
  polar_interleaver_impl il;
  il.interleave(span<uint8_t>(out, K), span<const uint8_t>(in, K),
                dir == 0 ? polar_interleaver_direction::tx : polar_interleaver_direction::rx);
  return 0;
}

// CPU baseline: decodes n codewords (cycling over n_sample LLR vectors of E each) with `threads` workers.
double srs_ref_polar_decode_many(unsigned      K,
                                 unsigned      E,
                                 unsigned      nMax,
                                 const int8_t* llrs,
                                 unsigned      n_sample,
                                 unsigned      n,
                                 unsigned      threads)
{
  auto                     t0 = std::chrono::steady_clock::now();
  std::vector<std::thread> pool;
  for (unsigned t = 0; t < threads; ++t) {
    pool.emplace_back([=]() {
      polar_code_impl code;
      code.set(K, E, nMax, polar_code_ibil::not_present);
      unsigned                          N = code.get_N();
      std::vector<log_likelihood_ratio> y(N);
      std::vector<uint8_t>              d(N), msg(K);
      polar_rate_dematcher_impl         dm;
      polar_decoder_impl                dec(std::make_unique<polar_encoder_impl>(), polar_code::NMAX_LOG);
      polar_deallocator_impl            dealloc;
      for (unsigned i = t; i < n; i += threads) {
        const int8_t* l = llrs + static_cast<size_t>(i % n_sample) * E;
        dm.rate_dematch(y, span<const log_likelihood_ratio>(reinterpret_cast<const log_likelihood_ratio*>(l), E), code);
        dec.decode(d, y, code);
        dealloc.deallocate(msg, d, code);
      }
    });
  }
  for (auto& th : pool) {
    th.join();
  }
  return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
}

} // extern "C"
