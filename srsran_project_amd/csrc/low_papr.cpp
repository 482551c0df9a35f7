// low_papr.cpp -- low-PAPR base sequences r_{u,v}(n) of TS 38.211 Section 5.2.2 (include/srsran_amd/low_papr.h),
// restating low_papr_sequence_generator_impl.cpp value for value: the phase index of every element is computed
// in integers (phase tables for M <= 24, the 31-point form for M = 30, Zadoff-Chu otherwise) and the value is
// read from a float table exp(j 2 pi k / (2 N_ZC)) built as complex_exponential_table builds it
// (include/srsran/phy/support/complex_exponential_table.h:43-49), so the floats are the reference's own.
#include "srsran_amd/low_papr.h"
#include "srsran_amd/ldpc.h"

#include "api_common.h"
#include "low_papr_tables.inc"
#include <cmath>
#include <complex>
#include <cstdint>
#include <vector>

namespace {

bool is_prime(unsigned n)
{
  if (n < 2) {
    return false;
  }
  for (unsigned d = 2; d * d <= n; ++d) {
    if (n % d == 0) {
      return false;
    }
  }
  return true;
}

// get_N_zc: the largest prime below M for M >= 36 (math_utils.cpp prime_lower_than), 31 for M = 30, else 4
// (the phase tables' exp(j pi phi / 4) as a 2 x 4-entry table).
unsigned nzc_of(unsigned M)
{
  if (M >= 36) {
    unsigned p = M - 1;
    while (!is_prime(p)) {
      --p;
    }
    return p;
  }
  return M == 30 ? 31u : 4u;
}

// zc_sequence_q (low_papr_sequence_generator_impl.cpp): the group / number root, in the reference's float /
// double arithmetic.
int zc_q(uint32_t u, uint32_t v, uint32_t N)
{
  const float n_sz  = static_cast<float>(N);
  const float q_hat = n_sz * static_cast<float>(u + 1) / 31;
  double      q;
  if ((static_cast<uint32_t>(2 * q_hat) % 2) == 0) {
    q = q_hat + 0.5 + v;
  } else {
    q = q_hat + 0.5 - v;
  }
  return static_cast<int>(q);
}

} // namespace

extern "C" {

int srs_amd_low_papr_length_valid(uint32_t M)
{
  for (unsigned short s : SRS_LOW_PAPR_SIZES) {
    if (s == M) {
      return 1;
    }
  }
  return 0;
}

int srs_amd_low_papr_sequence(float* out, uint32_t M, uint32_t u, uint32_t v)
{
  if (out == nullptr) {
    return srs_amd::fail(SRS_AMD_EINVAL, "null output");
  }
  if (!srs_amd_low_papr_length_valid(M)) {
    return srs_amd::fail(SRS_AMD_EINVAL, "Invalid sequence length %u.", M);
  }
  if (u >= 30 || v > 1 || (v != 0 && M < 72)) {
    return srs_amd::fail(SRS_AMD_EINVAL, "Invalid sequence group %u / number %u.", u, v);
  }
  const unsigned N     = nzc_of(M);
  const unsigned tsize = 2 * N;
  // the phase index of element n: exp(j 2 pi arg / tsize)
  std::vector<int> arg(M);
  for (unsigned n = 0; n != M; ++n) {
    if (M <= 24) {
      const signed char* phi = M == 6    ? SRS_LOW_PAPR_PHI_6[u]
                               : M == 12 ? SRS_LOW_PAPR_PHI_12[u]
                               : M == 18 ? SRS_LOW_PAPR_PHI_18[u]
                                         : SRS_LOW_PAPR_PHI_24[u];
      arg[n]                 = phi[n];
    } else if (M == 30) {
      arg[n] = -static_cast<int>(((u + 1L) * (n + 1L) * (n + 2L)) % (2 * 31));
    } else {
      const int64_t q = zc_q(u, v, N);
      const int64_t m = n % N;
      arg[n]          = -static_cast<int>((q * m * (m + 1)) % (2 * N));
    }
  }
  for (unsigned n = 0; n != M; ++n) {
    const unsigned k = static_cast<unsigned>((static_cast<int64_t>(tsize) + arg[n]) % tsize);
    const std::complex<float> x =
        std::polar(1.0F, static_cast<float>(2 * M_PI) * static_cast<float>(k) / static_cast<float>(tsize));
    out[2 * n]     = x.real();
    out[2 * n + 1] = x.imag();
  }
  return SRS_AMD_OK;
}

} // extern "C"
