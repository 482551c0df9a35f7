// modulation_api.cpp -- C-ABI of the MI355X modulation mapper, soft demapper
// and scrambling (include/srsran_amd/modulation.h).
//
// Host-side tables, computed once per object with the reference's own float
// operations:
//   modulation LUTs: modulation_mapper_lut_impl.cpp:35-60 (TS 38.211 5.1 levels,
//     scaled by sqrt(1 / average power));
//   soft-demapper interval lines: the max-log LLR of each Gray-mapped PAM axis
//     bit, slope 2a(o0 - o1), intercept (o1^2 - o0^2) / norm (the values of
//     demodulation_mapper_qam64.cpp:43-78 / _qam256.cpp:43-170), the least
//     significant axis bit on intervals of width 4a, the others 2a;
//   Gold-sequence jump matrices A^(2^k) of the two TS 38.211 5.2.1 LFSRs.
#include "srsran_amd/modulation.h"

#include <hip/hip_runtime.h>

#include "api_common.h"
#include "modulation_args.h"
#include <cmath>
#include <mutex>
#include <vector>

using namespace srs_amd;

namespace {

int bits_per_symbol(int qm)
{
  return qm <= 1 ? 1 : qm;
}

bool valid_qm(int qm)
{
  return qm == 0 || qm == 1 || qm == 2 || qm == 4 || qm == 6 || qm == 8;
}

// AVX2 block of demodulation_mapper_{qpsk,qam16,qam64,qam256}.cpp; the rest is scalar code.
uint32_t avx2_block(int qm)
{
  switch (qm) {
    case 2:
      return 16;
    case 4:
      return 8;
    case 6:
      return 16;
    case 8:
      return 4;
    default:
      return 0;
  }
}

// Axis bit k (0 = sign) of the PAM level with odd value o (TS 38.211 5.1).
int pam_bit(int m, int o, int k)
{
  for (int pat = 0; pat < (1 << m); ++pat) {
    int v = 1;
    for (int j = m - 1; j >= 1; --j) {
      v = (1 << (m - j)) - (1 - 2 * ((pat >> j) & 1)) * v;
    }
    v *= 1 - 2 * (pat & 1);
    if (v == o) {
      return (pat >> k) & 1;
    }
  }
  return -1;
}

demod_interval_table make_table(int m, int k, float a, float norm)
{
  demod_interval_table t{};
  const int            L  = 1 << m;
  const bool           lsb = (k == m - 1);
  t.n                     = lsb ? L / 2 : L;
  t.width                 = static_cast<float>(lsb ? 4 : 2) * a;
  t.inv_width             = 1.0f / t.width;
  const double w          = lsb ? 4.0 : 2.0;
  for (int i = 0; i < t.n; ++i) {
    const double x  = ((i - t.n / 2) + 0.5) * w;
    int          o0 = 0, o1 = 0;
    double       d0 = 1e30, d1 = 1e30;
    for (int li = 0; li < L; ++li) {
      const int    o = 2 * li - (L - 1);
      const double d = (x - o) * (x - o);
      if (pam_bit(m, o, k) == 0) {
        if (d < d0) {
          d0 = d;
          o0 = o;
        }
      } else if (d < d1) {
        d1 = d;
        o1 = o;
      }
    }
    t.slope[i] = static_cast<float>(2 * (o0 - o1)) * a;
    t.icpt[i]  = static_cast<float>(o1 * o1 - o0 * o0) / norm;
  }
  return t;
}

// One step of the x1 / x2 LFSRs (state bit i = x(n + i)).
uint32_t lfsr_step(uint32_t s, bool x2)
{
  const uint32_t nb = x2 ? (((s >> 3) ^ (s >> 2) ^ (s >> 1) ^ s) & 1u) : (((s >> 3) ^ s) & 1u);
  return (s >> 1) | (nb << 30);
}

uint32_t gf2_apply_host(const uint32_t* cols, uint32_t s)
{
  uint32_t r = 0;
  for (int j = 0; j < 31; ++j) {
    if ((s >> j) & 1u) {
      r ^= cols[j];
    }
  }
  return r;
}

} // namespace

std::vector<uint32_t> srs_amd::gold_jump_tables()
{
  std::vector<uint32_t> t(PRBS_NIB_OFF + 2 * PRBS_NIB_NK * 8 * 16, 0u);
  for (int which = 0; which < 2; ++which) {
    uint32_t* m0 = t.data() + (which * PRBS_NJUMP) * 31;
    for (int j = 0; j < 31; ++j) {
      m0[j] = lfsr_step(1u << j, which == 1);
    }
    for (int k = 1; k < PRBS_NJUMP; ++k) {
      const uint32_t* prev = t.data() + (which * PRBS_NJUMP + k - 1) * 31;
      uint32_t*       cur  = t.data() + (which * PRBS_NJUMP + k) * 31;
      for (int j = 0; j < 31; ++j) {
        cur[j] = gf2_apply_host(prev, prev[j]);
      }
    }
    // radix 16: A^(d 16^k) = A^((d-1) 16^k) A^(16^k), A^(16^k) = the binary matrix 4k
    for (int k = 0; k < PRBS_RADIX_DIGITS; ++k) {
      const uint32_t* base = t.data() + (which * PRBS_NJUMP + 4 * k) * 31;
      uint32_t*       row  = t.data() + PRBS_RADIX_OFF + ((which * PRBS_RADIX_DIGITS + k) * 16) * 31;
      for (int j = 0; j < 31; ++j) {
        row[31 + j] = base[j];
      }
      for (int d = 2; d < 16; ++d) {
        for (int j = 0; j < 31; ++j) {
          row[d * 31 + j] = gf2_apply_host(row + (d - 1) * 31, base[j]);
        }
      }
    }
    // nibble tables of A^(2^k): [q][v] = A^(2^k) (v << 4 q) (the state has 31 bits: nibble 7 holds bits 28..30)
    for (int k = 0; k < PRBS_NIB_NK; ++k) {
      const uint32_t* m   = t.data() + (which * PRBS_NJUMP + PRBS_NIB_K0 + k) * 31;
      uint32_t*       tab = t.data() + PRBS_NIB_OFF + ((which * PRBS_NIB_NK + k) * 8) * 16;
      for (int q = 0; q < 8; ++q) {
        for (uint32_t v = 0; v < 16; ++v) {
          tab[q * 16 + v] = gf2_apply_host(m, (v << (4 * q)) & 0x7fffffffu);
        }
      }
    }
  }
  return t;
}

std::vector<uint32_t> srs_amd::gold_word_basis()
{
  std::vector<uint32_t> t(32 * GOLD_BASIS_WORDS, 0u);
  for (int row = 0; row < 32; ++row) {
    // rows 0..30: x2 from c_init = 2^row; row 31: x1 (initial state 1)
    const bool x2 = row < 31;
    uint32_t   st = x2 ? (1u << row) : 1u;
    for (int n = 0; n < 1600; ++n) {
      st = lfsr_step(st, x2);
    }
    for (uint32_t w = 0; w < GOLD_BASIS_WORDS; ++w) {
      uint32_t word = 0;
      for (uint32_t b = 0; b < 32; ++b) {
        word |= (st & 1u) << b;
        st = lfsr_step(st, x2);
      }
      t[static_cast<size_t>(row) * GOLD_BASIS_WORDS + w] = word;
    }
  }
  return t;
}

struct srs_amd_modulator {
  int                  device = 0;
  hipStream_t          stream = nullptr;
  float*               d_tables = nullptr; // [4 (qm 2,4,6,8)][256][2]
  uint32_t*            d_jump   = nullptr;
  demod_interval_table tab64[3], tab256[4];
  float                qam16_scale = 0;
  void*                scratch      = nullptr;
  size_t               scratch_size = 0;
  std::mutex           mtx;
  ~srs_amd_modulator()
  {
    (void)hipSetDevice(device);
    if (stream) {
      (void)hipStreamSynchronize(stream);
      (void)hipStreamDestroy(stream);
    }
    (void)hipFree(d_tables);
    (void)hipFree(d_jump);
    (void)hipFree(scratch);
  }
  hipError_t ensure(size_t n)
  {
    if (n <= scratch_size) {
      return hipSuccess;
    }
    (void)hipFree(scratch);
    scratch      = nullptr;
    scratch_size = 0;
    hipError_t e = hipMalloc(&scratch, n);
    if (e == hipSuccess) {
      scratch_size = n;
    }
    return e;
  }
};

namespace {

const float* table_ptr(const srs_amd_modulator* m, int qm)
{
  const int slot = qm == 2 ? 0 : qm == 4 ? 1 : qm == 6 ? 2 : 3;
  return m->d_tables + slot * 512;
}

int check(srs_amd_modulator* m, int qm)
{
  if (m == nullptr) {
    return fail(SRS_AMD_EINVAL, "null modulator");
  }
  if (!valid_qm(qm)) {
    return fail(SRS_AMD_EINVAL, "Invalid modulation scheme %d.", qm);
  }
  return SRS_AMD_OK;
}

} // namespace

extern "C" {

int srs_amd_modulator_create(srs_amd_modulator** mod, int device)
{
  if (mod == nullptr) {
    return fail(SRS_AMD_EINVAL, "null handle pointer");
  }
  *mod   = nullptr;
  int rc = select_device(device);
  if (rc != SRS_AMD_OK) {
    return rc;
  }
  auto* m   = new srs_amd_modulator();
  m->device = device;
  // modulation_mapper_lut_impl.cpp:40-58
  std::vector<float> tables(4 * 512, 0.0f);
  for (int slot = 0; slot < 4; ++slot) {
    const int QM = 2 * (slot + 1);
    const int L  = 1 << QM;
    float     sum = 0;
    for (int i = 0; i < L; ++i) {
      float off = -1, re = 0, im = 0;
      for (int j = 0; j < QM / 2; ++j) {
        re += off;
        im += off;
        off *= 2;
        re *= ((i & (1 << (2 * j + 1))) != 0) ? +1 : -1;
        im *= ((i & (1 << (2 * j + 0))) != 0) ? +1 : -1;
      }
      tables[slot * 512 + 2 * i]     = re;
      tables[slot * 512 + 2 * i + 1] = im;
      sum += re * re + im * im; // integers: exact in any order
    }
    const float scaling = std::sqrt(1 / (sum / static_cast<float>(L)));
    for (int i = 0; i < 2 * L; ++i) {
      tables[slot * 512 + i] *= scaling;
    }
  }
  const float a64  = 1.0F / std::sqrt(42.0F);
  const float a256 = 1.0F / std::sqrt(170.0F);
  for (int k = 0; k < 3; ++k) {
    m->tab64[k] = make_table(3, k, a64, 42.0F);
  }
  for (int k = 0; k < 4; ++k) {
    m->tab256[k] = make_table(4, k, a256, 170.0F);
  }
  m->qam16_scale         = 1.0F / std::sqrt(10.0F);
  std::vector<uint32_t> j = gold_jump_tables();
  hipError_t            e = hipMalloc(&m->d_tables, tables.size() * sizeof(float));
  if (e == hipSuccess) {
    e = hipMemcpy(m->d_tables, tables.data(), tables.size() * sizeof(float), hipMemcpyHostToDevice);
  }
  if (e == hipSuccess) {
    e = hipMalloc(&m->d_jump, j.size() * sizeof(uint32_t));
  }
  if (e == hipSuccess) {
    e = hipMemcpy(m->d_jump, j.data(), j.size() * sizeof(uint32_t), hipMemcpyHostToDevice);
  }
  if (e == hipSuccess) {
    e = hipStreamCreateWithFlags(&m->stream, hipStreamNonBlocking);
  }
  if (e != hipSuccess) {
    delete m;
    return hip_fail(e, "modulator tables");
  }
  *mod = m;
  return SRS_AMD_OK;
}

void srs_amd_modulator_destroy(srs_amd_modulator* mod)
{
  delete mod;
}

int srs_amd_modulate_batch(srs_amd_modulator* mod, float* d_symbols, const uint8_t* d_bits, uint32_t nof_symbols,
                           int qm, void* stream)
{
  int rc = check(mod, qm);
  if (rc != SRS_AMD_OK) {
    return rc;
  }
  if (nof_symbols == 0) {
    return SRS_AMD_OK;
  }
  if (d_symbols == nullptr || d_bits == nullptr) {
    return fail(SRS_AMD_EINVAL, "null device buffer");
  }
  modulate_args a{};
  a.bits        = d_bits;
  a.symbols     = d_symbols;
  a.table       = qm >= 2 ? table_ptr(mod, qm) : nullptr;
  a.nof_symbols = nof_symbols;
  a.qm          = qm;
  std::lock_guard<std::mutex> lock(mod->mtx);
  hipError_t                  e = hipSetDevice(mod->device);
  if (e == hipSuccess) {
    e = launch_modulate(a, static_cast<hipStream_t>(stream));
  }
  return e == hipSuccess ? SRS_AMD_OK : hip_fail(e, "modulate_kernel launch");
}

int srs_amd_demodulate_soft_batch(srs_amd_modulator* mod,
                                  int8_t*            d_llrs,
                                  const float*       d_symbols,
                                  const float*       d_noise_vars,
                                  uint32_t           nof_symbols,
                                  int                qm,
                                  void*              stream)
{
  int rc = check(mod, qm);
  if (rc != SRS_AMD_OK) {
    return rc;
  }
  if (nof_symbols == 0) {
    return SRS_AMD_OK;
  }
  if (d_llrs == nullptr || d_symbols == nullptr || d_noise_vars == nullptr) {
    return fail(SRS_AMD_EINVAL, "null device buffer");
  }
  demodulate_args a = srs_amd::demodulate_args_for(mod, qm, nof_symbols);
  a.symbols         = d_symbols;
  a.noise_vars      = d_noise_vars;
  a.llrs            = d_llrs;
  std::lock_guard<std::mutex> lock(mod->mtx);
  hipError_t                  e = hipSetDevice(mod->device);
  if (e == hipSuccess) {
    e = launch_demodulate(a, static_cast<hipStream_t>(stream));
  }
  return e == hipSuccess ? SRS_AMD_OK : hip_fail(e, "demodulate_kernel launch");
}

int srs_amd_scramble_bits_batch(srs_amd_modulator* mod, uint8_t* d_out, const uint8_t* d_in, uint32_t nof_bits,
                                uint32_t c_init, void* stream)
{
  if (mod == nullptr || d_out == nullptr) {
    return fail(SRS_AMD_EINVAL, "null argument");
  }
  if (nof_bits >= (1u << PRBS_NJUMP) - 1600u - 32u) {
    return fail(SRS_AMD_EINVAL, "sequence length %u too large", nof_bits);
  }
  prbs_args a{};
  a.in_bits  = d_in;
  a.out_bits = d_out;
  a.jump     = mod->d_jump;
  a.c_init   = c_init;
  a.length   = nof_bits;
  std::lock_guard<std::mutex> lock(mod->mtx);
  hipError_t                  e = hipSetDevice(mod->device);
  if (e == hipSuccess) {
    e = launch_scramble_bits(a, static_cast<hipStream_t>(stream));
  }
  return e == hipSuccess ? SRS_AMD_OK : hip_fail(e, "scramble_bits_kernel launch");
}

int srs_amd_descramble_llrs_batch(srs_amd_modulator* mod, int8_t* d_out, const int8_t* d_in, uint32_t nof_llrs,
                                  uint32_t c_init, void* stream)
{
  if (mod == nullptr || d_out == nullptr || (d_in == nullptr && nof_llrs > 0)) {
    return fail(SRS_AMD_EINVAL, "null argument");
  }
  if (nof_llrs >= (1u << PRBS_NJUMP) - 1600u - 32u) {
    return fail(SRS_AMD_EINVAL, "sequence length %u too large", nof_llrs);
  }
  prbs_args a{};
  a.in_llrs  = d_in;
  a.out_llrs = d_out;
  a.jump     = mod->d_jump;
  a.c_init   = c_init;
  a.length   = nof_llrs;
  std::lock_guard<std::mutex> lock(mod->mtx);
  hipError_t                  e = hipSetDevice(mod->device);
  if (e == hipSuccess) {
    e = launch_descramble_llrs(a, static_cast<hipStream_t>(stream));
  }
  return e == hipSuccess ? SRS_AMD_OK : hip_fail(e, "descramble_llrs_kernel launch");
}

// ---- synchronous host forms: stage, launch, copy back --------------------

int srs_amd_modulate(srs_amd_modulator* mod, float* symbols, const uint8_t* bits, uint32_t nof_symbols, int qm)
{
  int rc = check(mod, qm);
  if (rc != SRS_AMD_OK) {
    return rc;
  }
  if (symbols == nullptr || bits == nullptr) {
    return fail(SRS_AMD_EINVAL, "null argument");
  }
  const size_t nb = (static_cast<size_t>(nof_symbols) * bits_per_symbol(qm) + 7) / 8, ns = nof_symbols * 8ull;
  uint8_t*     base = nullptr;
  {
    std::lock_guard<std::mutex> lock(mod->mtx);
    hipError_t                  e = hipSetDevice(mod->device);
    if (e == hipSuccess) {
      e = mod->ensure(ns + nb + 16);
    }
    base = static_cast<uint8_t*>(mod->scratch);
    if (e == hipSuccess && nb) {
      e = hipMemcpyAsync(base + ns, bits, nb, hipMemcpyHostToDevice, mod->stream);
    }
    if (e != hipSuccess) {
      return hip_fail(e, "staging bits");
    }
  }
  rc = srs_amd_modulate_batch(mod, reinterpret_cast<float*>(base), base + ns, nof_symbols, qm, mod->stream);
  if (rc != SRS_AMD_OK) {
    return rc;
  }
  hipError_t e = ns ? hipMemcpyAsync(symbols, base, ns, hipMemcpyDeviceToHost, mod->stream) : hipSuccess;
  if (e == hipSuccess) {
    e = hipStreamSynchronize(mod->stream);
  }
  return e == hipSuccess ? SRS_AMD_OK : hip_fail(e, "modulate");
}

int srs_amd_demodulate_soft(srs_amd_modulator* mod,
                            int8_t*            llrs,
                            const float*       symbols,
                            const float*       noise_vars,
                            uint32_t           nof_symbols,
                            int                qm)
{
  int rc = check(mod, qm);
  if (rc != SRS_AMD_OK) {
    return rc;
  }
  if (llrs == nullptr || symbols == nullptr || noise_vars == nullptr) {
    return fail(SRS_AMD_EINVAL, "null argument");
  }
  const size_t ns = nof_symbols * 8ull, nn = nof_symbols * 4ull, nl = static_cast<size_t>(nof_symbols) * bits_per_symbol(qm);
  uint8_t*     base = nullptr;
  {
    std::lock_guard<std::mutex> lock(mod->mtx);
    hipError_t                  e = hipSetDevice(mod->device);
    if (e == hipSuccess) {
      e = mod->ensure(ns + nn + nl + 16);
    }
    base = static_cast<uint8_t*>(mod->scratch);
    if (e == hipSuccess && ns) {
      e = hipMemcpyAsync(base, symbols, ns, hipMemcpyHostToDevice, mod->stream);
    }
    if (e == hipSuccess && nn) {
      e = hipMemcpyAsync(base + ns, noise_vars, nn, hipMemcpyHostToDevice, mod->stream);
    }
    if (e != hipSuccess) {
      return hip_fail(e, "staging symbols");
    }
  }
  rc = srs_amd_demodulate_soft_batch(mod, reinterpret_cast<int8_t*>(base + ns + nn), reinterpret_cast<float*>(base),
                                     reinterpret_cast<float*>(base + ns), nof_symbols, qm, mod->stream);
  if (rc != SRS_AMD_OK) {
    return rc;
  }
  hipError_t e = nl ? hipMemcpyAsync(llrs, base + ns + nn, nl, hipMemcpyDeviceToHost, mod->stream) : hipSuccess;
  if (e == hipSuccess) {
    e = hipStreamSynchronize(mod->stream);
  }
  return e == hipSuccess ? SRS_AMD_OK : hip_fail(e, "demodulate");
}

int srs_amd_scramble_bits(srs_amd_modulator* mod, uint8_t* out, const uint8_t* in, uint32_t nof_bits, uint32_t c_init)
{
  if (mod == nullptr || out == nullptr) {
    return fail(SRS_AMD_EINVAL, "null argument");
  }
  const size_t nb   = (nof_bits + 7) / 8;
  uint8_t*     base = nullptr;
  {
    std::lock_guard<std::mutex> lock(mod->mtx);
    hipError_t                  e = hipSetDevice(mod->device);
    if (e == hipSuccess) {
      e = mod->ensure(2 * nb + 16);
    }
    base = static_cast<uint8_t*>(mod->scratch);
    if (e == hipSuccess && in && nb) {
      e = hipMemcpyAsync(base, in, nb, hipMemcpyHostToDevice, mod->stream);
    }
    if (e != hipSuccess) {
      return hip_fail(e, "staging bits");
    }
  }
  int rc = srs_amd_scramble_bits_batch(mod, base + nb, in ? base : nullptr, nof_bits, c_init, mod->stream);
  if (rc != SRS_AMD_OK) {
    return rc;
  }
  hipError_t e = nb ? hipMemcpyAsync(out, base + nb, nb, hipMemcpyDeviceToHost, mod->stream) : hipSuccess;
  if (e == hipSuccess) {
    e = hipStreamSynchronize(mod->stream);
  }
  return e == hipSuccess ? SRS_AMD_OK : hip_fail(e, "scramble");
}

int srs_amd_descramble_llrs(srs_amd_modulator* mod, int8_t* out, const int8_t* in, uint32_t nof_llrs, uint32_t c_init)
{
  if (mod == nullptr || out == nullptr || in == nullptr) {
    return fail(SRS_AMD_EINVAL, "null argument");
  }
  uint8_t* base = nullptr;
  {
    std::lock_guard<std::mutex> lock(mod->mtx);
    hipError_t                  e = hipSetDevice(mod->device);
    if (e == hipSuccess) {
      e = mod->ensure(2ull * nof_llrs + 16);
    }
    base = static_cast<uint8_t*>(mod->scratch);
    if (e == hipSuccess && nof_llrs) {
      e = hipMemcpyAsync(base, in, nof_llrs, hipMemcpyHostToDevice, mod->stream);
    }
    if (e != hipSuccess) {
      return hip_fail(e, "staging LLRs");
    }
  }
  int rc = srs_amd_descramble_llrs_batch(mod, reinterpret_cast<int8_t*>(base + nof_llrs),
                                         reinterpret_cast<int8_t*>(base), nof_llrs, c_init, mod->stream);
  if (rc != SRS_AMD_OK) {
    return rc;
  }
  hipError_t e = nof_llrs ? hipMemcpyAsync(out, base + nof_llrs, nof_llrs, hipMemcpyDeviceToHost, mod->stream)
                          : hipSuccess;
  if (e == hipSuccess) {
    e = hipStreamSynchronize(mod->stream);
  }
  return e == hipSuccess ? SRS_AMD_OK : hip_fail(e, "descramble");
}

} // extern "C"

demodulate_args srs_amd::demodulate_args_for(const srs_amd_modulator* mod, int qm, uint32_t nof_symbols)
{
  demodulate_args a{};
  a.nof_symbols      = nof_symbols;
  a.qm               = qm;
  const uint32_t blk = avx2_block(qm);
  a.block_end        = blk ? (nof_symbols / blk) * blk : 0;
  a.qam16_scale      = mod->qam16_scale;
  if (qm == 6) {
    for (int k = 0; k < 3; ++k) {
      a.tab[k] = mod->tab64[k];
    }
  } else if (qm == 8) {
    for (int k = 0; k < 4; ++k) {
      a.tab[k] = mod->tab256[k];
    }
  }
  return a;
}

uint32_t srs_amd::demap_symbol_bounds(int qm, const uint32_t* sym_counts, uint32_t* sym_lo, uint32_t* simd_hi)
{
  // one demapper call per OFDM symbol: SIMD blocks of avx2_block(qm) symbols from each symbol's start
  const uint32_t blk = avx2_block(qm);
  uint32_t       s0  = 0;
  for (int l = 0; l < 14; ++l) {
    const uint32_t n = sym_counts[l];
    sym_lo[l]        = s0;
    simd_hi[l]       = s0 + (blk ? (n / blk) * blk : 0);
    s0 += n;
  }
  return s0;
}

int srs_amd::make_demap_item(srs_amd_modulator* mod, int qm, int8_t* d_llrs, const float* d_symbols,
                             const float* d_noise_vars, uint32_t grid_symbols, const uint32_t* sym_counts,
                             const uint32_t* d_jump, uint32_t c_init, demap_item& out)
{
  int rc = check(mod, qm);
  if (rc != SRS_AMD_OK) {
    return rc;
  }
  out              = demap_item{};
  out.a            = demodulate_args_for(mod, qm, grid_symbols);
  out.a.symbols    = d_symbols;
  out.a.noise_vars = d_noise_vars;
  out.d.llrs         = d_llrs;
  out.d.jump         = d_jump;
  out.d.grid_symbols = grid_symbols;
  out.d.c_init       = c_init;
  if (demap_symbol_bounds(qm, sym_counts, out.d.sym_lo, out.d.simd_hi) != grid_symbols) {
    return fail(SRS_AMD_EINVAL, "per-symbol counts do not add up to the grid symbols (%u)", grid_symbols);
  }
  return SRS_AMD_OK;
}

int srs_amd::demap_descramble_batch(srs_amd_modulator* mod, int qm, int8_t* d_llrs, uint64_t llr_stride,
                                    const float* d_symbols, const float* d_noise_vars, uint32_t grid_symbols,
                                    const uint32_t* sym_counts, uint32_t nof_grids, const uint32_t* d_jump,
                                    uint32_t c_init, void* stream)
{
  int rc = check(mod, qm);
  if (rc != SRS_AMD_OK) {
    return rc;
  }
  demodulate_args a = demodulate_args_for(mod, qm, grid_symbols);
  a.symbols         = d_symbols;
  a.noise_vars      = d_noise_vars;
  demap_descramble_args d{};
  d.llrs         = d_llrs;
  d.jump         = d_jump;
  d.llr_stride   = llr_stride;
  d.grid_symbols = grid_symbols;
  d.c_init       = c_init;
  const uint32_t s0 = demap_symbol_bounds(qm, sym_counts, d.sym_lo, d.simd_hi);
  if (s0 != grid_symbols) {
    return fail(SRS_AMD_EINVAL, "per-symbol counts (%u) do not add up to the grid symbols (%u)", s0, grid_symbols);
  }
  std::lock_guard<std::mutex> lock(mod->mtx);
  hipError_t                  e = hipSetDevice(mod->device);
  if (e == hipSuccess) {
    e = launch_demap_descramble(a, d, nof_grids, static_cast<hipStream_t>(stream));
  }
  return e == hipSuccess ? SRS_AMD_OK : hip_fail(e, "demap_descramble_kernel launch");
}
