// pdsch_modulator.hip -- MI355X PDSCH modulator and PDSCH DM-RS kernels.
//
// pdsch_map_kernel fuses what the reference does in four passes over a
// codeword (pdsch_modulator_impl.cpp:94-115): Gold-sequence scrambling,
// modulation to integer constellation points (ci8_t, modulation_mapper_lut_impl.cpp:37-67),
// layer mapping + precoding (channel_precoder_avx2.cpp:214-330) and RE mapping
// around the reserved / DM-RS REs (resource_grid_mapper_impl.cpp:341-460).
// One workgroup per (codeword, OFDM symbol, 256 subcarriers): thread t owns
// subcarrier k; its data-RE index j comes from the per-PRB table (prefix <<
// 12 | 12-bit mask, built once per plan on the host). The workgroup's data
// REs are contiguous in the codeword, so it scrambles exactly its bit range
// into LDS (four Gold words per thread: one jump-ahead, then word-parallel steps), then
// every thread gathers its L x Qm bits, builds the integer points and writes
// the precoded cbf16 RE of every port (coalesced 4-byte stores).
//
// dmrs_pdsch_kernel: one thread per (DM-RS symbol, RE of an allocated CRB), several grids per
// workgroup; the workgroup's Gold words computed once into LDS, CDM codes w_f / w_t
// (dmrs_helper.cpp:34-56), precoding with the same SIMD complex product, coalesced stores.
//
// Both are HBM-store bound: 4 bytes per RE and port written, Qm * L / 8 bytes
// per RE read.
#include <hip/hip_runtime.h>

#include "bf16_device.h"

#include "gold_sequence.h"
#include "pdsch_modulator_args.h"

#pragma clang fp contract(off)

namespace srs_amd {
namespace {

// x * w as _mm256_fmaddsub_ps(x, w.re, swap(x) * w.im).
__device__ __forceinline__ float2 cmul_simd(float2 x, float wr, float wi)
{
  return make_float2(__builtin_fmaf(x.x, wr, -(x.y * wi)), __builtin_fmaf(x.y, wr, x.x * wi));
}

// ps_to_cbf16: round half to even on the bit pattern.
__device__ __forceinline__ uint32_t to_bf16(float f)
{
  uint32_t u = __float_as_uint(f);
  u += 0x7fffu + ((u >> 16) & 1u);
  return u >> 16;
}

__device__ __forceinline__ uint32_t pack_cbf16(float2 v)
{
  return cbf16_pack(v.x, v.y); // == to_bf16(v.x) | to_bf16(v.y) << 16 (bf16_device.h)
}

// Integer constellation point of a Qm-bit index (modulation_mapper_lut_impl.cpp:44-56).
__device__ __forceinline__ float2 qam_point(uint32_t idx, int qm)
{
  float off = -1.0f, re = 0.0f, im = 0.0f;
  for (int j = 0; j < qm / 2; ++j) {
    re += off;
    im += off;
    off *= 2.0f;
    re = ((idx >> (2 * j + 1)) & 1u) ? re : -re;
    im = ((idx >> (2 * j)) & 1u) ? im : -im;
  }
  return make_float2(re, im);
}

// Data REs of symbol row `row` before subcarrier k (k may be nof_subc).
__device__ __forceinline__ uint32_t data_re_before(const uint32_t* row, uint32_t nof_prb, uint32_t k)
{
  const uint32_t prb = k / PDSCH_NRE;
  if (prb >= nof_prb) {
    const uint32_t e = row[nof_prb - 1];
    return (e >> 12) + __builtin_popcount(e & 0xfffu);
  }
  const uint32_t e = row[prb];
  return (e >> 12) + __builtin_popcount(e & ((1u << (k % PDSCH_NRE)) - 1u));
}

// Stream bits 32w .. 32w+31 of a packed MSB-first codeword, bit b at bit b (0 past the end).
__device__ __forceinline__ uint32_t codeword_word(const uint8_t* cw, uint32_t nof_bytes, uint32_t w)
{
  uint32_t v = 0;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const uint32_t p = 4 * w + q;
    const uint32_t b = p < nof_bytes ? cw[p] : 0u;
    v |= (__builtin_bitreverse32(b) >> 24) << (8 * q);
  }
  return v;
}

constexpr int MAX_WORDS = PDSCH_THREADS + 2; // 256 REs x 4 layers x 8 bits / 32 + 2

// The argument block of this workgroup: the launch's own (batch form) or that of PDU blockIdx.z (slot form).
template <bool MULTI, typename T>
__device__ __forceinline__ const T& item_of(const T& own, const T* items)
{
  if constexpr (MULTI) {
    return items[blockIdx.z];
  } else {
    return own;
  }
}

template <bool MULTI>
__global__ __launch_bounds__(PDSCH_THREADS) void pdsch_map_kernel(pdsch_map_args own, const pdsch_map_args* items)
{
  const pdsch_map_args& a = item_of<MULTI>(own, items);
  if (MULTI && (blockIdx.x >= a.nof_tiles || blockIdx.y >= a.nof_symbols)) {
    return;
  }
  __shared__ uint32_t scrambled[MAX_WORDS];
  __shared__ float2   s_qam[256]; // constellation point of every Qm-bit index (qm >= 2)

  const uint32_t  l   = a.first_symbol + blockIdx.y;
  const uint32_t  k0  = a.first_subc + blockIdx.x * PDSCH_THREADS;
  const uint32_t  k   = k0 + threadIdx.x;
  const uint32_t* row = a.re_table + l * a.nof_prb;
  const uint32_t  kend = min(k0 + PDSCH_THREADS, a.nof_subc);

  const uint32_t bits_per_re = static_cast<uint32_t>(a.nof_layers) * (a.qm < 2 ? 1u : static_cast<uint32_t>(a.qm));
  const uint32_t j_lo        = data_re_before(row, a.nof_prb, k0);
  const uint32_t j_hi        = data_re_before(row, a.nof_prb, kend);
  if (j_hi == j_lo) {
    return; // no data RE in this block (uniform over the workgroup)
  }
  const uint32_t w_lo = j_lo * bits_per_re / 32;
  const uint32_t w_hi = (j_hi * bits_per_re + 31) / 32;

  const uint8_t* cw        = a.codewords + static_cast<uint64_t>(blockIdx.z) * a.cw_stride;
  const uint32_t nof_bytes = (a.nof_bits + 7) / 8;
  if (a.qm >= 2 && threadIdx.x < (1u << a.qm)) {
    s_qam[threadIdx.x] = qam_point(threadIdx.x, a.qm);
  }
  // the block's codeword words XOR the plan's scrambling words (one word per thread)
  const uint32_t nw = w_hi - w_lo;
  for (uint32_t q = threadIdx.x; q < nw; q += PDSCH_THREADS) {
    scrambled[q] = codeword_word(cw, nof_bytes, w_lo + q) ^ a.scr[w_lo + q];
  }
  __syncthreads();

  if (k >= kend) {
    return;
  }
  const uint32_t e   = row[k / PDSCH_NRE];
  const uint32_t bit = k % PDSCH_NRE;
  if (((e >> bit) & 1u) == 0) {
    return;
  }
  const uint32_t j = (e >> 12) + __builtin_popcount(e & ((1u << bit) - 1u));
  if ((j + 1) * bits_per_re > a.nof_bits) {
    return; // past a shorter codeword: the reference's mapper stops when its symbol buffer runs empty
  }

  const int bps = a.qm < 2 ? 1 : a.qm;
  float2    x[4];
#pragma unroll
  for (int v = 0; v < 4; ++v) {
    if (v < a.nof_layers) {
      const uint32_t s   = j * a.nof_layers + v; // symbol index in the codeword
      const uint32_t o   = s * bps - w_lo * 32;  // bit offset in LDS
      const uint64_t win = static_cast<uint64_t>(scrambled[o / 32]) |
                           (static_cast<uint64_t>(scrambled[min(o / 32 + 1, static_cast<uint32_t>(MAX_WORDS - 1))])
                            << 32);
      const uint32_t seq = static_cast<uint32_t>(win >> (o % 32)) & ((1u << bps) - 1u); // bit i = i-th bit
      const uint32_t idx = __builtin_bitreverse32(seq) >> (32 - bps);                    // MSB-first index
      if (a.qm >= 2) {
        x[v] = s_qam[idx];
      } else {
        const float b = idx ? -1.0f : 1.0f;
        x[v]          = make_float2((a.qm == 0 && (s & 1u)) ? -b : b, b);
      }
    }
  }

  uint32_t* grid = a.grids + static_cast<uint64_t>(blockIdx.z) * a.grid_stride + l * a.nof_subc + k;
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    if (p < a.nof_ports) {
      float2 y = cmul_simd(x[0], a.w[0][p][0], a.w[0][p][1]);
#pragma unroll
      for (int v = 1; v < 4; ++v) {
        if (v < a.nof_layers) {
          const float2 t = cmul_simd(x[v], a.w[v][p][0], a.w[v][p][1]);
          y.x            = y.x + t.x;
          y.y            = y.y + t.y;
        }
      }
      grid[static_cast<uint64_t>(p) * a.port_stride] = pack_cbf16(y);
    }
  }
}

// DM-RS: one thread per resource element of an allocated CRB (12 per CRB, consecutive threads on consecutive
// subcarriers: coalesced stores), DMRS_GRIDS_PER_WG grids per workgroup (batch form: every grid of a launch
// carries the same sequence, so the Gold words are computed once per workgroup and written to several grids).
// The sequence words of the workgroup's CRBs are computed cooperatively (one jump per word, into LDS); a
// workgroup whose CRBs are spread over more than DMRS_MAX_WORDS words jumps per thread instead.
constexpr int DMRS_THREADS      = 256;
constexpr int DMRS_GRIDS_PER_WG = 4;
constexpr int DMRS_MAX_WORDS    = 64;

template <bool MULTI>
__global__ __launch_bounds__(DMRS_THREADS) void dmrs_pdsch_kernel(dmrs_pdsch_args own, const dmrs_pdsch_args* items,
                                                                 uint32_t nof_grids)
{
  const dmrs_pdsch_args& a = item_of<MULTI>(own, items);
  __shared__ uint32_t    s_words[DMRS_MAX_WORDS];
  const uint32_t         e0 = blockIdx.x * DMRS_THREADS;
  if (e0 >= a.nof_crb * PDSCH_NRE || (MULTI && blockIdx.y >= a.nof_dmrs_symbols)) {
    return; // uniform over the workgroup
  }
  const int      nd = a.type2 ? 4 : 6;
  const uint32_t l  = a.symbol[blockIdx.y];
  // sequence words covering the workgroup's CRBs (dmrs_helper.cpp:70-90: bits 2 nd (crb - ref) ..)
  const uint32_t i_lo   = e0 / PDSCH_NRE;
  const uint32_t i_hi   = min(a.nof_crb, (e0 + DMRS_THREADS + PDSCH_NRE - 1) / PDSCH_NRE) - 1;
  const uint32_t w_lo   = 2u * nd * (a.crbs[i_lo] - a.reference_point_k_rb) / 32;
  const uint32_t w_hi   = (2u * nd * (a.crbs[i_hi] - a.reference_point_k_rb) + 2u * nd - 1) / 32;
  const bool     shared = w_hi - w_lo < DMRS_MAX_WORDS;
  if (shared && threadIdx.x <= w_hi - w_lo) {
    uint32_t x1, x2;
    gold_state(a.jump, a.c_init[blockIdx.y], 32 * (w_lo + threadIdx.x), x1, x2);
    s_words[threadIdx.x] = gold_next32(x1, x2);
  }
  __syncthreads();
  const uint32_t e = e0 + threadIdx.x;
  const uint32_t i = e / PDSCH_NRE;
  const uint32_t r = e - i * PDSCH_NRE;
  if (i >= a.nof_crb) {
    return;
  }
  // resource element r of the CRB: CDM group g, sequence index t within the RB
  const uint32_t g = a.type2 ? (r % 6) / 2 : (r & 1u);
  const uint32_t t = a.type2 ? (r & 1u) + 2 * (r / 6) : (r >> 1);
  if (2 * static_cast<int>(g) >= a.nof_layers) {
    return; // no port of this PDU in CDM group g
  }
  const uint32_t crb = a.crbs[i];
  const uint32_t b   = 2u * nd * (crb - a.reference_point_k_rb) + 2 * t;
  uint32_t       word;
  if (shared) {
    word = s_words[b / 32 - w_lo];
  } else {
    uint32_t x1, x2;
    gold_state(a.jump, a.c_init[blockIdx.y], 32 * (b / 32), x1, x2);
    word = gold_next32(x1, x2);
  }
  const uint32_t bits = word >> (b % 32);
  const float    amp  = a.amplitude;
  const float2   base = make_float2((bits & 1u) ? -amp : amp, (bits & 2u) ? -amp : amp);
  // ports 2g and 2g+1 of the CDM group: w_f = -1 on odd sequence indices for the odd port, w_t = +1 for every
  // port < 4 (type 1) / < 6 (type 2) and every DM-RS symbol (dmrs_helper.cpp:34-56)
  const float2   seq1 = (t & 1u) ? make_float2(-base.x, -base.y) : base;
  const uint32_t sc   = crb * PDSCH_NRE + r;
  const uint32_t z0   = MULTI ? 0u : blockIdx.z * DMRS_GRIDS_PER_WG;
  const uint32_t z1   = MULTI ? 1u : min(nof_grids, z0 + DMRS_GRIDS_PER_WG);
  uint32_t       y[4];
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    if (p < a.nof_ports) {
      float2 v = cmul_simd(base, a.w[2 * g][p][0], a.w[2 * g][p][1]);
      if (2 * static_cast<int>(g) + 1 < a.nof_layers) {
        const float2 u = cmul_simd(seq1, a.w[2 * g + 1][p][0], a.w[2 * g + 1][p][1]);
        v.x            = v.x + u.x;
        v.y            = v.y + u.y;
      }
      y[p] = pack_cbf16(v);
    }
  }
  for (uint32_t z = z0; z < z1; ++z) {
    uint32_t* grid = a.grids + static_cast<uint64_t>(MULTI ? blockIdx.z : z) * a.grid_stride +
                     l * (a.port_stride / 14) + sc;
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      if (p < a.nof_ports) {
        grid[static_cast<uint64_t>(p) * a.port_stride] = y[p];
      }
    }
  }
}

} // namespace

hipError_t launch_pdsch_map(const pdsch_map_args& a, uint32_t nof_symbols, uint32_t span_subc, uint32_t nof_cws,
                            hipStream_t stream)
{
  if (nof_symbols == 0 || span_subc == 0 || nof_cws == 0) {
    return hipSuccess;
  }
  const dim3 grid((span_subc + PDSCH_THREADS - 1) / PDSCH_THREADS, nof_symbols, nof_cws);
  hipLaunchKernelGGL(pdsch_map_kernel<false>, grid, dim3(PDSCH_THREADS), 0, stream, a, nullptr);
  return hipGetLastError();
}

hipError_t launch_dmrs_pdsch(const dmrs_pdsch_args& a, uint32_t nof_grids, hipStream_t stream)
{
  if (a.nof_crb == 0 || a.nof_dmrs_symbols == 0 || nof_grids == 0) {
    return hipSuccess;
  }
  const dim3 grid((a.nof_crb * PDSCH_NRE + DMRS_THREADS - 1) / DMRS_THREADS, a.nof_dmrs_symbols,
                  (nof_grids + DMRS_GRIDS_PER_WG - 1) / DMRS_GRIDS_PER_WG);
  hipLaunchKernelGGL(dmrs_pdsch_kernel<false>, grid, dim3(DMRS_THREADS), 0, stream, a, nullptr, nof_grids);
  return hipGetLastError();
}

hipError_t launch_pdsch_map_items(const pdsch_map_args* items, uint32_t count, uint32_t max_tiles,
                                  uint32_t max_symbols, hipStream_t stream)
{
  if (count == 0 || max_tiles == 0 || max_symbols == 0) {
    return hipSuccess;
  }
  hipLaunchKernelGGL(pdsch_map_kernel<true>, dim3(max_tiles, max_symbols, count), dim3(PDSCH_THREADS), 0, stream,
                     pdsch_map_args{}, items);
  return hipGetLastError();
}

hipError_t launch_dmrs_pdsch_items(const dmrs_pdsch_args* items, uint32_t count, uint32_t max_crb_blocks,
                                   uint32_t max_symbols, hipStream_t stream)
{
  if (count == 0 || max_crb_blocks == 0 || max_symbols == 0) {
    return hipSuccess;
  }
  hipLaunchKernelGGL(dmrs_pdsch_kernel<true>, dim3(max_crb_blocks, max_symbols, count), dim3(DMRS_THREADS), 0,
                     stream, dmrs_pdsch_args{}, items, 1u);
  return hipGetLastError();
}

// PT-RS (ptrs_pdsch_generator_impl.cpp:30-130): one thread per (PT-RS PRB, symbol).  The reference generates the
// DM-RS-like sequence of the first DM-RS symbol from the pattern's first PRB and picks every rb_stride-th PRB's
// re_offset / 2-th element; the same values go on every PT-RS symbol, precoded per PRG (the generic mapper path,
// resource_grid_mapper_impl.cpp:258-286, PRG = CRB / prg_size).
__global__ __launch_bounds__(64) void ptrs_pdsch_kernel(const ptrs_pdsch_args* items)
{
  const ptrs_pdsch_args& a = items[blockIdx.z];
  const uint32_t         i = blockIdx.x * 64 + threadIdx.x;
  const uint32_t         l = blockIdx.y;
  if (i >= a.nof_prb || ((a.symbol_mask >> l) & 1u) == 0) {
    return;
  }
  const uint32_t b    = a.bit0 + i * a.bit_step; // even: both bits in one word
  const uint32_t bits = gold_word(a.jump, a.c_init, 32 * (b / 32)) >> (b % 32);
  const float2   x    = make_float2((bits & 1u) ? -a.amplitude : a.amplitude, (bits & 2u) ? -a.amplitude : a.amplitude);
  const uint32_t crb  = a.rb_begin + i * a.rb_stride;
  const float*   w    = a.w + 2 * (crb / a.prg_size) * a.nof_ports;
  uint32_t*      re   = a.grid + static_cast<uint64_t>(l) * a.nof_subc + crb * PDSCH_NRE + a.k;
  for (uint32_t p = 0; p < a.nof_ports; ++p) {
    re[static_cast<uint64_t>(p) * a.port_stride] = pack_cbf16(cmul_simd(x, w[2 * p], w[2 * p + 1]));
  }
}

hipError_t launch_ptrs_pdsch_items(const ptrs_pdsch_args* items, uint32_t count, uint32_t max_prb, hipStream_t stream)
{
  if (count == 0 || max_prb == 0) {
    return hipSuccess;
  }
  hipLaunchKernelGGL(ptrs_pdsch_kernel, dim3((max_prb + 63) / 64, PDSCH_NSYMB, count), dim3(64), 0, stream, items);
  return hipGetLastError();
}

} // namespace srs_amd
