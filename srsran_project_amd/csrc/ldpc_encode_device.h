// ldpc_encode_device.h -- the bit-sliced LDPC encoder core (TS 38.212 Section 5.3.2) as device code shared by
// ldpc_encode_bits_kernel (ldpc_encoder.hip) and the fused PDSCH codeblock kernel (pdsch_encoder.hip).
//
// The codeword lives in LDS as ONE linear bit vector (bit i = lifted column i / Z, row i % Z, at word
// i / 32, bit i % 32), so unpacking the MSB-first message and packing the output are word copies with a
// bit reversal.  A lane computes 32 rows of a parity column at once: each edge is a 32-row window of the
// variable column at the edge's cyclic shift (two LDS words and a funnel shift, a second pair where
// the window wraps), XOR-ed into the row's accumulator.  The base-graph structure the solve relies on is
// checked on the host (build_encode_params, ldpc_codec_api.cpp): see ldpc_encoder.hip.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace srs_amd {

__device__ __forceinline__ uint32_t lds_bits32(const uint32_t* W, uint32_t off)
{
  const uint32_t w = off >> 5;
  return __builtin_amdgcn_alignbit(W[w + 1], W[w], off & 31u);
}

// Rows x0 .. x0+31 of the column starting at bit cz, cyclically shifted by s: row x takes the column
// bit (x + s) mod Z (x0 < Z, s < Z; rows >= Z are don't-care).  For Z < 32 the one wrap covers every row < Z.
__device__ __forceinline__ uint32_t cyc32(const uint32_t* W, uint32_t cz, uint32_t Z, uint32_t x0, uint32_t s)
{
  uint32_t pos = x0 + s;
  pos -= pos >= Z ? Z : 0u;
  uint32_t v = lds_bits32(W, cz + pos);
  if (pos + 32 > Z) {
    const uint32_t n1 = Z - pos; // 1 .. 31
    v = (v & ((1u << n1) - 1u)) | (lds_bits32(W, cz) << n1);
  }
  return v;
}

// ORs the low n bits of v into the (zeroed) bits off .. off+n-1.
__device__ __forceinline__ void lds_or_bits(uint32_t* W, uint32_t off, uint32_t v, uint32_t n)
{
  v &= n < 32 ? (1u << n) - 1u : 0xffffffffu;
  const uint32_t w = off >> 5, sh = off & 31u;
  atomicOr(&W[w], v << sh);
  if (sh != 0) {
    atomicOr(&W[w + 1], v >> (32 - sh));
  }
}

// LDS words of the encoder state: codeword bits of K + M_eff columns (+2 guard words), four lambda
// columns, the lambda sum column (+2).
__host__ __device__ constexpr uint32_t enc_bits_cw_words(uint32_t K, uint32_t M_eff, uint32_t Z)
{
  return ((K + M_eff) * Z + 31) / 32 + 2;
}
__host__ __device__ constexpr uint32_t enc_bits_lds_words(uint32_t K, uint32_t M_eff, uint32_t Z)
{
  return enc_bits_cw_words(K, M_eff, Z) + 4 * ((Z + 31) / 32) + (Z + 31) / 32 + 2;
}

// Parity of one codeblock, NT threads (thread j).  On entry: cw holds the message bits [0, K Z) and zeros up to
// enc_bits_cw_words, ls[0, nq + 2) is zero, and a barrier has passed.  On exit (after a barrier) cw holds the
// high-rate parity columns and the extension columns K + 4 .. K + M_eff - 1.  row_start: the base graph's
// check-row edge offsets; edges: its lifted edges (var * Z | shift << 16).
template <int NT>
__device__ __forceinline__ void encode_bits_parity(uint32_t*       cw,
                                                   uint32_t*       lam,
                                                   uint32_t*       ls,
                                                   const uint32_t* edges,
                                                   const int32_t*  row_start,
                                                   int             bg,
                                                   uint32_t        K,
                                                   uint32_t        Z,
                                                   uint32_t        M_eff,
                                                   int32_t         p0_shift,
                                                   const int32_t (&core_a)[3],
                                                   uint32_t        j)
{
  const uint32_t kz = K * Z;
  const uint32_t nq = (Z + 31) / 32;
  // 1. Systematic part of the high-rate rows, 32 rows per task.
  for (uint32_t task = j; task < 4 * nq; task += NT) {
    const uint32_t r = task / nq, x0 = 32 * (task - r * nq);
    uint32_t       acc = 0;
    for (int e = row_start[r]; e < row_start[r + 1]; ++e) {
      const uint32_t ed   = edges[e];
      const uint32_t base = ed & 0xffffu;
      if (base >= kz) {
        break; // edges are sorted by column
      }
      acc ^= cyc32(cw, base, Z, x0, ed >> 16);
    }
    lam[task] = acc;
  }
  __syncthreads();
  for (uint32_t q = j; q < nq; q += NT) {
    const uint32_t n = min(32u, Z - 32 * q);
    const uint32_t v = lam[q] ^ lam[nq + q] ^ lam[2 * nq + q] ^ lam[3 * nq + q];
    ls[q]            = n < 32 ? v & ((1u << n) - 1u) : v;
  }
  __syncthreads();

  // 2. p0 = P^-s (lambda sum): row x takes the sum's row (x - s) mod Z.
  const uint32_t sh0 = (Z - static_cast<uint32_t>(p0_shift) % Z) % Z;
  for (uint32_t q = j; q < nq; q += NT) {
    lds_or_bits(cw, kz + 32 * q, cyc32(ls, 0, Z, 32 * q, sh0), min(32u, Z - 32 * q));
  }
  __syncthreads();

  // 3. p1 .. p3 (double diagonal).
  for (uint32_t q = j; q < nq; q += NT) {
    const uint32_t x0 = 32 * q, n = min(32u, Z - x0);
    auto           at = [&](int s) { return cyc32(cw, kz, Z, x0, static_cast<uint32_t>(s)); };
    uint32_t       p1, p2, p3;
    p1 = lam[q] ^ at(core_a[0]);
    if (bg == 1) {
      p2 = lam[nq + q] ^ at(core_a[1]) ^ p1;
      p3 = lam[2 * nq + q] ^ p2;
    } else {
      p2 = lam[nq + q] ^ p1;
      p3 = lam[2 * nq + q] ^ at(core_a[2]) ^ p2;
    }
    lds_or_bits(cw, kz + Z + x0, p1, n);
    lds_or_bits(cw, kz + 2 * Z + x0, p2, n);
    lds_or_bits(cw, kz + 3 * Z + x0, p3, n);
  }
  __syncthreads();

  // 4. Extension rows: independent single-parity rows over columns < K + 4.
  const uint32_t hz = kz + 4 * Z;
  for (uint32_t task = j; task < (M_eff - 4) * nq; task += NT) {
    const uint32_t rr = task / nq, r = 4 + rr, x0 = 32 * (task - rr * nq);
    uint32_t       acc = 0;
    for (int e = row_start[r]; e < row_start[r + 1]; ++e) {
      const uint32_t ed   = edges[e];
      const uint32_t base = ed & 0xffffu;
      if (base >= hz) {
        break;
      }
      acc ^= cyc32(cw, base, Z, x0, ed >> 16);
    }
    lds_or_bits(cw, (K + r) * Z + x0, acc, min(32u, Z - x0));
  }
  __syncthreads();
}

} // namespace srs_amd
