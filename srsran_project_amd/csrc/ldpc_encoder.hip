// ldpc_encoder.hip -- MI355X LDPC encoder (TS 38.212 Section 5.3.2), batched.
//
// Reference behaviour: lib/phy/upper/channel_coding/ldpc/ldpc_encoder_impl.cpp:44-80
// (encode), ldpc_encoder_generic.cpp (systematic preprocessing, high-rate
// region, extension region) -- every reference encoder returns the same
// codeword: the unique one satisfying H * c = 0 for the lifted base graph,
// with the first 2Z systematic bits removed (write_codeblock).
//
// Work decomposition: one workgroup per codeblock, lane j < Z owns lifted row
// j of every base-graph check row; the codeword is kept in LDS one bit per
// byte (BG1 Z=384: 26 KiB) and each edge is an LDS byte gather at the
// edge's cyclic shift.  Base-graph structure (checked on the host when the
// launch parameters are built, ldpc_encoder_api.cpp):
//   * high-rate region (rows 0..3, parity columns K_bg..K_bg+3): column K_bg
//     appears in three of the four rows with shifts a, b, c of which two are
//     equal, the other three parity columns form a double diagonal with shift 0.
//     Summing the four rows cancels p1..p3 and the two equal shifts, so
//     p0 = P^-s (lambda0 + lambda1 + lambda2 + lambda3), s the odd shift out,
//     lambda_r the systematic part of row r; p1..p3 then follow row by row.
//   * extension region (rows 4..M-1): row r is an identity on column K_bg + r
//     and otherwise touches only columns < K_bg + 4: p_(K_bg+r) is the XOR of
//     that row's other gathers -- all rows independent.  Only the rows whose
//     parity columns the rate matcher will read are computed (M_eff), and
//     only the leading pack_bits of the codeword are written: a high-rate
//     PDSCH codeblock (R = 0.93) needs 2 of BG1's 42 extension rows, and the
//     LDS footprint shrinks with them.
#include <hip/hip_runtime.h>

#include "ldpc_codec_args.h"
#include "ldpc_encode_device.h"

namespace srs_amd {


__device__ __forceinline__ uint32_t spread_nibble(uint32_t n)
{
  // bit k of n -> byte k (LSB-first)
  return (n * 0x00204081u) & 0x01010101u;
}

__global__ __launch_bounds__(MAX_LIFTING_SIZE) void ldpc_encode_kernel(encode_args a)
{
  extern __shared__ uint8_t lds[];
  const int Z    = a.Z;
  const int j    = threadIdx.x;
  uint8_t*  cw   = lds;                                    // [N_full][Z] bits, one per byte
  uint8_t*  lsum = lds + ((a.K + a.M_eff) * Z + 15) / 16 * 16; // [Z]
  const int kz   = a.K * Z;

  for (uint32_t cb = blockIdx.x; cb < a.nof_cbs; cb += gridDim.x) {
    // 1. Unpack the message (MSB-first) into LDS, 8 bits per thread-step.
    const uint8_t* msg    = a.msgs + static_cast<size_t>(cb) * a.msg_stride;
    const int      nbytes = (kz + 7) / 8;
    for (int q = j; q < nbytes; q += blockDim.x) {
      const uint32_t x  = __builtin_bitreverse32(static_cast<uint32_t>(msg[q])) >> 24;
      uint32_t*      d  = reinterpret_cast<uint32_t*>(cw + 8 * q);
      d[0]              = spread_nibble(x & 15u);
      d[1]              = spread_nibble(x >> 4);
    }
    __syncthreads();

    // 2. Systematic part of the high-rate rows.
    uint32_t lam[4] = {0, 0, 0, 0};
    if (j < Z) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        uint32_t acc = 0;
        for (int e = a.row_start[r]; e < a.row_start[r + 1]; ++e) {
          const uint32_t ed   = a.edges[e];
          const int      base = static_cast<int>(ed & 0xffffu);
          if (base >= kz) {
            break; // edges are sorted by column
          }
          int idx = j + static_cast<int>(ed >> 16);
          idx -= idx >= Z ? Z : 0;
          acc ^= cw[base + idx];
        }
        lam[r] = acc;
      }
      lsum[j] = static_cast<uint8_t>(lam[0] ^ lam[1] ^ lam[2] ^ lam[3]);
    }
    __syncthreads();

    // 3. First parity column: p0[j] = sum[(j - s) mod Z].
    if (j < Z) {
      int idx = j - a.p0_shift;
      idx += idx < 0 ? Z : 0;
      cw[kz + j] = lsum[idx];
    }
    __syncthreads();

    // 4. The other three high-rate parity columns (row by row, double diagonal).
    if (j < Z) {
      const uint8_t* p0 = cw + kz;
      auto           at = [&](int s) {
        int idx = j + s;
        idx -= idx >= Z ? Z : 0;
        return static_cast<uint32_t>(p0[idx]);
      };
      uint32_t p1, p2, p3;
      p1 = lam[0] ^ at(a.core_a[0]);
      if (a.bg == 1) {
        p2 = lam[1] ^ at(a.core_a[1]) ^ p1;
        p3 = lam[2] ^ p2;
      } else {
        p2 = lam[1] ^ p1;
        p3 = lam[2] ^ at(a.core_a[2]) ^ p2;
      }
      cw[kz + Z + j]     = static_cast<uint8_t>(p1);
      cw[kz + 2 * Z + j] = static_cast<uint8_t>(p2);
      cw[kz + 3 * Z + j] = static_cast<uint8_t>(p3);
    }
    __syncthreads();

    // 5. Extension region: independent single-parity rows.
    if (j < Z) {
      const int hz = kz + 4 * Z;
      for (int r = 4; r < a.M_eff; ++r) {
        uint32_t acc = 0;
        for (int e = a.row_start[r]; e < a.row_start[r + 1]; ++e) {
          const uint32_t ed   = a.edges[e];
          const int      base = static_cast<int>(ed & 0xffffu);
          if (base >= hz) {
            break;
          }
          int idx = j + static_cast<int>(ed >> 16);
          idx -= idx >= Z ? Z : 0;
          acc ^= cw[base + idx];
        }
        cw[(a.K + r) * Z + j] = static_cast<uint8_t>(acc);
      }
    }
    __syncthreads();

    // 6. Pack the shortened codeword (drop the first 2Z systematic bits), MSB-first.
    uint8_t*  out   = a.cws + static_cast<size_t>(cb) * a.cw_stride;
    const int nbits = a.pack_bits;
    const int nb    = (nbits + 7) / 8;
    for (int q = j; q < nb; q += blockDim.x) {
      uint32_t byte = 0;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int pos = 8 * q + k;
        const uint32_t bit = pos < nbits ? cw[2 * Z + pos] : 0u;
        byte |= bit << (7 - k);
      }
      out[q] = static_cast<uint8_t>(byte);
    }
    __syncthreads();
  }
}

// ---- bit-sliced encoder (ldpc_encode_device.h) ----------------------------------------------------------
// One wave per codeblock: the four high-rate rows of BG1 Z = 384 are 48 lane tasks.
constexpr int ENC_BITS_THREADS = 64;
constexpr uint32_t ENC_MSG_UNROLL = 5; // 1,056-byte BG1 Z = 384 message: 264 words, five per lane

__global__ __launch_bounds__(ENC_BITS_THREADS) void ldpc_encode_bits_kernel(encode_args a)
{
  extern __shared__ uint32_t lw[];
  const uint32_t K = static_cast<uint32_t>(a.K);
  const uint32_t j = threadIdx.x;

  for (uint32_t cb = blockIdx.x; cb < a.nof_cbs; cb += gridDim.x) {
    // lifting size and graph of this codeblock: the launch's, or its row descriptor's (mixed Z; the
    // launch's LDS is sized for the largest), made wave-uniform explicitly
    const bool      mixed     = a.rows != nullptr;
    const uint32_t  Z         = mixed ? __builtin_amdgcn_readfirstlane(a.rows[cb].Z) : static_cast<uint32_t>(a.Z);
    const uint32_t* edges     = mixed ? a.edges + __builtin_amdgcn_readfirstlane(a.rows[cb].edge_off) : a.edges;
    const uint32_t  M_eff     = mixed ? __builtin_amdgcn_readfirstlane(a.rows[cb].M_eff) : static_cast<uint32_t>(a.M_eff);
    const uint32_t  pack_bits = mixed ? __builtin_amdgcn_readfirstlane(a.rows[cb].pack_bits)
                                      : static_cast<uint32_t>(a.pack_bits);
    const int32_t   p0_shift  = mixed ? static_cast<int32_t>(__builtin_amdgcn_readfirstlane(a.rows[cb].p0_shift))
                                      : a.p0_shift;
    int32_t         core_a[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      core_a[c] = mixed ? static_cast<int32_t>(__builtin_amdgcn_readfirstlane(a.rows[cb].core_a[c])) : a.core_a[c];
    }
    const uint32_t kz  = K * Z;
    const uint32_t nq  = (Z + 31) / 32;
    const uint32_t ncw = enc_bits_cw_words(K, M_eff, Z);
    uint32_t*      cw  = lw;            // [ncw] codeword bits
    uint32_t*      lam = lw + ncw;      // [4][nq] systematic part of the high-rate rows
    uint32_t*      ls  = lam + 4 * nq;  // [nq + 2] lambda sum as a column at bit 0
    // 1. Message words (bit reversal of 4 MSB-first bytes), the rest zeroed.
    const uint8_t* msg    = a.msgs + static_cast<size_t>(cb) * a.msg_stride;
    const uint32_t nbytes = (kz + 7) / 8;
    const uint32_t nmw    = (kz + 31) / 32;
    // message words: every load of a lane issued before its LDS stores (ENC_MSG_UNROLL rounds of the wave)
    const bool al4 = (reinterpret_cast<uintptr_t>(msg) & 3u) == 0;
    for (uint32_t w0 = j; w0 < nmw; w0 += ENC_MSG_UNROLL * ENC_BITS_THREADS) {
      uint32_t be[ENC_MSG_UNROLL];
#pragma unroll
      for (uint32_t r = 0; r < ENC_MSG_UNROLL; ++r) {
        const uint32_t w = w0 + r * ENC_BITS_THREADS;
        be[r]            = 0;
        if (w < nmw) {
          if (al4 && 4 * w + 4 <= nbytes) {
            be[r] = __builtin_bswap32(reinterpret_cast<const uint32_t*>(msg)[w]);
          } else {
#pragma unroll
            for (int b = 0; b < 4; ++b) {
              const uint32_t q = 4 * w + b;
              be[r] |= (q < nbytes ? static_cast<uint32_t>(msg[q]) : 0u) << (24 - 8 * b);
            }
          }
        }
      }
#pragma unroll
      for (uint32_t r = 0; r < ENC_MSG_UNROLL; ++r) {
        const uint32_t w = w0 + r * ENC_BITS_THREADS;
        if (w < nmw) {
          uint32_t v = __builtin_bitreverse32(be[r]);
          if (32 * w + 32 > kz) {
            v &= (1u << (kz - 32 * w)) - 1u;
          }
          cw[w] = v;
        }
      }
    }
    for (uint32_t w = nmw + j; w < ncw; w += ENC_BITS_THREADS) {
      cw[w] = 0;
    }
    for (uint32_t w = j; w < nq + 2; w += ENC_BITS_THREADS) {
      ls[w] = 0;
    }
    __syncthreads();

    // 2-5. Parity (ldpc_encode_device.h).
    encode_bits_parity<ENC_BITS_THREADS>(cw, lam, ls, edges, a.row_start, a.bg, K, Z, M_eff, p0_shift, core_a, j);

    // 6. Pack the shortened codeword (from bit 2Z), MSB-first.
    uint8_t*       out   = a.cws + static_cast<size_t>(cb) * a.cw_stride;
    const uint32_t nbits = pack_bits;
    const uint32_t nb    = (nbits + 7) / 8;
    const bool     al    = ((reinterpret_cast<uintptr_t>(out)) & 3u) == 0;
    for (uint32_t m = j; 4 * m < nb; m += ENC_BITS_THREADS) {
      uint32_t v = lds_bits32(cw, 2 * Z + 32 * m);
      if (32 * m + 32 > nbits) {
        v &= (1u << (nbits - 32 * m)) - 1u;
      }
      const uint32_t x = __builtin_bswap32(__builtin_bitreverse32(v));
      if (al && 4 * m + 4 <= nb) {
        *reinterpret_cast<uint32_t*>(out + 4 * m) = x;
      } else {
        for (uint32_t b = 0; b < 4 && 4 * m + b < nb; ++b) {
          out[4 * m + b] = static_cast<uint8_t>(x >> (8 * b));
        }
      }
    }
    __syncthreads();
  }
}

size_t ldpc_encode_lds_bytes(int K, int M_eff, int Z)
{
  return static_cast<size_t>(((K + M_eff) * Z + 15) / 16 * 16 + Z);
}

hipError_t launch_ldpc_encode(const encode_args& a, int grid, hipStream_t stream)
{
  // (mixed Z: a.Z / a.M_eff are the largest of the launch, for the LDS size)
  if (a.Z >= 32 || a.rows != nullptr) {
    const size_t words = enc_bits_lds_words(a.K, a.M_eff, a.Z);
    hipLaunchKernelGGL(ldpc_encode_bits_kernel, dim3(grid), dim3(ENC_BITS_THREADS), words * 4, stream, a);
    return hipGetLastError();
  }
  const int threads = (a.Z + 63) / 64 * 64;
  hipLaunchKernelGGL(ldpc_encode_kernel, dim3(grid), dim3(threads), ldpc_encode_lds_bytes(a.K, a.M_eff, a.Z), stream, a);
  return hipGetLastError();
}

} // namespace srs_amd
