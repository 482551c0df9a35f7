// ldpc_decoder.hip -- batched layered normalised min-sum LDPC decoder for gfx950.
//
// Algorithm (bit-exact with the reference CPU decoders):
//   lib/phy/upper/channel_coding/ldpc/ldpc_decoder_impl.cpp:55   decode(): input trimming,
//       soft-bit loading (clamp to +-64), layer count from the input length,
//       layered schedule, CRC early stop after every iteration.
//   ldpc_decoder_impl.cpp:235    update_variable_to_check_messages
//   ldpc_decoder_impl.cpp:290    update_check_to_variable_messages (min / second min / index / sign)
//   ldpc_decoder_impl.cpp:270    update_soft_bits (promotion sum)
//   ldpc_decoder_avx2.cpp / ldpc_decoder_avx512.cpp (ARITH_SIMD) and
//   ldpc_decoder_generic.cpp (ARITH_GENERIC): the check-node scaling by 0.8.
//
// MI355X mapping:
//   * one workgroup per codeblock; workgroup = ceil(Z/64) wavefronts; lane j owns
//     check row j of every layer (all Z checks of a layer are independent, so a
//     layer is one data-parallel step and layers are separated by one barrier);
//   * the codeblock's soft bits (N_full x Z int8, <= 26 KiB) live in LDS for the
//     whole decode: every edge update is an LDS gather/scatter at a per-edge
//     cyclic shift, HBM is touched only to read the LLRs once and write the
//     packed hard bits once;
//   * check-to-variable messages: int8 per (edge, check row), kept in a per-slot
//     scratch region read/written with coalesced byte accesses (L2/MALL resident);
//   * the graph (per-layer edge list: variable node + shift) is a kernel
//     argument, read through the scalar cache;
//   * CRC early stop: the CRC is linear over GF(2), so each lane XORs the
//     precomputed remainders x^(n-1-i+L) mod g of its set hard bits and the
//     workgroup XOR-reduces -- one pass over LDS instead of a serial bit loop.
#include <hip/hip_runtime.h>

#include "ldpc_common.h"

namespace srs_amd {


__device__ __forceinline__ int clamp_i(int x, int lo, int hi)
{
  return x < lo ? lo : (x > hi ? hi : x);
}

template <int ARITH>
__device__ __forceinline__ int scale_mag(int mag)
{
  if (ARITH == ARITH_GENERIC) {
    return static_cast<int>(__builtin_roundf(static_cast<float>(mag) * 0.8f));
  }
  return (mag * 52428) >> 16;
}

// Block-wide reductions (wave64 shuffles, then one LDS slot per wave).
__device__ __forceinline__ uint32_t wave_xor(uint32_t v)
{
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    v ^= __shfl_xor(v, o, 64);
  }
  return v;
}
__device__ __forceinline__ uint32_t wave_or(uint32_t v)
{
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    v |= __shfl_xor(v, o, 64);
  }
  return v;
}
__device__ __forceinline__ int wave_max(int v)
{
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    int w = __shfl_xor(v, o, 64);
    v     = v > w ? v : w;
  }
  return v;
}

template <int MAXDEG, int ARITH>
__global__ void __launch_bounds__(MAX_LIFTING_SIZE) ldpc_decode_kernel(decode_args a, lifted_graph g)
{
  extern __shared__ __attribute__((aligned(16))) int8_t smem[];
  // smem layout: [0, 64) reduction slots (int32 x 16), then soft bits N_full*Z.
  int32_t* red  = reinterpret_cast<int32_t*>(smem);
  int8_t*  soft = smem + 64;

  const int  Z       = g.Z;
  const int  j       = threadIdx.x;
  const int  nthr    = blockDim.x;
  const bool active  = j < Z;
  const int  wave    = j >> 6;
  const int  nwaves  = nthr >> 6;
  const int  lane    = j & 63;
  const int  msg_len = g.K * Z;
  const int  NZ      = g.N_full * Z;
  int8_t*    c2v     = a.c2v_ws + static_cast<size_t>(blockIdx.x) * g.nedges * a.zpad;

  for (uint32_t cb = blockIdx.x; cb < a.nof_cbs; cb += gridDim.x) {
    const int8_t* in      = a.llrs + static_cast<size_t>(cb) * a.llr_stride;
    const int     n_llrs  = a.llr_lens ? static_cast<int>(a.llr_lens[cb]) : static_cast<int>(a.llr_len);
    uint8_t*      out     = a.out + static_cast<size_t>(cb) * a.out_stride;
    const int     obytes  = (msg_len + 7) >> 3;

    // ---- input trimming: position of the last non-zero LLR (ldpc_decoder_impl.cpp:86).
    int last = -1;
    for (int i = j; i < n_llrs; i += nthr) {
      if (in[i] != 0) {
        last = i;
      }
    }
    last = wave_max(last);
    __syncthreads();
    if (lane == 0) {
      red[wave] = last;
    }
    __syncthreads();
    int input_size = 0;
    for (int w = 0; w < nwaves; ++w) {
      input_size = red[w] + 1 > input_size ? red[w] + 1 : input_size;
    }

    if (input_size < msg_len && a.force_decoding) {
      // ldpc_decoder_impl.cpp:92: not enough soft bits -- all ones when no CRC,
      // output left untouched when a CRC is given (as the reference).
      for (int b = j; b < obytes && !a.crc_table; b += nthr) {
        uint8_t v = 0xff;
        if (b == obytes - 1 && (msg_len & 7)) {
          v &= static_cast<uint8_t>(0xff << (8 - (msg_len & 7)));
        }
        out[b] = v;
      }
      if (j == 0) {
        a.nof_iters[cb] = -1;
      }
      __syncthreads();
      continue;
    }

    // ---- load soft bits (ldpc_decoder_impl.cpp:160 load_soft_bits).
    {
      const int nof_full_nodes = n_llrs / Z + 2;
      const int tail           = n_llrs - (nof_full_nodes - 2) * Z;
      for (int node = 0; node < g.N_full; ++node) {
        for (int p = j; p < Z; p += nthr) {
          int v = 0;
          if (node >= 2 && node < nof_full_nodes) {
            v = clamp_i(in[(node - 2) * Z + p], -SOFT_CLAMP, SOFT_CLAMP);
          } else if (node == nof_full_nodes && p < tail) {
            v = in[(node - 2) * Z + p];
          }
          soft[node * Z + p] = static_cast<int8_t>(v);
        }
      }
    }
    int cb_len = input_size + 2 * Z;
    if (cb_len < msg_len + 4 * Z) {
      cb_len = msg_len + 4 * Z;
    }
    const int nof_layers     = (cb_len + Z - 1) / Z - g.K;
    const int nof_sig        = msg_len - a.nof_filler_bits;
    int       result         = -1;
    __syncthreads();

    for (int it = 0; it < a.max_iterations; ++it) {
      for (int l = 0; l < nof_layers; ++l) {
        const int e0  = g.row_start[l];
        const int deg = g.row_start[l + 1] - e0;
        int       v2c[MAXDEG];
        int       addr[MAXDEG];
        int       min1 = LLR_MAX, min2 = LLR_MAX, idx = 0, sgn = 0;
#pragma unroll
        for (int e = 0; e < MAXDEG; ++e) {
          if (e < deg) {
            const int var = g.var[e0 + e];
            int       p   = j + g.shift[e0 + e];
            p             = p >= Z ? p - Z : p;
            addr[e]       = var * Z + p;
            int sb        = active ? soft[addr[e]] : 0;
            int c         = (it > 0 && active) ? c2v[(e0 + e) * a.zpad + j] : 0;
            // v2c = soft - c2v saturated to +-LLR_MAX; infinite soft bits stay infinite.
            int v    = (sb == LLR_INFINITY || sb == -LLR_INFINITY) ? sb : clamp_i(sb - c, -LLR_MAX, LLR_MAX);
            v2c[e]   = v;
            int  av  = v < 0 ? -v : v;
            bool lt1 = av < min1;
            min2     = lt1 ? min1 : (av < min2 ? av : min2);
            idx      = lt1 ? e : idx;
            min1     = lt1 ? av : min1;
            sgn ^= (v < 0);
          }
        }
        const int s1 = scale_mag<ARITH>(min1);
        const int s2 = scale_mag<ARITH>(min2);
#pragma unroll
        for (int e = 0; e < MAXDEG; ++e) {
          if (e < deg) {
            const int v   = v2c[e];
            const int mag = (e == idx) ? s2 : s1;
            const int c   = (sgn ^ (v < 0)) ? -mag : mag;
            // promotion sum (log_likelihood_ratio.cpp:75); c is always finite.
            int s;
            if (c == -v) {
              s = 0;
            } else if (v == LLR_INFINITY || v == -LLR_INFINITY) {
              s = v;
            } else {
              s = c + v;
              s = s > LLR_MAX ? LLR_INFINITY : (s < -LLR_MAX ? -LLR_INFINITY : s);
            }
            if (active) {
              c2v[(e0 + e) * a.zpad + j] = static_cast<int8_t>(c);
              soft[addr[e]]              = static_cast<int8_t>(s);
            }
          }
        }
        __syncthreads();
      }

      if (a.crc_table) {
        // get_hard_bits + CRC early stop (ldpc_decoder_impl.cpp:125).
        uint32_t crc = 0, zero = 0;
        for (int i = j; i < msg_len; i += nthr) {
          int sb = soft[i];
          zero |= (sb == 0);
          if (i < nof_sig && sb <= 0) {
            crc ^= a.crc_table[nof_sig - 1 - i];
          }
        }
        crc  = wave_xor(crc);
        zero = wave_or(zero);
        if (lane == 0) {
          red[wave]      = static_cast<int32_t>(crc);
          red[8 + wave]  = static_cast<int32_t>(zero);
        }
        __syncthreads();
        uint32_t c_all = 0, z_all = 0;
        for (int w = 0; w < nwaves; ++w) {
          c_all ^= static_cast<uint32_t>(red[w]);
          z_all |= static_cast<uint32_t>(red[8 + w]);
        }
        __syncthreads();
        if (z_all == 0 && c_all == 0) {
          result = it + 1;
          break;
        }
      }
    }

    // ---- hard decision, packed MSB-first (log_likelihood_ratio.cpp hard_decision).
    for (int b = j; b < obytes; b += nthr) {
      uint32_t byte = 0;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        int i = b * 8 + k;
        if (i < msg_len && soft[i] <= 0) {
          byte |= 0x80u >> k;
        }
      }
      out[b] = static_cast<uint8_t>(byte);
    }
    if (a.soft_out) {
      int8_t* so = a.soft_out + static_cast<size_t>(cb) * NZ;
      for (int i = j; i < NZ; i += nthr) {
        so[i] = soft[i];
      }
    }
    if (j == 0) {
      a.nof_iters[cb] = result;
    }
    __syncthreads();
  }
}

// Host launcher (declared in ldpc_api.cpp).
hipError_t launch_ldpc_decode(const decode_args& args, const lifted_graph& g, int arith, int grid, hipStream_t stream)
{
  const int threads = ((g.Z + 63) / 64) * 64;
  const size_t lds  = 64 + ((static_cast<size_t>(g.N_full) * g.Z + 15) / 16) * 16;
  if (g.bg == 1) {
    if (arith == ARITH_GENERIC) {
      hipLaunchKernelGGL((ldpc_decode_kernel<BG1_MAX_DEGREE, ARITH_GENERIC>), dim3(grid), dim3(threads), lds, stream, args, g);
    } else {
      hipLaunchKernelGGL((ldpc_decode_kernel<BG1_MAX_DEGREE, ARITH_SIMD>), dim3(grid), dim3(threads), lds, stream, args, g);
    }
  } else {
    if (arith == ARITH_GENERIC) {
      hipLaunchKernelGGL((ldpc_decode_kernel<BG2_MAX_DEGREE, ARITH_GENERIC>), dim3(grid), dim3(threads), lds, stream, args, g);
    } else {
      hipLaunchKernelGGL((ldpc_decode_kernel<BG2_MAX_DEGREE, ARITH_SIMD>), dim3(grid), dim3(threads), lds, stream, args, g);
    }
  }
  return hipGetLastError();
}

} // namespace srs_amd
