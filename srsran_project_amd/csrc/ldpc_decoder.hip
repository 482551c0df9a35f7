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
//   * check-to-variable messages: int8 per (edge, check row), also in LDS
//     (BG1 Z=384: 26 KiB soft bits + 121 KiB messages = 147 KiB of the 160 KiB),
//     so the whole decoder state of a codeblock stays on chip;
//   * the graph (per-layer edge list, packed (var*Z) | shift<<16) is a kernel
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

// One layer (base-graph check row) for check row j of the lifted graph:
// ldpc_decoder_impl.cpp:235 (v2c), :290 (min / second min / sign, scaling),
// :270 (soft-bit promotion sum).  DEG is the row degree, so the body is
// straight-line code: all LDS gathers are issued before the first use.
template <int DEG, int ARITH>
__device__ __forceinline__ void
process_layer(int8_t* soft, int8_t* c2v, const uint32_t* edge, int e0, int Z, int j, bool active)
{
  int ad[DEG];
  int sb[DEG];
  int cv[DEG];
#pragma unroll
  for (int e = 0; e < DEG; ++e) {
    const uint32_t d = edge[e0 + e];
    int            p = j + static_cast<int>(d >> 16);
    p                = p >= Z ? p - Z : p;
    ad[e]            = static_cast<int>(d & 0xffffu) + p;
  }
#pragma unroll
  for (int e = 0; e < DEG; ++e) {
    sb[e] = soft[ad[e]];
    cv[e] = c2v[(e0 + e) * Z + j];
  }
  int min1 = LLR_MAX, min2 = LLR_MAX, idx = 0, sgn = 0;
#pragma unroll
  for (int e = 0; e < DEG; ++e) {
    // v2c = soft - c2v saturated to +-LLR_MAX; infinite soft bits stay infinite.
    const int  x   = sb[e];
    const bool inf = (x > LLR_MAX) || (x < -LLR_MAX);
    const int  v   = inf ? x : clamp_i(x - cv[e], -LLR_MAX, LLR_MAX);
    sb[e]          = v; // reuse as v2c
    const int  av  = v < 0 ? -v : v;
    const bool lt1 = av < min1;
    min2           = lt1 ? min1 : (av < min2 ? av : min2);
    idx            = lt1 ? e : idx;
    min1           = lt1 ? av : min1;
    sgn ^= (v < 0);
  }
  const int s1 = scale_mag<ARITH>(min1);
  const int s2 = scale_mag<ARITH>(min2);
#pragma unroll
  for (int e = 0; e < DEG; ++e) {
    const int  v   = sb[e];
    const int  mag = (e == idx) ? s2 : s1;
    const int  c   = (sgn ^ (v < 0)) ? -mag : mag;
    // promotion sum (log_likelihood_ratio.cpp:75); c is always finite, and
    // c == -v gives 0 through the plain sum.
    const bool inf = (v > LLR_MAX) || (v < -LLR_MAX);
    int        t   = c + v;
    t              = t > LLR_MAX ? LLR_INFINITY : (t < -LLR_MAX ? -LLR_INFINITY : t);
    cv[e]          = c;
    sb[e]          = inf ? v : t;
  }
  if (active) {
#pragma unroll
    for (int e = 0; e < DEG; ++e) {
      c2v[(e0 + e) * Z + j] = static_cast<int8_t>(cv[e]);
      soft[ad[e]]           = static_cast<int8_t>(sb[e]);
    }
  }
}

template <int MAXDEG, int ARITH>
__global__ void __launch_bounds__(MAX_LIFTING_SIZE) ldpc_decode_kernel(decode_args a, lifted_graph g)
{
  extern __shared__ __attribute__((aligned(16))) int8_t smem[];
  // smem layout: [0, 64) reduction slots (int32 x 16), then soft bits N_full*Z.
  const int Z    = g.Z;
  int32_t*  red  = reinterpret_cast<int32_t*>(smem);
  int8_t*   soft = smem + 64;
  int8_t*   c2v  = soft + ((g.N_full * Z + 15) & ~15); // [edge][check row]

  const int  j       = threadIdx.x;
  const int  nthr    = blockDim.x;
  const bool active  = j < Z;
  const int  jj      = active ? j : 0; // idle lanes gather valid addresses, store nothing
  const int  wave    = j >> 6;
  const int  nwaves  = nthr >> 6;
  const int  lane    = j & 63;
  const int  msg_len = g.K * Z;
  const int  NZ      = g.N_full * Z;

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

    // check-to-variable messages start at zero (ldpc_decoder_impl.cpp:244: an
    // uninitialised layer uses v2c = soft, identical to v2c = soft - 0).
    for (int i = j * 16; i < g.nedges * Z; i += nthr * 16) {
      *reinterpret_cast<int4*>(c2v + i) = make_int4(0, 0, 0, 0);
    }
    __syncthreads();

    for (int it = 0; it < a.max_iterations; ++it) {
      for (int l = 0; l < nof_layers; ++l) {
        const int e0  = g.row_start[l];
        const int deg = g.row_start[l + 1] - e0;
        switch (deg) {
          case 3: process_layer<3, ARITH>(soft, c2v, g.edge, e0, Z, jj, active); break;
          case 4: process_layer<4, ARITH>(soft, c2v, g.edge, e0, Z, jj, active); break;
          case 5: process_layer<5, ARITH>(soft, c2v, g.edge, e0, Z, jj, active); break;
          case 6: process_layer<6, ARITH>(soft, c2v, g.edge, e0, Z, jj, active); break;
          case 7: process_layer<7, ARITH>(soft, c2v, g.edge, e0, Z, jj, active); break;
          case 8: process_layer<8, ARITH>(soft, c2v, g.edge, e0, Z, jj, active); break;
          case 9: process_layer<9, ARITH>(soft, c2v, g.edge, e0, Z, jj, active); break;
          case 10: process_layer<10, ARITH>(soft, c2v, g.edge, e0, Z, jj, active); break;
          default: process_layer<19, ARITH>(soft, c2v, g.edge, e0, Z, jj, active); break;
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
size_t ldpc_decode_lds_bytes(const lifted_graph& g)
{
  return 64 + ((static_cast<size_t>(g.N_full) * g.Z + 15) / 16) * 16 + static_cast<size_t>(g.nedges) * g.Z;
}

hipError_t launch_ldpc_decode(const decode_args& args, const lifted_graph& g, int arith, int grid, hipStream_t stream)
{
  const int    threads = ((g.Z + 63) / 64) * 64;
  const size_t lds     = ldpc_decode_lds_bytes(g);
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
