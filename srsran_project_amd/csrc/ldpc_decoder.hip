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
//     check row j of every layer (the Z checks of a layer are independent, so a
//     layer is one data-parallel step and consecutive layers are separated by one
//     workgroup barrier);
//   * soft bits (N_full x Z int8, <= 26 KiB) live in LDS for the whole decode:
//     every edge update is an LDS gather/scatter at the edge's cyclic shift;
//   * check-to-variable messages live in VGPRs: lane j holds the int8 message of
//     every edge of check row j (BG1: 316 edges = 79 packed registers).  The
//     layer schedule is unrolled at compile time over the base graph's row
//     degrees, so every message has a fixed register and byte; extraction is
//     one v_bfe_i32, insertion one v_perm_b32.  With 26 KiB of LDS and <= 128
//     VGPRs per lane, two Z=384 codeblocks (12 waves) share a CU and hide each
//     other's barrier / LDS latency;
//   * HBM is touched only to read the LLRs once and write the packed hard bits;
//   * CRC early stop: the CRC is linear over GF(2), so each lane XORs the
//     precomputed remainders x^(n-1-i+L) mod g of its set hard bits and the
//     workgroup XOR-reduces -- one pass over LDS instead of a serial bit loop.
#include <hip/hip_runtime.h>

#include "ldpc_common.h"
#include <utility>

namespace srs_amd {

// Edge descriptors are read through the scalar unit (s_load from the constant
// address space), never as per-lane vector loads.
using const_u32_ptr = const __attribute__((address_space(4))) uint32_t*;

// Row degrees of the base graphs (TS 38.212 Tables 5.3.2-2/3); the host checks
// them against bg_tables.inc (ldpc_graph.cpp, check_row_degrees).
constexpr int BG1_DEG[46] = {19, 19, 19, 19, 3, 8, 9, 7, 10, 9, 7, 8, 7, 6, 7, 7, 6, 6, 6, 6, 6, 6, 5,
                             5,  6,  5,  5,  4, 5, 5, 5, 5,  5, 5, 5, 5, 5, 4, 5, 5, 4, 5, 4, 5, 5, 4};
constexpr int BG2_DEG[42] = {8, 10, 8, 10, 4, 6, 6, 6, 4, 5, 5, 5, 4, 5, 5, 4, 5, 5, 4, 4, 4,
                             4, 3,  4, 4,  3, 5, 3, 4, 3, 5, 3, 4, 4, 4, 4, 4, 3, 4, 4, 4, 4};

template <int BG>
struct bg_traits;
template <>
struct bg_traits<1> {
  static constexpr int M = 46, NEDGES = 316;
  static constexpr int deg(int l) { return BG1_DEG[l]; }
};
template <>
struct bg_traits<2> {
  static constexpr int M = 42, NEDGES = 197;
  static constexpr int deg(int l) { return BG2_DEG[l]; }
};
template <int BG>
constexpr int row_start(int l)
{
  int s = 0;
  for (int i = 0; i < l; ++i) {
    s += bg_traits<BG>::deg(i);
  }
  return s;
}
static_assert(row_start<1>(46) == 316, "BG1 degree table");
static_assert(row_start<2>(42) == 197, "BG2 degree table");

__device__ __forceinline__ int med3_i(int x, int lo, int hi)
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

// int8 message K of the packed register file.
template <int K, int NW>
__device__ __forceinline__ int c2v_get(const uint32_t (&r)[NW])
{
  return static_cast<int>(static_cast<int8_t>(r[K >> 2] >> (8 * (K & 3))));
}
template <int K, int NW>
__device__ __forceinline__ void c2v_set(uint32_t (&r)[NW], int c)
{
  // v_perm_b32: byte (K&3) from c, the other bytes from the old word.
  constexpr uint32_t sel = (K & 3) == 0 ? 0x07060500u : (K & 3) == 1 ? 0x07060004u : (K & 3) == 2 ? 0x07000504u : 0x00060504u;
  r[K >> 2]              = __builtin_amdgcn_perm(r[K >> 2], static_cast<uint32_t>(c), sel);
}

// Pass 1 for edge E: form v2c from the gathered soft bit and the old message
// and update the check-node statistics (ldpc_decoder_impl.cpp:235 / :290).
// v2c is kept packed (4 per register; pass 2 reads it back as a sign-extended
// SDWA byte operand, free on gfx950).
template <int E0, int E, int NW, int NX>
__device__ __forceinline__ void
edge_pass1(int s, uint32_t (&xp)[NX], const uint32_t (&c2v)[NW], int& min1, int& min2, int& idx, int& sgn)
{
  // v2c = soft - c2v saturated to +-LLR_MAX; infinite soft bits stay infinite.
  const bool inf = static_cast<unsigned>(s + LLR_MAX) > static_cast<unsigned>(2 * LLR_MAX);
  const int  v   = inf ? s : med3_i(s - c2v_get<E0 + E>(c2v), -LLR_MAX, LLR_MAX);
  const int  av  = v < 0 ? -v : v;
  const bool lt1 = av < min1;
  idx            = lt1 ? E : idx;
  // new second minimum = median(min1, |v|, min2)
  min2 = av < min1 ? min1 : (av < min2 ? av : min2);
  min1 = lt1 ? av : min1;
  sgn ^= v;
  c2v_set<E>(xp, v);
}

// Pass 2 for edge E: new c2v (scaled min / second min with the extrinsic sign)
// and the new soft bit, promotion sum c2v + v2c (ldpc_decoder_impl.cpp:310, :270).
template <int E0, int E, int NW, int NX>
__device__ __forceinline__ int edge_pass2(const uint32_t (&xp)[NX], uint32_t (&c2v)[NW], int s1, int s2, int idx, int sgn)
{
  const int v   = c2v_get<E>(xp);
  const int mag = (E == idx) ? s2 : s1;
  const int c   = ((sgn ^ v) < 0) ? -mag : mag;
  // promotion sum (log_likelihood_ratio.cpp:75); c is always finite, and
  // c == -v gives 0 through the plain sum.
  const bool inf = static_cast<unsigned>(v + LLR_MAX) > static_cast<unsigned>(2 * LLR_MAX);
  int        t   = c + v;
  t              = t > LLR_MAX ? LLR_INFINITY : (t < -LLR_MAX ? -LLR_INFINITY : t);
  c2v_set<E0 + E>(c2v, c);
  return inf ? v : t;
}

// One layer (base-graph check row) for check row j of the lifted graph.
// E0/DEG are compile-time, so the body is straight-line code: all DEG gathers
// are issued before the first use and all DEG scatters after the last, so no
// LDS read ever waits behind a (possibly aliasing) LDS write of the same layer.
// Idle lanes (j >= Z, only when Z is not a multiple of 64) are redirected to a
// private dummy slot, so no exec-mask branches are needed.
template <int E0, int ARITH, int NW, int... E>
__device__ __forceinline__ void process_layer(int8_t*                  soft,
                                              uint32_t (&c2v)[NW],
                                              const_u32_ptr            edge,
                                              int                      Z,
                                              int                      j,
                                              int                      idle_slot,
                                              std::integer_sequence<int, E...>)
{
  constexpr int DEG = sizeof...(E);
  constexpr int NX  = (DEG + 3) / 4;
  int           ad[DEG];
  int           x[DEG];
  uint32_t      xp[NX];
#pragma unroll
  for (int e = 0; e < DEG; ++e) {
    // gather address = var*Z + (j + shift) mod Z; (j + shift - Z) wraps as an
    // unsigned value exactly when j + shift < Z, so the mod is one v_min_u32.
    const uint32_t d     = edge[E0 + e];
    const uint32_t shift = d >> 16;
    const uint32_t t1    = static_cast<uint32_t>(j) + shift;
    const uint32_t t2    = static_cast<uint32_t>(j) + (shift - static_cast<uint32_t>(Z));
    ad[e]                = static_cast<int>((t1 < t2 ? t1 : t2) + (d & 0xffffu));
    if (idle_slot >= 0) {
      ad[e] = idle_slot;
    }
  }
#pragma unroll
  for (int e = 0; e < DEG; ++e) {
    x[e] = soft[ad[e]];
  }
#pragma unroll
  for (int w = 0; w < NX; ++w) {
    xp[w] = 0;
  }
  int min1 = LLR_MAX, min2 = LLR_MAX, idx = 0, sgn = 0;
  (edge_pass1<E0, E>(x[E], xp, c2v, min1, min2, idx, sgn), ...);
  const int s1 = scale_mag<ARITH>(min1);
  const int s2 = scale_mag<ARITH>(min2);
  ((x[E] = edge_pass2<E0, E>(xp, c2v, s1, s2, idx, sgn)), ...);
#pragma unroll
  for (int e = 0; e < DEG; ++e) {
    soft[ad[e]] = static_cast<int8_t>(x[e]);
  }
}

// Layers L .. M-1 of one iteration, stopping (uniformly) at nof_layers.
template <int BG, int L, int ARITH, int NW>
__device__ __forceinline__ void run_layers(int8_t*       soft,
                                           uint32_t (&c2v)[NW],
                                           const_u32_ptr edge,
                                           int           Z,
                                           int           j,
                                           int           idle_slot,
                                           int           nof_layers)
{
  if constexpr (L < bg_traits<BG>::M) {
    // A uniform branch around the layer (not an early return): the join after
    // it merges only the few message registers this layer writes, whereas 46
    // early exits would each merge the whole message file.
    if (L < nof_layers) {
      // Launder the graph pointer and Z per layer: the gather addresses are
      // iteration-invariant, and letting the compiler hoist (and keep live) the
      // addresses and descriptors of later layers would spill the register file.
      asm volatile("" : "+s"(edge), "+s"(Z));
      process_layer<row_start<BG>(L), ARITH>(
          soft, c2v, edge, Z, j, idle_slot, std::make_integer_sequence<int, bg_traits<BG>::deg(L)>{});
      __syncthreads();
    }
    run_layers<BG, L + 1, ARITH>(soft, c2v, edge, Z, j, idle_slot, nof_layers);
  }
}

template <int BG, int ARITH>
__global__ void __launch_bounds__(MAX_LIFTING_SIZE, 4) ldpc_decode_kernel(decode_args a, lifted_graph g)
{
  constexpr int NW = (bg_traits<BG>::NEDGES + 3) / 4;
  extern __shared__ __attribute__((aligned(16))) int8_t smem[];
  // smem layout: [0, 64) reduction slots (int32 x 16), then soft bits N_full*Z.
  const int Z    = g.Z;
  int32_t*  red  = reinterpret_cast<int32_t*>(smem);
  int8_t*   soft = smem + 64;

  const int  j       = threadIdx.x;
  const int  nthr    = blockDim.x;
  const bool active  = j < Z;
  // idle lanes (Z not a multiple of 64) work on a private dummy byte past the soft bits
  const int idle_slot = active ? -1 : ((g.N_full * Z + 15) & ~15) + (j & 63);
  const int  wave    = j >> 6;
  const int  nwaves  = nthr >> 6;
  const int  lane    = j & 63;
  const int  msg_len = g.K * Z;
  const int  NZ      = g.N_full * Z;

  for (uint32_t cb = blockIdx.x; cb < a.nof_cbs; cb += gridDim.x) {
    const int8_t* in     = a.llrs + static_cast<size_t>(cb) * a.llr_stride;
    const int     n_llrs = a.llr_lens ? static_cast<int>(a.llr_lens[cb]) : static_cast<int>(a.llr_len);
    uint8_t*      out    = a.out + static_cast<size_t>(cb) * a.out_stride;
    const int     obytes = (msg_len + 7) >> 3;

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
            v = med3_i(in[(node - 2) * Z + p], -SOFT_CLAMP, SOFT_CLAMP);
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
    const int nof_layers = (cb_len + Z - 1) / Z - g.K;
    const int nof_sig    = msg_len - a.nof_filler_bits;
    int       result     = -1;

    // check-to-variable messages start at zero (ldpc_decoder_impl.cpp:244: an
    // uninitialised layer uses v2c = soft, identical to v2c = soft - 0).
    uint32_t c2v[NW];
#pragma unroll
    for (int w = 0; w < NW; ++w) {
      c2v[w] = 0;
    }
    __syncthreads();

    for (int it = 0; it < a.max_iterations; ++it) {
      run_layers<BG, 0, ARITH>(soft, c2v, (const_u32_ptr)(a.edges), Z, j, idle_slot, nof_layers);

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
          red[wave]     = static_cast<int32_t>(crc);
          red[8 + wave] = static_cast<int32_t>(zero);
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

size_t ldpc_decode_lds_bytes(const lifted_graph& g)
{
  return 64 + ((static_cast<size_t>(g.N_full) * g.Z + 15) / 16) * 16 + 64;
}

hipError_t launch_ldpc_decode(const decode_args& args, const lifted_graph& g, int arith, int grid, hipStream_t stream)
{
  const int    threads = ((g.Z + 63) / 64) * 64;
  const size_t lds     = ldpc_decode_lds_bytes(g);
  if (g.bg == 1) {
    if (arith == ARITH_GENERIC) {
      hipLaunchKernelGGL((ldpc_decode_kernel<1, ARITH_GENERIC>), dim3(grid), dim3(threads), lds, stream, args, g);
    } else {
      hipLaunchKernelGGL((ldpc_decode_kernel<1, ARITH_SIMD>), dim3(grid), dim3(threads), lds, stream, args, g);
    }
  } else {
    if (arith == ARITH_GENERIC) {
      hipLaunchKernelGGL((ldpc_decode_kernel<2, ARITH_GENERIC>), dim3(grid), dim3(threads), lds, stream, args, g);
    } else {
      hipLaunchKernelGGL((ldpc_decode_kernel<2, ARITH_SIMD>), dim3(grid), dim3(threads), lds, stream, args, g);
    }
  }
  return hipGetLastError();
}

} // namespace srs_amd
