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
//   * check-to-variable messages: lane j holds the int8 message of every edge of
//     check row j.  The layer schedule is unrolled at compile time over the base
//     graph's row degrees, so every message has a fixed home: the light layers
//     (degree <= 10, 240 of BG1's 316 edges) in VGPRs packed 4 per register
//     (read as a sign-extended SDWA byte operand, written with one v_perm_b32),
//     the four degree-19 rows of BG1 in LDS ([edge][row], 29 KiB at Z=384).
//     That keeps a Z=384 codeblock at <= 128 VGPRs and 55 KiB of LDS, so two
//     codeblocks (12 waves) share a CU and hide each other's barrier and LDS
//     latency;
//   * for Z=384 (the 100 MHz workloads) the lifted graph is compile-time: shifts
//     and node offsets are literals (gather address = add, add, min); other Z
//     read packed edge descriptors through the scalar unit;
//   * HBM is touched only to read the LLRs once and write the packed hard bits;
//   * CRC early stop: the CRC is linear over GF(2), so each lane XORs the
//     precomputed remainders x^(n-1-i+L) mod g of its set hard bits and the
//     workgroup XOR-reduces -- one pass over LDS instead of a serial bit loop.
#include "kernel_probe.h"
#include "srsran_amd/profiling.h"
#include <hip/hip_runtime.h>

#include "ldpc_common.h"
#include <cstdlib>
#include <type_traits>
#include <utility>

namespace srs_amd {

#define SRS_BG_TABLE_QUAL constexpr
namespace tables {
#include "bg_tables.inc"
}
#undef SRS_BG_TABLE_QUAL

// Edge descriptors are read through the scalar unit (s_load from the constant
// address space), never as per-lane vector loads.
using const_u32_ptr = const __attribute__((address_space(4))) uint32_t*;

// LDS addressing.  The kernels declare no static LDS, so the dynamic segment
// starts at LDS address 0 and the carve-up offsets are plain integers: with a
// compile-time Z every gather/scatter offset folds into the ds instruction's
// immediate, and the compiler's occupancy model does not see a fixed 55 KiB
// block (which would let it trade the 4-waves/SIMD target for registers).
// Layout (bytes): [16,80) reductions | soft bits | LDS-resident messages | pad.
constexpr int LDS_RED_OFFSET  = 16;
constexpr int LDS_SOFT_OFFSET = 80;
using lds_i8                  = __attribute__((address_space(3))) int8_t;
using lds_i32                 = __attribute__((address_space(3))) int32_t;
using lds_u32                 = __attribute__((address_space(3))) uint32_t;


// Row degrees of the base graphs (TS 38.212 Tables 5.3.2-2/3).
constexpr int BG1_DEG[46] = {19, 19, 19, 19, 3, 8, 9, 7, 10, 9, 7, 8, 7, 6, 7, 7, 6, 6, 6, 6, 6, 6, 5,
                             5,  6,  5,  5,  4, 5, 5, 5, 5,  5, 5, 5, 5, 5, 4, 5, 5, 4, 5, 4, 5, 5, 4};
constexpr int BG2_DEG[42] = {8, 10, 8, 10, 4, 6, 6, 6, 4, 5, 5, 5, 4, 5, 5, 4, 5, 5, 4, 4, 4,
                             4, 3,  4, 4,  3, 5, 3, 4, 3, 5, 3, 4, 4, 4, 4, 4, 3, 4, 4, 4, 4};

template <int BG>
struct bg_traits;
template <>
struct bg_traits<1> {
  static constexpr int M = 46, NEDGES = 316, N_FULL = 68, K = 22;
  // leading rows whose messages live in LDS (the degree-19 rows)
  static constexpr int LDS_ROWS = 4, LDS_EDGES = 76;
  static constexpr int deg(int l) { return BG1_DEG[l]; }
};
template <>
struct bg_traits<2> {
  static constexpr int M = 42, NEDGES = 197, N_FULL = 52, K = 10;
  static constexpr int LDS_ROWS = 0, LDS_EDGES = 0;
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
static_assert(row_start<1>(46) == 316 && row_start<1>(4) == bg_traits<1>::LDS_EDGES, "BG1 degree table");
static_assert(row_start<2>(42) == 197, "BG2 degree table");
template <int BG>
constexpr int reg_words()
{
  return (bg_traits<BG>::NEDGES - bg_traits<BG>::LDS_EDGES + 3) / 4;
}

// TS 38.212 Table 5.3.2-1 set index of a lifting size (compile-time).
constexpr int lifting_index_c(int Z)
{
  int a = Z;
  while ((a & 1) == 0) {
    a >>= 1;
  }
  return a == 1 ? 0 : a == 3 ? 1 : a == 5 ? 2 : a == 7 ? 3 : a == 9 ? 4 : a == 11 ? 5 : a == 13 ? 6 : 7;
}

// Edge E of base graph BG lifted to a compile-time Z: variable node and shift.
template <int BG, int ZC, int E>
struct const_edge {
  static constexpr int var   = BG == 1 ? tables::SRS_BG1_EDGES[E][1] : tables::SRS_BG2_EDGES[E][1];
  static constexpr int shift = (BG == 1 ? tables::SRS_BG1_EDGES[E][2 + lifting_index_c(ZC)]
                                        : tables::SRS_BG2_EDGES[E][2 + lifting_index_c(ZC)]) %
                               ZC;
};

// LDS carve-up (bytes): [0,64) reductions | soft bits N_full*Z | LDS-resident
// messages LDS_EDGES*Z | 64-byte idle-lane pad.
template <int BG>
__host__ __device__ constexpr int lds_soft_bytes(int Z)
{
  return (bg_traits<BG>::N_FULL * Z + 15) & ~15;
}
template <int BG>
__host__ __device__ constexpr int lds_total_bytes(int Z)
{
  return 80 + lds_soft_bytes<BG>(Z) + ((bg_traits<BG>::LDS_EDGES * Z + 15) & ~15) + 64;
}

__device__ __forceinline__ int med3_i(int x, int lo, int hi)
{
  return x < lo ? lo : (x > hi ? hi : x);
}

// v_med3_i32 as an opaque instruction: left to itself the compiler rewrites
// some medians into compare + v_cndmask pairs (two instructions plus hazard
// s_nops each), which is what the branch-free formulations below avoid.
__device__ __forceinline__ int med3_op(int x, int y, int z)
{
  int r;
  asm("v_med3_i32 %0, %1, %2, %3" : "=v"(r) : "v"(x), "v"(y), "v"(z));
  return r;
}
// median(x, -120, 120): the +-LLR_MAX saturation.
__device__ __forceinline__ int sat120(int x)
{
  int r;
  asm("v_med3_i32 %0, %1, %2, %3" : "=v"(r) : "v"(x), "s"(-LLR_MAX), "v"(LLR_MAX));
  return r;
}
// a * K + b with a 24-bit signed multiply
template <int K>
__device__ __forceinline__ int mad24(int a, int b)
{
  int r;
  if constexpr (K >= -16 && K <= 64) {
    asm("v_mad_i32_i24 %0, %1, %2, %3" : "=v"(r) : "v"(a), "i"(K), "v"(b));
  } else { // not an inline constant: from an SGPR (VOP3 takes no literal here)
    asm("v_mad_i32_i24 %0, %1, %2, %3" : "=v"(r) : "v"(a), "s"(K), "v"(b));
  }
  return r;
}
// median(x, -1, 1)
__device__ __forceinline__ int sign3(int x)
{
  int r;
  asm("v_med3_i32 %0, %1, -1, 1" : "=v"(r) : "v"(x));
  return r;
}

// Soft bits in LDS encode the reference's +-LLR_INFINITY (127) as +-SOFT_INF = +-121, the first value past
// +-LLR_MAX: the promotion sum (log_likelihood_ratio.cpp:75: |a + b| > LLR_MAX -> +-infinity) is then a single
// clamp of a + b to +-SOFT_INF, and an infinite soft bit is the only value outside +-LLR_MAX.  Values are
// mapped at the two borders: the partial tail node of the input is clamped to +-SOFT_INF on load (a valid LLR
// is in +-LLR_MAX or +-127), and +-SOFT_INF is written out as +-127 in the soft-bit export.
constexpr int SOFT_INF = LLR_MAX + 1;
// v2c of an infinite soft bit: (s - sat(s)) * INF_BOOST + sat(s - c2v), |.| >= 200 + 25 (|c2v| <= 96), so it is
// never a minimum (> LLR_MAX), keeps its sign, and c2v + v2c always saturates back to +-SOFT_INF.
constexpr int INF_BOOST = 200;

// byte -> the reference's LLR value (+-SOFT_INF -> +-LLR_INFINITY)
__device__ __forceinline__ int soft_export(int v)
{
  return v == SOFT_INF ? LLR_INFINITY : (v == -SOFT_INF ? -LLR_INFINITY : v);
}
__device__ __forceinline__ uint32_t soft_export4(uint32_t w)
{
  uint32_t o = 0;
#pragma unroll
  for (int b = 0; b < 4; ++b) {
    o |= (static_cast<uint32_t>(soft_export(static_cast<int8_t>(w >> (8 * b)))) & 0xffu) << (8 * b);
  }
  return o;
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

// int8 value K of a packed register array.
template <int K, int NW>
__device__ __forceinline__ int byte_get(const uint32_t (&r)[NW])
{
  return static_cast<int>(static_cast<int8_t>(r[K >> 2] >> (8 * (K & 3))));
}
template <int K, int NW>
__device__ __forceinline__ void byte_set(uint32_t (&r)[NW], int c)
{
  // v_perm_b32: byte (K&3) from c, the other bytes from the old word.
  constexpr uint32_t sel = (K & 3) == 0 ? 0x07060500u : (K & 3) == 1 ? 0x07060004u : (K & 3) == 2 ? 0x07000504u : 0x00060504u;
  r[K >> 2]              = __builtin_amdgcn_perm(r[K >> 2], static_cast<uint32_t>(c), sel);
}

// Message of edge K (global edge index): a register byte, or (LDS-resident
// rows) the value gathered into cl[] at the start of the layer.
template <int BG, int K, int NW, int DEG>
__device__ __forceinline__ int c2v_old(const uint32_t (&c2v)[NW], const int (&cl)[DEG], int e)
{
  if constexpr (K < bg_traits<BG>::LDS_EDGES) {
    return cl[e];
  } else {
    return byte_get<K - bg_traits<BG>::LDS_EDGES>(c2v);
  }
}

// Pass 1 for edge E: v2c from the gathered soft bit and the old message, plus
// the check-node statistics (ldpc_decoder_impl.cpp:235 / :290).  An infinite
// soft bit (+-SOFT_INF) yields |v2c| >= 225 here: it can never be a minimum (> 120),
// its sign is right, and in pass 2 c2v + v2c always lands beyond +-120, so the
// promotion sum returns +-SOFT_INF with no separate infinity test.
template <int BG, int E0, int E, int NW, int DEG>
__device__ __forceinline__ int edge_pass1(int            s,
                                          const uint32_t (&c2v)[NW],
                                          const int (&cl)[DEG],
                                          int&           min1,
                                          int&           min2,
                                          int&           idx,
                                          int&           sgn)
{
  // v2c = soft - c2v saturated to +-LLR_MAX; infinite soft bits stay infinite.
  // Branch-free: s - med3(s, +-120) is 0 for a finite soft bit and +-1 for an
  // infinite one, which pushes v2c to +-[225, 320] (|v2c| > 120: never a
  // minimum; |c2v + v2c| >= 129: always promoted to +-SOFT_INF in pass 2).
  const int  v   = mad24<INF_BOOST>(s - sat120(s), sat120(s - c2v_old<BG, E0 + E>(c2v, cl, E)));
  const int  av  = v < 0 ? -v : v;
  const bool lt1 = av < min1;
  idx            = lt1 ? E : idx;
  // new second minimum = median(min1, |v|, min2)
  min2 = med3_op(min1, av, min2);
  min1 = lt1 ? av : min1;
  sgn ^= v;
  return v;
}

// Pass 2 for edge E: the new message (scaled min / second min with the
// extrinsic sign) and the new soft bit, the promotion sum message + v2c
// (ldpc_decoder_impl.cpp:310, :270).  Returns the soft bit; the message goes to
// its register byte or to cl[E].
template <int BG, int E0, int E, int NW, int DEG>
__device__ __forceinline__ int edge_pass2(int v, uint32_t (&c2v)[NW], int (&cl)[DEG], int s1, int s2, int idx, int sgn)
{
  const int mag = (E == idx) ? s2 : s1;
  // extrinsic sign: negate when the sign product without this edge is negative
  const int neg = (sgn ^ v) >> 31;
  const int c   = (mag ^ neg) - neg;
  // promotion sum (log_likelihood_ratio.cpp:75) as one median: |t| > 120 is
  // +-SOFT_INF.  c is always finite, c == -v gives 0 through the plain sum,
  // an infinite v2c (|v| >= 225) always overflows.
  const int out = med3_op(c + v, -SOFT_INF, SOFT_INF);
  if constexpr (E0 + E < bg_traits<BG>::LDS_EDGES) {
    cl[E] = c;
  } else {
    byte_set<E0 + E - bg_traits<BG>::LDS_EDGES>(c2v, c);
  }
  return out;
}

// v2c store of one layer between pass 1 and pass 2: plain registers for light
// rows, 16-bit pairs (read back as SDWA word operands) for degree > 10.
template <int DEG, bool PACKED = (DEG > 10)>
struct v2c_store {
  int v[DEG];
  template <int E>
  __device__ __forceinline__ void put(int x) { v[E] = x; }
  template <int E>
  __device__ __forceinline__ int get() const { return v[E]; }
};
template <int DEG>
struct v2c_store<DEG, true> {
  uint32_t w[(DEG + 1) / 2];
  template <int E>
  __device__ __forceinline__ void put(int x)
  {
    if constexpr ((E & 1) == 0) {
      w[E >> 1] = static_cast<uint32_t>(x) & 0xffffu;
    } else {
      w[E >> 1] = __builtin_amdgcn_perm(static_cast<uint32_t>(x), w[E >> 1], 0x05040100u);
    }
  }
  template <int E>
  __device__ __forceinline__ int get() const
  {
    return static_cast<int>(static_cast<int16_t>(w[E >> 1] >> (16 * (E & 1))));
  }
};

// Gather address of edge E0+E for lane j: var*Z + (j + shift) mod Z, where
// (j + shift - Z) wraps as an unsigned value exactly when j + shift < Z, so the
// mod is one v_min_u32.  Compile-time Z: shift and node offset are literals.
template <int BG, int ZC, int EI>
__device__ __forceinline__ int gather_addr(const_u32_ptr edge, int Z, int j)
{
  if constexpr (ZC > 0) {
    constexpr uint32_t s = const_edge<BG, ZC, EI>::shift;
    return static_cast<int>(__builtin_elementwise_min(static_cast<uint32_t>(j) + s,
                                                      static_cast<uint32_t>(j) + (s - static_cast<uint32_t>(ZC))) +
                            static_cast<uint32_t>(const_edge<BG, ZC, EI>::var * ZC));
  } else {
    const uint32_t d     = edge[EI];
    const uint32_t shift = d >> 16;
    const uint32_t t1    = static_cast<uint32_t>(j) + shift;
    const uint32_t t2    = static_cast<uint32_t>(j) + (shift - static_cast<uint32_t>(Z));
    return static_cast<int>((t1 < t2 ? t1 : t2) + (d & 0xffffu));
  }
}

// Edges of a layer are gathered and reduced in chunks of EDGE_CHUNK with a
// scheduling barrier in between, which bounds the registers a degree-19 row
// keeps in flight next to the message file.
constexpr int EDGE_CHUNK = 5;

// One layer (base-graph check row L) for check row j of the lifted graph.
// Straight-line code: every gather of the layer precedes every scatter, so no
// LDS read waits behind a (possibly aliasing) LDS write of the same layer.
// Idle lanes (j >= Z, only possible when Z is not a multiple of 64) are
// redirected to a private pad.  Rows of degree > 10 recompute their gather
// addresses for the scatter instead of holding 19 of them live.
template <int BG, int ZC, int L, int ARITH, int NW, int... E>
__device__ __forceinline__ void process_layer(lds_i8*       soft,
                                              lds_i8*       c2v_lds,
                                              uint32_t (&c2v)[NW],
                                              const_u32_ptr edge,
                                              int           Z,
                                              int           j,
                                              int           idle_slot,
                                              std::integer_sequence<int, E...>)
{
  constexpr int  E0     = row_start<BG>(L);
  constexpr int  DEG    = sizeof...(E);
  constexpr bool IN_LDS = L < bg_traits<BG>::LDS_ROWS;
  constexpr bool ALL_ON = ZC > 0 && (ZC % 64) == 0;
  constexpr bool KEEP   = DEG <= 10;
  int            ad[DEG];
  int            cl[DEG];
  v2c_store<DEG> vs;
  const int jl = ALL_ON ? j : (idle_slot >= 0 ? 0 : j);
  auto addr = [&](auto ec) {
    constexpr int e = decltype(ec)::value;
    const int     a = gather_addr<BG, ZC, E0 + e>(edge, Z, j);
    return ALL_ON ? a : (idle_slot >= 0 ? idle_slot : a);
  };
  int min1 = LLR_MAX, min2 = LLR_MAX, idx = 0, sgn = 0;
  (
      [&] {
        if constexpr (E % EDGE_CHUNK == 0 && E > 0) {
          __builtin_amdgcn_sched_barrier(0);
        }
        ad[E]       = addr(std::integral_constant<int, E>{});
        const int x = soft[ad[E]];
        if constexpr (IN_LDS) {
          cl[E] = c2v_lds[(E0 + E) * Z + jl];
        }
        vs.template put<E>(edge_pass1<BG, E0, E>(x, c2v, cl, min1, min2, idx, sgn));
      }(),
      ...);
  __builtin_amdgcn_sched_barrier(0);
  const int s1 = scale_mag<ARITH>(min1);
  const int s2 = scale_mag<ARITH>(min2);
  (
      [&] {
        if constexpr (E % EDGE_CHUNK == 0 && E > 0 && !KEEP) {
          __builtin_amdgcn_sched_barrier(0);
        }
        const int snew = edge_pass2<BG, E0, E>(vs.template get<E>(), c2v, cl, s1, s2, idx, sgn);
        const int a    = KEEP ? ad[E] : addr(std::integral_constant<int, E>{});
        soft[a]        = static_cast<int8_t>(snew);
        if constexpr (IN_LDS) {
          if (ALL_ON || idle_slot < 0) {
            c2v_lds[(E0 + E) * Z + j] = static_cast<int8_t>(cl[E]);
          }
        }
      }(),
      ...);
}

// Layers L .. M-1 of one iteration, skipping (uniformly) layers >= nof_layers.
template <int BG, int ZC, int L, int ARITH, int NW>
__device__ __forceinline__ void run_layers(lds_i8*       soft,
                                           lds_i8*       c2v_lds,
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
      // Launder the lane index, graph pointer and Z per layer: the gather
      // addresses are iteration-invariant, and letting the compiler hoist (and
      // keep live) the addresses of later layers would spill the register file.
      asm volatile("" : "+v"(j), "+s"(edge), "+s"(Z));
      process_layer<BG, ZC, L, ARITH>(
          soft, c2v_lds, c2v, edge, Z, j, idle_slot, std::make_integer_sequence<int, bg_traits<BG>::deg(L)>{});
      __syncthreads();
    }
    run_layers<BG, ZC, L + 1, ARITH>(soft, c2v_lds, c2v, edge, Z, j, idle_slot, nof_layers);
  }
}

// Occupancy target: 4 waves per SIMD (<= 128 VGPRs).  A Z=384 workgroup is 6
// waves; two of them fit a CU whatever SIMD the dispatcher starts them on only
// if every SIMD can hold 4 (at 3 per SIMD the second workgroup is mostly refused).
template <int BG, int ZC>
constexpr int waves_per_simd()
{
  return 4;
}

// Check rows per wavefront.  64 for every Z except the compile-time Z=384
// kernel, which may spread its 384 rows over 8 waves of 48 (lanes 48-63 then
// duplicate rows 32-47: identical values to identical addresses), so that two
// workgroups put exactly 2 + 2 waves on every SIMD instead of 2/2/1/1 + 1/1/2/2.
#ifndef Z384_CPW
#define Z384_CPW 48
#endif
constexpr int Z384_CHECKS_PER_WAVE = Z384_CPW;
template <int ZC>
constexpr int checks_per_wave()
{
  return ZC == 384 ? Z384_CHECKS_PER_WAVE : 64;
}
template <int ZC>
constexpr int max_threads()
{
  return ZC == 384 ? 64 * (384 / Z384_CHECKS_PER_WAVE) : MAX_LIFTING_SIZE;
}

template <int BG, int ARITH, int ZC>
__global__ void __launch_bounds__(max_threads<ZC>(), (waves_per_simd<BG, ZC>())) ldpc_decode_kernel(decode_args a, lifted_graph g)
{
  constexpr int NW      = reg_words<BG>();
  constexpr int N_FULL  = bg_traits<BG>::N_FULL;
  lds_i32*      red     = (lds_i32*)(uintptr_t)LDS_RED_OFFSET;
  lds_i8*       soft    = (lds_i8*)(uintptr_t)LDS_SOFT_OFFSET;

  const int  nthr    = blockDim.x;
  constexpr int CPW  = checks_per_wave<ZC>();

  for (uint32_t cb = blockIdx.x; cb < a.nof_cbs; cb += gridDim.x) {
    // lifting size, graph and CRC of this codeblock: the launch's, or its row descriptor's (mixed Z)
    // (row fields made wave-uniform explicitly: they feed scalar operands of the layer code)
    const bool      mixed     = ZC == 0 && a.rows != nullptr;
    const uint32_t  row_z     = mixed ? __builtin_amdgcn_readfirstlane(a.rows[cb].Z) : 0u;
    const uint32_t  row_e     = mixed ? __builtin_amdgcn_readfirstlane(a.rows[cb].edge_off) : 0u;
    const uint32_t  row_c     = mixed ? __builtin_amdgcn_readfirstlane(a.rows[cb].crc_off) : 0u;
    const int       Z         = ZC > 0 ? ZC : (mixed ? static_cast<int>(row_z) : g.Z);
    const uint32_t* edges     = mixed ? a.edges + row_e : a.edges;
    const uint32_t* crc_table = mixed ? (row_c == NO_CRC_ROW ? nullptr : a.crc_table + row_c) : a.crc_table;
    lds_i8*         c2v_lds   = soft + lds_soft_bytes<BG>(Z);
    const int       msg_len   = bg_traits<BG>::K * Z;
    const int       NZ        = N_FULL * Z;
    if (a.skip_flags && *reinterpret_cast<const int32_t*>(a.skip_flags + static_cast<size_t>(cb) * a.skip_stride)) {
      if (threadIdx.x == 0) {
        a.nof_iters[cb] = LDPC_ITERS_SKIPPED; // uniform over the workgroup
      }
      continue;
    }
    // Per-lane values are rebuilt from a laundered thread id in each phase, so
    // the compiler cannot hoist them out of the codeblock loop and keep them
    // live (spilled to scratch) across the iterations.
    int j = threadIdx.x;
    asm volatile("" : "+v"(j));
    const int8_t* in     = a.llrs + static_cast<size_t>(cb) * a.llr_stride;
    const int     n_llrs = a.llr_lens ? static_cast<int>(a.llr_lens[cb]) : static_cast<int>(a.llr_len);
    uint8_t*      out    = a.out + static_cast<size_t>(cb) * a.out_stride;
    const int     obytes = (msg_len + 7) >> 3;

    // ---- input trimming: position of the last non-zero LLR (ldpc_decoder_impl.cpp:86),
    // fused with the soft-bit load (ldpc_decoder_impl.cpp:160 load_soft_bits) when the rows
    // allow 4-byte accesses: soft[2Z + i] = clamp(in[i]) for i < B = (n_llrs / Z) Z, in[i]
    // unclamped for the partial tail node, zero elsewhere.
    if (j == 0) {
      red[0] = -1;
    }
    __syncthreads();
    const bool vec4 = a.aligned4 != 0 && (Z & 3) == 0;
    if (vec4) {
      const int       nw   = n_llrs >> 2;
      const int       B4   = (n_llrs / Z) * Z >> 2; // words of full (clamped) nodes
      const int32_t*  in4  = reinterpret_cast<const int32_t*>(in);
      lds_i32*        s4   = reinterpret_cast<lds_i32*>(soft);
      const int       off4 = (2 * Z) >> 2;
      int             last = -1;
      for (int w = j; w < off4; w += nthr) {
        s4[w] = 0;
      }
      for (int w = j; w < nw; w += nthr) {
        const uint32_t v = static_cast<uint32_t>(in4[w]);
        if (v != 0) {
          last = 4 * w + (31 - __builtin_clz(v)) / 8;
        }
        // full nodes clamped to +-SOFT_CLAMP, the partial tail node to the soft-bit range
        const int lim = w < B4 ? SOFT_CLAMP : SOFT_INF;
        uint32_t  o   = 0;
#pragma unroll
        for (int b = 0; b < 4; ++b) {
          const int x = static_cast<int8_t>(v >> (8 * b));
          o |= (static_cast<uint32_t>(med3_i(x, -lim, lim)) & 0xffu) << (8 * b);
        }
        s4[off4 + w] = static_cast<int32_t>(o);
      }
      // trailing bytes (n_llrs not a multiple of 4), then zeros up to N_FULL Z
      const int tb0 = nw << 2;
      if (j < n_llrs - tb0) {
        const int v = in[tb0 + j];
        if (v != 0) {
          last = max(last, tb0 + j);
        }
        soft[2 * Z + tb0 + j] = static_cast<int8_t>(med3_i(v, -SOFT_INF, SOFT_INF)); // partial tail node
      }
      const int z0 = 2 * Z + n_llrs; // first byte after the data
      for (int i = z0 + j; i < ((z0 + 3) & ~3) && i < NZ; i += nthr) {
        soft[i] = 0;
      }
      for (int w = ((z0 + 3) >> 2) + j; w < (NZ >> 2); w += nthr) {
        s4[w] = 0;
      }
      if (last >= 0) {
        __hip_atomic_fetch_max(&red[0], last, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
    } else {
      int last = -1;
      for (int i = j; i < n_llrs; i += nthr) {
        if (in[i] != 0) {
          last = i;
        }
      }
      if (last >= 0) {
        __hip_atomic_fetch_max(&red[0], last, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
    }
    __syncthreads();
    const int input_size = __builtin_amdgcn_readfirstlane(red[0] + 1);

    if (input_size < msg_len && a.force_decoding) {
      // ldpc_decoder_impl.cpp:92: not enough soft bits -- all ones when no CRC,
      // output left untouched when a CRC is given (as the reference).
      for (int b = j; b < obytes && !crc_table; b += nthr) {
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

    if (!vec4) {
      // ---- load soft bits (ldpc_decoder_impl.cpp:160 load_soft_bits).
      const int nof_full_nodes = n_llrs / Z + 2;
      const int tail           = n_llrs - (nof_full_nodes - 2) * Z;
      for (int node = 0; node < N_FULL; ++node) {
        for (int p = j; p < Z; p += nthr) {
          int v = 0;
          if (node >= 2 && node < nof_full_nodes) {
            v = med3_i(in[(node - 2) * Z + p], -SOFT_CLAMP, SOFT_CLAMP);
          } else if (node == nof_full_nodes && p < tail) {
            v = med3_i(in[(node - 2) * Z + p], -SOFT_INF, SOFT_INF);
          }
          soft[node * Z + p] = static_cast<int8_t>(v);
        }
      }
    }
    // LDS-resident messages start at zero, like the register ones below.
    for (int i = j; i < bg_traits<BG>::LDS_EDGES * Z / 4; i += nthr) {
      reinterpret_cast<lds_i32*>(c2v_lds)[i] = 0;
    }
    int cb_len = input_size + 2 * Z;
    if (cb_len < msg_len + 4 * Z) {
      cb_len = msg_len + 4 * Z;
    }
    const int nof_layers = (cb_len + Z - 1) / Z - bg_traits<BG>::K;
    const int nof_sig    = msg_len - (a.fillers ? a.fillers[cb] : a.nof_filler_bits);
    int       result     = -1;

    // check row of this lane (== j unless rows are spread 48 per wave)
    const int jc        = CPW == 64 ? j : (j >> 6) * CPW + ((j & 63) < CPW ? (j & 63) : (j & 63) - (64 - CPW));
    const bool active   = CPW == 64 ? j < Z : true;
    // idle lanes (Z not a multiple of 64) work on a private pad byte after the messages
    const int idle_slot = active ? -1 : lds_total_bytes<BG>(Z) - LDS_SOFT_OFFSET - 64 + (j & 63);

    // check-to-variable messages start at zero (ldpc_decoder_impl.cpp:244: an
    // uninitialised layer uses v2c = soft, identical to v2c = soft - 0).
    uint32_t c2v[NW];
#pragma unroll
    for (int w = 0; w < NW; ++w) {
      c2v[w] = 0;
    }
    __syncthreads();

    for (int it = 0; it < a.max_iterations; ++it) {
      run_layers<BG, ZC, 0, ARITH>(soft, c2v_lds, c2v, (const_u32_ptr)(edges), Z, jc, idle_slot, nof_layers);

      if (crc_table) {
        // get_hard_bits + CRC early stop (ldpc_decoder_impl.cpp:125): linear
        // CRC, every lane XORs the remainders of its set bits into LDS.
        int jj = threadIdx.x;
        asm volatile("" : "+v"(jj));
        if (jj == 0) {
          red[1] = 0;
          red[2] = 0;
        }
        __syncthreads();
        uint32_t crc = 0, zero = 0;
        // four soft bits per LDS read (msg_len = K_bg Z is even; a 2-bit remainder for odd Z)
        const int nq = msg_len >> 2;
        for (int q = jj; q < nq; q += nthr) {
          const uint32_t w4 = static_cast<uint32_t>(reinterpret_cast<lds_i32*>(soft)[q]);
#pragma unroll
          for (int b = 0; b < 4; ++b) {
            const int sb = static_cast<int8_t>(w4 >> (8 * b));
            const int i  = 4 * q + b;
            zero |= (sb == 0);
            if (i < nof_sig && sb <= 0) {
              crc ^= crc_table[nof_sig - 1 - i];
            }
          }
        }
        for (int i = 4 * nq + jj; i < msg_len; i += nthr) {
          const int sb = soft[i];
          zero |= (sb == 0);
          if (i < nof_sig && sb <= 0) {
            crc ^= crc_table[nof_sig - 1 - i];
          }
        }
        if (crc != 0) {
          __hip_atomic_fetch_xor(reinterpret_cast<lds_u32*>(&red[1]), crc, __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        if (zero != 0) {
          __hip_atomic_fetch_or(reinterpret_cast<lds_u32*>(&red[2]), zero, __ATOMIC_RELAXED,
                                __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        __syncthreads();
        const uint32_t c_all = __builtin_amdgcn_readfirstlane(red[1]);
        const uint32_t z_all = __builtin_amdgcn_readfirstlane(red[2]);
        __syncthreads();
        if (z_all == 0 && c_all == 0) {
          result = it + 1;
          break;
        }
      }
    }

    // ---- hard decision, packed MSB-first (log_likelihood_ratio.cpp hard_decision).
    int je = threadIdx.x;
    asm volatile("" : "+v"(je));
    for (int b = je; b < obytes; b += nthr) {
      uint32_t byte = 0;
      if (b * 8 + 8 <= msg_len) {
        // 8 soft bits from two aligned LDS words; bit k set when soft <= 0
        const uint32_t w0 = static_cast<uint32_t>(reinterpret_cast<lds_i32*>(soft)[2 * b]);
        const uint32_t w1 = static_cast<uint32_t>(reinterpret_cast<lds_i32*>(soft)[2 * b + 1]);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const int sb = static_cast<int8_t>((k < 4 ? w0 : w1) >> (8 * (k & 3)));
          byte |= sb <= 0 ? (0x80u >> k) : 0u;
        }
      } else {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          int i = b * 8 + k;
          if (i < msg_len && soft[i] <= 0) {
            byte |= 0x80u >> k;
          }
        }
      }
      out[b] = static_cast<uint8_t>(byte);
    }
    if (a.soft_out) {
      int8_t* so = a.soft_out + static_cast<size_t>(cb) * NZ;
      for (int i = je; i < NZ; i += nthr) {
        so[i] = static_cast<int8_t>(soft_export(soft[i]));
      }
    }
    if (je == 0) {
      a.nof_iters[cb] = result;
    }
    __syncthreads();
  }
}

// ============================================================================
// High-rate BG1 / Z = 384 decoder: two check rows per lane in packed int16.
//
// A high-rate codeblock (the 256QAM R ~ 0.93 PUSCH of the 100 MHz workloads)
// has input_size <= (20 + MAXL) Z, so the reference processes only its first
// nof_layers <= MAXL layers (ldpc_decoder_impl.cpp:104-113) and touches only
// variable nodes 0 .. 21 + MAXL.  The host selects this kernel when the row
// length bounds nof_layers by MAXL (launch_ldpc_decode), so:
//   * lane t in [0, 192) owns check rows t and t + 192 of every layer; both
//     rows' values travel as the two halves of one VGPR and every check-node
//     operation is one v_pk_* instruction for both (3 waves per codeblock,
//     every lane busy);
//   * the check-to-variable messages of all MAXL layers live in registers
//     (int16 pairs), so LDS holds only the 22 + MAXL soft-bit nodes (10 KiB
//     for MAXL = 4) and several codeblocks share a CU;
//   * gather addresses: for each edge one of the two rows never wraps around
//     the cyclic shift, so its address is the lane index plus an immediate
//     offset; the other takes add, add, min;
//   * no argmin index: an edge takes the second minimum exactly when its
//     |v2c| equals the minimum (when two edges tie, min1 == min2 and the
//     choice does not matter), computed as min(|v2c| - min1, 1);
//   * CRC early stop: the remainder is only tested for zero, so it is
//     accumulated as CRC(msg) x^(K Z - nof_sig) mod g (a unit multiple: zero
//     iff the CRC is zero) from one fixed table order, which makes the four
//     remainders of a soft-bit word one aligned 16-byte load.
// Bit-exact with ldpc_decode_kernel (same per-edge arithmetic, identical
// outputs, iteration counts and final soft bits).
// ============================================================================

typedef short pk16 __attribute__((ext_vector_type(2)));

constexpr int HR_Z       = 384;
constexpr int HR_HALF    = HR_Z / 2; // lanes per codeblock

__device__ __forceinline__ pk16 pk_splat(int v)
{
  return pk16{static_cast<short>(v), static_cast<short>(v)};
}
__device__ __forceinline__ pk16 pk_min(pk16 a, pk16 b)
{
  return __builtin_elementwise_min(a, b);
}
__device__ __forceinline__ pk16 pk_max(pk16 a, pk16 b)
{
  return __builtin_elementwise_max(a, b);
}
__device__ __forceinline__ pk16 pk_clamp(pk16 x, int lim)
{
  return pk_min(pk_max(x, pk_splat(-lim)), pk_splat(lim));
}

template <int MAXL>
__host__ __device__ constexpr int hr_lds_bytes()
{
  return LDS_SOFT_OFFSET + (22 + MAXL) * HR_Z;
}

// LDS byte offset of the soft bit that row (t + KOFF + H) of edge EI reads, H = 0 or 192, t + KOFF < 192.
// One of the two rows of an edge never wraps: its address is t + literal.
template <int EI, int H, int KOFF = 0>
__device__ __forceinline__ uint32_t hr_addr(uint32_t t)
{
  constexpr uint32_t s    = (const_edge<1, HR_Z, EI>::shift + H) % HR_Z;
  constexpr uint32_t base = LDS_SOFT_OFFSET + const_edge<1, HR_Z, EI>::var * HR_Z;
  if constexpr (s <= HR_HALF) {
    return t + (base + KOFF + s); // t + KOFF < 192: t + KOFF + s < 384
  } else {
    return __builtin_elementwise_min(t + (KOFF + s), t + (KOFF + s - HR_Z)) + base;
  }
}

// Compile-time loop: f(std::integral_constant<int, 0>) ... f(std::integral_constant<int, N - 1>).
template <int N, typename F, int... I>
__device__ __forceinline__ void static_for_impl(F&& f, std::integer_sequence<int, I...>)
{
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, typename F>
__device__ __forceinline__ void static_for(F&& f)
{
  static_for_impl<N>(f, std::make_integer_sequence<int, N>{});
}

// Check-to-variable messages of the first MAXL layers, register resident: one int16 pair per edge
// (default), or (HR_PACK8) two edges per VGPR as int8 pairs, edge 2w in the high byte and edge 2w+1
// in the low byte of each 16-bit half, unpacked with one or two packed shifts and repacked with one
// v_perm_b32.  Measured (tools/ldpc_hr_probe.py, 4,544 codeblocks): the layers are VALU-bound, and
// the 2.5 extra VALU per edge of the int8 form cost more (75.6 vs 70.2 us per iteration) than its
// occupancy gain (98 vs 128 VGPRs) returns; the edge chunking (5, 10, 19) changes nothing.
#ifndef HR_PACK8
#define HR_PACK8 0
#endif
template <int NE, bool PACK8 = HR_PACK8>
struct hr_msgs {
  pk16 m[NE];
  __device__ __forceinline__ void zero()
  {
#pragma unroll
    for (int e = 0; e < NE; ++e) {
      m[e] = pk16{0, 0};
    }
  }
  template <int E>
  __device__ __forceinline__ pk16 get() const { return m[E]; }
  template <int E>
  __device__ __forceinline__ void set(pk16 c) { m[E] = c; }
};
template <int NE>
struct hr_msgs<NE, true> {
  uint32_t w[(NE + 1) / 2];
  __device__ __forceinline__ void zero()
  {
#pragma unroll
    for (int e = 0; e < (NE + 1) / 2; ++e) {
      w[e] = 0;
    }
  }
  template <int E>
  __device__ __forceinline__ pk16 get() const
  {
    const pk16 x = __builtin_bit_cast(pk16, w[E >> 1]);
    if constexpr ((E & 1) == 0) {
      return x >> 8;
    } else {
      return (x << 8) >> 8;
    }
  }
  template <int E>
  __device__ __forceinline__ void set(pk16 c)
  {
    const uint32_t cv = __builtin_bit_cast(uint32_t, c);
    // v_perm_b32(src0 = c, src1 = w): selector bytes 0-3 pick w, 4-7 pick c
    w[E >> 1] = __builtin_amdgcn_perm(cv, w[E >> 1], (E & 1) == 0 ? 0x06020400u : 0x03060104u);
    // pin the repacked word here: left alone the compiler sinks the v_perm_b32 to the end of the
    // iteration and keeps every new message unpacked (and spilled) until then
    asm volatile("" : "+v"(w[E >> 1]));
  }
};

template <int ARITH>
__device__ __forceinline__ pk16 pk_scale(pk16 m)
{
  return pk16{static_cast<short>(scale_mag<ARITH>(m.x)), static_cast<short>(scale_mag<ARITH>(m.y))};
}

typedef unsigned short pku16 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ pk16 as_pk(uint32_t w)
{
  return __builtin_bit_cast(pk16, w);
}
__device__ __forceinline__ uint32_t as_u32(pk16 v)
{
  return __builtin_bit_cast(uint32_t, v);
}
// per 16-bit half: 0 if the half is zero, 1 otherwise -- one v_pk_min_u16 kept opaque: the compiler otherwise
// turns min(x, 1) into a per-half compare and v_cndmask selects (no packed select exists)
__device__ __forceinline__ pk16 pk_nonzero(uint32_t w)
{
  uint32_t r;
  // op_sel_hi:[1,0]: the high half also reads the inline constant's low 16 bits (a splat 1)
  asm("v_pk_min_u16 %0, %1, 1 op_sel_hi:[1,0]" : "=v"(r) : "v"(w));
  return __builtin_bit_cast(pk16, r);
}

// scale_mag of both halves in 16-bit arithmetic (minima are <= LLR_MAX; both forms equal scale_mag on 0..120):
// ARITH_SIMD floor(m 52428 / 2^16) = max((205 m - 52) >> 8, 0), ARITH_GENERIC round(0.8 m) = (205 m + 102) >> 8
template <int ARITH>
__device__ __forceinline__ pk16 pk_scale16(pk16 m)
{
  if constexpr (ARITH == ARITH_GENERIC) {
    return (m * pk_splat(205) + pk_splat(102)) >> 8;
  } else {
    return pk_max((m * pk_splat(205) - pk_splat(52)) >> 8, pk_splat(0));
  }
}

// a * b + c in both halves as one v_pk_mad_u16 (the low 16 bits of the product are sign-agnostic); opaque, so
// the compiler does not split it into a multiply and a subtract
__device__ __forceinline__ pk16 pk_mad(pk16 a, pk16 b, pk16 c)
{
  uint32_t r;
  asm("v_pk_mad_u16 %0, %1, %2, %3" : "=v"(r) : "v"(as_u32(a)), "v"(as_u32(b)), "v"(as_u32(c)));
  return as_pk(r);
}
// a * 32 + E (E an inline constant), one v_pk_mad_u16
template <int E>
__device__ __forceinline__ pk16 pk_key(pk16 a)
{
  uint32_t r;
  asm("v_pk_mad_u16 %0, %1, 32, %2 op_sel_hi:[1,0,0]" : "=v"(r) : "v"(as_u32(a)), "i"(E));
  return as_pk(r);
}

// Edges per scheduling group in the two passes of a layer (bounds the gathered values in flight).
#ifndef HR_CHUNK1
#define HR_CHUNK1 5
#endif
#ifndef HR_CHUNK2
#define HR_CHUNK2 5
#endif
#ifndef HR_PIN_X
#define HR_PIN_X 0
#endif
// argmin as the low bits of min(|v2c| << 5 | e) (as the full-length kernel below): pass 2 tests e == idx with two
// instructions instead of recomputing |v2c| - min1 (four)
#ifndef HR_KEYS
#define HR_KEYS 0
#endif

// One layer (base-graph row L, global edges E0 .. E0 + DEG - 1) for the NP row pairs of lane t:
// rows t + k T and t + k T + 192, T = 192 / NP, k < NP (message of edge e, pair k: index e NP + k).
//
// Instruction scheduling (gfx950): a packed-math (VOP3P) result read by the very next VOP3P instruction costs a
// hazard s_nop, and those nops took ~35 % of the issue slots of a dependent v_pk_* chain at 4 waves per SIMD
// (scratch microbenchmark; the kernel is VALU-issue bound at ~4.3 cycles per v_pk_* wave instruction).  So the
// check-node reduction runs as two independent chains (even / odd edges, merged at the end of pass 1), and pass 2
// leaves the scheduler free to interleave consecutive edges (no ordering fence between them).
template <int L, int ARITH, int NP, typename MSGS, int... E>
__device__ __forceinline__ void hr_layer(lds_i8* lds, MSGS& c2v, uint32_t t, std::integer_sequence<int, E...>)
{
  constexpr int E0  = row_start<1>(L);
  constexpr int DEG = sizeof...(E);
  constexpr int T   = HR_HALF / NP;
  pk16          v[DEG][NP];
  pk16          min1[2][NP], min2[2][NP], sgn[NP];
#pragma unroll
  for (int k = 0; k < NP; ++k) {
    // HR_KEYS: minima of the keys |v2c| << 5 | e (the initial key stands for LLR_MAX with no edge index)
    min1[0][k] = min1[1][k] = pk_splat(HR_KEYS ? LLR_MAX * 32 + 31 : LLR_MAX);
    min2[0][k] = min2[1][k] = pk_splat(HR_KEYS ? LLR_MAX * 32 + 31 : LLR_MAX);
    sgn[k]                  = pk_splat(0);
  }
  // pass 1 (ldpc_decoder_impl.cpp:235 / :290): v2c and the check-node statistics
  (
      [&] {
        if constexpr (E % HR_CHUNK1 == 0 && E > 0) {
          __builtin_amdgcn_sched_barrier(0);
        }
        static_for<NP>([&](auto kc) {
          constexpr int k = decltype(kc)::value;
          constexpr int h = E & 1; // reduction chain
          const pk16    s = pk16{static_cast<short>(lds[hr_addr<E0 + E, 0, k * T>(t)]),
                              static_cast<short>(lds[hr_addr<E0 + E, HR_HALF, k * T>(t)])};
          const pk16 sat = pk_clamp(s, LLR_MAX);
          // infinite soft bits (+-SOFT_INF) push |v2c| beyond 220 (see edge_pass1)
          const pk16 x = (s - sat) * pk_splat(INF_BOOST) + pk_clamp(s - c2v.template get<(E0 + E) * NP + k>(), LLR_MAX);
#if HR_KEYS
          const pk16 ax = pk_key<E>(__builtin_elementwise_abs(x));
#else
          const pk16 ax = __builtin_elementwise_abs(x);
#endif
          min2[h][k]    = pk_max(min1[h][k], pk_min(ax, min2[h][k])); // median(min1, |v|, min2)
          min1[h][k]    = pk_min(min1[h][k], ax);
          sgn[k] ^= x;
          v[E][k] = x;
        });
      }(),
      ...);
  __builtin_amdgcn_sched_barrier(0);
  pk16 m1[NP], s1[NP], s2[NP], d12[NP];
#pragma unroll
  for (int k = 0; k < NP; ++k) {
    // merge the two chains: min1 = min(a1, b1), min2 = min(max(a1, b1), min(a2, b2))
    m1[k]  = pk_min(min1[0][k], min1[1][k]);
    const pk16 mn2 = pk_min(pk_max(min1[0][k], min1[1][k]), pk_min(min2[0][k], min2[1][k]));
#if HR_KEYS
    s1[k]  = pk_scale16<ARITH>(m1[k] >> 5);
    s2[k]  = pk_scale16<ARITH>(mn2 >> 5);
    m1[k]  = as_pk(as_u32(m1[k]) & 0x001f001fu); // index of the first minimum
#else
    s1[k]  = pk_scale<ARITH>(m1[k]);
    s2[k]  = pk_scale<ARITH>(mn2);
#endif
    d12[k] = s1[k] - s2[k];
  }
  // pass 2 (ldpc_decoder_impl.cpp:310, :270): new message and promotion sum
  (
      [&] {
        if constexpr (E % HR_CHUNK2 == 0 && E > 0) {
          __builtin_amdgcn_sched_barrier(0);
        }
        static_for<NP>([&](auto kc) {
          constexpr int k = decltype(kc)::value;
          pk16          x = v[E][k];
#if HR_PIN_X
          // opaque: otherwise |x| of pass 1 is kept live (19 more VGPRs) instead of being recomputed
          asm volatile("" : "+v"(x));
#endif
#if HR_KEYS
          const pk16 f   = pk_nonzero(as_u32(m1[k]) ^ (static_cast<uint32_t>(E) * 0x10001u)); // 0: edge E holds min1
#else
          const pk16 f   = pk_min(__builtin_elementwise_abs(x) - m1[k], pk_splat(1)); // 0: this edge holds min1
#endif
          const pk16 mag = f * d12[k] + s2[k];
          const pk16 neg = (sgn[k] ^ x) >> 15;
          const pk16 c   = (mag ^ neg) - neg;
          // promotion sum: |c + x| > LLR_MAX is +-SOFT_INF (see edge_pass2)
          const pk16 out = pk_clamp(c + x, SOFT_INF);
          c2v.template set<(E0 + E) * NP + k>(c);
          lds[hr_addr<E0 + E, 0, k * T>(t)]       = static_cast<int8_t>(out.x);
          lds[hr_addr<E0 + E, HR_HALF, k * T>(t)] = static_cast<int8_t>(out.y);
        });
      }(),
      ...);
}

// hr_layer with the edges taken two at a time (HR_PAIRS=1, an r06 A/B kept for the record, not the default): each
// packed operation of an edge pair is two independent v_pk_* instructions on a four-element vector (edge a's row
// pair, edge b's row pair), so consecutive VOP3P instructions of one wave no longer depend on each other and the
// hazard s_nop between dependent packed instructions goes (878 -> 224 in the headline decoder's code).  The even
// edges feed the low half's reduction chain and the odd edges the high half's, exactly the two chains of hr_layer,
// so outputs and iteration counts are identical (decoder and golden tests pass).  Measured slower: 388 vs 345 us
// per in-step launch (profiles/r06_ldpc_pairs_ab.md) -- the pairs cost 80 extra v_perm_b32 and ~32 VGPRs of
// scratch spills, and with eight waves per SIMD the nops of one wave were already covered by the others' issue.
#ifndef HR_PAIRS
#define HR_PAIRS 0
#endif
#ifndef HR_PCHUNK
#define HR_PCHUNK 3
#endif
typedef short pk4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ pk4 pk_cat(pk16 a, pk16 b)
{
  return __builtin_shufflevector(a, b, 0, 1, 2, 3);
}
__device__ __forceinline__ pk16 pk_lo(pk4 v)
{
  return __builtin_shufflevector(v, v, 0, 1);
}
__device__ __forceinline__ pk16 pk_hi(pk4 v)
{
  return __builtin_shufflevector(v, v, 2, 3);
}
__device__ __forceinline__ pk4 pk4_splat(int v)
{
  const short x = static_cast<short>(v);
  return pk4{x, x, x, x};
}
__device__ __forceinline__ pk4 pk4_clamp(pk4 x, int lim)
{
  return __builtin_elementwise_min(__builtin_elementwise_max(x, pk4_splat(-lim)), pk4_splat(lim));
}

template <int L, int ARITH, int NP, typename MSGS, int... P>
__device__ __forceinline__ void hr_layer_pairs(lds_i8* lds, MSGS& c2v, uint32_t t, std::integer_sequence<int, P...>)
{
  static_assert(!HR_KEYS, "the paired layer keeps |v2c| minima");
  constexpr int E0  = row_start<1>(L);
  constexpr int DEG = bg_traits<1>::deg(L);
  constexpr int T   = HR_HALF / NP;
  pk16          v[DEG][NP];
  pk4           mn1[NP], mn2[NP], sg[NP]; // low half: the even edges' chain, high half: the odd edges'
#pragma unroll
  for (int k = 0; k < NP; ++k) {
    mn1[k] = mn2[k] = pk4_splat(LLR_MAX);
    sg[k]           = pk4_splat(0);
  }
  // pass 1 (ldpc_decoder_impl.cpp:235 / :290): v2c and the check-node statistics
  (
      [&] {
        constexpr int Ea = 2 * P, Eb = 2 * P + 1;
        if constexpr (P % HR_PCHUNK == 0 && P > 0) {
          __builtin_amdgcn_sched_barrier(0);
        }
        static_for<NP>([&](auto kc) {
          constexpr int k  = decltype(kc)::value;
          const pk16    sa = pk16{static_cast<short>(lds[hr_addr<E0 + Ea, 0, k * T>(t)]),
                               static_cast<short>(lds[hr_addr<E0 + Ea, HR_HALF, k * T>(t)])};
          if constexpr (Eb < DEG) {
            const pk16 sb  = pk16{static_cast<short>(lds[hr_addr<E0 + Eb, 0, k * T>(t)]),
                                 static_cast<short>(lds[hr_addr<E0 + Eb, HR_HALF, k * T>(t)])};
            const pk4  s   = pk_cat(sa, sb);
            const pk4  c   = pk_cat(c2v.template get<(E0 + Ea) * NP + k>(), c2v.template get<(E0 + Eb) * NP + k>());
            const pk4  sat = pk4_clamp(s, LLR_MAX);
            // infinite soft bits (+-SOFT_INF) push |v2c| beyond 220 (see edge_pass1)
            const pk4 x  = (s - sat) * pk4_splat(INF_BOOST) + pk4_clamp(s - c, LLR_MAX);
            const pk4 ax = __builtin_elementwise_abs(x);
            mn2[k]       = __builtin_elementwise_max(mn1[k], __builtin_elementwise_min(ax, mn2[k]));
            mn1[k]       = __builtin_elementwise_min(mn1[k], ax);
            sg[k] ^= x;
            v[Ea][k] = pk_lo(x);
            v[Eb][k] = pk_hi(x);
          } else { // the last edge of an odd degree: the even chain
            const pk16 sat = pk_clamp(sa, LLR_MAX);
            const pk16 x = (sa - sat) * pk_splat(INF_BOOST) + pk_clamp(sa - c2v.template get<(E0 + Ea) * NP + k>(), LLR_MAX);
            const pk16 ax = __builtin_elementwise_abs(x);
            pk16       a1 = pk_lo(mn1[k]), a2 = pk_lo(mn2[k]);
            a2            = pk_max(a1, pk_min(ax, a2));
            a1            = pk_min(a1, ax);
            mn1[k]        = pk_cat(a1, pk_hi(mn1[k]));
            mn2[k]        = pk_cat(a2, pk_hi(mn2[k]));
            sg[k]         = pk_cat(pk_lo(sg[k]) ^ x, pk_hi(sg[k]));
            v[Ea][k]      = x;
          }
        });
      }(),
      ...);
  __builtin_amdgcn_sched_barrier(0);
  pk4 m1q[NP], s2q[NP], d12q[NP], sgq[NP];
#pragma unroll
  for (int k = 0; k < NP; ++k) {
    // merge the two chains: min1 = min(a1, b1), min2 = min(max(a1, b1), min(a2, b2))
    const pk16 a1 = pk_lo(mn1[k]), b1 = pk_hi(mn1[k]);
    const pk16 m1  = pk_min(a1, b1);
    const pk16 mn2v = pk_min(pk_max(a1, b1), pk_min(pk_lo(mn2[k]), pk_hi(mn2[k])));
    const pk16 s1  = pk_scale<ARITH>(m1);
    const pk16 s2  = pk_scale<ARITH>(mn2v);
    const pk16 sgn = pk_lo(sg[k]) ^ pk_hi(sg[k]);
    m1q[k]         = pk_cat(m1, m1);
    s2q[k]         = pk_cat(s2, s2);
    d12q[k]        = pk_cat(s1 - s2, s1 - s2);
    sgq[k]         = pk_cat(sgn, sgn);
  }
  // pass 2 (ldpc_decoder_impl.cpp:310, :270): new message and promotion sum
  (
      [&] {
        constexpr int Ea = 2 * P, Eb = 2 * P + 1;
        if constexpr (P % HR_PCHUNK == 0 && P > 0) {
          __builtin_amdgcn_sched_barrier(0);
        }
        static_for<NP>([&](auto kc) {
          constexpr int k = decltype(kc)::value;
          if constexpr (Eb < DEG) {
            const pk4 x   = pk_cat(v[Ea][k], v[Eb][k]);
            const pk4 f   = __builtin_elementwise_min(__builtin_elementwise_abs(x) - m1q[k], pk4_splat(1));
            const pk4 mag = f * d12q[k] + s2q[k];
            const pk4 neg = (sgq[k] ^ x) >> 15;
            const pk4 c   = (mag ^ neg) - neg;
            // promotion sum: |c + x| > LLR_MAX is +-SOFT_INF (see edge_pass2)
            const pk4 out = pk4_clamp(c + x, SOFT_INF);
            c2v.template set<(E0 + Ea) * NP + k>(pk_lo(c));
            c2v.template set<(E0 + Eb) * NP + k>(pk_hi(c));
            lds[hr_addr<E0 + Ea, 0, k * T>(t)]       = static_cast<int8_t>(out.x);
            lds[hr_addr<E0 + Ea, HR_HALF, k * T>(t)] = static_cast<int8_t>(out.y);
            lds[hr_addr<E0 + Eb, 0, k * T>(t)]       = static_cast<int8_t>(out.z);
            lds[hr_addr<E0 + Eb, HR_HALF, k * T>(t)] = static_cast<int8_t>(out.w);
          } else {
            const pk16 x   = v[Ea][k];
            const pk16 f   = pk_min(__builtin_elementwise_abs(x) - pk_lo(m1q[k]), pk_splat(1));
            const pk16 mag = f * pk_lo(d12q[k]) + pk_lo(s2q[k]);
            const pk16 neg = (pk_lo(sgq[k]) ^ x) >> 15;
            const pk16 c   = (mag ^ neg) - neg;
            const pk16 out = pk_clamp(c + x, SOFT_INF);
            c2v.template set<(E0 + Ea) * NP + k>(c);
            lds[hr_addr<E0 + Ea, 0, k * T>(t)]       = static_cast<int8_t>(out.x);
            lds[hr_addr<E0 + Ea, HR_HALF, k * T>(t)] = static_cast<int8_t>(out.y);
          }
        });
      }(),
      ...);
}

template <int L, int MAXL, int ARITH, int NP, typename MSGS>
__device__ __forceinline__ void hr_layers(lds_i8* lds, MSGS& c2v, uint32_t t, int nof_layers)
{
  if constexpr (L < MAXL) {
    if (L < 4 || L < nof_layers) {
      asm volatile("" : "+v"(t));
      if constexpr (HR_PAIRS && !HR_KEYS) {
        hr_layer_pairs<L, ARITH, NP>(lds, c2v, t, std::make_integer_sequence<int, (bg_traits<1>::deg(L) + 1) / 2>{});
      } else {
        hr_layer<L, ARITH, NP>(lds, c2v, t, std::make_integer_sequence<int, bg_traits<1>::deg(L)>{});
      }
      if constexpr (NP == 1) {
        __syncthreads();
      } else {
        // one wave per codeblock: the wave's LDS instructions execute in issue order, so the next layer's
        // gathers see this layer's scatters of every lane; only the compiler must not move LDS accesses
        // across the layer boundary (it cannot see the cross-lane dependencies)
        asm volatile("" ::: "memory");
      }
    }
    hr_layers<L + 1, MAXL, ARITH, NP>(lds, c2v, t, nof_layers);
  }
}

// ============================================================================
// Full-length BG1 / Z = 384 codeblocks (any layer count, e.g. the rate-1/3 codeblocks of configs[1]): the
// high-rate layout above -- two check rows per lane in packed int16, three waves per codeblock, no argmin
// index register -- with the check-to-variable messages of all 46 layers held COMPRESSED in registers.
//
// A min-sum message is a function of four values of its check row (ldpc_decoder_impl.cpp:290-310): the scaled
// minima s1 <= s2, the edge index of the first minimum and the sign of each edge's message, c_e = +-(e == idx ?
// s2 : s1).  Per row pair (rows t and t + 192, one per 16-bit half) the registers hold exactly that:
//   word A: s2 (bits 0-6) | idx (bits 7-11) | signs of edges 0-3 (bits 12-15)
//   word B: s2 - s1 (bits 0-6) | signs of edges 4-12 (bits 7-15)
//   word C (the degree-19 rows only): signs of edges 13-18 (bits 0-5)
// 96 VGPRs for all 46 layers, where int16 messages would take 316 and int8 pairs 158: the kernel runs at
// three waves per SIMD, four codeblocks (12 waves, 4 x 26 KiB of soft bits) per CU with every SIMD equally
// loaded.  Rebuilding an old message costs 7 packed instructions (index test, min-select, sign extract, sign
// apply); the index of the first minimum comes out of pass 1 as the low bits of min(|v2c| << 5 | e).
// Bit-exact with ldpc_decode_kernel (same per-edge arithmetic; identical outputs, iteration counts, final
// soft bits).
// ============================================================================

// compressed state words of BG1 layer l, and the offset of layer l's words
constexpr int fr_words(int l)
{
  return bg_traits<1>::deg(l) > 13 ? 3 : 2;
}
constexpr int fr_off(int l)
{
  int s = 0;
  for (int i = 0; i < l; ++i) {
    s += fr_words(i);
  }
  return s;
}
constexpr int FR_STATE_WORDS = fr_off(bg_traits<1>::M);
static_assert(FR_STATE_WORDS == 96, "BG1 compressed message state");
// word and bit (of each 16-bit half) holding the sign of edge e of a row
constexpr int fr_sign_word(int e)
{
  return e < 4 ? 0 : (e < 13 ? 1 : 2);
}
constexpr int fr_sign_bit(int e)
{
  return e < 4 ? 12 + e : (e < 13 ? e + 3 : e - 13);
}

// v_pk_mad_u16 as opaque asm for the old-message magnitude and the argmin key (fewer instructions; 1 = on)
#ifndef FR_ASM_MAD
#define FR_ASM_MAD 1
#endif
#ifndef FR_SIGN_SHIFT
#define FR_SIGN_SHIFT 1
#endif
#ifndef FR_KEEP_ADDR
#define FR_KEEP_ADDR 19
#endif

// compressed message state of the first NW / (2 or 3) layers (all 46: fr_state)
template <int NW>
struct fr_state_n {
  uint32_t w[NW];
  __device__ __forceinline__ void zero()
  {
#pragma unroll
    for (int i = 0; i < NW; ++i) {
      w[i] = 0;
    }
  }
};
using fr_state = fr_state_n<FR_STATE_WORDS>;

// One layer (BG1 row L) for the row pair of lane t, messages rebuilt from / folded into the compressed state.
template <int L, int ARITH, typename ST, int... E>
__device__ __forceinline__ void fr_layer(lds_i8* lds, ST& st, uint32_t t, std::integer_sequence<int, E...>)
{
  constexpr int  E0  = row_start<1>(L);
  constexpr int  DEG = sizeof...(E);
  constexpr int  O   = fr_off(L);
  constexpr bool W3  = fr_words(L) == 3;
  const uint32_t wold[3] = {st.w[O], st.w[O + 1], W3 ? st.w[O + 2] : 0u};
  const pk16     s2o     = as_pk(wold[0] & 0x007f007fu);
  const uint32_t imo     = wold[0] & 0x0f800f80u;
  const pk16     dno     = pk_splat(0) - as_pk(wold[1] & 0x007f007fu); // s1 - s2 of the old messages
  pk16           v[DEG];
  pk16           min1[2], min2[2];
  pk16           sgn = pk_splat(0);
  // keys |v2c| << 5 | e; the initial key stands for the reference's LLR_MAX start value (no edge index)
  min1[0] = min1[1] = min2[0] = min2[1] = pk_splat(LLR_MAX * 32 + 31);
  // pass 1 (ldpc_decoder_impl.cpp:235 / :290): old message, v2c, check-node statistics
  (
      [&] {
        if constexpr (E % HR_CHUNK1 == 0 && E > 0) {
          __builtin_amdgcn_sched_barrier(0);
        }
        constexpr int h = E & 1; // reduction chain
        const pk16    s = pk16{static_cast<short>(lds[hr_addr<E0 + E, 0>(t)]),
                            static_cast<short>(lds[hr_addr<E0 + E, HR_HALF>(t)])};
        // old message: +-(e == idx ? s2 : s1)
        const pk16 f   = pk_nonzero(imo ^ ((static_cast<uint32_t>(E) << 7) * 0x10001u));
#if FR_ASM_MAD
        const pk16 mag = pk_mad(f, dno, s2o);
#else
        const pk16 mag = f * dno + s2o;
#endif
        const pk16 ng  = (as_pk(wold[fr_sign_word(E)]) << pk_splat(15 - fr_sign_bit(E))) >> 15;
        const pk16 c   = (mag ^ ng) - ng;
        const pk16 sat = pk_clamp(s, LLR_MAX);
        // infinite soft bits (+-SOFT_INF) push |v2c| beyond 220 (see edge_pass1)
        const pk16 x   = (s - sat) * pk_splat(INF_BOOST) + pk_clamp(s - c, LLR_MAX);
#if FR_ASM_MAD
        const pk16 key = pk_key<E>(__builtin_elementwise_abs(x));
#else
        const pk16 key = __builtin_elementwise_abs(x) * pk_splat(32) + pk_splat(E);
#endif
        min2[h]        = pk_max(min1[h], pk_min(key, min2[h])); // median(min1, key, min2)
        min1[h]        = pk_min(min1[h], key);
        sgn ^= x;
        v[E] = x;
      }(),
      ...);
  __builtin_amdgcn_sched_barrier(0);
  const pk16     k1  = pk_min(min1[0], min1[1]);
  const pk16     k2  = pk_min(pk_max(min1[0], min1[1]), pk_min(min2[0], min2[1]));
  const pk16     s1  = pk_scale16<ARITH>(k1 >> 5);
  const pk16     s2  = pk_scale16<ARITH>(k2 >> 5);
  const pk16     d12 = s1 - s2;
  const uint32_t idx = as_u32(k1) & 0x001f001fu;
  uint32_t       acc[3] = {(idx << 7) | as_u32(s2), as_u32(s2 - s1), 0u};
  if constexpr (DEG > FR_KEEP_ADDR) {
    // rows of high degree recompute their scatter addresses instead of holding DEG of them live
    asm volatile("" : "+v"(t));
  }
  // pass 2 (ldpc_decoder_impl.cpp:310, :270): new message, promotion sum, new state
  (
      [&] {
        if constexpr (E % HR_CHUNK2 == 0 && E > 0) {
          __builtin_amdgcn_sched_barrier(0);
        }
        const pk16 x   = v[E];
        const pk16 f   = pk_nonzero(idx ^ (static_cast<uint32_t>(E) * 0x10001u)); // 0: this edge holds min1
        const pk16 mag = f * d12 + s2;
        const pk16 sx  = sgn ^ x;
        const pk16 ng  = sx >> 15;
        const pk16 c   = (mag ^ ng) - ng;
        // promotion sum: |c + x| > LLR_MAX is +-SOFT_INF (see edge_pass2)
        const pk16 out = pk_clamp(c + x, SOFT_INF);
#if FR_SIGN_SHIFT
        // sign bit into both halves of the state word: (sx >>> 15) << bit, one v_lshl_or_b32 with an inline shift
        const uint32_t nb = __builtin_bit_cast(uint32_t, __builtin_bit_cast(pku16, sx) >> 15);
        acc[fr_sign_word(E)] |= nb << fr_sign_bit(E);
#else
        // sign mask of both halves into the state word: one v_and_or_b32 (mask constant in an SGPR)
        acc[fr_sign_word(E)] |= as_u32(ng) & ((1u << fr_sign_bit(E)) * 0x10001u);
#endif
        lds[hr_addr<E0 + E, 0>(t)]       = static_cast<int8_t>(out.x);
        lds[hr_addr<E0 + E, HR_HALF>(t)] = static_cast<int8_t>(out.y);
      }(),
      ...);
  // pin the assembled words here: left alone the compiler sinks the sign-bit ORs past the layer's join and
  // keeps (and spills) the separate bits until the next iteration reads the words
  asm volatile("" : "+v"(acc[0]), "+v"(acc[1]));
  st.w[O]     = acc[0];
  st.w[O + 1] = acc[1];
  if constexpr (W3) {
    asm volatile("" : "+v"(acc[2]));
    st.w[O + 2] = acc[2];
  }
}

// Barrier groups of BG1 layers (r06): consecutive layers that share no variable node read and write disjoint soft
// bits, so no workgroup barrier is needed between them -- the result is the sequential one, bit for bit.  A layer
// starts a new group when one of its columns is a column of a layer of the current group.  BG1 (the lower part is
// built of orthogonal row pairs): 32 groups for 46 layers, layers 16-17, 20-21, 22-23, ..., 44-45 paired.
#ifndef FR_GROUPS
#define FR_GROUPS 1
#endif
template <int BG>
struct bg_groups_t {
  int first[bg_traits<BG>::M] = {}; // first layer of the group of layer l
  int count                   = 0;
  constexpr bg_groups_t()
  {
    int rs[bg_traits<BG>::M + 1] = {};
    for (int l = 0; l < bg_traits<BG>::M; ++l) {
      rs[l + 1] = rs[l] + bg_traits<BG>::deg(l);
    }
    auto col = [](int e) { return BG == 1 ? tables::SRS_BG1_EDGES[e][1] : tables::SRS_BG2_EDGES[e][1]; };
    int  gs  = 0;
    for (int l = 0; l < bg_traits<BG>::M; ++l) {
      bool share = l == 0;
      for (int a = gs; a < l && !share; ++a) {
        for (int i = rs[a]; i < rs[a + 1] && !share; ++i) {
          for (int j = rs[l]; j < rs[l + 1] && !share; ++j) {
            share = col(i) == col(j);
          }
        }
      }
      if (share) {
        gs = l;
        ++count;
      }
      first[l] = gs;
    }
  }
};
template <int BG>
inline constexpr bg_groups_t<BG> BG_GROUPS{};
template <int BG>
constexpr int bg_group_start(int l)
{
  return BG_GROUPS<BG>.first[l];
}
constexpr int bg1_group_start(int l)
{
  return bg_group_start<1>(l);
}
static_assert(BG_GROUPS<1>.count == 32 && BG_GROUPS<2>.count == 28, "BG1 / BG2 barrier groups of the decoders");

template <int L, int ARITH, int MAXL, typename ST>
__device__ __forceinline__ void fr_layers(lds_i8* lds, ST& st, uint32_t t, int nof_layers)
{
  if constexpr (L < MAXL) {
    // laundered per layer: otherwise the 42 layer conditions are hoisted out of the iteration loop as 64-bit
    // lane masks (84 SGPRs, spilled)
    asm volatile("" : "+s"(nof_layers));
    if (L < 4 || L < nof_layers) { // uniform; nof_layers >= 4
      asm volatile("" : "+v"(t));
      fr_layer<L, ARITH>(lds, st, t, std::make_integer_sequence<int, bg_traits<1>::deg(L)>{});
      // a barrier before the next layer unless it continues this one's group (and runs); always one after the last
      constexpr bool next_joins = FR_GROUPS && L + 1 < MAXL && bg1_group_start(L + 1) != L + 1;
      if (!next_joins || !(L + 1 < 4 || L + 1 < nof_layers)) {
        __syncthreads();
      } else {
        asm volatile("" ::: "memory"); // (program order of this lane's LDS accesses; the layers touch disjoint bytes)
      }
    }
    fr_layers<L + 1, ARITH, MAXL>(lds, st, t, nof_layers);
  }
}

// NP row pairs per lane: NP = 1 -> 192 threads (3 waves) per codeblock, NP = 3 -> one wave per codeblock
// (no workgroup barriers, three independent pair streams per lane).
#ifndef HR_WAVES
#define HR_WAVES 4
#endif
#ifndef FR_WAVES
#define FR_WAVES 3
#endif
// HR_CMP: the high-rate kernel holds its MAXL layers' messages compressed (fr_layer) instead of as int16 pairs
#ifndef HR_CMP
#define HR_CMP 0
#endif
// HR_OLD_LOAD: the codeword-fed load deinterleaves raw bytes and clamps / completes / scans the row in a second pass
// (r05 form, kept for A/B)
#ifndef HR_OLD_LOAD
#define HR_OLD_LOAD 0
#endif
#ifndef HR_CMP_WAVES
#define HR_CMP_WAVES 8
#endif
template <int NP, int MAXL>
constexpr int hr_waves_per_simd()
{
  return MAXL == bg_traits<1>::M ? FR_WAVES : (NP == 1 ? (HR_CMP ? HR_CMP_WAVES : HR_WAVES) : 2);
}

// threadIdx.x rebuilt from the wave's first thread (wave-uniform) and the lane id: opaque (volatile), so it is
// recomputed where it is asked for instead of being held in a VGPR (or hoisted) across the codeblock loop
__device__ __forceinline__ uint32_t hr_thread(uint32_t wave_base)
{
  uint32_t l;
  asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
  return wave_base + l;
}

// MAXL < 46: the high-rate kernel (int16 messages of the first MAXL layers in registers); MAXL == 46: the
// full-length kernel (compressed messages of every layer).
template <int ARITH, int MAXL, int NP>
__global__ void __launch_bounds__(HR_HALF / NP, (hr_waves_per_simd<NP, MAXL>())) ldpc_decode_hr_kernel(decode_args a)
{
  constexpr bool FULL   = MAXL == bg_traits<1>::M;
  constexpr bool CMP    = FULL || (HR_CMP && NP == 1); // compressed message state
  static_assert(!FULL || NP == 1, "full-length codeblocks: one row pair per lane");
  constexpr int Z       = HR_Z;
  constexpr int K       = 22 * Z;
  constexpr int NODES   = 22 + MAXL;
  constexpr int NE      = row_start<1>(MAXL) * NP;
  constexpr int MAX_LLR = (NODES - 2) * Z; // host guarantees llr_len <= MAX_LLR
  constexpr int NT      = HR_HALF / NP;
  lds_i32*      red     = (lds_i32*)(uintptr_t)LDS_RED_OFFSET;
  lds_i8*       lds     = (lds_i8*)(uintptr_t)0;
  lds_i8*       soft    = lds + LDS_SOFT_OFFSET;
  lds_i32*      soft4   = reinterpret_cast<lds_i32*>(soft);

  // The thread index is rebuilt per codeblock from the wave's first lane (an SGPR) and the lane id (v_mbcnt, opaque
  // so that nothing derived from it is hoisted out of the codeblock loop): no VGPR holds threadIdx.x across the
  // loop (held next to the message file, it was spilled -- scratch traffic of ~25 MB per headline launch).
  const uint32_t wave_base = __builtin_amdgcn_readfirstlane(threadIdx.x) & ~63u;
  for (uint32_t cb = blockIdx.x; cb < a.nof_cbs; cb += gridDim.x) {
    uint32_t t = hr_thread(wave_base);
    if (a.skip_flags && *reinterpret_cast<const int32_t*>(a.skip_flags + static_cast<size_t>(cb) * a.skip_stride)) {
      if (t == 0) {
        a.nof_iters[cb] = LDPC_ITERS_SKIPPED; // uniform over the workgroup
      }
      continue;
    }
    asm volatile("" : "+v"(t));
    const int8_t* in     = a.llrs + static_cast<size_t>(cb) * a.llr_stride;
    const int     n_llrs = static_cast<int>(a.llr_len);
    uint8_t*      out    = a.out + static_cast<size_t>(cb) * a.out_stride;

    // ---- input scan (last non-zero LLR, ldpc_decoder_impl.cpp:86) fused with the soft-bit load
    // (:160): clamped full nodes, the partial tail node unclamped, zeros elsewhere.
    if constexpr (NT > 64) {
      if (t == 0) {
        red[0] = -1;
        red[1] = 0;
        red[2] = 0;
      }
      __syncthreads();
    }
    int input_size;
    if (a.cw_llrs != nullptr) {
      // ---- rate dematching fused into the load (decode_args::cw_llrs): the codeblock's E received LLRs are
      // deinterleaved straight into the LDS row (symbol i, bit j -> deinterleaver index j Kq + i -> row position
      // p, shifted past the filler block), then each word is completed (fillers +infinity, zeros from E + F),
      // clamped and scanned exactly as a dematched row read from HBM (ldpc_rate_dematch_kernel's first pass).
      const uint32_t E     = a.cw_lengths[cb];
      const int8_t*  src   = a.cw_llrs + a.cw_offsets[cb];
      const uint32_t Qm    = a.cw_qm;
      const uint32_t Kq    = E / Qm;
      const uint32_t ninfo = a.cw_nof_info;
      const uint32_t F     = a.cw_filler;
      lds_i8*        row   = soft + 2 * Z;
      if (Qm == 8 && ((reinterpret_cast<uintptr_t>(src) & 7u) == 0) && n_llrs % Z == 0 && !HR_OLD_LOAD) {
        // Whole nodes only (the fused launches' prefix is whole nodes): every byte of the row is a full-node soft
        // bit, clamped to +-SOFT_CLAMP as it is stored, so the row needs no second pass.  Fillers (+infinity)
        // are stored as +SOFT_CLAMP and the bytes from E + F on as zeros (disjoint from the deinterleaved bytes,
        // so one barrier covers all three).  Clamp of a byte pair: offset binary (b ^ 0x80), each byte into the
        // low byte of a 16-bit half by one v_perm_b32, v_pk_max_u16 / v_pk_min_u16 against 128 -+ SOFT_CLAMP,
        // back by ^ 0x80; the two halves go out with ds_write_b8 / ds_write_b8_d16_hi.
        const uint32_t lane = t & 63u;
        for (uint32_t i = t; i < Kq; i += NT) {
          const uint2    v  = reinterpret_cast<const uint2*>(src)[i];
          const uint32_t ox = v.x ^ 0x80808080u, oy = v.y ^ 0x80808080u;
          uint32_t       q[4];
          // [b0 | b1], [b2 | b3] of x, then of y: selector bytes 0-3 pick S1 (= the second operand), 12 gives 0x00
          q[0] = __builtin_amdgcn_perm(0u, ox, 0x0c010c00u);
          q[1] = __builtin_amdgcn_perm(0u, ox, 0x0c030c02u);
          q[2] = __builtin_amdgcn_perm(0u, oy, 0x0c010c00u);
          q[3] = __builtin_amdgcn_perm(0u, oy, 0x0c030c02u);
#pragma unroll
          for (int h = 0; h < 4; ++h) {
            const pku16 u = __builtin_elementwise_min(
                __builtin_elementwise_max(__builtin_bit_cast(pku16, q[h]), pku16{128 - SOFT_CLAMP, 128 - SOFT_CLAMP}),
                pku16{128 + SOFT_CLAMP, 128 + SOFT_CLAMP});
            q[h] = __builtin_bit_cast(uint32_t, u) ^ 0x00800080u;
          }
          // the wave's first symbol index (uniform): the row position of bit j is d = j Kq + i, moved past the
          // filler block when d >= ninfo -- uniform for the whole wave except in at most one (wave, j)
          const uint32_t iw = __builtin_amdgcn_readfirstlane(i - lane);
#pragma unroll
          for (uint32_t j = 0; j < 8; ++j) {
            const uint32_t lo = j * Kq + iw;
            uint32_t       p  = j * Kq + i;
            if (lo >= ninfo) {
              p += F;
            } else if (lo + 63 >= ninfo) {
              p = p < ninfo ? p : p + F;
            }
            const uint32_t w = q[j >> 1];
            if ((j & 1u) == 0) {
              row[p] = static_cast<int8_t>(w);
            } else {
              row[p] = static_cast<int8_t>(w >> 16);
            }
          }
        }
        for (uint32_t p = ninfo + t; p < ninfo + F; p += NT) {
          row[p] = static_cast<int8_t>(SOFT_CLAMP);
        }
        {
          // zeros from E + F to the end of the row: the bytes up to the next word boundary, then words
          constexpr uint32_t ROW = (NODES - 2) * Z;
          const uint32_t     e0  = E + F;
          const uint32_t     w0  = (e0 + 3u) & ~3u;
          if (t < w0 - e0) {
            row[e0 + t] = 0;
          }
          lds_i32* row4 = soft4 + (2 * Z) / 4;
          for (uint32_t w = w0 / 4 + t; w < ROW / 4; w += NT) {
            row4[w] = 0;
          }
        }
        for (int w = t; w < 2 * Z / 4; w += NT) {
          soft4[w] = 0;
        }
        __syncthreads();
        if (FULL || a.force_decoding) {
          // last non-zero soft bit (only the layer count of a full-length row and force_decoding read it; a clamp
          // keeps zero and non-zero bytes apart, fillers are non-zero)
          const int nw   = n_llrs >> 2;
          int       last = -1;
          for (int w = static_cast<int>(t); w < nw; w += NT) {
            const uint32_t v = static_cast<uint32_t>(soft4[(2 * Z) / 4 + w]);
            if (v != 0) {
              last = 4 * w + (31 - __builtin_clz(v)) / 8;
            }
          }
          if constexpr (NT == 64) {
            input_size = __builtin_amdgcn_readfirstlane(wave_max(last) + 1);
          } else {
            if (last >= 0) {
              __hip_atomic_fetch_max(&red[0], last, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            }
            __syncthreads();
            input_size = __builtin_amdgcn_readfirstlane(red[0] + 1);
          }
        } else {
          // MAXL layers whatever the last non-zero position (<= (NODES - 2) Z): cb_len below gives MAXL
          input_size = n_llrs;
        }
      } else {
      if (Qm == 8 && ((reinterpret_cast<uintptr_t>(src) & 7u) == 0)) {
        for (uint32_t i = t; i < Kq; i += NT) {
          const uint2 v = reinterpret_cast<const uint2*>(src)[i];
#pragma unroll
          for (uint32_t j = 0; j < 8; ++j) {
            const uint32_t d = j * Kq + i;
            row[d < ninfo ? d : d + F] = static_cast<int8_t>((j < 4 ? v.x : v.y) >> (8 * (j & 3u)));
          }
        }
      } else {
        for (uint32_t i = t; i < Kq; i += NT) {
          for (uint32_t j = 0; j < Qm; ++j) {
            const uint32_t d = j * Kq + i;
            row[d < ninfo ? d : d + F] = src[i * Qm + j];
          }
        }
      }
      __syncthreads();
      const int nw   = n_llrs >> 2; // n_llrs % 4 == 0 (ldpc_hr_takes)
      const int B4   = (n_llrs / Z) * Z >> 2;
      const int end  = static_cast<int>(E + F);
      int       last = -1;
#pragma unroll
      for (int k = 0; k < (MAX_LLR / 4 + NT - 1) / NT; ++k) {
        const int w = static_cast<int>(t) + k * NT;
        uint32_t  v = 0;
        if (w < nw) {
          v = static_cast<uint32_t>(soft4[(2 * Z) / 4 + w]);
#pragma unroll
          for (int b = 0; b < 4; ++b) {
            const int      pb   = 4 * w + b;
            const uint32_t mask = 0xffu << (8 * b);
            v                   = pb >= end ? (v & ~mask) : v;
            v = (pb >= static_cast<int>(ninfo) && pb < static_cast<int>(ninfo + F)) ? ((v & ~mask) | (0x7fu << (8 * b))) : v;
          }
        }
        if (v != 0) {
          last = 4 * w + (31 - __builtin_clz(v)) / 8;
        }
        const int lim = w < B4 ? SOFT_CLAMP : SOFT_INF;
        uint32_t  o   = 0;
#pragma unroll
        for (int b = 0; b < 4; ++b) {
          const int x = static_cast<int8_t>(v >> (8 * b));
          o |= (static_cast<uint32_t>(med3_i(x, -lim, lim)) & 0xffu) << (8 * b);
        }
        if (w < (NODES - 2) * Z / 4) {
          soft4[(2 * Z) / 4 + w] = static_cast<int32_t>(o);
        }
      }
      for (int w = t; w < 2 * Z / 4; w += NT) {
        soft4[w] = 0;
      }
      if constexpr (NT == 64) {
        input_size = __builtin_amdgcn_readfirstlane(wave_max(last) + 1);
      } else {
        if (last >= 0) {
          __hip_atomic_fetch_max(&red[0], last, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        __syncthreads();
        input_size = __builtin_amdgcn_readfirstlane(red[0] + 1);
      }
      }
    } else {
      const int      nw  = n_llrs >> 2;
      const int      B4  = (n_llrs / Z) * Z >> 2;
      const int32_t* in4 = reinterpret_cast<const int32_t*>(in);
      const int      tail = n_llrs & 3; // trailing bytes of the partial word nw (tail node: unclamped)
      int            last = -1;
      uint32_t       w_in[(MAX_LLR / 4 + NT - 1) / NT];
#pragma unroll
      for (int k = 0; k < (MAX_LLR / 4 + NT - 1) / NT; ++k) {
        const int w = static_cast<int>(t) + k * NT;
        uint32_t  v = w < nw ? static_cast<uint32_t>(in4[w]) : 0u;
        if (w == nw && tail != 0) {
          for (int b = 0; b < tail; ++b) {
            v |= static_cast<uint32_t>(static_cast<uint8_t>(in[4 * nw + b])) << (8 * b);
          }
        }
        w_in[k] = v;
      }
#pragma unroll
      for (int k = 0; k < (MAX_LLR / 4 + NT - 1) / NT; ++k) {
        const int      w = static_cast<int>(t) + k * NT;
        const uint32_t v = w_in[k];
        if (v != 0) {
          last = 4 * w + (31 - __builtin_clz(v)) / 8;
        }
        // full nodes clamped to +-SOFT_CLAMP, the partial tail node to the soft-bit range
        const int lim = w < B4 ? SOFT_CLAMP : SOFT_INF;
        uint32_t  o   = 0;
#pragma unroll
        for (int b = 0; b < 4; ++b) {
          const int x = static_cast<int8_t>(v >> (8 * b));
          o |= (static_cast<uint32_t>(med3_i(x, -lim, lim)) & 0xffu) << (8 * b);
        }
        if (w < (NODES - 2) * Z / 4) {
          soft4[(2 * Z) / 4 + w] = static_cast<int32_t>(o); // words past nw hold zeros
        }
      }
      // punctured nodes 0 and 1
      for (int w = t; w < 2 * Z / 4; w += NT) {
        soft4[w] = 0;
      }
      if constexpr (NT == 64) {
        input_size = __builtin_amdgcn_readfirstlane(wave_max(last) + 1);
      } else {
        if (last >= 0) {
          __hip_atomic_fetch_max(&red[0], last, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        __syncthreads();
        input_size = __builtin_amdgcn_readfirstlane(red[0] + 1);
      }
    }

    if (input_size < K && a.force_decoding) {
      // ldpc_decoder_impl.cpp:92 (see ldpc_decode_kernel)
      const uint32_t tf = hr_thread(wave_base);
      for (int b = tf; b < K / 8 && !a.crc_table; b += NT) {
        out[b] = 0xff;
      }
      if (tf == 0) {
        a.nof_iters[cb] = -1;
      }
      if constexpr (NT > 64) {
        __syncthreads();
      }
      continue;
    }
    const int cb_len     = max(input_size + 2 * Z, K + 4 * Z);
    const int nof_layers = (cb_len + Z - 1) / Z - 22;
    // wave-uniform (an SGPR, not a VGPR held across the iterations)
    const int nof_sig    = __builtin_amdgcn_readfirstlane(K - (a.fillers ? a.fillers[cb] : a.nof_filler_bits));
    int       result     = -1;

    std::conditional_t<CMP, fr_state_n<fr_off(MAXL)>, hr_msgs<NE>> c2v;
    c2v.zero();

    for (int it = 0; it < a.max_iterations; ++it) {
      if constexpr (CMP) {
        fr_layers<0, ARITH, MAXL>(lds, c2v, t, nof_layers);
      } else {
        hr_layers<0, MAXL, ARITH, NP>(lds, c2v, t, nof_layers);
      }

      if (a.crc_table) {
        // hard bits + CRC early stop (ldpc_decoder_impl.cpp:125), remainder up to a unit factor:
        // bit i contributes crc_table[K - 1 - i]; the word of soft bits 4q .. 4q+3 reads the
        // remainders [K - 4 - 4q, K - 1 - 4q] as one 16-byte load.
        const uint32_t tq = hr_thread(wave_base);
        uint32_t crc = 0, zero = 0;
        // chunks of CRC_CHUNK words with a scheduling barrier in between: all eleven 16-byte remainder
        // loads in flight at once would need 44 VGPRs next to the message file
        constexpr int CRC_CHUNK = 4;
#pragma unroll
        for (int k = 0; k < K / 4 / NT; ++k) {
          if (k % CRC_CHUNK == 0 && k > 0) {
            __builtin_amdgcn_sched_barrier(0);
          }
          const int      q  = static_cast<int>(tq) + k * NT;
          const uint32_t w4 = static_cast<uint32_t>(soft4[q]);
          const uint4    r  = *reinterpret_cast<const uint4*>(a.crc_table + (K - 4 - 4 * q));
          zero |= (w4 - 0x01010101u) & ~w4 & 0x80808080u; // some byte is zero
          // bit 8b + 7 of d: soft bit 4q + b <= 0 (per-byte sign of x - 1, SWAR without borrows)
          const uint32_t d     = ((w4 | 0x80808080u) - 0x01010101u) ^ (~w4 & 0x80808080u);
          const uint32_t rr[4] = {r.w, r.z, r.y, r.x};
#pragma unroll
          for (int b = 0; b < 4; ++b) {
            // one bit-field extract (sign-extended) as the select mask: no compare / v_cndmask per bit
            crc ^= rr[b] & static_cast<uint32_t>(__builtin_amdgcn_sbfe(static_cast<int>(d), 8 * b + 7, 1));
          }
        }
        // filler bits (positions >= nof_sig) take no part in the CRC: cancel what the loop above added for them
        // (at most one word per lane; with the PUSCH's +infinity fillers nothing is set)
        for (int q = (nof_sig >> 2) + static_cast<int>(tq); q < K / 4; q += NT) {
          const uint32_t w4 = static_cast<uint32_t>(soft4[q]);
          const uint32_t d  = ((w4 | 0x80808080u) - 0x01010101u) ^ (~w4 & 0x80808080u);
#pragma unroll
          for (int b = 0; b < 4; ++b) {
            if (4 * q + b >= nof_sig && ((d >> (8 * b + 7)) & 1u)) {
              crc ^= a.crc_table[K - 1 - (4 * q + b)];
            }
          }
        }
        if constexpr (NT == 64) {
          // one wave: shuffle reductions, no LDS round trip and no barrier
          const uint32_t c_all = __builtin_amdgcn_readfirstlane(wave_xor(crc));
          const uint32_t z_all = __builtin_amdgcn_readfirstlane(wave_or(zero));
          if (z_all == 0 && c_all == 0) {
            result = it + 1;
            break;
          }
          continue;
        }
        lds_u32* acc = reinterpret_cast<lds_u32*>(&red[1 + 2 * (it & 1)]);
        if (crc != 0) {
          __hip_atomic_fetch_xor(&acc[0], crc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        if (zero != 0) {
          __hip_atomic_fetch_or(&acc[1], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        __syncthreads();
        const uint32_t c_all = __builtin_amdgcn_readfirstlane(acc[0]);
        const uint32_t z_all = __builtin_amdgcn_readfirstlane(acc[1]);
        if (tq == 0) {
          // the other slot was read before this iteration's barrier: reset it for the next check
          lds_u32* nxt = reinterpret_cast<lds_u32*>(&red[1 + 2 * ((it + 1) & 1)]);
          nxt[0]       = 0;
          nxt[1]       = 0;
        }
        if (z_all == 0 && c_all == 0) {
          result = it + 1;
          break;
        }
      }
    }

    // ---- hard decision, packed MSB-first: 4 output bytes per task
    const uint32_t te = hr_thread(wave_base);
    // 16 output bytes (128 soft bits) per task: one 16-byte store per lane when the row is 16-byte aligned
    static_assert(K % 128 == 0, "whole 16-byte hard-decision tasks");
    for (int task = te; task < K / 128; task += NT) {
      uint32_t o[4];
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        o[c] = 0;
#pragma unroll
        for (int h = 0; h < 8; ++h) {
          const uint32_t w = static_cast<uint32_t>(soft4[32 * task + 8 * c + h]);
          // per-byte (x <= 0) = sign of x - 1 (SWAR subtract, no borrow between bytes)
          const uint32_t d    = ((w | 0x80808080u) - 0x01010101u) ^ (~w & 0x80808080u);
          const uint32_t nib  = (((d & 0x80808080u) >> 7) * 0x08040201u) >> 24; // byte0 -> bit 3
          const int      byte = h >> 1;
          o[c] |= (nib & 0xfu) << (8 * byte + ((h & 1) ? 0 : 4));
        }
      }
      uint8_t* ob = out + 16 * task;
      if (((reinterpret_cast<uintptr_t>(ob)) & 15u) == 0) {
        *reinterpret_cast<uint4*>(ob) = uint4{o[0], o[1], o[2], o[3]};
      } else {
#pragma unroll
        for (int b = 0; b < 16; ++b) {
          ob[b] = static_cast<uint8_t>(o[b >> 2] >> (8 * (b & 3)));
        }
      }
    }
    if (a.soft_out) {
      int32_t* so = reinterpret_cast<int32_t*>(a.soft_out + static_cast<size_t>(cb) * (68 * Z));
      for (int i = te; i < 68 * Z / 4; i += NT) {
        so[i] = i < NODES * Z / 4 ? static_cast<int32_t>(soft_export4(static_cast<uint32_t>(soft4[i]))) : 0;
      }
    }
    if (te == 0) {
      a.nof_iters[cb] = result;
    }
    if constexpr (NT > 64) {
      __syncthreads();
    } else {
      asm volatile("" ::: "memory"); // the next codeblock's soft-bit stores follow this one's reads
    }
  }
}

// ============================================================================
// Packed decoder for every other lifted graph -- BG2, BG1 with Z < 384 and the mixed-Z launches of a slot --
// when Z is a multiple of 4: the full-length kernel's layout with the lifting size known only at run time.
//   * lane t owns check rows t and t + H (H = Z / 2) of every layer, one per 16-bit half; W = ceil(H / 64)
//     waves per codeblock (W = 1 for Z <= 128: one wave and no barriers; W = 2 for Z <= 256; W = 3).  Lanes
//     t >= H repeat lane t mod H, and odd rows past Z are rows mod Z: a repeated row computes the same
//     values from the same soft bits and writes them to the same addresses;
//   * soft bits in LDS at a compile-time stride of 128 W bytes per variable node, so the node offset of an
//     edge is a literal in the ds instruction's immediate, and only (row + shift) mod Z is computed per row:
//     two adds and a min on the lane index, the shift and shift - Z coming from the scalar unit;
//   * the compressed messages of every layer in registers (fr_layer): BG1 96 VGPRs, BG2 84;
//   * the LLR row, the CRC and the hard decision address the node-strided LDS through i / Z computed as
//     umulhi(i, ceil(2^32 / Z)) (exact for i < 2^16).
// Bit-exact with ldpc_decode_kernel (same per-edge arithmetic; identical outputs, iteration counts, soft bits).
// ============================================================================

template <int BG>
constexpr int pk_words(int l)
{
  return bg_traits<BG>::deg(l) > 13 ? 3 : 2;
}
template <int BG>
constexpr int pk_off(int l)
{
  int s = 0;
  for (int i = 0; i < l; ++i) {
    s += pk_words<BG>(i);
  }
  return s;
}
static_assert(pk_off<1>(46) == FR_STATE_WORDS && pk_off<2>(42) == 84, "compressed message state");

template <int BG>
struct pk_state {
  uint32_t w[pk_off<BG>(bg_traits<BG>::M)];
  __device__ __forceinline__ void zero()
  {
#pragma unroll
    for (int i = 0; i < pk_off<BG>(bg_traits<BG>::M); ++i) {
      w[i] = 0;
    }
  }
};

// base-graph variable node of edge E (compile time)
template <int BG, int E>
constexpr int bg_var()
{
  return BG == 1 ? tables::SRS_BG1_EDGES[E][1] : tables::SRS_BG2_EDGES[E][1];
}

// The lifted graph of one codeblock, wave-uniform.
struct pk_geo {
  const_u32_ptr edge; // lifted_graph::edge: var * Z | shift << 16
  uint32_t      Z, H;
};

// Positions (row + shift) mod Z of rows t and t + H of edge EI within its variable node (t + H + shift < 2 Z).
template <int EI>
__device__ __forceinline__ void pk_rows(const pk_geo& g, uint32_t t, uint32_t& lo, uint32_t& hi)
{
  const uint32_t s  = g.edge[EI] >> 16;
  uint32_t       sh = s + g.H;
  sh                = sh >= g.Z ? sh - g.Z : sh;
  lo                = __builtin_elementwise_min(t + s, t + (s - g.Z));
  hi                = __builtin_elementwise_min(t + sh, t + (sh - g.Z));
}

// rows of degree <= PK_KEEP_ADDR keep their gather positions for the scatter; longer rows recompute them
#ifndef PK_KEEP_ADDR
#define PK_KEEP_ADDR 10
#endif

// One layer (row L of base graph BG) for the row pair of lane t (fr_layer with run-time positions).
template <int BG, int L, int ARITH, int STRIDE, int... E>
__device__ __forceinline__ void pk_layer(lds_i8* lds, pk_state<BG>& st, uint32_t t, const pk_geo& g,
                                         std::integer_sequence<int, E...>)
{
  constexpr int  E0   = row_start<BG>(L);
  constexpr int  DEG  = sizeof...(E);
  constexpr int  O    = pk_off<BG>(L);
  constexpr bool W3   = pk_words<BG>(L) == 3;
  constexpr bool KEEP = DEG <= PK_KEEP_ADDR;
  const uint32_t wold[3] = {st.w[O], st.w[O + 1], W3 ? st.w[O + 2] : 0u};
  const pk16     s2o     = as_pk(wold[0] & 0x007f007fu);
  const uint32_t imo     = wold[0] & 0x0f800f80u;
  const pk16     dno     = pk_splat(0) - as_pk(wold[1] & 0x007f007fu); // s1 - s2 of the old messages
  pk16           v[DEG];
  uint32_t       plo[KEEP ? DEG : 1], phi[KEEP ? DEG : 1];
  pk16           min1[2], min2[2];
  pk16           sgn = pk_splat(0);
  min1[0] = min1[1] = min2[0] = min2[1] = pk_splat(LLR_MAX * 32 + 31);
  // pass 1 (ldpc_decoder_impl.cpp:235 / :290): old message, v2c, check-node statistics
  (
      [&] {
        if constexpr (E % HR_CHUNK1 == 0 && E > 0) {
          __builtin_amdgcn_sched_barrier(0);
        }
        constexpr int      h    = E & 1; // reduction chain
        constexpr uint32_t node = LDS_SOFT_OFFSET + bg_var<BG, E0 + E>() * STRIDE;
        uint32_t           lo, hi;
        pk_rows<E0 + E>(g, t, lo, hi);
        if constexpr (KEEP) {
          plo[E] = lo;
          phi[E] = hi;
        }
        const pk16 s   = pk16{static_cast<short>(lds[lo + node]), static_cast<short>(lds[hi + node])};
        const pk16 f   = pk_nonzero(imo ^ ((static_cast<uint32_t>(E) << 7) * 0x10001u));
        const pk16 mag = pk_mad(f, dno, s2o);
        const pk16 ng  = (as_pk(wold[fr_sign_word(E)]) << pk_splat(15 - fr_sign_bit(E))) >> 15;
        const pk16 c   = (mag ^ ng) - ng;
        const pk16 sat = pk_clamp(s, LLR_MAX);
        const pk16 x   = (s - sat) * pk_splat(INF_BOOST) + pk_clamp(s - c, LLR_MAX);
        const pk16 key = pk_key<E>(__builtin_elementwise_abs(x));
        min2[h]        = pk_max(min1[h], pk_min(key, min2[h])); // median(min1, key, min2)
        min1[h]        = pk_min(min1[h], key);
        sgn ^= x;
        v[E] = x;
      }(),
      ...);
  __builtin_amdgcn_sched_barrier(0);
  const pk16     k1     = pk_min(min1[0], min1[1]);
  const pk16     k2     = pk_min(pk_max(min1[0], min1[1]), pk_min(min2[0], min2[1]));
  const pk16     s1     = pk_scale16<ARITH>(k1 >> 5);
  const pk16     s2     = pk_scale16<ARITH>(k2 >> 5);
  const pk16     d12    = s1 - s2;
  const uint32_t idx    = as_u32(k1) & 0x001f001fu;
  uint32_t       acc[3] = {(idx << 7) | as_u32(s2), as_u32(s2 - s1), 0u};
  if constexpr (!KEEP) {
    asm volatile("" : "+v"(t));
  }
  // pass 2 (ldpc_decoder_impl.cpp:310, :270): new message, promotion sum, new state
  (
      [&] {
        if constexpr (E % HR_CHUNK2 == 0 && E > 0) {
          __builtin_amdgcn_sched_barrier(0);
        }
        constexpr uint32_t node = LDS_SOFT_OFFSET + bg_var<BG, E0 + E>() * STRIDE;
        const pk16         x    = v[E];
        const pk16         f    = pk_nonzero(idx ^ (static_cast<uint32_t>(E) * 0x10001u)); // 0: edge E holds min1
        const pk16         mag  = f * d12 + s2;
        const pk16         sx   = sgn ^ x;
        const pk16         ng   = sx >> 15;
        const pk16         c    = (mag ^ ng) - ng;
        const pk16         out  = pk_clamp(c + x, SOFT_INF);
        const uint32_t     nb   = __builtin_bit_cast(uint32_t, __builtin_bit_cast(pku16, sx) >> 15);
        acc[fr_sign_word(E)] |= nb << fr_sign_bit(E);
        uint32_t lo, hi;
        if constexpr (KEEP) {
          lo = plo[E];
          hi = phi[E];
        } else {
          pk_rows<E0 + E>(g, t, lo, hi);
        }
        lds[lo + node] = static_cast<int8_t>(out.x);
        lds[hi + node] = static_cast<int8_t>(out.y);
      }(),
      ...);
  asm volatile("" : "+v"(acc[0]), "+v"(acc[1]));
  st.w[O]     = acc[0];
  st.w[O + 1] = acc[1];
  if constexpr (W3) {
    asm volatile("" : "+v"(acc[2]));
    st.w[O + 2] = acc[2];
  }
}

// own: the lane owns its row pair (threadIdx.x < H).  A repeating lane (t >= H, rows of lane t mod H) sits in another
// wave than its owner when H is not a multiple of 64 (Z = 136..252 or 264..380 with Z / 2 mod 64 != 0): with no
// barrier between a layer's gathers and scatters, the owner's wave can scatter a row's new soft bits before the
// repeating wave gathers them, which then computes -- and scatters -- different values (BG2 Z = 288 soft bits
// differed in 0.6 % of positions, intermittently).  Repeating lanes therefore skip the layers: they only fill the
// workgroup for the CRC, hard-decision and export loops, which index words by threadIdx.x.
template <int BG, int L, int ARITH, int W>
__device__ __forceinline__ void pk_layers(lds_i8* lds, pk_state<BG>& st, uint32_t t, pk_geo g, int nof_layers, bool own)
{
  if constexpr (L < bg_traits<BG>::M) {
    asm volatile("" : "+s"(nof_layers));
    if (L < 4 || L < nof_layers) { // uniform; nof_layers >= 4
      // laundered per layer: the positions are iteration-invariant, hoisted they would spill
      asm volatile("" : "+v"(t), "+s"(g.edge), "+s"(g.Z), "+s"(g.H));
      if (own) {
        pk_layer<BG, L, ARITH, 128 * W>(lds, st, t, g, std::make_integer_sequence<int, bg_traits<BG>::deg(L)>{});
      }
      // no barrier before a next layer of the same group (disjoint columns, see bg_groups_t); always one after
      // the last layer that runs
      constexpr bool next_joins = FR_GROUPS && L + 1 < bg_traits<BG>::M && bg_group_start<BG>(L + 1) != L + 1;
      if constexpr (W > 1) {
        if (!next_joins || !(L + 1 < 4 || L + 1 < nof_layers)) {
          __syncthreads();
        } else {
          asm volatile("" ::: "memory");
        }
      } else {
        asm volatile("" ::: "memory"); // one wave: LDS accesses execute in issue order
      }
    }
    pk_layers<BG, L + 1, ARITH, W>(lds, st, t, g, nof_layers, own);
  }
}

#ifndef PK_WAVES_BG1
#define PK_WAVES_BG1 3
#endif
#ifndef PK_WAVES_BG2
#define PK_WAVES_BG2 3
#endif

__host__ __device__ constexpr int pk_lds_bytes(int bg, int w)
{
  return LDS_SOFT_OFFSET + (bg == 1 ? 68 : 52) * 128 * w;
}

template <int BG, int ARITH, int W>
__global__ void __launch_bounds__(64 * W, (BG == 1 ? PK_WAVES_BG1 : PK_WAVES_BG2))
    ldpc_decode_pk_kernel(decode_args a, uint32_t launch_z, uint32_t launch_magic)
{
  constexpr int      NT     = 64 * W;
  constexpr uint32_t STRIDE = 128 * W;
  constexpr int      KB     = bg_traits<BG>::K;
  constexpr int      NF     = bg_traits<BG>::N_FULL;
  lds_i32*           red    = (lds_i32*)(uintptr_t)LDS_RED_OFFSET;
  lds_i8*            lds    = (lds_i8*)(uintptr_t)0;

  for (uint32_t cb = blockIdx.x; cb < a.nof_cbs; cb += gridDim.x) {
    const bool      mixed = a.rows != nullptr;
    const uint32_t  Z     = mixed ? __builtin_amdgcn_readfirstlane(a.rows[cb].Z) : launch_z;
    const uint32_t  magic = mixed ? __builtin_amdgcn_readfirstlane(a.rows[cb].zmagic) : launch_magic;
    const uint32_t  e_off = mixed ? __builtin_amdgcn_readfirstlane(a.rows[cb].edge_off) : 0u;
    const uint32_t  c_off = mixed ? __builtin_amdgcn_readfirstlane(a.rows[cb].crc_off) : 0u;
    const uint32_t* crc_table = mixed ? (c_off == NO_CRC_ROW ? nullptr : a.crc_table + c_off) : a.crc_table;
    if (a.skip_flags && *reinterpret_cast<const int32_t*>(a.skip_flags + static_cast<size_t>(cb) * a.skip_stride)) {
      if (threadIdx.x == 0) {
        a.nof_iters[cb] = LDPC_ITERS_SKIPPED; // uniform over the workgroup
      }
      continue;
    }
    const uint32_t gap = STRIDE - Z; // LDS bytes of a node row past its Z soft bits
    // LDS byte of soft bit i (node i / Z, position i mod Z)
    auto lds_at = [&](uint32_t i) { return LDS_SOFT_OFFSET + i + __umulhi(i, magic) * gap; };
    uint32_t t = threadIdx.x;
    asm volatile("" : "+v"(t));
    const int8_t*  in     = a.llrs + static_cast<size_t>(cb) * a.llr_stride;
    const uint32_t n_llrs = a.llr_lens ? a.llr_lens[cb] : a.llr_len;
    uint8_t*       out    = a.out + static_cast<size_t>(cb) * a.out_stride;
    const uint32_t KZ     = KB * Z;

    if constexpr (W > 1) {
      if (t == 0) {
        red[0] = -1;
        red[1] = red[2] = red[3] = red[4] = 0;
      }
      __syncthreads();
    }
    // ---- input scan (last non-zero LLR, ldpc_decoder_impl.cpp:86) fused with the soft-bit load (:160):
    // LLR i is soft bit 2 Z + i; full nodes clamped to +-SOFT_CLAMP, the partial tail node to the soft-bit range,
    // zeros past the input; nodes 0, 1 and the nodes past the input that a layer or the export reads zeroed.
    int input_size;
    {
      const uint32_t in_nodes = __umulhi(n_llrs + Z - 1, magic); // nodes holding input
      const uint32_t B4       = __umulhi(n_llrs, magic) * Z >> 2; // words of full (clamped) nodes
      const uint32_t nw       = n_llrs >> 2;
      const uint32_t wend     = in_nodes * Z >> 2;
      const uint32_t tail     = n_llrs & 3;
      const bool     al4      = a.aligned4 != 0;
      const int32_t* in4      = reinterpret_cast<const int32_t*>(in);
      int            last     = -1;
      for (uint32_t w = t; w < wend; w += NT) {
        uint32_t v = 0;
        if (w < nw) {
          if (al4) {
            v = static_cast<uint32_t>(in4[w]);
          } else {
#pragma unroll
            for (int b = 0; b < 4; ++b) {
              v |= static_cast<uint32_t>(static_cast<uint8_t>(in[4 * w + b])) << (8 * b);
            }
          }
        } else if (w == nw) {
          for (uint32_t b = 0; b < tail; ++b) {
            v |= static_cast<uint32_t>(static_cast<uint8_t>(in[4 * w + b])) << (8 * b);
          }
        }
        if (v != 0) {
          last = static_cast<int>(4 * w + (31 - __builtin_clz(v)) / 8);
        }
        const int lim = w < B4 ? SOFT_CLAMP : SOFT_INF;
        uint32_t  o   = 0;
#pragma unroll
        for (int b = 0; b < 4; ++b) {
          const int x = static_cast<int8_t>(v >> (8 * b));
          o |= (static_cast<uint32_t>(med3_i(x, -lim, lim)) & 0xffu) << (8 * b);
        }
        *reinterpret_cast<lds_u32*>(lds + lds_at(2 * Z + 4 * w)) = o;
      }
      // nodes 0 and 1 (punctured), then the nodes after the input up to the last one read
      const uint32_t zend = a.soft_out ? NF : min(static_cast<uint32_t>(NF), max(2 + in_nodes, KB + 4u));
      const uint32_t z0   = (2 + in_nodes) * Z >> 2;
      const uint32_t nz   = (Z >> 1) + (zend > 2 + in_nodes ? (zend - 2 - in_nodes) * Z >> 2 : 0u);
      for (uint32_t q = t; q < nz; q += NT) {
        const uint32_t w = q < (Z >> 1) ? q : z0 + q - (Z >> 1);
        *reinterpret_cast<lds_u32*>(lds + lds_at(4 * w)) = 0;
      }
      if constexpr (W == 1) {
        input_size = __builtin_amdgcn_readfirstlane(wave_max(last) + 1);
      } else {
        if (last >= 0) {
          __hip_atomic_fetch_max(&red[0], last, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        __syncthreads();
        input_size = __builtin_amdgcn_readfirstlane(red[0] + 1);
      }
    }

    if (input_size < static_cast<int>(KZ) && a.force_decoding) {
      // ldpc_decoder_impl.cpp:92 (see ldpc_decode_kernel); K Z is a multiple of 8 here
      for (uint32_t b = t; b < KZ / 8 && !crc_table; b += NT) {
        out[b] = 0xff;
      }
      if (t == 0) {
        a.nof_iters[cb] = -1;
      }
      if constexpr (W > 1) {
        __syncthreads();
      }
      continue;
    }
    const uint32_t cb_len     = max(static_cast<uint32_t>(input_size) + 2 * Z, KZ + 4 * Z);
    const int      nof_layers = static_cast<int>(__umulhi(cb_len + Z - 1, magic)) - KB;
    const int      nof_sig    = static_cast<int>(KZ) - (a.fillers ? a.fillers[cb] : a.nof_filler_bits);
    int            result     = -1;
    const uint32_t H          = Z >> 1;
    const pk_geo   geo{(const_u32_ptr)(a.edges + e_off), Z, H};
    const uint32_t tr         = t < H ? t : t % H; // the row pair of this lane (lanes t >= H repeat one)

    pk_state<BG> st;
    st.zero();

    for (int it = 0; it < a.max_iterations; ++it) {
      pk_layers<BG, 0, ARITH, W>(lds, st, tr, geo, nof_layers, t < H);

      if (crc_table) {
        // hard bits + CRC early stop (ldpc_decoder_impl.cpp:125), remainder up to a unit factor (see the
        // high-rate kernel): word q (soft bits 4q .. 4q+3, one node) reads remainders [KZ - 4 - 4q, KZ - 1 - 4q]
        uint32_t tq = threadIdx.x;
        asm volatile("" : "+v"(tq));
        uint32_t crc = 0, zero = 0;
        for (uint32_t q = tq; q < KZ / 4; q += NT) {
          const uint32_t w4 = *reinterpret_cast<const lds_u32*>(lds + lds_at(4 * q));
          const uint4    r  = *reinterpret_cast<const uint4*>(crc_table + (KZ - 4 - 4 * q));
          zero |= (w4 - 0x01010101u) & ~w4 & 0x80808080u;
          const uint32_t d     = ((w4 | 0x80808080u) - 0x01010101u) ^ (~w4 & 0x80808080u);
          const uint32_t rr[4] = {r.w, r.z, r.y, r.x};
#pragma unroll
          for (int b = 0; b < 4; ++b) {
            crc ^= rr[b] & static_cast<uint32_t>(__builtin_amdgcn_sbfe(static_cast<int>(d), 8 * b + 7, 1));
          }
        }
        // filler bits take no part in the CRC
        for (uint32_t q = (static_cast<uint32_t>(nof_sig) >> 2) + tq; q < KZ / 4; q += NT) {
          const uint32_t w4 = *reinterpret_cast<const lds_u32*>(lds + lds_at(4 * q));
          const uint32_t d  = ((w4 | 0x80808080u) - 0x01010101u) ^ (~w4 & 0x80808080u);
#pragma unroll
          for (uint32_t b = 0; b < 4; ++b) {
            if (4 * q + b >= static_cast<uint32_t>(nof_sig) && ((d >> (8 * b + 7)) & 1u)) {
              crc ^= crc_table[KZ - 1 - (4 * q + b)];
            }
          }
        }
        if constexpr (W == 1) {
          const uint32_t c_all = __builtin_amdgcn_readfirstlane(wave_xor(crc));
          const uint32_t z_all = __builtin_amdgcn_readfirstlane(wave_or(zero));
          if (z_all == 0 && c_all == 0) {
            result = it + 1;
            break;
          }
          continue;
        } else {
          lds_u32* acc = reinterpret_cast<lds_u32*>(&red[1 + 2 * (it & 1)]);
          if (crc != 0) {
            __hip_atomic_fetch_xor(&acc[0], crc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          }
          if (zero != 0) {
            __hip_atomic_fetch_or(&acc[1], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          }
          __syncthreads();
          const uint32_t c_all = __builtin_amdgcn_readfirstlane(acc[0]);
          const uint32_t z_all = __builtin_amdgcn_readfirstlane(acc[1]);
          if (tq == 0) {
            lds_u32* nxt = reinterpret_cast<lds_u32*>(&red[1 + 2 * ((it + 1) & 1)]);
            nxt[0]       = 0;
            nxt[1]       = 0;
          }
          if (z_all == 0 && c_all == 0) {
            result = it + 1;
            break;
          }
        }
      }
    }

    // ---- hard decision, packed MSB-first: one output byte (two soft-bit words of one node each) per task
    uint32_t te = threadIdx.x;
    asm volatile("" : "+v"(te));
    for (uint32_t b = te; b < KZ / 8; b += NT) {
      uint32_t o = 0;
#pragma unroll
      for (uint32_t h = 0; h < 2; ++h) {
        const uint32_t w   = *reinterpret_cast<const lds_u32*>(lds + lds_at(8 * b + 4 * h));
        const uint32_t d   = ((w | 0x80808080u) - 0x01010101u) ^ (~w & 0x80808080u);
        const uint32_t nib = (((d & 0x80808080u) >> 7) * 0x08040201u) >> 24; // byte0 -> bit 3
        o |= (nib & 0xfu) << (h ? 0 : 4);
      }
      out[b] = static_cast<uint8_t>(o);
    }
    if (a.soft_out) {
      int32_t* so = reinterpret_cast<int32_t*>(a.soft_out + static_cast<size_t>(cb) * (NF * Z));
      for (uint32_t q = te; q < NF * Z / 4; q += NT) {
        so[q] = static_cast<int32_t>(soft_export4(*reinterpret_cast<const lds_u32*>(lds + lds_at(4 * q))));
      }
    }
    if (te == 0) {
      a.nof_iters[cb] = result;
    }
    if constexpr (W > 1) {
      __syncthreads();
    } else {
      asm volatile("" ::: "memory");
    }
  }
}

// Waves per codeblock of the packed kernel for a lifting size, 0 when it does not take it.
int ldpc_pk_waves(int bg, int Z)
{
  // read per call (A/B timing and the parity tests switch it per launch)
  const char* mode    = std::getenv("SRSRAN_AMD_LDPC_PK");
  const bool  enabled = mode == nullptr || mode[0] != '0';
  if (!enabled || (bg != 1 && bg != 2) || Z < 4 || (Z & 3) != 0 || Z > MAX_LIFTING_SIZE) {
    return 0;
  }
  return (Z / 2 + 63) / 64;
}

uint32_t ldpc_z_magic(uint32_t Z)
{
  return static_cast<uint32_t>((1ull << 32) / Z + 1);
}

template <int BG, int ARITH>
static void launch_pk(const decode_args& args, int W, uint32_t Z, int grid, hipStream_t stream)
{
  const uint32_t magic = ldpc_z_magic(Z);
  if (W == 1) {
    hipLaunchKernelGGL((ldpc_decode_pk_kernel<BG, ARITH, 1>), dim3(grid), dim3(64), pk_lds_bytes(BG, 1), stream, args,
                       Z, magic);
  } else if (W == 2) {
    hipLaunchKernelGGL((ldpc_decode_pk_kernel<BG, ARITH, 2>), dim3(grid), dim3(128), pk_lds_bytes(BG, 2), stream,
                       args, Z, magic);
  } else {
    hipLaunchKernelGGL((ldpc_decode_pk_kernel<BG, ARITH, 3>), dim3(grid), dim3(192), pk_lds_bytes(BG, 3), stream,
                       args, Z, magic);
  }
}

constexpr int HR_MAXL = 4;
#ifndef HR_NP_DEFAULT
#define HR_NP_DEFAULT 1
#endif
constexpr int HR_NP = HR_NP_DEFAULT; // row pairs per lane (1: three waves per codeblock, 3: one wave)

bool ldpc_decode_hr_eligible(const decode_args& args, const lifted_graph& g)
{
  // SRSRAN_AMD_LDPC_HR=0 keeps every launch on ldpc_decode_kernel (A/B timing, cross-checks).
  static const bool enabled = [] {
    const char* e = std::getenv("SRSRAN_AMD_LDPC_HR");
    return e == nullptr || e[0] != '0';
  }();
  return enabled && g.bg == 1 && g.Z == HR_Z && args.llr_lens == nullptr && args.aligned4 != 0 &&
         args.llr_len <= static_cast<uint32_t>((20 + HR_MAXL) * HR_Z) &&
         ((reinterpret_cast<uintptr_t>(args.soft_out) | (args.soft_out ? 68u * HR_Z : 0u)) & 3u) == 0;
}

// BG1 Z = 384 codeblocks of any length through the packed full-length kernel (same launch conditions as the
// high-rate kernel otherwise).  SRSRAN_AMD_LDPC_FULL (read per launch): 0 keeps them on ldpc_decode_kernel,
// 1 takes the full-length kernel whatever the batch size (A/B timing, parity tests on small batches).
static bool ldpc_decode_full_eligible(const decode_args& args, const lifted_graph& g)
{
  const char* mode    = std::getenv("SRSRAN_AMD_LDPC_FULL");
  const bool  enabled = mode == nullptr || mode[0] != '0';
  const bool  forced  = mode != nullptr && mode[0] == '1';
  if (!(enabled && g.bg == 1 && g.Z == HR_Z && args.llr_lens == nullptr && args.aligned4 != 0 &&
        ((reinterpret_cast<uintptr_t>(args.soft_out) | (args.soft_out ? 68u * HR_Z : 0u)) & 3u) == 0)) {
    return false;
  }
  if (forced) {
    return true;
  }
  // Batch size: the full-length kernel keeps 4 codeblocks per CU in flight with 3 waves each, ldpc_decode_kernel
  // 2 per CU with 8 waves each, and one of its codeblocks takes ~1.6x less time (configs[1]: 1.57 vs 1.26 M
  // codeblocks/s at full occupancy).  A launch that fills only part of a round (e.g. a small slot bucket) is
  // latency-bound, so take the full-length kernel only when it needs fewer codeblock-rounds in time.
  static const uint32_t cus = [] {
    int dev = 0, n = 0;
    return (hipGetDevice(&dev) == hipSuccess &&
            hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && n > 0)
               ? static_cast<uint32_t>(n)
               : 256u;
  }();
  const uint64_t rounds_general = (args.nof_cbs + 2ull * cus - 1) / (2ull * cus);
  const uint64_t rounds_full    = (args.nof_cbs + 4ull * cus - 1) / (4ull * cus);
  return 16 * rounds_full < 10 * rounds_general;
}

size_t ldpc_decode_lds_bytes(const lifted_graph& g)
{
  return g.bg == 1 ? lds_total_bytes<1>(g.Z) : lds_total_bytes<2>(g.Z);
}

template <int BG, int ARITH>
static void launch_bg(const decode_args& args, const lifted_graph& g, int grid, int threads, hipStream_t stream)
{
  // Specialised kernels for the largest lifting size (the 100 MHz workloads);
  // every other Z runs the runtime-Z instantiation.
  const size_t lds = lds_total_bytes<BG>(g.Z);
  if (g.Z == 384) {
    hipLaunchKernelGGL((ldpc_decode_kernel<BG, ARITH, 384>), dim3(grid), dim3(max_threads<384>()), lds, stream, args, g);
  } else {
    hipLaunchKernelGGL((ldpc_decode_kernel<BG, ARITH, 0>), dim3(grid), dim3(threads), lds, stream, args, g);
  }
}

bool ldpc_hr_takes(int bg, int Z, uint32_t llr_len)
{
  static const bool enabled = [] {
    const char* e = std::getenv("SRSRAN_AMD_LDPC_HR");
    return e == nullptr || e[0] != '0';
  }();
  return enabled && bg == 1 && Z == HR_Z && llr_len <= static_cast<uint32_t>((20 + HR_MAXL) * HR_Z) &&
         (llr_len & 3u) == 0;
}

hipError_t launch_ldpc_decode(const decode_args& args, const lifted_graph& g, int arith, int grid, hipStream_t stream)
{
  if (args.cw_llrs != nullptr && !(ldpc_decode_hr_eligible(args, g) && ldpc_hr_takes(g.bg, g.Z, args.llr_len))) {
    return hipErrorInvalidValue; // codeword-fed rows are the high-rate kernel's only
  }
  if (ldpc_decode_hr_eligible(args, g)) {
    // The crc table of the high-rate kernel is indexed from K Z - 1 down, 16-byte aligned.
    constexpr size_t lds = hr_lds_bytes<HR_MAXL>();
    constexpr int    NT  = HR_HALF / HR_NP;
    // live in-step timing when armed (profiling.h)
    if (arith == ARITH_GENERIC) {
      SRS_PROBED_LAUNCH(SRS_AMD_PROBE_LDPC_HR, (ldpc_decode_hr_kernel<ARITH_GENERIC, HR_MAXL, HR_NP>), dim3(grid),
                        dim3(NT), lds, stream, args);
    } else {
      SRS_PROBED_LAUNCH(SRS_AMD_PROBE_LDPC_HR, (ldpc_decode_hr_kernel<ARITH_SIMD, HR_MAXL, HR_NP>), dim3(grid),
                        dim3(NT), lds, stream, args);
    }
    return hipGetLastError();
  }
  if (ldpc_decode_full_eligible(args, g)) {
    constexpr int    MAXL = bg_traits<1>::M;
    constexpr size_t lds  = hr_lds_bytes<MAXL>();
    if (arith == ARITH_GENERIC) {
      SRS_PROBED_LAUNCH(SRS_AMD_PROBE_LDPC_FULL, (ldpc_decode_hr_kernel<ARITH_GENERIC, MAXL, 1>), dim3(grid),
                        dim3(HR_HALF), lds, stream, args);
    } else {
      SRS_PROBED_LAUNCH(SRS_AMD_PROBE_LDPC_FULL, (ldpc_decode_hr_kernel<ARITH_SIMD, MAXL, 1>), dim3(grid),
                        dim3(HR_HALF), lds, stream, args);
    }
    return hipGetLastError();
  }
  // every other graph with Z a multiple of 4: the packed runtime-Z kernel (BG1 Z = 384 keeps the compile-time
  // kernels above and below)
  const int pkw = ldpc_pk_waves(g.bg, g.Z);
  if (pkw > 0 && !(g.bg == 1 && g.Z == HR_Z) && (reinterpret_cast<uintptr_t>(args.soft_out) & 3u) == 0) {
    if (g.bg == 1) {
      arith == ARITH_GENERIC ? launch_pk<1, ARITH_GENERIC>(args, pkw, g.Z, grid, stream)
                             : launch_pk<1, ARITH_SIMD>(args, pkw, g.Z, grid, stream);
    } else {
      arith == ARITH_GENERIC ? launch_pk<2, ARITH_GENERIC>(args, pkw, g.Z, grid, stream)
                             : launch_pk<2, ARITH_SIMD>(args, pkw, g.Z, grid, stream);
    }
    return hipGetLastError();
  }
  const int threads = ((g.Z + 63) / 64) * 64;
  if (g.bg == 1) {
    if (arith == ARITH_GENERIC) {
      launch_bg<1, ARITH_GENERIC>(args, g, grid, threads, stream);
    } else {
      launch_bg<1, ARITH_SIMD>(args, g, grid, threads, stream);
    }
  } else {
    if (arith == ARITH_GENERIC) {
      launch_bg<2, ARITH_GENERIC>(args, g, grid, threads, stream);
    } else {
      launch_bg<2, ARITH_SIMD>(args, g, grid, threads, stream);
    }
  }
  return hipGetLastError();
}

} // namespace srs_amd
