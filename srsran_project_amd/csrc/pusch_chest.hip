// pusch_chest.hip -- MI355X PUSCH DM-RS channel estimator (dmrs_pusch_estimator_impl
// + port_channel_estimator_average_impl, DM-RS type 1, one hop).
//
// Two launches per batch of grids (a third when the per-RE estimates are wanted):
//   chest_pilot_kernel   one 256-thread workgroup per (grid, rx port, slice = layer x LSE symbol), so the
//                        slices of a port run concurrently: the DM-RS Gold words into LDS (jump-ahead, one wave
//                        per DM-RS symbol); the port's CFO from the first two DM-RS symbols over every layer of
//                        every CDM group (computed by each slice of the port, the same value in each);
//                        LSE (rx * conj(pilot)), CFO compensation and time accumulation, CDM
//                        pair averaging (lane shuffle), scaling, FD smoothing in LDS (mean, or virtual
//                        pilots + raised-cosine FIR), the slice's RSRP share, linear interpolation to
//                        every RE of the allocation (port_channel_estimator_average_impl.cpp:130-506), and
//                        the slice's time-alignment IDFT of its smoothed pilots (fused Stockham engine,
//                        |.|^2 into the slice's correlation row, time_alignment_estimator_dft_impl.cpp:122-200).
//   chest_stats_kernel   one workgroup per (grid, port): EPRE and the noise energy per CDM group from the
//                        smoothed pilots of every slice (estimate_noise, :594-690), the correlations
//                        summed, peak search and quadratic refinement (:248-310), and the per-port
//                        measurements (noise variance, EPRE, RSRP, SNR, CFO).
//   chest_expand_kernel  one thread per (subcarrier, port, layer), every symbol: the time-domain strategy
//                        (average or interpolation between DM-RS symbols), bf16
//                        rounding and the CFO phase of the symbol -- the only
//                        HBM-heavy step (4 bytes per RE x layer x port written).
// (r04 ran the Gold words, the CFO, the slices and the IDFTs as four launches: 87 us of a 64-cell step.)
// Complex products follow the reference's AVX2+FMA srsran_simd_cf_prod
// (re = fma(a.re, b.re, -a.im b.im), im = fma(a.re, b.im, a.im b.re)); sums
// are reassociated by the reductions (float tolerance).
#include <hip/hip_runtime.h>

#include "dft_engine.h"
#include "gold_sequence.h"
#include "chest_device.h"
#include "pusch_chest_args.h"

#pragma clang fp contract(off)

namespace srs_amd {
namespace {

// Phase probe (tools/chest_probe.py; never in the product build): -DSRS_AMD_CHEST_PROBE records per-workgroup
// s_memtime stamps of the pilot and statistics kernels' phases, read back by srs_amd_chest_probe_read.
#ifdef SRS_AMD_CHEST_PROBE
constexpr uint32_t CHEST_PROBE_WG = 4096;
__device__ uint64_t g_chest_probe[2][CHEST_PROBE_WG][16];
#define CHEST_STAMP(k, i)                                                                                            \
  do {                                                                                                               \
    if (threadIdx.x == 0) {                                                                                          \
      const uint32_t wg_ = (blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x;                           \
      if (wg_ < CHEST_PROBE_WG) {                                                                                    \
        g_chest_probe[k][wg_][i] = (i) == 0 || (i) == 15 ? __builtin_amdgcn_s_memrealtime()                          \
                                                         : __builtin_amdgcn_s_memtime();                             \
      }                                                                                                              \
    }                                                                                                                \
  } while (0)
#else
#define CHEST_STAMP(k, i)                                                                                            \
  do {                                                                                                               \
  } while (0)
#endif


using chdev::bf16_bits;
using chdev::cmul;
using chdev::from_cbf16;
using chdev::polar1;
using chdev::to_cbf16;
using chdev::TWOPI_F;
using chdev::virtual_pilots_wave;
constexpr float AMP = 0.70710678118654752440f; // M_SQRT1_2 as float

__device__ __forceinline__ float2 cmulc(float2 a, float2 b) // a * conj(b)
{
  return cmul(a, make_float2(b.x, -b.y));
}
__device__ __forceinline__ float2 cadd(float2 a, float2 b)
{
  return make_float2(a.x + b.x, a.y + b.y);
}
__device__ __forceinline__ float2 csub(float2 a, float2 b)
{
  return make_float2(a.x - b.x, a.y - b.y);
}
__device__ __forceinline__ float2 cscale(float2 a, float s)
{
  return make_float2(a.x * s, a.y * s);
}

// Sum of 4 floats over the workgroup (result broadcast). red: >= 4 * 16 floats.
__device__ float4 block_sum4(float4 v, float* red)
{
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    v.x += __shfl_xor(v.x, o);
    v.y += __shfl_xor(v.y, o);
    v.z += __shfl_xor(v.z, o);
    v.w += __shfl_xor(v.w, o);
  }
  const int wave = threadIdx.x / 64, nw = blockDim.x / 64;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) {
    red[4 * wave + 0] = v.x;
    red[4 * wave + 1] = v.y;
    red[4 * wave + 2] = v.z;
    red[4 * wave + 3] = v.w;
  }
  __syncthreads();
  float4 r = make_float4(0, 0, 0, 0);
  for (int w = 0; w < nw; ++w) {
    r.x += red[4 * w + 0];
    r.y += red[4 * w + 1];
    r.z += red[4 * w + 2];
    r.w += red[4 * w + 3];
  }
  return r;
}

// Pilot of layer v at DM-RS symbol d, index m (dmrs_pusch_estimator_impl.cpp:72-184): amplitude
// M_SQRT1_2, w_f = -1 on odd indices of odd layers (w_t = +1 for layers < 4).  Transform precoding: the
// low-PAPR sequence of the allocation, one layer, the same in every DM-RS symbol (:86-92).
__device__ __forceinline__ float2 pilot(const chest_args& a, const uint32_t (*seq)[CH_SEQWORDS], uint32_t bit0, int d,
                                        int v, uint32_t m)
{
  if (a.lp_seq != nullptr) {
    return a.lp_seq[m];
  }
  const uint32_t b  = bit0 + 2 * m;
  const uint32_t c0 = (seq[d][b >> 5] >> (b & 31)) & 1u;
  const uint32_t c1 = (seq[d][(b + 1) >> 5] >> ((b + 1) & 31)) & 1u;
  float2         p  = make_float2(c0 ? -AMP : AMP, c1 ? -AMP : AMP);
  if ((v & 1) && (m & 1)) {
    p = make_float2(-p.x, -p.y);
  }
  return p;
}

// Allocations of at most CH_SMALL_NPIL pilots per DM-RS symbol (68 PRBs: time-alignment IDFTs of <= 512 points)
// take the narrow workgroups of the pilot and statistics kernels.
constexpr uint32_t CH_SMALL_NPIL = 412;
__device__ __host__ __forceinline__ bool chest_small(const chest_args& a)
{
  return a.npil <= CH_SMALL_NPIL;
}

// Words of the DM-RS Gold sequences (bits 2 x 6 x prb_lo .. of every DM-RS symbol), shared by every grid
// and port of the batch.
__device__ __forceinline__ uint32_t dmrs_nof_words(const chest_args& a, uint32_t& w_first)
{
  const uint32_t bit_first = 12u * a.prb_lo;
  w_first                  = bit_first / 32;
  return (bit_first + 2 * a.npil + 31) / 32 - w_first;
}

// The DM-RS words of the item into LDS, one thread per word (nds x nwords <= 4 x 106) from the word basis
// (gold_basis_word: 32 independent loads per word, no dependent jump-ahead chain).  Workgroup (0, 0) of the item
// also keeps them in a.dmrs_seq for the statistics kernel.  Returns the bit offset of the first allocated pilot in
// word 0.
__device__ __forceinline__ uint32_t dmrs_words_gen(const chest_args& a, uint32_t (*seq)[CH_SEQWORDS])
{
  uint32_t       w_first;
  const uint32_t nwords = dmrs_nof_words(a, w_first);
  const bool     keep   = blockIdx.x == 0 && blockIdx.y == 0;
#pragma unroll 1
  for (uint32_t i = threadIdx.x; i < a.nds * nwords; i += blockDim.x) {
    const uint32_t d    = i / nwords, w = i % nwords;
    const uint32_t word = gold_basis_word(a.gold_basis, a.c_init[d], w_first + w);
    seq[d][w]           = word;
    if (keep) {
      a.dmrs_seq[d * CH_SEQWORDS + w] = word;
    }
  }
  return 12u * a.prb_lo - 32 * w_first;
}

// The item's DM-RS words from a.dmrs_seq into LDS (statistics kernel).
__device__ __forceinline__ uint32_t dmrs_words(const chest_args& a, uint32_t (*seq)[CH_SEQWORDS])
{
  uint32_t       w_first;
  const uint32_t nwords = dmrs_nof_words(a, w_first);
  for (uint32_t i = threadIdx.x; i < nwords * a.nds; i += blockDim.x) {
    const uint32_t d = i / nwords, w = i % nwords;
    seq[d][w]        = a.dmrs_seq[d * CH_SEQWORDS + w];
  }
  return 12u * a.prb_lo - 32 * w_first;
}

// Time alignment of one slice: the N-point IDFT of its smoothed pilots with the fused Stockham engine and |.|^2
// into the slice's correlation row (time_alignment_estimator_dft_impl.cpp:122-200).
// N <= 512 (npil <= 412): plan<N> on the workgroup's first plan<N>::T threads, input from the pilots in LDS,
// work area in the unused upper half of the pilot buffer.
template <int N>
__device__ __forceinline__ void slice_ta_small(const chest_args& a, const float2* pil, dft::cf* lds, float* corr)
{
  using dft::cf;
  const int npil = static_cast<int>(a.npil);
  auto      load = [&](int i) -> cf {
    if (i < npil) {
      const float2 v = pil[i];
      return cf{v.x, v.y};
    }
    return cf{0, 0};
  };
  auto store = [&](int k, cf v) { corr[k] = v.x * v.x + v.y * v.y; };
  static_assert(dft::plan<N>::T <= CS_THREADS, "IDFT plan wider than the slice workgroup");
  dft::plan<N>::template engine<+1>::run_guarded(lds, reinterpret_cast<const cf*>(a.ta_tw), load, store);
}
// N = 1024 / 2048: 256-thread plans whose first pass takes the thread's own pilots m = tid + 256 r straight from
// its registers x[r] (N / R_first = 256), work area the whole pilot buffer (after a barrier).
using ta_plan_1024 = dft::stockham<1024, CS_THREADS, +1, 4, 4, 4, 4, 4>;
using ta_plan_2048 = dft::stockham<2048, CS_THREADS, +1, 8, 8, 8, 4>;
template <class Plan, int R>
__device__ __forceinline__ void slice_ta_regs(const chest_args& a, const float2 (&x)[CS_PPT], dft::cf* lds,
                                              float* corr)
{
  using dft::cf;
  static_assert(R <= CS_PPT, "first radix beyond the thread's pilots");
  const uint32_t      npil = a.npil;
  dft::reg_input<R> load;
#pragma unroll
  for (int r = 0; r < R; ++r) {
    load.v[r] = threadIdx.x + r * CS_THREADS < npil ? cf{x[r].x, x[r].y} : cf{0, 0};
  }
  auto store = [&](int k, cf v) { corr[k] = v.x * v.x + v.y * v.y; };
  Plan::run(lds, reinterpret_cast<const cf*>(a.ta_tw), load, store);
}

// Pilot buffer of the slice kernel: the FD filter's input, then the smoothed pilots, then the IDFT's work area.
constexpr int CH_ENL = dft::lds_complex<2048>() > CH_MAXPIL + 2 * CH_MAXV ? dft::lds_complex<2048>()
                                                                          : CH_MAXPIL + 2 * CH_MAXV;
static_assert(1024 + dft::lds_complex<512>() <= CH_ENL, "small IDFT work area exceeds the pilot buffer");

// One workgroup per (grid, rx port, slice = layer x LSE symbol): every slice of a port is estimated
// concurrently.  The port's CFO from the first two DM-RS symbols over every layer of every CDM group
// (preprocess_pilots_and_estimate_cfo, :390-445) is computed by each slice workgroup of the port (the same
// operations in the same order, so the same value; slice 0 keeps it in acc for the statistics, expansion and
// equalizer kernels).  Per slice: LSE (rx * conj(pilot)), CFO compensation and time accumulation, CDM pair
// averaging (lane shuffle), scaling, FD smoothing in LDS (mean, or virtual pilots + raised-cosine FIR), the
// slice's RSRP share, linear interpolation to every RE of the allocation
// (port_channel_estimator_average_impl.cpp:130-506), the slice's time-alignment IDFT.
//
// T = 256 threads (eight pilots each, up to 2,048), or T = 64 for allocations of at most CH_SMALL_NPIL pilots (68
// PRBs): one wave per slice, so the small PDUs of a multi-UE slot -- most of its workgroups -- do not hold three idle
// waves through every barrier (the slot form launches both widths, each workgroup leaving at once when its item
// belongs to the other).
template <bool MULTI, int T>
__global__ __launch_bounds__(T) __attribute__((amdgpu_waves_per_eu(T == 256 && !MULTI ? 5 : 4))) void
chest_pilot_kernel(chest_args a_in, chest_items items)
{
  const chest_args& a = item_args<MULTI>(a_in, items);
  if (MULTI && (blockIdx.x >= a.nof_ports || blockIdx.y >= a.L * a.nof_lse || chest_small(a) != (T == 64))) {
    return;
  }
  constexpr int CS_THREADS = T;
  // pilot buffer: the FD filter's input, then (after a barrier) the smoothed pilots the interpolation and the IDFT
  // read, then the IDFT's work area (from WORK_OFF for N <= 512)
  constexpr int ENL      = T == 64 ? CH_SMALL_NPIL + 2 * CH_MAXV + dft::lds_complex<512>() : CH_ENL;
  constexpr int WORK_OFF = T == 64 ? CH_SMALL_NPIL + 2 * CH_MAXV : 1024;
  __shared__ uint32_t seq[CH_MAXDMRS][CH_SEQWORDS];
  __shared__ float2   enl_in[ENL];
  float2* const       enl_out = enl_in;
  __shared__ float    red[4 * 16];
  __shared__ float2   s_rot[CH_MAXDMRS];
  __shared__ int      s_has_cfo;

  const uint32_t gp    = blockIdx.x; // grid * nof_ports + port
  const uint32_t slice = blockIdx.y; // layer * nof_lse + LSE symbol
  const uint32_t grid  = gp / a.nof_ports;
  const uint32_t port  = gp % a.nof_ports;
  const uint32_t tid   = threadIdx.x;
  const uint32_t npil  = a.npil;
  const int      nds   = static_cast<int>(a.nds);
  const int      L     = static_cast<int>(a.L);
  const int      v     = static_cast<int>(slice / a.nof_lse);
  const int      s     = static_cast<int>(slice % a.nof_lse);
  const int      g     = v / 2;
  CHEST_STAMP(0, 0);
  CHEST_STAMP(0, 1);

  const uint32_t* gridp = a.grids + grid * a.grid_stride + static_cast<uint64_t>(port) * CH_NSYMB * a.nsubc +
                          12 * a.prb_lo;
  // received pilot m of CDM group gg in DM-RS symbol d (subcarrier 12 prb_lo + 2m + gg)
  auto rxv = [&](int gg, int d, uint32_t m) { return from_cbf16(gridp[a.dmrs_sym[d] * a.nsubc + 2 * m + gg]); };
  // The thread's pilots of both CDM groups in the first two DM-RS symbols, loaded before the Gold words are
  // generated (their latency hides behind it); the CFO and the slice's LSE of those symbols read them here.
  uint32_t r01[CS_PPT][2][2];
#pragma unroll
  for (int k = 0; k < CS_PPT; ++k) {
    const uint32_t m = tid + k * CS_THREADS;
#pragma unroll
    for (int gg = 0; gg < 2; ++gg) {
#pragma unroll
      for (int d = 0; d < 2; ++d) {
        r01[k][gg][d] = (m < npil && gg < static_cast<int>(a.ncdm) && d < nds)
                            ? gridp[a.dmrs_sym[d] * a.nsubc + 2 * m + gg]
                            : 0u;
      }
    }
  }
  // pilot k of group gg (runtime) in DM-RS symbol d (runtime): the registers above for d < 2
  auto rxk = [&](int k, int gg, int d, uint32_t m) {
    if (d >= 2) {
      return rxv(gg, d, m);
    }
    const uint32_t u0 = gg == 0 ? r01[k][0][0] : r01[k][1][0];
    const uint32_t u1 = gg == 0 ? r01[k][0][1] : r01[k][1][1];
    return from_cbf16(d == 0 ? u0 : u1);
  };
  const uint32_t bit0 = dmrs_words_gen(a, seq);
  __syncthreads(); // seq ready
  CHEST_STAMP(0, 2);

  // The port's CFO: sum over the layers v of (rx_1 conj(p_1,v)) conj(rx_0 conj(p_0,v)).  The two layers of a CDM
  // group differ in their pilots by w_f = -1 on odd indices in both symbols, which cancels in the product: the
  // term of layer 2 gg is added once per layer of the group (as a loop over the layers adds it).
  if (nds >= 2) {
    float4 acc = make_float4(0, 0, 0, 0); // (re, im) of CDM group 0, then 1
#pragma unroll
    for (int k = 0; k < CS_PPT; ++k) {
      const uint32_t m = tid + k * CS_THREADS;
      if (m < npil) {
#pragma unroll
        for (int gg = 0; gg < 2; ++gg) {
          const int nl = min(2, L - 2 * gg); // layers of the group
          if (nl <= 0) {
            continue;
          }
          const float2 p0 = cmulc(from_cbf16(r01[k][gg][0]), pilot(a, seq, bit0, 0, 2 * gg, m));
          const float2 p1 = cmulc(from_cbf16(r01[k][gg][1]), pilot(a, seq, bit0, 1, 2 * gg, m));
          const float2 t  = cmulc(p1, p0);
          for (int r = 0; r < nl; ++r) {
            if (gg == 0) {
              acc.x += t.x;
              acc.y += t.y;
            } else {
              acc.z += t.x;
              acc.w += t.y;
            }
          }
        }
      }
    }
    acc = block_sum4(acc, red);
    // thread d < nds: the rotation of DM-RS symbol d (every such thread computes the same cfo)
    if (tid < static_cast<uint32_t>(nds)) {
      const float de  = a.epoch[a.dmrs_sym[1]] - a.epoch[a.dmrs_sym[0]];
      float       cfo = atan2f(acc.y, acc.x) / TWOPI_F / de;
      if (a.ncdm > 1) {
        cfo += atan2f(acc.w, acc.z) / TWOPI_F / de;
      }
      cfo /= static_cast<float>(a.ncdm);
      s_rot[tid] = a.compensate_cfo ? polar1(-TWOPI_F * a.epoch[a.dmrs_sym[tid]] * cfo) : make_float2(1, 0);
      s_has_cfo = 1;
      if (slice == 0 && tid == 0) {
        float* out = a.acc + static_cast<uint64_t>(gp) * CH_ACC;
        out[3]     = 1.0f;
        out[4]     = cfo;
      }
    }
  } else if (tid == 0) {
    s_rot[0]  = make_float2(1, 0);
    s_has_cfo = 0;
    if (slice == 0) {
      float* out = a.acc + static_cast<uint64_t>(gp) * CH_ACC;
      out[3]     = 0.0f;
      out[4]     = 0.0f;
    }
  }
  __syncthreads(); // rotations ready
  CHEST_STAMP(0, 3);
  const bool  has_cfo  = s_has_cfo != 0;
  const bool  rotate   = has_cfo && a.compensate_cfo;
  const float total    = a.td == SRS_AMD_CHEST_TD_AVERAGE ? (1.0f / a.beta) / static_cast<float>(nds) : 1.0f / a.beta;
  const float rsrp_nrm = a.beta * a.beta * static_cast<float>(nds) / static_cast<float>(a.nof_lse);
  // Pair averaging (average_pairs): one DM-RS symbol -> layers of two-layer CDM groups; more -> every layer if L > 1.
  const bool pair_avg = nds == 1 ? (2 * g + 2 <= L) : (L > 1);

  float2 x[CS_PPT];
#pragma unroll
  for (int k = 0; k < CS_PPT; ++k) {
    const uint32_t m = tid + k * CS_THREADS;
    float2         y = make_float2(0, 0);
    if (m < npil) {
      if (a.td == SRS_AMD_CHEST_TD_AVERAGE) {
        y = cmulc(rxk(k, g, 0, m), pilot(a, seq, bit0, 0, v, m));
        if (rotate) {
          y = cmul(y, s_rot[0]);
        }
#pragma unroll
        for (int d = 1; d < CH_MAXDMRS; ++d) {
          if (d >= nds) {
            break;
          }
          float2 t = cmulc(rxk(k, g, d, m), pilot(a, seq, bit0, d, v, m));
          if (rotate) {
            t = cmul(t, s_rot[d]);
          }
          y = cadd(y, t);
        }
      } else {
        y = cmulc(rxk(k, g, s, m), pilot(a, seq, bit0, s, v, m));
        if (rotate) {
          y = cmul(y, s_rot[s]);
        }
      }
    }
    const float2 o = make_float2(__shfl_xor(y.x, 1), __shfl_xor(y.y, 1));
    if (pair_avg && m < npil) {
      const float2 sum = (m & 1) ? cadd(o, y) : cadd(y, o);
      y                = make_float2(sum.x / 2.0f, sum.y / 2.0f);
    }
    x[k] = cscale(y, total);
  }
  CHEST_STAMP(0, 4);

  // FD smoothing (apply_fd_smoothing, port_channel_estimator_helpers.cpp:213-260).
  bool staged = false; // smoothed pilots already in enl_out
  if (a.fd == SRS_AMD_CHEST_FD_MEAN) {
    float4 sm = make_float4(0, 0, 0, 0);
#pragma unroll
    for (int k = 0; k < CS_PPT; ++k) {
      if (tid + k * CS_THREADS < npil) {
        sm.x += x[k].x;
        sm.y += x[k].y;
      }
    }
    sm              = block_sum4(sm, red);
    const float2 mu = make_float2(sm.x / npil, sm.y / npil);
#pragma unroll
    for (int k = 0; k < CS_PPT; ++k) {
      x[k] = mu;
    }
  } else if (a.fd == SRS_AMD_CHEST_FD_FILTER) {
    const int nv = a.nof_v;
    // the pilots between zero pads of CH_MAXV (the virtual pilots overwrite nv of each pad)
    if (tid < 2 * CH_MAXV) {
      enl_in[tid < CH_MAXV ? tid : npil + tid] = make_float2(0, 0);
    }
#pragma unroll
    for (int k = 0; k < CS_PPT; ++k) {
      const uint32_t m = tid + k * CS_THREADS;
      if (m < npil) {
        enl_in[CH_MAXV + m] = x[k];
      }
    }
    __syncthreads();
    CHEST_STAMP(0, 10);
    if (T == 64) { // one wave: both ends in turn
      virtual_pilots_wave(enl_in + CH_MAXV - nv, enl_in + CH_MAXV, nv, true);
      virtual_pilots_wave(enl_in + CH_MAXV + npil, enl_in + CH_MAXV + npil - nv, nv, false);
    } else if (tid < 64) {
      virtual_pilots_wave(enl_in + CH_MAXV - nv, enl_in + CH_MAXV, nv, true);
    } else if (tid < 128) {
      virtual_pilots_wave(enl_in + CH_MAXV + npil, enl_in + CH_MAXV + npil - nv, nv, false);
    }
    __syncthreads();
    CHEST_STAMP(0, 11);
    // Blocked FIR: thread t filters pilots FB t .. FB t + FB - 1 from one window of FB + 15 LDS values (22 reads
    // instead of one per tap and pilot).  Inputs outside [-nv, npil + nv) read the zero pads: the reference skips
    // them, and adding a +-0 product leaves every partial sum unchanged, so the per-tap order and values are the
    // reference's.  FB = 7: an odd stride of 14 dwords between lanes spreads a wave's window reads over every LDS
    // bank (FB = 8, a 16-dword stride, measured 7.4 us per launch in 16-way bank conflicts).
    constexpr int FB   = 7;
    static_assert(FB * 64 >= static_cast<int>(CH_SMALL_NPIL) && FB * 256 >= 6 * 275, "FIR outputs per thread");
    constexpr int NWIN = FB + CH_MAXV + 3;
    const int     half = a.nof_taps / 2;
    const int     m0   = static_cast<int>(tid) * FB;
    float2        y[FB];
    if (m0 < static_cast<int>(npil)) {
      float2 win[NWIN];
#pragma unroll
      for (int q = 0; q < NWIN; ++q) {
        win[q] = enl_in[CH_MAXV + m0 - half + q];
      }
      // the coefficients once, all loads issued together (a runtime-indexed a.rc read per tap and output was one
      // dependent scalar load each: 6.2 us of the launch)
      float rcv[CH_MAXV + 4];
#pragma unroll
      for (int j = 0; j < CH_MAXV + 4; ++j) {
        rcv[j] = a.rc[max(a.nof_taps - 1 - j, 0)];
      }
#pragma unroll
      for (int i = 0; i < FB; ++i) {
        y[i] = make_float2(0, 0);
      }
#pragma unroll
      for (int j = 0; j < CH_MAXV + 4; ++j) {
        if (j < a.nof_taps) { // per output, taps in ascending order as before
#pragma unroll
          for (int i = 0; i < FB; ++i) {
            y[i].x = y[i].x + win[i + j].x * rcv[j]; // srsran_simd_f_mul then _add
            y[i].y = y[i].y + win[i + j].y * rcv[j];
          }
        }
      }
    }
    __syncthreads(); // every FIR read of enl_in is done before the smoothed pilots overwrite it
    CHEST_STAMP(0, 12);
    if (m0 < static_cast<int>(npil)) {
#pragma unroll
      for (int i = 0; i < FB; ++i) {
        if (m0 + i < static_cast<int>(npil)) {
          enl_out[m0 + i] = y[i];
        }
      }
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < CS_PPT; ++k) {
      const uint32_t m = tid + k * CS_THREADS;
      x[k]             = m < npil ? enl_out[m] : make_float2(0, 0);
    }
    staged = true;
  }

  // RSRP share, store the smoothed pilots, stage them for the interpolation (the blocked FIR staged them already).
  if (!staged) {
    __syncthreads(); // every read of enl_in is done before the smoothed pilots overwrite it
  }
  CHEST_STAMP(0, 5);
  float   rsrp = 0;
  float2* filt = a.filt + (static_cast<uint64_t>(gp) * a.L * a.nof_lse + slice) * npil;
#pragma unroll
  for (int k = 0; k < CS_PPT; ++k) {
    const uint32_t m = tid + k * CS_THREADS;
    if (m < npil) {
      rsrp    = __builtin_fmaf(x[k].x * x[k].x + x[k].y * x[k].y, rsrp_nrm, rsrp);
      filt[m] = x[k];
      if (!staged) {
        enl_out[m] = x[k];
      }
    }
  }
  if (!staged) {
    __syncthreads();
  }
  CHEST_STAMP(0, 6);
  // Linear interpolation (interpolator_linear_impl.cpp): pilots at offset g + 2i.
  float2* fr = a.freq + (static_cast<uint64_t>(gp) * a.L * a.nof_lse + slice) * a.nof_re;
  constexpr uint32_t IU = 4; // outputs per thread and round: their LDS reads issued together
  for (uint32_t k0 = tid; k0 < a.nof_re; k0 += IU * CS_THREADS) {
    float2 out[IU];
#pragma unroll
    for (uint32_t u = 0; u < IU; ++u) {
      const uint32_t kk = min(k0 + u * CS_THREADS, a.nof_re - 1);
      if (kk <= static_cast<uint32_t>(g)) {
        out[u] = enl_out[0];
      } else {
        const uint32_t j = (kk - g) / 2, r = (kk - g) % 2;
        if (j + 1 < npil) {
          const float2 p0 = enl_out[j], p1 = enl_out[j + 1];
          out[u] = r ? make_float2((p1.x - p0.x) * 0.5f + p0.x, (p1.y - p0.y) * 0.5f + p0.y) : p0;
        } else {
          out[u] = enl_out[npil - 1];
        }
      }
    }
#pragma unroll
    for (uint32_t u = 0; u < IU; ++u) {
      if (k0 + u * CS_THREADS < a.nof_re) {
        fr[k0 + u * CS_THREADS] = out[u];
      }
    }
  }
  // the slice's time-alignment correlation row (every thread takes part in the engine's barriers)
  CHEST_STAMP(0, 7);
  float*   corr = a.corr + (static_cast<uint64_t>(gp) * a.L * a.nof_lse + slice) * a.ta_n;
  auto*    work = reinterpret_cast<dft::cf*>(enl_in);
  switch (a.ta_n) {
    case 128: slice_ta_small<128>(a, enl_out, work + WORK_OFF, corr); break;
    case 256: slice_ta_small<256>(a, enl_out, work + WORK_OFF, corr); break;
    case 512: slice_ta_small<512>(a, enl_out, work + WORK_OFF, corr); break;
    default:
      if constexpr (T == 256) {
        __syncthreads(); // the interpolation's reads of the pilot buffer are done
        if (a.ta_n == 1024) {
          slice_ta_regs<ta_plan_1024, 4>(a, x, work, corr);
        } else { // 2048 (the host admits N <= 2048)
          slice_ta_regs<ta_plan_2048, 8>(a, x, work, corr);
        }
      }
      break;
  }
  const float4 tot = block_sum4(make_float4(rsrp, 0, 0, 0), red);
  CHEST_STAMP(0, 8);
  if (tid == 0) {
    a.acc[static_cast<uint64_t>(gp) * CH_ACC + CH_ACC_RSRP + slice] = tot.x;
  }
  CHEST_STAMP(0, 9);
  CHEST_STAMP(0, 15);
}

// Per-port measurements, one workgroup per (grid, port): EPRE over every received DM-RS RE, the noise energy per
// CDM group from the smoothed pilots of every slice (estimate_noise, :594-690), the slices' correlations summed in slice order (the
// reference accumulates them symbol-major; the sum is order-free up to rounding), the peak search and
// quadratic refinement (time_alignment_estimator_dft_impl.cpp:248-310) and noise variance, EPRE, RSRP,
// SNR and CFO (do_compute tail, port_channel_estimator_average_impl.cpp:160-199).
// ST = 1,024 threads, or 256 for allocations of at most CH_SMALL_NPIL pilots (as the pilot kernel's widths).
template <bool MULTI, int ST>
__global__ __launch_bounds__(ST) void chest_stats_kernel(chest_args a_in, chest_items items)
{
  const chest_args& a = item_args<MULTI>(a_in, items);
  if (MULTI && (blockIdx.x >= a.nof_ports || chest_small(a) != (ST == 256))) {
    return;
  }
  constexpr int ST_THREADS = ST;
  __shared__ uint32_t seq[CH_MAXDMRS][CH_SEQWORDS];
  __shared__ float    corr[CH_TA_MAXN];
  __shared__ float    red[4 * 16];
  const uint32_t      gp   = blockIdx.x;
  const uint32_t      grid = gp / a.nof_ports;
  const uint32_t      port = gp % a.nof_ports;
  const uint32_t      tid  = threadIdx.x;
  const uint32_t      npil = a.npil;
  const int           nds  = static_cast<int>(a.nds);
  const int           L    = static_cast<int>(a.L);
  const uint32_t      N    = a.ta_n;
  CHEST_STAMP(1, 0);
  CHEST_STAMP(1, 1);
  const float*        acc  = a.acc + static_cast<uint64_t>(gp) * CH_ACC;
  const uint32_t      bit0 = dmrs_words(a, seq);
  const uint32_t      nsl  = a.L * a.nof_lse;
  const float*        crow = a.corr + static_cast<uint64_t>(gp) * nsl * N;
  for (uint32_t k = tid; k < N; k += ST_THREADS) {
    // compile-time bound (every slice's load in flight at once), sum in slice order
    float v[CH_MAXL * CH_MAXDMRS];
#pragma unroll
    for (uint32_t sl = 0; sl < CH_MAXL * CH_MAXDMRS; ++sl) {
      v[sl] = sl < nsl ? crow[static_cast<uint64_t>(sl) * N + k] : 0.0f;
    }
    float c = 0;
#pragma unroll
    for (uint32_t sl = 0; sl < CH_MAXL * CH_MAXDMRS; ++sl) {
      if (sl < nsl) {
        c += v[sl];
      }
    }
    corr[k] = c;
  }
  __syncthreads(); // seq, corr ready
  CHEST_STAMP(1, 2);

  const bool rotate = acc[3] != 0.0f && a.compensate_cfo;
  float2     rot_fwd[CH_MAXDMRS]; // the noise predictor's phase
#pragma unroll
  for (int d = 0; d < CH_MAXDMRS; ++d) {
    rot_fwd[d] = d < nds ? polar1(TWOPI_F * a.epoch[a.dmrs_sym[d]] * acc[4]) : make_float2(1, 0);
  }
  CHEST_STAMP(1, 10);
  const uint32_t* gridp = a.grids + grid * a.grid_stride + static_cast<uint64_t>(port) * CH_NSYMB * a.nsubc +
                          12 * a.prb_lo;
  const float2*   filt  = a.filt + static_cast<uint64_t>(gp) * a.L * a.nof_lse * npil;
  float           noise0 = 0, noise1 = 0, epre = 0;
  const float     sf     = a.beta / static_cast<float>(a.nof_lse);
  const int nlse = static_cast<int>(a.nof_lse);
  // At most two pilots per thread (npil <= 1,650 with 1,024 threads, <= 412 with 256).  Every load of both is issued
  // before the first is used: the smoothed pilots and received DM-RS REs go into registers from clamped (always
  // valid) addresses, the arithmetic then masks what does not exist -- loads under the runtime guards waited one
  // memory latency per guard.  One LSE slice per layer (average TD strategy) takes this path.
  static_assert(2 * ST_THREADS >= (ST_THREADS == 256 ? static_cast<int>(CH_SMALL_NPIL) : 6 * 275), "pilots per thread");
  float2   F[2][CH_MAXL];       // [pilot][layer]: smoothed pilots (one LSE slice)
  uint32_t R[2][2][CH_MAXDMRS]; // [pilot][CDM group][DM-RS symbol]: received DM-RS REs
  if (nlse == 1) {
#pragma unroll
    for (uint32_t it = 0; it < 2; ++it) {
      const uint32_t mc = min(tid + it * ST_THREADS, npil - 1);
#pragma unroll
      for (int v = 0; v < CH_MAXL; ++v) {
        F[it][v] = filt[static_cast<uint64_t>(min(v, L - 1)) * npil + mc];
      }
#pragma unroll
      for (int g = 0; g < 2; ++g) {
#pragma unroll
        for (int d = 0; d < CH_MAXDMRS; ++d) {
          R[it][g][d] = gridp[a.dmrs_sym[min(d, nds - 1)] * a.nsubc + 2 * mc + min(g, static_cast<int>(a.ncdm) - 1)];
        }
      }
    }
  }
#pragma unroll
  for (uint32_t it = 0; it < 2; ++it) {
    const uint32_t m = tid + it * ST_THREADS;
    if (m >= npil) {
      continue;
    }
    // compile-time bounds on CDM groups, layers, LSE symbols and DM-RS symbols: every load of an iteration is
    // issued before the first is used (the runtime-bounded loops waited one memory latency per load)
#pragma unroll
    for (int g = 0; g < 2; ++g) {
      if (g >= static_cast<int>(a.ncdm)) {
        continue;
      }
      const int v0 = 2 * g, v1 = min(2 * g + 2, L);
      float2    sc0 = make_float2(0, 0), sc1 = make_float2(0, 0);
#pragma unroll
      for (int vi = 0; vi < 2; ++vi) {
        const int v = v0 + vi;
        if (v >= v1) {
          continue;
        }
        float2 t;
        if (nlse == 1) {
          t = cscale(F[it][v], sf);
        } else {
          const float2* fv = filt + static_cast<uint64_t>(v) * a.nof_lse * npil + m;
          t                = cscale(fv[0], sf);
#pragma unroll
          for (int s = 1; s < CH_MAXDMRS; ++s) {
            if (s < nlse) {
              t = cadd(cscale(fv[static_cast<uint64_t>(s) * npil], sf), t);
            }
          }
        }
        if (vi == 0) {
          sc0 = t;
        } else {
          sc1 = t;
        }
      }
#pragma unroll
      for (int d = 0; d < CH_MAXDMRS; ++d) {
        if (d >= nds) {
          continue;
        }
        float2 pred = cmul(sc0, pilot(a, seq, bit0, d, v0, m));
        if (rotate) {
          pred = cmul(pred, rot_fwd[d]);
        }
        if (v1 - v0 == 2) {
          float2 po = cmul(sc1, pilot(a, seq, bit0, d, v0 + 1, m));
          if (rotate) {
            po = cmul(po, rot_fwd[d]);
          }
          pred = cadd(pred, po);
        }
        const float2 rx = from_cbf16(nlse == 1 ? R[it][g][d] : gridp[a.dmrs_sym[d] * a.nsubc + 2 * m + g]);
        epre            = __builtin_fmaf(rx.x, rx.x, __builtin_fmaf(rx.y, rx.y, epre));
        const float2 n  = csub(rx, pred);
        const float  e  = __builtin_fmaf(n.x, n.x, n.y * n.y);
        if (g == 0) {
          noise0 += e;
        } else {
          noise1 += e;
        }
      }
    }
  }
  const float4 tot = block_sum4(make_float4(noise0, noise1, epre, 0), red);
  CHEST_STAMP(1, 3);

  // Peak search of estimate_ta_correlation (time_alignment_estimator_dft_impl.cpp:248-310) over wave 0 instead
  // of a serial scan by one thread: the first maximum (strict >) of corr[0, max_taps) and of
  // corr[N - max_taps, N), each lane scanning a strided subset and the wave keeping the larger value or, on
  // equal values, the smaller index.
  int   i_d = 0, i_a = 0;
  float v_d = 0.0f, v_a = 0.0f;
  if (tid < 64) {
    const int max_taps = a.ta_max_taps;
    float     bd = -__builtin_inff(), ba = -__builtin_inff();
    int       id = 0x7fffffff, ia = 0x7fffffff;
    for (int i = static_cast<int>(tid); i < max_taps; i += 64) {
      const float cd = corr[i];
      const float ca = corr[N - max_taps + i];
      if (i == 0 || cd > bd) {
        bd = cd;
        id = i;
      }
      if (i == 0 || ca > ba) {
        ba = ca;
        ia = i;
      }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float obd = __shfl_xor(bd, o), oba = __shfl_xor(ba, o);
      const int   oid = __shfl_xor(id, o), oia = __shfl_xor(ia, o);
      if (obd > bd || (obd == bd && oid < id)) {
        bd = obd;
        id = oid;
      }
      if (oba > ba || (oba == ba && oia < ia)) {
        ba = oba;
        ia = oia;
      }
    }
    i_d = id;
    v_d = bd;
    i_a = ia;
    v_a = ba;
    if (max_taps <= 0) { // empty ranges (never for a valid configuration): the scan's initial values
      i_d = i_a = 0;
      v_d = corr[0];
      v_a = corr[min(N - max_taps, static_cast<uint32_t>(CH_TA_MAXN - 1))];
    }
  }

  if (tid == 0) {
    float nsum = 0;
    nsum += (isnormal(tot.x) ? tot.x : 0.0f);
    if (a.ncdm > 1) {
      nsum += (isnormal(tot.y) ? tot.y : 0.0f);
    }
    float rsrp_sum = 0;
    for (uint32_t sl = 0; sl < nsl; ++sl) {
      rsrp_sum += acc[CH_ACC_RSRP + sl];
    }
    // estimate_ta_correlation (time_alignment_estimator_dft_impl.cpp:248-310).
    const int max_taps = a.ta_max_taps;
    int       idx      = -(max_taps - i_a);
    if (v_d >= v_a) {
      idx = i_d;
    }
    double frac = 0.0;
    if (a.ta_frac) {
      const int nt = max_taps > 2 ? 5 : 3;
      float     pk[5];
      for (int i = 0; i < nt; ++i) {
        pk[i] = corr[(idx + i + N - nt / 2) % N];
      }
      float num, den, corr_f;
      if (nt == 5) {
        num    = -0.4f * pk[0] + -0.2f * pk[1] + 0.0f * pk[2] + 0.2f * pk[3] + 0.4f * pk[4];
        den    = 0.571429f * pk[0] + -0.285714f * pk[1] + -0.571429f * pk[2] + -0.285714f * pk[3] + 0.571429f * pk[4];
        corr_f = 1.0f;
      } else {
        num    = -0.5f * pk[0] + 0.5f * pk[2];
        den    = 0.5f * pk[0] - pk[1] + 0.5f * pk[2];
        corr_f = 0.5f;
      }
      const float r = -corr_f * num / den;
      frac          = (isnan(r) || isinf(r) || fabsf(r) > 1.0f) ? 0.0 : static_cast<double>(r);
    }
    const double ta_s = (static_cast<double>(idx) + frac) / a.ta_fs;
    // phy_time_unit::from_seconds (phy_time_unit.h:275-283) -> to_seconds.
    constexpr double T_C = 1.0 / (480000.0 * 4096.0);
    const long       tcx = static_cast<long>(ta_s / T_C * 10.0);
    const long       tc  = tcx / 10 + (tcx % 10) / 5;

    // do_compute tail (port_channel_estimator_average_impl.cpp:160-199).
    const float npilt  = static_cast<float>(npil * a.nds);
    const float rsrp   = rsrp_sum / (npilt * static_cast<float>(a.L));
    const float epre   = tot.z / npilt;
    float       nvar   = nsum / (npilt * static_cast<float>(a.ncdm) - 1.0f);
    nvar               = fmaxf(rsrp / 1e10f, nvar);
    const float datarp = rsrp * static_cast<float>(a.L) / a.beta / a.beta;
    const float snr    = isnormal(nvar) ? datarp / nvar : 0.0f;

    srs_amd_chest_port_stats st;
    st.noise_var        = nvar;
    st.epre             = epre;
    st.rsrp             = rsrp;
    st.snr              = snr;
    st.time_alignment_s = static_cast<float>(static_cast<double>(tc) * T_C);
    st.cfo_hz           = acc[3] != 0.0f ? acc[4] * a.scs_hz : __builtin_nanf("");
    a.stats[gp]         = st;
  }
  CHEST_STAMP(1, 4);
  CHEST_STAMP(1, 15);
}

// Channel estimates: one thread per (grid, port, layer, symbol, subcarrier). Inside the
// allocation the time-domain strategy and bf16 rounding; the CFO phase then multiplies the
// whole OFDM symbol (do_compute, port_channel_estimator_average_impl.cpp:184-193), so REs
// outside the allocation are rotated in place, as the reference does.
template <bool MULTI>
__global__ __launch_bounds__(256) void chest_expand_kernel(chest_args a_in, chest_items items)
{
  const chest_args& a = item_args<MULTI>(a_in, items);
  if (MULTI && blockIdx.y >= a.nof_ports * a.L) {
    return;
  }
  // one thread per subcarrier and (grid, port, layer): the LSE estimates of the subcarrier are read
  // once and every OFDM symbol of the allocation written from them
  __shared__ float2 s_ph[CH_NSYMB];
  const uint32_t    sc   = blockIdx.x * 256 + threadIdx.x;
  const uint32_t    gpv  = blockIdx.y; // (grid * nof_ports + port) * L + layer
  const uint32_t    gp   = gpv / a.L;
  const uint32_t    v    = gpv % a.L;
  const uint32_t    grid = gp / a.nof_ports, port = gp % a.nof_ports;
  const float*      acc  = a.acc + static_cast<uint64_t>(gp) * CH_ACC;
  const bool        rot  = chdev::cfo_rotates(a, acc);
  if (rot && threadIdx.x < a.nof_symbols) {
    const uint32_t l  = a.first_symbol + threadIdx.x;
    s_ph[threadIdx.x] = chdev::cfo_phase(a, acc, l);
  }
  __syncthreads();
  if (sc >= a.nsubc) {
    return;
  }
  uint32_t*      est = a.estimates + grid * a.est_stride + (static_cast<uint64_t>(port) * a.L + v) * CH_NSYMB * a.nsubc + sc;
  const uint32_t kk  = sc - 12 * a.prb_lo; // wraps for sc below the allocation
  const bool     in  = kk < a.nof_re;
  if (!in && !rot) {
    return;
  }
  float2 x[CH_MAXDMRS];
  if (in) {
    const float2* fr = a.freq + (static_cast<uint64_t>(gp) * a.L + v) * a.nof_lse * a.nof_re + kk;
#pragma unroll
    for (int s = 0; s < CH_MAXDMRS; ++s) {
      x[s] = s < static_cast<int>(a.nof_lse) ? fr[static_cast<uint64_t>(s) * a.nof_re] : make_float2(0, 0);
    }
  }
  for (uint32_t n = 0; n < a.nof_symbols; ++n) {
    const uint32_t l = a.first_symbol + n;
    uint32_t       out;
    if (in) {
      out = chdev::expand_value(a, x, l, rot, rot ? s_ph[n] : make_float2(1, 0));
    } else {
      out = est[static_cast<uint64_t>(l) * a.nsubc];
      if (rot) {
        out = to_cbf16(cmul(from_cbf16(out), s_ph[n]));
      }
    }
    est[static_cast<uint64_t>(l) * a.nsubc] = out;
  }
}

} // namespace

#ifdef SRS_AMD_CHEST_PROBE
extern "C" int srs_amd_chest_probe_read(void* host, uint64_t bytes, int clear)
{
  if (bytes > sizeof(g_chest_probe)) {
    bytes = sizeof(g_chest_probe);
  }
  if (hipMemcpyFromSymbol(host, HIP_SYMBOL(g_chest_probe), bytes) != hipSuccess) {
    return -2;
  }
  if (clear) {
    static const uint64_t zero[2 * CHEST_PROBE_WG * 16] = {};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_chest_probe), zero, sizeof(zero)) != hipSuccess) {
      return -2;
    }
  }
  return 0;
}
#endif

hipError_t launch_chest(const chest_args& a, uint32_t nof_grids, hipStream_t stream, bool expand)
{
  const uint32_t nb = nof_grids * a.nof_ports;
  if (nb == 0) {
    return hipSuccess;
  }
  if (a.ta_n > 2048) { // the pilot kernel's largest IDFT (4096 npil / (275 x 12), npil <= 1650)
    return hipErrorInvalidValue;
  }
  const dim3 slices(nb, a.L * a.nof_lse);
  if (chest_small(a)) {
    hipLaunchKernelGGL((chest_pilot_kernel<false, 64>), slices, dim3(64), 0, stream, a, chest_items{});
  } else {
    hipLaunchKernelGGL((chest_pilot_kernel<false, 256>), slices, dim3(256), 0, stream, a, chest_items{});
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    return e;
  }
  if (chest_small(a)) {
    hipLaunchKernelGGL((chest_stats_kernel<false, 256>), dim3(nb), dim3(256), 0, stream, a, chest_items{});
  } else {
    hipLaunchKernelGGL((chest_stats_kernel<false, 1024>), dim3(nb), dim3(1024), 0, stream, a, chest_items{});
  }
  e = hipGetLastError();
  if (e != hipSuccess) {
    return e;
  }
  if (!expand) {
    return hipSuccess; // the consumer rebuilds the estimates from a.freq / a.acc (chest_device.h)
  }
  hipLaunchKernelGGL(chest_expand_kernel<false>, dim3((a.nsubc + 255) / 256, nb * a.L), dim3(256), 0, stream, a,
                     chest_items{});
  return hipGetLastError();
}

hipError_t launch_chest_items(const chest_items& items, uint32_t nof_items, uint32_t max_ports, uint32_t max_slices,
                              uint32_t nof_small, hipStream_t stream)
{
  if (nof_items == 0) {
    return hipSuccess;
  }
  const chest_args none{};
  const dim3       slices(max_ports, max_slices, nof_items);
  hipError_t       e = hipSuccess;
  // each launch covers every item; the workgroups of the other width's items leave at once
  if (nof_small != 0) {
    hipLaunchKernelGGL((chest_pilot_kernel<true, 64>), slices, dim3(64), 0, stream, none, items);
    e = hipGetLastError();
  }
  if (e == hipSuccess && nof_small != nof_items) {
    hipLaunchKernelGGL((chest_pilot_kernel<true, 256>), slices, dim3(256), 0, stream, none, items);
    e = hipGetLastError();
  }
  if (e == hipSuccess && nof_small != 0) {
    hipLaunchKernelGGL((chest_stats_kernel<true, 256>), dim3(max_ports, 1, nof_items), dim3(256), 0, stream, none,
                       items);
    e = hipGetLastError();
  }
  if (e == hipSuccess && nof_small != nof_items) {
    hipLaunchKernelGGL((chest_stats_kernel<true, 1024>), dim3(max_ports, 1, nof_items), dim3(1024), 0, stream, none,
                       items);
    e = hipGetLastError();
  }
  return e;
}

} // namespace srs_amd
