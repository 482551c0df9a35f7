// ulsch_demux.hip -- MI355X UL-SCH demultiplexer kernel (include/srsran_amd/ulsch_demux.h): one thread per
// (codeword, data RE) copies the RE's layers x Qm LLRs to its stream position(s) from the plan's placement
// table (ulsch_demultiplex_impl.cpp:446-590), reverting the scrambling of the repetition placeholders of
// 1/2-bit UCI (on_uci_placeholder_1bit / _2bit, :92-194) from the codeword's Gold words.  HBM-bound: every
// codeword byte read once, every stream byte written once.
#include <hip/hip_runtime.h>

#include "ulsch_demux_args.h"

namespace srs_amd {
namespace {

constexpr int DMX_THREADS = 256;
constexpr int DMX_MAXB    = 32; // layers x Qm <= 4 x 8

__device__ __forceinline__ uint32_t scr_bit(const uint32_t* scr, uint32_t n)
{
  return (scr[n >> 5] >> (n & 31)) & 1u;
}

// MULTI: one argument block per codeword (items[blockIdx.y], row 0), the slot form of the PUSCH processor
template <bool MULTI>
__global__ __launch_bounds__(DMX_THREADS) void ulsch_demux_kernel(demux_args own, const demux_args* items)
{
  const demux_args& a   = MULTI ? items[blockIdx.y] : own;
  const uint32_t    re  = blockIdx.x * DMX_THREADS + threadIdx.x;
  const uint64_t    row = MULTI ? 0u : blockIdx.y;
  if (re >= a.nof_re || (MULTI && a.sel != nullptr && *a.sel != a.sel_val)) {
    return;
  }
  const uint32_t s = a.sch_map[re];
  const uint32_t u = a.uci_map[re];
  const int8_t*  in = a.cws + row * a.cw_stride + static_cast<uint64_t>(re) * a.bpre;
  int8_t         v[DMX_MAXB];
  for (uint32_t b = 0; b < a.bpre; ++b) {
    v[b] = in[b];
  }
  const uint32_t n0 = re * a.bpre; // codeword bit of the RE's first LLR
  // one UCI stream's copy of the RE, the placeholder scrambling of a 1/2-bit payload reverted
  auto put_uci = [&](int8_t* out, uint32_t ph, bool zero) {
    for (uint32_t b = 0; b < a.bpre; ++b) {
      int8_t x = zero ? int8_t(0) : v[b];
      if (ph != 0 && a.qm > 1) {
        const uint32_t k = b % a.qm; // bit of the modulation symbol
        if (k >= 2) {
          // placeholder x: revert the scrambling
          x = scr_bit(a.scr, n0 + b) ? static_cast<int8_t>(-x) : x;
        } else if (k == 1 && ph == 1) {
          // placeholder y: revert the second bit's scrambling and apply the first bit's mask
          x = (scr_bit(a.scr, n0 + b - 1) ^ scr_bit(a.scr, n0 + b)) ? static_cast<int8_t>(-x) : x;
        }
      }
      out[b] = x;
    }
  };
  if (u != DMX_NONE) {
    const uint32_t kind = u >> DMX_KIND_SHIFT;
    int8_t*        out  = kind == DMX_ACK ? a.ack + row * a.ack_stride : a.csi1 + row * a.csi1_stride;
    put_uci(out + static_cast<uint64_t>(u & DMX_INDEX_MASK) * a.bpre, kind == DMX_ACK ? a.ack_ph : a.csi1_ph, false);
  }
  if (a.csi2_map != nullptr) {
    // CSI part 2 after HARQ-ACK: a RE it shares with a 1/2-bit HARQ-ACK was zeroed by the HARQ-ACK extraction
    const uint32_t c2 = a.csi2_map[re];
    if (c2 != DMX_NONE) {
      put_uci(a.csi2 + row * a.csi2_stride + static_cast<uint64_t>(c2 & ~DMX_ZERO) * a.bpre, a.csi2_ph,
              (c2 & DMX_ZERO) != 0);
    }
  }
  if (s != DMX_NONE) {
    int8_t*    out  = a.sch + row * a.sch_stride + static_cast<uint64_t>(s & ~DMX_ZERO) * a.bpre;
    const bool zero = (s & DMX_ZERO) != 0;
    for (uint32_t b = 0; b < a.bpre; ++b) {
      out[b] = zero ? int8_t(0) : v[b];
    }
  }
}

} // namespace

hipError_t launch_ulsch_demux(const demux_args& a, uint32_t nof_cws, hipStream_t stream)
{
  if (a.nof_re == 0 || nof_cws == 0) {
    return hipSuccess;
  }
  hipLaunchKernelGGL(ulsch_demux_kernel<false>, dim3((a.nof_re + DMX_THREADS - 1) / DMX_THREADS, nof_cws),
                     dim3(DMX_THREADS), 0, stream, a, nullptr);
  return hipGetLastError();
}

hipError_t launch_ulsch_demux_items(const demux_args* items, uint32_t n, uint32_t max_re, hipStream_t stream)
{
  if (n == 0 || max_re == 0) {
    return hipSuccess;
  }
  hipLaunchKernelGGL(ulsch_demux_kernel<true>, dim3((max_re + DMX_THREADS - 1) / DMX_THREADS, n), dim3(DMX_THREADS),
                     0, stream, demux_args{}, items);
  return hipGetLastError();
}

} // namespace srs_amd
