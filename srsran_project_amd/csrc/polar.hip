// polar.hip -- MI355X polar encoder / decoder chains (PDCCH / PUCCH / PUSCH UCI).
//
// One wavefront per codeword, 4 codewords per workgroup; everything lives in
// LDS (N <= 1024).  Per-code tables (polar_code.cpp) turn the reference's
// sequential pieces into gathers:
//   encode (pdcch_encoder_impl chain: polar_allocator_impl.cpp:29-69,
//   polar_encoder_impl.cpp:29-82, polar_rate_matcher_impl.cpp:29-106):
//     u[msg_pos[k]] = message[k]; parity-check bits by the reference's 5-register
//     cyclic shift (one lane, only codes with K <= 25); x = polar transform of u
//     (log2 N butterfly stages); out[k] = x[tx_map[k]].
//   decode (polar_rate_dematcher_impl.cpp:29-118, polar_decoder_impl.cpp:28-350,
//   polar_deallocator_impl.cpp:27-42):
//     L_n[blk[j]] = y[j], y from the received LLRs by the channel deinterleaver,
//     repetition (promotion sums in index order), puncturing (0) or shortening
//     (+inf); then the SSC program: F (min-sum soft xor), G (saturated
//     switch-combine), XOR (partial-sum combine), R1 (hard decision + re-encode);
//     message[k] = u_hat[msg_pos[k]].
// LLR arithmetic is the reference's int8 LLR type (log_likelihood_ratio.cpp):
// sums saturate at +-120, +-127 is infinity, opposite infinities cancel.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "polar_args.h"

namespace srs_amd {
namespace {

constexpr int WAVES = 4;

__device__ __forceinline__ void wave_sync()
{
  // Lanes of one wave exchange data through LDS; LDS operations of a wave
  // complete in order, this only stops the compiler from reordering them.
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ bool llr_isinf(int a)
{
  return a > 120 || a < -120;
}

// a += b (log_likelihood_ratio.cpp:58)
__device__ __forceinline__ int llr_sum(int a, int b)
{
  if (a == -b) {
    return 0;
  }
  if (llr_isinf(a)) {
    return a;
  }
  if (llr_isinf(b)) {
    return b;
  }
  return min(max(a + b, -120), 120);
}

// log_likelihood_ratio::promotion_sum (log_likelihood_ratio.cpp:75)
__device__ __forceinline__ int llr_promotion_sum(int a, int b)
{
  if (a == -b) {
    return 0;
  }
  if (llr_isinf(a)) {
    return a;
  }
  if (llr_isinf(b)) {
    return b;
  }
  const int s = a + b;
  return s > 120 ? 127 : (s < -120 ? -127 : s);
}

// log_likelihood_ratio::soft_xor (log_likelihood_ratio.h:207)
__device__ __forceinline__ int soft_xor(int x, int y)
{
  const int m = min(abs(x), abs(y));
  return (x * y < 0) ? -m : m;
}

// In-place polar transform of n_bits bits at p (stage_function recursion of
// polar_encoder_impl.cpp, bottom-up).
__device__ __forceinline__ void transform(uint8_t* b, int n_bits, int lane)
{
  for (int d = 1; d < n_bits; d <<= 1) {
    for (int i = lane; i < n_bits / 2; i += 64) {
      const int lo = (i / d) * 2 * d + (i % d);
      b[lo] ^= b[lo + d];
    }
    wave_sync();
  }
}

} // namespace

__global__ __launch_bounds__(64 * WAVES) void polar_encode_kernel(polar_args a)
{
  __shared__ uint8_t ubuf[WAVES][1024];
  const int          wave = threadIdx.x >> 6;
  const int          lane = threadIdx.x & 63;
  const uint32_t     cw   = blockIdx.x * WAVES + wave;
  if (cw >= a.nof) {
    return;
  }
  uint8_t*       u   = ubuf[wave];
  const uint8_t* msg = a.msgs + static_cast<size_t>(cw) * a.msg_stride;
  const int      N   = static_cast<int>(a.N);
  for (int i = lane; i < N; i += 64) {
    u[i] = 0;
  }
  wave_sync();
  for (int k = lane; k < static_cast<int>(a.K); k += 64) {
    u[a.msg_pos[k]] = msg[k] & 1u;
  }
  wave_sync();
  if (a.nPC > 0 && lane == 0) {
    // polar_allocator_impl.cpp:44-67: parity-check bits from a cyclic shift register.
    uint32_t y0 = 0, y1 = 0, y2 = 0, y3 = 0, y4 = 0, ipc = 0;
    for (int i = 0; i < N; ++i) {
      const uint32_t t = y0;
      y0               = y1;
      y1               = y2;
      y2               = y3;
      y3               = y4;
      y4               = t;
      if (a.kset[i]) {
        if (ipc < a.nPC && static_cast<uint32_t>(i) == a.pc_set[ipc]) {
          ++ipc;
          u[i] = static_cast<uint8_t>(y0);
        } else {
          y0 ^= u[i];
        }
      }
    }
  }
  wave_sync();
  transform(u, N, lane);
  uint8_t* out = a.cws + static_cast<size_t>(cw) * a.cw_stride;
  for (int k = lane; k < static_cast<int>(a.E); k += 64) {
    out[k] = u[a.tx_map[k]];
  }
}

// MULTI: one argument block (one codeword, its own code) per wave: items[blockIdx.x * WAVES + wave], nof items
template <bool MULTI>
__global__ __launch_bounds__(64 * WAVES) void polar_decode_kernel(polar_args own, const polar_args* items,
                                                                   uint32_t nof)
{
  __shared__ int8_t  llr_all[WAVES][2048]; // stage s at offset 2^s - 1
  __shared__ uint8_t est_all[WAVES][1024];
  __shared__ uint8_t msg_all[WAVES][1024];
  const int          wave = threadIdx.x >> 6;
  const int          lane = threadIdx.x & 63;
  const uint32_t     w    = blockIdx.x * WAVES + wave;
  if (w >= (MULTI ? nof : own.nof)) {
    return;
  }
  const polar_args& a  = MULTI ? items[w] : own;
  const uint32_t    cw = MULTI ? 0u : w;
  if (MULTI && a.pred != nullptr && *a.pred != a.pred_val) {
    return; // one wave per item: nothing else of the workgroup waits for it
  }
  int8_t*       llr = llr_all[wave];
  uint8_t*      est = est_all[wave];
  uint8_t*      dec = msg_all[wave];
  const int8_t* in  = a.llrs + static_cast<size_t>(cw) * a.llr_stride;
  const int     N   = static_cast<int>(a.N);
  const int     E   = static_cast<int>(a.E);

  // ---- rate dematching: L_n[blk[j]] = y[j]
  int8_t* top = llr + (N - 1);
  for (int j = lane; j < N; j += 64) {
    int v;
    if (a.mode == 0) { // repetition: promotion sums in index order
      v = in[a.rx_e2f[j]];
      for (int k = j + N; k < E; k += N) {
        v = llr_promotion_sum(v, in[a.rx_e2f[k]]);
      }
    } else if (a.mode == 1) { // puncturing: the first N - E bits unknown
      v = j < N - E ? 0 : in[a.rx_e2f[j - (N - E)]];
    } else { // shortening: the last N - E bits known zero
      v = j < E ? in[a.rx_e2f[j]] : 127;
    }
    top[a.blk[j]] = static_cast<int8_t>(v);
    est[j]        = 0;
    dec[j]        = 0;
  }
  wave_sync();

  // ---- SSC program (the next operation's word is loaded one step ahead, behind the current step's LDS work)
  uint32_t next = a.prog_len != 0 ? a.program[0] : 0u;
  for (uint32_t o = 0; o < a.prog_len; ++o) {
    const uint32_t op = next;
    if (o + 1 < a.prog_len) {
      next = a.program[o + 1];
    }
    const int      type = op & 3;
    const int      s    = (op >> 2) & 63;
    const int      p    = op >> 8;
    const int      size = 1 << s;
    const int8_t*  L    = llr + (size - 1);
    if (type == POLAR_OP_R1) {
      for (int i = lane; i < size; i += 64) {
        const uint8_t b = L[i] <= 0;
        est[p + i]      = b;
        dec[p + i]      = b;
      }
      wave_sync();
      if (s > 0) {
        transform(dec + p, size, lane);
      }
      continue;
    }
    const int h  = size >> 1;
    int8_t*   Lc = llr + (h - 1);
    if (type == POLAR_OP_F) {
      for (int i = lane; i < h; i += 64) {
        Lc[i] = static_cast<int8_t>(soft_xor(L[i], L[i + h]));
      }
    } else if (type == POLAR_OP_G) {
      for (int i = lane; i < h; i += 64) {
        // switch_combine(llr1, llr0, b): b == 0 ? llr0 += llr1 : (-llr0) += llr1
        const int x = L[i];
        Lc[i]       = static_cast<int8_t>(llr_sum(est[p + i] ? -x : x, L[i + h]));
      }
    } else {
      for (int i = lane; i < h; i += 64) {
        est[p + i] ^= est[p + h + i];
      }
    }
    wave_sync();
  }

  // ---- deallocation
  uint8_t* msg = a.msgs_out + static_cast<size_t>(cw) * a.msg_stride;
  for (int k = lane; k < static_cast<int>(a.K); k += 64) {
    msg[k] = dec[a.msg_pos[k]];
  }
}

hipError_t launch_polar_encode(const polar_args& a, hipStream_t stream)
{
  if (a.nof == 0) {
    return hipSuccess;
  }
  hipLaunchKernelGGL(polar_encode_kernel, dim3((a.nof + WAVES - 1) / WAVES), dim3(64 * WAVES), 0, stream, a);
  return hipGetLastError();
}

hipError_t launch_polar_decode(const polar_args& a, hipStream_t stream)
{
  if (a.nof == 0) {
    return hipSuccess;
  }
  hipLaunchKernelGGL(polar_decode_kernel<false>, dim3((a.nof + WAVES - 1) / WAVES), dim3(64 * WAVES), 0, stream, a,
                     nullptr, 0u);
  return hipGetLastError();
}

hipError_t launch_polar_decode_items(const polar_args* items, uint32_t n, hipStream_t stream)
{
  if (n == 0) {
    return hipSuccess;
  }
  hipLaunchKernelGGL(polar_decode_kernel<true>, dim3((n + WAVES - 1) / WAVES), dim3(64 * WAVES), 0, stream,
                     polar_args{}, items, n);
  return hipGetLastError();
}

} // namespace srs_amd
