// ldpc_rate_matching.hip -- MI355X kernels for LDPC rate matching (PDSCH) and
// rate dematching (PUSCH), TS 38.212 Section 5.4.2.
//
// Both kernels are gathers over the circular buffer (rate_matching_common.h):
// HBM traffic is one read of the source and one write of the destination, so
// they are HBM/latency bound and trivial next to the decoder; what matters is
// being exact and never needing a host round trip.
//
// Dematching (ldpc_rate_dematcher_impl.cpp:36-217) is recast from the
// reference's sequential walk over the input into a per-OUTPUT-position rule,
// so every soft-buffer byte is produced by one thread with no write conflicts:
//   * deinterleaving (…:200 deinterleave_bits_Qm): input index t reads
//     in[(t mod K) * Qm + t div K], K = E / Qm;
//   * position p (non-filler, p < Ncb) receives inputs t0(p) + c*L, c = 0, 1, …
//     with t0(p) = (walk(p) - rank0) mod L;
//   * new data (…:123 allot_llrs copy mode): the reference's first loop pass
//     (the walk from k0 to the end of the buffer, t < L1 = L - rank0) copies,
//     everything after combines; before copying it zeroes [0, k0) when k0 lies
//     in the information part, else [0, nof_info), and sets the filler bits to
//     +inf (127); when the input ends inside the first pass it zeroes the LAST
//     Ncb - tmp positions of the N-long buffer (…:214, out.last()), tmp being
//     where the walk stopped (skips to nof_sys if it stopped in the systematic
//     part); positions it does not cover keep their old value.
//   * combining is the LLR saturated sum new += old (log_likelihood_ratio.cpp:58):
//     two infinities of opposite sign give 0, otherwise an infinite operand
//     (|x| > 120) wins -- the new one first -- otherwise clamp to +-120.
//
// Rate matching (ldpc_rate_matcher_impl.cpp:93-170): output bit o of a
// codeblock is e[(o mod Qm) * K + o div Qm] (bit interleaver), e[t] the
// codeblock bit at walk index (rank0 + t) mod L.  One thread per output BYTE
// of the concatenated codeword; a byte that straddles two codeblocks' segments
// is owned by the codeblock holding its first bit, which also computes the
// following codeblocks' bits, so no two threads write one byte.
#include <hip/hip_runtime.h>

#include <type_traits>

#include "ldpc_common.h"
#include "ldpc_codec_args.h"
#include "rate_match_device.h"

namespace srs_amd {

namespace {


// LLR saturated sum a += b, a = new input, b = old soft bit (log_likelihood_ratio.cpp:38-74).
__device__ __forceinline__ int llr_sum(int a, int b)
{
  if (a == -b) {
    return 0;
  }
  if (a > LLR_MAX || a < -LLR_MAX) {
    return a;
  }
  if (b > LLR_MAX || b < -LLR_MAX) {
    return b;
  }
  return min(max(a + b, -LLR_MAX), LLR_MAX);
}

} // namespace


constexpr int DEMATCH_THREADS   = 256;
constexpr int DEMATCH_PER_THREAD = 16;
constexpr uint32_t DEMATCH_UNROLL = 4; // staging loads in flight per thread
constexpr uint32_t DEMATCH_LDS   = 12288; // received LLRs of a codeblock staged in LDS up to this length (8 resident workgroups per CU)

// One workgroup per codeblock: the codeblock's received LLRs (deinterleaver input) are staged in LDS
// with coalesced loads when they fit, then each thread produces 16 consecutive soft-buffer bytes.
// RAGGED: per-codeblock geometry (a.row_geo / a.geos / a.geo_write_end), a separate instantiation so the
// uniform launch keeps its geometry in kernel arguments.
template <bool RAGGED>
__global__ __launch_bounds__(DEMATCH_THREADS) void ldpc_rate_dematch_kernel(dematch_args a)
{
  __shared__ __attribute__((aligned(16))) int8_t s_in[DEMATCH_LDS];
  for (uint32_t cb = blockIdx.y; cb < a.nof_cbs; cb += gridDim.y) {
    const uint32_t    gi        = RAGGED ? a.row_geo[cb] : 0u;
    const rm_geometry g         = RAGGED ? a.geos[gi] : a.g;
    const uint32_t    write_end = RAGGED ? a.geo_write_end[gi] : a.write_end;
    const uint32_t flags    = RAGGED && a.row_flags != nullptr ? a.row_flags[cb] : 0u;
    const int32_t  new_data = RAGGED && a.row_flags != nullptr ? static_cast<int32_t>(flags & 1u) : a.new_data;
    const int32_t  fresh    = RAGGED && a.row_flags != nullptr ? static_cast<int32_t>((flags >> 1) & 1u) : a.fresh;
    const uint32_t E   = a.rm_lengths[cb];
    const int8_t*  in  = a.in + a.in_offsets[cb];
    int8_t*        buf = a.soft + static_cast<size_t>(cb) * a.soft_stride;
    const uint32_t Kq  = E / g.Qm;
    const fast_div divK(Kq);
    // Staged in LDS already deinterleaved (s_in[t], t = j Kq + i <- in[i Qm + j]): consecutive soft-buffer
    // positions then read consecutive LDS bytes (the interleaved order put the lanes of a wave 16 Qm
    // bytes apart, a 32-way bank conflict per read).
    const bool staged = E <= DEMATCH_LDS && Kq * g.Qm == E;
    if (staged) {
      __syncthreads(); // s_in of the previous codeblock is no longer read
      const fast_div divQ(g.Qm);
      auto           put = [&](uint32_t x, int8_t v) {
        uint32_t j;
        const uint32_t i = divQ.div(x, j);
        s_in[j * Kq + i] = v;
      };
      // one thread per modulation symbol i: its Qm LLRs (one load) to rows j = 0 .. Qm-1
      auto by_symbol = [&](auto qm_tag) {
        constexpr uint32_t QM = decltype(qm_tag)::value;
        using word            = typename std::conditional<QM == 8, uint2, typename std::conditional<QM == 4, uint32_t, uint16_t>::type>::type;
        // DEMATCH_UNROLL symbols per thread per round, all loads issued before the LDS stores (a
        // load-then-store loop waits one memory latency per symbol)
        for (uint32_t i0 = threadIdx.x; i0 < Kq; i0 += DEMATCH_UNROLL * DEMATCH_THREADS) {
          union {
            word   w;
            int8_t b[QM];
          } u[DEMATCH_UNROLL];
#pragma unroll
          for (uint32_t r = 0; r < DEMATCH_UNROLL; ++r) {
            const uint32_t i = i0 + r * DEMATCH_THREADS;
            u[r].w           = i < Kq ? reinterpret_cast<const word*>(in)[i] : word{};
          }
#pragma unroll
          for (uint32_t r = 0; r < DEMATCH_UNROLL; ++r) {
            const uint32_t i = i0 + r * DEMATCH_THREADS;
            if (i < Kq) {
#pragma unroll
              for (uint32_t j = 0; j < QM; ++j) {
                s_in[j * Kq + i] = u[r].b[j];
              }
            }
          }
        }
      };
      const uintptr_t ia = reinterpret_cast<uintptr_t>(in);
      if (g.Qm == 8 && (ia & 15u) == 0 && (Kq & 3u) == 0) {
        // four symbols per thread and round: 32 LLR bytes (two 16-byte loads), transposed into the eight
        // rows' 4-byte words (v_perm_b32) and stored with one aligned ds_write_b32 per row -- byte stores put
        // four lanes on every LDS dword
        const uint32_t ng = Kq / 4;
        for (uint32_t q0 = threadIdx.x; q0 < ng; q0 += DEMATCH_UNROLL * DEMATCH_THREADS) {
          uint4 u[DEMATCH_UNROLL][2];
#pragma unroll
          for (uint32_t r = 0; r < DEMATCH_UNROLL; ++r) {
            const uint32_t q = q0 + r * DEMATCH_THREADS;
            u[r][0]          = q < ng ? reinterpret_cast<const uint4*>(in)[2 * q] : uint4{};
            u[r][1]          = q < ng ? reinterpret_cast<const uint4*>(in)[2 * q + 1] : uint4{};
          }
#pragma unroll
          for (uint32_t r = 0; r < DEMATCH_UNROLL; ++r) {
            const uint32_t q = q0 + r * DEMATCH_THREADS;
            if (q < ng) {
              // symbol s of the group: LLR bytes s0 = (u[s/2] word 2(s%2)), s1 = (word 2(s%2) + 1)
              const uint32_t lo[4] = {u[r][0].x, u[r][0].z, u[r][1].x, u[r][1].z}; // LLRs 0-3 of symbols 0-3
              const uint32_t hi[4] = {u[r][0].y, u[r][0].w, u[r][1].y, u[r][1].w}; // LLRs 4-7
#pragma unroll
              for (uint32_t j = 0; j < 8; ++j) {
                const uint32_t* w  = j < 4 ? lo : hi;
                const uint32_t  b  = j & 3u;
                // bytes b of w[0], w[1] into the low half, of w[2], w[3] into the high half
                const uint32_t  p01 = __builtin_amdgcn_perm(w[1], w[0], (b) | ((4 + b) << 8) | 0x0c0c0000u);
                const uint32_t  p23 = __builtin_amdgcn_perm(w[3], w[2], (b) | ((4 + b) << 8) | 0x0c0c0000u);
                reinterpret_cast<uint32_t*>(s_in + j * Kq)[q] = p01 | (p23 << 16);
              }
            }
          }
        }
      } else if (g.Qm == 8 && (ia & 7u) == 0) {
        by_symbol(std::integral_constant<uint32_t, 8>{});
      } else if (g.Qm == 4 && (ia & 3u) == 0) {
        by_symbol(std::integral_constant<uint32_t, 4>{});
      } else if (g.Qm == 2 && (ia & 1u) == 0) {
        by_symbol(std::integral_constant<uint32_t, 2>{});
      } else if (((reinterpret_cast<uintptr_t>(in) | E) & 15u) == 0) {
        for (uint32_t x = threadIdx.x; x < E / 16; x += DEMATCH_THREADS) {
          union {
            uint4  v;
            int8_t b[16];
          } w;
          w.v = reinterpret_cast<const uint4*>(in)[x];
#pragma unroll
          for (int k = 0; k < 16; ++k) {
            put(16 * x + k, w.b[k]);
          }
        }
      } else {
        for (uint32_t x = threadIdx.x; x < E; x += DEMATCH_THREADS) {
          put(x, in[x]);
        }
      }
      __syncthreads();
    }
    // received LLR of deinterleaver index t = j Kq + i
    auto llr_in = [&](uint32_t t, uint32_t i, uint32_t j) -> int { return staged ? s_in[t] : in[i * g.Qm + j]; };

    // First loop pass of the reference (copy mode), see the file header.
    const bool     first_pass = new_data && E > 0;
    const uint32_t L1         = g.L - g.rank0;
    const uint32_t ncopy      = first_pass ? min(E, L1) : 0u;
    const bool     k0_in_info = g.k0 < g.nof_info;
    const uint32_t zero_end   = first_pass ? (k0_in_info ? g.k0 : g.nof_info) : 0u;
    uint32_t       zero_from  = g.N; // final tail zeroing
    if (new_data) {
      uint32_t tmp;
      if (E == 0) {
        tmp = g.k0;
      } else if (g.rank0 < g.nof_info) {
        const uint32_t n1 = min(g.nof_info - g.rank0, E);
        tmp               = (g.nof_sys + (E - n1)) % g.Ncb;
      } else {
        tmp = (g.rank0 + g.F + E) % g.Ncb;
      }
      if (E <= L1 && tmp != 0) {
        zero_from = g.N - (g.Ncb - tmp);
      }
    }

    // With new data, k0 = 0 and no limited-buffer rate matching, the first pass covers [0, E + F) (the
    // walk skips to nof_sys when the input ends in the information part) and the tail zeroing starts
    // where it stopped: once E >= nof_info nothing of the old contents survives.
    const bool read_old = !fresh && !(new_data && E >= g.nof_info && g.k0 == 0 && g.Ncb == g.N);
    const bool vec      = (reinterpret_cast<uintptr_t>(buf) & 3u) == 0 && (g.N & 15u) == 0;
    const bool vec16    = (reinterpret_cast<uintptr_t>(buf) & 15u) == 0; // PUSCH soft rows are 64-byte aligned
    auto       store16  = [&](uint32_t* o, uint4 v) {
      if (vec16) {
        *reinterpret_cast<uint4*>(o) = v;
      } else {
        o[0] = v.x;
        o[1] = v.y;
        o[2] = v.z;
        o[3] = v.w;
      }
    };
    const uint32_t step = gridDim.x * DEMATCH_THREADS * DEMATCH_PER_THREAD;
    if (staged && vec && first_pass && E <= L1) {
      // Single first pass (no combining), branch-free: every position selects between its old value,
      // zero, +inf (filler) and its input, whose LDS read is always issued at a clamped index.
      for (uint32_t p0 = (blockIdx.x * DEMATCH_THREADS + threadIdx.x) * DEMATCH_PER_THREAD; p0 < write_end; p0 += step) {
        union {
          uint4  v;
          int8_t b[16];
        } old, out;
        // deinterleaver index of the run's first position; along the run t advances by one (i + 1,
        // wrapping to the next j at Kq) unless the run crosses the filler block or the k0 wrap, where
        // each position divides on its own
        auto t_of = [&](uint32_t p) {
          const uint32_t w = p < g.nof_info ? p : p - g.F;
          return w >= g.rank0 ? w - g.rank0 : w + L1;
        };
        const uint32_t t0     = t_of(p0);
        const bool     linear = Kq >= DEMATCH_PER_THREAD && t_of(p0 + DEMATCH_PER_THREAD - 1) == t0 + DEMATCH_PER_THREAD - 1 &&
                            (p0 + DEMATCH_PER_THREAD <= g.nof_info || p0 >= g.nof_sys);
        uint32_t i0;
        const uint32_t j0 = divK.div(min(t0, E - 1), i0);
        uint32_t*      o4 = reinterpret_cast<uint32_t*>(buf + p0);
        constexpr uint32_t R = DEMATCH_PER_THREAD;
        if (p0 >= zero_from) {
          // the whole run lies in the tail zeroing (most of a high-rate codeblock)
          store16(o4, make_uint4(0, 0, 0, 0));
          continue;
        }
        if (linear && t0 + R <= E && p0 >= zero_end && p0 + R <= zero_from && p0 + R <= g.Ncb) {
          // pure copy run: 16 consecutive deinterleaved LLRs
          if ((t0 & 3u) == 0) {
            const uint32_t* w4 = reinterpret_cast<const uint32_t*>(s_in + t0);
            out.v              = make_uint4(w4[0], w4[1], w4[2], w4[3]);
          } else {
#pragma unroll
            for (uint32_t k = 0; k < R; ++k) {
              out.b[k] = s_in[t0 + k];
            }
          }
          store16(o4, out.v);
          continue;
        }
        old.v = read_old ? make_uint4(o4[0], o4[1], o4[2], o4[3]) : make_uint4(0, 0, 0, 0);
#pragma unroll
        for (int k = 0; k < DEMATCH_PER_THREAD; ++k) {
          const uint32_t p      = p0 + k;
          const bool     filler = p >= g.nof_info && p < g.nof_sys;
          const uint32_t t      = t_of(p);
          uint32_t       i, j;
          if (linear) {
            i = i0 + k;
            j = j0;
            if (i >= Kq) {
              i -= Kq;
              ++j;
            }
            i = t < E ? i : 0u; // past the input: any in-range index (the value is not used)
            j = t < E ? j : 0u;
          } else {
            j = divK.div(min(t, E - 1), i);
          }
          const int x = s_in[min(t, E - 1)];
          int            v = p < zero_end ? 0 : old.b[k];
          v                = filler ? LLR_INFINITY : v;
          v                = (!filler && p < g.Ncb && t < E) ? x : v;
          v                = p >= zero_from ? 0 : v;
          out.b[k]         = static_cast<int8_t>(v);
        }
        store16(o4, out.v);
      }
      continue;
    }
    for (uint32_t p0 = (blockIdx.x * DEMATCH_THREADS + threadIdx.x) * DEMATCH_PER_THREAD; p0 < write_end; p0 += step) {
      union {
        uint4  v;
        int8_t b[16];
      } old, out;
      if (read_old && vec) {
        const uint32_t* o4 = reinterpret_cast<const uint32_t*>(buf + p0);
        old.v              = make_uint4(o4[0], o4[1], o4[2], o4[3]);
      }
      // deinterleaver index (i, j) of the previous input, advanced incrementally along the run
      uint32_t t_prev = 0xfffffffeu, i = 0, j = 0; // t_prev + 1 matches no t
#pragma unroll
      for (int k = 0; k < DEMATCH_PER_THREAD; ++k) {
        const uint32_t p = p0 + k;
        if (!vec && p >= g.N) {
          continue; // vec: N is a multiple of 16, every run is whole
        }
        int v = read_old ? (vec ? old.b[k] : buf[p]) : 0;
        if (p < zero_end) {
          v = 0;
        }
        const bool filler = p >= g.nof_info && p < g.nof_sys;
        if (first_pass && filler) {
          v = LLR_INFINITY;
        }
        if (!filler && p < g.Ncb) {
          const uint32_t w = p < g.nof_info ? p : p - g.F;
          uint32_t       t = w >= g.rank0 ? w - g.rank0 : w + L1;
          if (t < ncopy) {
            if (t == t_prev + 1) {
              if (++i == Kq) {
                i = 0;
                ++j;
              }
            } else {
              j = divK.div(t, i);
            }
            t_prev = t;
            v      = llr_in(t, i, j);
            t += g.L;
          }
          for (; t < E; t += g.L) {
            uint32_t ii, jj;
            jj = divK.div(t, ii);
            v  = llr_sum(llr_in(t, ii, jj), v);
          }
        }
        if (p >= zero_from) {
          v = 0;
        }
        if (vec) {
          out.b[k] = static_cast<int8_t>(v);
        } else {
          buf[p] = static_cast<int8_t>(v);
        }
      }
      if (vec) {
        uint32_t* o4 = reinterpret_cast<uint32_t*>(buf + p0);
        o4[0]        = out.v.x;
        o4[1]        = out.v.y;
        o4[2]        = out.v.z;
        o4[3]        = out.v.w;
      }
    }
  }
}


constexpr int      RATE_MATCH_THREADS = 256;
constexpr uint32_t RM_MAX_CW_BYTES    = 66 * 384 / 8; // circular buffer of BG1, Z = 384

// Output byte b of the concatenated codeword, bits of segment cb and (when it straddles) the following
// segments.
__device__ uint32_t rm_byte(const rate_match_args& a, const rm_geometry& g, const fast_div& divL, uint32_t cb,
                            uint32_t b)
{
  uint32_t c = cb, off_c = a.out_offsets[cb], E_c = a.rm_lengths[cb];
  uint32_t byte = 0;
  for (int k = 0; k < 8; ++k) {
    const uint32_t gbit = 8 * b + k;
    bool           have = true;
    while (gbit >= off_c + E_c) {
      if (++c >= a.nof_cbs) {
        have = false;
        break;
      }
      off_c = a.out_offsets[c];
      E_c   = a.rm_lengths[c];
    }
    if (!have) {
      break;
    }
    if (gbit < off_c) {
      continue; // gap between segments
    }
    const uint32_t o = gbit - off_c;
    uint32_t       i, j;
    if (g.Qm == 6) {
      i = __umulhi(o >> 1, 0xAAAAAAABu) >> 1;
      j = o - 6 * i;
    } else {
      const uint32_t sh = g.Qm == 8 ? 3 : g.Qm == 4 ? 2 : g.Qm == 2 ? 1 : 0;
      i                 = o >> sh;
      j                 = o & (g.Qm - 1);
    }
    const uint32_t t = j * (E_c / g.Qm) + i;
    uint32_t       w;
    divL.div(g.rank0 + t, w);
    const uint32_t p   = w < g.nof_info ? w : w + g.F;
    const uint8_t* src = a.cw + static_cast<size_t>(c) * a.cw_stride;
    byte |= ((src[p >> 3] >> (7 - (p & 7))) & 1u) << (7 - k);
  }
  return byte;
}

// One workgroup per codeblock: the circular buffer (Ncb bits of the packed codeword) is staged in LDS
// with coalesced loads.  When the segment starts on a byte boundary, one thread per group of 8 modulation
// symbols (Qm output bytes): for each interleaver row j < Qm the 8 bits of the group are 8 consecutive walk
// positions (one two-byte LDS read), and an 8 x 8 bit transpose turns rows into symbols.  The remaining
// bytes (partial last group, unaligned segments, Qm = 1): one thread per output byte gathering its 8 bits
// (bit selection + interleaver as index arithmetic); a byte straddling the next segment is built from global
// memory.
template <bool RAGGED>
__global__ __launch_bounds__(RATE_MATCH_THREADS) void ldpc_rate_match_kernel(rate_match_args a)
{
  __shared__ uint8_t s_cw[RM_MAX_CW_BYTES + 4]; // + the second byte of a two-byte read at the end
  for (uint32_t cb = blockIdx.y; cb < a.nof_cbs; cb += gridDim.y) {
    const rm_geometry g = RAGGED ? a.geos[a.row_geo[cb]] : a.g;
    const fast_div    divL(g.L);
    const uint32_t    cw_bytes = (g.Ncb + 7) / 8;
    const uint32_t off   = a.out_offsets[cb];
    const uint32_t E     = a.rm_lengths[cb];
    const uint32_t first = (off + 7) / 8;
    const uint32_t last  = (off + E + 7) / 8;
    const uint32_t whole = (off + E) / 8; // bytes [first, whole) hold only bits of this segment
    const uint32_t Kq    = E / g.Qm;
    const uint8_t* src   = a.cw + static_cast<size_t>(cb) * a.cw_stride;
    __syncthreads(); // s_cw of the previous codeblock is no longer read
    const uint32_t nw4 = (reinterpret_cast<uintptr_t>(src) & 3u) == 0 ? cw_bytes / 4 : 0;
    for (uint32_t x0 = threadIdx.x; x0 < nw4; x0 += 4 * RATE_MATCH_THREADS) {
      uint32_t v[4]; // every load of the round in flight before the LDS stores
#pragma unroll
      for (uint32_t r = 0; r < 4; ++r) {
        const uint32_t x = x0 + r * RATE_MATCH_THREADS;
        v[r]             = x < nw4 ? reinterpret_cast<const uint32_t*>(src)[x] : 0u;
      }
#pragma unroll
      for (uint32_t r = 0; r < 4; ++r) {
        const uint32_t x = x0 + r * RATE_MATCH_THREADS;
        if (x < nw4) {
          reinterpret_cast<uint32_t*>(s_cw)[x] = v[r];
        }
      }
    }
    for (uint32_t x = 4 * nw4 + threadIdx.x; x < cw_bytes; x += RATE_MATCH_THREADS) {
      s_cw[x] = src[x];
    }
    __syncthreads();
    // groups of 8 symbols (Qm bytes each) of a byte-aligned segment
    const uint32_t G        = ((off & 7u) == 0 && g.Qm >= 2) ? Kq / 8 : 0;
    const uint32_t fast_end = first + G * g.Qm;
    for (uint32_t gi = blockIdx.x * RATE_MATCH_THREADS + threadIdx.x; gi < G; gi += gridDim.x * RATE_MATCH_THREADS) {
      uint64_t x = 0;
#pragma unroll
      for (uint32_t j = 0; j < 8; ++j) {
        if (j < g.Qm) {
          uint32_t w = g.rank0 + j * Kq + 8 * gi;
          if (w >= g.L) {
            w -= g.L;
            if (w >= g.L) {
              divL.div(w, w); // repetition beyond one more turn
            }
          }
          x |= static_cast<uint64_t>(rm_walk_byte(s_cw, g, w)) << (56 - 8 * j);
        }
      }
      x = transpose8x8(x); // byte s: bits j = 0 .. Qm - 1 of symbol 8 gi + s, MSB first
      uint64_t acc = 0;
#pragma unroll
      for (uint32_t q = 0; q < 8; ++q) {
        acc = (acc << g.Qm) | ((x >> (64 - 8 * q - g.Qm)) & ((1u << g.Qm) - 1u));
      }
      uint8_t* o = a.out + fast_end - (G - gi) * g.Qm;
      for (uint32_t q = 0; q < g.Qm; ++q) {
        o[q] = static_cast<uint8_t>(acc >> (8 * (g.Qm - 1 - q)));
      }
    }
    for (uint32_t b = fast_end + blockIdx.x * RATE_MATCH_THREADS + threadIdx.x; b < last;
         b += gridDim.x * RATE_MATCH_THREADS) {
      if (b >= whole) {
        a.out[b] = static_cast<uint8_t>(rm_byte(a, g, divL, cb, b));
        continue;
      }
      uint32_t byte = 0;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const uint32_t o = 8 * b + k - off;
        uint32_t       i, j;
        if (g.Qm == 6) {
          i = __umulhi(o >> 1, 0xAAAAAAABu) >> 1;
          j = o - 6 * i;
        } else {
          const uint32_t sh = g.Qm == 8 ? 3 : g.Qm == 4 ? 2 : g.Qm == 2 ? 1 : 0;
          i                 = o >> sh;
          j                 = o & (g.Qm - 1);
        }
        uint32_t w = g.rank0 + j * Kq + i;
        if (w >= g.L) {
          w -= g.L;
          if (w >= g.L) {
            divL.div(w, w); // repetition beyond one more turn
          }
        }
        const uint32_t p = w < g.nof_info ? w : w + g.F;
        byte |= ((s_cw[p >> 3] >> (7 - (p & 7))) & 1u) << (7 - k);
      }
      a.out[b] = static_cast<uint8_t>(byte);
    }
  }
}

hipError_t launch_rate_dematch(const dematch_args& a, hipStream_t stream)
{
  // one workgroup per codeblock: splitting a codeblock over several (each staging its input) measured
  // twice as slow
  dim3 grid(1, a.nof_cbs < 65535u ? a.nof_cbs : 65535u);
  if (a.row_geo != nullptr) {
    hipLaunchKernelGGL(ldpc_rate_dematch_kernel<true>, grid, dim3(DEMATCH_THREADS), 0, stream, a);
  } else {
    hipLaunchKernelGGL(ldpc_rate_dematch_kernel<false>, grid, dim3(DEMATCH_THREADS), 0, stream, a);
  }
  return hipGetLastError();
}

hipError_t launch_rate_match(const rate_match_args& a, uint32_t max_rm_length, hipStream_t stream)
{
  // one workgroup per codeblock: the staged circular buffer is loaded once
  (void)max_rm_length;
  dim3 grid(1, a.nof_cbs < 65535u ? a.nof_cbs : 65535u);
  if (a.row_geo != nullptr) {
    hipLaunchKernelGGL(ldpc_rate_match_kernel<true>, grid, dim3(RATE_MATCH_THREADS), 0, stream, a);
  } else {
    hipLaunchKernelGGL(ldpc_rate_match_kernel<false>, grid, dim3(RATE_MATCH_THREADS), 0, stream, a);
  }
  return hipGetLastError();
}

} // namespace srs_amd
