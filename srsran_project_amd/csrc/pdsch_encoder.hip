// pdsch_encoder.hip -- the PDSCH encoder chain of pdsch_encoder_impl::encode
// (lib/phy/upper/channel_processors/pdsch/pdsch_encoder_impl.cpp:28-80) in two launches:
//
//   pdsch_tb_crc_kernel  the TB CRC (CRC16 / CRC24A, crc_calculator_generic_impl.cpp) of every transport block
//                        as partials of PE_TB_CHUNK bytes, each moved to the TB end (crc_device.h), so no
//                        accumulator has to be zeroed and no atomics are needed; the workgroups of chunk 0 also
//                        zero the codeword bytes that two rate-matched segments share.
//   pdsch_cb_kernel      one workgroup per codeblock, everything in LDS:
//                          segmentation (ldpc_segmenter_tx_impl.cpp:137-207): the message bytes straight from
//                            the TB, the TB CRC (XOR of the partials) on the last segment, zero padding;
//                          the CRC24B of segmented TBs (ldpc_segmenter_tx_impl.cpp:196), byte table in LDS;
//                          LDPC encoding (ldpc_encoder_impl.cpp:44-80) by the bit-sliced core
//                            (ldpc_encode_device.h), only the circular-buffer window the rate matcher reads;
//                          rate matching + bit interleaving (ldpc_rate_matcher_impl.cpp:95-160) into the
//                            codeword: whole bytes stored, the bytes shared with the neighbouring segments ORed
//                            in (zeroed by launch 1).
// Replaces the five launches of pdsch_api.cpp (TB CRC, finalize, segmentation + CB CRC, encoder, rate
// matcher) and the message / codeblock round trips through HBM.
#include <hip/hip_runtime.h>

#include "crc_device.h"
#include "ldpc_codec_args.h"
#include "ldpc_common.h"
#include "ldpc_encode_device.h"
#include "rate_match_device.h"
#include "sch_args.h"

namespace srs_amd {
namespace {

constexpr int      PE_THREADS      = 256;
constexpr uint32_t PE_TB_PER       = PE_TB_CHUNK / PE_THREADS; // TB bytes per thread of the CRC kernel
constexpr uint32_t PE_CW_BYTES     = 66 * MAX_LIFTING_SIZE / 8; // circular buffer of BG1, Z = 384
constexpr uint32_t PE_ENC_WORDS    = enc_bits_lds_words(22, 46, MAX_LIFTING_SIZE);

// TB CRC partials: workgroup (chunk, t) divides TB bytes [chunk * PE_TB_CHUNK, +PE_TB_CHUNK) and stores its
// remainder moved to the TB end; chunk 0 zeroes the codeword bytes shared by consecutive segments of t.
__global__ __launch_bounds__(PE_THREADS) void pdsch_tb_crc_kernel(pdsch_fused_args a)
{
  __shared__ uint32_t partial[PE_THREADS / 64];
  __shared__ uint32_t T[256];
  __shared__ __attribute__((aligned(16))) uint8_t s_chunk[PE_TB_CHUNK];
  uint32_t table_order = 0, table_poly = 0;
  for (uint32_t t = blockIdx.y; t < a.nof_tbs; t += gridDim.y) {
    const tb_desc  d      = a.tds[t];
    const uint32_t nbytes = d.tbs_bits / 8;
    const uint32_t c0     = blockIdx.x * PE_TB_CHUNK;
    if (c0 >= nbytes) {
      continue; // uniform over the workgroup
    }
    if (blockIdx.x == 0) {
      // bytes holding bits of two segments (or the codeword's zero-padded last byte): ORed by pdsch_cb_kernel
      for (uint32_t r = threadIdx.x; r < d.nof_segments; r += PE_THREADS) {
        const uint32_t row = d.row0 + r;
        const uint32_t o0 = a.row_out[row], o1 = o0 + a.row_E[row];
        if ((o0 & 7u) != 0) {
          a.cw[o0 >> 3] = 0;
        }
        if ((o1 & 7u) != 0) {
          a.cw[o1 >> 3] = 0;
        }
      }
    }
    const bool      c16   = d.tb_crc_bits == 16;
    const uint32_t  poly  = c16 ? a.crc16_poly : a.crc24a_poly;
    const uint32_t* table = c16 ? a.crc16_table : a.crc24a_table;
    __syncthreads(); // T and s_chunk of the previous TB are no longer read
    if (table_order != d.tb_crc_bits || table_poly != poly) {
      crc_table8_init<PE_THREADS>(T, d.tb_crc_bits, poly);
      table_order = d.tb_crc_bits;
      table_poly  = poly;
    }
    crc_stage_bytes<PE_THREADS>(s_chunk, a.tbs + d.tb_offset, c0, min(PE_TB_CHUNK, nbytes - c0)); // coalesced
    __syncthreads();
    const uint32_t b0 = c0 + threadIdx.x * PE_TB_PER;
    const uint32_t b1 = min(nbytes, b0 + PE_TB_PER);
    const uint32_t to = min(d.tbs_bits, (c0 + PE_TB_CHUNK) * 8); // moved to the TB end once per workgroup
    const uint32_t x  = crc_block_xor<PE_THREADS>(
        crc_chunk_contrib(lds_chunk_fetch{s_chunk, c0}, b0, b1, d.tbs_bits, d.tb_crc_bits, poly, table, T, to),
        partial);
    if (threadIdx.x == 0) {
      a.tb_parts[static_cast<size_t>(t) * a.part_stride + blockIdx.x] =
          crc_move(x, d.tbs_bits - to, d.tb_crc_bits, table);
    }
  }
}

// Output byte b of the segment (bits [off, off + E) of the codeword): the bits of this segment, zeros elsewhere.
__device__ __forceinline__ uint32_t pe_out_byte(const uint8_t* s_cw, const rm_geometry& g, const fast_div& divL,
                                                uint32_t off, uint32_t E, uint32_t Kq, uint32_t b)
{
  uint32_t byte = 0;
#pragma unroll
  for (uint32_t k = 0; k < 8; ++k) {
    const uint32_t gbit = 8 * b + k;
    if (gbit < off || gbit >= off + E) {
      continue;
    }
    const uint32_t o = gbit - off;
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
  return byte;
}

__global__ __launch_bounds__(PE_THREADS) void pdsch_cb_kernel(pdsch_fused_args a)
{
  __shared__ uint32_t T[256]; // CRC24B byte table
  __shared__ uint32_t partial[PE_THREADS / 64];
  __shared__ uint32_t lw[PE_ENC_WORDS];
  // the message (MSB-first bytes), then the encoded circular-buffer window (+ the second byte of a two-byte read)
  __shared__ __attribute__((aligned(16))) uint8_t s_cw[PE_CW_BYTES + 8];
  crc_table8_init<PE_THREADS>(T, 24, a.crc24b_poly);
  const uint32_t j = threadIdx.x;

  for (uint32_t cb = blockIdx.x; cb < a.nof_cbs; cb += gridDim.x) {
    const uint32_t     t   = a.row_tb[cb];
    const tb_desc      d   = a.tds[t];
    const rm_geometry  g   = a.geos[a.row_geo[cb]];
    const enc_row_desc er  = a.enc_rows[cb];
    const uint32_t     E   = a.row_E[cb];
    const uint32_t     off = a.row_out[cb];
    const uint32_t     Z   = er.Z;
    const uint32_t     Kb  = g.nof_sys / Z + 2;
    const int          bg  = Kb == 22 ? 1 : 2;
    const uint32_t     r   = cb - d.row0;
    const uint32_t     C   = d.nof_segments;
    const bool         last   = r == C - 1;
    const uint32_t     cbi    = d.cb_info_bits;
    const uint32_t     n_data = last ? cbi - d.tb_crc_bits - d.zero_pad : cbi;
    const uint32_t     kz     = Kb * Z;
    const uint32_t     nmb    = (kz + 7) / 8; // message bytes incl. fillers

    // ---- 1. message bytes (MSB first) into s_cw: TB data, TB CRC on the last segment, zeros up to K Z
    uint32_t tb_crc = 0;
    if (last) {
      const uint32_t np = (d.tbs_bits / 8 + PE_TB_CHUNK - 1) / PE_TB_CHUNK;
      for (uint32_t i = 0; i < np; ++i) {
        tb_crc ^= a.tb_parts[static_cast<size_t>(t) * a.part_stride + i];
      }
    }
    // (a plan may count the TB CRC outside cb_info_bits, pdsch_encoder_hw_impl's single segment: bits up to the CRC)
    const uint32_t seg_end = last ? n_data + d.tb_crc_bits : n_data;
    const uint8_t* tb      = a.tbs + d.tb_offset;
    const uint32_t ob = r * cbi; // first TB bit of the segment
    __syncthreads(); // s_cw / lw of the previous codeblock are no longer read
    for (uint32_t q = j; q < (nmb + 3) / 4; q += PE_THREADS) {
      uint32_t w = 0;
#pragma unroll
      for (uint32_t b = 0; b < 4; ++b) {
        const uint32_t jb = 4 * q + b;
        uint32_t       v  = 0;
        if (8 * jb + 8 <= n_data) {
          // 8 TB bits: one or two byte loads
          const uint32_t p  = ob + 8 * jb;
          const uint32_t sh = p & 7u;
          uint32_t       x  = static_cast<uint32_t>(tb[p >> 3]) << 8;
          if (sh != 0) {
            x |= tb[(p >> 3) + 1];
          }
          v = (x >> (8 - sh)) & 0xffu;
        } else if (8 * jb < seg_end) {
#pragma unroll
          for (uint32_t k = 0; k < 8; ++k) {
            const uint32_t p = 8 * jb + k;
            uint32_t       x = 0;
            if (p < n_data) {
              x = (tb[(ob + p) >> 3] >> (7 - ((ob + p) & 7))) & 1u;
            } else if (last && p < n_data + d.tb_crc_bits) {
              x = (tb_crc >> (d.tb_crc_bits - 1 - (p - n_data))) & 1u;
            }
            v |= x << (7 - k);
          }
        }
        w |= v << (8 * b);
      }
      reinterpret_cast<uint32_t*>(s_cw)[q] = w;
    }
    __syncthreads();
    // ---- 2. CRC24B of segmented TBs over the cbi message bits, attached MSB-first after them
    if (C > 1) {
      const uint32_t nb  = (cbi + 7) / 8;
      const uint32_t per = (nb + PE_THREADS - 1) / PE_THREADS;
      const uint32_t b0  = j * per;
      const uint32_t crc = crc_block_xor<PE_THREADS>(
          crc_chunk_contrib(lds_chunk_fetch{s_cw, 0}, b0, min(nb, b0 + per), cbi, 24, a.crc24b_poly, a.crc24b_table, T),
          partial);
      if (j == 0) {
        attach_crc_bits(s_cw, cbi, 24, crc);
      }
      __syncthreads();
    }
    // ---- 3. message words of the bit-linear codeword (bit i at word i / 32, bit i % 32), the rest zeroed
    const uint32_t nq  = (Z + 31) / 32;
    const uint32_t ncw = enc_bits_cw_words(Kb, er.M_eff, Z);
    uint32_t*      cwb = lw;
    uint32_t*      lam = lw + ncw;
    uint32_t*      ls  = lam + 4 * nq;
    const uint32_t nmw = (kz + 31) / 32;
    for (uint32_t w = j; w < ncw; w += PE_THREADS) {
      uint32_t v = 0;
      if (w < nmw) {
        v = __builtin_bitreverse32(__builtin_bswap32(reinterpret_cast<const uint32_t*>(s_cw)[w]));
        if (32 * w + 32 > kz) {
          v &= (1u << (kz - 32 * w)) - 1u;
        }
      }
      cwb[w] = v;
    }
    for (uint32_t w = j; w < nq + 2; w += PE_THREADS) {
      ls[w] = 0;
    }
    __syncthreads();
    // ---- 4. parity of the encoded window
    const int32_t core_a[3] = {static_cast<int32_t>(er.core_a[0]), static_cast<int32_t>(er.core_a[1]),
                               static_cast<int32_t>(er.core_a[2])};
    encode_bits_parity<PE_THREADS>(cwb, lam, ls, a.edges + er.edge_off, a.row_start[bg - 1], bg, Kb, Z, er.M_eff,
                                   static_cast<int32_t>(er.p0_shift), core_a, j);
    // ---- 5. the shortened codeword window (from bit 2Z) as MSB-first bytes into s_cw
    const uint32_t nbits = er.pack_bits;
    for (uint32_t m = j; m < (nbits + 31) / 32; m += PE_THREADS) {
      uint32_t v = lds_bits32(cwb, 2 * Z + 32 * m);
      if (32 * m + 32 > nbits) {
        v &= (1u << (nbits - 32 * m)) - 1u;
      }
      reinterpret_cast<uint32_t*>(s_cw)[m] = __builtin_bswap32(__builtin_bitreverse32(v));
    }
    __syncthreads();
    // ---- 6. rate matching + bit interleaving into codeword bits [off, off + E)
    const fast_div divL(g.L);
    const uint32_t Kq    = E / g.Qm;
    const uint32_t first = (off + 7) / 8;
    const uint32_t whole = (off + E) / 8; // bytes [first, whole) hold only bits of this segment
    // groups of 8 symbols (Qm bytes each) of a byte-aligned segment
    const uint32_t G        = ((off & 7u) == 0 && g.Qm >= 2) ? Kq / 8 : 0;
    const uint32_t fast_end = first + G * g.Qm;
    for (uint32_t gi = j; gi < G; gi += PE_THREADS) {
      uint64_t x = 0;
#pragma unroll
      for (uint32_t jj = 0; jj < 8; ++jj) {
        if (jj < g.Qm) {
          uint32_t w = g.rank0 + jj * Kq + 8 * gi;
          if (w >= g.L) {
            w -= g.L;
            if (w >= g.L) {
              divL.div(w, w);
            }
          }
          x |= static_cast<uint64_t>(rm_walk_byte(s_cw, g, w)) << (56 - 8 * jj);
        }
      }
      x            = transpose8x8(x);
      uint64_t acc = 0;
#pragma unroll
      for (uint32_t q = 0; q < 8; ++q) {
        acc = (acc << g.Qm) | ((x >> (64 - 8 * q - g.Qm)) & ((1u << g.Qm) - 1u));
      }
      uint8_t* o = a.cw + first + gi * g.Qm;
      for (uint32_t q = 0; q < g.Qm; ++q) {
        o[q] = static_cast<uint8_t>(acc >> (8 * (g.Qm - 1 - q)));
      }
    }
    for (uint32_t b = fast_end + j; b < whole; b += PE_THREADS) {
      a.cw[b] = static_cast<uint8_t>(pe_out_byte(s_cw, g, divL, off, E, Kq, b));
    }
    // bytes shared with the previous / next segment (zeroed by pdsch_tb_crc_kernel): ORed in
    if (j < 2) {
      const uint32_t b = j == 0 ? off / 8 : whole;
      // (j = 1: the end byte, unless it is the start byte that j = 0 already covers)
      const bool partial_byte =
          j == 0 ? (off & 7u) != 0 : ((off + E) & 7u) != 0 && (whole != off / 8 || (off & 7u) == 0);
      if (partial_byte) {
        const uint32_t v = pe_out_byte(s_cw, g, divL, off, E, Kq, b);
        atomicOr(reinterpret_cast<uint32_t*>(a.cw + (b & ~3u)), v << (8 * (b & 3u)));
      }
    }
  }
}

} // namespace

hipError_t launch_pdsch_fused(const pdsch_fused_args& a, hipStream_t stream)
{
  if (a.nof_cbs == 0) {
    return hipSuccess;
  }
  hipLaunchKernelGGL(pdsch_tb_crc_kernel,
                     dim3((a.max_tb_bytes + PE_TB_CHUNK - 1) / PE_TB_CHUNK, a.nof_tbs < 65535u ? a.nof_tbs : 65535u),
                     dim3(PE_THREADS), 0, stream, a);
  hipLaunchKernelGGL(pdsch_cb_kernel, dim3(a.nof_cbs < 65535u ? a.nof_cbs : 65535u), dim3(PE_THREADS), 0, stream, a);
  return hipGetLastError();
}

} // namespace srs_amd
