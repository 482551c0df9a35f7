// pdsch_encoder.hip -- the PDSCH encoder chain of pdsch_encoder_impl::encode
// (lib/phy/upper/channel_processors/pdsch/pdsch_encoder_impl.cpp:28-80):
//   pdsch_tb_crc_kernel  the TB CRC (CRC16 / CRC24A, crc_calculator_generic_impl.cpp) as partials of PE_TB_CHUNK
//                        bytes: byte-table remainders per thread combined in a tree, one move to the TB end per
//                        chunk (crc_device.h); no accumulator to reset, no atomics;
//   pdsch_cb_kernel      one wave per codeblock, everything in LDS:
//                          segmentation (ldpc_segmenter_tx_impl.cpp:137-207): the message straight from the TB, the
//                            TB CRC (XOR of the partials) on the last segment;
//                          the CRC24B of segmented TBs (ldpc_segmenter_tx_impl.cpp:196), byte table in LDS;
//                          LDPC encoding (ldpc_encoder_impl.cpp:44-80) by the bit-sliced core (ldpc_encode_device.h)
//                            with the lifted graph staged in LDS, only the circular-buffer window the rate matcher
//                            reads;
//                          rate matching + bit interleaving (ldpc_rate_matcher_impl.cpp:95-160) into the codeword:
//                            whole bytes stored, the bytes shared with the neighbouring segments written with AND / OR
//                            atomics on the segment's own bits (the codeword's padding bits cleared by the TB's last
//                            segment), so no zeroing pass is needed.
// The TB CRC kernel runs concurrently with the codeblock kernel over every codeblock but the TBs' last ones, which a
// second codeblock launch encodes once the partials are in (pdsch_api.cpp).  (Gathering the TB CRC inside one launch
// through a last-arriving workgroup needs an agent-scope fence per codeblock, which on the multi-XCD MI355X writes
// back / invalidates L2 and measured twice as slow.)
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "crc_device.h"
#include "ldpc_codec_args.h"
#include "ldpc_common.h"
#include "ldpc_encode_device.h"
#include "rate_match_device.h"
#include "sch_args.h"

namespace srs_amd {
namespace {

constexpr uint32_t PE_CW_BYTES  = 66 * MAX_LIFTING_SIZE / 8; // circular buffer of BG1, Z = 384
constexpr uint32_t PE_ENC_WORDS = enc_bits_lds_words(22, 46, MAX_LIFTING_SIZE);

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

struct pe_lds {
  uint32_t T24b[256]; // CRC24B byte table
  uint32_t Ttb[256];  // byte table of the TB CRC polynomial in use (tb_order / tb_poly)
  uint32_t lw[PE_ENC_WORDS];
  uint32_t edges[MAX_EDGES]; // the codeblock's lifted graph (the rows the encoder computes)
  // the message (MSB-first bytes), then the encoded circular-buffer window (+ the second byte of a two-byte read)
  __attribute__((aligned(16))) uint8_t s_cw[PE_CW_BYTES + 8];
  uint32_t partial[4]; // block reductions (NT > 64)
  uint32_t bcast[2];   // arrival count, TB CRC (NT > 64)
};

// XOR of v over the NT threads of the block (to every thread).
template <int NT>
__device__ __forceinline__ uint32_t pe_xor(uint32_t v, uint32_t* partial)
{
  if constexpr (NT == 64) {
    return crc_wave_xor(v);
  } else {
    return crc_block_xor<NT>(v, partial);
  }
}

// The segment of codeblock row `cb` (its TB's data bits only: zero from the data end) into s_cw as MSB-first bytes,
// K Z bits in all.
template <int NT>
__device__ __forceinline__ void pe_message(const pdsch_fused_args& a, const tb_desc& d, uint32_t r, uint32_t n_data,
                                           uint32_t kz, uint8_t* s_cw, uint32_t j)
{
  const uint8_t* tb  = a.tbs + d.tb_offset;
  const uint32_t ob  = r * d.cb_info_bits; // first TB bit of the segment
  const uint32_t nmb = (kz + 7) / 8;
  if ((ob & 7u) == 0) {
    // byte-aligned segment: message word q = TB bytes B .. B + 3 (B = ob / 8 + 4q), one funnel shift of the two
    // aligned dwords that hold them; the partial / last words below
    const uintptr_t base  = reinterpret_cast<uintptr_t>(tb) + ob / 8;
    const uint32_t  nfull = n_data / 32;
    for (uint32_t q = j; q < nfull; q += NT) {
      const uintptr_t  addr = base + 4 * q;
      const uint32_t*  p4   = reinterpret_cast<const uint32_t*>(addr & ~uintptr_t(3));
      const uint32_t   sh   = static_cast<uint32_t>(addr & 3u);
      const uint32_t   lo   = p4[0];
      const uint32_t   hi   = sh != 0 ? p4[1] : 0u;
      reinterpret_cast<uint32_t*>(s_cw)[q] = sh != 0 ? __builtin_amdgcn_alignbyte(hi, lo, sh) : lo;
    }
    for (uint32_t q = nfull + j; q < (nmb + 3) / 4; q += NT) {
      uint32_t w = 0;
      for (uint32_t b = 0; b < 4; ++b) {
        const uint32_t jb = 4 * q + b;
        uint32_t       v  = 0;
        for (uint32_t k = 0; k < 8 && 8 * jb + k < n_data; ++k) {
          const uint32_t p = ob + 8 * jb + k;
          v |= ((tb[p >> 3] >> (7 - (p & 7))) & 1u) << (7 - k);
        }
        w |= v << (8 * b);
      }
      reinterpret_cast<uint32_t*>(s_cw)[q] = w;
    }
    return;
  }
  for (uint32_t q = j; q < (nmb + 3) / 4; q += NT) {
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
      } else if (8 * jb < n_data) {
        for (uint32_t k = 0; k < 8 && 8 * jb + k < n_data; ++k) {
          const uint32_t p = ob + 8 * jb + k;
          v |= ((tb[p >> 3] >> (7 - (p & 7))) & 1u) << (7 - k);
        }
      }
      w |= v << (8 * b);
    }
    reinterpret_cast<uint32_t*>(s_cw)[q] = w;
  }
}

// CRC24B (C > 1), LDPC encoding and rate matching of codeblock row `cb` whose message is in s_cw.

template <int NT>
__device__ __forceinline__ void pe_finish(const pdsch_fused_args& a, pe_lds& s, uint32_t cb, const tb_desc& d,
                                          uint32_t j)
{
  const rm_geometry  g   = a.geos[a.row_geo[cb]];
  const enc_row_desc er  = a.enc_rows[cb];
  const uint32_t     E   = a.row_E[cb];
  const uint32_t     off = a.row_out[cb];
  const uint32_t     Z   = er.Z;
  const uint32_t     Kb  = g.nof_sys / Z + 2;
  const int          bg  = Kb == 22 ? 1 : 2;
  const uint32_t     kz  = Kb * Z;
  uint8_t*           s_cw = s.s_cw;
  // ---- CRC24B of segmented TBs over the cbi message bits, attached MSB-first after them
  if (d.nof_segments > 1) {
    const uint32_t cbi = d.cb_info_bits;
    const uint32_t nb  = (cbi + 7) / 8;
    const uint32_t per = (nb + NT - 1) / NT;
    const uint32_t b0  = j * per;
    const uint32_t crc = pe_xor<NT>(
        crc_chunk_contrib(lds_chunk_fetch{s_cw, 0}, b0, min(nb, b0 + per), cbi, 24, a.crc24b_poly, a.crc24b_table,
                          s.T24b),
        s.partial);
    if (j == 0) {
      attach_crc_bits(s_cw, cbi, 24, crc);
    }
    __syncthreads();
  }
  // ---- message words of the bit-linear codeword (bit i at word i / 32, bit i % 32), the rest zeroed
  const uint32_t nq  = (Z + 31) / 32;
  const uint32_t ncw = enc_bits_cw_words(Kb, er.M_eff, Z);
  uint32_t*      cwb = s.lw;
  uint32_t*      lam = s.lw + ncw;
  uint32_t*      ls  = lam + 4 * nq;
  const uint32_t nmw = (kz + 31) / 32;
  for (uint32_t w = j; w < ncw; w += NT) {
    uint32_t v = 0;
    if (w < nmw) {
      v = __builtin_bitreverse32(__builtin_bswap32(reinterpret_cast<const uint32_t*>(s_cw)[w]));
      if (32 * w + 32 > kz) {
        v &= (1u << (kz - 32 * w)) - 1u;
      }
    }
    cwb[w] = v;
  }
  for (uint32_t w = j; w < nq + 2; w += NT) {
    ls[w] = 0;
  }
  const uint32_t* ge = a.edges + er.edge_off;
  const uint32_t  ne = static_cast<uint32_t>(a.row_start[bg - 1][er.M_eff]);
  for (uint32_t e = j; e < ne; e += NT) {
    s.edges[e] = ge[e];
  }
  __syncthreads();
  // ---- parity of the encoded window (edge descriptors from LDS: every edge read is then an LDS latency)
  const int32_t core_a[3] = {static_cast<int32_t>(er.core_a[0]), static_cast<int32_t>(er.core_a[1]),
                             static_cast<int32_t>(er.core_a[2])};
  encode_bits_parity<NT>(cwb, lam, ls, s.edges, a.row_start[bg - 1], bg, Kb, Z, er.M_eff,
                                 static_cast<int32_t>(er.p0_shift), core_a, j);
  // ---- the shortened codeword window (from bit 2Z) as MSB-first bytes into s_cw
  const uint32_t nbits = er.pack_bits;
  for (uint32_t m = j; m < (nbits + 31) / 32; m += NT) {
    uint32_t v = lds_bits32(cwb, 2 * Z + 32 * m);
    if (32 * m + 32 > nbits) {
      v &= (1u << (nbits - 32 * m)) - 1u;
    }
    reinterpret_cast<uint32_t*>(s_cw)[m] = __builtin_bswap32(__builtin_bitreverse32(v));
  }
  __syncthreads();
  // ---- rate matching + bit interleaving into codeword bits [off, off + E)
  const fast_div divL(g.L);
  const uint32_t Kq    = E / g.Qm;
  const uint32_t first = (off + 7) / 8;
  const uint32_t whole = (off + E) / 8; // bytes [first, whole) hold only bits of this segment
  // groups of 8 symbols (Qm bytes each) of a byte-aligned segment
  const uint32_t G        = ((off & 7u) == 0 && g.Qm >= 2) ? Kq / 8 : 0;
  const uint32_t fast_end = first + G * g.Qm;
  for (uint32_t gi = j; gi < G; gi += NT) {
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
  for (uint32_t b = fast_end + j; b < whole; b += NT) {
    a.cw[b] = static_cast<uint8_t>(pe_out_byte(s_cw, g, divL, off, E, Kq, b));
  }
  // bytes shared with the previous / next segment: clear this segment's bits (and, for the TB's last segment, the
  // codeword's padding bits after them), then set its ones -- the neighbour's bits are never touched
  if (j < 2) {
    const bool     last_seg = cb == d.row0 + d.nof_segments - 1;
    const uint32_t b        = j == 0 ? off / 8 : whole;
    // (j = 1: the end byte, unless it is the start byte that j = 0 already covers)
    const bool partial =
        j == 0 ? (off & 7u) != 0 : ((off + E) & 7u) != 0 && (whole != off / 8 || (off & 7u) == 0);
    if (partial) {
      uint32_t mask = 0;
      for (uint32_t k = 0; k < 8; ++k) {
        const uint32_t gbit = 8 * b + k;
        mask |= (gbit >= off && (gbit < off + E || last_seg)) ? (0x80u >> k) : 0u;
      }
      const uint32_t v  = pe_out_byte(s_cw, g, divL, off, E, Kq, b);
      uint32_t*      w4 = reinterpret_cast<uint32_t*>(a.cw + (b & ~3u));
      const uint32_t sh = 8 * (b & 3u);
      atomicAnd(w4, ~(mask << sh));
      atomicOr(w4, v << sh);
    }
  }
  __syncthreads(); // s_cw / lw are rewritten by the next codeblock
}

// TB CRC partials: workgroup (chunk, t) divides TB bytes [chunk * PE_TB_CHUNK, + PE_TB_CHUNK), PE_TB_PER contiguous
// bytes per thread by the byte table, combines the threads' remainders pairwise in a tree (left x^(bits of right) +
// right, the powers from the linear table's first entries, hot in L2) and stores the chunk's remainder moved to the
// TB end in tb_parts[t][chunk]: one move per chunk instead of one per thread, no accumulator, no atomics.
constexpr int      PE_CRC_THREADS = 256;
constexpr uint32_t PE_TB_PER      = PE_TB_CHUNK / PE_CRC_THREADS;

__global__ __launch_bounds__(PE_CRC_THREADS) void pdsch_tb_crc_kernel(pdsch_fused_args a)
{
  __shared__ uint32_t T[256];
  __shared__ uint32_t R[PE_CRC_THREADS];
  __shared__ __attribute__((aligned(16))) uint8_t s_chunk[PE_TB_CHUNK];
  uint32_t       table_order = 0, table_poly = 0;
  const uint32_t i           = threadIdx.x;
  for (uint32_t t = blockIdx.y; t < a.nof_tbs; t += gridDim.y) {
    const tb_desc  d      = a.tds[t];
    const uint32_t nbytes = d.tbs_bits / 8;
    const uint32_t c0     = blockIdx.x * PE_TB_CHUNK;
    if (c0 >= nbytes) {
      continue; // uniform over the workgroup
    }
    const uint32_t  L     = d.tb_crc_bits;
    const uint32_t  poly  = L == 16 ? a.crc16_poly : a.crc24a_poly;
    const uint32_t* table = L == 16 ? a.crc16_table : a.crc24a_table;
    const uint32_t  n     = min(PE_TB_CHUNK, nbytes - c0);
    __syncthreads(); // T, R and s_chunk of the previous TB are no longer read
    if (table_order != L || table_poly != poly) {
      crc_table8_init<PE_CRC_THREADS>(T, L, poly);
      table_order = L;
      table_poly  = poly;
    }
    crc_stage_bytes<PE_CRC_THREADS>(s_chunk, a.tbs + d.tb_offset, c0, n); // coalesced
    __syncthreads();
    const uint32_t b0 = min(n, i * PE_TB_PER), b1 = min(n, b0 + PE_TB_PER);
    R[i]              = crc_chunk_rem(lds_chunk_fetch{s_chunk, 0}, b0, b1, L, T);
    __syncthreads();
    // tree: R[i] <- R[i] x^(8 bytes of the right half) + R[i + h] over the threads' contiguous byte ranges
#pragma unroll
    for (uint32_t h = 1; h < PE_CRC_THREADS; h <<= 1) {
      if ((i & (2 * h - 1)) == 0) {
        const uint32_t rb0 = min(n, (i + h) * PE_TB_PER), rb1 = min(n, (i + 2 * h) * PE_TB_PER);
        R[i] = crc_mulmod(R[i], crc_xpow(8 * (rb1 - rb0), L, table), L, poly) ^ R[i + h];
      }
      __syncthreads();
    }
    if (i == 0) {
      // the chunk's message remainder, times x^(L + TB bits after the chunk)
      a.tb_parts[static_cast<size_t>(t) * a.part_stride + blockIdx.x] =
          crc_move(R[0], L + (d.tbs_bits - 8 * (c0 + n)), L, table);
    }
  }
}

template <int NT>
__global__ __launch_bounds__(NT) void pdsch_cb_kernel(pdsch_fused_args a)
{
  __shared__ pe_lds s;
  crc_table8_init<NT>(s.T24b, 24, a.crc24b_poly);
  const uint32_t j = threadIdx.x;

  // last_only 1: the TBs' last codeblocks (a.last_rows, one per TB, after the TB CRC partials); 0: every other
  // codeblock (those carry no TB CRC and run while the partials are computed); 2: every codeblock (after the partials)
  const uint32_t n = a.last_only == 1 ? a.nof_tbs : a.nof_cbs;
  for (uint32_t k = blockIdx.x; k < n; k += gridDim.x) {
    const uint32_t cb   = a.last_only == 1 ? a.last_rows[k] : k;
    const uint32_t t    = a.row_tb[cb];
    const tb_desc  d    = a.tds[t];
    const uint32_t r    = cb - d.row0;
    const uint32_t C    = d.nof_segments;
    const bool     last = r == C - 1;
    if (a.last_only == 0 && last) {
      continue; // uniform over the workgroup
    }
    const uint32_t L    = d.tb_crc_bits;
    // TB data bits of the segment (the last one: up to the TB CRC; a plan may count that CRC outside cb_info_bits,
    // as pdsch_encoder_hw_impl's single segment does)
    const uint32_t n_data = last ? d.cb_info_bits - L - d.zero_pad : d.cb_info_bits;
    const uint32_t kz     = (a.geos[a.row_geo[cb]].nof_sys / a.enc_rows[cb].Z + 2) * a.enc_rows[cb].Z;
    // ---- 1. the segment's TB data bits; the last segment: the TB CRC (XOR of the partials) after them
    uint32_t tb_crc = 0;
    if (last) {
      const uint32_t np = (d.tbs_bits / 8 + PE_TB_CHUNK - 1) / PE_TB_CHUNK;
      for (uint32_t i = j; i < np; i += NT) {
        tb_crc ^= a.tb_parts[static_cast<size_t>(t) * a.part_stride + i];
      }
      tb_crc = pe_xor<NT>(tb_crc, s.partial);
    }
    pe_message<NT>(a, d, r, n_data, kz, s.s_cw, j);
    __syncthreads();
    if (last && j == 0) {
      attach_crc_bits(s.s_cw, n_data, L, tb_crc); // zero padding stays zero after it
    }
    __syncthreads();
    // ---- 2. CB CRC, encoding, rate matching
    pe_finish<NT>(a, s, cb, d, j);
  }
}

} // namespace

hipError_t launch_pdsch_fused(const pdsch_fused_args& a, hipStream_t crc_stream, hipStream_t cb_stream, hipStream_t stream,
                              int phase)
{
  if (a.nof_cbs == 0) {
    return hipSuccess;
  }
  // threads per codeblock: SRSRAN_AMD_PDSCH_WG (read per launch) 256, else one wave
  const char* wg  = std::getenv("SRSRAN_AMD_PDSCH_WG");
  const bool  big = wg != nullptr && wg[0] == '2';
  auto cb_launch = [&](const pdsch_fused_args& x, uint32_t n, hipStream_t st) {
    const dim3 grid(n < 65535u ? n : 65535u);
    if (big) {
      hipLaunchKernelGGL(pdsch_cb_kernel<256>, grid, dim3(256), 0, st, x);
    } else {
      hipLaunchKernelGGL(pdsch_cb_kernel<64>, grid, dim3(64), 0, st, x);
    }
  };
  if (phase == 2) {
    // one stream: the TB CRC partials, then every codeblock
    hipLaunchKernelGGL(pdsch_tb_crc_kernel,
                       dim3((a.max_tb_bytes + PE_TB_CHUNK - 1) / PE_TB_CHUNK, a.nof_tbs < 65535u ? a.nof_tbs : 65535u),
                       dim3(PE_CRC_THREADS), 0, stream, a);
    pdsch_fused_args b = a;
    b.last_only        = 2;
    cb_launch(b, a.nof_cbs, stream);
  } else if (phase == 0) {
    // the TB CRC partials and the codeblocks without a TB CRC, concurrently
    hipLaunchKernelGGL(pdsch_tb_crc_kernel,
                       dim3((a.max_tb_bytes + PE_TB_CHUNK - 1) / PE_TB_CHUNK, a.nof_tbs < 65535u ? a.nof_tbs : 65535u),
                       dim3(PE_CRC_THREADS), 0, crc_stream, a);
    pdsch_fused_args b = a;
    b.last_only        = 0;
    cb_launch(b, a.nof_cbs, cb_stream);
  } else {
    // the TBs' last codeblocks, once the partials are in
    pdsch_fused_args b = a;
    b.last_only        = 1;
    cb_launch(b, a.nof_tbs, stream);
  }
  return hipGetLastError();
}

} // namespace srs_amd
