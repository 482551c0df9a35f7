// sch.hip -- transport-block kernels of the PDSCH encoder and PUSCH decoder.
//
//   segment_kernel   TX segmentation (ldpc_segmenter_tx_impl.cpp:137-207): one
//                    thread per output byte of a (TB, segment) message row.
//   asm_copy_kernel  HARQ message copies into the soft buffer, one thread per
//                    4 message bytes of the batch;
//   assemble_kernel  RX tail of pusch_decoder_impl.cpp:309-500: one workgroup per
//                    TB; CB CRC status + HARQ flags, LDPC statistics, codeblock
//                    copies of single-codeblock TBs;
//   asm_tb_kernel    codeblock concatenation (concatenate_codeblocks, :460-503)
//                    and the TB CRC24A computed from the concatenated bytes as
//                    they are produced, 2 KiB of a TB per workgroup (linear
//                    CRC, crc_device.h, partials XOR-ed with atomics);
//   asm_final_kernel the TB CRC verdict and the HARQ flag reset.
// Heterogeneous slots (srs_amd_pdsch_encode_slot / srs_amd_pusch_decode_slot) read per-TB descriptors
// (tb_desc): the assembly kernels above through view_of(), and the TX kernels
//   tx_tb_crc_kernel  TB CRC16 / CRC24A per TB, 8 KiB of a TB per workgroup, partials XOR-ed per TB;
//   tx_segment_kernel segmentation with per-TB geometry, one thread per message byte;
//   tx_cb_crc_kernel  CRC24B attachment of the codeblocks of segmented TBs, one wave per codeblock.
// Both are byte-gather kernels far below any roofline next to the LDPC
// kernels they sit between (a few hundred KB per slot).
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "crc_device.h"
#include "sch_args.h"

namespace srs_amd {
namespace {

constexpr int SEG_THREADS = 256;
constexpr int ASM_THREADS = 256;
constexpr uint32_t CRC24A_POLY = 0x1864cfb;
constexpr uint32_t SCH_MAX_SEGMENTS = 512;
constexpr uint32_t ASM_TB_PER       = 32;                        // TB bytes per thread
constexpr uint32_t ASM_TB_CHUNK     = ASM_THREADS * ASM_TB_PER;  // TB bytes per workgroup

__device__ __forceinline__ uint32_t bit_at(const uint8_t* b, uint32_t p)
{
  return (b[p >> 3] >> (7 - (p & 7))) & 1u;
}

// Byte j of segment message row: n_data TB bits from bit tb_off, then (last segment) the TB CRC, zeros after.
__device__ __forceinline__ uint8_t segment_byte(const uint8_t* tb, uint32_t tb_off, uint32_t n_data, bool last,
                                                uint32_t crc, uint32_t tb_crc_bits, uint32_t j)
{
  if (8 * j + 8 <= n_data) {
    // all 8 bits from the TB: one or two byte loads
    const uint32_t q  = tb_off + 8 * j;
    const uint32_t sh = q & 7u;
    uint32_t       w  = static_cast<uint32_t>(tb[q >> 3]) << 8;
    if (sh != 0) {
      w |= tb[(q >> 3) + 1];
    }
    return static_cast<uint8_t>(w >> (8 - sh));
  }
  uint32_t byte = 0;
  for (int k = 0; k < 8; ++k) {
    const uint32_t p = 8 * j + k;
    uint32_t       v = 0;
    if (p < n_data) {
      v = bit_at(tb, tb_off + p);
    } else if (last && p < n_data + tb_crc_bits) {
      v = (crc >> (tb_crc_bits - 1 - (p - n_data))) & 1u;
    }
    byte |= v << (7 - k);
  }
  return static_cast<uint8_t>(byte);
}

__global__ __launch_bounds__(SEG_THREADS) void segment_kernel(segment_args a)
{
  const uint32_t row = blockIdx.y;
  const uint32_t j   = blockIdx.x * SEG_THREADS + threadIdx.x;
  if (row >= a.nof_rows || j >= a.msg_bytes) {
    return;
  }
  const uint32_t t      = row / a.nof_segments;
  const uint32_t r      = row - t * a.nof_segments;
  const bool     last   = r == a.nof_segments - 1;
  const uint32_t n_data = last ? a.last_data_bits : a.cb_info_bits;
  const uint8_t* tb     = a.tbs + static_cast<size_t>(t) * a.tb_stride;
  a.msgs[static_cast<size_t>(row) * a.msg_stride + j] =
      segment_byte(tb, r * a.cb_info_bits, n_data, last, a.tb_crcs[t], a.tb_crc_bits, j);
}

// Segmentation and CRC24B attachment in one pass (C > 1): one wave per (TB, segment) row.  Lane l builds
// the contiguous message bytes [l per, (l + 1) per) in registers (segment_byte), divides them into its CRC
// contribution, the wave XOR-reduces the codeblock CRC, every lane patches the CRC bits that fall into its
// own bytes and stores them: the message row is written once and never read back.
constexpr int      SEGCRC_THREADS = 64;
constexpr uint32_t SEGCRC_PER     = 20; // bytes per lane: 64 x 20 >= 1,056 (BG1 K = 8,448 bits)

__global__ __launch_bounds__(SEGCRC_THREADS) void segment_crc_kernel(segment_args a)
{
  __shared__ uint32_t T[256];
  // the segment's TB bytes (coalesced loads), then the message row (coalesced stores)
  __shared__ __attribute__((aligned(16))) uint8_t s_io[SEGCRC_THREADS * SEGCRC_PER + 8];
  crc_table8_init<SEGCRC_THREADS>(T, 24, a.cb_crc_poly);
  const uint32_t row = blockIdx.x;
  const uint32_t t   = row / a.nof_segments;
  const uint32_t r   = row - t * a.nof_segments;
  const bool     last   = r == a.nof_segments - 1;
  const uint32_t n_data = last ? a.last_data_bits : a.cb_info_bits;
  const uint8_t* tb     = a.tbs + static_cast<size_t>(t) * a.tb_stride;
  const uint32_t crc_t  = a.tb_crcs[t];
  const uint32_t b0     = threadIdx.x * SEGCRC_PER;
  const uint32_t off    = r * a.cb_info_bits;        // first TB bit of the segment
  const uint32_t q0     = off >> 3;                   // its byte
  const uint32_t nsrc   = (off + n_data + 7) / 8 - q0; // TB bytes the segment touches (<= msg_bytes + 1)
  for (uint32_t i = threadIdx.x; i < nsrc; i += SEGCRC_THREADS) {
    s_io[i] = tb[q0 + i];
  }
  __syncthreads(); // T, s_io ready
  uint32_t v[SEGCRC_PER];
#pragma unroll
  for (uint32_t k = 0; k < SEGCRC_PER; ++k) {
    const uint32_t j = b0 + k;
    v[k]             = j < a.msg_bytes ? segment_byte(s_io, off & 7u, n_data, last, crc_t, a.tb_crc_bits, j) : 0u;
  }
  // CRC contribution of this lane's bits below n = cb_info_bits, moved to n (crc_device.h)
  const uint32_t n    = a.cb_info_bits;
  const uint32_t full = n / 8;
  uint32_t       rem  = 0;
#pragma unroll
  for (uint32_t k = 0; k < SEGCRC_PER; ++k) {
    const uint32_t j = b0 + k;
    if (j < full) {
      rem = T[rem >> 16] ^ ((rem << 8) & 0xffffffu) ^ v[k];
    } else if (j == full && (n & 7u) != 0) {
      for (uint32_t i = 0; i < (n & 7u); ++i) {
        rem = (rem << 1) | ((v[k] >> (7 - i)) & 1u);
        if (rem & 0x1000000u) {
          rem ^= a.cb_crc_poly;
        }
      }
    }
  }
  uint32_t contrib = 0;
  if (b0 * 8 < n) {
    const uint32_t e = min(n, (b0 + SEGCRC_PER) * 8);
#pragma unroll
    for (uint32_t i = 0; i < 24; ++i) {
      contrib ^= a.cb_crc_table[n - e + i] & (0u - ((rem >> i) & 1u));
    }
  }
  const uint32_t crc = crc_wave_xor(contrib);
  __syncthreads(); // every lane has read its TB bytes from s_io
#pragma unroll
  for (uint32_t k = 0; k < SEGCRC_PER; ++k) {
    s_io[b0 + k] = static_cast<uint8_t>(v[k]);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    attach_crc_bits(s_io, n, 24, crc); // the CRC bits [n, n + 24): at most four LDS bytes
  }
  __syncthreads();
  uint8_t* m = a.msgs + static_cast<size_t>(row) * a.msg_stride;
  if ((reinterpret_cast<uintptr_t>(m) & 3u) == 0) {
    for (uint32_t w = threadIdx.x; w < (a.msg_bytes + 3) / 4; w += SEGCRC_THREADS) {
      reinterpret_cast<uint32_t*>(m)[w] = reinterpret_cast<const uint32_t*>(s_io)[w]; // row padded to 64 B
    }
  } else {
    for (uint32_t i = threadIdx.x; i < a.msg_bytes; i += SEGCRC_THREADS) {
      m[i] = s_io[i];
    }
  }
}

// ---- PDSCH encoder of a heterogeneous batch (srs_amd_pdsch_encode_slot) ----

// TB CRC (CRC16 / CRC24A per TB): one workgroup per ASM_TB_CHUNK bytes of a TB, partials XOR-ed into acc[t].
__global__ __launch_bounds__(ASM_THREADS) void tx_tb_crc_kernel(tx_slot_args a)
{
  __shared__ uint32_t partial[ASM_THREADS / 64];
  __shared__ uint32_t T[256];
  const uint32_t      t      = blockIdx.y;
  const tb_desc       d      = a.tds[t];
  const uint32_t      nbytes = d.tbs_bits / 8;
  const uint32_t      c0     = blockIdx.x * ASM_TB_CHUNK;
  if (c0 >= nbytes) {
    return; // uniform over the workgroup
  }
  const bool      c16   = d.tb_crc_bits == 16;
  const uint32_t  poly  = c16 ? a.crc16_poly : a.crc24a_poly;
  const uint32_t* table = c16 ? a.crc16_table : a.crc24a_table;
  __shared__ __attribute__((aligned(16))) uint8_t s_chunk[ASM_TB_CHUNK];
  crc_table8_init<ASM_THREADS>(T, d.tb_crc_bits, poly);
  crc_stage_bytes<ASM_THREADS>(s_chunk, a.tbs + d.tb_offset, c0, min(ASM_TB_CHUNK, nbytes - c0)); // coalesced
  __syncthreads();
  const uint32_t b0 = c0 + threadIdx.x * ASM_TB_PER;
  const uint32_t b1 = min(nbytes, b0 + ASM_TB_PER);
  const uint32_t to = min(d.tbs_bits, (c0 + ASM_TB_CHUNK) * 8); // moved to the TB end once per workgroup
  const uint32_t x  = crc_block_xor<ASM_THREADS>(
      crc_chunk_contrib(lds_chunk_fetch{s_chunk, c0}, b0, b1, d.tbs_bits, d.tb_crc_bits, poly, table, T, to),
      partial);
  if (threadIdx.x == 0 && x != 0) {
    atomicXor(a.acc + t, crc_move(x, d.tbs_bits - to, d.tb_crc_bits, table));
  }
}

// Segmentation (ldpc_segmenter_tx_impl.cpp:137-207) with per-TB geometry: one thread per message byte.
__global__ __launch_bounds__(SEG_THREADS) void tx_segment_kernel(tx_slot_args a)
{
  const uint32_t row = blockIdx.y;
  const uint32_t j   = blockIdx.x * SEG_THREADS + threadIdx.x;
  const uint32_t t   = a.row_tb[row];
  const tb_desc  d   = a.tds[t];
  if (j >= d.msg_bytes) {
    return;
  }
  const uint32_t r      = row - d.row0;
  const bool     last   = r == d.nof_segments - 1;
  const uint32_t n_data = last ? d.cb_info_bits - d.tb_crc_bits - d.zero_pad : d.cb_info_bits;
  a.msgs[static_cast<size_t>(row) * a.msg_stride + j] =
      segment_byte(a.tbs + d.tb_offset, r * d.cb_info_bits, n_data, last, a.acc[t], d.tb_crc_bits, j);
}

// CRC24B attachment to the codeblocks of segmented TBs (ldpc_segmenter_tx_impl.cpp:196): one wave per row,
// the CRC bits MSB-first into message bits [cb_info_bits, cb_info_bits + 24).
__global__ __launch_bounds__(64) void tx_cb_crc_kernel(tx_slot_args a)
{
  __shared__ uint32_t partial[1];
  __shared__ uint32_t T[256];
  const uint32_t      row = blockIdx.x;
  const tb_desc       d   = a.tds[a.row_tb[row]];
  if (d.nof_segments == 1) {
    return;
  }
  crc_table8_init<64>(T, 24, a.crc24b_poly);
  __syncthreads();
  uint8_t*       m   = a.msgs + static_cast<size_t>(row) * a.msg_stride;
  const uint32_t n   = d.cb_info_bits;
  const uint32_t crc = block_crc_bytes<64>(row_fetch{m}, n, 24, a.crc24b_poly, a.crc24b_table, T, partial);
  if (threadIdx.x == 0) {
    attach_crc_bits(m, n, 24, crc);
  }
}

// TB byte j (bits 8j..8j+7) gathered from the concatenated codeblock data bits.
struct tb_gather {
  const uint8_t* base;
  uint32_t       stride;
  uint32_t       cbi;
  float          rcp; // 1 / cbi: the codeblock of bit b from a float estimate and one correction (b < 2^24)
  __device__ tb_gather(const uint8_t* base_, uint32_t stride_, uint32_t cbi_) :
    base(base_), stride(stride_), cbi(cbi_), rcp(1.0f / static_cast<float>(cbi_))
  {
  }
  __device__ uint32_t operator()(uint32_t j) const
  {
    uint32_t byte = 0;
    uint32_t b    = 8 * j;
    uint32_t r    = static_cast<uint32_t>(static_cast<float>(b) * rcp);
    int32_t  x    = static_cast<int32_t>(b - r * cbi);
    if (x < 0) {
      r -= 1;
      x += static_cast<int32_t>(cbi);
    } else if (x >= static_cast<int32_t>(cbi)) {
      r += 1;
      x -= static_cast<int32_t>(cbi);
    }
    uint32_t o = static_cast<uint32_t>(x);
    if (o + 8 <= cbi) {
      // the 8 bits lie in one codeblock: one or two byte loads
      const uint8_t* m  = base + static_cast<size_t>(r) * stride + (o >> 3);
      const uint32_t sh = o & 7u;
      uint32_t       w  = static_cast<uint32_t>(m[0]) << 8;
      if (sh != 0) {
        w |= m[1];
      }
      return (w >> (8 - sh)) & 0xffu;
    }
    for (int k = 0; k < 8; ++k) {
      byte |= bit_at(base + static_cast<size_t>(r) * stride, o) << (7 - k);
      if (++o == cbi) {
        o = 0;
        ++r;
      }
    }
    return byte;
  }
};

// HARQ message copies (pusch_decoder_impl.cpp:334-375): every decoded codeblock not already OK from an
// earlier transmission stores its message in its soft-buffer row. One thread per 4 message bytes over
// all codeblocks of the batch; runs before assemble_kernel rewrites the CRC flags it reads.
__global__ __launch_bounds__(ASM_THREADS) void asm_copy_kernel(assemble_args a, uint32_t nof_cbs, uint32_t nw)
{
  const uint32_t x = blockIdx.x * ASM_THREADS + threadIdx.x;
  if (x >= nof_cbs * nw) {
    return;
  }
  const uint32_t cb   = x / nw;
  const uint32_t w    = x - cb * nw;
  uint8_t*       srow = a.soft + static_cast<size_t>(cb) * a.lay.row_bytes;
  if (!a.new_data && *reinterpret_cast<const int32_t*>(srow + a.lay.flag_offset) != 0) {
    return; // kept from a previous transmission
  }
  const uint32_t msg_bytes = a.lay.flag_offset - a.lay.msg_offset;
  const uint8_t* m         = a.msgs + static_cast<size_t>(cb) * a.msg_stride;
  if ((((reinterpret_cast<uintptr_t>(a.soft) | reinterpret_cast<uintptr_t>(a.msgs)) | a.lay.row_bytes |
        a.lay.msg_offset | a.msg_stride | msg_bytes) & 3u) == 0) {
    reinterpret_cast<uint32_t*>(srow + a.lay.msg_offset)[w] = reinterpret_cast<const uint32_t*>(m)[w];
    return;
  }
  for (uint32_t j = 4 * w; j < min(msg_bytes, 4 * w + 4); ++j) {
    srow[a.lay.msg_offset + j] = m[j];
  }
}

// Transport block t of a batch: uniform plan, or its descriptor in a heterogeneous batch.
struct tb_view {
  uint8_t* tb;
  uint32_t row0, C, cbi, tbs_bits;
};

__device__ __forceinline__ tb_view view_of(const assemble_args& a, uint32_t t)
{
  if (a.tds != nullptr) {
    const tb_desc d = a.tds[t];
    return {a.tbs + d.tb_offset, d.row0, d.nof_segments, d.cb_info_bits, d.tbs_bits};
  }
  return {a.tbs + static_cast<size_t>(t) * a.tb_stride, t * a.nof_segments, a.nof_segments, a.cb_info_bits,
          a.tbs_bits};
}

// CB CRC status, LDPC statistics, HARQ flags, single-codeblock TBs and the result row of TB t (one workgroup).
// zero_acc: clear the TB's CRC accumulator for asm_tb_kernel (launched after this kernel); the merged form
// (asm_merged_kernel) relies on asm_final_kernel having cleared it after its previous use instead.
__device__ __forceinline__ void assemble_tb(const assemble_args& a, uint32_t t, bool zero_acc)
{
  __shared__ uint32_t s_ok, s_sum, s_min, s_max, s_tb_ok;
  __shared__ uint8_t  s_fresh[SCH_MAX_SEGMENTS]; // decoded in this call (not OK from a previous transmission)
  __shared__ uint8_t  s_cb_ok[SCH_MAX_SEGMENTS];
  __shared__ uint16_t s_stat[SCH_MAX_SEGMENTS]; // iterations of the freshly decoded codeblocks
  const tb_view       v = view_of(a, t);
  if (zero_acc && threadIdx.x == 0 && a.acc != nullptr) {
    a.acc[t] = 0; // the TB CRC accumulator of asm_tb_kernel (launched after this kernel): no memset launch
  }
  const uint32_t      C = v.C;
  if (threadIdx.x == 0) {
    s_ok    = 0;
    s_sum   = 0;
    s_min   = 0xffffffffu;
    s_max   = 0;
    s_tb_ok = 0;
  }
  __syncthreads();
  // 1. CB CRC status (pusch_decoder_impl.cpp:334-375) and LDPC statistics.
  for (uint32_t r = threadIdx.x; r < C; r += ASM_THREADS) {
    const uint32_t cb   = v.row0 + r;
    const uint8_t* srow = a.soft ? a.soft + static_cast<size_t>(cb) * a.lay.row_bytes : nullptr;
    // the soft-buffer flag of a codeblock OK from an earlier transmission holds that decoding's iteration
    // count, which the reference's statistics keep for it (cb_stats is not updated, :333-345)
    const int32_t  flag = srow && !a.new_data ? *reinterpret_cast<const int32_t*>(srow + a.lay.flag_offset) : 0;
    const bool     prev = flag != 0;
    const int32_t  it   = a.iters[cb];
    const bool     dec  = !prev && (a.crc_checks ? (a.crc_checks[cb] == 0) : (it >= 0));
    const uint32_t stat = prev  ? static_cast<uint32_t>(flag)
                          : dec ? (a.crc_checks ? a.max_iterations : static_cast<uint32_t>(it))
                                : a.max_iterations;
    const bool     ok   = prev || dec;
    s_fresh[r]          = prev ? 0 : 1;
    s_cb_ok[r]          = ok ? 1 : 0;
    if (a.cb_iterations) {
      // slot form: the caller's per-codeblock index of the TB's first codeblock (tb_desc::pad)
      a.cb_iterations[a.tds != nullptr ? a.tds[t].pad + r : cb] = ok ? static_cast<int32_t>(stat) : -1;
    }
    if (!prev && a.soft) {
      s_stat[r] = stat;
    }
    atomicAdd(&s_ok, ok ? 1u : 0u);
    atomicAdd(&s_sum, stat);
    atomicMin(&s_min, stat);
    atomicMax(&s_max, stat);
  }
  __syncthreads();
  // 2. HARQ: CRC flags of the freshly decoded codeblocks into the soft buffer.
  const uint8_t* src = a.msgs + static_cast<size_t>(v.row0) * a.msg_stride;
  if (a.soft) {
    // the fresh messages were copied by asm_copy_kernel (launched before this kernel, which then
    // overwrites the flags it read)
    for (uint32_t r = threadIdx.x; r < C; r += ASM_THREADS) {
      if (s_fresh[r]) {
        *reinterpret_cast<int32_t*>(a.soft + static_cast<size_t>(v.row0 + r) * a.lay.row_bytes + a.lay.flag_offset) =
            s_cb_ok[r] ? static_cast<int32_t>(s_stat[r]) : 0;
      }
    }
    __syncthreads();
    src = a.soft + static_cast<size_t>(v.row0) * a.lay.row_bytes + a.lay.msg_offset;
  }
  // 3. Transport block (pusch_decoder_impl.cpp:416-437).
  uint8_t*       tb     = v.tb;
  const uint32_t nbytes = v.tbs_bits / 8;
  const bool     all_ok = s_ok == C;
  if (C == 1) {
    if (all_ok) {
      for (uint32_t j = threadIdx.x; j < nbytes; j += ASM_THREADS) {
        tb[j] = src[j];
      }
    }
    if (threadIdx.x == 0) {
      s_tb_ok = all_ok ? 1 : 0;
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    srs_amd_pusch_decoder_result res{};
    res.tb_crc_ok             = static_cast<int32_t>(s_tb_ok); // C > 1: set by asm_final_kernel
    res.nof_codeblocks_total  = C;
    res.ldpc_iterations_sum   = s_sum;
    res.ldpc_iterations_min   = s_min;
    res.ldpc_iterations_max   = s_max;
    res.nof_codeblocks_crc_ok = s_ok;
    a.results[t]              = res;
  }
}

__global__ __launch_bounds__(ASM_THREADS) void assemble_kernel(assemble_args a)
{
  assemble_tb(a, blockIdx.x, true);
}

// Source of the concatenated codeblock messages of TB t (the soft-buffer copies when HARQ state is kept).
__device__ __forceinline__ const uint8_t* asm_source(const assemble_args& a, const tb_view& v, uint32_t& stride)
{
  if (a.soft) {
    stride = a.lay.row_bytes;
    return a.soft + static_cast<size_t>(v.row0) * a.lay.row_bytes + a.lay.msg_offset;
  }
  stride = a.msg_stride;
  return a.msgs + static_cast<size_t>(v.row0) * a.msg_stride;
}

struct lds_fetch {
  const uint8_t* chunk;
  uint32_t       first;
  __device__ uint32_t operator()(uint32_t j) const { return chunk[j - first]; }
};

// C > 1, every codeblock OK: concatenation (concatenate_codeblocks, pusch_decoder_impl.cpp:460-503) and
// TB CRC24A contributions, one workgroup per TB_CHUNK bytes of a TB: the chunk is gathered with consecutive
// threads on consecutive bytes (coalesced codeblock reads and TB writes) into LDS, then each thread folds
// its TB_PER contiguous bytes into a CRC contribution.
// Chunk `chunk` of TB t when every codeblock of the TB is OK (all_ok: from the assembly's result row, or computed
// by the caller in the merged form).
__device__ __forceinline__ void asm_tb_chunk(const assemble_args& a, uint32_t t, uint32_t chunk, bool use_results)
{
  __shared__ uint32_t partial[ASM_THREADS / 64];
  __shared__ uint32_t T[256];
  __shared__ uint8_t  s_chunk[ASM_TB_CHUNK];
  __shared__ uint32_t s_bad;
  const tb_view       v = view_of(a, t);
  const uint32_t      c0 = chunk * ASM_TB_CHUNK;
  if (v.C == 1 || c0 >= v.tbs_bits / 8) {
    return; // uniform over the workgroup
  }
  if (use_results) {
    if (a.results[t].nof_codeblocks_crc_ok != v.C) {
      return;
    }
  } else {
    // no HARQ state (a.soft null): a codeblock is OK exactly when this call decoded it with a CRC pass, as
    // assemble_tb counts it
    if (threadIdx.x == 0) {
      s_bad = 0;
    }
    __syncthreads();
    for (uint32_t r = threadIdx.x; r < v.C; r += ASM_THREADS) {
      const uint32_t cb = v.row0 + r;
      const bool     ok = a.crc_checks ? (a.crc_checks[cb] == 0) : (a.iters[cb] >= 0);
      if (!ok) {
        s_bad = 1;
      }
    }
    __syncthreads();
    if (s_bad != 0) {
      return;
    }
  }
  crc_table8_init<ASM_THREADS>(T, 24, CRC24A_POLY);
  uint32_t        stride;
  const uint8_t*  src    = asm_source(a, v, stride);
  const tb_gather g{src, stride, v.cbi};
  uint8_t*        tb     = v.tb;
  const uint32_t  nbytes = v.tbs_bits / 8;
  const uint32_t  n      = min(ASM_TB_CHUNK, nbytes - c0);
  constexpr uint32_t U = 8; // gathers in flight per thread before their stores
  for (uint32_t i0 = threadIdx.x; i0 < n; i0 += U * ASM_THREADS) {
    uint32_t v[U];
#pragma unroll
    for (uint32_t r = 0; r < U; ++r) {
      const uint32_t i = i0 + r * ASM_THREADS;
      v[r]             = i < n ? g(c0 + i) : 0u;
    }
#pragma unroll
    for (uint32_t r = 0; r < U; ++r) {
      const uint32_t i = i0 + r * ASM_THREADS;
      if (i < n) {
        s_chunk[i] = static_cast<uint8_t>(v[r]);
        tb[c0 + i] = static_cast<uint8_t>(v[r]);
      }
    }
  }
  __syncthreads();
  const uint32_t b0 = c0 + threadIdx.x * ASM_TB_PER;
  const uint32_t b1 = min(nbytes, b0 + ASM_TB_PER);
  const uint32_t to = min(v.tbs_bits, (c0 + ASM_TB_CHUNK) * 8); // moved to the TB end once per workgroup
  const uint32_t x  = crc_block_xor<ASM_THREADS>(
      crc_chunk_contrib(lds_fetch{s_chunk, c0}, b0, b1, v.tbs_bits, 24, CRC24A_POLY, a.crc24a_table, T, to),
      partial);
  if (threadIdx.x == 0 && x != 0) {
    atomicXor(a.acc + t, crc_move(x, v.tbs_bits - to, 24, a.crc24a_table));
  }
}

__global__ __launch_bounds__(ASM_THREADS) void asm_tb_kernel(assemble_args a)
{
  asm_tb_chunk(a, blockIdx.y, blockIdx.x, true);
}

// No HARQ state (a.soft null): the assembly of TB blockIdx.y (last workgroup of its row) and its concatenation /
// CRC chunks (the other workgroups) in one launch -- one launch and one dependency fewer on the PUSCH critical path.
__global__ __launch_bounds__(ASM_THREADS) void asm_merged_kernel(assemble_args a)
{
  if (blockIdx.x == gridDim.x - 1) {
    assemble_tb(a, blockIdx.y, false);
  } else {
    asm_tb_chunk(a, blockIdx.y, blockIdx.x, false);
  }
}

// TB CRC verdict (pusch_decoder_impl.cpp:416-437): the checksum is the 24 bits after the TB data in the
// last codeblock; a mismatch flags a false CB CRC positive and resets the kept CB flags.
__global__ __launch_bounds__(64) void asm_final_kernel(assemble_args a, uint32_t nof_tbs)
{
  const uint32_t t = blockIdx.x * 64 + threadIdx.x;
  if (t >= nof_tbs) {
    return;
  }
  const tb_view  v = view_of(a, t);
  const uint32_t C = v.C;
  // the accumulator is read and cleared on every path (the merged form relies on zero accumulators at its start)
  const uint32_t acc = a.acc != nullptr ? a.acc[t] : 0u;
  if (a.acc != nullptr) {
    a.acc[t] = 0;
  }
  if (C == 1 || a.results[t].nof_codeblocks_crc_ok != C) {
    return;
  }
  uint32_t       stride;
  const uint8_t* src = asm_source(a, v, stride);
  const uint32_t off = v.tbs_bits - (C - 1) * v.cbi;
  const uint8_t* m   = src + static_cast<size_t>(C - 1) * stride;
  uint32_t       chk = 0;
  for (uint32_t k = 0; k < 24; ++k) {
    chk = (chk << 1) | bit_at(m, off + k);
  }
  const bool ok           = acc == chk;
  a.results[t].tb_crc_ok  = ok ? 1 : 0;
  if (!ok && a.soft) {
    for (uint32_t r = 0; r < C; ++r) {
      uint8_t* srow = a.soft + static_cast<size_t>(v.row0 + r) * a.lay.row_bytes;
      *reinterpret_cast<int32_t*>(srow + a.lay.flag_offset) = 0;
    }
  }
}

} // namespace

// ---- HARQ state of the slot decoder (sch_args.h harq_args) ----------------------------------------------------------
constexpr uint32_t HARQ_THREADS = 256;

// Copies n bytes (4-byte words when both ends allow it) with the workgroup's threads, chunk blockIdx.x.
__device__ __forceinline__ void harq_copy(uint8_t* dst, const uint8_t* src, uint32_t n)
{
  const uint32_t chunk = HARQ_THREADS * 16;
  const uint32_t b0    = blockIdx.x * chunk;
  const uint32_t b1    = min(n, b0 + chunk);
  if (b0 >= b1) {
    return;
  }
  if (((reinterpret_cast<uintptr_t>(dst) | reinterpret_cast<uintptr_t>(src)) & 3u) == 0) {
    const uint32_t w1 = b1 / 4;
    for (uint32_t w = b0 / 4 + threadIdx.x; w < w1; w += HARQ_THREADS) {
      reinterpret_cast<uint32_t*>(dst)[w] = reinterpret_cast<const uint32_t*>(src)[w];
    }
    for (uint32_t j = max(b0, w1 * 4) + threadIdx.x; j < b1; j += HARQ_THREADS) {
      dst[j] = src[j];
    }
    return;
  }
  for (uint32_t j = b0 + threadIdx.x; j < b1; j += HARQ_THREADS) {
    dst[j] = src[j];
  }
}

__global__ __launch_bounds__(HARQ_THREADS) void harq_gather_kernel(harq_args a)
{
  const harq_row_desc d = a.rows[blockIdx.y];
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    // new data: every CRC flag starts cleared (pusch_decoder_impl.cpp:133-135)
    a.prev[blockIdx.y] = d.new_data ? 0 : *reinterpret_cast<const int32_t*>(d.soft_row + d.flag_offset);
  }
  if (!d.new_data) { // combining reads the earlier transmissions' soft bits
    harq_copy(reinterpret_cast<uint8_t*>(a.internal) + static_cast<size_t>(d.row) * a.S, d.soft_row, d.soft_bytes);
  }
}

__global__ __launch_bounds__(HARQ_THREADS) void harq_scatter_kernel(harq_args a)
{
  const harq_row_desc d    = a.rows[blockIdx.y];
  bool                keep = true;
  if (d.lazy) {
    // new data kept only for a retransmission: the soft LLRs matter only if some codeblock of the TB failed
    int fail = 0;
    for (uint32_t c = threadIdx.x; c < d.tb_C; c += HARQ_THREADS) {
      fail |= a.iters[d.tb_row0 + c] < 0 ? 1 : 0;
    }
    keep = __syncthreads_or(fail) != 0;
  }
  if (keep) {
    harq_copy(d.soft_row, reinterpret_cast<const uint8_t*>(a.internal) + static_cast<size_t>(d.row) * a.S,
              d.soft_bytes);
  }
  if (blockIdx.x != 0) {
    return;
  }
  const int32_t prev = a.prev[blockIdx.y];
  uint8_t*      m    = a.msgs + static_cast<size_t>(d.row) * a.M;
  uint8_t*      sm   = d.soft_row + d.msg_offset;
  if (prev != 0) {
    // OK from an earlier transmission: its stored message and iteration count (:333-345, cb_stats not updated)
    for (uint32_t j = threadIdx.x; j < d.msg_bytes; j += HARQ_THREADS) {
      m[j] = sm[j];
    }
    if (threadIdx.x == 0) {
      a.iters[d.row] = prev;
    }
    return;
  }
  const int32_t it = a.iters[d.row];
  if (it >= 0) { // decoded now: the message and the flag (its iteration count) kept for later transmissions
    for (uint32_t j = threadIdx.x; j < d.msg_bytes; j += HARQ_THREADS) {
      sm[j] = m[j];
    }
  }
  if (threadIdx.x == 0) {
    *reinterpret_cast<int32_t*>(d.soft_row + d.flag_offset) = it >= 0 ? it : 0;
  }
}

// one workgroup per TB
__global__ __launch_bounds__(HARQ_THREADS) void harq_final_kernel(harq_args a)
{
  const harq_tb_desc                  d = a.tbs[blockIdx.x];
  const srs_amd_pusch_decoder_result& r = a.results[d.result];
  // every codeblock passed but not the TB CRC: reset_codeblocks_crc (pusch_decoder_impl.cpp:425-437)
  if (d.C > 1 && r.nof_codeblocks_crc_ok == d.C && !r.tb_crc_ok) {
    for (uint32_t c = threadIdx.x; c < d.C; c += HARQ_THREADS) {
      *reinterpret_cast<int32_t*>(d.soft + static_cast<size_t>(c) * d.row_bytes + d.flag_offset) = 0;
    }
    if (d.lazy) {
      // the scatter skipped the soft LLRs (no codeblock failed): the retransmission combines with them
      for (uint32_t c = 0; c < d.C; ++c) {
        const uint8_t* src = reinterpret_cast<const uint8_t*>(a.internal) + static_cast<size_t>(d.row0 + c) * a.S;
        uint8_t*       dst = d.soft + static_cast<size_t>(c) * d.row_bytes;
        for (uint32_t j = threadIdx.x; j < d.soft_bytes; j += HARQ_THREADS) {
          dst[j] = src[j];
        }
      }
    }
  }
}

hipError_t launch_harq_gather(const harq_args& a, uint32_t max_soft_bytes, hipStream_t stream)
{
  if (a.nof_rows == 0) {
    return hipSuccess;
  }
  const uint32_t gx = max_soft_bytes > HARQ_THREADS * 16 ? (max_soft_bytes + HARQ_THREADS * 16 - 1) / (HARQ_THREADS * 16)
                                                         : 1u;
  hipLaunchKernelGGL(harq_gather_kernel, dim3(gx, a.nof_rows), dim3(HARQ_THREADS), 0, stream, a);
  return hipGetLastError();
}

hipError_t launch_harq_scatter(const harq_args& a, uint32_t max_soft_bytes, hipStream_t stream)
{
  if (a.nof_rows == 0) {
    return hipSuccess;
  }
  const uint32_t gx = max_soft_bytes > HARQ_THREADS * 16 ? (max_soft_bytes + HARQ_THREADS * 16 - 1) / (HARQ_THREADS * 16)
                                                         : 1u;
  hipLaunchKernelGGL(harq_scatter_kernel, dim3(gx, a.nof_rows), dim3(HARQ_THREADS), 0, stream, a);
  return hipGetLastError();
}

__global__ __launch_bounds__(64) void slot_row_patch_kernel(const slot_row_patch* items)
{
  const slot_row_patch& p = items[blockIdx.x];
  const int32_t         s = *p.sel;
  if (s < 0) {
    return;
  }
  for (uint32_t r = threadIdx.x; r < p.C; r += 64) {
    p.row_E[r]  = p.cand_E[static_cast<size_t>(s) * p.C + r];
    p.row_in[r] = p.llr_offset + p.cand_off[static_cast<size_t>(s) * p.C + r];
  }
}

hipError_t launch_slot_row_patch(const slot_row_patch* items, uint32_t n, hipStream_t stream)
{
  if (n == 0) {
    return hipSuccess;
  }
  hipLaunchKernelGGL(slot_row_patch_kernel, dim3(n), dim3(64), 0, stream, items);
  return hipGetLastError();
}

hipError_t launch_harq_final(const harq_args& a, hipStream_t stream)
{
  if (a.nof_tbs == 0) {
    return hipSuccess;
  }
  hipLaunchKernelGGL(harq_final_kernel, dim3(a.nof_tbs), dim3(HARQ_THREADS), 0, stream, a);
  return hipGetLastError();
}


__global__ __launch_bounds__(256) void rm_arrays_kernel(uint32_t* arrays, uint32_t rows, uint32_t C, uint32_t S,
                                                       uint32_t e_short, uint32_t e_long, uint32_t tb_units)
{
  const uint32_t row = blockIdx.x * 256 + threadIdx.x;
  if (row < rows) {
    const uint32_t tb = row / C, r = row - tb * C;
    arrays[row]        = r < S ? e_short : e_long;
    arrays[rows + row] = tb * tb_units + (r < S ? r * e_short : S * e_short + (r - S) * e_long);
  }
}

hipError_t launch_rm_arrays(uint32_t* arrays, uint32_t nof_tbs, uint32_t C, uint32_t nof_short, uint32_t e_short,
                            uint32_t e_long, uint32_t tb_units, hipStream_t stream)
{
  const uint32_t rows = nof_tbs * C;
  hipLaunchKernelGGL(rm_arrays_kernel, dim3((rows + 255) / 256), dim3(256), 0, stream, arrays, rows, C, nof_short,
                     e_short, e_long, tb_units);
  return hipGetLastError();
}

bool segment_attaches_crc(const segment_args& a)
{
  return a.cb_crc_table != nullptr && a.msg_bytes <= SEGCRC_THREADS * SEGCRC_PER;
}

hipError_t launch_segment(const segment_args& a, hipStream_t stream)
{
  if (a.nof_rows == 0) {
    return hipSuccess;
  }
  if (segment_attaches_crc(a)) {
    hipLaunchKernelGGL(segment_crc_kernel, dim3(a.nof_rows), dim3(SEGCRC_THREADS), 0, stream, a);
    return hipGetLastError();
  }
  dim3 grid((a.msg_bytes + SEG_THREADS - 1) / SEG_THREADS, a.nof_rows);
  hipLaunchKernelGGL(segment_kernel, grid, dim3(SEG_THREADS), 0, stream, a);
  return hipGetLastError();
}

hipError_t launch_tx_slot_segment(const tx_slot_args& a, hipStream_t stream)
{
  if (a.nof_tbs == 0) {
    return hipSuccess;
  }
  hipError_t e = hipMemsetAsync(a.acc, 0, sizeof(uint32_t) * a.nof_tbs, stream);
  if (e != hipSuccess) {
    return e;
  }
  hipLaunchKernelGGL(tx_tb_crc_kernel, dim3((a.max_tb_bytes + ASM_TB_CHUNK - 1) / ASM_TB_CHUNK, a.nof_tbs),
                     dim3(ASM_THREADS), 0, stream, a);
  hipLaunchKernelGGL(tx_segment_kernel, dim3((a.max_msg_bytes + SEG_THREADS - 1) / SEG_THREADS, a.nof_rows),
                     dim3(SEG_THREADS), 0, stream, a);
  hipLaunchKernelGGL(tx_cb_crc_kernel, dim3(a.nof_rows), dim3(64), 0, stream, a);
  return hipGetLastError();
}

hipError_t launch_assemble(const assemble_args& a, uint32_t nof_tbs, hipStream_t stream)
{
  if (nof_tbs == 0) {
    return hipSuccess;
  }
  if (a.soft) {
    const uint32_t nw  = (a.lay.flag_offset - a.lay.msg_offset + 3) / 4;
    const uint32_t ncb = nof_tbs * a.nof_segments;
    hipLaunchKernelGGL(asm_copy_kernel, dim3((ncb * nw + ASM_THREADS - 1) / ASM_THREADS), dim3(ASM_THREADS), 0,
                       stream, a, ncb, nw);
  }
  const uint32_t nbytes = (a.tds != nullptr ? a.max_tb_bits : a.tbs_bits) / 8;
  const char*    mv     = std::getenv("SRSRAN_AMD_ASM_MERGED"); // read per call: 0 keeps the three-launch form
  if (a.soft == nullptr && !(a.tds == nullptr && a.nof_segments == 1) && !(mv != nullptr && mv[0] == '0')) {
    // the accumulators start at zero (allocation) and asm_final_kernel clears each one it reads
    hipLaunchKernelGGL(asm_merged_kernel, dim3((nbytes + ASM_TB_CHUNK - 1) / ASM_TB_CHUNK + 1, nof_tbs),
                       dim3(ASM_THREADS), 0, stream, a);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
      return e;
    }
    hipLaunchKernelGGL(asm_final_kernel, dim3((nof_tbs + 63) / 64), dim3(64), 0, stream, a, nof_tbs);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(assemble_kernel, dim3(nof_tbs), dim3(ASM_THREADS), 0, stream, a);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess || (a.tds == nullptr && a.nof_segments == 1)) {
    return e;
  }
  // a.acc was zeroed by assemble_kernel
  hipLaunchKernelGGL(asm_tb_kernel, dim3((nbytes + ASM_TB_CHUNK - 1) / ASM_TB_CHUNK, nof_tbs), dim3(ASM_THREADS), 0,
                     stream, a);
  e = hipGetLastError();
  if (e != hipSuccess) {
    return e;
  }
  hipLaunchKernelGGL(asm_final_kernel, dim3((nof_tbs + 63) / 64), dim3(64), 0, stream, a, nof_tbs);
  return hipGetLastError();
}

} // namespace srs_amd
