// crc_device.h -- linear CRC of rows of packed bits (device code shared by
// crc.hip and sch.hip).
//
// The CRC is linear, so a row is split into contiguous byte chunks, one per
// thread (and, for long rows, several workgroups per row): a thread divides
// its chunk, R_t = chunk_t(x) mod g, byte by byte with a 256-entry table in
// LDS (T[t] = t(x) x^L mod g; bitwise for the partial last byte and for
// L < 8, the shift register of crc_calculator_generic_impl.cpp:98-127), moves
// it to the row's end with table[k] = x^(k+L) mod g (R_t(x) x^(n - e_t + L)
// mod g = XOR of table[j + n - e_t] over the set bits j of R_t) and the
// contributions are XOR-reduced (wave shuffles, LDS, atomics across
// workgroups).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace srs_amd {

__device__ __forceinline__ uint32_t crc_wave_xor(uint32_t v)
{
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    v ^= static_cast<uint32_t>(__shfl_xor(static_cast<int>(v), o, 64));
  }
  return v;
}

// T[t] = t(x) x^L mod g for t < 256 (L >= 8). All threads of the block call it.
template <int THREADS>
__device__ __forceinline__ void crc_table8_init(uint32_t* T, uint32_t order, uint32_t polynom)
{
  if (order < 8) {
    return;
  }
  const uint32_t highbit = 1u << order;
  for (uint32_t t = threadIdx.x; t < 256; t += THREADS) {
    uint32_t r = t << (order - 8);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      r <<= 1;
      if (r & highbit) {
        r ^= polynom;
      }
    }
    T[t] = r;
  }
}

// Bytes fetched per batch before the division chain consumes them: the loads of a batch are independent
// and all in flight at once (a fetch-then-divide loop per byte waits one memory latency per byte).
constexpr uint32_t CRC_FETCH_BATCH = 16;
// Largest CRC order of the path (CRC24A/B/C): the remainder move below is unrolled to it.
constexpr uint32_t CRC_MAX_ORDER = 24;

// This thread's contribution to the CRC of the n-bit message (byte j = fetch(j), MSB first) from
// its bytes [b0, b1), as if the message ended at bit `to` (to = n: the contribution itself; a workgroup
// that sums its threads' contributions at the end of its chunk moves the sum to n once, crc_move, instead of
// every thread reading the far end of the table).
template <typename Fetch>
__device__ __forceinline__ uint32_t crc_chunk_contrib(const Fetch&    fetch,
                                                      uint32_t        b0,
                                                      uint32_t        b1,
                                                      uint32_t        n,
                                                      uint32_t        order,
                                                      uint32_t        polynom,
                                                      const uint32_t* table,
                                                      const uint32_t* T,
                                                      uint32_t        to = 0xffffffffu)
{
  to = to == 0xffffffffu ? n : to;
  if (b0 >= b1) {
    return 0;
  }
  const uint32_t highbit = 1u << order;
  const uint32_t mask    = highbit - 1u;
  const uint32_t full    = min(b1, n / 8); // whole bytes
  uint32_t       r       = 0;
  uint32_t       b       = b0;
  if (order >= 8) {
    const uint32_t sh = order - 8;
    for (; b < full; b += CRC_FETCH_BATCH) {
      uint32_t v[CRC_FETCH_BATCH];
#pragma unroll
      for (uint32_t k = 0; k < CRC_FETCH_BATCH; ++k) {
        v[k] = b + k < full ? fetch(b + k) : 0u;
      }
#pragma unroll
      for (uint32_t k = 0; k < CRC_FETCH_BATCH; ++k) {
        if (b + k < full) {
          r = T[r >> sh] ^ ((r << 8) & mask) ^ v[k];
        }
      }
    }
    b = max(b0, full);
  }
  for (; b < b1; ++b) {
    const uint32_t byte = fetch(b);
    const int      nb   = (b * 8 + 8 <= n) ? 8 : static_cast<int>(n - b * 8);
    for (int i = 0; i < nb; ++i) {
      r = (r << 1) | ((byte >> (7 - i)) & 1u);
      if (r & highbit) {
        r ^= polynom;
      }
    }
  }
  // move the remainder to the message end: XOR of table[j + n - e] over the set bits j of r (independent
  // loads, unrolled so that they are all in flight together)
  const uint32_t  e       = min(n, b1 * 8);
  const uint32_t* tj      = table + (to - e);
  uint32_t        contrib = 0;
#pragma unroll
  for (uint32_t j = 0; j < CRC_MAX_ORDER; ++j) {
    if (j < order) {
      contrib ^= tj[j] & (0u - ((r >> j) & 1u));
    }
  }
  return contrib;
}

// R(x) x^d mod g for a remainder R of degree < order: bit j moves to x^(j + d), reduced through the linear
// table (table[k] = x^(k + order) mod g) when j + d >= order.  Branch-free: the table words of every bit position
// are loaded unconditionally (all in flight together, one memory latency) and masked by the bits of R.
__device__ __forceinline__ uint32_t crc_move(uint32_t R, uint32_t d, uint32_t order, const uint32_t* table)
{
  uint32_t out = 0;
#pragma unroll
  for (uint32_t j = 0; j < CRC_MAX_ORDER; ++j) {
    const uint32_t k    = j + d;
    const uint32_t word = k >= order ? table[k - order] : 0u;
    const uint32_t v    = k < order ? (1u << (k & 31u)) : word;
    out ^= (j < order) ? (v & (0u - ((R >> j) & 1u))) : 0u;
  }
  return out;
}

// The remainder M(x) mod g of the message bytes [b0, b1) alone (byte j = fetch(j), MSB first, every byte whole),
// by the byte table T (crc_table8_init; order >= 8).
template <typename Fetch>
__device__ __forceinline__ uint32_t crc_chunk_rem(const Fetch& fetch, uint32_t b0, uint32_t b1, uint32_t order,
                                                  const uint32_t* T)
{
  const uint32_t mask = (1u << order) - 1u;
  const uint32_t sh   = order - 8;
  uint32_t       r    = 0;
  for (uint32_t b = b0; b < b1; b += CRC_FETCH_BATCH) {
    uint32_t v[CRC_FETCH_BATCH];
#pragma unroll
    for (uint32_t k = 0; k < CRC_FETCH_BATCH; ++k) {
      v[k] = b + k < b1 ? fetch(b + k) : 0u;
    }
#pragma unroll
    for (uint32_t k = 0; k < CRC_FETCH_BATCH; ++k) {
      if (b + k < b1) {
        r = T[r >> sh] ^ ((r << 8) & mask) ^ v[k];
      }
    }
  }
  return r;
}

// a(x) c(x) mod g for a, c of degree < order (GF(2) multiplication, the reduction folded into the shifts of c);
// polynom includes the x^order term (crc_params).
__device__ __forceinline__ uint32_t crc_mulmod(uint32_t a, uint32_t c, uint32_t order, uint32_t polynom)
{
  const uint32_t mask = (1u << order) - 1u;
  const uint32_t top  = 1u << (order - 1);
  uint32_t       r    = 0;
#pragma unroll
  for (uint32_t i = 0; i < CRC_MAX_ORDER; ++i) {
    if (i < order) {
      r ^= c & (0u - ((a >> i) & 1u));
      const uint32_t hi = c & top;
      c                 = ((c << 1) & mask) ^ (hi ? (polynom & mask) : 0u);
    }
  }
  return r;
}

// x^m mod g from the linear table (table[k] = x^(k + order) mod g).
__device__ __forceinline__ uint32_t crc_xpow(uint32_t m, uint32_t order, const uint32_t* table)
{
  return m < order ? (1u << m) : table[m - order];
}

// XOR of v over the block (result to all threads). `partial`: __shared__, THREADS / 64 words.
template <int THREADS>
__device__ __forceinline__ uint32_t crc_block_xor(uint32_t v, uint32_t* partial)
{
  v = crc_wave_xor(v);
  __syncthreads(); // `partial` may still be read by a previous call
  if ((threadIdx.x & 63) == 0) {
    partial[threadIdx.x >> 6] = v;
  }
  __syncthreads();
  uint32_t crc = 0;
#pragma unroll
  for (int w = 0; w < THREADS / 64; ++w) {
    crc ^= partial[w];
  }
  return crc;
}

// Every thread of the block must call it; returns the CRC of the whole n-bit message to all
// threads. T: the crc_table8_init table (LDS). `partial` is __shared__ storage of THREADS / 64 words.
template <int THREADS, typename Fetch>
__device__ uint32_t block_crc_bytes(const Fetch&    fetch,
                                    uint32_t        n,
                                    uint32_t        order,
                                    uint32_t        polynom,
                                    const uint32_t* table,
                                    const uint32_t* T,
                                    uint32_t*       partial)
{
  const uint32_t nbytes = (n + 7) / 8;
  const uint32_t per    = (nbytes + THREADS - 1) / THREADS;
  const uint32_t b0     = threadIdx.x * per;
  const uint32_t b1     = min(nbytes, b0 + per);
  return crc_block_xor<THREADS>(crc_chunk_contrib(fetch, b0, b1, n, order, polynom, table, T), partial);
}

// Writes the order-bit checksum MSB-first into bits [n, n + order) of a packed MSB-first row, keeping the other
// bits of the touched bytes: every touched byte (at most 4) is loaded before any is written back, so the
// read-modify-write costs one memory round trip instead of one per byte.
__device__ __forceinline__ void attach_crc_bits(uint8_t* row, uint32_t n, uint32_t order, uint32_t crc)
{
  const uint32_t first = n >> 3, last = (n + order - 1) >> 3; // last - first <= 3 (order <= 24)
  uint32_t       bytes[4];
#pragma unroll
  for (uint32_t k = 0; k < 4; ++k) {
    bytes[k] = first + k <= last ? row[first + k] : 0u;
  }
#pragma unroll
  for (uint32_t k = 0; k < 4; ++k) {
    if (first + k <= last) {
      uint32_t byte = bytes[k];
#pragma unroll
      for (uint32_t b = 0; b < 8; ++b) {
        const uint32_t pos = 8 * (first + k) + b;
        if (pos >= n && pos < n + order) {
          const uint32_t mask = 0x80u >> b;
          byte                = (byte & ~mask) | (((crc >> (order - 1 - (pos - n))) & 1u) ? mask : 0u);
        }
      }
      row[first + k] = static_cast<uint8_t>(byte);
    }
  }
}

// Bytes [c0, c0 + n) of a row into LDS, consecutive threads on consecutive words (4-byte loads when the
// source is aligned), every load of a thread issued before its stores.
template <int THREADS>
__device__ __forceinline__ void crc_stage_bytes(uint8_t* dst, const uint8_t* row, uint32_t c0, uint32_t n)
{
  const uint8_t* src = row + c0;
  uint32_t       nw  = (reinterpret_cast<uintptr_t>(src) & 3u) == 0 ? n / 4 : 0;
  constexpr int  U   = 8;
  for (uint32_t w0 = threadIdx.x; w0 < nw; w0 += U * THREADS) {
    uint32_t v[U];
#pragma unroll
    for (int r = 0; r < U; ++r) {
      const uint32_t w = w0 + r * THREADS;
      v[r]             = w < nw ? reinterpret_cast<const uint32_t*>(src)[w] : 0u;
    }
#pragma unroll
    for (int r = 0; r < U; ++r) {
      const uint32_t w = w0 + r * THREADS;
      if (w < nw) {
        reinterpret_cast<uint32_t*>(dst)[w] = v[r];
      }
    }
  }
  for (uint32_t i = 4 * nw + threadIdx.x; i < n; i += THREADS) {
    dst[i] = src[i];
  }
}

struct row_fetch {
  const uint8_t* row;
  __device__ uint32_t operator()(uint32_t j) const { return row[j]; }
};

// byte j of a message whose bytes [first, first + staged) are in LDS
struct lds_chunk_fetch {
  const uint8_t* chunk;
  uint32_t       first;
  __device__ uint32_t operator()(uint32_t j) const { return chunk[j - first]; }
};

} // namespace srs_amd
