// gold_sequence.h -- TS 38.211 5.2.1 pseudo-random (Gold) sequence at any
// offset, shared by the scrambling, PDSCH modulator and DM-RS kernels.
//
// c(n) = x1(n + 1600) ^ x2(n + 1600); the two 31-bit LFSR states are jumped to
// n + 1600 with the GF(2) matrices A^(2^k) (columns, built once on the host by
// gold_jump_tables()), then advanced 32 bits at a time with word-parallel shifts (gold_next32).  Same sequence as
// lib/phy/upper/sequence_generators/pseudo_random_generator_impl.cpp.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <vector>

namespace srs_amd {

constexpr int PRBS_NJUMP = 24; // jumps by 2^k, k < 24 (sequences up to 2^24 - 1600 bits)

constexpr int PRBS_RADIX_DIGITS = 6;                        // 4-bit digits of a jump (24 bits)
constexpr int PRBS_RADIX_OFF    = 2 * PRBS_NJUMP * 31;      // start of the radix-16 matrices

// Nibble tables of the binary matrices A^(2^k), k = PRBS_NIB_K0 .. PRBS_NIB_K0 + PRBS_NIB_NK - 1: entry [q][v] =
// M x (v << 4 q), so a product is eight table reads and seven XORs (gf2_apply_nib) instead of 31 masked XORs.
constexpr int PRBS_NIB_K0  = 5;
constexpr int PRBS_NIB_NK  = 7;
constexpr int PRBS_NIB_OFF = PRBS_RADIX_OFF + 2 * PRBS_RADIX_DIGITS * 16 * 31;

// [2][PRBS_NJUMP][31] jump matrices A^(2^k) (columns), x1 then x2, followed by the radix-16 matrices
// [2][PRBS_RADIX_DIGITS][16][31] A^(d 16^k) (d = 0 unused) and the nibble tables [2][PRBS_NIB_NK][8][16].
std::vector<uint32_t> gold_jump_tables();

// Word basis of the sequence from its start: c is linear in c_init, so word w (bits c(32 w .. 32 w + 31)) of any c_init
// is row 31 (the x1 part) XOR the rows j < 31 of the set bits j of c_init (x2 from c_init = 2^j), table
// [32][GOLD_BASIS_WORDS].  A word then costs 32 independent loads instead of a chain of dependent jump-ahead products.
constexpr uint32_t GOLD_BASIS_WORDS = 224; // bits 0 .. 7,167 (a DM-RS symbol's last pilot bit: 12 x 274 + 2 x 1,650)
std::vector<uint32_t> gold_word_basis();

__device__ __forceinline__ uint32_t gold_basis_word(const uint32_t* basis, uint32_t c_init, uint32_t w)
{
  uint32_t t[32];
#pragma unroll
  for (int j = 0; j < 32; ++j) {
    t[j] = basis[j * GOLD_BASIS_WORDS + w]; // every load issued before the first use
  }
  uint32_t r = t[31];
#pragma unroll
  for (int j = 0; j < 31; ++j) {
    r ^= t[j] & (0u - ((c_init >> j) & 1u));
  }
  return r;
}

// state' = M * state over GF(2), M given by its 31 columns.
__device__ __forceinline__ uint32_t gf2_apply(const uint32_t* cols, uint32_t state)
{
  uint32_t r = 0;
#pragma unroll
  for (int j = 0; j < 31; ++j) {
    r ^= cols[j] & (0u - ((state >> j) & 1u));
  }
  return r;
}

// LFSR states advanced by `steps` positions (steps < 2^PRBS_NJUMP): one matrix-vector product per
// set bit of steps.
__device__ __forceinline__ void gold_advance(const uint32_t* jump, uint32_t steps, uint32_t& x1, uint32_t& x2)
{
  for (int k = 0; k < PRBS_NJUMP; ++k) {
    if ((steps >> k) & 1u) {
      x1 = gf2_apply(jump + (0 * PRBS_NJUMP + k) * 31, x1);
      x2 = gf2_apply(jump + (1 * PRBS_NJUMP + k) * 31, x2);
    }
  }
}

// LFSR states advanced by `steps` (< 2^24) positions: one product per non-zero 4-bit digit (half the
// products of the binary decomposition).
__device__ __forceinline__ void gold_advance16(const uint32_t* jump, uint32_t steps, uint32_t& x1, uint32_t& x2)
{
  const uint32_t* r = jump + PRBS_RADIX_OFF;
  for (int k = 0; k < PRBS_RADIX_DIGITS; ++k) {
    const uint32_t d = (steps >> (4 * k)) & 15u;
    if (d != 0) {
      x1 = gf2_apply(r + ((0 * PRBS_RADIX_DIGITS + k) * 16 + d) * 31, x1);
      x2 = gf2_apply(r + ((1 * PRBS_RADIX_DIGITS + k) * 16 + d) * 31, x2);
    }
  }
}

// States whose next output is c(n0).
__device__ __forceinline__ void gold_state(const uint32_t* jump, uint32_t c_init, uint32_t n0, uint32_t& x1,
                                           uint32_t& x2)
{
  x1 = 1u;
  x2 = c_init & 0x7fffffffu;
  gold_advance16(jump, n0 + 1600u, x1, x2);
}

// The next 32 outputs from the states (the b-th output at bit b), word-parallel: with the state
// s = x(n .. n+30) in bits 0..30, x1(n+31+i) = x1(n+3+i) ^ x1(n+i) gives 28 new bits in one shift/xor
// (x2: taps 3, 2, 1, 0), a second round the next 4; the states advance by 32.
__device__ __forceinline__ uint32_t gold_next32(uint32_t& x1, uint32_t& x2)
{
  uint64_t a = x1;
  a |= static_cast<uint64_t>(((a >> 3) ^ a) & 0x0fffffffu) << 31;
  a |= static_cast<uint64_t>(((a >> 31) ^ (a >> 28)) & 0xfu) << 59;
  uint64_t b = x2;
  b |= static_cast<uint64_t>(((b >> 3) ^ (b >> 2) ^ (b >> 1) ^ b) & 0x0fffffffu) << 31;
  b |= static_cast<uint64_t>(((b >> 31) ^ (b >> 30) ^ (b >> 29) ^ (b >> 28)) & 0xfu) << 59;
  x1 = static_cast<uint32_t>(a >> 32) & 0x7fffffffu;
  x2 = static_cast<uint32_t>(b >> 32) & 0x7fffffffu;
  return static_cast<uint32_t>(a ^ b);
}

__device__ __forceinline__ uint32_t gold_emit32(uint32_t x1, uint32_t x2)
{
  return gold_next32(x1, x2);
}

// 32 sequence bits c(n0 .. n0+31), c(n0 + b) at bit b.
__device__ inline uint32_t gold_word(const uint32_t* jump, uint32_t c_init, uint32_t n0)
{
  uint32_t x1, x2;
  gold_state(jump, c_init, n0, x1, x2);
  return gold_emit32(x1, x2);
}

// States whose next output is c(n_wave + off), n_wave the same for every lane of the wave: the jump
// to n_wave runs once per wave on the scalar unit (readfirstlane makes its inputs uniform), each lane
// then applies one product per non-zero 4-bit digit of its own offset.
__device__ __forceinline__ void gold_state_wave(const uint32_t* jump, uint32_t c_init, uint32_t n_wave, uint32_t off,
                                                uint32_t& x1, uint32_t& x2)
{
  gold_state(jump, __builtin_amdgcn_readfirstlane(c_init), __builtin_amdgcn_readfirstlane(n_wave), x1, x2);
  gold_advance16(jump, off, x1, x2);
}

// state' = A^(2^k) x state (k in [PRBS_NIB_K0, PRBS_NIB_K0 + PRBS_NIB_NK)) by its nibble table.
__device__ __forceinline__ uint32_t gf2_apply_nib(const uint32_t* jump, int which, int k, uint32_t state)
{
  const uint32_t* t = jump + PRBS_NIB_OFF + ((which * PRBS_NIB_NK + (k - PRBS_NIB_K0)) * 8) * 16;
  uint32_t        r = 0;
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    r ^= t[q * 16 + ((state >> (4 * q)) & 15u)];
  }
  return r;
}

// States whose next output is c(n_wave + 32 lane), n_wave the same for every lane of the wave: the jump to n_wave on
// the scalar unit, then the lane's offset by doubling rounds over bits 0..5 of lane with the nibble tables of
// A^(32 2^k) (eight reads of one 64-byte row per product, the same matrix in every lane).
__device__ __forceinline__ void gold_state_lanes(const uint32_t* jump, uint32_t c_init, uint32_t n_wave, uint32_t lane,
                                                 uint32_t& x1, uint32_t& x2)
{
  gold_state(jump, __builtin_amdgcn_readfirstlane(c_init), __builtin_amdgcn_readfirstlane(n_wave), x1, x2);
#pragma unroll
  for (int k = 0; k < 6; ++k) {
    const uint32_t y1 = gf2_apply_nib(jump, 0, 5 + k, x1);
    const uint32_t y2 = gf2_apply_nib(jump, 1, 5 + k, x2);
    const bool     b  = ((lane >> k) & 1u) != 0;
    x1                = b ? y1 : x1;
    x2                = b ? y2 : x2;
  }
}

// States advanced by 2^k positions (k in [PRBS_NIB_K0, PRBS_NIB_K0 + PRBS_NIB_NK), the same k in every lane).
__device__ __forceinline__ void gold_advance_pow2(const uint32_t* jump, int k, uint32_t& x1, uint32_t& x2)
{
  x1 = gf2_apply_nib(jump, 0, k, x1);
  x2 = gf2_apply_nib(jump, 1, k, x2);
}

} // namespace srs_amd
