// Issue cost of single VALU opcodes on gfx950, per SIMD, at 8 waves per SIMD with 8 independent chains per lane
// (throughput form), plus the wave-count sweep of a few opcodes.  r06: v_pk_*_i16 and v_max_i32 / v_mad_u32_u24
// measured ~1.75x the cost of v_add_u32 (tools/valu_rate_probe.hip, profiles/r06_valu_rate.txt), so the issue cost of
// the LDPC decoders depends on the opcode mix, not on the packed form alone.
//   hipcc --offload-arch=gfx950 -O3 tools/valu_rate_probe.hip -o tools/_build/valu_rate_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

#define CHECK(x)                                                                                                       \
  do {                                                                                                                 \
    hipError_t e_ = (x);                                                                                               \
    if (e_ != hipSuccess) {                                                                                            \
      std::printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__);                                          \
      return 1;                                                                                                        \
    }                                                                                                                  \
  } while (0)

constexpr int ITERS = 2048;

// one kernel per opcode: INSN is the instruction text with %0 the chain register (read and written), %1 and %2 two
// loop-invariant registers
#define RATE_KERNEL(NAME, INSN)                                                                                        \
  template <int CH>                                                                                                    \
  __global__ void __launch_bounds__(256) NAME(uint32_t* out, uint32_t seed)                                            \
  {                                                                                                                    \
    uint32_t a[8];                                                                                                     \
    _Pragma("unroll") for (int i = 0; i < 8; ++i) { a[i] = seed * (threadIdx.x + 1) + i; }                            \
    const uint32_t b = seed ^ threadIdx.x, c = seed + threadIdx.x;                                                     \
    for (int it = 0; it < ITERS; ++it) {                                                                               \
      _Pragma("unroll") for (int r = 0; r < 8 / CH; ++r)                                                               \
      {                                                                                                                \
        _Pragma("unroll") for (int i = 0; i < CH; ++i) { asm volatile(INSN : "+v"(a[i]) : "v"(b), "v"(c)); }           \
      }                                                                                                                \
    }                                                                                                                  \
    uint32_t s = 0;                                                                                                    \
    _Pragma("unroll") for (int i = 0; i < 8; ++i) { s ^= a[i]; }                                                       \
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;                                                                    \
  }

RATE_KERNEL(k_add_u32, "v_add_u32 %0, %0, %1")
RATE_KERNEL(k_max_i32, "v_max_i32 %0, %0, %1")
RATE_KERNEL(k_max_i16, "v_max_i16 %0, %0, %1")
RATE_KERNEL(k_min_i16, "v_min_i16 %0, %0, %1")
RATE_KERNEL(k_max_u16, "v_max_u16 %0, %0, %1")
RATE_KERNEL(k_min_u16, "v_min_u16 %0, %0, %1")
RATE_KERNEL(k_sub_u16, "v_sub_u16 %0, %0, %1")
RATE_KERNEL(k_subrev_u16, "v_subrev_u16 %0, %0, %1")
RATE_KERNEL(k_lshlrev_b16, "v_lshlrev_b16 %0, 1, %0")
RATE_KERNEL(k_lshrrev_b16, "v_lshrrev_b16 %0, 1, %0")
RATE_KERNEL(k_ashrrev_i16, "v_ashrrev_i16 %0, 1, %0")
RATE_KERNEL(k_lshrrev_b32, "v_lshrrev_b32 %0, 1, %0")
RATE_KERNEL(k_lshlrev_b32, "v_lshlrev_b32 %0, 1, %0")
RATE_KERNEL(k_min_i32, "v_min_i32 %0, %0, %1")
RATE_KERNEL(k_max_u32, "v_max_u32 %0, %0, %1")
RATE_KERNEL(k_sub_i32, "v_sub_i32 %0, %0, %1")
RATE_KERNEL(k_mad_i16, "v_mad_i16 %0, %0, %1, %2")
RATE_KERNEL(k_mad_u16, "v_mad_u16 %0, %0, %1, %2")
RATE_KERNEL(k_med3_i16, "v_med3_i16 %0, %0, %1, %2")
RATE_KERNEL(k_max3_i16, "v_max3_i16 %0, %0, %1, %2")
RATE_KERNEL(k_mul_lo_u16, "v_mul_lo_u16 %0, %0, %1")
RATE_KERNEL(k_bitop3_b32, "v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96")
RATE_KERNEL(k_or3_b32, "v_or3_b32 %0, %0, %1, %2")
RATE_KERNEL(k_bfi_b32, "v_bfi_b32 %0, %0, %1, %2")
RATE_KERNEL(k_alignbyte, "v_alignbyte_b32 %0, %0, %1, 1")
RATE_KERNEL(k_lshl_add_u32, "v_lshl_add_u32 %0, %0, 1, %1")
RATE_KERNEL(k_pk_min_u16, "v_pk_min_u16 %0, %0, %1")
RATE_KERNEL(k_pk_sub_u16, "v_pk_sub_u16 %0, %0, %1")
RATE_KERNEL(k_min_f32, "v_min_f32 %0, %0, %1")
RATE_KERNEL(k_mul_f32, "v_mul_f32 %0, %0, %1")
RATE_KERNEL(k_sub_f16, "v_sub_f16 %0, %0, %1")
RATE_KERNEL(k_max_f16, "v_max_f16 %0, %0, %1")
RATE_KERNEL(k_pk_max_f16, "v_pk_max_f16 %0, %0, %1")
RATE_KERNEL(k_pk_add_f16, "v_pk_add_f16 %0, %0, %1")
RATE_KERNEL(k_cmp_cnd, "v_cmp_gt_i32 vcc, %0, %1\n\tv_cndmask_b32 %0, %0, %1, vcc")
RATE_KERNEL(k_cmp_lt, "v_cmp_lt_i32 vcc, %0, %1")
RATE_KERNEL(k_cnd_s, "v_cndmask_b32_e64 %0, %0, %1, s[40:41]")
RATE_KERNEL(k_mix_pk_xor, "v_pk_max_i16 %0, %0, %1\n\tv_xor_b32 %0, %0, %2")
RATE_KERNEL(k_mix_pk_add, "v_pk_max_i16 %0, %0, %1\n\tv_add_u32 %0, %0, %2")
RATE_KERNEL(k_mix_maxi16_xor, "v_max_i16 %0, %0, %1\n\tv_xor_b32 %0, %0, %2")
RATE_KERNEL(k_mix_pk2_xor2, "v_pk_max_i16 %0, %0, %1\n\tv_pk_min_i16 %0, %0, %2\n\tv_xor_b32 %0, %0, %2\n\tv_add_u32 %0, %0, %1")

template <typename K>
static int run(K kernel, const char* name, int waves_per_simd, int cus, int ch)
{
  // one 256-thread workgroup = 4 waves, one per SIMD; waves_per_simd workgroups per CU
  const int blocks = cus * waves_per_simd;
  uint32_t* out;
  CHECK(hipMalloc(&out, sizeof(uint32_t) * blocks * 256));
  hipLaunchKernelGGL(kernel, dim3(blocks), dim3(256), 0, 0, out, 7u);
  CHECK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  CHECK(hipEventRecord(e0));
  for (int r = 0; r < 3; ++r) {
    hipLaunchKernelGGL(kernel, dim3(blocks), dim3(256), 0, 0, out, 9u);
  }
  CHECK(hipEventRecord(e1));
  CHECK(hipEventSynchronize(e1));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  ms /= 3;
  const double wave_insts_per_simd = static_cast<double>(ITERS) * 8 * waves_per_simd;
  const double ns                  = ms * 1e6 / wave_insts_per_simd;
  std::printf("%-18s ch=%d waves/SIMD=%d  %.3f ns per wave-instruction per SIMD\n", name, ch, waves_per_simd, ns);
  CHECK(hipFree(out));
  CHECK(hipEventDestroy(e0));
  CHECK(hipEventDestroy(e1));
  return 0;
}

#define RUN(K, W, CH) run(K<CH>, #K, W, cus, CH)

int main()
{
  hipDeviceProp_t p;
  if (hipGetDeviceProperties(&p, 0) != hipSuccess) {
    return 1;
  }
  const int cus = p.multiProcessorCount;
  std::printf("%s, %d CUs\n", p.gcnArchName, cus);
  for (int w : {8}) {
    RUN(k_add_u32, w, 8);
    RUN(k_max_i32, w, 8);
    RUN(k_max_i16, w, 8);
    RUN(k_min_i16, w, 8);
    RUN(k_max_u16, w, 8);
    RUN(k_min_u16, w, 8);
    RUN(k_sub_u16, w, 8);
    RUN(k_subrev_u16, w, 8);
    RUN(k_lshlrev_b16, w, 8);
    RUN(k_lshrrev_b16, w, 8);
    RUN(k_ashrrev_i16, w, 8);
    RUN(k_lshrrev_b32, w, 8);
    RUN(k_lshlrev_b32, w, 8);
    RUN(k_min_i32, w, 8);
    RUN(k_max_u32, w, 8);
    RUN(k_sub_i32, w, 8);
    RUN(k_mad_i16, w, 8);
    RUN(k_mad_u16, w, 8);
    RUN(k_med3_i16, w, 8);
    RUN(k_max3_i16, w, 8);
    RUN(k_mul_lo_u16, w, 8);
    RUN(k_bitop3_b32, w, 8);
    RUN(k_or3_b32, w, 8);
    RUN(k_bfi_b32, w, 8);
    RUN(k_alignbyte, w, 8);
    RUN(k_lshl_add_u32, w, 8);
    RUN(k_pk_min_u16, w, 8);
    RUN(k_pk_sub_u16, w, 8);
    RUN(k_min_f32, w, 8);
    RUN(k_mul_f32, w, 8);
    RUN(k_sub_f16, w, 8);
    RUN(k_max_f16, w, 8);
    RUN(k_pk_max_f16, w, 8);
    RUN(k_pk_add_f16, w, 8);
    RUN(k_cmp_cnd, w, 8);
    RUN(k_cmp_lt, w, 8);
    RUN(k_cnd_s, w, 8);
    RUN(k_mix_pk_xor, w, 8);
    RUN(k_mix_pk_add, w, 8);
    RUN(k_mix_maxi16_xor, w, 8);
    RUN(k_mix_pk2_xor2, w, 8);
  }
  return 0;
}
