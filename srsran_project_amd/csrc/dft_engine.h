// dft_engine.h -- device-side batched DFT building blocks for gfx950.
//
// One workgroup transforms one N-point complex float vector with the
// Stockham autosort formulation (natural order in, natural order out, no bit
// reversal), radix passes R in {2, 3, 4, 8, 16}:
//   pass with radix R after sub-transforms of length Ns (1, R0, R0*R1, ...):
//     butterfly j in [0, N/R): k = j mod Ns
//       v[r] = x[j + r*N/R] * W_{Ns*R}^{r*k}            (twiddle, r = 0..R-1)
//       v    = DFT_R(v)
//       y[(j div Ns)*Ns*R + k + r*Ns] = v[r]
// The first pass reads straight from HBM through a caller-supplied loader
// (which also performs the OFDM subcarrier mapping / CP skip / bf16
// conversion), the last pass writes straight to HBM through a storer (scaling,
// CP insertion, bf16 rounding, subcarrier demapping): the vector crosses HBM
// exactly once each way and LDS only between passes.  For the last pass,
// (j div Ns) = 0, so thread j writes y[j + r*Ns]: consecutive lanes write
// consecutive samples (coalesced).
//
// LDS holds the vector padded by one complex every 16 (index i -> i + i/16):
// the first pass's stride-R writes then spread over all 64 banks.
// Pass twiddles: the base W_N^m of each butterfly comes from a per-size table
// (double-precision values rounded to float, L2-resident), its powers are
// formed in registers; the DFT_R kernels' internal twiddles are compile-time
// constants.
//
// Accuracy: float32 arithmetic with exactly rounded twiddles; the error is that
// of any radix-R float FFT, O(eps * log N) of the RMS (tests state the bound).
#pragma once

#include <type_traits>

#include <hip/hip_runtime.h>

#include <cstdint>
#include <utility>

namespace srs_amd {
namespace dft {

struct cf {
  float x, y;
};

__device__ __forceinline__ cf operator+(cf a, cf b)
{
  return {a.x + b.x, a.y + b.y};
}
__device__ __forceinline__ cf operator-(cf a, cf b)
{
  return {a.x - b.x, a.y - b.y};
}
__device__ __forceinline__ cf cmul(cf a, cf b)
{
  return {a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x};
}
__device__ __forceinline__ cf scale(cf a, float s)
{
  return {a.x * s, a.y * s};
}
// a * (S i)
template <int S>
__device__ __forceinline__ cf mul_si(cf a)
{
  return S > 0 ? cf{-a.y, a.x} : cf{a.y, -a.x};
}

// ---- compile-time twiddles exp(S * 2*pi*i * m / n) ----------------------------
constexpr double PI_D = 3.14159265358979323846264338327950288;

constexpr double taylor_cos(double x)
{
  double term = 1.0, sum = 1.0;
  for (int k = 1; k < 30; ++k) {
    term *= -x * x / ((2.0 * k - 1.0) * (2.0 * k));
    sum += term;
  }
  return sum;
}
constexpr double taylor_sin(double x)
{
  double term = x, sum = x;
  for (int k = 1; k < 30; ++k) {
    term *= -x * x / ((2.0 * k) * (2.0 * k + 1.0));
    sum += term;
  }
  return sum;
}
// angle 2*pi*m/n reduced to [-pi, pi]
constexpr double reduced_angle(long m, long n)
{
  long r = ((m % n) + n) % n;
  if (2 * r > n) {
    r -= n;
  }
  return 2.0 * PI_D * static_cast<double>(r) / static_cast<double>(n);
}
template <int S, long M, long NN>
__device__ __forceinline__ constexpr cf twiddle()
{
  constexpr double a = reduced_angle(M, NN);
  return cf{static_cast<float>(taylor_cos(a)), static_cast<float>(S * taylor_sin(a))};
}

// ---- small DFTs in registers ---------------------------------------------------
template <int R, int S>
struct small_dft;

template <int S>
struct small_dft<1, S> {
  __device__ __forceinline__ static void run(cf*) {}
};

template <int S>
struct small_dft<2, S> {
  __device__ __forceinline__ static void run(cf* v)
  {
    cf a = v[0];
    v[0] = a + v[1];
    v[1] = a - v[1];
  }
};

template <int S>
struct small_dft<3, S> {
  __device__ __forceinline__ static void run(cf* v)
  {
    constexpr float h = 0.866025403784438646763723170752936183f; // sqrt(3)/2
    cf t = v[1] + v[2];
    cf m = {v[0].x - 0.5f * t.x, v[0].y - 0.5f * t.y};
    cf d = v[1] - v[2];
    d    = mul_si<S>(scale(d, h));
    v[0] = v[0] + t;
    v[1] = m + d;
    v[2] = m - d;
  }
};

template <int S>
struct small_dft<4, S> {
  __device__ __forceinline__ static void run(cf* v)
  {
    cf a0 = v[0] + v[2], a1 = v[0] - v[2];
    cf a2 = v[1] + v[3], a3 = mul_si<S>(v[1] - v[3]);
    v[0] = a0 + a2;
    v[2] = a0 - a2;
    v[1] = a1 + a3;
    v[3] = a1 - a3;
  }
};

// Two-level decomposition R = A*B: n = b + B*a, k = k_a + A*k_b.
template <int A, int B, int S>
struct split_dft {
  template <int b, int ka>
  __device__ __forceinline__ static cf tw_ab(cf x)
  {
    if constexpr (b == 0 || ka == 0) {
      return x;
    } else {
      return cmul(x, twiddle<S, static_cast<long>(b) * ka, static_cast<long>(A) * B>());
    }
  }
  template <int b>
  __device__ __forceinline__ static void stage1(cf* v, cf (*y)[A])
  {
    cf u[A];
#pragma unroll
    for (int a = 0; a < A; ++a) {
      u[a] = v[b + B * a];
    }
    small_dft<A, S>::run(u);
    [&]<int... ka>(std::integer_sequence<int, ka...>) { ((y[b][ka] = tw_ab<b, ka>(u[ka])), ...); }
    (std::make_integer_sequence<int, A>{});
  }
  __device__ __forceinline__ static void run(cf* v)
  {
    cf y[B][A];
    [&]<int... b>(std::integer_sequence<int, b...>) { (stage1<b>(v, y), ...); }
    (std::make_integer_sequence<int, B>{});
#pragma unroll
    for (int ka = 0; ka < A; ++ka) {
      cf z[B];
#pragma unroll
      for (int b = 0; b < B; ++b) {
        z[b] = y[b][ka];
      }
      small_dft<B, S>::run(z);
#pragma unroll
      for (int kb = 0; kb < B; ++kb) {
        v[ka + A * kb] = z[kb];
      }
    }
  }
};

template <int S>
struct small_dft<8, S> : split_dft<2, 4, S> {};
template <int S>
struct small_dft<16, S> : split_dft<4, 4, S> {};

// ---- Stockham passes -------------------------------------------------------------
__device__ __forceinline__ int pad(int i)
{
  return i + (i >> 4);
}

template <int N>
constexpr int lds_complex()
{
  return N + N / 16;
}

template <int R, int... Rest>
struct first_of {
  static constexpr int value = R;
};

// w[r] = w1^r, r = 1..R-1, by squarings and one multiply each (error grows
// with the depth, <= 6 products for R = 16).
template <int R>
__device__ __forceinline__ void twiddle_powers(cf w1, cf* w)
{
  w[1] = w1;
#pragma unroll
  for (int r = 2; r < R; ++r) {
    w[r] = (r & 1) ? cmul(w[r - 1], w1) : cmul(w[r / 2], w[r / 2]);
  }
}

// First-pass input held in registers: thread t's samples t + T r, r < K (plans whose first pass has N / R = T
// butterflies, one per thread); passed as the engine's Load.
template <int K>
struct reg_input {
  cf v[K];
};
template <class L>
struct is_reg_input : std::false_type {};
template <int K>
struct is_reg_input<reg_input<K>> : std::true_type {};

// Runs the passes Rs... over one N-point vector with T threads.
//   load(i)       -> cf  : input sample i (first pass only)
//   store(i, v)          : output sample i (last pass only)
//   tw                   : table W_N^m = exp(-2*pi*i*m/N), m in [0, N) (conjugated for S = +1)
// Each butterfly of a later pass needs W_{Ns*R}^{r*k}, r = 1..R-1: only the
// base W_{Ns*R}^k is read from the table -- one HBM/L2 load per butterfly,
// issued a whole pass ahead so its latency hides behind the previous pass --
// and the powers are formed in registers.
template <int N, int T, int S, int... Rs>
struct stockham {
  template <int Ns, int R>
  static constexpr int per()
  {
    return N / R / T;
  }

  // G: the workgroup may hold more than T threads; threads T.. only take part in the barriers
  template <bool G, int Ns, int R, int... Rest, class Load, class Store>
  __device__ __forceinline__ static void pass(cf* lds, const cf* tw, Load& load, Store& store, const cf* wbase)
  {
    constexpr int  NB    = N / R;           // butterflies in this pass
    constexpr int  PER   = NB / T;          // butterflies per thread
    constexpr bool FIRST = Ns == 1;
    constexpr bool LAST  = sizeof...(Rest) == 0;
    static_assert(NB % T == 0, "butterflies must divide evenly over the threads");
    const int  tid = threadIdx.x;
    const bool act = !G || tid < T;

    // prefetch the next pass's twiddle bases
    constexpr int R2   = LAST ? 1 : first_of<Rest..., 1>::value;
    constexpr int Ns2  = Ns * R;
    constexpr int PER2 = LAST ? 1 : N / R2 / T;
    cf            wnext[PER2];
    if constexpr (!LAST) {
#pragma unroll
      for (int b = 0; b < PER2; ++b) {
        const int j2 = tid + b * T;
        wnext[b]     = act ? tw[(j2 % Ns2) * (N / (Ns2 * R2))] : cf{1, 0};
      }
    }

    cf v[PER][R];
#pragma unroll
    for (int b = 0; b < PER; ++b) {
      const int j = tid + b * T;
#pragma unroll
      for (int r = 0; r < R; ++r) {
        if constexpr (FIRST && is_reg_input<Load>::value) {
          static_assert(PER == 1, "register input needs one first-pass butterfly per thread");
          v[b][r] = load.v[r];
        } else if constexpr (FIRST) {
          v[b][r] = act ? load(j + r * NB) : cf{0, 0};
        } else {
          v[b][r] = act ? lds[pad(j + r * NB)] : cf{0, 0};
        }
      }
    }
#pragma unroll
    for (int b = 0; b < PER; ++b) {
      if constexpr (!FIRST) {
        cf w1 = wbase[b];
        if (S > 0) {
          w1.y = -w1.y;
        }
        cf w[R];
        twiddle_powers<R>(w1, w);
#pragma unroll
        for (int r = 1; r < R; ++r) {
          v[b][r] = cmul(v[b][r], w[r]);
        }
      }
      small_dft<R, S>::run(v[b]);
    }
    if constexpr (LAST) {
#pragma unroll
      for (int b = 0; b < PER; ++b) {
        const int j = tid + b * T; // j < Ns here
#pragma unroll
        for (int r = 0; r < R; ++r) {
          if (act) {
            store(j + r * Ns, v[b][r]);
          }
        }
      }
    } else {
      if constexpr (!FIRST) {
        __syncthreads(); // everyone has read this pass's input
      }
#pragma unroll
      for (int b = 0; b < PER; ++b) {
        const int j    = tid + b * T;
        const int k    = j % Ns;
        const int base = (j / Ns) * Ns * R + k;
#pragma unroll
        for (int r = 0; r < R; ++r) {
          if (act) {
            lds[pad(base + r * Ns)] = v[b][r];
          }
        }
      }
      __syncthreads();
      pass<G, Ns * R, Rest...>(lds, tw, load, store, wnext);
    }
  }

  template <class Load, class Store>
  __device__ __forceinline__ static void run(cf* lds, const cf* tw, Load& load, Store& store)
  {
    pass<false, 1, Rs...>(lds, tw, load, store, nullptr);
  }
  // the same transform in a workgroup of more than T threads (all of them reach this call)
  template <class Load, class Store>
  __device__ __forceinline__ static void run_guarded(cf* lds, const cf* tw, Load& load, Store& store)
  {
    pass<true, 1, Rs...>(lds, tw, load, store, nullptr);
  }
};

// Plans: threads per transform and radix sequence for each supported size.
template <int N>
struct plan;
#define SRS_DFT_PLAN(NN, TT, ...)                                                                                      \
  template <>                                                                                                          \
  struct plan<NN> {                                                                                                    \
    static constexpr int T = TT;                                                                                       \
    template <int S>                                                                                                   \
    using engine = stockham<NN, TT, S, __VA_ARGS__>;                                                                   \
  };
SRS_DFT_PLAN(128, 32, 4, 4, 4, 2)
SRS_DFT_PLAN(256, 64, 4, 4, 4, 4)
SRS_DFT_PLAN(384, 32, 4, 4, 4, 2, 3)
SRS_DFT_PLAN(512, 64, 8, 8, 8)
SRS_DFT_PLAN(768, 64, 4, 4, 4, 4, 3)
SRS_DFT_PLAN(1024, 64, 16, 16, 4)
SRS_DFT_PLAN(1536, 64, 8, 8, 8, 3)
SRS_DFT_PLAN(2048, 128, 16, 16, 8)
SRS_DFT_PLAN(3072, 256, 4, 4, 4, 4, 4, 3)
SRS_DFT_PLAN(4096, 256, 16, 16, 16)
SRS_DFT_PLAN(6144, 256, 8, 8, 8, 4, 3)
SRS_DFT_PLAN(8192, 256, 16, 16, 16, 2)
#undef SRS_DFT_PLAN

// Sizes with a plan, in the order used by the host dispatch tables.
#define SRS_DFT_FOR_EACH_SIZE(X) X(128) X(256) X(384) X(512) X(768) X(1024) X(1536) X(2048) X(3072) X(4096) X(6144) X(8192)

} // namespace dft
} // namespace srs_amd
