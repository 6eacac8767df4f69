// Dense products for nn.Linear layers on the hot path (BiLSTM output projection,
// model/model.py:157,162; CTC head) and their gradients, on the
// shared MFMA GEMM core.
#include "gemm.hpp"
#include "gemm256.hpp"
#include "crnn_internal.hpp"

using namespace gemm;

namespace {

template <typename T, bool ROW8 = false> struct OutEpi {
  static constexpr bool kStats = false;
  // ROW8 (CRNN_OPT_LINEAR_ROW8, 256-row kernel only): the accumulators go through the wave's LDS and a lane
  // stores 8 consecutive columns (one 16-B bf16 store, gemm256.hpp row8_epilogue) instead of 4
  static constexpr bool kRow8 = ROW8;
  void* c;
  int ldc, M, N, c_f32, accumulate, atomic;
  const float* bias;
  __device__ __forceinline__ void store(int m, int n, f32x4 v, int kz) const {
    if (m >= M || n >= N) return;
    if (bias && (!atomic || kz == 0)) {   // split-K partials: the bias once, with the first K split
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] += (n + r < N) ? bias[n + r] : 0.f;
    }
    size_t o = (size_t)m * ldc + n;
    if (c_f32) {
      float* p = (float*)c + o;
      if (atomic) {
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (n + r < N) atomicAdd(p + r, v[r]);
        return;
      }
      if (n + 4 <= N && (ldc % 4) == 0) {
        if (accumulate) v += *reinterpret_cast<const f32x4*>(p);
        *reinterpret_cast<f32x4*>(p) = v;
      } else {
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (n + r < N) p[r] = accumulate ? p[r] + v[r] : v[r];
      }
    } else {
      T* p = (T*)c + o;
      if (n + 4 <= N && (ldc % 4) == 0) {
        if (accumulate) v += ld4f<T>(p);
        st4<T>(p, v);
      } else {
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (n + r < N) p[r] = fromf<T>(accumulate ? tof(p[r]) + v[r] : v[r]);
      }
    }
  }
  // 8 consecutive columns n..n+7 of row m (the same per-element arithmetic as two store() calls)
  __device__ __forceinline__ void store8(int m, int n, f32x4 lo, f32x4 hi, int kz) const {
    if constexpr (sizeof(T) == 2) {
      if (!c_f32 && !atomic && n + 8 <= N && (ldc % 8) == 0) {
        if (m >= M) return;
        if (bias) {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            lo[r] += bias[n + r];
            hi[r] += bias[n + 4 + r];
          }
        }
        T* p = (T*)c + (size_t)m * ldc + n;
        if (accumulate) {
          lo += ld4f<T>(p);
          hi += ld4f<T>(p + 4);
        }
        bf16x8 v;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          v[r] = (bf16)lo[r];
          v[4 + r] = (bf16)hi[r];
        }
        *reinterpret_cast<bf16x8*>(p) = v;
        return;
      }
    }
    store(m, n, lo, kz);
    store(m, n + 4, hi, kz);
  }
  __device__ __forceinline__ void stats(int, int, f32x4, f32x4) const {}
};

// DEEP = false: the register-staged kernels only (loaders without an LDS-DMA form, gemm::Bf16Of)
template <typename T, bool DEEP = true, class LA, class LB>
int run(const LA& la, const LB& lb, const OutEpi<T>& ep, int M, int N, int K, int splits, hipStream_t st) {
  long work = (long)M * N;
  if constexpr (sizeof(T) == 2 && DEEP) {
    // the deep 256-row kernel when the grid alone fills most CUs (no split-K for these outputs)
    const long cu = crnn_cu_count();
    if (crnn_option(CRNN_OPT_DEEP_LINEAR) && splits == 1 && K >= 256) {
      const long t256 = (long)((M + 255) / 256) * ((N + 255) / 256);
      const long t128 = (long)((M + 255) / 256) * ((N + 127) / 128);
      const OutEpi<T, true> ep8{ep.c, ep.ldc, ep.M, ep.N, ep.c_f32, ep.accumulate, ep.atomic, ep.bias};
      // 16-B row stores need a 16-B aligned C and row pitch (a view offset by 4 elements is only 8-B aligned)
      const bool row8 = crnn_option(CRNN_OPT_LINEAR_ROW8) != 0 && ep.ldc % 8 == 0 && ((uintptr_t)ep.c & 15) == 0;
      if (N >= 256 && t256 * 4 >= cu * 3)
        return row8 ? launch256<256, 256>(la, lb, ep8, M, N, K, st) : launch256<256, 256>(la, lb, ep, M, N, K, st);
      if (N >= 128 && t128 * 4 >= cu * 3)
        return row8 ? launch256<256, 128>(la, lb, ep8, M, N, K, st) : launch256<256, 128>(la, lb, ep, M, N, K, st);
    }
  }
  if (M >= 128 && N >= 128 && work >= 128L * 128 * 128) return launch<T, 128, 128>(la, lb, ep, M, N, K, splits, st);
  if (work >= 64L * 64 * 128) return launch<T, 64, 64>(la, lb, ep, M, N, K, splits, st);
  return launch<T, 32, 32>(la, lb, ep, M, N, K, splits, st);
}

template <typename T>
int gemm_nt_t(const void* A, int lda, const void* B, int ldb, void* C, int ldc, const float* bias, int M, int N, int K,
              int c_f32, int acc, hipStream_t st) {
  RowMajorK<T> la{(const T*)A, lda, M, K};
  RowMajorK<T> lb{(const T*)B, ldb, N, K};
  OutEpi<T> ep{C, ldc, M, N, c_f32, acc, 0, bias};
  return run<T>(la, lb, ep, M, N, K, 1, st);
}

template <typename T>
int gemm_nn_t(const void* A, int lda, const void* B, int ldb, void* C, int ldc, int M, int N, int K, int c_f32, int acc,
              hipStream_t st) {
  RowMajorK<T> la{(const T*)A, lda, M, K};
  ColMajorK<T> lb{(const T*)B, ldb, N, K};
  OutEpi<T> ep{C, ldc, M, N, c_f32, acc, 0, nullptr};
  return run<T>(la, lb, ep, M, N, K, 1, st);
}

template <typename T>
int gemm_tn_t(const void* A, int lda, const void* B, int ldb, float* C, int ldc, int M, int N, int K, int acc,
              hipStream_t st) {
  ColMajorK<T> la{(const T*)A, lda, M, K};
  ColMajorK<T> lb{(const T*)B, ldb, N, K};
  int b = (M >= 128 && N >= 128) ? 128 : (M >= 64 && N >= 64 ? 64 : 32);
  long tiles = (long)((M + b - 1) / b) * ((N + b - 1) / b);
  long want = (512 + tiles - 1) / tiles;
  long maxs = (K + 4 * BK - 1) / (4 * BK);
  if (want > maxs) want = maxs;
  if (want < 1) want = 1;
  int splits = eff_splits(K, (int)want);
  if (splits > 1 && !acc) {
    for (int m = 0; m < 1; ++m) {
      hipError_t e = ldc == N ? hipMemsetAsync(C, 0, (size_t)M * N * sizeof(float), st)
                              : hipMemset2DAsync(C, (size_t)ldc * sizeof(float), 0, (size_t)N * sizeof(float), M, st);
      if (e != hipSuccess) return (int)e;
    }
  }
  OutEpi<T> ep{C, ldc, M, N, 1, acc, splits > 1 ? 1 : 0, nullptr};
  if (b == 128) return launch<T, 128, 128>(la, lb, ep, M, N, K, splits, st);
  if (b == 64) return launch<T, 64, 64>(la, lb, ep, M, N, K, splits, st);
  return launch<T, 32, 32>(la, lb, ep, M, N, K, splits, st);
}

// CRNN_F32_BF16MMA: fp32 operands in memory, staged as bf16 (gemm::Bf16Of), bf16 MFMA, fp32 accumulation and
// fp32 output — the attention decoder's training GEMMs (the reference's fp16 autocast, training/train.py:499)
// The decoder's per-step products are small (M = batch: 256 x 1280 x 1024 and 256 x 1024 x 1280 per step): one
// K-serial tile per workgroup, and the fp32 operands cost twice the bytes of bf16 ones. Measured on the MI355X
// (profiles/r06/r06w_gemm_mix_plans.log, us for nn / nt): 32 x 32 tiles with 128-deep stages 12.4 / 12.9, the same
// with 64-deep stages 13.5 / 15.5, 256-deep 15.4 / 12.4, 64 x 64 x 128 13.8 / 13.6, 64 x 64 x 256 12.7 / 12.8;
// split-K with fp32 atomics ~20 (and not bit-reproducible); bf16 operands on the LDS-DMA kernels 8.0 / 7.5;
// hipBLASLt bf16 19.1 / 19.8. The 256^3 products stay on the default plan (~4 us, launch-bound).
template <class LA, class LB>
int run_mix(const LA& la, const LB& lb, void* C, int ldc, const float* bias, int M, int N, int K, int acc,
            hipStream_t st) {
  const OutEpi<bf16> ep{C, ldc, M, N, 1, acc, 0, bias};
  const long t64 = (long)((M + 63) / 64) * ((N + 63) / 64);
  if (t64 >= 2 * crnn_cu_count() || K < 512) return run<bf16, false>(la, lb, ep, M, N, K, 1, st);
  return launch<bf16, 32, 32, 128>(la, lb, ep, M, N, K, 1, st);
}

int gemm_nt_mix(const void* A, int lda, const void* B, int ldb, void* C, int ldc, const float* bias, int M, int N,
                int K, int acc, hipStream_t st) {
  Bf16Of<RowMajorK<float>> la{RowMajorK<float>{(const float*)A, lda, M, K}};
  Bf16Of<RowMajorK<float>> lb{RowMajorK<float>{(const float*)B, ldb, N, K}};
  return run_mix(la, lb, C, ldc, bias, M, N, K, acc, st);
}

int gemm_nn_mix(const void* A, int lda, const void* B, int ldb, void* C, int ldc, int M, int N, int K, int acc,
                hipStream_t st) {
  Bf16Of<RowMajorK<float>> la{RowMajorK<float>{(const float*)A, lda, M, K}};
  Bf16Of<ColMajorK<float>> lb{ColMajorK<float>{(const float*)B, ldb, N, K}};
  return run_mix(la, lb, C, ldc, nullptr, M, N, K, acc, st);
}

int gemm_tn_mix(const void* A, int lda, const void* B, int ldb, float* C, int ldc, int M, int N, int K, int acc,
                hipStream_t st) {
  Bf16Of<ColMajorK<float>> la{ColMajorK<float>{(const float*)A, lda, M, K}};
  Bf16Of<ColMajorK<float>> lb{ColMajorK<float>{(const float*)B, ldb, N, K}};
  int b = (M >= 128 && N >= 128) ? 128 : (M >= 64 && N >= 64 ? 64 : 32);
  long tiles = (long)((M + b - 1) / b) * ((N + b - 1) / b);
  long want = (512 + tiles - 1) / tiles;
  long maxs = (K + 4 * BK - 1) / (4 * BK);
  if (want > maxs) want = maxs;
  if (want < 1) want = 1;
  int splits = eff_splits(K, (int)want);
  if (splits > 1 && !acc) {
    hipError_t e = ldc == N ? hipMemsetAsync(C, 0, (size_t)M * N * sizeof(float), st)
                            : hipMemset2DAsync(C, (size_t)ldc * sizeof(float), 0, (size_t)N * sizeof(float), M, st);
    if (e != hipSuccess) return (int)e;
  }
  OutEpi<bf16> ep{C, ldc, M, N, 1, acc, splits > 1 ? 1 : 0, nullptr};
  if (b == 128) return launch<bf16, 128, 128>(la, lb, ep, M, N, K, splits, st);
  if (b == 64) return launch<bf16, 64, 64>(la, lb, ep, M, N, K, splits, st);
  return launch<bf16, 32, 32>(la, lb, ep, M, N, K, splits, st);
}

// ---- the attention decoder's gate GEMM with its LSTM cell in the epilogue (crnn_attn_gates_cell)
// W rows gate-interleaved (row 4u + q = the reference's row q*H + u, q = i f g o): the MFMA epilogue hands a lane 4
// consecutive columns of one row, i.e. the four gates of one unit of one sample, and the cell runs right there. The
// arithmetic is attn.hip attn_cell_kernel's, in the same order, so the fused step equals GEMM + cell bit for bit.
struct AttnCellEpi {
  static constexpr bool kStats = false;
  const float *b_ih, *b_hh;   // [4H] interleaved
  const float* wv;            // [V][4H] interleaved one-hot columns of W_ih
  const int* ch;
  int ch_stride;
  float *h, *c, *hx;
  int ldx;
  float* hs;
  int ld_hs;
  float *gact, *cs;
  int B, H, C;
  __device__ __forceinline__ void store(int m, int n, f32x4 v, int) const {
    if (m >= B || n >= 4 * H) return;
    const int u = n >> 2;
    const float* wr = wv + (size_t)ch[(size_t)m * ch_stride] * 4 * H + n;
    float g[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) g[q] = v[q] + b_ih[n + q] + b_hh[n + q] + wr[q];
    const float ig = 1.f / (1.f + expf(-g[0])), fg = 1.f / (1.f + expf(-g[1])), gg = tanhf(g[2]),
                og = 1.f / (1.f + expf(-g[3]));
    const size_t e = (size_t)m * H + u;
    const float cn = fg * c[e] + ig * gg;
    const float hn = og * tanhf(cn);
    c[e] = cn;
    h[e] = hn;
    hx[(size_t)m * ldx + C + u] = hn;
    if (hs) hs[(size_t)m * ld_hs + u] = hn;
    if (gact) {   // saved for the backward in the reference's gate-block order
      float* gr = gact + (size_t)m * 4 * H;
      gr[u] = ig;
      gr[H + u] = fg;
      gr[2 * H + u] = gg;
      gr[3 * H + u] = og;
      cs[e] = cn;
    }
  }
  __device__ __forceinline__ void stats(int, int, f32x4, f32x4) const {}
};

// the tile plans of crnn_gemm_nt (run / run_mix) with another epilogue
template <typename T, class LA, class LB, class EPI>
int run_plain(const LA& la, const LB& lb, const EPI& ep, int M, int N, int K, hipStream_t st) {
  const long work = (long)M * N;
  if (M >= 128 && N >= 128 && work >= 128L * 128 * 128) return launch<T, 128, 128>(la, lb, ep, M, N, K, 1, st);
  if (work >= 64L * 64 * 128) return launch<T, 64, 64>(la, lb, ep, M, N, K, 1, st);
  return launch<T, 32, 32>(la, lb, ep, M, N, K, 1, st);
}

// split-K partials of C = A^T B into fp32 slabs [S][M][N] (deterministic; fp32 atomics from every
// split are several times slower on this chip), then one fixed-order reduce into C (ldc, +=)
struct TnSlabEpi {
  static constexpr bool kStats = false;
  float* ws;
  int M, N;
  __device__ __forceinline__ void store(int m, int n, f32x4 v, int kz) const {
    if (m < M && n < N) *reinterpret_cast<f32x4*>(ws + ((size_t)kz * M + m) * N + n) = v;
  }
  __device__ __forceinline__ void stats(int, int, f32x4, f32x4) const {}
};

__global__ __launch_bounds__(256) void tn_reduce_kernel(const float* __restrict__ ws, int S, int M, int N,
                                                        float* __restrict__ C, int ldc, int accumulate) {
  const long total = (long)M * N;
  for (long i4 = blockIdx.x * (long)blockDim.x + threadIdx.x; 4 * i4 < total; i4 += (long)gridDim.x * blockDim.x) {
    const long i = 4 * i4;
    f32x4 s = {0.f, 0.f, 0.f, 0.f};
    int z = 0;
    for (; z + 8 <= S; z += 8) {
      f32x4 v[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) v[q] = *reinterpret_cast<const f32x4*>(ws + (size_t)(z + q) * total + i);
#pragma unroll
      for (int q = 0; q < 8; ++q) s += v[q];
    }
    for (; z < S; ++z) s += *reinterpret_cast<const f32x4*>(ws + (size_t)z * total + i);
    const int m = (int)(i / N), n = (int)(i - (long)m * N);
    float* o = C + (size_t)m * ldc + n;
#pragma unroll
    for (int e = 0; e < 4; ++e) o[e] = accumulate ? o[e] + s[e] : s[e];
  }
}

inline int tn_slab_splits(int M, int N, int K) {
  const long tiles = (long)((M + 127) / 128) * ((N + 127) / 128);
  long s = (256 + tiles - 1) / tiles;
  const long smax = (K + 16 * 64 - 1) / (16 * 64);   // >= 16 K-tiles per split
  if (s > smax) s = smax;
  if (s < 1) s = 1;
  return eff_splits(K, (int)s);
}

// out[n] (+)= sum_m X[m][n] (bias gradients), in a FIXED order: block = 16 columns; thread = (4-column
// quarter q = tid & 3, row lane rl = tid >> 2 of 256) sums rows rl, rl + 256, ... with 8 rows' 4-column
// loads in flight, then a fixed tree over the row lanes in LDS. One launch, no atomics: the r01-r03
// version added row-chunk sums with fp32 atomics, whose last bits followed the arrival order.
constexpr int CS_RL = 256;
template <typename T>
__global__ __launch_bounds__(1024) void colsum_kernel(const T* __restrict__ X, int ld, long M, int N,
                                                      float* __restrict__ out, int accumulate, int vec) {
  __shared__ f32x4 red[1024];
  const int tid = threadIdx.x, q = tid & 3, rl = tid >> 2;
  const int n = blockIdx.x * 16 + 4 * q;
  const bool okn = n < N;
  // 16-B loads only for a quarter whose 4 columns are all < N (vec: ld % 4 == 0, 16-B aligned X): the
  // last row of a strided view may end at column N, so a ragged last quarter loads element-wise
  const bool vq = vec && n + 4 <= N;
  f32x4 s = {0.f, 0.f, 0.f, 0.f};
  for (long mb = rl; mb < M; mb += 8 * CS_RL) {
    f32x4 v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const long m = mb + (long)u * CS_RL;
      const bool ok = okn && m < M;
      // clamped address, masked value: the loads stay unconditional (all 8 in flight)
      const T* p = X + (size_t)(m < M ? m : M - 1) * ld + (okn ? n : 0);
      if (vq) {
        v[u] = ld4f<T>(p);
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) v[u][e] = tof(p[n + e < N ? e : 0]);
      }
      if (!ok) v[u] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) s += v[u];
  }
  red[tid] = s;
  __syncthreads();
  for (int st = CS_RL / 2; st >= 1; st >>= 1) {   // lane rl += lane rl + st, fixed order
    if (rl < st) red[tid] = red[tid] + red[tid + 4 * st];
    __syncthreads();
  }
  if (rl == 0 && okn) {
    const f32x4 r = red[q];
#pragma unroll
    for (int e = 0; e < 4; ++e)
      if (n + e < N) out[n + e] = accumulate ? out[n + e] + r[e] : r[e];
  }
}

}  // namespace

extern "C" {

int crnn_gemm_nt(int dtype, const void* A, int lda, const void* B, int ldb, void* C, int ldc, const float* bias, int M,
                 int N, int K, int c_f32, int accumulate, void* stream) {
  if (K % 8 || lda % 8 || ldb % 8) return crnn_set_error(hipErrorInvalidValue, "gemm_nt: K/lda/ldb must be multiples of 8");
  hipStream_t st = (hipStream_t)stream;
  if (dtype == CRNN_F32_BF16MMA) return gemm_nt_mix(A, lda, B, ldb, C, ldc, bias, M, N, K, accumulate, st);
  return dtype == CRNN_BF16 ? gemm_nt_t<bf16>(A, lda, B, ldb, C, ldc, bias, M, N, K, c_f32, accumulate, st)
                            : gemm_nt_t<float>(A, lda, B, ldb, C, ldc, bias, M, N, K, c_f32, accumulate, st);
}

int crnn_gemm_nn(int dtype, const void* A, int lda, const void* B, int ldb, void* C, int ldc, int M, int N, int K,
                 int c_f32, int accumulate, void* stream) {
  if (K % 8 || N % 8 || lda % 8 || ldb % 8) return crnn_set_error(hipErrorInvalidValue, "gemm_nn: K/N/ld must be multiples of 8");
  hipStream_t st = (hipStream_t)stream;
  if (dtype == CRNN_F32_BF16MMA) return gemm_nn_mix(A, lda, B, ldb, C, ldc, M, N, K, accumulate, st);
  return dtype == CRNN_BF16 ? gemm_nn_t<bf16>(A, lda, B, ldb, C, ldc, M, N, K, c_f32, accumulate, st)
                            : gemm_nn_t<float>(A, lda, B, ldb, C, ldc, M, N, K, c_f32, accumulate, st);
}

int crnn_gemm_tn(int dtype, const void* A, int lda, const void* B, int ldb, float* C, int ldc, int M, int N, int K,
                 int accumulate, void* stream) {
  if (M % 8 || N % 8 || lda % 8 || ldb % 8) return crnn_set_error(hipErrorInvalidValue, "gemm_tn: M/N/ld must be multiples of 8");
  hipStream_t st = (hipStream_t)stream;
  if (dtype == CRNN_F32_BF16MMA) return gemm_tn_mix(A, lda, B, ldb, C, ldc, M, N, K, accumulate, st);
  return dtype == CRNN_BF16 ? gemm_tn_t<bf16>(A, lda, B, ldb, C, ldc, M, N, K, accumulate, st)
                            : gemm_tn_t<float>(A, lda, B, ldb, C, ldc, M, N, K, accumulate, st);
}

int crnn_colsum(int dtype, const void* X, int ld, long M, int N, float* out, int accumulate, int x_f32, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (ld < N || M < 0 || N < 0) return crnn_set_error(hipErrorInvalidValue, "colsum: ld >= N >= 0, M >= 0");
  if (N == 0) return 0;
  if (M == 0) return accumulate ? 0 : (int)hipMemsetAsync(out, 0, (size_t)N * sizeof(float), st);
  const int vec = ld % 4 == 0 && ((uintptr_t)X % 16) == 0;
  dim3 grid((N + 15) / 16);
  if (x_f32 || dtype != CRNN_BF16)
    hipLaunchKernelGGL(colsum_kernel<float>, grid, dim3(1024), 0, st, (const float*)X, ld, M, N, out, accumulate, vec);
  else
    hipLaunchKernelGGL(colsum_kernel<bf16>, grid, dim3(1024), 0, st, (const bf16*)X, ld, M, N, out, accumulate, vec);
  return (int)hipGetLastError();
}

size_t crnn_gemm_tn_workspace(int M, int N, int K) {
  return (size_t)tn_slab_splits(M, N, K) * M * N * sizeof(float);
}

int crnn_gemm_tn_slab(const void* A, int lda, const void* B, int ldb, float* C, int ldc, int M, int N, int K,
                      int accumulate, float* ws, size_t ws_bytes, void* stream) {
  if (M % 8 || N % 8 || lda % 8 || ldb % 8) return crnn_set_error(hipErrorInvalidValue, "gemm_tn: M/N/ld must be multiples of 8");
  if (ws_bytes < crnn_gemm_tn_workspace(M, N, K)) return crnn_set_error(hipErrorInvalidValue, "gemm_tn: workspace too small");
  hipStream_t st = (hipStream_t)stream;
  const int S = tn_slab_splits(M, N, K);
  ColMajorK<bf16> la{(const bf16*)A, lda, M, K};
  ColMajorK<bf16> lb{(const bf16*)B, ldb, N, K};
  TnSlabEpi ep{ws, M, N};
  int rc = launch<bf16, 128, 128>(la, lb, ep, M, N, K, S, st);
  if (rc) return rc;
  int blocks = (int)(((long)M * N / 4 + 255) / 256);
  if (blocks > 2048) blocks = 2048;
  hipLaunchKernelGGL(tn_reduce_kernel, dim3(blocks), dim3(256), 0, st, ws, S, M, N, C, ldc, accumulate);
  return (int)hipGetLastError();
}

int crnn_attn_gates_cell(int dtype, const float* X, int ldx, const float* W, int ldw, const float* b_ih,
                         const float* b_hh, const float* wv, const int* ch, int ch_stride, float* h, float* c,
                         float* hx, int ldhx, float* hs, int ld_hs, float* gact, float* cs, int B, int H, int C,
                         void* stream) {
  const int K = C + H;
  if (K % 8 || ldx % 8 || ldw % 8) return crnn_set_error(hipErrorInvalidValue, "attn_gates_cell: K/ld must be multiples of 8");
  if (hx == X) return crnn_set_error(hipErrorInvalidValue, "attn_gates_cell: hx must not alias X (read by the GEMM)");
  hipStream_t st = (hipStream_t)stream;
  const AttnCellEpi ep{b_ih, b_hh, wv, ch, ch_stride, h, c, hx, ldhx, hs, ld_hs, gact, cs, B, H, C};
  const int M = B, N = 4 * H;
  if (dtype == CRNN_F32_BF16MMA) {   // crnn_gemm_nt's run_mix plan
    Bf16Of<RowMajorK<float>> la{RowMajorK<float>{X, ldx, M, K}};
    Bf16Of<RowMajorK<float>> lb{RowMajorK<float>{W, ldw, N, K}};
    const long t64 = (long)((M + 63) / 64) * ((N + 63) / 64);
    if (t64 >= 2 * crnn_cu_count() || K < 512) return run_plain<bf16>(la, lb, ep, M, N, K, st);
    return launch<bf16, 32, 32, 128>(la, lb, ep, M, N, K, 1, st);
  }
  RowMajorK<float> la{X, ldx, M, K};
  RowMajorK<float> lb{W, ldw, N, K};
  return run_plain<float>(la, lb, ep, M, N, K, st);
}

}  // extern "C"
