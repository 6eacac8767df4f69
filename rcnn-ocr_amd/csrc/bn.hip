// BatchNorm / ReLU / MaxPool / SE / residual / height-collapse kernels, NHWC.
//
// Reference semantics:
//   nn.BatchNorm2d train/eval (torch defaults eps 1e-5, momentum 0.1)   model/seresnet31.py:40-45
//   nn.ReLU, nn.MaxPool2d(2,2)                                          model/seresnet31.py:83-88
//   SELayer: mean_hw -> Linear(C,C/16,no bias) -> ReLU -> Linear(C/16,C) -> sigmoid -> x*s
//                                                                       model/seresnet31.py:5-20
//   SEBasicBlock tail: relu(se(bn2(conv2)) + identity|bn_d(conv_d(x)))   model/seresnet31.py:55-67
//   AdaptiveAvgPool2d((1,None)) + squeeze(2) + permute(0,2,1)           model/model.py:191, 216-218
// All elementwise passes move 8 channels (16 B bf16 / 32 B f32) per lane.
#include "common.hpp"
#include "crnn_internal.hpp"

namespace {

constexpr int NT = 256;

// ------------------------------------------------------------ channel reductions
// Block b reduces rows [b*rpb, (b+1)*rpb) of an [M][C] tensor into row b of two
// [rows][C] partial buffers. Threads: cg = C/8 channel groups x (256/cg) row lanes.
template <class F>
__global__ __launch_bounds__(NT) void chan_reduce_kernel(F f, long M, int C, long rpb, float* __restrict__ p0,
                                                         float* __restrict__ p1) {
  extern __shared__ float red[];  // [2][rl][C]
  const int cg = C / 8, rl = NT / cg;
  const int tid = threadIdx.x, c8 = (tid % cg) * 8, r = tid / cg;
  float a0[8], a1[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) a0[i] = a1[i] = 0.f;
  const long m0 = blockIdx.x * rpb, m1 = min(M, m0 + rpb);
  if (r < rl)
    for (long m = m0 + r; m < m1; m += rl) f(m, c8, a0, a1);
  if (r < rl) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      red[r * C + c8 + i] = a0[i];
      red[(rl + r) * C + c8 + i] = a1[i];
    }
  }
  __syncthreads();
  for (int c = tid; c < C; c += NT) {
    float s0 = 0.f, s1 = 0.f;
    for (int q = 0; q < rl; ++q) {
      s0 += red[q * C + c];
      s1 += red[(rl + q) * C + c];
    }
    p0[(size_t)blockIdx.x * C + c] = s0;
    p1[(size_t)blockIdx.x * C + c] = s1;
  }
}

// (sum, M2) partials of a streamed [M][C] tensor: block-local two-pass (the block's rows
// are re-read for the second pass, they are L2-resident) — matches the conv epilogue format.
template <typename T>
__global__ __launch_bounds__(NT) void chan_stats_kernel(const T* __restrict__ x, long M, int C, long rpb,
                                                        float* __restrict__ p0, float* __restrict__ p1) {
  extern __shared__ float red[];  // [rl][C] + [C] block means
  const int cg = C / 8, rl = NT / cg;
  const int tid = threadIdx.x, c8 = (tid % cg) * 8, r = tid / cg;
  const long m0 = blockIdx.x * rpb, m1 = min(M, m0 + rpb);
  const long n = m1 > m0 ? m1 - m0 : 0;
  float* mu = red + rl * C;
  float a[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) a[i] = 0.f;
  if (r < rl)
    for (long m = m0 + r; m < m1; m += rl) {
      float v[8];
      unpack8<T>(ld8<T>(x + m * C + c8), v);
#pragma unroll
      for (int i = 0; i < 8; ++i) a[i] += v[i];
    }
  if (r < rl)
#pragma unroll
    for (int i = 0; i < 8; ++i) red[r * C + c8 + i] = a[i];
  __syncthreads();
  for (int c = tid; c < C; c += NT) {
    float s = 0.f;
    for (int q = 0; q < rl; ++q) s += red[q * C + c];
    p0[(size_t)blockIdx.x * C + c] = s;
    mu[c] = n > 0 ? s / (float)n : 0.f;
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 8; ++i) a[i] = 0.f;
  if (r < rl)
    for (long m = m0 + r; m < m1; m += rl) {
      float v[8];
      unpack8<T>(ld8<T>(x + m * C + c8), v);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        float d = v[i] - mu[c8 + i];
        a[i] += d * d;
      }
    }
  __syncthreads();
  if (r < rl)
#pragma unroll
    for (int i = 0; i < 8; ++i) red[r * C + c8 + i] = a[i];
  __syncthreads();
  for (int c = tid; c < C; c += NT) {
    float s = 0.f;
    for (int q = 0; q < rl; ++q) s += red[q * C + c];
    p1[(size_t)blockIdx.x * C + c] = s;
  }
}

// upstream gradient g of a BN output, by mode (see crnn_hip.h CRNN_BNG_*)
template <typename T>
__device__ __forceinline__ void bn_g(const crnn_bn_bwd_desc& d, unsigned m, int c8, const float* zz, float* g) {
  float dy[8];
  unpack8<T>(ld8<T>((const T*)d.dy + (size_t)m * d.C + c8), dy);
  if (d.mode == CRNN_BNG_PLAIN) {
#pragma unroll
    for (int i = 0; i < 8; ++i) g[i] = dy[i];
  } else if (d.mode == CRNN_BNG_RELU) {
#pragma unroll
    for (int i = 0; i < 8; ++i) g[i] = (zz[i] * d.scale[c8 + i] + d.shift[c8 + i]) > 0.f ? dy[i] : 0.f;
  } else {
    float y[8];
    unpack8<T>(ld8<T>((const T*)d.y + (size_t)m * d.C + c8), y);
    if (d.mode == CRNN_BNG_RESID) {
#pragma unroll
      for (int i = 0; i < 8; ++i) g[i] = y[i] > 0.f ? dy[i] : 0.f;
    } else {
      const unsigned b = m / (unsigned)d.HW;
      const float* s = d.s + (size_t)b * d.C + c8;
      const float* dp = d.dpool + (size_t)b * d.C + c8;
#pragma unroll
      for (int i = 0; i < 8; ++i) g[i] = (y[i] > 0.f ? dy[i] * s[i] : 0.f) + dp[i];
    }
  }
}

int cg_shift(int C) {
  if (C % 8) return -1;
  int g = C / 8, s = 0;
  while ((1 << s) < g) ++s;
  return (1 << s) == g ? s : -1;
}

int rows_for(long M) {
  long r = (M + 63) / 64;
  if (r > 1024) r = 1024;
  if (r < 1) r = 1;
  return (int)r;
}

template <class F> int chan_reduce(F f, long M, int C, float* p0, float* p1, int rows, hipStream_t st) {
  if (C % 8 || C / 8 > NT || NT % (C / 8)) return crnn_set_error(hipErrorInvalidValue, "channel reduce: bad C");
  long rpb = (M + rows - 1) / rows;
  int rl = NT / (C / 8);
  size_t sm = (size_t)2 * rl * C * sizeof(float);
  hipLaunchKernelGGL((chan_reduce_kernel<F>), dim3(rows), dim3(NT), sm, st, f, M, C, rpb, p0, p1);
  return (int)hipGetLastError();
}

// ------------------------------------------------------------ finalize
// Up to FIN_FUSED_ROWS partial rows (C % 8 == 0): one launch (fin_one_kernel below). Otherwise two
// launches:
//  (1) fin_chunk_kernel, grid (C/64, P): block y folds partial rows [y*chunk, ...) of 64 channels
//      (4 row lanes per channel, 8 loads in flight per lane) into one chunk partial. Chan mode
//      (forward): rows hold (sum, M2 about the row's own mean) covering rpp data rows, the chunk
//      result is (sum, M2 about the chunk mean), two-pass over the L2-resident rows; plain mode
//      (backward): two independent sums. P adapts so a block folds ~16 rows.
//  (2) fin_combine_kernel, grid C/16: 16 lanes per channel fold the P (<= 256) chunk partials
//      in double — one batch of 16 loads per lane, full chunks share one reciprocal.
constexpr int FIN_P = 256;   // max chunk partials
constexpr int FIN_CNT = 64;  // reserved head of the workspace (floats)

__device__ __forceinline__ long span_rows(long r0, long r1, long rpp, long count) {
  long a = r0 * rpp, b = r1 * rpp;
  if (b > count) b = count;
  return b > a ? b - a : 0;
}

struct FinFwd {  // forward: batch statistics -> running stats, mean/invstd, affine scale/shift
  const float* gamma;
  const float* beta;
  float* rmean;
  float* rvar;
  float momentum, eps;
  float* mean_o;
  float* inv_o;
  float* scale_o;
  float* shift_o;
};
struct FinBwd {  // backward: sum(g), sum(g xhat) -> dbeta, dgamma, their means
  float* dgamma;
  float* dbeta;
  float* mean_g;
  float* mean_gx;
  int acc;
};

__device__ __forceinline__ void write_affine(const FinFwd& a, int c, double mean, double var, bool train, long count) {
  if (train) {
    if (a.rmean) {
      double unb = count > 1 ? var * (double)count / (double)(count - 1) : var;
      a.rmean[c] = (float)((1.0 - a.momentum) * a.rmean[c] + a.momentum * mean);
      a.rvar[c] = (float)((1.0 - a.momentum) * a.rvar[c] + a.momentum * unb);
    }
  } else {
    mean = a.rmean[c];
    var = a.rvar[c];
  }
  double inv = 1.0 / sqrt(var + (double)a.eps);
  double sc = (double)a.gamma[c] * inv;
  if (a.mean_o) a.mean_o[c] = (float)mean;
  if (a.inv_o) a.inv_o[c] = (float)inv;
  a.scale_o[c] = (float)sc;
  a.shift_o[c] = (float)((double)a.beta[c] - mean * sc);
}

template <bool CHAN>
__global__ __launch_bounds__(256) void fin_chunk_kernel(const float* __restrict__ p0, const float* __restrict__ p1,
                                                        int rows, long rpp, int C, long count, int chunk,
                                                        float* __restrict__ o0, float* __restrict__ o1) {
  __shared__ float red[2][4][64];
  const int lc = threadIdx.x & 63, ln = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + lc;
  const int r0 = blockIdx.y * chunk, r1 = min(rows, r0 + chunk);
  float s = 0.f, q = 0.f;
  if (c < C)
    for (int rb = r0 + ln; rb < r1; rb += 32) {  // 8 independent loads in flight per lane
      float a[8], b[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int r = rb + 4 * u;
        a[u] = r < r1 ? p0[(size_t)r * C + c] : 0.f;
        b[u] = (!CHAN && r < r1) ? p1[(size_t)r * C + c] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        s += a[u];
        q += b[u];
      }
    }
  red[0][ln][lc] = s;
  red[1][ln][lc] = q;
  __syncthreads();
  const float S = red[0][0][lc] + red[0][1][lc] + red[0][2][lc] + red[0][3][lc];
  if (CHAN) {
    const long n = span_rows(r0, r1, rpp, count);
    const float mu = n > 0 ? S / (float)n : 0.f;
    const float rr = 1.f / (float)rpp;
    q = 0.f;
    if (c < C)
      for (int rb = r0 + ln; rb < r1; rb += 32) {
        float a[8], b[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int r = rb + 4 * u;
          a[u] = r < r1 ? p0[(size_t)r * C + c] : 0.f;
          b[u] = r < r1 ? p1[(size_t)r * C + c] : 0.f;
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int r = rb + 4 * u;
          const long nr = r < r1 ? span_rows(r, r + 1, rpp, count) : 0;
          if (nr == 0) continue;
          const float d = a[u] * (nr == rpp ? rr : 1.f / (float)nr) - mu;
          q += b[u] + (float)nr * d * d;
        }
      }
    __syncthreads();
    red[1][ln][lc] = q;
    __syncthreads();
  }
  if (ln == 0 && c < C) {
    o0[(size_t)blockIdx.y * C + c] = S;
    o1[(size_t)blockIdx.y * C + c] = red[1][0][lc] + red[1][1][lc] + red[1][2][lc] + red[1][3][lc];
  }
}

template <bool CHAN, class A>
__global__ __launch_bounds__(256) void fin_combine_kernel(const float* __restrict__ o0, const float* __restrict__ o1,
                                                          int P, long crows, int C, long count, A args) {
  __shared__ double dred[2][16][16];
  const int lc = threadIdx.x & 15, ln = threadIdx.x >> 4;
  const int c = blockIdx.x * 16 + lc;
  const bool okc = c < C;
  float v[16], w[16];
#pragma unroll
  for (int u = 0; u < 16; ++u) {  // P <= 256: one batch
    const int p = ln + 16 * u;
    v[u] = (okc && p < P) ? o0[(size_t)p * C + c] : 0.f;
    w[u] = (okc && p < P) ? o1[(size_t)p * C + c] : 0.f;
  }
  double s = 0.0, q = 0.0;
#pragma unroll
  for (int u = 0; u < 16; ++u) {
    s += v[u];
    if (!CHAN) q += w[u];
  }
  dred[0][ln][lc] = s;
  dred[1][ln][lc] = q;
  __syncthreads();
  s = 0.0;
  q = 0.0;
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    s += dred[0][k][lc];
    q += dred[1][k][lc];
  }
  if constexpr (CHAN) {
    const double mean = s / (double)count;
    const double rfull = 1.0 / (double)crows;
    double m2 = 0.0;
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int p = ln + 16 * u;
      const long n = p < P ? span_rows(p, p + 1, crows, count) : 0;
      if (n == 0) continue;
      const double d = (double)v[u] * (n == crows ? rfull : 1.0 / (double)n) - mean;
      m2 += (double)w[u] + (double)n * d * d;
    }
    __syncthreads();
    dred[1][ln][lc] = m2;
    __syncthreads();
    if (ln != 0 || !okc) return;
    m2 = 0.0;
#pragma unroll
    for (int k = 0; k < 16; ++k) m2 += dred[1][k][lc];
    double var = m2 / (double)count;
    if (var < 0.0) var = 0.0;
    write_affine(args, c, mean, var, true, count);
  } else {
    if (ln != 0 || !okc) return;
    if (args.dgamma) args.dgamma[c] = (float)(args.acc ? args.dgamma[c] + q : q);
    if (args.dbeta) args.dbeta[c] = (float)(args.acc ? args.dbeta[c] + s : s);
    args.mean_g[c] = (float)(s / (double)count);
    args.mean_gx[c] = (float)(q / (double)count);
  }
}

constexpr int FIN_FUSED_ROWS = 2048;

// One-launch finalize with NO inter-workgroup hand-off (r04, the default for <= FIN_FUSED_ROWS rows):
// block = 8 channels; thread = (4-channel half h = tid & 1, row lane rl = tid >> 1 of 128). Each thread
// holds its NR rows (rl, rl + 128, ...; 16-B buffer loads all in flight, out-of-range rows read 0) in
// registers. Backward: the two sums in double. Forward (CHAN): two passes over the registers, no
// per-row division — the batch mean from the row sums, then M2 = sum_r (M2_r + n_r (mean_r - mean)^2)
// (every row holds rpp samples except at most the one at count / rpp). Block sums: an xor butterfly
// over the wave's 32 row lanes (commutative adds: every lane ends with the same bits), then the four
// waves' values from LDS in a fixed order. A block reads only what the previous kernel wrote, so the
// launch boundary is the only hand-off. (r01-r03 handed chunk results to the group's last block by
// 4-B sc1 stores / loads + a ticket: a form the guide measures valid only at one workgroup per CU;
// under load it read stale chunk results, DESIGN.md §6. Removed in r06.)
constexpr int FIN1_RL = 128;

template <int K>
__device__ __forceinline__ void fin1_block_sum(double (&v)[K], double (*sh)[2][K], int wv, int h, int rl) {
#pragma unroll
  for (int o = 2; o < 64; o <<= 1)
#pragma unroll
    for (int k = 0; k < K; ++k) v[k] += __shfl_xor(v[k], o);
  if ((rl & 31) == 0)
#pragma unroll
    for (int k = 0; k < K; ++k) sh[wv][h][k] = v[k];
  __syncthreads();
#pragma unroll
  for (int k = 0; k < K; ++k) v[k] = ((sh[0][h][k] + sh[1][h][k]) + sh[2][h][k]) + sh[3][h][k];
}

template <bool CHAN, int NR, class A>
__global__ __launch_bounds__(256) void fin_one_kernel(const float* __restrict__ p0, const float* __restrict__ p1,
                                                      int rows, long rpp, int C, long count, A args) {
  __shared__ double sh1[4][2][8], sh2[4][2][4];
  const int tid = threadIdx.x, h = tid & 1, rl = tid >> 1, wv = tid >> 6;
  const int c = blockIdx.x * 8 + 4 * h;
  const uint32_t bytes = (uint32_t)((size_t)rows * C * sizeof(float));
  const __amdgpu_buffer_rsrc_t r0s = mk_rsrc(p0, bytes), r1s = mk_rsrc(p1, bytes);
  f32x4 a[NR], b[NR];
#pragma unroll
  for (int u = 0; u < NR; ++u) {
    const int r = rl + u * FIN1_RL;
    const uint32_t off = r < rows ? (uint32_t)(((size_t)r * C + c) * 4) : OOB;
    a[u] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r0s, off, 0, 0));
    b[u] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r1s, off, 0, 0));
  }
  if constexpr (CHAN) {
    double v[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int u = 0; u < NR; ++u)
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] += (double)a[u][i];
    fin1_block_sum<4>(v, (double(*)[2][4])sh2, wv, h, rl);
    double mean[4], q[4];
    const double rc = 1.0 / (double)count;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      mean[i] = v[i] * rc;
      q[i] = 0.0;
    }
    // row r holds nb(r) = rpp samples for r < rfull, count % rpp at r == rfull, none beyond
    const long rfull = count / rpp;
    const double npart = (double)(count - rfull * rpp), rr = 1.0 / (double)rpp;
    const double rpart = npart > 0.0 ? 1.0 / npart : 0.0;
#pragma unroll
    for (int u = 0; u < NR; ++u) {
      const long r = rl + u * FIN1_RL;
      const double nb = r < rfull ? (double)rpp : (r == rfull ? npart : 0.0);
      const double rnb = r < rfull ? rr : (r == rfull ? rpart : 0.0);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const double d = (double)a[u][i] * rnb - mean[i];
        q[i] += nb > 0.0 ? (double)b[u][i] + nb * d * d : 0.0;
      }
    }
    double w[8];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      w[i] = q[i];
      w[4 + i] = 0.0;
    }
    fin1_block_sum<8>(w, sh1, wv, h, rl);
    if (rl != 0) return;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      double var = w[i] * rc;
      if (var < 0.0) var = 0.0;
      write_affine(args, c + i, mean[i], var, true, count);
    }
  } else {
    double v[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = 0.0;
#pragma unroll
    for (int u = 0; u < NR; ++u)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        v[i] += (double)a[u][i];
        v[4 + i] += (double)b[u][i];
      }
    fin1_block_sum<8>(v, sh1, wv, h, rl);
    if (rl != 0) return;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const double s = v[i], q = v[4 + i];
      if (args.dgamma) args.dgamma[c + i] = (float)(args.acc ? args.dgamma[c + i] + q : q);
      if (args.dbeta) args.dbeta[c + i] = (float)(args.acc ? args.dbeta[c + i] + s : s);
      args.mean_g[c + i] = (float)(s / (double)count);
      args.mean_gx[c + i] = (float)(q / (double)count);
    }
  }
}

// eval mode: running statistics only
__global__ void bn_eval_affine_kernel(int C, FinFwd a) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c < C) write_affine(a, c, 0.0, 1.0, false, 0);
}

template <bool CHAN, class A>
int launch_fin(const float* p0, const float* p1, int rows, long rpp, int C, long count, float* ws, const A& args,
               hipStream_t st) {
  if (rows <= FIN_FUSED_ROWS && C % 8 == 0) {
    const dim3 g(C / 8), t(256);
    if (rows <= 2 * FIN1_RL)
      hipLaunchKernelGGL((fin_one_kernel<CHAN, 2, A>), g, t, 0, st, p0, p1, rows, rpp, C, count, args);
    else if (rows <= 4 * FIN1_RL)
      hipLaunchKernelGGL((fin_one_kernel<CHAN, 4, A>), g, t, 0, st, p0, p1, rows, rpp, C, count, args);
    else if (rows <= 8 * FIN1_RL)
      hipLaunchKernelGGL((fin_one_kernel<CHAN, 8, A>), g, t, 0, st, p0, p1, rows, rpp, C, count, args);
    else
      hipLaunchKernelGGL((fin_one_kernel<CHAN, 16, A>), g, t, 0, st, p0, p1, rows, rpp, C, count, args);
    return (int)hipGetLastError();
  }
  int P = rows / 16;  // ~16 partial rows per stage-1 block (4 per lane)
  if (P > FIN_P) P = FIN_P;
  if (P < 1) P = 1;
  const int chunk = (rows + P - 1) / P;
  P = (rows + chunk - 1) / chunk;
  float* part = ws + FIN_CNT;
  hipLaunchKernelGGL((fin_chunk_kernel<CHAN>), dim3((C + 63) / 64, P), dim3(256), 0, st, p0, p1, rows, rpp, C, count,
                     chunk, part, part + (size_t)FIN_P * C);
  hipLaunchKernelGGL((fin_combine_kernel<CHAN, A>), dim3((C + 15) / 16), dim3(256), 0, st, part,
                     part + (size_t)FIN_P * C, P, (long)chunk * rpp, C, count, args);
  return (int)hipGetLastError();
}

// maxpool 2x2/2 over relu(z*sc+sh); NHWC, one lane = 8 channels of one output pixel
template <typename T>
__global__ void bn_relu_maxpool_kernel(const T* __restrict__ z, const float* __restrict__ sc, const float* __restrict__ sh,
                                       T* __restrict__ y, int B, int H, int W, int C) {
  const int Ho = H / 2, Wo = W / 2, cg = C / 8;
  const long n = (long)B * Ho * Wo * cg;   // < 2^31 (host check): 32-bit index arithmetic
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const uint32_t iu = (uint32_t)i;
    int c8 = (int)(iu % (uint32_t)cg) * 8;
    const uint32_t p = iu / (uint32_t)cg;
    int wo = (int)(p % (uint32_t)Wo);
    const uint32_t q = p / (uint32_t)Wo;
    int ho = (int)(q % (uint32_t)Ho);
    int b = (int)(q / (uint32_t)Ho);
    float best[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) best[k] = -INFINITY;
#pragma unroll
    for (int dh = 0; dh < 2; ++dh)
#pragma unroll
      for (int dw = 0; dw < 2; ++dw) {
        float v[8];
        unpack8<T>(ld8<T>(z + (((size_t)b * H + 2 * ho + dh) * W + 2 * wo + dw) * C + c8), v);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          float a = fmaxf(v[k] * sc[c8 + k] + sh[c8 + k], 0.f);
          best[k] = a > best[k] ? a : best[k];
        }
      }
    st8<T>(y + (((size_t)b * Ho + ho) * Wo + wo) * C + c8, pack8<T>(best));
  }
}

// route d(pool) to the first maximum (scan order h, w — torch's max_pool2d index)
template <typename T>
__global__ void maxpool_bwd_kernel(const T* __restrict__ z, const float* __restrict__ sc, const float* __restrict__ sh,
                                   const T* __restrict__ dp, T* __restrict__ dy, int B, int H, int W, int C) {
  const int Ho = H / 2, Wo = W / 2, cg = C / 8;
  const long n = (long)B * Ho * Wo * cg;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    int c8 = (int)(i % cg) * 8;
    long p = i / cg;
    int wo = (int)(p % Wo);
    long q = p / Wo;
    int ho = (int)(q % Ho);
    int b = (int)(q / Ho);
    float a[4][8], best[8], g[8];
    int arg[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) { best[k] = -INFINITY; arg[k] = 0; }
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      unpack8<T>(ld8<T>(z + (((size_t)b * H + 2 * ho + (t >> 1)) * W + 2 * wo + (t & 1)) * C + c8), a[t]);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        float v = fmaxf(a[t][k] * sc[c8 + k] + sh[c8 + k], 0.f);
        if (v > best[k]) { best[k] = v; arg[k] = t; }
      }
    }
    unpack8<T>(ld8<T>(dp + (((size_t)b * Ho + ho) * Wo + wo) * C + c8), g);
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      float o[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) o[k] = arg[k] == t ? g[k] : 0.f;
      st8<T>(dy + (((size_t)b * H + 2 * ho + (t >> 1)) * W + 2 * wo + (t & 1)) * C + c8, pack8<T>(o));
    }
  }
}

// ------------------------------------------------------------ SE
// SELayer.fc (model/seresnet31.py:9-14, 16-20): Linear(C, C/16, bias=False) -> ReLU ->
// Linear(C/16, C, bias=False) -> Sigmoid on the pooled [B][C] vector, and its backward.
// Tiny GEMMs whose cost is memory round trips, not FLOPs: every global access is a 16-B vector,
// all of a phase's loads are issued before its first FMA, and they are UNCONDITIONAL (clamped
// addresses, masked values) — a load under a runtime condition makes hipcc branch around it and
// wait for it on the spot (cdna_hip_programming.md §5, trap 4(c)), serialising the batch.
// C is a template parameter (the SE-ResNet31 widths 256 / 512; Cr = C/16); SB samples per block
// share each weight read.
constexpr int SE_SB = 4;

// butterfly reduce-scatter: 32 values per lane summed over the 64 lanes of the wave; on return
// v[0] of lanes 2i and 2i+1 holds the full sum of value i (halving exchanges at xor 32..2, then 1)
__device__ __forceinline__ void reduce_scatter32(float (&v)[32], int lane) {
#pragma unroll
  for (int step = 0; step < 5; ++step) {
    const int o = 32 >> step, h = 16 >> step;
    const bool hi = (lane & o) != 0;
#pragma unroll
    for (int i = 0; i < h; ++i) {
      const float send = hi ? v[i] : v[i + h];
      const float keep = hi ? v[i + h] : v[i];
      v[i] = keep + __shfl_xor(send, o, 64);
    }
  }
  v[0] += __shfl_xor(v[0], 1, 64);
}

__device__ __forceinline__ float dot4(f32x4 a, f32x4 b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2] + a[3] * b[3]; }

// the squeeze from conv2's BN partial sums (crnn_se_pool_partials' arithmetic, same order), computed
// in the excitation kernel's load stage when FP: psum [B * per_b][C] rows, pooled written out for
// the backward
struct SePoolSrc {
  const float* psum;
  const float* scale;
  const float* shift;
  float* pooled;
  int per_b, HW;
};

template <int C, bool FP = false>
__global__ __launch_bounds__(256) void se_mlp_fwd_kernel(const float* __restrict__ pooled, const float* __restrict__ w1,
                                                         const float* __restrict__ w2, float* __restrict__ hid,
                                                         float* __restrict__ s, int B, SePoolSrc src = {}) {
  constexpr int Cr = C / 16, KC = C / 256;   // KC: 16-B column pieces per lane per w1 row
  __shared__ __attribute__((aligned(16))) float p[SE_SB][C];
  __shared__ __attribute__((aligned(16))) float h[SE_SB][Cr];
  const int b0 = blockIdx.x * SE_SB, tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int nb = min(SE_SB, B - b0);
#pragma unroll
  for (int q = 0; q < SE_SB * C / 1024; ++q) {
    const int i = 4 * tid + 1024 * q, sb = i / C;
    const int bb = b0 + min(sb, nb - 1), c = i % C;
    f32x4 v;
    if constexpr (FP) {
      f32x4 a = {0.f, 0.f, 0.f, 0.f};
      for (int k = 0; k < src.per_b; ++k) a += *reinterpret_cast<const f32x4*>(src.psum + ((size_t)bb * src.per_b + k) * C + c);
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = src.scale[c + r] * (a[r] / (float)src.HW) + src.shift[c + r];
      if (sb < nb) *reinterpret_cast<f32x4*>(src.pooled + (size_t)bb * C + c) = v;
    } else {
      v = *reinterpret_cast<const f32x4*>(pooled + (size_t)bb * C + c);
    }
    *reinterpret_cast<f32x4*>(&p[0][0] + i) = sb < nb ? v : f32x4{0.f, 0.f, 0.f, 0.f};
  }
  __syncthreads();
  // hidden = relu(p . W1^T): thread (row r = tid % Cr, channel chunk ck = tid / Cr of CK channels)
  // accumulates its chunk's dot products for the SB samples; chunks fold through LDS (no
  // cross-lane shuffles)
  {
    constexpr int NCK = 256 / Cr, CK = C / NCK;
    __shared__ float red[NCK][SE_SB][Cr];
    const int r = tid % Cr, ck = tid / Cr, cbeg = ck * CK;
    f32x4 wv[CK / 4];
#pragma unroll
    for (int q = 0; q < CK / 4; ++q) wv[q] = *reinterpret_cast<const f32x4*>(w1 + (size_t)r * C + cbeg + 4 * q);
#pragma unroll
    for (int sb = 0; sb < SE_SB; ++sb) {
      float a = 0.f;
#pragma unroll
      for (int q = 0; q < CK / 4; ++q) a += dot4(*reinterpret_cast<const f32x4*>(&p[sb][cbeg + 4 * q]), wv[q]);
      red[ck][sb][r] = a;
    }
    __syncthreads();
    if (tid < SE_SB * Cr) {
      const int sb = tid / Cr, rr = tid % Cr;
      float a = 0.f;
#pragma unroll
      for (int k = 0; k < NCK; ++k) a += red[k][sb][rr];
      a = fmaxf(a, 0.f);
      h[sb][rr] = a;
      if (sb < nb) hid[(size_t)(b0 + sb) * Cr + rr] = a;
    }
  }
  __syncthreads();
  // s = sigmoid(h . W2^T): lane = (row group rg = lane % G of 4 hidden units, channel sub-row
  // cs = lane / G): one instruction reads R whole w2 rows (contiguous); the G lanes of a row fold
  // their 4-unit partials with DPP moves (quad / half-row permutes, no LDS round trip)
  {
    constexpr int G = Cr / 4, R = 64 / G, CQ = C / 4, NI = CQ / R;
    const int rg = lane % G, cs = lane / G, cbeg = wid * CQ;
    f32x4 wv[NI];
#pragma unroll
    for (int k = 0; k < NI; ++k) wv[k] = *reinterpret_cast<const f32x4*>(w2 + (size_t)(cbeg + k * R + cs) * Cr + 4 * rg);
#pragma unroll
    for (int k = 0; k < NI; ++k) {
      const int c = cbeg + k * R + cs;
      float out = 0.f;
#pragma unroll
      for (int sb = 0; sb < SE_SB; ++sb) {
        float a = dot4(*reinterpret_cast<const f32x4*>(&h[sb][4 * rg]), wv[k]);
        a = rowgroup_sum<G>(a);
        out = rg == sb ? a : out;
      }
      if (rg < nb) s[(size_t)(b0 + rg) * C + c] = 1.f / (1.f + expf(-out));
    }
  }
}

// backward for SB samples per block: dsig = ds*s(1-s); dhid = (hid>0) * W2^T dsig;
// dpool = W1^T dhid / HW (the pool's mean folded in)
template <int C>
__global__ __launch_bounds__(256) void se_mlp_bwd_kernel(const float* __restrict__ ds, const float* __restrict__ hid,
                                                         const float* __restrict__ s, const float* __restrict__ w1,
                                                         const float* __restrict__ w2, float* __restrict__ dsig,
                                                         float* __restrict__ dhid, float* __restrict__ dpool, int B,
                                                         float inv_hw, const float* __restrict__ abc,
                                                         float* __restrict__ pg, float* __restrict__ pgx, int HW) {
  constexpr int Cr = C / 16;
  constexpr int G = Cr / 4, R = 64 / G;   // lanes per w2 row (16 B each), w2 rows per wave-instruction
  constexpr int CQ = C / 4, NI = CQ / R;  // channels per wave, load instructions per lane
  __shared__ __attribute__((aligned(16))) float dg[SE_SB][C];
  __shared__ __attribute__((aligned(16))) float red[4][SE_SB][Cr];
  __shared__ __attribute__((aligned(16))) float dh[SE_SB][Cr];
  const int b0 = blockIdx.x * SE_SB, tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int nb = min(SE_SB, B - b0);
#pragma unroll
  for (int q = 0; q < SE_SB * C / 1024; ++q) {
    const int i = 4 * tid + 1024 * q, sb = i / C;
    const size_t o = (size_t)(b0 + min(sb, nb - 1)) * C + i % C;
    const f32x4 sv = *reinterpret_cast<const f32x4*>(s + o);
    const f32x4 dv = *reinterpret_cast<const f32x4*>(ds + o);
    f32x4 v;
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = dv[e] * sv[e] * (1.f - sv[e]);
    if (sb < nb) *reinterpret_cast<f32x4*>(dsig + o) = v;
    *reinterpret_cast<f32x4*>(&dg[0][0] + i) = sb < nb ? v : f32x4{0.f, 0.f, 0.f, 0.f};
  }
  __syncthreads();
  // W2^T dg: lane = (row group rg = lane % G, channel sub-row cs = lane / G); wave w sums the
  // channels [w*CQ, (w+1)*CQ): NI 16-B loads per lane, all issued first
  {
    const int rg = lane % G, cs = lane / G, cbeg = wid * CQ;
    f32x4 wv[NI];
#pragma unroll
    for (int k = 0; k < NI; ++k) wv[k] = *reinterpret_cast<const f32x4*>(w2 + (size_t)(cbeg + k * R + cs) * Cr + 4 * rg);
    f32x4 acc[SE_SB];
#pragma unroll
    for (int sb = 0; sb < SE_SB; ++sb) {
      acc[sb] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int k = 0; k < NI; ++k) acc[sb] += dg[sb][cbeg + k * R + cs] * wv[k];
    }
    // fold the R channel sub-rows (lanes with equal rg): xor over the lane bits above G
#pragma unroll
    for (int sb = 0; sb < SE_SB; ++sb)
#pragma unroll
      for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int o = G; o < 64; o <<= 1) acc[sb][e] += __shfl_xor(acc[sb][e], o, 64);
    if (cs == 0)
#pragma unroll
      for (int sb = 0; sb < SE_SB; ++sb) *reinterpret_cast<f32x4*>(&red[wid][sb][4 * rg]) = acc[sb];
  }
  __syncthreads();
  if (tid < SE_SB * Cr) {
    const int sb = tid / Cr, r = tid % Cr;
    const float a = red[0][sb][r] + red[1][sb][r] + red[2][sb][r] + red[3][sb][r];
    const float hv = hid[(size_t)(b0 + min(sb, nb - 1)) * Cr + r];
    const float v = sb < nb && hv > 0.f ? a : 0.f;
    dh[sb][r] = v;
    if (sb < nb) dhid[(size_t)(b0 + sb) * Cr + r] = v;
  }
  __syncthreads();
  // dpool: thread = 4 consecutive channels, w1 columns by 16-B loads over all Cr rows
  if (4 * tid < C) {
    const int c4 = 4 * tid;
    f32x4 wv[Cr];
#pragma unroll
    for (int r = 0; r < Cr; ++r) wv[r] = *reinterpret_cast<const f32x4*>(w1 + (size_t)r * C + c4);
#pragma unroll
    for (int sb = 0; sb < SE_SB; ++sb) {
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int r = 0; r < Cr; ++r) acc += dh[sb][r] * wv[r];
      const f32x4 dp = acc * inv_hw;
      if (sb < nb) *reinterpret_cast<f32x4*>(dpool + (size_t)(b0 + sb) * C + c4) = dp;
      if (abc != nullptr && sb < nb) {   // the CRNN_BNG_SE BatchNorm sums (se_bn_partials_kernel's rows)
        const size_t b = (size_t)(b0 + sb);
        const f32x4 sv = *reinterpret_cast<const f32x4*>(s + b * C + c4);
        const f32x4 o0 = *reinterpret_cast<const f32x4*>(abc + b * 3 * C + c4);
        const f32x4 o1 = *reinterpret_cast<const f32x4*>(abc + b * 3 * C + C + c4);
        const f32x4 o2 = *reinterpret_cast<const f32x4*>(abc + b * 3 * C + 2 * C + c4);
        f32x4 q0, q1;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          q0[e] = sv[e] * o0[e] + (float)HW * dp[e];
          q1[e] = sv[e] * o1[e] + dp[e] * o2[e];
        }
        *reinterpret_cast<f32x4*>(pg + b * C + c4) = q0;
        *reinterpret_cast<f32x4*>(pgx + b * C + c4) = q1;
      }
    }
  }
}

// dw2[c][r] = sum_b dsig[b][c] hid[b][r] ; dw1[r][c] = sum_b dhid[b][r] pooled[b][c]
// block (x, y): 64 channels (16 groups of 4, one 16-B load each) x rows r0 = 8y .. 8y+7;
// 16 batch lanes (4 per wave x 4 waves) take interleaved samples; fixed-order combine
// (shuffles inside a wave, then LDS across waves): deterministic.
// Diagnostic build only (-DCRNN_SE_PROBE=1, tools/se_probe.py): every se_wgrad block records, per
// launch, the fixed-order sums of the four inputs as its lanes READ them and of its results, so a
// run-to-run difference can be placed before (read-time) or after (arithmetic) the loads.
#ifndef CRNN_SE_PROBE
#define CRNN_SE_PROBE 0
#endif
#if CRNN_SE_PROBE
constexpr int SE_PROBE_LAUNCHES = 32, SE_PROBE_BLOCKS = 64, SE_PROBE_VALS = 6;
__device__ float g_se_probe[SE_PROBE_LAUNCHES * SE_PROBE_BLOCKS * SE_PROBE_VALS];
static int g_se_probe_launch = 0;
#endif

template <int C>
__global__ __launch_bounds__(256) void se_wgrad_kernel(const float* __restrict__ dsig, const float* __restrict__ hid,
                                                       const float* __restrict__ dhid,
                                                       const float* __restrict__ pooled, float* __restrict__ dw1,
                                                       float* __restrict__ dw2, int B, int accumulate,
                                                       int probe_launch = 0) {
  constexpr int Cr = C / 16;
  __shared__ __attribute__((aligned(16))) f32x4 red[4][16][16];   // [wave][value][c-group]
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int cgp = lane & 15, bl = (lane >> 4) + 4 * wid;         // channel group, batch lane 0..15
  const int c4 = blockIdx.x * 64 + 4 * cgp, r0 = blockIdx.y * 8;
  f32x4 a2[8], a1[8];   // a2[rr] = dw2[c4..c4+3][r0+rr], a1[rr] = dw1[r0+rr][c4..c4+3]
#pragma unroll
  for (int rr = 0; rr < 8; ++rr) a2[rr] = a1[rr] = f32x4{0.f, 0.f, 0.f, 0.f};
  const __amdgpu_buffer_rsrc_t rds = mk_rsrc(dsig, (uint32_t)(B * C * 4)), rpo = mk_rsrc(pooled, (uint32_t)(B * C * 4));
  const __amdgpu_buffer_rsrc_t rhi = mk_rsrc(hid, (uint32_t)(B * Cr * 4)), rdh = mk_rsrc(dhid, (uint32_t)(B * Cr * 4));
  // device-scope (sc1) loads of the SE backward's small per-width buffers: with plain loads, a second
  // process on the device made this kernel's se.fc gradients differ run to run while the buffers
  // held identical values afterwards (tools/det_load.py)
  auto ldc = [](__amdgpu_buffer_rsrc_t r, size_t e) {
    return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, (uint32_t)(e * 4), 0, 16));
  };
#if CRNN_SE_PROBE
  float pin[4] = {0.f, 0.f, 0.f, 0.f};
#endif
  for (int bb = bl; bb < B; bb += 64) {   // 4 samples per lane per batch, all loads first
    f32x4 dv[4], pv[4], hv[4][2], dhv[4][2];
    float mk[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int b = min(bb + 16 * j, B - 1);   // clamped: the value is masked below
      mk[j] = bb + 16 * j < B ? 1.f : 0.f;
      dv[j] = ldc(rds, (size_t)b * C + c4);
      pv[j] = ldc(rpo, (size_t)b * C + c4);
#pragma unroll
      for (int hq = 0; hq < 2; ++hq) {
        hv[j][hq] = ldc(rhi, (size_t)b * Cr + r0 + 4 * hq);
        dhv[j][hq] = ldc(rdh, (size_t)b * Cr + r0 + 4 * hq);
      }
    }
#if CRNN_SE_PROBE
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        pin[0] += mk[j] * dv[j][e];
        pin[1] += mk[j] * pv[j][e];
        pin[2] += mk[j] * (hv[j][0][e] + hv[j][1][e]);
        pin[3] += mk[j] * (dhv[j][0][e] + dhv[j][1][e]);
      }
#endif
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const f32x4 dm = dv[j] * mk[j], pm = pv[j] * mk[j];
#pragma unroll
      for (int rr = 0; rr < 8; ++rr) {
        a2[rr] += dm * hv[j][rr >> 2][rr & 3];
        a1[rr] += dhv[j][rr >> 2][rr & 3] * pm;
      }
    }
  }
  // fold the 4 batch lanes of this wave (lane bits 4, 5), then the 4 waves
#pragma unroll
  for (int rr = 0; rr < 8; ++rr)
#pragma unroll
    for (int e = 0; e < 4; ++e)
#pragma unroll
      for (int o = 16; o < 64; o <<= 1) {
        a2[rr][e] += __shfl_xor(a2[rr][e], o, 64);
        a1[rr][e] += __shfl_xor(a1[rr][e], o, 64);
      }
  if (lane < 16)
#pragma unroll
    for (int rr = 0; rr < 8; ++rr) {
      red[wid][rr][cgp] = a2[rr];
      red[wid][8 + rr][cgp] = a1[rr];
    }
  __syncthreads();
  // finalise: thread (value k = tid / 16, c-group = tid % 16)
  const int k = threadIdx.x >> 4, cg2 = threadIdx.x & 15;
  const int rr = k & 7, r = r0 + rr, cc = blockIdx.x * 64 + 4 * cg2;
  const f32x4 v = red[0][k][cg2] + red[1][k][cg2] + red[2][k][cg2] + red[3][k][cg2];
  if (k < 8) {   // dw2[cc + e][r], stride Cr
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float* p = dw2 + (size_t)(cc + e) * Cr + r;
      *p = accumulate ? *p + v[e] : v[e];
    }
  } else {
    f32x4* p = reinterpret_cast<f32x4*>(dw1 + (size_t)r * C + cc);
    *p = accumulate ? *p + v : v;
  }
#if CRNN_SE_PROBE
  // block sums in a fixed order: per-thread values through LDS (red is free again after a barrier)
  __syncthreads();
  float* pr = reinterpret_cast<float*>(&red[0][0][0]);
#pragma unroll
  for (int q = 0; q < 4; ++q) pr[q * 256 + threadIdx.x] = pin[q];
  pr[4 * 256 + threadIdx.x] = k < 8 ? v[0] + v[1] + v[2] + v[3] : 0.f;
  pr[5 * 256 + threadIdx.x] = k < 8 ? 0.f : v[0] + v[1] + v[2] + v[3];
  __syncthreads();
  const int blk = blockIdx.y * gridDim.x + blockIdx.x;
  if (threadIdx.x < SE_PROBE_VALS && probe_launch < SE_PROBE_LAUNCHES && blk < SE_PROBE_BLOCKS) {
    float a = 0.f;
    for (int t = 0; t < 256; ++t) a += pr[threadIdx.x * 256 + t];
    g_se_probe[(probe_launch * SE_PROBE_BLOCKS + blk) * SE_PROBE_VALS + threadIdx.x] = a;
  }
#endif
}

// ------------------------------------------------------------ height collapse
template <typename T>
__global__ void hpool_fwd_kernel(const T* __restrict__ z, const float* __restrict__ sc, const float* __restrict__ sh,
                                 T* __restrict__ seq, int B, int Hh, int W, int C) {
  const int cg = C / 8;
  const long n = (long)B * W * cg;
  const float inv = 1.f / (float)Hh;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    int c8 = (int)(i % cg) * 8;
    long p = i / cg;
    int w = (int)(p % W), b = (int)(p / W);
    float acc[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) acc[k] = 0.f;
    for (int h = 0; h < Hh; ++h) {
      float v[8];
      unpack8<T>(ld8<T>(z + (((size_t)b * Hh + h) * W + w) * C + c8), v);
#pragma unroll
      for (int k = 0; k < 8; ++k) acc[k] += fmaxf(v[k] * sc[c8 + k] + sh[c8 + k], 0.f);
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) acc[k] *= inv;
    st8<T>(seq + ((size_t)b * W + w) * C + c8, pack8<T>(acc));
  }
}

template <typename T>
__global__ void hpool_bwd_kernel(const T* __restrict__ dseq, T* __restrict__ dy, int B, int Hh, int W, int C) {
  const int cg = C / 8;
  const long n = (long)B * Hh * W * cg;
  const float inv = 1.f / (float)Hh;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    int c8 = (int)(i % cg) * 8;
    long p = i / cg;
    int w = (int)(p % W);
    long q = p / W;
    int b = (int)(q / Hh);
    float v[8];
    unpack8<T>(ld8<T>(dseq + ((size_t)b * W + w) * C + c8), v);
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] *= inv;
    st8<T>(dy + p * C + c8, pack8<T>(v));
  }
}

// ------------------------------------------------------------ layout / packing
template <typename T>
__global__ void nchw_to_nhwc_kernel(const float* __restrict__ x, T* __restrict__ y, int B, int C, int H, int W, int Cp) {
  const long n = (long)B * H * W;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    long b = i / ((long)H * W), hw = i - b * H * W;
    if (Cp == 8 && C <= 8) {   // the encoder input: one 16-B (bf16) / 32-B (fp32) vector store per pixel
      float v[8];
#pragma unroll
      for (int c = 0; c < 8; ++c) v[c] = c < C ? x[(b * C + c) * H * W + hw] : 0.f;
      st8<T>(y + i * 8, pack8<T>(v));
      continue;
    }
    for (int c = 0; c < Cp; ++c) {
      float v = c < C ? x[(b * C + c) * H * W + hw] : 0.f;
      y[i * Cp + c] = fromf<T>(v);
    }
  }
}

template <typename T>
__global__ void cast_kernel(const float* __restrict__ s, T* __restrict__ d, long n) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    d[i] = fromf<T>(s[i]);
}

template <typename T>
__global__ void pack_conv_kernel(const float* __restrict__ w, T* __restrict__ o, int Co, int Ci, int KH, int KW, int Cip) {
  const long n = (long)Co * KH * KW * Cip;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    int ci = (int)(i % Cip);
    long t = i / Cip;
    int kw = (int)(t % KW);
    t /= KW;
    int kh = (int)(t % KH);
    int co = (int)(t / KH);
    float v = ci < Ci ? w[(((size_t)co * Ci + ci) * KH + kh) * KW + kw] : 0.f;
    o[i] = fromf<T>(v);
  }
}

template <typename T>
__global__ void pack_rows_kernel(const float* __restrict__ src, T* __restrict__ o, const int* __restrict__ perm,
                                 int rows_out, int rows_src, int cols) {
  const long n = (long)rows_out * cols;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    int r = (int)(i / cols), c = (int)(i - (long)r * cols);
    int sr = perm ? perm[r] : r;
    float v = (r < rows_src && sr >= 0) ? src[(size_t)sr * cols + c] : 0.f;
    o[i] = fromf<T>(v);
  }
}

// all pack jobs in one launch: block b owns elements [b*chunk, (b+1)*chunk) of the concatenation
// (chunk a multiple of 8) and walks the (start-sorted) job table from the job holding its first
// element. Jobs whose start and size are multiples of 8 (every job the engine builds) go 8 output
// elements per thread: 16-B stores, and for row gathers two 16-B source loads when the source is
// 16-B aligned (parameters are views into the flat buffer at arbitrary offsets, so checked per job);
// the transposed gathers (W_hh^T) read 8 rows of one column. Other jobs: one element per thread.
template <typename T>
__device__ __forceinline__ float pack_elem(const crnn_pack_job& jb, int i) {
  if (jb.kind == CRNN_PACK_CONV) {
    const int Ci = jb.b, KH = jb.c, KW = jb.d, Cip = jb.e;
    const int ci = i % Cip;
    int t = i / Cip;
    const int kw = t % KW;
    t /= KW;
    const int kh = t % KH, co = t / KH;
    return ci < Ci ? jb.src[(((size_t)co * Ci + ci) * KH + kh) * KW + kw] : 0.f;
  }
  if (jb.kind == CRNN_PACK_TRANSPOSE) {
    const int rows = jb.a;
    const int c = i / rows, r = i - c * rows;
    const int sr = jb.perm ? jb.perm[r] : r;
    return (r < jb.b && sr >= 0) ? jb.src[(size_t)sr * jb.c + c] : 0.f;
  }
  const int cols = jb.c;
  const int r = i / cols, c = i - r * cols;
  const int sr = jb.perm ? jb.perm[r] : r;
  const bool ok = r < jb.b && sr >= 0;
  float v = ok ? jb.src[(size_t)sr * cols + c] : 0.f;
  if (jb.kind == CRNN_PACK_ROWS_SUM && ok) v += jb.src2[(size_t)sr * cols + c];
  return v;
}

template <typename T>
__device__ __forceinline__ void pack_store8(const crnn_pack_job& jb, int i, const float* v) {
  if (jb.out_f32) {
    f32x4* d = reinterpret_cast<f32x4*>((float*)jb.dst + i);
    d[0] = f32x4{v[0], v[1], v[2], v[3]};
    d[1] = f32x4{v[4], v[5], v[6], v[7]};
  } else if constexpr (sizeof(T) == 2) {
    *reinterpret_cast<bf16x8*>((T*)jb.dst + i) = pack8<T>(v);
  } else {
    f32x4* d = reinterpret_cast<f32x4*>((T*)jb.dst + i);
    d[0] = f32x4{v[0], v[1], v[2], v[3]};
    d[1] = f32x4{v[4], v[5], v[6], v[7]};
  }
}

template <typename T>
__device__ __forceinline__ void pack_job8(const crnn_pack_job& jb, long a0, long a1) {
  const int kind = jb.kind;
  const bool rows = kind == CRNN_PACK_ROWS || kind == CRNN_PACK_ROWS_SUM;
  const int cols = jb.c;
  const bool vsrc = rows && cols % 8 == 0 && ((uintptr_t)jb.src & 15) == 0 &&
                    (kind != CRNN_PACK_ROWS_SUM || ((uintptr_t)jb.src2 & 15) == 0);
  for (long g = a0 + 8 * (long)threadIdx.x; g < a1; g += 8L * blockDim.x) {
    const int i = (int)(g - jb.start);
    float v[8];
    if (rows && cols % 8 == 0) {   // 8 consecutive columns of one row
      const int r = i / cols, c = i - r * cols;
      const int sr = jb.perm ? jb.perm[r] : r;
      const bool ok = r < jb.b && sr >= 0;
      const size_t o = (size_t)(ok ? sr : 0) * cols + c;
      if (vsrc) {
        f32x4 x0 = *reinterpret_cast<const f32x4*>(jb.src + o), x1 = *reinterpret_cast<const f32x4*>(jb.src + o + 4);
        if (kind == CRNN_PACK_ROWS_SUM) {
          x0 += *reinterpret_cast<const f32x4*>(jb.src2 + o);
          x1 += *reinterpret_cast<const f32x4*>(jb.src2 + o + 4);
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          v[q] = ok ? x0[q] : 0.f;
          v[4 + q] = ok ? x1[q] : 0.f;
        }
      } else {
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          float x = jb.src[o + q];
          if (kind == CRNN_PACK_ROWS_SUM) x += jb.src2[o + q];
          v[q] = ok ? x : 0.f;
        }
      }
    } else if (rows) {                // cols == 1: 8 consecutive rows (bias vectors)
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const int r = i + q;
        const int sr = jb.perm ? jb.perm[r] : r;
        const bool ok = r < jb.b && sr >= 0;
        float x = jb.src[ok ? sr : 0];
        if (kind == CRNN_PACK_ROWS_SUM) x += jb.src2[ok ? sr : 0];
        v[q] = ok ? x : 0.f;
      }
    } else {                          // transpose: 8 consecutive rows of one source column
      const int R = jb.a;
      const int c = i / R, r0 = i - c * R;
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const int r = r0 + q;
        const int sr = jb.perm ? jb.perm[r] : r;
        const bool ok = r < jb.b && sr >= 0;
        const float x = jb.src[(size_t)(ok ? sr : 0) * jb.c + c];
        v[q] = ok ? x : 0.f;
      }
    }
    pack_store8<T>(jb, i, v);
  }
}

template <typename T>
__global__ __launch_bounds__(256) void pack_batch_kernel(const crnn_pack_job* __restrict__ jobs, int njobs, long total,
                                                         long chunk) {
  const long e0 = blockIdx.x * chunk, e1 = min(total, e0 + chunk);
  if (e0 >= e1) return;
  int lo = 0, hi = njobs - 1;
  while (lo < hi) {  // last job with start <= e0
    const int mid = (lo + hi + 1) >> 1;
    if (jobs[mid].start <= e0) lo = mid;
    else hi = mid - 1;
  }
  for (int j = lo; j < njobs; ++j) {
    const crnn_pack_job jb = jobs[j];
    const long jend = j + 1 < njobs ? jobs[j + 1].start : total;
    const long a0 = max(e0, jb.start), a1 = min(e1, jend);
    if (a0 >= a1) {
      if (jb.start >= e1) break;
      continue;
    }
    const bool v8 = jb.start % 8 == 0 && jend % 8 == 0 && e0 % 8 == 0 && a1 % 8 == 0 &&
                    ((jb.kind == CRNN_PACK_ROWS || jb.kind == CRNN_PACK_ROWS_SUM) ? (jb.c % 8 == 0 || jb.c == 1)
                     : jb.kind == CRNN_PACK_TRANSPOSE ? jb.a % 8 == 0 : false);
    if (v8) {
      pack_job8<T>(jb, a0, a1);
      continue;
    }
    // element index inside a job fits 32 bits (the largest tensor is 2.4 M elements): 32-bit
    // divisions, not the 64-bit ones that dominated this kernel
    for (long g = a0 + threadIdx.x; g < a1; g += blockDim.x) {
      const int i = (int)(g - jb.start);
      const float v = pack_elem<T>(jb, i);
      if (jb.out_f32) ((float*)jb.dst)[i] = v;
      else ((T*)jb.dst)[i] = fromf<T>(v);
    }
  }
}

// conv weights, one block per output channel co: the OIHW source slab [Ci][KH][KW] (contiguous) is
// staged in LDS with coalesced reads, then written as the OHWI slab [KH][KW][Cip] (contiguous) —
// both sides coalesced, unlike the per-element gather of pack_batch_kernel (stride KH*KW reads).
// A 16-B aligned slab (every conv but the 3-channel input one) is read as 16-B vectors with all of
// a thread's loads in flight before its LDS stores (<= 5 per thread at Ci * KH * KW <= 5120), and
// the OHWI row is written 8 channels (16 B) per store: the scalar load-store loop ran at the memory
// latency (85 us per step for 42 M weights). LDS reads at stride KH*KW words: conflict-free for 3x3
// (9 is odd), 4-way at worst for 2x2.
template <typename T>
__global__ __launch_bounds__(256) void pack_conv_kernel(const crnn_pack_job* __restrict__ jobs, int njobs) {
  extern __shared__ float slab[];
  const long row = blockIdx.x;
  int lo = 0, hi = njobs - 1;
  while (lo < hi) {  // last job with start (first output channel) <= row
    const int mid = (lo + hi + 1) >> 1;
    if (jobs[mid].start <= row) lo = mid;
    else hi = mid - 1;
  }
  const crnn_pack_job jb = jobs[lo];
  const int co = (int)(row - jb.start), Ci = jb.b, KHW = jb.c * jb.d, Cip = jb.e;
  const int n = Ci * KHW;
  const float* src = jb.src + (size_t)co * n;
  constexpr int PER = 5;
  if (n % 4 == 0 && n <= 4 * 256 * PER && ((uintptr_t)src & 15) == 0) {
    f32x4 v[PER];
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      const int k = threadIdx.x + 256 * u;
      v[u] = *reinterpret_cast<const f32x4*>(src + 4 * (4 * k < n ? k : 0));   // clamped: unconditional
    }
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      const int k = threadIdx.x + 256 * u;
      if (4 * k < n) *reinterpret_cast<f32x4*>(&slab[4 * k]) = v[u];
    }
  } else {
    for (int i = threadIdx.x; i < n; i += blockDim.x) slab[i] = src[i];
  }
  __syncthreads();
  T* dst = (T*)jb.dst + (size_t)co * KHW * Cip;
  if (Cip % 8 == 0) {
    for (int i = 8 * threadIdx.x; i < KHW * Cip; i += 8 * blockDim.x) {
      const int t = i / Cip, c0 = i - t * Cip;
      float f[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) f[q] = c0 + q < Ci ? slab[(c0 + q) * KHW + t] : 0.f;
      if constexpr (sizeof(T) == 2) {
        *reinterpret_cast<bf16x8*>(dst + i) = pack8<T>(f);
      } else {
        *reinterpret_cast<f32x4*>(dst + i) = f32x4{f[0], f[1], f[2], f[3]};
        *reinterpret_cast<f32x4*>(dst + i + 4) = f32x4{f[4], f[5], f[6], f[7]};
      }
    }
  } else {
    for (int i = threadIdx.x; i < KHW * Cip; i += blockDim.x) {
      const int t = i / Cip, ci = i - t * Cip;
      dst[i] = fromf<T>(ci < Ci ? slab[ci * KHW + t] : 0.f);
    }
  }
}

// transposed, flipped conv kernel (crnn_conv_dgrad_tw's B operand): one workgroup per (64 co x 16 ci)
// tile of a job. With KH = KW = 1 and a row permutation it is a plain tiled transpose of a gathered
// matrix: the BiLSTM's W_hh'^T (perm = the gate interleave), whose per-element gather in
// pack_batch_kernel read one source column per block (32x L2 traffic). The source rows [co][ci0 .. ci0+15][KH*KW] are contiguous runs, read as 16-B vectors,
// all of a thread's loads in flight before its LDS stores (a load-store-load loop runs at the
// memory latency); LDS row pitch 16*KHW + 1 words (the read-back's 64 consecutive co on distinct
// banks); the destination rows [ci][tap'][co0 .. co0+63] are written as whole 128-B lines of
// consecutive co. KHW is a template parameter (3x3 and 2x2 kernels): no runtime divisions.
constexpr int PT_CO = 64, PT_CI = 16;
template <typename T, int KHW>
__device__ __forceinline__ void pack_conv_t_tile(const crnn_pack_job& jb, int tl, float* tile) {
  const int Co = jb.a, Ci = jb.b;
  const int tci = (Ci + PT_CI - 1) / PT_CI;
  const int co0 = (tl / tci) * PT_CO, ci0 = (tl % tci) * PT_CI;
  const int nco = min(PT_CO, Co - co0);
  constexpr int RUN = PT_CI * KHW, V4 = RUN / 4, P = RUN + 1, NV = PT_CO * V4;
  constexpr int PER = (NV + 255) / 256;
  f32x4 v[PER];
#pragma unroll
  for (int u = 0; u < PER; ++u) {
    const int k = threadIdx.x + 256 * u, r = k / V4, e = k - r * V4;
    const int rr = (k < NV && r < nco) ? r : 0;   // clamped: every load unconditional
    const int srow = jb.perm ? jb.perm[co0 + rr] : co0 + rr;   // row gather (BiLSTM gate order)
    v[u] = *reinterpret_cast<const f32x4*>(jb.src + ((size_t)srow * Ci + ci0) * KHW + 4 * e);
  }
#pragma unroll
  for (int u = 0; u < PER; ++u) {
    const int k = threadIdx.x + 256 * u, r = k / V4, e = k - r * V4;
    if (k < NV)
#pragma unroll
      for (int q = 0; q < 4; ++q) tile[r * P + 4 * e + q] = r < nco ? v[u][q] : 0.f;
  }
  __syncthreads();
  T* dst = (T*)jb.dst;
  // 8 consecutive co per thread: one 16-B (bf16) store instead of eight 2-B ones
  constexpr int G = PT_CO / 8, NR = RUN * G;
  const bool vec = (Co & 7) == 0;
#pragma unroll
  for (int u = 0; u < (NR + 255) / 256; ++u) {
    const int i = threadIdx.x + 256 * u;
    const int cb = 8 * (i % G), rest = i / G;
    const int tp = rest % KHW, ci = rest / KHW;   // destination tap (flipped source tap KHW-1-tp)
    if (i < NR && cb < nco) {
      float f[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) f[q] = tile[(cb + q) * P + ci * KHW + (KHW - 1 - tp)];
      T* o = dst + ((size_t)(ci0 + ci) * KHW + tp) * Co + co0 + cb;
      if (vec && cb + 8 <= nco) {
        st8<T>(o, pack8<T>(f));
      } else {
        for (int q = 0; q < 8 && cb + q < nco; ++q) o[q] = fromf<T>(f[q]);
      }
    }
  }
  if (jb.dst2) {   // the plain OHWI pack of the same tile: rows (co, tap) of 16 ci, two 8-channel pieces each
    T* d2 = (T*)jb.dst2;
    constexpr int NS = PT_CO * KHW * 2;
#pragma unroll
    for (int u = 0; u < (NS + 255) / 256; ++u) {
      const int k = threadIdx.x + 256 * u;
      const int hf = k & 1, rest = k >> 1, tp = rest % KHW, co = rest / KHW;
      if (k < NS && co < nco) {
        float f[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) f[q] = tile[co * P + (8 * hf + q) * KHW + tp];
        st8<T>(d2 + ((size_t)(co0 + co) * KHW + tp) * Ci + ci0 + 8 * hf, pack8<T>(f));
      }
    }
  }
}

template <typename T>
__global__ __launch_bounds__(256) void pack_conv_t_kernel(const crnn_pack_job* __restrict__ jobs, int njobs) {
  __shared__ float tile[PT_CO * (PT_CI * 9 + 1)];   // KH*KW <= 9 (the header's contract)
  const long bid = blockIdx.x;
  int lo = 0, hi = njobs - 1;
  while (lo < hi) {  // last job with start (first tile) <= bid
    const int mid = (lo + hi + 1) >> 1;
    if (jobs[mid].start <= bid) lo = mid;
    else hi = mid - 1;
  }
  const crnn_pack_job jb = jobs[lo];
  const int KHW = jb.c * jb.d, tl = (int)(bid - jb.start);
  if (jb.b % PT_CI) return;   // the header's contract: Ci % 16 == 0 (16-B source rows)
  if (KHW == 9) pack_conv_t_tile<T, 9>(jb, tl, tile);
  else if (KHW == 4) pack_conv_t_tile<T, 4>(jb, tl, tile);
  else if (KHW == 1) pack_conv_t_tile<T, 1>(jb, tl, tile);
}

// ------------------------------------------------------------ dropout (enc_dropout, model/model.py:201,220)
// Counter-based: element i of a call with seed s is kept iff hash(s, i) >= p * 2^32, so the
// backward regenerates the forward's mask from (seed, index) and nothing is stored. The hash is
// splitmix64's finalizer on s ^ (i * golden ratio); torch's Philox stream is not reproduced (the
// masks are equal in distribution, not bit for bit). drop_hash: common.hpp.
template <typename T>
__global__ void dropout_kernel(const T* __restrict__ x, T* __restrict__ y, long n, uint32_t thr, float scale,
                               unsigned long long seed) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    y[i] = fromf<T>(drop_hash(seed, (unsigned long long)i) >= thr ? tof(x[i]) * scale : 0.f);
}

// ------------------------------------------------------------ DropBlock2d (model/seresnet31.py:49-53,62)
// torchvision.ops.drop_block2d in training mode, restated: bs = min(block_size, H, W); the seeds of
// each (n, c) plane live on the (H-bs+1) x (W-bs+1) grid and are Bernoulli(gamma) with gamma =
// p*H*W / (bs^2 (H-bs+1)(W-bs+1)); a seed at (i, j) zeroes rows i..i+bs-1, cols j..j+bs-1 (the
// padded bs x bs stride-1 max-pool of the seed map); the kept elements are scaled by numel /
// (1e-6 + kept). Seed (n, c, i, j) is drawn as drop_hash(seed, ((n*C + c)*Hs + i)*Ws + j) < thr:
// counter based, so the backward reuses the stored keep bytes and a test regenerates the mask
// (oracle: dropblock_keep); torch's Philox stream is not reproduced.
// Thread = (pixel, 8-channel group) of the NHWC map; keep is u8 [B][H][W][C]; *kept counts the
// kept elements (an integer sum: the total does not depend on the order of the adds).
__global__ __launch_bounds__(256) void dropblock_mask_kernel(uint8_t* __restrict__ keep,
                                                             unsigned long long* __restrict__ kept, int H, int W, int C,
                                                             int bs, uint32_t thr, unsigned long long seed,
                                                             long total8) {
  const int C8 = C >> 3, Hs = H - bs + 1, Ws = W - bs + 1;
  unsigned int nk = 0;
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < total8; e += (long)gridDim.x * blockDim.x) {
    const long pix = e / C8;
    const int c0 = (int)(e - pix * C8) * 8;
    const int w = (int)(pix % W);
    const long nh = pix / W;
    const int h = (int)(nh % H);
    const long n = nh / H;
    const int i0 = max(0, h - bs + 1), i1 = min(h, Hs - 1), j0 = max(0, w - bs + 1), j1 = min(w, Ws - 1);
    uint64_t kb = 0;
    for (int k = 0; k < 8; ++k) {
      const unsigned long long plane = (unsigned long long)(n * C + c0 + k) * Hs;
      bool drop = false;
      for (int i = i0; i <= i1 && !drop; ++i)
        for (int j = j0; j <= j1 && !drop; ++j) drop = drop_hash(seed, (plane + i) * Ws + j) < thr;
      if (!drop) {
        kb |= 1ull << (8 * k);
        ++nk;
      }
    }
    *reinterpret_cast<uint64_t*>(keep + e * 8) = kb;
  }
  for (int off = 32; off > 0; off >>= 1) nk += __shfl_xor(nk, off);
  if ((threadIdx.x & 63) == 0 && nk) atomicAdd(kept, (unsigned long long)nk);
}

// y = x * keep * numel / (1e-6 + kept), 8 elements per thread (the backward's SE-side gradient)
template <typename T>
__global__ __launch_bounds__(256) void dropblock_apply_kernel(const T* __restrict__ x, T* __restrict__ y,
                                                              const uint8_t* __restrict__ keep,
                                                              const unsigned long long* __restrict__ kept, long n8) {
  const float scale = (float)(n8 * 8) / (1e-6f + (float)*kept);
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < n8; e += (long)gridDim.x * blockDim.x) {
    const uint64_t kb = *reinterpret_cast<const uint64_t*>(keep + e * 8);
    float v[8];
    unpack8<T>(ld8<T>(x + e * 8), v);
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = ((kb >> (8 * i)) & 0xff) ? v[i] * scale : 0.f;
    st8<T>(y + e * 8, pack8<T>(v));
  }
}

// ------------------------------------------------------------ row-streaming elementwise kernels
// Thread = (8-channel group c8, row lane r): the group is fixed for the thread's lifetime so
// per-channel coefficients live in registers; a block streams a contiguous chunk of rows
// (per-sample SE values are re-fetched only when the row crosses into the next sample).
struct RowMap {
  int cg, rl, c8, r;
};
__device__ __forceinline__ RowMap rowmap(int C) {
  RowMap q;
  q.cg = C >> 3;
  q.rl = NT / q.cg;
  q.c8 = (threadIdx.x % q.cg) * 8;
  q.r = threadIdx.x / q.cg;
  return q;
}

__device__ __forceinline__ void ld8f(const float* p, float* o) {
  f32x4 a = *reinterpret_cast<const f32x4*>(p), b = *reinterpret_cast<const f32x4*>(p + 4);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    o[i] = a[i];
    o[4 + i] = b[i];
  }
}

// upstream gradient g by mode, with per-thread cached channel / sample constants
template <typename T, int MODE>
__device__ __forceinline__ void bng(const crnn_bn_bwd_desc& d, size_t o, const float* z, const float* sc,
                                    const float* sh, const float* s8, const float* dp8, float* g) {
  float dy[8];
  unpack8<T>(ld8<T>((const T*)d.dy + o), dy);
  if constexpr (MODE == CRNN_BNG_PLAIN) {
#pragma unroll
    for (int i = 0; i < 8; ++i) g[i] = dy[i];
  } else if constexpr (MODE == CRNN_BNG_RELU) {
#pragma unroll
    for (int i = 0; i < 8; ++i) g[i] = (z[i] * sc[i] + sh[i]) > 0.f ? dy[i] : 0.f;
  } else {
    float y[8];
    unpack8<T>(ld8<T>((const T*)d.y + o), y);
    if constexpr (MODE == CRNN_BNG_RESID) {
#pragma unroll
      for (int i = 0; i < 8; ++i) g[i] = y[i] > 0.f ? dy[i] : 0.f;
    } else {
#pragma unroll
      for (int i = 0; i < 8; ++i) g[i] = (y[i] > 0.f ? dy[i] * s8[i] : 0.f) + dp8[i];
    }
  }
}

// CRNN_BNG_POOL — BN -> ReLU -> MaxPool2d(2,2) of the stem (model/seresnet31.py:83-88) with the
// max-pool backward fused in: d.dy is the POOLED gradient [B][H/2][W/2][C] and d.HW the full-res
// width W. Window i (pooled pixel) covers full-res rows (2*(i / Wo) + dh) * W + 2*(i % Wo) + dw; the
// gradient of each row is dpool at the window's first maximum of relu(z*scale+shift) (torch's
// max_pool2d index, scan order h then w) when that value is > 0, else 0.
template <typename T>
__device__ __forceinline__ void pool_window(const crnn_bn_bwd_desc& d, const FastDiv& dWo, long i, int c8,
                                            const float* sc, const float* sh, float (&z)[4][8], float (&g)[4][8],
                                            size_t (&o)[4]) {
  uint32_t wo;
  const uint32_t bho = dWo.divmod((uint32_t)i, wo);
  const int W = d.HW;
  float best[8];
  int arg[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    best[k] = -INFINITY;
    arg[k] = 0;
  }
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    o[t] = ((size_t)(2 * bho + (t >> 1)) * W + 2 * wo + (t & 1)) * d.C + c8;
    unpack8<T>(ld8<T>((const T*)d.z + o[t]), z[t]);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const float v = fmaxf(z[t][k] * sc[k] + sh[k], 0.f);
      if (v > best[k]) {
        best[k] = v;
        arg[k] = t;
      }
    }
  }
  float dp[8];
  unpack8<T>(ld8<T>((const T*)d.dy + (size_t)i * d.C + c8), dp);
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int k = 0; k < 8; ++k) g[t][k] = (arg[k] == t && z[t][k] * sc[k] + sh[k] > 0.f) ? dp[k] : 0.f;
}

// CRNN_BNG_POOL_OUT: the pool-mode sums from the pooled output y and the pooled gradient dy (one row
// per window): y > 0 means the window's first maximum got dy, and that maximum's z is (y - shift) /
// scale. That z carries y's bf16 rounding: an xhat error of 2^-8 |xhat + beta/gamma|, which grows with
// |beta/gamma| as BN parameters train. A thread whose 8 channels include one with
// |beta/gamma| > POOL_OUT_BG (or scale == 0: all four values tie at relu(shift)) takes the full
// window from z instead (CRNN_BNG_POOL's arithmetic for those rows); the common path never touches
// the full-resolution tensor.
constexpr float POOL_OUT_BG = 4.f;
template <typename T>
__global__ __launch_bounds__(NT) void bnb_reduce_pool_out_kernel(crnn_bn_bwd_desc d, FastDiv dWo, long rpb,
                                                                 float* __restrict__ p0, float* __restrict__ p1) {
  extern __shared__ float red[];  // [2][rl][C]
  const int C = d.C;
  const RowMap q = rowmap(C);
  float mean[8], inv[8], sc[8], sh[8], rsc[8], a0[8], a1[8];
  ld8f(d.mean + q.c8, mean);
  ld8f(d.invstd + q.c8, inv);
  ld8f(d.scale + q.c8, sc);
  ld8f(d.shift + q.c8, sh);
  bool wide = false;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    a0[i] = a1[i] = 0.f;
    // beta / gamma = (shift + mean * scale) * invstd / scale
    wide |= sc[i] == 0.f || fabsf((sh[i] + mean[i] * sc[i]) * inv[i]) > POOL_OUT_BG * fabsf(sc[i]);
    rsc[i] = sc[i] != 0.f ? 1.f / sc[i] : 0.f;
  }
  const long mend = d.M / 4;
  const long m0 = blockIdx.x * rpb, m1 = min(mend, m0 + rpb);
  if (__builtin_expect(wide, 0)) {
    for (long m = m0 + q.r; m < m1; m += q.rl) {
      float z[4][8], g[4][8];
      size_t o[4];
      pool_window<T>(d, dWo, m, q.c8, sc, sh, z, g, o);
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          a0[i] += g[t][i];
          a1[i] += g[t][i] * ((z[t][i] - mean[i]) * inv[i]);
        }
    }
  } else {
    for (long m = m0 + q.r; m < m1; m += q.rl) {
      const size_t o = (size_t)m * C + q.c8;
      float y[8], dp[8];
      unpack8<T>(ld8<T>((const T*)d.y + o), y);
      unpack8<T>(ld8<T>((const T*)d.dy + o), dp);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const float g = y[i] > 0.f ? dp[i] : 0.f;
        const float z = (y[i] - sh[i]) * rsc[i];
        a0[i] += g;
        a1[i] += g * ((z - mean[i]) * inv[i]);
      }
    }
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    red[q.r * C + q.c8 + i] = a0[i];
    red[(q.rl + q.r) * C + q.c8 + i] = a1[i];
  }
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += NT) {
    float s0 = 0.f, s1 = 0.f;
    for (int k = 0; k < q.rl; ++k) {
      s0 += red[k * C + c];
      s1 += red[(q.rl + k) * C + c];
    }
    p0[(size_t)blockIdx.x * C + c] = s0;
    p1[(size_t)blockIdx.x * C + c] = s1;
  }
}

template <typename T, int MODE>
__global__ __launch_bounds__(NT) void bnb_reduce_kernel(crnn_bn_bwd_desc d, FastDiv dHW, long rpb,
                                                        float* __restrict__ p0, float* __restrict__ p1) {
  extern __shared__ float red[];  // [2][rl][C]
  const int C = d.C;
  const RowMap q = rowmap(C);
  float mean[8], inv[8], sc[8], sh[8], s8[8], dp8[8], a0[8], a1[8];
  ld8f(d.mean + q.c8, mean);
  ld8f(d.invstd + q.c8, inv);
  if (MODE == CRNN_BNG_RELU || MODE == CRNN_BNG_POOL) {
    ld8f(d.scale + q.c8, sc);
    ld8f(d.shift + q.c8, sh);
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) a0[i] = a1[i] = 0.f;
  const long mend = MODE == CRNN_BNG_POOL ? d.M / 4 : d.M;  // pool mode: rows = windows
  const long m0 = blockIdx.x * rpb, m1 = min(mend, m0 + rpb);
  uint32_t cb = 0xffffffffu;
  if constexpr (MODE == CRNN_BNG_POOL) {
    for (long m = m0 + q.r; m < m1; m += q.rl) {
      float z[4][8], g[4][8];
      size_t o[4];
      pool_window<T>(d, dHW, m, q.c8, sc, sh, z, g, o);
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          a0[i] += g[t][i];
          a1[i] += g[t][i] * ((z[t][i] - mean[i]) * inv[i]);
        }
    }
  } else
  for (long m = m0 + q.r; m < m1; m += q.rl) {
    const size_t o = (size_t)m * C + q.c8;
    if constexpr (MODE == CRNN_BNG_SE) {
      const uint32_t bb = dHW.div((uint32_t)m);
      if (bb != cb) {
        cb = bb;
        ld8f(d.s + (size_t)bb * C + q.c8, s8);
        ld8f(d.dpool + (size_t)bb * C + q.c8, dp8);
      }
    }
    float z[8], g[8];
    unpack8<T>(ld8<T>((const T*)d.z + o), z);
    bng<T, MODE>(d, o, z, sc, sh, s8, dp8, g);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      a0[i] += g[i];
      a1[i] += g[i] * ((z[i] - mean[i]) * inv[i]);
    }
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    red[q.r * C + q.c8 + i] = a0[i];
    red[(q.rl + q.r) * C + q.c8 + i] = a1[i];
  }
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += NT) {
    float s0 = 0.f, s1 = 0.f;
    for (int k = 0; k < q.rl; ++k) {
      s0 += red[k * C + c];
      s1 += red[(q.rl + k) * C + c];
    }
    p0[(size_t)blockIdx.x * C + c] = s0;
    p1[(size_t)blockIdx.x * C + c] = s1;
  }
}

// dz = A g - Bx xhat - Cg with A = scale, Bx = scale*mgx, Cg = scale*mg, xhat = (z - mean)*invstd.
// (Folding xhat into z-coefficients would cancel catastrophically on channels with |mean| >> std.)
template <typename T, int MODE>
__global__ __launch_bounds__(NT) void bnb_apply_kernel(crnn_bn_bwd_desc d, FastDiv dHW, const float* __restrict__ mg,
                                                       const float* __restrict__ mgx, T* __restrict__ dz, long rpb) {
  const int C = d.C;
  const RowMap q = rowmap(C);
  float A[8], Bx[8], Cg[8], mean[8], inv[8], sc[8], sh[8], s8[8], dp8[8];
  {
    float g1[8], g2[8];
    ld8f(d.mean + q.c8, mean);
    ld8f(d.invstd + q.c8, inv);
    ld8f(d.scale + q.c8, A);
    ld8f(mg + q.c8, g1);
    ld8f(mgx + q.c8, g2);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      Bx[i] = A[i] * g2[i];
      Cg[i] = A[i] * g1[i];
    }
  }
  if (MODE == CRNN_BNG_RELU || MODE == CRNN_BNG_POOL) {
    ld8f(d.scale + q.c8, sc);
    ld8f(d.shift + q.c8, sh);
  }
  const long mend = MODE == CRNN_BNG_POOL ? d.M / 4 : d.M;
  const long m0 = blockIdx.x * rpb, m1 = min(mend, m0 + rpb);
  uint32_t cb = 0xffffffffu;
  if constexpr (MODE == CRNN_BNG_POOL) {
    for (long m = m0 + q.r; m < m1; m += q.rl) {
      float z[4][8], g[4][8];
      size_t o[4];
      pool_window<T>(d, dHW, m, q.c8, sc, sh, z, g, o);
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        float out[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) out[i] = A[i] * g[t][i] - Bx[i] * ((z[t][i] - mean[i]) * inv[i]) - Cg[i];
        st8<T>(dz + o[t], pack8<T>(out));
      }
    }
    return;
  }
  for (long m = m0 + q.r; m < m1; m += q.rl) {
    const size_t o = (size_t)m * C + q.c8;
    if constexpr (MODE == CRNN_BNG_SE) {
      const uint32_t bb = dHW.div((uint32_t)m);
      if (bb != cb) {
        cb = bb;
        ld8f(d.s + (size_t)bb * C + q.c8, s8);
        ld8f(d.dpool + (size_t)bb * C + q.c8, dp8);
      }
    }
    float z[8], g[8], out[8];
    unpack8<T>(ld8<T>((const T*)d.z + o), z);
    bng<T, MODE>(d, o, z, sc, sh, s8, dp8, g);
#pragma unroll
    for (int i = 0; i < 8; ++i) out[i] = A[i] * g[i] - Bx[i] * ((z[i] - mean[i]) * inv[i]) - Cg[i];
    st8<T>(dz + o, pack8<T>(out));
  }
}

// DROP: the block's DropBlock2d between the SE gate and the residual add (model/seresnet31.py:61-62):
// the SE output is multiplied by keep * numel / (1e-6 + kept) (dropblock_mask_kernel below).
template <typename T, bool DROP>
__global__ __launch_bounds__(NT) void se_residual2_kernel(const T* __restrict__ z, const float* __restrict__ scp,
                                                          const float* __restrict__ shp, const float* __restrict__ s,
                                                          const T* __restrict__ idn, const float* __restrict__ iscp,
                                                          const float* __restrict__ ishp, T* __restrict__ y, long M,
                                                          int C, FastDiv dHW, long rpb,
                                                          const uint8_t* __restrict__ keep,
                                                          const unsigned long long* __restrict__ kept) {
  const RowMap q = rowmap(C);
  float sc[8], sh[8], isc[8], ish[8], s8[8];
  float dscale = 1.f;
  if constexpr (DROP) dscale = (float)(M * C) / (1e-6f + (float)*kept);
  ld8f(scp + q.c8, sc);
  ld8f(shp + q.c8, sh);
  if (iscp) {
    ld8f(iscp + q.c8, isc);
    ld8f(ishp + q.c8, ish);
  } else {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      isc[i] = 1.f;
      ish[i] = 0.f;
    }
  }
  const long m0 = blockIdx.x * rpb, m1 = min(M, m0 + rpb);
  uint32_t cb = 0xffffffffu;
  for (long m = m0 + q.r; m < m1; m += q.rl) {
    const uint32_t bb = dHW.div((uint32_t)m);
    if (bb != cb) {
      cb = bb;
      ld8f(s + (size_t)bb * C + q.c8, s8);
    }
    const size_t o = (size_t)m * C + q.c8;
    float v[8], dd[8];
    unpack8<T>(ld8<T>(z + o), v);
    unpack8<T>(ld8<T>(idn + o), dd);
    float km[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) km[i] = s8[i];
    if constexpr (DROP) {
      const uint64_t kb = *reinterpret_cast<const uint64_t*>(keep + o);
#pragma unroll
      for (int i = 0; i < 8; ++i) km[i] = ((kb >> (8 * i)) & 0xff) ? s8[i] * dscale : 0.f;
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = fmaxf((v[i] * sc[i] + sh[i]) * km[i] + dd[i] * isc[i] + ish[i], 0.f);
    st8<T>(y + o, pack8<T>(v));
  }
}

template <typename T>
__global__ __launch_bounds__(NT) void bn_act2_kernel(const T* __restrict__ z, const float* __restrict__ scp,
                                                     const float* __restrict__ shp, T* __restrict__ y, long M, int C,
                                                     int relu, long rpb) {
  const RowMap q = rowmap(C);
  float sc[8], sh[8];
  ld8f(scp + q.c8, sc);
  ld8f(shp + q.c8, sh);
  const long m0 = blockIdx.x * rpb, m1 = min(M, m0 + rpb);
  for (long m = m0 + q.r; m < m1; m += q.rl) {
    const size_t o = (size_t)m * C + q.c8;
    float v[8];
    unpack8<T>(ld8<T>(z + o), v);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      v[i] = v[i] * sc[i] + sh[i];
      if (relu) v[i] = fmaxf(v[i], 0.f);
    }
    st8<T>(y + o, pack8<T>(v));
  }
}

// per-sample spatial reductions with hoisted channel constants; block per sample
template <typename T, int KIND>  // KIND 0: SE pool (mean of z*sc+sh); 1: SE bwd (sum dy*(y>0)*(z*sc+sh))
__global__ __launch_bounds__(NT) void se_reduce_kernel(const T* __restrict__ z, const float* __restrict__ scp,
                                                       const float* __restrict__ shp, const T* __restrict__ dy,
                                                       const T* __restrict__ y, int HW, int C,
                                                       float* __restrict__ out, float mul) {
  extern __shared__ float red[];
  const RowMap q = rowmap(C);
  const int b = blockIdx.x;
  float sc[8], sh[8], a[8];
  ld8f(scp + q.c8, sc);
  ld8f(shp + q.c8, sh);
#pragma unroll
  for (int i = 0; i < 8; ++i) a[i] = 0.f;
  for (int hw = q.r; hw < HW; hw += q.rl) {
    const size_t o = ((size_t)b * HW + hw) * C + q.c8;
    float v[8];
    unpack8<T>(ld8<T>(z + o), v);
    if constexpr (KIND == 0) {
#pragma unroll
      for (int i = 0; i < 8; ++i) a[i] += v[i] * sc[i] + sh[i];
    } else {
      float dd[8], yy[8];
      unpack8<T>(ld8<T>(dy + o), dd);
      unpack8<T>(ld8<T>(y + o), yy);
#pragma unroll
      for (int i = 0; i < 8; ++i) a[i] += yy[i] > 0.f ? dd[i] * (v[i] * sc[i] + sh[i]) : 0.f;
    }
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) red[q.r * C + q.c8 + i] = a[i];
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += NT) {
    float s = 0.f;
    for (int k = 0; k < q.rl; ++k) s += red[k * C + c];
    out[(size_t)b * C + c] = s * mul;
  }
}

// SE squeeze from the conv's BatchNorm partial sums (training forward): when the partial rows
// (rpp data rows each, conv.hip's FwdEpi / halo layout) tile every sample's HW rows exactly,
// sum_hw z[b][c] is the sum of the sample's partial rows, so pooled = scale * that / HW + shift
// needs no pass over z. Block per sample, thread per channel.
__global__ void se_pool_partials_kernel(const float* __restrict__ psum, int per_b, const float* __restrict__ scale,
                                        const float* __restrict__ shift, float* __restrict__ pooled, int HW, int C) {
  const int b = blockIdx.x;
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    float s = 0.f;
    for (int k = 0; k < per_b; ++k) s += psum[((size_t)b * per_b + k) * C + c];
    pooled[(size_t)b * C + c] = scale[c] * (s / (float)HW) + shift[c];
  }
}

// SE block backward, one pass for both reductions over the tensor (block per sample b):
//   dy_m = dy * (y > 0), xhat = (z - mean) * invstd
//   A = sum_hw dy_m, Bx = sum_hw dy_m xhat, Cx = sum_hw xhat        -> abc[b][3][C]
//   ds[b][c] = sum_hw dy_m (z scale + shift) = gamma Bx + beta A     (the SE gate gradient)
// The BN sums of g = dy_m s + dpool (CRNN_BNG_SE) then follow per sample without a second pass
// (se_bn_partials_kernel): sum g = s A + HW dpool, sum g xhat = s Bx + dpool Cx.
template <typename T>
__global__ __launch_bounds__(NT) void se_bn_bwd_reduce_kernel(const T* __restrict__ dy, const T* __restrict__ y,
                                                              const T* __restrict__ z, const float* __restrict__ meanp,
                                                              const float* __restrict__ invp,
                                                              const float* __restrict__ gamma,
                                                              const float* __restrict__ beta, int HW, int C,
                                                              float* __restrict__ ds, float* __restrict__ abc) {
  extern __shared__ float red[];  // [3][rl][C]
  const RowMap q = rowmap(C);
  const int b = blockIdx.x;
  float mean[8], inv[8], a[8], bx[8], cx[8];
  ld8f(meanp + q.c8, mean);
  ld8f(invp + q.c8, inv);
#pragma unroll
  for (int i = 0; i < 8; ++i) a[i] = bx[i] = cx[i] = 0.f;
  for (int hw = q.r; hw < HW; hw += q.rl) {
    const size_t o = ((size_t)b * HW + hw) * C + q.c8;
    float zz[8], dd[8], yy[8];
    unpack8<T>(ld8<T>(z + o), zz);
    unpack8<T>(ld8<T>(dy + o), dd);
    unpack8<T>(ld8<T>(y + o), yy);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const float xh = (zz[i] - mean[i]) * inv[i];
      const float dm = yy[i] > 0.f ? dd[i] : 0.f;
      a[i] += dm;
      bx[i] += dm * xh;
      cx[i] += xh;
    }
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    red[q.r * C + q.c8 + i] = a[i];
    red[(q.rl + q.r) * C + q.c8 + i] = bx[i];
    red[(2 * q.rl + q.r) * C + q.c8 + i] = cx[i];
  }
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += NT) {
    float s0 = 0.f, s1 = 0.f, s2 = 0.f;
    for (int k = 0; k < q.rl; ++k) {
      s0 += red[k * C + c];
      s1 += red[(q.rl + k) * C + c];
      s2 += red[(2 * q.rl + k) * C + c];
    }
    float* o = abc + (size_t)b * 3 * C;
    o[c] = s0;
    o[C + c] = s1;
    o[2 * C + c] = s2;
    ds[(size_t)b * C + c] = gamma[c] * s1 + beta[c] * s0;
  }
}

__global__ void se_bn_partials_kernel(const float* __restrict__ abc, const float* __restrict__ sg,
                                      const float* __restrict__ dpool, int HW, int C, float* __restrict__ p0,
                                      float* __restrict__ p1) {
  const int b = blockIdx.x;
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    const float* o = abc + (size_t)b * 3 * C;
    const float sv = sg[(size_t)b * C + c], dp = dpool[(size_t)b * C + c];
    p0[(size_t)b * C + c] = sv * o[c] + (float)HW * dp;
    p1[(size_t)b * C + c] = sv * o[C + c] + dp * o[2 * C + c];
  }
}

inline bool rowmap_ok(int C) { return C % 8 == 0 && C / 8 <= NT && NT % (C / 8) == 0; }

// blocks for a row-streaming launch: enough to fill the chip, each a contiguous row chunk
inline void stream_grid(long M, int C, int* blocks, long* rpb) {
  const int rl = NT / (C / 8);
  long nb = (M + rl * 8 - 1) / (rl * 8);  // >= 8 rows per thread
  if (nb > 4096) nb = 4096;
  if (nb < 1) nb = 1;
  *rpb = (M + nb - 1) / nb;
  *blocks = (int)((M + *rpb - 1) / *rpb);
}

#define DISPATCH(dtype, ...)            \
  if ((dtype) == CRNN_BF16) {           \
    using T = bf16;                     \
    __VA_ARGS__;                        \
  } else {                              \
    using T = float;                    \
    __VA_ARGS__;                        \
  }

}  // namespace

namespace {
template <typename T>
int bnb_reduce_launch(const crnn_bn_bwd_desc* d, float* pg, float* pgx, int rows, hipStream_t st) {
  const bool pool = d->mode == CRNN_BNG_POOL || d->mode == CRNN_BNG_POOL_OUT;
  const long rpb = ((pool ? d->M / 4 : d->M) + rows - 1) / rows;
  const int rl = NT / (d->C / 8);
  const size_t sm = (size_t)2 * rl * d->C * sizeof(float);
  const FastDiv dHW(pool ? d->HW / 2 : (d->HW > 0 ? d->HW : 1));  // pool mode: pooled width Wo
  switch (d->mode) {
    case CRNN_BNG_POOL:
      hipLaunchKernelGGL((bnb_reduce_kernel<T, CRNN_BNG_POOL>), dim3(rows), dim3(NT), sm, st, *d, dHW, rpb, pg, pgx);
      break;
    case CRNN_BNG_POOL_OUT:
      hipLaunchKernelGGL((bnb_reduce_pool_out_kernel<T>), dim3(rows), dim3(NT), sm, st, *d, dHW, rpb, pg, pgx);
      break;
    case CRNN_BNG_PLAIN:
      hipLaunchKernelGGL((bnb_reduce_kernel<T, CRNN_BNG_PLAIN>), dim3(rows), dim3(NT), sm, st, *d, dHW, rpb, pg, pgx);
      break;
    case CRNN_BNG_RELU:
      hipLaunchKernelGGL((bnb_reduce_kernel<T, CRNN_BNG_RELU>), dim3(rows), dim3(NT), sm, st, *d, dHW, rpb, pg, pgx);
      break;
    case CRNN_BNG_RESID:
      hipLaunchKernelGGL((bnb_reduce_kernel<T, CRNN_BNG_RESID>), dim3(rows), dim3(NT), sm, st, *d, dHW, rpb, pg, pgx);
      break;
    default:
      hipLaunchKernelGGL((bnb_reduce_kernel<T, CRNN_BNG_SE>), dim3(rows), dim3(NT), sm, st, *d, dHW, rpb, pg, pgx);
  }
  return (int)hipGetLastError();
}

template <typename T>
int bnb_apply_launch(const crnn_bn_bwd_desc* d, const float* mg, const float* mgx, void* dz, hipStream_t st) {
  int nb;
  long rpb;
  const bool pool = d->mode == CRNN_BNG_POOL;
  stream_grid(pool ? d->M / 4 : d->M, d->C, &nb, &rpb);
  const FastDiv dHW(pool ? d->HW / 2 : (d->HW > 0 ? d->HW : 1));
  switch (d->mode) {
    case CRNN_BNG_POOL:
      hipLaunchKernelGGL((bnb_apply_kernel<T, CRNN_BNG_POOL>), dim3(nb), dim3(NT), 0, st, *d, dHW, mg, mgx, (T*)dz, rpb);
      break;
    case CRNN_BNG_PLAIN:
      hipLaunchKernelGGL((bnb_apply_kernel<T, CRNN_BNG_PLAIN>), dim3(nb), dim3(NT), 0, st, *d, dHW, mg, mgx, (T*)dz, rpb);
      break;
    case CRNN_BNG_RELU:
      hipLaunchKernelGGL((bnb_apply_kernel<T, CRNN_BNG_RELU>), dim3(nb), dim3(NT), 0, st, *d, dHW, mg, mgx, (T*)dz, rpb);
      break;
    case CRNN_BNG_RESID:
      hipLaunchKernelGGL((bnb_apply_kernel<T, CRNN_BNG_RESID>), dim3(nb), dim3(NT), 0, st, *d, dHW, mg, mgx, (T*)dz, rpb);
      break;
    default:
      hipLaunchKernelGGL((bnb_apply_kernel<T, CRNN_BNG_SE>), dim3(nb), dim3(NT), 0, st, *d, dHW, mg, mgx, (T*)dz, rpb);
  }
  return (int)hipGetLastError();
}

}  // namespace

extern "C" {

int crnn_bn_rows(long M) { return rows_for(M); }

int crnn_channel_stats(int dtype, const void* x, long M, int C, float* psum, float* psq, int rows, void* stream) {
  if (C % 8 || C / 8 > NT || NT % (C / 8)) return crnn_set_error(hipErrorInvalidValue, "channel_stats: bad C");
  long rpb = (M + rows - 1) / rows;
  int rl = NT / (C / 8);
  size_t sm = (size_t)(rl + 1) * C * sizeof(float);
  DISPATCH(dtype, hipLaunchKernelGGL(chan_stats_kernel<T>, dim3(rows), dim3(NT), sm, (hipStream_t)stream, (const T*)x, M,
                                     C, rpb, psum, psq));
  return (int)hipGetLastError();
}

size_t crnn_bn_finalize_workspace(int C) {
  return (size_t)FIN_CNT * sizeof(unsigned) + (size_t)2 * FIN_P * C * sizeof(float);
}

int crnn_bn_finalize(const float* psum, const float* psq, int rows, long rows_per_partial, int C, long count,
                     const float* gamma, const float* beta, float* running_mean, float* running_var, float momentum,
                     float eps, int train, float* mean, float* invstd, float* scale, float* shift, float* ws,
                     void* stream) {
  hipStream_t st = (hipStream_t)stream;
  FinFwd a{gamma, beta, running_mean, running_var, momentum, eps, mean, invstd, scale, shift};
  if (!train) {
    hipLaunchKernelGGL(bn_eval_affine_kernel, dim3((C + 255) / 256), dim3(256), 0, st, C, a);
    return (int)hipGetLastError();
  }
  return launch_fin<true>(psum, psq, rows, rows_per_partial, C, count, ws, a, st);
}

int crnn_bn_act(int dtype, const void* z, const float* scale, const float* shift, void* y, long M, int C, int relu,
                void* stream) {
  if (!rowmap_ok(C)) return crnn_set_error(hipErrorInvalidValue, "bn_act: C/8 must divide 256");
  int nb;
  long rpb;
  stream_grid(M, C, &nb, &rpb);
  DISPATCH(dtype, hipLaunchKernelGGL(bn_act2_kernel<T>, dim3(nb), dim3(NT), 0, (hipStream_t)stream, (const T*)z, scale,
                                     shift, (T*)y, M, C, relu, rpb));
  return (int)hipGetLastError();
}

int crnn_bn_relu_maxpool(int dtype, const void* z, const float* scale, const float* shift, void* y, int B, int H,
                         int W, int C, void* stream) {
  long n = (long)B * (H / 2) * (W / 2) * (C / 8);
  if (n >= (1L << 31)) return crnn_set_error(hipErrorInvalidValue, "bn_relu_maxpool: > 2^31 pooled 8-channel groups");
  DISPATCH(dtype, hipLaunchKernelGGL(bn_relu_maxpool_kernel<T>, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream,
                                     (const T*)z, scale, shift, (T*)y, B, H, W, C));
  return (int)hipGetLastError();
}

int crnn_maxpool_bwd(int dtype, const void* z, const float* scale, const float* shift, const void* dpool,
                     void* dy_full, int B, int H, int W, int C, void* stream) {
  if ((H & 1) || (W & 1)) return crnn_set_error(hipErrorInvalidValue, "maxpool_bwd: H and W must be even");
  long n = (long)B * (H / 2) * (W / 2) * (C / 8);
  DISPATCH(dtype, hipLaunchKernelGGL(maxpool_bwd_kernel<T>, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream,
                                     (const T*)z, scale, shift, (const T*)dpool, (T*)dy_full, B, H, W, C));
  return (int)hipGetLastError();
}

int crnn_bn_bwd_reduce(int dtype, const crnn_bn_bwd_desc* d, float* pg, float* pgx, int rows, void* stream) {
  if (!rowmap_ok(d->C)) return crnn_set_error(hipErrorInvalidValue, "bn_bwd_reduce: C/8 must divide 256");
  hipStream_t st = (hipStream_t)stream;
  return dtype == CRNN_BF16 ? bnb_reduce_launch<bf16>(d, pg, pgx, rows, st) : bnb_reduce_launch<float>(d, pg, pgx, rows, st);
}

int crnn_bn_bwd_finalize(const float* pg, const float* pgx, int rows, int C, long count, float* dgamma, float* dbeta,
                         float* mean_g, float* mean_gx, int accumulate, float* ws, void* stream) {
  FinBwd a{dgamma, dbeta, mean_g, mean_gx, accumulate};
  return launch_fin<false>(pg, pgx, rows, 1, C, count, ws, a, (hipStream_t)stream);
}

int crnn_bn_bwd_apply(int dtype, const crnn_bn_bwd_desc* d, const float* mean_g, const float* mean_gx, void* dz,
                      void* stream) {
  if (!rowmap_ok(d->C)) return crnn_set_error(hipErrorInvalidValue, "bn_bwd_apply: C/8 must divide 256");
  if (d->mode == CRNN_BNG_POOL_OUT) return crnn_set_error(hipErrorInvalidValue, "bn_bwd_apply: POOL_OUT is a reduce-only mode");
  hipStream_t st = (hipStream_t)stream;
  return dtype == CRNN_BF16 ? bnb_apply_launch<bf16>(d, mean_g, mean_gx, dz, st)
                            : bnb_apply_launch<float>(d, mean_g, mean_gx, dz, st);
}

int crnn_se_pool(int dtype, const void* z2, const float* scale, const float* shift, float* pooled, int B, int HW, int C,
                 void* stream) {
  if (C % 8 || NT % (C / 8)) return crnn_set_error(hipErrorInvalidValue, "se_pool: bad C");
  size_t sm = (size_t)(NT / (C / 8)) * C * sizeof(float);
  DISPATCH(dtype, hipLaunchKernelGGL((se_reduce_kernel<T, 0>), dim3(B), dim3(NT), sm, (hipStream_t)stream,
                                     (const T*)z2, scale, shift, (const T*)nullptr, (const T*)nullptr, HW, C, pooled,
                                     1.f / (float)HW));
  return (int)hipGetLastError();
}

int crnn_se_pool_partials(const float* psum, int rows, long rows_per_partial, const float* scale,
                          const float* shift, float* pooled, int B, int HW, int C, void* stream) {
  if (rows_per_partial <= 0 || HW % rows_per_partial || (long)rows * rows_per_partial != (long)B * HW)
    return crnn_set_error(hipErrorInvalidValue, "se_pool_partials: partial rows must tile every sample");
  hipLaunchKernelGGL(se_pool_partials_kernel, dim3(B), dim3(256), 0, (hipStream_t)stream, psum,
                     (int)(HW / rows_per_partial), scale, shift, pooled, HW, C);
  return (int)hipGetLastError();
}

int crnn_se_pool_mlp_fwd(const float* psum, int rows, long rows_per_partial, const float* scale, const float* shift,
                         float* pooled, const float* w1, const float* w2, float* hid, float* s, int B, int HW, int C,
                         int Cr, void* stream) {
  if (rows_per_partial <= 0 || HW % rows_per_partial || (long)rows * rows_per_partial != (long)B * HW)
    return crnn_set_error(hipErrorInvalidValue, "se_pool_mlp_fwd: partial rows must tile every sample");
  if (Cr * 16 != C || (C != 256 && C != 512)) return crnn_set_error(hipErrorInvalidValue, "se_pool_mlp_fwd: C in {256, 512}, Cr = C/16");
  const SePoolSrc src{psum, scale, shift, pooled, (int)(HW / rows_per_partial), HW};
  const dim3 grid((B + SE_SB - 1) / SE_SB);
  if (C == 256)
    hipLaunchKernelGGL((se_mlp_fwd_kernel<256, true>), grid, dim3(256), 0, (hipStream_t)stream, nullptr, w1, w2, hid, s,
                       B, src);
  else
    hipLaunchKernelGGL((se_mlp_fwd_kernel<512, true>), grid, dim3(256), 0, (hipStream_t)stream, nullptr, w1, w2, hid, s,
                       B, src);
  return (int)hipGetLastError();
}

int crnn_se_bn_bwd_reduce(int dtype, const void* dy, const void* y, const void* z2, const float* mean,
                          const float* invstd, const float* gamma, const float* beta, float* ds, float* abc, int B,
                          int HW, int C, void* stream) {
  if (!rowmap_ok(C)) return crnn_set_error(hipErrorInvalidValue, "se_bn_bwd_reduce: C/8 must divide 256");
  size_t sm = (size_t)3 * (NT / (C / 8)) * C * sizeof(float);
  DISPATCH(dtype, hipLaunchKernelGGL((se_bn_bwd_reduce_kernel<T>), dim3(B), dim3(NT), sm, (hipStream_t)stream,
                                     (const T*)dy, (const T*)y, (const T*)z2, mean, invstd, gamma, beta, HW, C, ds,
                                     abc));
  return (int)hipGetLastError();
}

int crnn_se_bn_partials(const float* abc, const float* s, const float* dpool, float* pg, float* pgx, int B, int HW,
                        int C, void* stream) {
  hipLaunchKernelGGL(se_bn_partials_kernel, dim3(B), dim3(256), 0, (hipStream_t)stream, abc, s, dpool, HW, C, pg,
                     pgx);
  return (int)hipGetLastError();
}

int crnn_se_mlp_fwd(const float* pooled, const float* w1, const float* w2, float* hid, float* s, int B, int C, int Cr,
                    void* stream) {
  if (Cr * 16 != C || (C != 256 && C != 512)) return crnn_set_error(hipErrorInvalidValue, "se_mlp: C in {256, 512}, Cr = C/16");
  const dim3 grid((B + SE_SB - 1) / SE_SB);
  if (C == 256)
    hipLaunchKernelGGL(se_mlp_fwd_kernel<256>, grid, dim3(256), 0, (hipStream_t)stream, pooled, w1, w2, hid, s, B);
  else
    hipLaunchKernelGGL(se_mlp_fwd_kernel<512>, grid, dim3(256), 0, (hipStream_t)stream, pooled, w1, w2, hid, s, B);
  return (int)hipGetLastError();
}

int crnn_se_residual_fwd(int dtype, const void* z2, const float* scale, const float* shift, const float* s,
                         const void* idn, const float* iscale, const float* ishift, void* y, int B, int HW, int C,
                         void* stream) {
  if (!rowmap_ok(C)) return crnn_set_error(hipErrorInvalidValue, "se_residual: C/8 must divide 256");
  const long M = (long)B * HW;
  int nb;
  long rpb;
  stream_grid(M, C, &nb, &rpb);
  DISPATCH(dtype, hipLaunchKernelGGL((se_residual2_kernel<T, false>), dim3(nb), dim3(NT), 0, (hipStream_t)stream,
                                     (const T*)z2, scale, shift, s, (const T*)idn, iscale, ishift, (T*)y, M, C,
                                     FastDiv(HW), rpb, nullptr, nullptr));
  return (int)hipGetLastError();
}

int crnn_se_residual_drop_fwd(int dtype, const void* z2, const float* scale, const float* shift, const float* s,
                              const void* idn, const float* iscale, const float* ishift, void* y, int B, int HW,
                              int C, const unsigned char* keep, const unsigned long long* kept, void* stream) {
  if (!rowmap_ok(C)) return crnn_set_error(hipErrorInvalidValue, "se_residual: C/8 must divide 256");
  if (!keep || !kept) return crnn_set_error(hipErrorInvalidValue, "se_residual_drop: keep / kept missing");
  const long M = (long)B * HW;
  int nb;
  long rpb;
  stream_grid(M, C, &nb, &rpb);
  DISPATCH(dtype, hipLaunchKernelGGL((se_residual2_kernel<T, true>), dim3(nb), dim3(NT), 0, (hipStream_t)stream,
                                     (const T*)z2, scale, shift, s, (const T*)idn, iscale, ishift, (T*)y, M, C,
                                     FastDiv(HW), rpb, keep, kept));
  return (int)hipGetLastError();
}

int crnn_dropblock_mask(unsigned char* keep, unsigned long long* kept, int B, int H, int W, int C, float p,
                        int block_size, unsigned long long seed, void* stream) {
  if (B <= 0 || H <= 0 || W <= 0 || C <= 0 || C % 8)
    return crnn_set_error(hipErrorInvalidValue, "dropblock_mask: B, H, W > 0 and C % 8 == 0 required");
  if (!(p >= 0.f && p <= 1.f)) return crnn_set_error(hipErrorInvalidValue, "dropblock_mask: p must be in [0, 1]");
  const int hw = H < W ? H : W, bs = block_size < hw ? block_size : hw;
  if (bs < 1 || bs % 2 == 0)
    return crnn_set_error(hipErrorInvalidValue,
                          "dropblock_mask: min(block_size, H, W) must be odd (drop_block2d's mask is "
                          "(H+2) x (W+2) for an even block and does not broadcast against the input)");
  const double gamma = (double)p * H * W / ((double)bs * bs * (double)(H - bs + 1) * (W - bs + 1));
  if (gamma > 1.0) return crnn_set_error(hipErrorInvalidValue, "dropblock_mask: Bernoulli rate above 1");
  const double t = gamma * 4294967296.0;
  const uint32_t thr = t >= 4294967295.0 ? 0xffffffffu : (uint32_t)t;
  hipError_t e = hipMemsetAsync(kept, 0, sizeof(unsigned long long), (hipStream_t)stream);
  if (e != hipSuccess) return crnn_set_error(e, "dropblock_mask: memset");
  const long total8 = (long)B * H * W * (C / 8);
  hipLaunchKernelGGL(dropblock_mask_kernel, dim3(grid_for(total8)), dim3(256), 0, (hipStream_t)stream, keep, kept,
                     H, W, C, bs, thr, seed, total8);
  return (int)hipGetLastError();
}

int crnn_dropblock_apply(int dtype, const void* x, void* y, const unsigned char* keep,
                         const unsigned long long* kept, long n, void* stream) {
  if (n % 8) return crnn_set_error(hipErrorInvalidValue, "dropblock_apply: n % 8 != 0");
  DISPATCH(dtype, hipLaunchKernelGGL(dropblock_apply_kernel<T>, dim3(grid_for(n / 8)), dim3(256), 0,
                                     (hipStream_t)stream, (const T*)x, (T*)y, keep, kept, n / 8));
  return (int)hipGetLastError();
}

int crnn_se_bwd_reduce(int dtype, const void* dy, const void* y, const void* z2, const float* scale,
                       const float* shift, float* ds, int B, int HW, int C, void* stream) {
  if (C % 8 || NT % (C / 8)) return crnn_set_error(hipErrorInvalidValue, "se_bwd_reduce: bad C");
  size_t sm = (size_t)(NT / (C / 8)) * C * sizeof(float);
  DISPATCH(dtype, hipLaunchKernelGGL((se_reduce_kernel<T, 1>), dim3(B), dim3(NT), sm, (hipStream_t)stream,
                                     (const T*)z2, scale, shift, (const T*)dy, (const T*)y, HW, C, ds, 1.f));
  return (int)hipGetLastError();
}

int crnn_se_mlp_bwd(const float* ds, const float* pooled, const float* hid, const float* s, const float* w1,
                    const float* w2, float* dsig, float* dhid, float* dpool, float* dw1, float* dw2, int B, int C,
                    int Cr, int HW, int accumulate, void* stream) {
  return crnn_se_mlp_bwd_partials(ds, pooled, hid, s, w1, w2, dsig, dhid, dpool, dw1, dw2, nullptr, nullptr, nullptr,
                                  B, C, Cr, HW, accumulate, stream);
}

int crnn_se_mlp_bwd_partials(const float* ds, const float* pooled, const float* hid, const float* s, const float* w1,
                             const float* w2, float* dsig, float* dhid, float* dpool, float* dw1, float* dw2,
                             const float* abc, float* pg, float* pgx, int B, int C, int Cr, int HW, int accumulate,
                             void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (Cr * 16 != C || (C != 256 && C != 512)) return crnn_set_error(hipErrorInvalidValue, "se_mlp: C in {256, 512}, Cr = C/16");
  const dim3 grid((B + SE_SB - 1) / SE_SB), wgrid(C / 64, Cr / 8);
  const float inv = 1.f / (float)HW;
  if (C == 256) {
    hipLaunchKernelGGL(se_mlp_bwd_kernel<256>, grid, dim3(256), 0, st, ds, hid, s, w1, w2, dsig, dhid, dpool, B, inv,
                       abc, pg, pgx, HW);
#if CRNN_SE_PROBE
    hipLaunchKernelGGL(se_wgrad_kernel<256>, wgrid, dim3(256), 0, st, dsig, hid, dhid, pooled, dw1, dw2, B, accumulate,
                       g_se_probe_launch++);
#else
    hipLaunchKernelGGL(se_wgrad_kernel<256>, wgrid, dim3(256), 0, st, dsig, hid, dhid, pooled, dw1, dw2, B, accumulate);
#endif
  } else {
    hipLaunchKernelGGL(se_mlp_bwd_kernel<512>, grid, dim3(256), 0, st, ds, hid, s, w1, w2, dsig, dhid, dpool, B, inv,
                       abc, pg, pgx, HW);
#if CRNN_SE_PROBE
    hipLaunchKernelGGL(se_wgrad_kernel<512>, wgrid, dim3(256), 0, st, dsig, hid, dhid, pooled, dw1, dw2, B, accumulate,
                       g_se_probe_launch++);
#else
    hipLaunchKernelGGL(se_wgrad_kernel<512>, wgrid, dim3(256), 0, st, dsig, hid, dhid, pooled, dw1, dw2, B, accumulate);
#endif
  }
  return (int)hipGetLastError();
}

#if CRNN_SE_PROBE
// diagnostic build only (not in crnn_hip.h): copy the probe records out and restart the launch count
int crnn_diag_se_probe(float* host, int n) {
  const int all = SE_PROBE_LAUNCHES * SE_PROBE_BLOCKS * SE_PROBE_VALS;
  hipError_t e = hipMemcpyFromSymbol(host, HIP_SYMBOL(g_se_probe), (size_t)(n < all ? n : all) * sizeof(float), 0,
                                     hipMemcpyDeviceToHost);
  g_se_probe_launch = 0;
  return (int)e;
}
#endif

int crnn_hpool_fwd(int dtype, const void* z, const float* scale, const float* shift, void* seq, int B, int Hh, int W,
                   int C, void* stream) {
  long n = (long)B * W * (C / 8);
  DISPATCH(dtype, hipLaunchKernelGGL(hpool_fwd_kernel<T>, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream,
                                     (const T*)z, scale, shift, (T*)seq, B, Hh, W, C));
  return (int)hipGetLastError();
}

int crnn_hpool_bwd(int dtype, const void* dseq, void* dy_full, int B, int Hh, int W, int C, void* stream) {
  long n = (long)B * Hh * W * (C / 8);
  DISPATCH(dtype, hipLaunchKernelGGL(hpool_bwd_kernel<T>, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream,
                                     (const T*)dseq, (T*)dy_full, B, Hh, W, C));
  return (int)hipGetLastError();
}

int crnn_nchw_to_nhwc(int dtype, const float* x, void* y, int B, int C, int H, int W, int Cp, void* stream) {
  long n = (long)B * H * W;
  DISPATCH(dtype, hipLaunchKernelGGL(nchw_to_nhwc_kernel<T>, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, x,
                                     (T*)y, B, C, H, W, Cp));
  return (int)hipGetLastError();
}

int crnn_dropout(int dtype, const void* x, void* y, long n, float p, unsigned long long seed, void* stream) {
  if (!(p >= 0.f && p < 1.f)) return crnn_set_error(hipErrorInvalidValue, "dropout: p must be in [0, 1)");
  const uint32_t thr = drop_threshold(p);
  DISPATCH(dtype, hipLaunchKernelGGL(dropout_kernel<T>, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream,
                                     (const T*)x, (T*)y, n, thr, 1.f / (1.f - p), seed));
  return (int)hipGetLastError();
}

int crnn_cast_f32(int dtype, const float* src, void* dst, long n, void* stream) {
  DISPATCH(dtype, hipLaunchKernelGGL(cast_kernel<T>, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, src, (T*)dst,
                                     n));
  return (int)hipGetLastError();
}

int crnn_pack_conv_weight(int dtype, const float* w, void* out, int Co, int Ci, int KH, int KW, int Cip, void* stream) {
  long n = (long)Co * KH * KW * Cip;
  DISPATCH(dtype, hipLaunchKernelGGL(pack_conv_kernel<T>, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, w,
                                     (T*)out, Co, Ci, KH, KW, Cip));
  return (int)hipGetLastError();
}

int crnn_pack_batch(int dtype, const crnn_pack_job* jobs, int njobs, long total, void* stream) {
  if (njobs <= 0 || total <= 0) return 0;
  // ~4 elements per thread: the element loop is load-latency bound (one dependent load per
  // element, strided for the conv repack), so parallelism comes from many small blocks
  long blocks = (total + 2047) / 2048;
  if (blocks > (1L << 20)) blocks = 1L << 20;
  const long chunk = ((total + blocks - 1) / blocks + 7) / 8 * 8;   // whole 8-element groups per block
  DISPATCH(dtype, hipLaunchKernelGGL(pack_batch_kernel<T>, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream,
                                     jobs, njobs, total, chunk));
  return (int)hipGetLastError();
}

int crnn_pack_conv_t_tiles(int Co, int Ci) { return ((Co + PT_CO - 1) / PT_CO) * ((Ci + PT_CI - 1) / PT_CI); }

int crnn_pack_conv_t_batch(int dtype, const crnn_pack_job* jobs, int njobs, long total_tiles, void* stream) {
  if (njobs <= 0 || total_tiles <= 0) return 0;
  DISPATCH(dtype, hipLaunchKernelGGL(pack_conv_t_kernel<T>, dim3((unsigned)total_tiles), dim3(256), 0,
                                     (hipStream_t)stream, jobs, njobs));
  return (int)hipGetLastError();
}

int crnn_pack_conv_batch(int dtype, const crnn_pack_job* jobs, int njobs, long total_rows, int max_slab,
                         void* stream) {
  if (njobs <= 0 || total_rows <= 0 || max_slab <= 0 || max_slab > 16384)
    return crnn_set_error(hipErrorInvalidValue, "pack_conv_batch: bad job table / slab size");
  DISPATCH(dtype, hipLaunchKernelGGL(pack_conv_kernel<T>, dim3((unsigned)total_rows), dim3(256),
                                     (size_t)max_slab * sizeof(float), (hipStream_t)stream, jobs, njobs));
  return (int)hipGetLastError();
}

int crnn_pack_rows(int dtype, const float* src, void* out, const int* perm, int rows_out, int rows_src, int cols,
                   void* stream) {
  long n = (long)rows_out * cols;
  DISPATCH(dtype, hipLaunchKernelGGL(pack_rows_kernel<T>, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, src,
                                     (T*)out, perm, rows_out, rows_src, cols));
  return (int)hipGetLastError();
}

}  // extern "C"
