// Implicit-GEMM convolutions, NHWC, for the SE-ResNet31 backbone
// (reference: model/seresnet31.py:37-45, :82-86, :130-134, :153-154 — nn.Conv2d, bias=False).
//
//   fwd   : y[m=(b,ho,wo)][co]      = sum_{k=(kh,kw,ci)} x_im2col[m][k] * W[co][k]
//   dgrad : dx[m=(b,hi,wi)][ci]     = sum_{k=(kh,kw,co)} dy[b,(hi+p-kh)/s,(wi+p-kw)/s][co] * W[co][kh][kw][ci]
//   wgrad : dW[co][k'=(kh,kw,ci)]   = sum_{m=(b,ho,wo)} dy[m][co] * x_im2col[m][k']
//
// Weights are packed OHWI ([Co][KH][KW][Cip], Cip = Ci padded to a multiple of 8)
// in the compute dtype; dgrad reads them transposed straight from that layout
// (row-contiguous loader + ds_read_b64_tr_b16), so no transposed copy exists.
// fwd also emits per-column (channel) partial sum / sum-of-squares of the fp32
// accumulators for training-mode BatchNorm (two rows per 128-row M tile).
#include "gemm.hpp"
#include "crnn_internal.hpp"

using namespace gemm;

namespace {

struct Geo {
  int B, Hi, Wi, Ci, Ho, Wo, Co, KH, KW, sh, sw, ph, pw;
  // magic divisors for the im2col decodes (no hardware integer division on the GPU)
  FastDiv dCi, dCo, dKW, dWo, dHoWo, dWi, dHiWi, dsh, dsw;
};

inline Geo geo(const crnn_conv_desc* d) {
  Geo g{d->B, d->Hi, d->Wi, d->Ci, d->Ho, d->Wo, d->Co, d->KH, d->KW, d->sh, d->sw, d->ph, d->pw};
  g.dCi = FastDiv(d->Ci);
  g.dCo = FastDiv(d->Co);
  g.dKW = FastDiv(d->KW);
  g.dWo = FastDiv(d->Wo);
  g.dHoWo = FastDiv(d->Ho * d->Wo);
  g.dWi = FastDiv(d->Wi);
  g.dHiWi = FastDiv(d->Hi * d->Wi);
  g.dsh = FastDiv(d->sh);
  g.dsw = FastDiv(d->sw);
  return g;
}

// ---- fwd A: im2col rows of x (NHWC [B][Hi][Wi][Ci]), K-contiguous
template <typename T> struct FwdA {
  static constexpr bool kRowVec = false;
  const T* x;
  Geo g;
  int M, K;
  struct Ctx { const T* base; int hb, wb; bool ok; };
  __device__ __forceinline__ Ctx row_ctx(int m) const {
    Ctx c;
    c.ok = m < M;
    uint32_t r, wo;
    uint32_t b = g.dHoWo.divmod(c.ok ? m : 0, r);
    uint32_t ho = g.dWo.divmod(r, wo);
    c.hb = ho * g.sh - g.ph;
    c.wb = wo * g.sw - g.pw;
    c.base = x + (size_t)b * g.Hi * g.Wi * g.Ci;
    return c;
  }
  __device__ __forceinline__ typename VT<T>::v8 load(const Ctx& c, int k) const {
    if (!c.ok || k >= K) return zero8<T>();
    uint32_t ci, kw;
    uint32_t tap = g.dCi.divmod(k, ci);
    uint32_t kh = g.dKW.divmod(tap, kw);
    int hi = c.hb + (int)kh, wi = c.wb + (int)kw;
    if ((unsigned)hi >= (unsigned)g.Hi || (unsigned)wi >= (unsigned)g.Wi) return zero8<T>();
    return ld8<T>(c.base + (uint32_t)((hi * g.Wi + wi) * g.Ci + (int)ci));
  }
};

// ---- dgrad A: gather of dy for input pixel rows, K = (kh,kw,co) contiguous in co
template <typename T> struct DgradA {
  static constexpr bool kRowVec = false;
  const T* dy;
  Geo g;
  int M, K;
  struct Ctx { const T* base; int hp, wp; bool ok; };
  __device__ __forceinline__ Ctx row_ctx(int m) const {
    Ctx c;
    c.ok = m < M;
    uint32_t r, wi;
    uint32_t b = g.dHiWi.divmod(c.ok ? m : 0, r);
    uint32_t hi = g.dWi.divmod(r, wi);
    c.hp = hi + g.ph;
    c.wp = wi + g.pw;
    c.base = dy + (size_t)b * g.Ho * g.Wo * g.Co;
    return c;
  }
  __device__ __forceinline__ typename VT<T>::v8 load(const Ctx& c, int k) const {
    if (!c.ok || k >= K) return zero8<T>();
    uint32_t co, kw;
    uint32_t tap = g.dCo.divmod(k, co);
    uint32_t kh = g.dKW.divmod(tap, kw);
    int th = c.hp - (int)kh, tw = c.wp - (int)kw;
    if (th < 0 || tw < 0) return zero8<T>();
    uint32_t rh, rw;
    int ho = (int)g.dsh.divmod(th, rh), wo = (int)g.dsw.divmod(tw, rw);
    if (rh | rw || ho >= g.Ho || wo >= g.Wo) return zero8<T>();
    return ld8<T>(c.base + (uint32_t)((ho * g.Wo + wo) * g.Co + (int)co));
  }
};

// ---- dgrad B: W^T rows (ci), k = (kh,kw,co), read from OHWI: 8 consecutive ci at fixed (co,kh,kw)
template <typename T> struct DgradB {
  static constexpr bool kRowVec = true;
  const T* w;  // [Co][KH][KW][Ci]
  Geo g;
  int K;       // KH*KW*Co
  struct Ctx { int ci; bool ok; };
  __device__ __forceinline__ Ctx row_ctx(int r8) const { return Ctx{r8, r8 < g.Ci}; }
  __device__ __forceinline__ typename VT<T>::v8 load(const Ctx& c, int k) const {
    if (!c.ok || k >= K) return zero8<T>();
    uint32_t co;
    uint32_t tap = g.dCo.divmod(k, co);
    return ld8<T>(w + (uint32_t)(((int)co * g.KH * g.KW + (int)tap) * g.Ci + c.ci));
  }
};

// ---- wgrad A: dy rows = co, k = output pixel m (row-contiguous: dy[m][co..co+7])
template <typename T> struct WgradA {
  static constexpr bool kRowVec = true;
  const T* dy;
  int Co, M;
  struct Ctx { const T* base; bool ok; };
  __device__ __forceinline__ Ctx row_ctx(int r8) const { return Ctx{dy + r8, r8 < Co}; }
  __device__ __forceinline__ typename VT<T>::v8 load(const Ctx& c, int k) const {
    if (!c.ok || k >= M) return zero8<T>();
    return ld8<T>(c.base + (size_t)k * Co);
  }
};

// ---- wgrad B: im2col columns k' = (kh,kw,ci) as rows, k = output pixel m
template <typename T> struct WgradB {
  static constexpr bool kRowVec = true;
  const T* x;
  Geo g;
  int Kp, M;  // Kp = KH*KW*Ci
  struct Ctx { int kh, kw, ci; bool ok; };
  __device__ __forceinline__ Ctx row_ctx(int r8) const {
    Ctx c;
    c.ok = r8 < Kp;
    uint32_t ci, kw;
    uint32_t tap = g.dCi.divmod(c.ok ? r8 : 0, ci);
    uint32_t kh = g.dKW.divmod(tap, kw);
    c.ci = ci;
    c.kh = kh;
    c.kw = kw;
    return c;
  }
  __device__ __forceinline__ typename VT<T>::v8 load(const Ctx& c, int m) const {
    if (!c.ok || m >= M) return zero8<T>();
    uint32_t r, wo;
    uint32_t b = g.dHoWo.divmod(m, r);
    uint32_t ho = g.dWo.divmod(r, wo);
    int hi = (int)ho * g.sh - g.ph + c.kh, wi = (int)wo * g.sw - g.pw + c.kw;
    if ((unsigned)hi >= (unsigned)g.Hi || (unsigned)wi >= (unsigned)g.Wi) return zero8<T>();
    return ld8<T>(x + (size_t)b * g.Hi * g.Wi * g.Ci + (uint32_t)((hi * g.Wi + wi) * g.Ci + c.ci));
  }
};

// ---- epilogues
template <typename T> struct FwdEpi {
  static constexpr bool kStats = true;
  T* y;
  float* psum;
  float* psq;
  int M, N;
  __device__ __forceinline__ void store(int m, int n, f32x4 v, int) const {
    if (m < M && n < N) st4<T>(y + (size_t)m * N + n, v);
  }
  __device__ __forceinline__ void stats(int row, int n, f32x4 s, f32x4 q) const {
    if (psum == nullptr || n >= N) return;
    *reinterpret_cast<f32x4*>(psum + (size_t)row * N + n) = s;
    *reinterpret_cast<f32x4*>(psq + (size_t)row * N + n) = q;
  }
};

// dx = acc (+ dx if accumulate) (+ dres * (yres > 0): the identity branch of a
// residual block whose output went through ReLU, model/seresnet31.py:66)
template <typename T> struct DgradEpi {
  static constexpr bool kStats = false;
  T* dx;
  const T* dres;
  const T* yres;
  int M, N, accumulate;
  __device__ __forceinline__ void store(int m, int n, f32x4 v, int) const {
    if (m >= M || n >= N) return;
    size_t o = (size_t)m * N + n;
    if (accumulate) v += ld4f<T>(dx + o);
    if (dres) {
      f32x4 d = ld4f<T>(dres + o), yy = ld4f<T>(yres + o);
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] += yy[r] > 0.f ? d[r] : 0.f;
    }
    st4<T>(dx + o, v);
  }
  __device__ __forceinline__ void stats(int, int, f32x4, f32x4) const {}
};

struct SlabEpi {
  static constexpr bool kStats = false;
  float* ws;  // [nsplit][Mrows][N]
  int M, N;
  __device__ __forceinline__ void store(int m, int n, f32x4 v, int kz) const {
    if (m >= M || n >= N) return;
    *reinterpret_cast<f32x4*>(ws + ((size_t)kz * M + m) * N + n) = v;
  }
  __device__ __forceinline__ void stats(int, int, f32x4, f32x4) const {}
};

// sum split-K slabs [S][Co][KH*KW*Cip] and scatter into an OIHW fp32 gradient
__global__ void wgrad_reduce_kernel(const float* __restrict__ ws, int S, float* __restrict__ dw,
                                    int Co, int Ci, int Cip, int KH, int KW, float beta) {
  const int Kp = KH * KW * Cip;
  const long total = (long)Co * Kp;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    int co = (int)(i / Kp), k = (int)(i - (long)co * Kp);
    int tap = k / Cip, ci = k - tap * Cip;
    if (ci >= Ci) continue;
    float s = 0.f;
    for (int z = 0; z < S; ++z) s += ws[(size_t)z * total + i];
    int kh = tap / KW, kw = tap - kh * KW;
    size_t o = (((size_t)co * Ci + ci) * KH + kh) * KW + kw;
    dw[o] = beta != 0.f ? beta * dw[o] + s : s;
  }
}

template <typename T> int conv_fwd_t(const crnn_conv_desc* d, const void* x, const void* w, void* y,
                                     float* psum, float* psq, hipStream_t st) {
  Geo g = geo(d);
  int M = g.B * g.Ho * g.Wo, N = g.Co, K = g.KH * g.KW * g.Ci;
  FwdA<T> la{(const T*)x, g, M, K};
  RowMajorK<T> lb{(const T*)w, K, N, K};
  FwdEpi<T> ep{(T*)y, psum, psq, M, N};
  int bm, bn;
  crnn_conv_fwd_tile(d, &bm, &bn);
  if (bm == 128 && bn == 128) return launch<T, 128, 128>(la, lb, ep, M, N, K, 1, st);
  if (bm == 128 && bn == 64) return launch<T, 128, 64>(la, lb, ep, M, N, K, 1, st);
  return launch<T, 64, 64>(la, lb, ep, M, N, K, 1, st);
}

template <typename T> int conv_dgrad_t(const crnn_conv_desc* d, const void* dy, const void* w, void* dx,
                                       const void* dres, const void* yres, int accumulate, hipStream_t st) {
  Geo g = geo(d);
  int M = g.B * g.Hi * g.Wi, N = g.Ci, K = g.KH * g.KW * g.Co;
  DgradA<T> la{(const T*)dy, g, M, K};
  DgradB<T> lb{(const T*)w, g, K};
  DgradEpi<T> ep{(T*)dx, (const T*)dres, (const T*)yres, M, N, accumulate};
  if (N >= 128 && (long)M * N >= 128L * 128 * 256) return launch<T, 128, 128>(la, lb, ep, M, N, K, 1, st);
  if (N <= 64 && (long)M * N >= 128L * 64 * 256) return launch<T, 128, 64>(la, lb, ep, M, N, K, 1, st);
  return launch<T, 64, 64>(la, lb, ep, M, N, K, 1, st);
}

template <typename T> int conv_wgrad_t(const crnn_conv_desc* d, const void* dy, const void* x, float* dw,
                                       float* ws, size_t ws_bytes, float beta, hipStream_t st) {
  Geo g = geo(d);
  int Mp = g.B * g.Ho * g.Wo, Kp = g.KH * g.KW * g.Ci;
  int bm, bn, splits;
  crnn_conv_wgrad_plan(d, &bm, &bn, &splits);
  size_t need = (size_t)splits * g.Co * Kp * sizeof(float);
  if (ws_bytes < need) return crnn_set_error(hipErrorInvalidValue, "conv_wgrad: workspace too small");
  WgradA<T> la{(const T*)dy, g.Co, Mp};
  WgradB<T> lb{(const T*)x, g, Kp, Mp};
  SlabEpi ep{ws, g.Co, Kp};
  int rc;
  if (bm == 128) rc = launch<T, 128, 128>(la, lb, ep, g.Co, Kp, Mp, splits, st);
  else rc = launch<T, 64, 64>(la, lb, ep, g.Co, Kp, Mp, splits, st);
  if (rc) return rc;
  int ci_real = d->Ci_real > 0 ? d->Ci_real : g.Ci;
  long total = (long)g.Co * Kp;
  int blocks = (int)((total + 255) / 256);
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(wgrad_reduce_kernel, dim3(blocks), dim3(256), 0, st, ws, splits, dw, g.Co, ci_real,
                     g.Ci, g.KH, g.KW, beta);
  return (int)hipGetLastError();
}

}  // namespace

extern "C" {

void crnn_conv_fwd_tile(const crnn_conv_desc* d, int* bm, int* bn) {
  long M = (long)d->B * d->Ho * d->Wo;
  if (d->Co <= 64) { *bm = 128; *bn = 64; }
  else if (M * d->Co >= 128L * 128 * 192) { *bm = 128; *bn = 128; }
  else { *bm = 64; *bn = 64; }
}

int crnn_conv_stat_rows_per_partial(const crnn_conv_desc* d) {
  int bm, bn;
  crnn_conv_fwd_tile(d, &bm, &bn);
  return bm / 2;
}

int crnn_conv_stat_rows(const crnn_conv_desc* d) {
  int bm, bn;
  crnn_conv_fwd_tile(d, &bm, &bn);
  long M = (long)d->B * d->Ho * d->Wo;
  return (int)(((M + bm - 1) / bm) * 2);
}

void crnn_conv_wgrad_plan(const crnn_conv_desc* d, int* bm, int* bn, int* splits) {
  long Mp = (long)d->B * d->Ho * d->Wo;
  int Kp = d->KH * d->KW * d->Ci;
  int b = (d->Co >= 128 && Kp >= 128) ? 128 : 64;
  *bm = b; *bn = b;
  long tiles = ((d->Co + b - 1) / b) * (long)((Kp + b - 1) / b);
  long want = (768 + tiles - 1) / tiles;        // ~3 waves of blocks over 256 CUs
  long maxs = (Mp + 8 * BK - 1) / (8 * BK);     // keep >= 8 K-steps per split
  if (want > maxs) want = maxs;
  if (want < 1) want = 1;
  if (want > 256) want = 256;
  *splits = eff_splits((int)Mp, (int)want);
}

size_t crnn_conv_wgrad_workspace(const crnn_conv_desc* d) {
  int bm, bn, s;
  crnn_conv_wgrad_plan(d, &bm, &bn, &s);
  return (size_t)s * d->Co * d->KH * d->KW * d->Ci * sizeof(float);
}

int crnn_conv_fwd(int dtype, const crnn_conv_desc* d, const void* x, const void* w, void* y,
                  float* psum, float* psq, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (d->Ci % 8 || d->Co % 8) return crnn_set_error(hipErrorInvalidValue, "conv_fwd: channels must be multiples of 8");
  return dtype == CRNN_BF16 ? conv_fwd_t<bf16>(d, x, w, y, psum, psq, st)
                            : conv_fwd_t<float>(d, x, w, y, psum, psq, st);
}

int crnn_conv_dgrad(int dtype, const crnn_conv_desc* d, const void* dy, const void* w, void* dx,
                    const void* dres, const void* yres, int accumulate, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (d->Ci % 8 || d->Co % 8) return crnn_set_error(hipErrorInvalidValue, "conv_dgrad: channels must be multiples of 8");
  return dtype == CRNN_BF16 ? conv_dgrad_t<bf16>(d, dy, w, dx, dres, yres, accumulate, st)
                            : conv_dgrad_t<float>(d, dy, w, dx, dres, yres, accumulate, st);
}

int crnn_conv_wgrad(int dtype, const crnn_conv_desc* d, const void* dy, const void* x, float* dw_oihw,
                    float* ws, size_t ws_bytes, float beta, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (d->Ci % 8 || d->Co % 8) return crnn_set_error(hipErrorInvalidValue, "conv_wgrad: channels must be multiples of 8");
  return dtype == CRNN_BF16 ? conv_wgrad_t<bf16>(d, dy, x, dw_oihw, ws, ws_bytes, beta, st)
                            : conv_wgrad_t<float>(d, dy, x, dw_oihw, ws, ws_bytes, beta, st);
}

}  // extern "C"
