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
#include "gemm256.hpp"
#include "gemm256hw.hpp"
#include "crnn_internal.hpp"

using namespace gemm;

// conv_halo.hip: direct 3x3 / stride-1 kernel for the full-resolution stem conv
bool conv_halo_fits(const crnn_conv_desc* d, bool dgrad);
int conv_halo_fwd(const crnn_conv_desc* d, const void* x, const void* w, void* y, float* psum, float* psq,
                  hipStream_t st, const float* esc = nullptr, const float* esh = nullptr);
int conv_halo_dgrad(const crnn_conv_desc* d, const void* dy, const void* w, void* dx, hipStream_t st);
bool conv_halo_pool_fits(const crnn_conv_desc* d);
int conv_halo_fwd_pool(const crnn_conv_desc* d, const void* x, const void* w, void* y, const float* esc,
                       const float* esh, hipStream_t st);
int conv_halo_wgrad_slabs(const crnn_conv_desc* d);
int conv_halo_wgrad(const crnn_conv_desc* d, const void* dy, const void* x, float* ws, hipStream_t st);
static bool use_halo(int dtype, const crnn_conv_desc* d, bool dgrad) {
  return dtype == CRNN_BF16 && crnn_option(CRNN_OPT_HALO_CONV) != 0 && conv_halo_fits(d, dgrad);
}

// target grid of the deep split-K wgrad (tuning knob; slab bytes grow with the split count)
#ifndef CRNN_WGRAD_BLOCKS
#define CRNN_WGRAD_BLOCKS 256
#endif
// smallest Co that takes the deep-pipelined fwd kernel (tuning knob)
#ifndef CRNN_DEEP_MIN_CO
#define CRNN_DEEP_MIN_CO 128
#endif

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

// Per-stage K decode shared by the loaders whose K = (tap, channel) with channel-minor order.
// When the channel count C is a multiple of the stage depth (every conv except the 8-channel
// stem input), a stage never straddles a tap: tap / channel base are wave-uniform scalars.
struct TapPrep {
  int tap;   // kh*KW + kw (>= KH*KW means past K: masked)
  int kh, kw;
  int c0;    // channel of k0
};

__device__ __forceinline__ TapPrep tap_prep(const FastDiv& dC, const FastDiv& dKW, int k0) {
  TapPrep p;
  uint32_t c, kw;
  uint32_t tap = dC.divmod((uint32_t)k0, c);
  uint32_t kh = dKW.divmod(tap, kw);
  p.tap = (int)tap;
  p.kh = (int)kh;
  p.kw = (int)kw;
  p.c0 = (int)c;
  return p;
}

// ---- fwd A: im2col rows of x (NHWC [B][Hi][Wi][Ci]), K-contiguous, K = (kh, kw, ci)
// UT: the stage never straddles a tap (Ci % stage depth == 0)
template <typename T, bool UT> struct FwdA {
  static constexpr bool kRowVec = false;
  const T* x;
  Geo g;
  int M, K;
  uint32_t bytes;
  struct Ctx { int off; uint32_t mask; int hb, wb; };  // off = element offset of (b, hb, wb, 0)
  typedef TapPrep Prep;
  __device__ __forceinline__ Ctx row_ctx(int m) const {
    Ctx c;
    uint32_t r, wo;
    uint32_t b = g.dHoWo.divmod(m < M ? m : 0, r);
    uint32_t ho = g.dWo.divmod(r, wo);
    c.hb = (int)ho * g.sh - g.ph;
    c.wb = (int)wo * g.sw - g.pw;
    c.off = (((int)b * g.Hi + c.hb) * g.Wi + c.wb) * g.Ci;
    c.mask = 0;
    if (m < M)
      for (int kh = 0; kh < g.KH; ++kh)
        for (int kw = 0; kw < g.KW; ++kw)
          if ((unsigned)(c.hb + kh) < (unsigned)g.Hi && (unsigned)(c.wb + kw) < (unsigned)g.Wi)
            c.mask |= 1u << (kh * g.KW + kw);
    return c;
  }
  __device__ __forceinline__ Prep prep(int k0) const {
    if constexpr (UT) return tap_prep(g.dCi, g.dKW, k0);
    TapPrep p;
    p.tap = k0;
    return p;
  }
  __device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc() const { return mk_rsrc(x, bytes); }
  // byte offset of elements (row, k0+kofs .. +7), or OOB (reads zeros) — UT only
  __device__ __forceinline__ uint32_t offs(const Ctx& c, const Prep& p, int kofs) const {
    const bool ok = (c.mask >> p.tap) & 1u;
    return boff<T>((uint32_t)(c.off + (p.kh * g.Wi + p.kw) * g.Ci + p.c0 + kofs), ok);
  }
  __device__ __forceinline__ typename VT<T>::v8 load(const Ctx& c, const Prep& p, int kofs) const {
    auto rs = mk_rsrc(x, bytes);
    if constexpr (UT) {
      return bld8<T>(rs, offs(c, p, kofs));
    } else {
      const int k = p.tap + kofs;
      uint32_t ci, kw;
      uint32_t tap = g.dCi.divmod((uint32_t)k, ci);
      uint32_t kh = g.dKW.divmod(tap, kw);
      const bool ok = k < K && ((c.mask >> tap) & 1u);
      const int off = c.off + ((int)kh * g.Wi + (int)kw) * g.Ci + (int)ci;
      return bld8<T>(rs, boff<T>((uint32_t)off, ok));
    }
  }
};

// ---- dgrad A: for input pixel rows (b, hi, wi), K = (kh, kw, co): dy at
// ((hi+ph-kh)/sh, (wi+pw-kw)/sw). Strides are 1 or 2 (lsh/lsw = log2), so for a valid tap
// (in range, divisible) the output row is (hp>>lsh) - (kh>>lsh): linear in a per-row base
// plus a per-stage scalar.
template <typename T> struct DgradA {
  static constexpr bool kRowVec = false;
  const T* dy;
  Geo g;
  int M, K, lsh, lsw;
  uint32_t bytes;
  struct Ctx { int off; uint32_t mask; };
  typedef TapPrep Prep;
  __device__ __forceinline__ Ctx row_ctx(int m) const {
    Ctx c;
    uint32_t r, wi;
    uint32_t b = g.dHiWi.divmod(m < M ? m : 0, r);
    uint32_t hi = g.dWi.divmod(r, wi);
    const int hp = (int)hi + g.ph, wp = (int)wi + g.pw;
    c.off = (((int)b * g.Ho + (hp >> lsh)) * g.Wo + (wp >> lsw)) * g.Co;
    c.mask = 0;
    if (m < M)
      for (int kh = 0; kh < g.KH; ++kh)
        for (int kw = 0; kw < g.KW; ++kw) {
          const int th = hp - kh, tw = wp - kw;
          if (th < 0 || tw < 0) continue;
          if ((th & ((1 << lsh) - 1)) || (tw & ((1 << lsw) - 1))) continue;
          if ((th >> lsh) >= g.Ho || (tw >> lsw) >= g.Wo) continue;
          c.mask |= 1u << (kh * g.KW + kw);
        }
    return c;
  }
  __device__ __forceinline__ Prep prep(int k0) const { return tap_prep(g.dCo, g.dKW, k0); }
  __device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc() const { return mk_rsrc(dy, bytes); }
  __device__ __forceinline__ uint32_t offs(const Ctx& c, const Prep& p, int kofs) const {
    const bool ok = (c.mask >> p.tap) & 1u;
    return boff<T>((uint32_t)(c.off - ((p.kh >> lsh) * g.Wo + (p.kw >> lsw)) * g.Co + p.c0 + kofs), ok);
  }
  __device__ __forceinline__ typename VT<T>::v8 load(const Ctx& c, const Prep& p, int kofs) const {
    return bld8<T>(rsrc(), offs(c, p, kofs));
  }
};

// ---- dgrad B: W^T rows (ci), k = (kh,kw,co), read from OHWI: 8 consecutive ci at fixed (co,kh,kw)
template <typename T> struct DgradB {
  static constexpr bool kRowVec = true;
  const T* w;  // [Co][KH][KW][Ci]
  Geo g;
  int K;       // KH*KW*Co
  uint32_t bytes;
  struct Ctx { int ci; bool ok; };
  typedef TapPrep Prep;
  __device__ __forceinline__ Ctx row_ctx(int r8) const { return Ctx{r8, r8 < g.Ci}; }
  __device__ __forceinline__ Prep prep(int k0) const { return tap_prep(g.dCo, g.dKW, k0); }
  __device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc() const { return mk_rsrc(w, bytes); }
  __device__ __forceinline__ uint32_t offs(const Ctx& c, const Prep& p, int kofs) const {
    const bool ok = c.ok && p.tap < g.KH * g.KW;
    return boff<T>((uint32_t)(((p.c0 + kofs) * g.KH * g.KW + p.tap) * g.Ci + c.ci), ok);
  }
  __device__ __forceinline__ typename VT<T>::v8 load(const Ctx& c, const Prep& p, int kofs) const {
    return bld8<T>(rsrc(), offs(c, p, kofs));
  }
};

// 8 consecutive columns (two f32x4) as one row vector of T
template <typename T> __device__ __forceinline__ void st8f(T* p, f32x4 lo, f32x4 hi) {
  typename VT<T>::v8 v;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    v[r] = fromf<T>(lo[r]);
    v[4 + r] = fromf<T>(hi[r]);
  }
  st8<T>(p, v);
}
template <typename T> __device__ __forceinline__ void ld8f(const T* p, f32x4& lo, f32x4& hi) {
  const typename VT<T>::v8 v = ld8<T>(p);
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    lo[r] = tof(v[r]);
    hi[r] = tof(v[4 + r]);
  }
}

// ---- strided dgrad by parity class (sub-pixel decomposition)
// Input pixels with (hi % sh, wi % sw) == (pc_h, pc_w) only receive gradient from taps with
// kh = (pc_h + ph) mod sh (same for w); for those taps ho = i + dh, wo = j + dw, linear in the
// class coordinates (hi = sh*i + pc_h). Each class is a dense GEMM over its own taps only.
// a TapTable entry by selects (static indices only: the grouped class kernel keeps its loaders in
// registers, where a dynamic array index would spill the table to scratch)
__device__ __forceinline__ int sel4(const int (&a)[4], int i) {
  return i == 0 ? a[0] : (i == 1 ? a[1] : (i == 2 ? a[2] : a[3]));
}

struct TapTable {
  int n;
  int dh[4], dw[4], id[4];  // per class tap: ho offset, wo offset, kh*KW + kw
  // fused 1x1 stride-2 downsample (crnn_conv_dgrad_ds): tap xtap reads the downsample's gradient,
  // stored right after dy (A: dw = B*Ho*Wo rows further, always in range), and its [Co][Ci]
  // weights, stored right after w (B: rows of Ci from element xb); -1 when absent
  int xtap = -1;
  int xb = 0;
};


template <typename T> struct DgradClsA {
  static constexpr bool kRowVec = false;
  const T* dy;
  Geo g;
  TapTable tt;
  int Hc, Wc, M, K;  // K = n * Co
  FastDiv dWc, dHcWc;
  uint32_t bytes;
  struct Ctx { int off; uint32_t mask; };
  typedef TapPrep Prep;
  __device__ __forceinline__ Ctx row_ctx(int m) const {
    Ctx c;
    uint32_t r, j;
    uint32_t b = dHcWc.divmod(m < M ? m : 0, r);
    uint32_t i = dWc.divmod(r, j);
    c.off = (((int)b * g.Ho + (int)i) * g.Wo + (int)j) * g.Co;
    c.mask = 0;
    if (m < M)
#pragma unroll
      for (int t = 0; t < 4; ++t)   // static bound: the table stays in registers (sel4)
        if (t < tt.n && (t == tt.xtap || ((unsigned)((int)i + tt.dh[t]) < (unsigned)g.Ho &&
                                          (unsigned)((int)j + tt.dw[t]) < (unsigned)g.Wo)))
          c.mask |= 1u << t;
    return c;
  }
  __device__ __forceinline__ Prep prep(int k0) const {
    TapPrep p;
    uint32_t co;
    p.tap = (int)g.dCo.divmod((uint32_t)k0, co);
    p.c0 = (int)co;
    const int t = p.tap < tt.n ? p.tap : 0;
    p.kh = sel4(tt.dh, t);
    p.kw = sel4(tt.dw, t);
    return p;
  }
  __device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc() const { return mk_rsrc(dy, bytes); }
  __device__ __forceinline__ uint32_t offs(const Ctx& c, const Prep& p, int kofs) const {
    const bool ok = (c.mask >> p.tap) & 1u;
    return boff<T>((uint32_t)(c.off + (p.kh * g.Wo + p.kw) * g.Co + p.c0 + kofs), ok);
  }
  __device__ __forceinline__ typename VT<T>::v8 load(const Ctx& c, const Prep& p, int kofs) const {
    return bld8<T>(rsrc(), offs(c, p, kofs));
  }
};

template <typename T> struct DgradClsB {
  static constexpr bool kRowVec = true;
  const T* w;  // [Co][KH][KW][Ci]
  Geo g;
  TapTable tt;
  int K;
  uint32_t bytes;
  struct Ctx { int ci; bool ok; };
  typedef TapPrep Prep;
  __device__ __forceinline__ Ctx row_ctx(int r8) const { return Ctx{r8, r8 < g.Ci}; }
  __device__ __forceinline__ Prep prep(int k0) const {
    TapPrep p;
    uint32_t co;
    p.tap = (int)g.dCo.divmod((uint32_t)k0, co);
    p.c0 = (int)co;
    p.kh = sel4(tt.id, p.tap < tt.n ? p.tap : 0);
    p.kw = p.tap == tt.xtap;  // the downsample's weights: rows of Ci after w
    return p;
  }
  __device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc() const { return mk_rsrc(w, bytes); }
  __device__ __forceinline__ uint32_t offs(const Ctx& c, const Prep& p, int kofs) const {
    const bool ok = c.ok && p.tap < tt.n;
    const int e = p.kw ? tt.xb + (p.c0 + kofs) * g.Ci + c.ci : ((p.c0 + kofs) * g.KH * g.KW + p.kh) * g.Ci + c.ci;
    return boff<T>((uint32_t)e, ok);
  }
  __device__ __forceinline__ typename VT<T>::v8 load(const Ctx& c, const Prep& p, int kofs) const {
    return bld8<T>(rsrc(), offs(c, p, kofs));
  }
};

// dx at class pixel (b, sh*i + pc_h, sw*j + pc_w) (+= if accumulate) (+ residual)
template <typename T> struct DgradClsEpi {
  static constexpr bool kStats = false;
  static constexpr bool kRow8 = true;
  T* dx;
  const T* dres;
  const T* yres;
  Geo g;
  int M, N, accumulate, pch, pcw;
  FastDiv dWc, dHcWc;
  __device__ __forceinline__ void store(int m, int n, f32x4 v, int) const {
    if (m >= M || n >= N) return;
    uint32_t r, j;
    uint32_t b = dHcWc.divmod(m, r);
    uint32_t i = dWc.divmod(r, j);
    const int hi = (int)i * g.sh + pch, wi = (int)j * g.sw + pcw;
    size_t o = ((size_t)((int)b * g.Hi + hi) * g.Wi + wi) * N + n;
    if (accumulate) v += ld4f<T>(dx + o);
    if (dres) {
      f32x4 d = ld4f<T>(dres + o), yy = ld4f<T>(yres + o);
#pragma unroll
      for (int q = 0; q < 4; ++q) v[q] += yy[q] > 0.f ? d[q] : 0.f;
    }
    st4<T>(dx + o, v);
  }
  // 8 consecutive channels of one class pixel: one 16-B store (gemm256 row8 epilogue)
  __device__ __forceinline__ void store8(int m, int n, f32x4 lo, f32x4 hi, int) const {
    if (m >= M || n >= N) return;
    uint32_t r, j;
    const uint32_t b = dHcWc.divmod(m, r);
    const uint32_t i = dWc.divmod(r, j);
    const int hi_ = (int)i * g.sh + pch, wi = (int)j * g.sw + pcw;
    const size_t o = ((size_t)((int)b * g.Hi + hi_) * g.Wi + wi) * N + n;
    if (accumulate) {
      f32x4 a, c;
      ld8f<T>(dx + o, a, c);
      lo += a;
      hi += c;
    }
    if (dres) {
      f32x4 d0, d1, y0, y1;
      ld8f<T>(dres + o, d0, d1);
      ld8f<T>(yres + o, y0, y1);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        lo[q] += y0[q] > 0.f ? d0[q] : 0.f;
        hi[q] += y1[q] > 0.f ? d1[q] : 0.f;
      }
    }
    st8f<T>(dx + o, lo, hi);
  }
  __device__ __forceinline__ void stats(int, int, f32x4, f32x4) const {}
};

// ---- wgrad A: dy rows = co, k = output pixel m (row-contiguous: dy[m][co..co+7])
template <typename T> struct WgradA {
  static constexpr bool kRowVec = true;
  const T* dy;
  int Co, M;
  uint32_t bytes;
  struct Ctx { int co; bool ok; };
  typedef int Prep;
  __device__ __forceinline__ Ctx row_ctx(int r8) const { return Ctx{r8, r8 < Co}; }
  __device__ __forceinline__ Prep prep(int k0) const { return k0; }
  __device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc() const { return mk_rsrc(dy, bytes); }
  __device__ __forceinline__ uint32_t offs(const Ctx& c, Prep k0, int kofs) const {
    const int m = k0 + kofs;
    return boff<T>((uint32_t)(m * Co + c.co), c.ok && m < M);
  }
  __device__ __forceinline__ typename VT<T>::v8 load(const Ctx& c, Prep k0, int kofs) const {
    return bld8<T>(rsrc(), offs(c, k0, kofs));
  }
};

// ---- wgrad B: im2col columns k' = (kh,kw,ci) as rows, k = output pixel m
template <typename T> struct WgradB {
  static constexpr bool kRowVec = true;
  const T* x;
  Geo g;
  int Kp, M;  // Kp = KH*KW*Ci
  uint32_t bytes;
  struct Ctx { int kh, kw, ci; bool ok; };
  typedef int Prep;
  __device__ __forceinline__ Ctx row_ctx(int r8) const {
    Ctx c;
    c.ok = r8 < Kp;
    uint32_t ci, kw;
    uint32_t tap = g.dCi.divmod(c.ok ? r8 : 0, ci);
    uint32_t kh = g.dKW.divmod(tap, kw);
    c.ci = (int)ci;
    c.kh = (int)kh - g.ph;
    c.kw = (int)kw - g.pw;
    return c;
  }
  __device__ __forceinline__ Prep prep(int k0) const { return k0; }
  __device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc() const { return mk_rsrc(x, bytes); }
  __device__ __forceinline__ uint32_t offs(const Ctx& c, Prep k0, int kofs) const {
    const int m = k0 + kofs;
    uint32_t r, wo;
    uint32_t b = g.dHoWo.divmod((uint32_t)m, r);
    uint32_t ho = g.dWo.divmod(r, wo);
    const int hi = (int)ho * g.sh + c.kh, wi = (int)wo * g.sw + c.kw;
    const bool ok = c.ok && m < M && (unsigned)hi < (unsigned)g.Hi && (unsigned)wi < (unsigned)g.Wi;
    return boff<T>((uint32_t)((((int)b * g.Hi + hi) * g.Wi + wi) * g.Ci + c.ci), ok);
  }
  __device__ __forceinline__ typename VT<T>::v8 load(const Ctx& c, Prep k0, int kofs) const {
    return bld8<T>(rsrc(), offs(c, k0, kofs));
  }
};

// ---- wgrad loaders for 64-aligned pixel tiles (the 256-row kernel's common case): every K-tile
// (64 output pixels, k0 % 64 == 0) lies inside one image (Ho*Wo % 64 == 0) and starts at a row
// start (Wo | 64) or inside one row (64 | Wo), so a pixel k0 + kr splits into per-tile scalars
// (image, first row, first column: SALU, once per K-tile) plus per-lane constants of the lane's
// k-row kr (hoisted out of the K-loop). The generic loaders above re-derive (b, ho, wo) per lane
// and per K-tile with 64-bit multiply-adds: 3x the VALU of the fwd loop.
template <typename T> struct WgradAF {
  static constexpr bool kRowVec = true;
  const T* dy;
  int Co;
  uint32_t bytes;
  struct Ctx { int co; bool ok; };
  typedef int Prep;   // k0 * Co
  __device__ __forceinline__ Ctx row_ctx(int r8) const { return Ctx{r8, r8 < Co}; }
  __device__ __forceinline__ Prep prep(int k0) const { return k0 * Co; }
  __device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc() const { return mk_rsrc(dy, bytes); }
  __device__ __forceinline__ uint32_t offs(const Ctx& c, Prep base, int kr) const {
    return c.ok ? (uint32_t)(base + kr * Co + c.co) * (uint32_t)sizeof(T) : OOB;
  }
  __device__ __forceinline__ typename VT<T>::v8 load(const Ctx& c, Prep p, int kofs) const {
    return bld8<T>(rsrc(), offs(c, p, kofs));
  }
};

template <typename T, bool WIDE> struct WgradBF {   // WIDE: Wo % 64 == 0, else 64 % Wo == 0
  static constexpr bool kRowVec = true;
  const T* x;
  Geo g;
  int Kp, lwo;        // lwo = log2(Wo) (narrow rows)
  uint32_t bytes;
  struct Ctx { int kh, kw, ci; bool ok; };
  struct Prep { int base, hs, ws; };   // element offset of (b, ho0*sh, wo0*sw, 0); row / column bases
  __device__ __forceinline__ Ctx row_ctx(int r8) const {
    Ctx c;
    c.ok = r8 < Kp;
    uint32_t ci, kw;
    uint32_t tap = g.dCi.divmod(c.ok ? r8 : 0, ci);
    uint32_t kh = g.dKW.divmod(tap, kw);
    c.ci = (int)ci;
    c.kh = (int)kh - g.ph;
    c.kw = (int)kw - g.pw;
    return c;
  }
  __device__ __forceinline__ Prep prep(int k0) const {
    uint32_t r, wo0;
    const uint32_t b = g.dHoWo.divmod((uint32_t)k0, r);
    const uint32_t ho0 = g.dWo.divmod(r, wo0);
    Prep p;
    p.hs = (int)ho0 * g.sh;
    p.ws = WIDE ? (int)wo0 * g.sw : 0;
    p.base = (((int)b * g.Hi + p.hs) * g.Wi + p.ws) * g.Ci;
    return p;
  }
  __device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc() const { return mk_rsrc(x, bytes); }
  __device__ __forceinline__ uint32_t offs(const Ctx& c, const Prep& p, int kr) const {
    // lane constants (loop-invariant): row / column offsets of this lane's pixel and tap
    const int dho = WIDE ? 0 : kr >> lwo;
    const int dwo = WIDE ? kr : kr & ((1 << lwo) - 1);
    const int lh = dho * g.sh + c.kh, lw = dwo * g.sw + c.kw;
    const int lc = (lh * g.Wi + lw) * g.Ci + c.ci;
    const bool okw = c.ok && (WIDE || (unsigned)lw < (unsigned)g.Wi);
    const bool ok = okw && (unsigned)(p.hs + lh) < (unsigned)g.Hi && (!WIDE || (unsigned)(p.ws + lw) < (unsigned)g.Wi);
    return ok ? (uint32_t)(p.base + lc) * (uint32_t)sizeof(T) : OOB;
  }
  __device__ __forceinline__ typename VT<T>::v8 load(const Ctx& c, const Prep& p, int kofs) const {
    return bld8<T>(rsrc(), offs(c, p, kofs));
  }
};

// the fast loaders' geometry condition (see WgradAF); 0 = generic, 1 = narrow rows, 2 = wide rows
inline int wgrad_fast_kind(const Geo& g) {
  const int HoWo = g.Ho * g.Wo;
  if (crnn_option(CRNN_OPT_WGRAD_FAST) == 0 || HoWo % 64) return 0;
  if (g.Wo % 64 == 0) return 2;
  if (64 % g.Wo == 0) return 1;
  return 0;
}

// ---- epilogues
// y = acc, or (eval-mode BN, esc != nullptr) y = ReLU(acc * esc[n] + esh[n]): the running-stat
// affine and the ReLU applied to the fp32 accumulators, so no z tensor and no bn_act pass

template <typename T> struct FwdEpi {
  static constexpr bool kStats = true;
  static constexpr bool kRow8 = true;
  T* y;
  float* psum;
  float* psq;
  int M, N;
  const float* esc = nullptr;
  const float* esh = nullptr;
  __device__ __forceinline__ void store(int m, int n, f32x4 v, int) const {
    if (m >= M || n >= N) return;
    if (esc) {
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = fmaxf(fmaf(v[r], esc[n + r], esh[n + r]), 0.f);
    }
    st4<T>(y + (size_t)m * N + n, v);
  }
  __device__ __forceinline__ void store8(int m, int n, f32x4 lo, f32x4 hi, int) const {
    if (m >= M || n >= N) return;
    if (esc) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        lo[r] = fmaxf(fmaf(lo[r], esc[n + r], esh[n + r]), 0.f);
        hi[r] = fmaxf(fmaf(hi[r], esc[n + 4 + r], esh[n + 4 + r]), 0.f);
      }
    }
    st8f<T>(y + (size_t)m * N + n, lo, hi);
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
  static constexpr bool kRow8 = true;
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
  __device__ __forceinline__ void store8(int m, int n, f32x4 lo, f32x4 hi, int) const {
    if (m >= M || n >= N) return;
    const size_t o = (size_t)m * N + n;
    if (accumulate) {
      f32x4 a, b;
      ld8f<T>(dx + o, a, b);
      lo += a;
      hi += b;
    }
    if (dres) {
      f32x4 d0, d1, y0, y1;
      ld8f<T>(dres + o, d0, d1);
      ld8f<T>(yres + o, y0, y1);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        lo[r] += y0[r] > 0.f ? d0[r] : 0.f;
        hi[r] += y1[r] > 0.f ? d1[r] : 0.f;
      }
    }
    st8f<T>(dx + o, lo, hi);
  }
  __device__ __forceinline__ void stats(int, int, f32x4, f32x4) const {}
};

// dgrad of a conv whose input went through BN -> ReLU (the next layer's BN backward, CRNN_BNG_RELU):
// stores dx and, per 128-row partial (the wave's rows of a 256-row tile), the BN sums
// sum g and sum g x^ over its rows, g = dx * (z scale + shift > 0), x^ = (z - mean) invstd, from
// the fp32 accumulators — the reduce pass over (dx, z) that would follow is not needed.
template <typename T> struct DgradBnEpi {
  static constexpr bool kStats = false;
  static constexpr bool kTileHook = true;
  static constexpr int kPrefer4W = 4;
  T* dx;
  int M, N;
  const T* z;
  const float* mean;
  const float* inv;
  const float* scale;
  const float* shift;
  float* pg;
  float* pgx;
  static constexpr bool kRow8 = true;
  __device__ __forceinline__ void store(int m, int n, f32x4 v, int) const {
    if (m < M && n < N) st4<T>(dx + (size_t)m * N + n, v);
  }
  __device__ __forceinline__ void store8(int m, int n, f32x4 lo, f32x4 hi, int) const {
    if (m < M && n < N) st8f<T>(dx + (size_t)m * N + n, lo, hi);
  }
  __device__ __forceinline__ void stats(int, int, f32x4, f32x4) const {}
  template <int MI, int NI>
  __device__ __forceinline__ void tile(const f32x4 (&acc)[MI][NI], int Mr, int rbase, int prow, int ncol0,
                                       int lane) const {
    const int mr = lane & 15, nq = 4 * (lane >> 4);
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      const int n = ncol0 + j * 16 + nq;
      const int nc = n < N ? n : N - 4;   // clamped: loads stay unconditional
      const f32x4 mu = *reinterpret_cast<const f32x4*>(mean + nc), iv = *reinterpret_cast<const f32x4*>(inv + nc);
      const f32x4 sc = *reinterpret_cast<const f32x4*>(scale + nc), sh = *reinterpret_cast<const f32x4*>(shift + nc);
      f32x4 s = {0.f, 0.f, 0.f, 0.f}, q = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        const int m = rbase + i * 16 + mr;
        const float ok = m < Mr ? 1.f : 0.f;
        const f32x4 zz = ld4f<T>(z + (size_t)(m < Mr ? m : Mr - 1) * N + nc);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float g = (zz[r] * sc[r] + sh[r]) > 0.f ? acc[i][j][r] * ok : 0.f;
          s[r] += g;
          q[r] += g * ((zz[r] - mu[r]) * iv[r]);
        }
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        s[r] = rowgroup_sum<16>(s[r]);
        q[r] = rowgroup_sum<16>(q[r]);
      }
      if (mr == 0 && n < N) {
        *reinterpret_cast<f32x4*>(pg + (size_t)prow * N + n) = s;
        *reinterpret_cast<f32x4*>(pgx + (size_t)prow * N + n) = q;
      }
    }
  }
};

struct SlabEpi {
  static constexpr bool kStats = false;
  static constexpr int kPrefer4W = 2;
  float* ws;  // [nsplit][Mrows][N], fp32 or (bf != 0, CRNN_OPT_WGRAD_SLAB_BF16) bf16
  int M, N, bf;
  __device__ __forceinline__ void store(int m, int n, f32x4 v, int kz) const {
    if (m >= M || n >= N) return;
    const size_t o = ((size_t)kz * M + m) * N + n;
    if (bf) st4<bf16>(reinterpret_cast<bf16*>(ws) + o, v);
    else *reinterpret_cast<f32x4*>(ws + o) = v;
  }
  __device__ __forceinline__ void stats(int, int, f32x4, f32x4) const {}
};

// sum split-K slabs [S][Co][KH*KW*Cip] and scatter into an OIHW fp32 gradient. A thread owns 4
// consecutive k' (one tap, 4 channels: Cip % 8 == 0) of one output row: 16-B slab loads, 8 slabs
// in flight per batch (the loop is otherwise latency-bound), fixed summation order.
// slab element loads: 4 consecutive fp32, or 4 bf16 (CRNN_OPT_WGRAD_SLAB_BF16) widened
template <bool BF> __device__ __forceinline__ f32x4 slab4(const float* ws, size_t o) {
  if constexpr (BF) return ld4f<bf16>(reinterpret_cast<const bf16*>(ws) + o);
  else return *reinterpret_cast<const f32x4*>(ws + o);
}

template <bool BF>
__global__ __launch_bounds__(256) void wgrad_reduce_kernel(const float* __restrict__ ws, int S,
                                                           float* __restrict__ dw, int Co, int Ci, int Cip, int KH,
                                                           int KW, float beta) {
  const int Kp = KH * KW * Cip;
  const long total = (long)Co * Kp, n4 = total / 4;
  for (long i4 = blockIdx.x * (long)blockDim.x + threadIdx.x; i4 < n4; i4 += (long)gridDim.x * blockDim.x) {
    const long i = 4 * i4;
    f32x4 s = {0.f, 0.f, 0.f, 0.f};
    int z = 0;
    for (; z + 8 <= S; z += 8) {
      f32x4 v[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) v[q] = slab4<BF>(ws, (size_t)(z + q) * total + i);
#pragma unroll
      for (int q = 0; q < 8; ++q) s += v[q];
    }
    for (; z < S; ++z) s += slab4<BF>(ws, (size_t)z * total + i);
    const int co = (int)(i / Kp), k = (int)(i - (long)co * Kp);
    const int tap = k / Cip, ci = k - tap * Cip;
    const int kh = tap / KW, kw = tap - kh * KW;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      if (ci + e >= Ci) break;
      const size_t o = (((size_t)co * Ci + ci + e) * KH + kh) * KW + kw;
      dw[o] = beta != 0.f ? beta * dw[o] + s[e] : s[e];
    }
  }
}

// the same sum, tiled: one workgroup per (co, 64-channel chunk of Cip). Slab loads as above (16 B,
// coalesced along ci; T * 16 vectors per slab, the slabs split over G = 256 / (T * 16) thread groups
// when the tile is narrow), partial sums transposed through LDS (pitch cc + 1: taps of one channel
// on different banks), then the OIHW rows [ci][kh][kw] of the chunk written contiguously. The
// flat kernel's 4-B stores land KH*KW floats apart; here every store is a coalesced run.
template <bool BF>
__global__ __launch_bounds__(256) void wgrad_reduce_tiled_kernel(const float* __restrict__ ws, int S,
                                                                 float* __restrict__ dw, int Ci, int Cip, int T,
                                                                 float beta) {
  __shared__ float red[2112];
  const int nchunk = (Cip + 63) / 64;
  const int co = blockIdx.x / nchunk, c0 = (blockIdx.x - co * nchunk) * 64;
  const int cc = min(64, Cip - c0), cv = cc / 4, nv = T * cv, P = cc + 1;
  const int G = max(1, 256 / nv);
  const long Kp = (long)T * Cip, total = Kp * (long)gridDim.x / nchunk;
  const int t = threadIdx.x, g = t / nv, v = t - g * nv;
  if (g < G) {
    const int tap = v / cv, c = 4 * (v - tap * cv);
    const size_t src = (size_t)co * Kp + (size_t)tap * Cip + c0 + c;
    f32x4 s = {0.f, 0.f, 0.f, 0.f};
    int z = g;
    for (; z + 7 * G < S; z += 8 * G) {
      f32x4 r[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) r[q] = slab4<BF>(ws, src + (size_t)(z + q * G) * total);
#pragma unroll
      for (int q = 0; q < 8; ++q) s += r[q];
    }
    for (; z < S; z += G) s += slab4<BF>(ws, src + (size_t)z * total);
    float* d = red + (g * T + tap) * P + c;
#pragma unroll
    for (int e = 0; e < 4; ++e) d[e] = s[e];
  }
  __syncthreads();
  const int cr = min(cc, Ci - c0);  // real (unpadded) channels of the chunk
  float* out = dw + ((size_t)co * Ci + c0) * T;
  for (int o = t; o < cr * T; o += 256) {
    const int ci = o / T, tap = o - ci * T;
    float a = 0.f;
    for (int q = 0; q < G; ++q) a += red[(q * T + tap) * P + ci];
    out[o] = beta != 0.f ? beta * out[o] + a : a;
  }
}

inline uint32_t nbytes(long elems, size_t es) { return (uint32_t)((size_t)elems * es); }

// the 256-row kernel's padding-row fragment skip (gemm256.hpp SKIP): a 3x3 / stride-1 / pad-1 conv
// over 4-row maps of 128 pixels (layer3 / layer4: 4 x 32), so each wave's 128 rows are one image
// and the rows reading only padding are the same two fragment rows in every wave
inline bool pad_skip_ok(const Geo& g, int rows, int cols) {
  return crnn_option(CRNN_OPT_PAD_SKIP) != 0 && g.KH == 3 && g.KW == 3 && g.sh == 1 && g.sw == 1 && g.ph == 1 &&
         g.pw == 1 && rows == 4 && rows * cols == 128;
}

// the W-halo A image kernel (gemm256hw.hpp) for this forward-form geometry, or -1
inline int halo_w_lwo(const Geo& g) {
  if (!crnn_option(CRNN_OPT_CONV_HALO_W)) return -1;
  if (g.KH != 3 || g.KW != 3 || g.sh != 1 || g.sw != 1 || g.ph != 1 || g.pw != 1) return -1;
  if (g.Hi != g.Ho || g.Wi != g.Wo || g.Ci % 64) return -1;
  return gemm::halo_w_log2(g.Wo);
}

// the 256-row launch of a forward-form conv (FwdA loader, K-contiguous weights [N][K]): the W-halo kernel
// when the geometry takes it, else gemm256 (with the padding-row skip on 4-row maps)
template <class EPI>
int launch_fwd256(const Geo& g, const FwdA<bf16, true>& la, const RowMajorK<bf16>& lb, const EPI& ep, int M, int N,
                  int K, int bn, hipStream_t st, bool dgrad = false) {
  const bool skip = pad_skip_ok(g, g.Ho, g.Wo);
  const int lwo = halo_w_lwo(g);
  // (the image contexts pack element offsets in 29 bits; the padding-skip form with the BN-backward tile
  // hook at BN = 256 exceeds the 256-register budget inside the K loop: the K-tile images there, so on
  // 4-row maps the dgrad's plain and BN-ReLU forms sum K in different orders)
  (void)dgrad;
  if (lwo >= 0 && la.bytes < (1u << 30) && !(gemm::has_tile_hook<EPI>::value && skip && bn == 256)) {
    const gemm::HaloWDesc a{la.x, la.bytes, g.B, g.Ho, g.Wo, g.Ci, lwo, g.Ci / 64};
    if (skip) {
      if (bn == 256) return gemm::launch256hw<256, 1>(a, lb, ep, M, N, st);
      return gemm::launch256hw<128, 1>(a, lb, ep, M, N, st);
    }
    if (bn == 256) return gemm::launch256hw<256, 0>(a, lb, ep, M, N, st);
    return gemm::launch256hw<128, 0>(a, lb, ep, M, N, st);
  }
  if (skip) {
    const int ktk = g.KW * g.Ci / 64;
    if (bn == 256) return launch256<256, 256, 1>(la, lb, ep, M, N, K, st, 1, 1, ktk);
    return launch256<256, 128, 1>(la, lb, ep, M, N, K, st, 1, 1, ktk);
  }
  if (bn == 256) return launch256<256, 256>(la, lb, ep, M, N, K, st);
  return launch256<256, 128>(la, lb, ep, M, N, K, st);
}


template <typename T, bool UT>
int conv_fwd_tt(const Geo& g, const crnn_conv_desc* d, const void* x, const void* w, void* y, float* psum,
                float* psq, const float* esc, const float* esh, hipStream_t st) {
  int M = g.B * g.Ho * g.Wo, N = g.Co, K = g.KH * g.KW * g.Ci;
  FwdA<T, UT> la{(const T*)x, g, M, K, nbytes((long)g.B * g.Hi * g.Wi * g.Ci, sizeof(T))};
  RowMajorK<T> lb{(const T*)w, K, N, K};
  FwdEpi<T> ep{(T*)y, psum, psq, M, N, esc, esh};
  if (crnn_option(CRNN_OPT_DIAG) & 1) ep.M = 0;   // diagnostic: no output stores
  int bm, bn;
  crnn_conv_fwd_tile(sizeof(T) == 2 ? CRNN_BF16 : CRNN_F32, d, &bm, &bn);
  if constexpr (sizeof(T) == 2 && UT) {
    if (bm == 256 && (bn == 256 || bn == 128)) return launch_fwd256(g, la, lb, ep, M, N, K, bn, st);
  }
  if (bm == 128 && bn == 128) return launch<T, 128, 128>(la, lb, ep, M, N, K, 1, st);
  if (bm == 128 && bn == 64) return launch<T, 128, 64>(la, lb, ep, M, N, K, 1, st);
  return launch<T, 64, 64>(la, lb, ep, M, N, K, 1, st);
}

template <typename T> int conv_fwd_t(const crnn_conv_desc* d, const void* x, const void* w, void* y,
                                     float* psum, float* psq, hipStream_t st, const float* esc = nullptr,
                                     const float* esh = nullptr) {
  Geo g = geo(d);
  if (g.Ci % kstage<T>() == 0) return conv_fwd_tt<T, true>(g, d, x, w, y, psum, psq, esc, esh, st);
  return conv_fwd_tt<T, false>(g, d, x, w, y, psum, psq, esc, esh, st);
}

inline int ilog2s(int s) { return s == 1 ? 0 : (s == 2 ? 1 : -1); }

// BN of the deep dgrad kernel for an (M = input pixels, N = Ci) GEMM, or 0 for the 128/64 kernels
// min_tiles: the grid must hold at least this many 256-row tiles (1 block per CU)
template <typename T> int deep_dgrad_bn(long M, int N, int Co, long min_tiles) {
  if (sizeof(T) != 2 || Co % 64 || N % 128) return 0;
  if (N % 256 == 0 && M * N >= 256L * 256 * min_tiles) return 256;
  if (M * N >= 256L * 128 * min_tiles) return 128;
  return 0;
}

// the 256-row kernel's share of the CUs in its last round of tiles (1 block per CU): a grid of
// 264 tiles runs two rounds, the second nearly empty
inline double round_eff(long tiles) {
  const long ncu = crnn_cu_count();
  return (double)tiles / (double)(((tiles + ncu - 1) / ncu) * ncu);
}
// CRNN_OPT_QUANT_TILE: a deep-kernel grid that fills its last round this badly runs on the 128x128
// kernel (two blocks per CU, 4x the tiles, balanced) instead. The 128x128 kernel's rate relative to
// the 256-row kernel (measured on conv_out: ~0.4 of the 256 x 256 tile, ~0.6 of the 256 x 128
// tile) is the break-even share of the CUs: below it the smaller tiles finish first
inline double quant_eff(int bn) { return bn == 256 ? 0.4 : 0.6; }

// ---- all parity classes of a strided dgrad in ONE launch (CRNN_OPT_DGRAD_GROUP): a grouped tile
// table over the classes' GEMMs (same N = Ci and tile shape, own M, K and taps), longest K first so
// the long tiles start in the first round. Per launch this removes the class launches' partial last
// rounds and their launch gaps (a class GEMM is short-K: 1-4 taps x Co). Each block picks its class
// from the table (wave-uniform), rebuilds the class's loaders from the shared base and runs the
// ordinary 256-row work item.
struct ClsRec {
  TapTable tt;
  int Hc, Wc, M, K, pch, pcw, start, tiles;
  FastDiv dWc, dHcWc;
};
constexpr int MAX_CLS = 4;
template <typename T> struct ClsGroup {
  DgradClsA<T> la;
  DgradClsB<T> lb;
  DgradClsEpi<T> ep;
  ClsRec c[MAX_CLS];
  int ng, tn, total;
};

template <typename T, int BN>
__global__ __launch_bounds__(512) void dgrad_cls_group_kernel(const ClsGroup<T> G, int stagger) {
  // blocks in table order (dispatch is round-robin over the XCDs, so every class spreads evenly over
  // them); the XCD-contiguous remap only WITHIN a class (over the whole table it gave the first XCDs
  // all of the longest class: 1.4x slower)
  const int wb = blockIdx.x;
  int g = 0;
#pragma unroll
  for (int i = 1; i < MAX_CLS; ++i) g += (i < G.ng && wb >= G.c[i].start) ? 1 : 0;
  // the class record by wave-uniform selects (a dynamic index into the kernel-argument array would
  // copy it to scratch)
  ClsRec r = G.c[0];
#pragma unroll
  for (int i = 1; i < MAX_CLS; ++i)
    if (g == i) r = G.c[i];
  DgradClsA<T> la = G.la;
  la.tt = r.tt;
  la.Hc = r.Hc;
  la.Wc = r.Wc;
  la.M = r.M;
  la.K = r.K;
  la.dWc = r.dWc;
  la.dHcWc = r.dHcWc;
  DgradClsB<T> lb = G.lb;
  lb.tt = r.tt;
  lb.K = r.K;
  DgradClsEpi<T> ep = G.ep;
  ep.M = r.M;
  ep.pch = r.pch;
  ep.pcw = r.pcw;
  ep.dWc = r.dWc;
  ep.dHcWc = r.dHcWc;
  const int local = xcd_remap(wb - r.start, r.tiles);
  gemm256_item<256, BN, 0>(la, lb, ep, r.M, r.K, r.K, local / G.tn, local % G.tn, 0, stagger, 0);
}

// rows: row classes (each input row its own class, Hc = 1) instead of parity classes in height —
// for maps of 1-2 output rows (conv_out[1]: Ho = 1), where half of a generic dgrad's taps read
// nothing but padding rows; the stride may then be 1
// ds: the 1x1 stride-2 downsample of the same block is fused in (crnn_conv_dgrad_ds): its gradient
// (B*Ho*Wo*Co, right after dy) and weights ([Co][Ci], right after w) are one more tap of the class
// (0, 0), whose pixels (2i, 2j) it reaches from output (i, j)
template <typename T>
int conv_dgrad_strided(const Geo& g, const void* dy, const void* w, void* dx, const void* dres, const void* yres,
                       int accumulate, hipStream_t st, bool rows = false, bool ds = false) {
  const long dyn = (long)g.B * g.Ho * g.Wo * g.Co, wn = (long)g.Co * g.KH * g.KW * g.Ci;
  const uint32_t dyb = nbytes(ds ? 2 * dyn : dyn, sizeof(T));
  const uint32_t wb = nbytes(ds ? wn + (long)g.Co * g.Ci : wn, sizeof(T));
  // grouped form: every class on the 256 x 128 tile of the 256-row kernel (bf16, Ci % 128 == 0)
  ClsRec recs[MAX_CLS];
  int nrec = 0;
  bool group = sizeof(T) == 2 && crnn_option(CRNN_OPT_DGRAD_GROUP) != 0 && !rows && g.Ci % 128 == 0 &&
               g.Co % 64 == 0 && g.sh * g.sw <= MAX_CLS;
  for (int pass = group ? 0 : 1; pass < 2; ++pass) {
  for (int pch = 0; pch < (rows ? g.Hi : g.sh); ++pch)
    for (int pcw = 0; pcw < g.sw; ++pcw) {
      TapTable tt{};
      for (int kh = 0; kh < g.KH; ++kh) {
        if (((pch + g.ph - kh) % g.sh + g.sh) % g.sh) continue;
        if (rows && (pch + g.ph - kh < 0 || (pch + g.ph - kh) / g.sh >= g.Ho)) continue;
        for (int kw = 0; kw < g.KW; ++kw) {
          if (((pcw + g.pw - kw) % g.sw + g.sw) % g.sw) continue;
          if (tt.n >= 4) return crnn_set_error(hipErrorInvalidValue, "conv_dgrad: > 4 taps per parity class");
          tt.dh[tt.n] = (pch + g.ph - kh) / g.sh;
          tt.dw[tt.n] = (pcw + g.pw - kw) / g.sw;
          tt.id[tt.n] = kh * g.KW + kw;
          ++tt.n;
        }
      }
      if (ds && pch == 0 && pcw == 0) {
        if (tt.n >= 4) return crnn_set_error(hipErrorInvalidValue, "conv_dgrad_ds: class (0, 0) is full");
        tt.xtap = tt.n;
        tt.xb = (int)wn;
        tt.dh[tt.n] = 0;
        tt.dw[tt.n] = g.B * g.Ho * g.Wo;  // A rows: the downsample's gradient follows dy
        tt.id[tt.n] = 0;
        ++tt.n;
      }
      const int Hc = rows ? 1 : (g.Hi - pch + g.sh - 1) / g.sh, Wc = (g.Wi - pcw + g.sw - 1) / g.sw;
      if (Hc <= 0 || Wc <= 0) continue;
      // a class no tap reaches contributes 0: with accumulate and no residual term it leaves dx
      // as it is (the 1x1 stride-2 downsample: 3 of 4 classes), so skip its read + write pass
      if (tt.n == 0 && accumulate && dres == nullptr) continue;
      const int M = g.B * Hc * Wc, N = g.Ci, K = tt.n * g.Co;
      FastDiv dWc(Wc), dHcWc(Hc * Wc);
      if (pass == 0) {   // grouped form: collect the class; a class off the 256 x 128 tile ends the group
        if (tt.n == 0 || deep_dgrad_bn<T>(M, N, g.Co, 64) == 0) {
          group = false;
          break;
        }
        recs[nrec++] = ClsRec{tt, Hc, Wc, M, K, pch, pcw, 0, 0, dWc, dHcWc};
        continue;
      }
      DgradClsA<T> la{(const T*)dy, g, tt, Hc, Wc, M, K, dWc, dHcWc, dyb};
      DgradClsB<T> lb{(const T*)w, g, tt, K, wb};
      DgradClsEpi<T> ep{(T*)dx, (const T*)dres, (const T*)yres, g, M, N, accumulate, pch, pcw, dWc, dHcWc};
      int rc = 0;
      int deep = deep_dgrad_bn<T>(M, N, g.Co, 256);
      if (deep && crnn_option(CRNN_OPT_QUANT_TILE) && round_eff((M + 255) / 256 * (N / deep)) < quant_eff(deep)) deep = 0;
      if constexpr (sizeof(T) == 2) {
        if (deep == 256) rc = launch256<256, 256>(la, lb, ep, M, N, K, st);
        else if (deep == 128) rc = launch256<256, 128>(la, lb, ep, M, N, K, st);
      }
      if (deep) {
      } else if (N >= 128 && (long)M * N >= 128L * 128 * 256) rc = launch<T, 128, 128>(la, lb, ep, M, N, K, 1, st);
      else rc = launch<T, 64, 64>(la, lb, ep, M, N, K, 1, st);
      if (rc) return rc;
    }
    if (pass == 0) {
      if (!group || nrec == 0) continue;    // fall back: a launch per class
      // longest K first (insertion sort, <= 4 records), then the tile table
      for (int i = 1; i < nrec; ++i)
        for (int j = i; j > 0 && recs[j].K > recs[j - 1].K; --j) std::swap(recs[j], recs[j - 1]);
      ClsGroup<T> G{};
      // CRNN_OPT_DGRAD_GROUP = 2: 256 x 256 tiles when Ci allows (half the tiles, each A row gathered once
      // for 256 output channels instead of twice)
      const int bn = crnn_option(CRNN_OPT_DGRAD_GROUP) == 2 && g.Ci % 256 == 0 ? 256 : 128;
      const int tn = g.Ci / bn;
      int total = 0;
      for (int i = 0; i < nrec; ++i) {
        recs[i].start = total;
        recs[i].tiles = (recs[i].M + 255) / 256 * tn;
        total += recs[i].tiles;
        G.c[i] = recs[i];
      }
      const ClsRec& r0 = recs[0];
      G.la = DgradClsA<T>{(const T*)dy, g, r0.tt, r0.Hc, r0.Wc, r0.M, r0.K, r0.dWc, r0.dHcWc, dyb};
      G.lb = DgradClsB<T>{(const T*)w, g, r0.tt, r0.K, wb};
      G.ep = DgradClsEpi<T>{(T*)dx, (const T*)dres, (const T*)yres, g, r0.M, g.Ci, accumulate, r0.pch, r0.pcw,
                            r0.dWc, r0.dHcWc};
      G.ng = nrec;
      G.tn = tn;
      G.total = total;
      if constexpr (sizeof(T) == 2) {
        if (bn == 256)
          hipLaunchKernelGGL((dgrad_cls_group_kernel<T, 256>), dim3(total), dim3(512), 0, st, G,
                             crnn_option(CRNN_OPT_GEMM_STAGGER));
        else
          hipLaunchKernelGGL((dgrad_cls_group_kernel<T, 128>), dim3(total), dim3(512), 0, st, G,
                             crnn_option(CRNN_OPT_GEMM_STAGGER));
        return (int)hipGetLastError();
      }
    }
  }
  return 0;
}

template <typename T> int conv_dgrad_t(const crnn_conv_desc* d, const void* dy, const void* w, void* dx,
                                       const void* dres, const void* yres, int accumulate, hipStream_t st) {
  Geo g = geo(d);
  if ((g.sh > 1 || g.sw > 1) && g.Co % kstage<T>() == 0)
    return conv_dgrad_strided<T>(g, dy, w, dx, dres, yres, accumulate, st);
  if (g.Hi <= 2 && g.KH > 1 && g.Co % kstage<T>() == 0 && crnn_option(CRNN_OPT_ROW_CLASS))
    return conv_dgrad_strided<T>(g, dy, w, dx, dres, yres, accumulate, st, true);
  int M = g.B * g.Hi * g.Wi, N = g.Ci, K = g.KH * g.KW * g.Co;
  int lsh = ilog2s(g.sh), lsw = ilog2s(g.sw);
  if (lsh < 0 || lsw < 0 || g.Co % kstage<T>())
    return crnn_set_error(hipErrorInvalidValue, "conv_dgrad: strides must be 1 or 2, Co a multiple of the stage depth");
  DgradA<T> la{(const T*)dy, g, M, K, lsh, lsw, nbytes((long)g.B * g.Ho * g.Wo * g.Co, sizeof(T))};
  DgradB<T> lb{(const T*)w, g, K, nbytes((long)g.Co * g.KH * g.KW * g.Ci, sizeof(T))};
  DgradEpi<T> ep{(T*)dx, (const T*)dres, (const T*)yres, M, N, accumulate};
  if (crnn_option(CRNN_OPT_DIAG) & 1) ep.M = 0;   // diagnostic: no output stores
  if constexpr (sizeof(T) == 2) {
    int deep = deep_dgrad_bn<T>(M, N, g.Co, 128);
    if (deep && crnn_option(CRNN_OPT_QUANT_TILE) && round_eff(((long)M + 255) / 256 * (N / deep)) < quant_eff(deep)) deep = 0;
    if (deep && pad_skip_ok(g, g.Hi, g.Wi)) {
      const int ktk = g.KW * g.Co / 64;
      if (deep == 256) return launch256<256, 256, 2>(la, lb, ep, M, N, K, st, 1, 1, ktk);
      return launch256<256, 128, 2>(la, lb, ep, M, N, K, st, 1, 1, ktk);
    }
    if (deep == 256) return launch256<256, 256>(la, lb, ep, M, N, K, st);
    if (deep == 128) return launch256<256, 128>(la, lb, ep, M, N, K, st);
  }
  if (N >= 128 && (long)M * N >= 128L * 128 * 256) return launch<T, 128, 128>(la, lb, ep, M, N, K, 1, st);
  if (N <= 64 && (long)M * N >= 128L * 64 * 256) return launch<T, 128, 64>(la, lb, ep, M, N, K, 1, st);
  return launch<T, 64, 64>(la, lb, ep, M, N, K, 1, st);
}

// stride-1 dgrad on the 256-row kernel with the BN-ReLU backward sums (DgradBnEpi); the number of
// partial rows, or 0 when the geometry does not take the 256-row path (caller: unfused)
inline int dgrad_bnrelu_rows(const crnn_conv_desc* d) {
  if (d->sh != 1 || d->sw != 1 || d->Co % 64 || d->Ci % 8) return 0;
  const long M = (long)d->B * d->Hi * d->Wi;
  const int deep = deep_dgrad_bn<bf16>(M, d->Ci, d->Co, 128);
  if (!deep) return 0;
  // the plain dgrad of this geometry would leave the 256-row kernel (CRNN_OPT_QUANT_TILE): so does
  // the fused one (callers then run the unfused pair)
  if (crnn_option(CRNN_OPT_QUANT_TILE) && round_eff((M + 255) / 256 * (d->Ci / deep)) < quant_eff(deep)) return 0;
  return (int)((M + 255) / 256 * 2);
}

int conv_dgrad_bnrelu(const crnn_conv_desc* d, const void* dy, const void* w, void* dx, const void* z,
                      const float* mean, const float* inv, const float* scale, const float* shift, float* pg,
                      float* pgx, hipStream_t st) {
  using T = bf16;
  Geo g = geo(d);
  const int M = g.B * g.Hi * g.Wi, N = g.Ci, K = g.KH * g.KW * g.Co;
  DgradA<T> la{(const T*)dy, g, M, K, 0, 0, nbytes((long)g.B * g.Ho * g.Wo * g.Co, sizeof(T))};
  DgradB<T> lb{(const T*)w, g, K, nbytes((long)g.Co * g.KH * g.KW * g.Ci, sizeof(T))};
  DgradBnEpi<T> ep{(T*)dx, M, N, (const T*)z, mean, inv, scale, shift, pg, pgx};
  const int deep = deep_dgrad_bn<T>(M, N, g.Co, 128);
  if (pad_skip_ok(g, g.Hi, g.Wi)) {
    const int ktk = g.KW * g.Co / 64;
    if (deep == 256) return launch256<256, 256, 2>(la, lb, ep, M, N, K, st, 1, 1, ktk);
    return launch256<256, 128, 2>(la, lb, ep, M, N, K, st, 1, 1, ktk);
  }
  if (deep == 256) return launch256<256, 256>(la, lb, ep, M, N, K, st);
  return launch256<256, 128>(la, lb, ep, M, N, K, st);
}

// ---- stride-1 dgrad on the FORWARD conv path ("tw": transposed weights)
// dgrad(dy)[b,hi,wi,ci] = sum_{kh',kw',co} dy[b, hi - (KH-1-ph) + kh', wi - (KW-1-pw) + kw', co] * wt[ci][kh'][kw'][co]
// with wt[ci][kh'][kw'][co] = w[co][KH-1-kh'][KW-1-kw'][ci]: a forward conv of dy (Ci' = Co, Co' = Ci,
// pad' = K-1-pad) with the flipped, transposed kernel, packed K-contiguous like a forward weight. So
// the dgrad runs the forward's A loader, its K-contiguous B fragments (ds_read_b128, not the
// row-contiguous transposed reads of DgradB), its tile rules and its padding-row skip, with the
// dgrad epilogues (DgradEpi / DgradBnEpi store by (input pixel, ci) exactly like the native path).
inline crnn_conv_desc dgrad_fwd_desc(const crnn_conv_desc* d) {
  crnn_conv_desc t{d->B, d->Ho, d->Wo, d->Co, d->Hi, d->Wi, d->Ci, d->KH, d->KW, 1, 1,
                   d->KH - 1 - d->ph, d->KW - 1 - d->pw, d->Co};
  return t;
}

// the tw path takes this geometry: bf16, stride 1, whole 64-channel K stages, the 256-row tile
inline bool dgrad_tw_ok(const crnn_conv_desc* d) {
  if (d->sh != 1 || d->sw != 1 || d->Co % 64 || d->Ci % 8) return false;
  if (d->ph > d->KH - 1 || d->pw > d->KW - 1) return false;
  if (use_halo(CRNN_BF16, d, true)) return false;
  const crnn_conv_desc t = dgrad_fwd_desc(d);
  if (t.Ho != d->Hi || t.Wo != d->Wi) return false;
  int bm, bn;
  crnn_conv_fwd_tile(CRNN_BF16, &t, &bm, &bn);
  return bm == 256;
}

template <class EPI>
int conv_dgrad_tw_launch(const crnn_conv_desc* d, const void* dy, const void* wt, const EPI& ep, hipStream_t st) {
  using T = bf16;
  const crnn_conv_desc t = dgrad_fwd_desc(d);
  const Geo g = geo(&t);
  const int M = g.B * g.Ho * g.Wo, N = g.Co, K = g.KH * g.KW * g.Ci;
  FwdA<T, true> la{(const T*)dy, g, M, K, nbytes((long)g.B * g.Hi * g.Wi * g.Ci, sizeof(T))};
  RowMajorK<T> lb{(const T*)wt, K, N, K};
  int bm, bn;
  crnn_conv_fwd_tile(CRNN_BF16, &t, &bm, &bn);
  if (bm != 256) return crnn_set_error(hipErrorInvalidValue, "conv_dgrad_tw: geometry not on the 256-row path");
  return launch_fwd256(g, la, lb, ep, M, N, K, bn, st, true);
}

// bf16 partial slabs (CRNN_OPT_WGRAD_SLAB_BF16, default on): only for bf16 operands on the GEMM forms (the
// halo stem kernels write their own fp32 slabs; fp32 convs keep fp32 slabs). Each partial is rounded to bf16
// once and the reduce sums in fp32: about one bf16 rounding of the gradient, as a bf16 weight gradient under
// the reference's AMP has, for half the slab bytes written and re-read.
template <typename T> bool wgrad_slab_bf16(int bm) {
  return sizeof(T) == 2 && bm != 0 && crnn_option(CRNN_OPT_WGRAD_SLAB_BF16) != 0;
}

// phases: bit 0 = the split-K GEMM into the fp32 slabs, bit 1 = the slab reduce into the OIHW gradient
// (crnn_conv_wgrad_gemm / _reduce run them apart, so the reduce can go to another stream)
template <typename T> int conv_wgrad_t(const crnn_conv_desc* d, const void* dy, const void* x, float* dw,
                                       float* ws, size_t ws_bytes, float beta, hipStream_t st, int phases = 3) {
  Geo g = geo(d);
  int Mp = g.B * g.Ho * g.Wo, Kp = g.KH * g.KW * g.Ci;
  int bm, bn, splits;
  crnn_conv_wgrad_plan(sizeof(T) == 2 ? CRNN_BF16 : CRNN_F32, d, &bm, &bn, &splits);
  size_t need = (size_t)splits * g.Co * Kp * sizeof(float);
  if (ws_bytes < need) return crnn_set_error(hipErrorInvalidValue, "conv_wgrad: workspace too small");
  int rc = 0;
  if (!(phases & 1)) {
  } else if (bm == 0) {  // halo-tiled direct kernel (plan: bm = bn = 0), one slab per workgroup
    rc = conv_halo_wgrad(d, dy, x, ws, st);
  } else {
  WgradA<T> la{(const T*)dy, g.Co, Mp, nbytes((long)Mp * g.Co, sizeof(T))};
  WgradB<T> lb{(const T*)x, g, Kp, Mp, nbytes((long)g.B * g.Hi * g.Wi * g.Ci, sizeof(T))};
  SlabEpi ep{ws, g.Co, Kp, wgrad_slab_bf16<T>(bm) ? 1 : 0};
  if (crnn_option(CRNN_OPT_DIAG) & 1) ep.M = 0;   // diagnostic: no slab stores
  if constexpr (sizeof(T) == 2) {
    const int fk = bm == 256 ? wgrad_fast_kind(g) : 0;
    if (fk) {
      WgradAF<T> fa{(const T*)dy, g.Co, la.bytes};
      int lwo = 0;
      while ((1 << lwo) < g.Wo) ++lwo;
      WgradBF<T, true> fbw{(const T*)x, g, Kp, lwo, lb.bytes};
      WgradBF<T, false> fbn{(const T*)x, g, Kp, lwo, lb.bytes};
      if (bn == 256) rc = fk == 2 ? launch256<256, 256>(fa, fbw, ep, g.Co, Kp, Mp, st, splits)
                                  : launch256<256, 256>(fa, fbn, ep, g.Co, Kp, Mp, st, splits);
      else rc = fk == 2 ? launch256<256, 128>(fa, fbw, ep, g.Co, Kp, Mp, st, splits)
                        : launch256<256, 128>(fa, fbn, ep, g.Co, Kp, Mp, st, splits);
    } else if (bm == 256 && bn == 256) rc = launch256<256, 256>(la, lb, ep, g.Co, Kp, Mp, st, splits);
    else if (bm == 256 && bn == 128) rc = launch256<256, 128>(la, lb, ep, g.Co, Kp, Mp, st, splits);
  }
  if (bm == 256) {
  } else if (bm == 128) rc = launch<T, 128, 128>(la, lb, ep, g.Co, Kp, Mp, splits, st);
  else rc = launch<T, 64, 64>(la, lb, ep, g.Co, Kp, Mp, splits, st);
  }
  if (rc || !(phases & 2)) return rc;
  int ci_real = d->Ci_real > 0 ? d->Ci_real : g.Ci;
  long total = (long)g.Co * Kp;
  const bool bfr = wgrad_slab_bf16<T>(bm);   // as the GEMM phase wrote them
  if (crnn_option(CRNN_OPT_WGRAD_REDUCE) != 0 && g.KH * g.KW <= 16 && g.Ci % 8 == 0) {
    if (bfr)
      hipLaunchKernelGGL(wgrad_reduce_tiled_kernel<true>, dim3(g.Co * ((g.Ci + 63) / 64)), dim3(256), 0, st, ws,
                         splits, dw, ci_real, g.Ci, g.KH * g.KW, beta);
    else
      hipLaunchKernelGGL(wgrad_reduce_tiled_kernel<false>, dim3(g.Co * ((g.Ci + 63) / 64)), dim3(256), 0, st, ws,
                         splits, dw, ci_real, g.Ci, g.KH * g.KW, beta);
    return (int)hipGetLastError();
  }
  int blocks = (int)((total / 4 + 255) / 256);
  if (blocks > 4096) blocks = 4096;
  if (bfr)
    hipLaunchKernelGGL(wgrad_reduce_kernel<true>, dim3(blocks), dim3(256), 0, st, ws, splits, dw, g.Co, ci_real,
                       g.Ci, g.KH, g.KW, beta);
  else
    hipLaunchKernelGGL(wgrad_reduce_kernel<false>, dim3(blocks), dim3(256), 0, st, ws, splits, dw, g.Co, ci_real,
                       g.Ci, g.KH, g.KW, beta);
  return (int)hipGetLastError();
}

}  // namespace

extern "C" {

void crnn_conv_fwd_tile(int dtype, const crnn_conv_desc* d, int* bm, int* bn) {
  long M = (long)d->B * d->Ho * d->Wo;
  // the 256-row kernel: bf16, whole 64-deep K-tiles inside one tap, >= ~1 block per CU
  const bool deep = dtype == CRNN_BF16 && d->Ci % 64 == 0 && d->Co % 128 == 0 && d->Co >= CRNN_DEEP_MIN_CO;
  if (deep && d->Co >= 256 && M * d->Co >= 256L * 256 * 128) { *bm = 256; *bn = 256; }
  else if (deep && M * d->Co >= 256L * 128 * 128) { *bm = 256; *bn = 128; }
  else { *bm = 0; }
  if (*bm == 256 && crnn_option(CRNN_OPT_QUANT_TILE) && round_eff((M + 255) / 256 * (d->Co / *bn)) < quant_eff(*bn))
    *bm = 0;
  if (*bm == 256) return;
  if (d->Co <= 64) { *bm = 128; *bn = 64; }
  else if (M * d->Co >= 128L * 128 * 192) { *bm = 128; *bn = 128; }
  else { *bm = 64; *bn = 64; }
}

int crnn_conv_stat_rows_per_partial(int dtype, const crnn_conv_desc* d) {
  if (use_halo(dtype, d, false)) return 64;  // one partial per wave: 64 pixels
  int bm, bn;
  crnn_conv_fwd_tile(dtype, d, &bm, &bn);
  return bm / 2;
}

int crnn_conv_stat_rows(int dtype, const crnn_conv_desc* d) {
  if (use_halo(dtype, d, false)) return (int)((long)d->B * d->Ho * d->Wo / 64);
  int bm, bn;
  crnn_conv_fwd_tile(dtype, d, &bm, &bn);
  long M = (long)d->B * d->Ho * d->Wo;
  return (int)(((M + bm - 1) / bm) * 2);
}

void crnn_conv_wgrad_plan(int dtype, const crnn_conv_desc* d, int* bm, int* bn, int* splits) {
  if (use_halo(dtype, d, false)) {  // conv_halo.hip (the fwd instances): bm = bn = 0, slab per workgroup
    *bm = 0;
    *bn = 0;
    *splits = conv_halo_wgrad_slabs(d);
    return;
  }
  long Mp = (long)d->B * d->Ho * d->Wo;
  int Kp = d->KH * d->KW * d->Ci;
  if (dtype == CRNN_BF16 && d->Co % 256 == 0 && Kp % 128 == 0 && Mp >= 256L * 64) {
    // deep kernel: 1 block per CU, ~2 blocks per CU over the split-K grid, >= 8 K-tiles per split
    // tuning (crnn_set_option CRNN_OPT_WGRAD_TILE): 0 = 256x256 when Kp allows, 1 = 256x128
    // (twice the tiles, about half the split-K slabs), 2.. = target grid of 128 * value blocks
    const int opt = crnn_option(CRNN_OPT_WGRAD_TILE);
    *bm = 256;
    // Kp = 256 (the 1x1 downsample of 256 channels): 256 x 128 tiles, twice the tiles and half the split-K
    // slabs (30.9 -> 25.2 us, profiles/r05y/kbench_opt3)
    *bn = (Kp % 256 == 0 && Kp > 256 && opt != 1) ? 256 : 128;
    long tiles = (long)(d->Co / 256) * (Kp / *bn);
    const long target = opt >= 2 ? 128L * opt : CRNN_WGRAD_BLOCKS;
    long want = target / tiles;                 // whole rounds of 1-block-per-CU waves
    long maxs = (Mp + 512 - 1) / 512;
    if (maxs > 128) maxs = 128;                 // >= 128 slabs cost more to reduce than CUs gain
    if (want > maxs) want = maxs;
    if (want < 1) want = 1;
    if (want > 256) want = 256;
    *splits = eff_splits((int)Mp, (int)want);
    return;
  }
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

size_t crnn_conv_wgrad_workspace(int dtype, const crnn_conv_desc* d) {
  int bm, bn, s;
  crnn_conv_wgrad_plan(dtype, d, &bm, &bn, &s);
  return (size_t)s * d->Co * d->KH * d->KW * d->Ci * sizeof(float);
}

int crnn_conv_fwd(int dtype, const crnn_conv_desc* d, const void* x, const void* w, void* y,
                  float* psum, float* psq, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (d->Ci % 8 || d->Co % 8) return crnn_set_error(hipErrorInvalidValue, "conv_fwd: channels must be multiples of 8");
  if (use_halo(dtype, d, false)) return conv_halo_fwd(d, x, w, y, psum, psq, st);
  return dtype == CRNN_BF16 ? conv_fwd_t<bf16>(d, x, w, y, psum, psq, st)
                            : conv_fwd_t<float>(d, x, w, y, psum, psq, st);
}

int crnn_conv_fwd_bnrelu_supported(int dtype, const crnn_conv_desc* d) {
  return d->Ci % 8 == 0 && d->Co % 8 == 0 ? 1 : 0;
}

int crnn_conv_fwd_bnrelu(int dtype, const crnn_conv_desc* d, const void* x, const void* w, void* y,
                         const float* scale, const float* shift, void* stream) {
  if (!crnn_conv_fwd_bnrelu_supported(dtype, d))
    return crnn_set_error(hipErrorInvalidValue, "conv_fwd_bnrelu: channels must be multiples of 8");
  if (scale == nullptr || shift == nullptr) return crnn_set_error(hipErrorInvalidValue, "conv_fwd_bnrelu: null affine");
  hipStream_t st = (hipStream_t)stream;
  if (use_halo(dtype, d, false)) return conv_halo_fwd(d, x, w, y, nullptr, nullptr, st, scale, shift);
  return dtype == CRNN_BF16 ? conv_fwd_t<bf16>(d, x, w, y, nullptr, nullptr, st, scale, shift)
                            : conv_fwd_t<float>(d, x, w, y, nullptr, nullptr, st, scale, shift);
}

int crnn_conv_dgrad(int dtype, const crnn_conv_desc* d, const void* dy, const void* w, void* dx,
                    const void* dres, const void* yres, int accumulate, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (d->Ci % 8 || d->Co % 8) return crnn_set_error(hipErrorInvalidValue, "conv_dgrad: channels must be multiples of 8");
  if (dres == nullptr && !accumulate && use_halo(dtype, d, true)) return conv_halo_dgrad(d, dy, w, dx, st);
  return dtype == CRNN_BF16 ? conv_dgrad_t<bf16>(d, dy, w, dx, dres, yres, accumulate, st)
                            : conv_dgrad_t<float>(d, dy, w, dx, dres, yres, accumulate, st);
}

int crnn_conv_fwd_bnrelu_pool_supported(int dtype, const crnn_conv_desc* d) {
  return dtype == CRNN_BF16 && use_halo(dtype, d, false) && conv_halo_pool_fits(d) ? 1 : 0;
}

int crnn_conv_fwd_bnrelu_pool(int dtype, const crnn_conv_desc* d, const void* x, const void* w, void* y,
                              const float* scale, const float* shift, void* stream) {
  if (!crnn_conv_fwd_bnrelu_pool_supported(dtype, d))
    return crnn_set_error(hipErrorInvalidValue, "conv_fwd_bnrelu_pool: not the halo stem geometry");
  if (scale == nullptr || shift == nullptr) return crnn_set_error(hipErrorInvalidValue, "conv_fwd_bnrelu_pool: null affine");
  return conv_halo_fwd_pool(d, x, w, y, scale, shift, (hipStream_t)stream);
}

int crnn_conv_dgrad_ds_supported(int dtype, const crnn_conv_desc* d, const crnn_conv_desc* dds) {
  const int ks = dtype == CRNN_BF16 ? kstage<bf16>() : kstage<float>();
  // the concatenated gradient (dz1 | dzd) and weights (conv1 | downsample) are each addressed by one
  // 32-bit buffer-resource range (nbytes): guard on their BYTE sizes in this dtype
  const long es = dtype == CRNN_BF16 ? 2 : 4;
  const long dyn = (long)d->B * d->Ho * d->Wo * d->Co, wn = (long)d->Co * d->KH * d->KW * d->Ci + (long)d->Co * d->Ci;
  return d->KH == 3 && d->KW == 3 && d->sh == 2 && d->sw == 2 && d->ph == 1 && d->pw == 1 && dds->KH == 1 &&
                 dds->KW == 1 && dds->sh == 2 && dds->sw == 2 && dds->ph == 0 && dds->pw == 0 && d->B == dds->B &&
                 d->Hi == dds->Hi && d->Wi == dds->Wi && d->Ci == dds->Ci && d->Ho == dds->Ho && d->Wo == dds->Wo &&
                 d->Co == dds->Co && d->Ci % 8 == 0 && d->Co % ks == 0 && d->Hi == 2 * d->Ho && d->Wi == 2 * d->Wo &&
                 2 * dyn * es < (1L << 32) && wn * es < (1L << 32)
             ? 1
             : 0;
}

int crnn_conv_dgrad_ds(int dtype, const crnn_conv_desc* d, const crnn_conv_desc* dds, const void* dy, const void* w,
                       void* dx, void* stream) {
  if (!crnn_conv_dgrad_ds_supported(dtype, d, dds))
    return crnn_set_error(hipErrorInvalidValue, "conv_dgrad_ds: not a 3x3/2 conv + 1x1/2 downsample pair");
  Geo g = geo(d);
  hipStream_t st = (hipStream_t)stream;
  return dtype == CRNN_BF16 ? conv_dgrad_strided<bf16>(g, dy, w, dx, nullptr, nullptr, 0, st, false, true)
                            : conv_dgrad_strided<float>(g, dy, w, dx, nullptr, nullptr, 0, st, false, true);
}

int crnn_conv_dgrad_bnrelu_rows(int dtype, const crnn_conv_desc* d) {
  return dtype == CRNN_BF16 ? dgrad_bnrelu_rows(d) : 0;
}

int crnn_conv_dgrad_bnrelu(int dtype, const crnn_conv_desc* d, const void* dy, const void* w, void* dx, const void* z,
                           const float* mean, const float* invstd, const float* scale, const float* shift, float* pg,
                           float* pgx, void* stream) {
  if (dtype != CRNN_BF16 || dgrad_bnrelu_rows(d) == 0)
    return crnn_set_error(hipErrorInvalidValue, "conv_dgrad_bnrelu: geometry not on the 256-row path");
  return conv_dgrad_bnrelu(d, dy, w, dx, z, mean, invstd, scale, shift, pg, pgx, (hipStream_t)stream);
}

int crnn_conv_dgrad_tw_rows(int dtype, const crnn_conv_desc* d) {
  return dtype == CRNN_BF16 && dgrad_tw_ok(d) ? (int)(((long)d->B * d->Hi * d->Wi + 255) / 256 * 2) : 0;
}

int crnn_conv_dgrad_tw(int dtype, const crnn_conv_desc* d, const void* dy, const void* wt, void* dx, const void* dres,
                       const void* yres, int accumulate, void* stream) {
  if (!crnn_conv_dgrad_tw_rows(dtype, d))
    return crnn_set_error(hipErrorInvalidValue, "conv_dgrad_tw: not a bf16 stride-1 geometry on the 256-row path");
  const int M = d->B * d->Hi * d->Wi, N = d->Ci;
  DgradEpi<bf16> ep{(bf16*)dx, (const bf16*)dres, (const bf16*)yres, M, N, accumulate};
  if (crnn_option(CRNN_OPT_DIAG) & 1) ep.M = 0;   // diagnostic: no output stores
  return conv_dgrad_tw_launch(d, dy, wt, ep, (hipStream_t)stream);
}

int crnn_conv_dgrad_bnrelu_tw(int dtype, const crnn_conv_desc* d, const void* dy, const void* wt, void* dx,
                              const void* z, const float* mean, const float* invstd, const float* scale,
                              const float* shift, float* pg, float* pgx, void* stream) {
  if (!crnn_conv_dgrad_tw_rows(dtype, d))
    return crnn_set_error(hipErrorInvalidValue, "conv_dgrad_bnrelu_tw: not a bf16 stride-1 geometry on the 256-row path");
  const int M = d->B * d->Hi * d->Wi, N = d->Ci;
  DgradBnEpi<bf16> ep{(bf16*)dx, M, N, (const bf16*)z, mean, invstd, scale, shift, pg, pgx};
  return conv_dgrad_tw_launch(d, dy, wt, ep, (hipStream_t)stream);
}

#if CRNN_GEMM_STAMPS
// diagnostic build only (not in crnn_hip.h): the 256-row GEMM stamps of this TU's kernels
int crnn_diag_gemm_stamps(unsigned long long* host, int nblocks) {
  const size_t n = (size_t)(nblocks < GEMM_STAMP_BLOCKS ? nblocks : GEMM_STAMP_BLOCKS) * GEMM_STAMP_SLOTS;
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_gemm_stamps), n * sizeof(unsigned long long), 0,
                                  hipMemcpyDeviceToHost);
}
#endif

int crnn_conv_wgrad(int dtype, const crnn_conv_desc* d, const void* dy, const void* x, float* dw_oihw,
                    float* ws, size_t ws_bytes, float beta, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (d->Ci % 8 || d->Co % 8) return crnn_set_error(hipErrorInvalidValue, "conv_wgrad: channels must be multiples of 8");
  return dtype == CRNN_BF16 ? conv_wgrad_t<bf16>(d, dy, x, dw_oihw, ws, ws_bytes, beta, st)
                            : conv_wgrad_t<float>(d, dy, x, dw_oihw, ws, ws_bytes, beta, st);
}

int crnn_conv_wgrad_gemm(int dtype, const crnn_conv_desc* d, const void* dy, const void* x, float* ws,
                         size_t ws_bytes, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (d->Ci % 8 || d->Co % 8) return crnn_set_error(hipErrorInvalidValue, "conv_wgrad: channels must be multiples of 8");
  return dtype == CRNN_BF16 ? conv_wgrad_t<bf16>(d, dy, x, nullptr, ws, ws_bytes, 0.f, st, 1)
                            : conv_wgrad_t<float>(d, dy, x, nullptr, ws, ws_bytes, 0.f, st, 1);
}

int crnn_conv_wgrad_reduce(int dtype, const crnn_conv_desc* d, float* dw_oihw, const float* ws, size_t ws_bytes,
                           float beta, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (d->Ci % 8 || d->Co % 8) return crnn_set_error(hipErrorInvalidValue, "conv_wgrad: channels must be multiples of 8");
  return dtype == CRNN_BF16 ? conv_wgrad_t<bf16>(d, nullptr, nullptr, dw_oihw, (float*)ws, ws_bytes, beta, st, 2)
                            : conv_wgrad_t<float>(d, nullptr, nullptr, dw_oihw, (float*)ws, ws_bytes, beta, st, 2);
}

}  // extern "C"
