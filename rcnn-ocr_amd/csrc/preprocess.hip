// GPU input pipeline: the reference's ResizeAndPadA + A.Normalize(0.5, 0.5)
// + ToTensorV2 (data/transforms.py:62-120, :185-193) for a ragged batch of uint8 crops, written
// straight into the encoder's input layout.
//
// One thread per output pixel (all 3 channels). Per crop, the host computes the reference's
// geometry (scale, new size, alignment offsets, interpolation choice :78-118, in Python so its
// rounding is the reference's) into a crnn_crop_desc; the kernel evaluates
//   INTER_LINEAR (upscale): OpenCV 4.x generic fixed-point path — 11-bit coefficients from the
//     float source coordinate, integer horizontal taps, (b0 r0 + b1 r1 + 2^21) >> 22 vertically;
//     columns clamp the tap (fx = 0 at the borders), rows keep the coefficients and clamp the
//     row index;
//   INTER_AREA (downscale): integer factors -> the cell sum ((s + 2) >> 2 for 2x2, else
//     cvRound(s * (1/area))); other factors -> the computeResizeAreaTab weights, accumulated in
//     float in OpenCV's order (row partial sums over ascending x, then beta-weighted rows over
//     ascending y), no FMA contraction, cvRound;
//   equal sizes: a copy; outside the resized box: white (255);
// then (v - 127.5) * (1 / 127.5) in fp32 (albumentations' Normalize). The CPU restatement it is
// held bit-exact to is oracle/preprocess_oracle.py (parity vs cv2 itself unpinned: not installed).
// HBM-bound: each source byte is read about once (neighbouring threads share taps through L1/L2),
// each output element written once.
#include "common.hpp"
#include "crnn_internal.hpp"

// OpenCV's float accumulation is rounded after every multiply and add: no FMA contraction here
// (__fmul_rn / __fadd_rn alone do not stop hipcc from fusing them; the Makefile also builds this
// file with -ffp-contract=off, since the default -ffp-contract=fast ignores the pragma)
#pragma clang fp contract(off)

namespace {

constexpr int COEF_BITS = 11;
constexpr float COEF_SCALE = 2048.f;

__device__ __forceinline__ int cv_round(float x) { return (int)rintf(x); }  // ties to even

// linear taps for destination index d: sources (s0, s1), coefficients (c0, c1)
__device__ __forceinline__ void linear_tap(int d, int ssize, double scale, bool clamp_coef, int& s0, int& s1,
                                           int& c0, int& c1) {
  float f = (float)((d + 0.5) * scale - 0.5);
  int s = (int)floorf(f);
  f = __fsub_rn(f, (float)s);
  if (clamp_coef) {
    if (s < 0) {
      f = 0.f;
      s = 0;
    }
    if (s >= ssize - 1) {
      f = 0.f;
      s = ssize - 1;
    }
  }
  c0 = cv_round(__fmul_rn(__fsub_rn(1.f, f), COEF_SCALE));
  c1 = cv_round(__fmul_rn(f, COEF_SCALE));
  s0 = min(max(s, 0), ssize - 1);
  s1 = min(max(s + 1, 0), ssize - 1);
}

// computeResizeAreaTab for one destination index: first / last source index, edge weights
struct AreaTab {
  int lo, hi;          // source range [lo, hi]
  float wlo, wmid, whi;  // weight of lo (if partial), of the interior, of hi (if partial)
  bool plo, phi;       // lo / hi are partial entries
};

__device__ __forceinline__ AreaTab area_tab(int d, int ssize, double scale) {
  const double fs1 = d * scale, fs2 = fs1 + scale;
  const double cell = fmin(scale, ssize - fs1);
  int s2 = (int)floor(fs2);
  s2 = min(s2, ssize - 1);
  const int s1 = min((int)ceil(fs1), s2);
  AreaTab t;
  t.plo = s1 - fs1 > 1e-3;
  t.phi = fs2 - s2 > 1e-3;
  t.lo = t.plo ? s1 - 1 : s1;
  t.hi = t.phi ? s2 : s2 - 1;
  t.wlo = (float)((s1 - fs1) / cell);
  t.wmid = (float)(1.0 / cell);
  t.whi = (float)(fmin(fmin(fs2 - s2, 1.0), cell) / cell);
  return t;
}

template <typename T>
__device__ __forceinline__ void store_px(int kind, void* out, int b, int y, int x, int H, int W, const int v[3]) {
  const float den = 1.f / 127.5f;
  if (kind == 2) {  // u8 canvas [B][H][W][3]
    uint8_t* o = (uint8_t*)out + (((size_t)b * H + y) * W + x) * 3;
    o[0] = (uint8_t)v[0];
    o[1] = (uint8_t)v[1];
    o[2] = (uint8_t)v[2];
    return;
  }
  float n[3];
#pragma unroll
  for (int c = 0; c < 3; ++c) n[c] = __fmul_rn(__fsub_rn((float)v[c], 127.5f), den);
  if (kind == 0) {  // fp32 NCHW [B][3][H][W] (ToTensorV2 of the reference)
    float* o = (float*)out;
#pragma unroll
    for (int c = 0; c < 3; ++c) o[(((size_t)b * 3 + c) * H + y) * W + x] = n[c];
  } else {  // encoder input [B][H][W][8] in T, channels 3..7 zero
    typename VT<T>::v8 pk;
#pragma unroll
    for (int c = 0; c < 8; ++c) pk[c] = fromf<T>(c < 3 ? n[c] : 0.f);
    *(typename VT<T>::v8*)((T*)out + (((size_t)b * H + y) * W + x) * 8) = pk;
  }
}

// per destination column / row of a crop: the resampling taps, computed once per launch
// (tab_kernel) instead of once per output pixel
struct Tap {
  int lo, hi;            // linear: s0, s1 ; area: source range [lo, hi]
  int c0, c1;            // linear: 11-bit coefficients ; area: plo, phi flags
  float wlo, wmid, whi;  // area weights
  int pad;
};

__global__ __launch_bounds__(256) void tab_kernel(const crnn_crop_desc* __restrict__ desc, int H, int W,
                                                  Tap* __restrict__ tabs) {
  const int b = blockIdx.y, i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= W + H) return;
  const crnn_crop_desc d = desc[b];
  const bool isx = i < W;
  const int k = isx ? i : i - W;
  const int dsize = isx ? d.new_w : d.new_h, ssize = isx ? d.w : d.h;
  if (k >= dsize) return;
  const double scale = (double)ssize / dsize;
  Tap t = {};
  if (d.interp == 0) {
    linear_tap(k, ssize, scale, isx, t.lo, t.hi, t.c0, t.c1);
  } else {
    const AreaTab a = area_tab(k, ssize, scale);
    t.lo = a.lo;
    t.hi = a.hi;
    t.c0 = a.plo;
    t.c1 = a.phi;
    t.wlo = a.wlo;
    t.wmid = a.wmid;
    t.whi = a.whi;
  }
  tabs[(size_t)b * (W + H) + i] = t;
}

__device__ __forceinline__ float tap_w(const Tap& t, int s) {
  if (t.c0 && s == t.lo) return t.wlo;
  if (t.c1 && s == t.hi) return t.whi;
  return t.wmid;
}

template <typename T>
__global__ __launch_bounds__(256) void preprocess_kernel(const uint8_t* __restrict__ src,
                                                         const crnn_crop_desc* __restrict__ desc,
                                                         const Tap* __restrict__ tabs, int H, int W, int kind,
                                                         void* __restrict__ out) {
  const int x = blockIdx.x * blockDim.x + threadIdx.x, y = blockIdx.y, b = blockIdx.z;
  if (x >= W) return;
  const crnn_crop_desc d = desc[b];
  int v[3] = {255, 255, 255};
  const int dy = y - d.y0, dx = x - d.x0;
  if (dy >= 0 && dy < d.new_h && dx >= 0 && dx < d.new_w) {
    const uint8_t* s = src + d.offset;
    const int cs = d.c, rs = d.w * d.c;  // channel / row strides
    const int cm = d.c == 1 ? 0 : 1;     // GRAY: channel 0 read for all three (COLOR_GRAY2RGB)
    // every load below is unconditional (clamped indices) and issued before its uses: a load under
    // a runtime condition makes the compiler wait for it on the spot, serializing the taps
    auto px = [&](int yy, int xx, int c) -> int { return s[(size_t)yy * rs + xx * cs + c * cm]; };
    if (d.new_h == d.h && d.new_w == d.w) {
#pragma unroll
      for (int c = 0; c < 3; ++c) v[c] = px(dy, dx, c);
    } else if (d.interp == 0) {
      const Tap tx = tabs[(size_t)b * (W + H) + dx], ty = tabs[(size_t)b * (W + H) + W + dy];
      int p[2][2][3];
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        p[0][0][c] = px(ty.lo, tx.lo, c);
        p[0][1][c] = px(ty.lo, tx.hi, c);
        p[1][0][c] = px(ty.hi, tx.lo, c);
        p[1][1][c] = px(ty.hi, tx.hi, c);
      }
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        const long h0 = (long)p[0][0][c] * tx.c0 + (long)p[0][1][c] * tx.c1;
        const long h1 = (long)p[1][0][c] * tx.c0 + (long)p[1][1][c] * tx.c1;
        const long q = (ty.c0 * h0 + ty.c1 * h1 + (1l << (2 * COEF_BITS - 1))) >> (2 * COEF_BITS);
        v[c] = (int)min(255l, max(0l, q));
      }
    } else {
      const double scx = (double)d.w / d.new_w, scy = (double)d.h / d.new_h;
      const int ix = (int)rint(scx), iy = (int)rint(scy);
      if (fabs(scx - ix) < 2.220446049250313e-16 && fabs(scy - iy) < 2.220446049250313e-16) {  // resizeAreaFast
        int sum[3] = {0, 0, 0};
        const int x1 = (dx + 1) * ix - 1;
        for (int yy = dy * iy; yy < (dy + 1) * iy; ++yy)
          for (int xx = dx * ix; xx <= x1; xx += 4) {
            int q[4][3];
#pragma unroll
            for (int k = 0; k < 4; ++k)
#pragma unroll
              for (int c = 0; c < 3; ++c) q[k][c] = px(yy, min(xx + k, x1), c);
#pragma unroll
            for (int k = 0; k < 4; ++k)
#pragma unroll
              for (int c = 0; c < 3; ++c) sum[c] += xx + k <= x1 ? q[k][c] : 0;
          }
        const float inv = 1.f / (float)(ix * iy);
#pragma unroll
        for (int c = 0; c < 3; ++c) {
          const int q = (ix == 2 && iy == 2) ? (sum[c] + 2) >> 2 : cv_round(__fmul_rn((float)sum[c], inv));
          v[c] = min(255, max(0, q));
        }
      } else {
        const Tap tx = tabs[(size_t)b * (W + H) + dx], ty = tabs[(size_t)b * (W + H) + W + dy];
        float acc[3] = {0.f, 0.f, 0.f};
        for (int yy = ty.lo; yy <= ty.hi; ++yy) {
          const float beta = tap_w(ty, yy);
          float buf[3] = {0.f, 0.f, 0.f};
          for (int xx = tx.lo; xx <= tx.hi; xx += 4) {  // OpenCV's order: ascending x, one add at a time
            int q[4][3];
#pragma unroll
            for (int k = 0; k < 4; ++k)
#pragma unroll
              for (int c = 0; c < 3; ++c) q[k][c] = px(yy, min(xx + k, tx.hi), c);
#pragma unroll
            for (int k = 0; k < 4; ++k) {
              if (xx + k > tx.hi) break;
              const float alpha = tap_w(tx, xx + k);
#pragma unroll
              for (int c = 0; c < 3; ++c) buf[c] = __fadd_rn(buf[c], __fmul_rn((float)q[k][c], alpha));
            }
          }
#pragma unroll
          for (int c = 0; c < 3; ++c) {
            const float term = __fmul_rn(beta, buf[c]);
            acc[c] = yy == ty.lo ? term : __fadd_rn(acc[c], term);
          }
        }
#pragma unroll
        for (int c = 0; c < 3; ++c) v[c] = min(255, max(0, cv_round(acc[c])));
      }
    }
  }
  store_px<T>(kind, out, b, y, x, H, W, v);
}

}  // namespace

extern "C" long crnn_preprocess_workspace(int B, int H, int W) { return (long)B * (H + W) * (long)sizeof(Tap); }

extern "C" int crnn_preprocess(const unsigned char* src, const crnn_crop_desc* desc, int B, int H, int W, int out_kind,
                               int dtype, void* out, void* ws, long ws_bytes, void* stream) {
  if (B <= 0 || H <= 0 || W <= 0 || B > 65535 || H > 65535)
    return crnn_set_error(hipErrorInvalidValue, "preprocess: bad batch / canvas size");
  if (out_kind < 0 || out_kind > 2) return crnn_set_error(hipErrorInvalidValue, "preprocess: out_kind 0, 1 or 2");
  if (ws_bytes < crnn_preprocess_workspace(B, H, W))
    return crnn_set_error(hipErrorInvalidValue, "preprocess: workspace too small");
  hipStream_t st = (hipStream_t)stream;
  Tap* tabs = (Tap*)ws;
  hipLaunchKernelGGL(tab_kernel, dim3((W + H + 255) / 256, B), dim3(256), 0, st, desc, H, W, tabs);
  const dim3 grid((W + 255) / 256, H, B);
  if (out_kind == 1 && dtype == CRNN_BF16)
    hipLaunchKernelGGL(preprocess_kernel<bf16>, grid, dim3(256), 0, st, src, desc, tabs, H, W, out_kind, out);
  else
    hipLaunchKernelGGL(preprocess_kernel<float>, grid, dim3(256), 0, st, src, desc, tabs, H, W, out_kind, out);
  return (int)hipGetLastError();
}
