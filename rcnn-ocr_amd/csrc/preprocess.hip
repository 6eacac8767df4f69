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

__device__ __forceinline__ float area_w(const AreaTab& t, int s, int s1, int s2) {
  if (t.plo && s == t.lo) return t.wlo;
  if (t.phi && s == t.hi) return t.whi;
  return t.wmid;
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

template <typename T>
__global__ __launch_bounds__(256) void preprocess_kernel(const uint8_t* __restrict__ src,
                                                         const crnn_crop_desc* __restrict__ desc, int H, int W,
                                                         int kind, void* __restrict__ out) {
  const int x = blockIdx.x * blockDim.x + threadIdx.x, y = blockIdx.y, b = blockIdx.z;
  if (x >= W) return;
  const crnn_crop_desc d = desc[b];
  int v[3] = {255, 255, 255};
  const int dy = y - d.y0, dx = x - d.x0;
  if (dy >= 0 && dy < d.new_h && dx >= 0 && dx < d.new_w) {
    const uint8_t* s = src + d.offset;
    const int cs = d.c, rs = d.w * d.c;  // channel / row strides (GRAY: 1 channel replicated)
    const int nc = d.c == 1 ? 1 : 3;
    if (d.new_h == d.h && d.new_w == d.w) {
      for (int c = 0; c < nc; ++c) v[c] = s[(size_t)dy * rs + dx * cs + c];
    } else if (d.interp == 0) {
      int sx0, sx1, a0, a1, sy0, sy1, b0, b1;
      linear_tap(dx, d.w, (double)d.w / d.new_w, true, sx0, sx1, a0, a1);
      linear_tap(dy, d.h, (double)d.h / d.new_h, false, sy0, sy1, b0, b1);
      const uint8_t* r0 = s + (size_t)sy0 * rs;
      const uint8_t* r1 = s + (size_t)sy1 * rs;
      for (int c = 0; c < nc; ++c) {
        const long h0 = (long)r0[sx0 * cs + c] * a0 + (long)r0[sx1 * cs + c] * a1;
        const long h1 = (long)r1[sx0 * cs + c] * a0 + (long)r1[sx1 * cs + c] * a1;
        const long q = (b0 * h0 + b1 * h1 + (1l << (2 * COEF_BITS - 1))) >> (2 * COEF_BITS);
        v[c] = (int)min(255l, max(0l, q));
      }
    } else {
      const double scx = (double)d.w / d.new_w, scy = (double)d.h / d.new_h;
      const int ix = (int)rint(scx), iy = (int)rint(scy);
      if (fabs(scx - ix) < 2.220446049250313e-16 && fabs(scy - iy) < 2.220446049250313e-16) {  // resizeAreaFast
        int sum[3] = {0, 0, 0};
        for (int yy = dy * iy; yy < (dy + 1) * iy; ++yy)
          for (int xx = dx * ix; xx < (dx + 1) * ix; ++xx)
            for (int c = 0; c < nc; ++c) sum[c] += s[(size_t)yy * rs + xx * cs + c];
        const float inv = 1.f / (float)(ix * iy);
        for (int c = 0; c < nc; ++c) {
          const int q = (ix == 2 && iy == 2) ? (sum[c] + 2) >> 2 : cv_round(__fmul_rn((float)sum[c], inv));
          v[c] = min(255, max(0, q));
        }
      } else {
        const AreaTab tx = area_tab(dx, d.w, scx), ty = area_tab(dy, d.h, scy);
        float acc[3] = {0.f, 0.f, 0.f};
        for (int yy = ty.lo; yy <= ty.hi; ++yy) {
          const float beta = area_w(ty, yy, ty.lo, ty.hi);
          float buf[3] = {0.f, 0.f, 0.f};
          for (int xx = tx.lo; xx <= tx.hi; ++xx) {
            const float alpha = area_w(tx, xx, tx.lo, tx.hi);
            for (int c = 0; c < nc; ++c)
              buf[c] = __fadd_rn(buf[c], __fmul_rn((float)s[(size_t)yy * rs + xx * cs + c], alpha));
          }
          for (int c = 0; c < nc; ++c) {
            const float term = __fmul_rn(beta, buf[c]);
            acc[c] = yy == ty.lo ? term : __fadd_rn(acc[c], term);
          }
        }
        for (int c = 0; c < nc; ++c) v[c] = min(255, max(0, cv_round(acc[c])));
      }
    }
    if (nc == 1) v[1] = v[2] = v[0];  // COLOR_GRAY2RGB
  }
  store_px<T>(kind, out, b, y, x, H, W, v);
}

}  // namespace

extern "C" int crnn_preprocess(const unsigned char* src, const crnn_crop_desc* desc, int B, int H, int W, int out_kind,
                               int dtype, void* out, void* stream) {
  if (B <= 0 || H <= 0 || W <= 0 || B > 65535 || H > 65535)
    return crnn_set_error(hipErrorInvalidValue, "preprocess: bad batch / canvas size");
  if (out_kind < 0 || out_kind > 2) return crnn_set_error(hipErrorInvalidValue, "preprocess: out_kind 0, 1 or 2");
  const dim3 grid((W + 255) / 256, H, B);
  if (out_kind == 1 && dtype == CRNN_BF16)
    hipLaunchKernelGGL(preprocess_kernel<bf16>, grid, dim3(256), 0, (hipStream_t)stream, src, desc, H, W, out_kind,
                       out);
  else
    hipLaunchKernelGGL(preprocess_kernel<float>, grid, dim3(256), 0, (hipStream_t)stream, src, desc, H, W, out_kind,
                       out);
  return (int)hipGetLastError();
}
