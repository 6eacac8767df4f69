// Halo-tiled direct 3x3 convolution (stride 1, pad 1, NHWC bf16) for the two full-resolution stem
// convs of SE-ResNet31 (reference: model/seresnet31.py:82-86, nn.Conv2d(3, 64, 3, 1, 1) and
// nn.Conv2d(64, 128, 3, 1, 1)) — their forward, and the second one's input gradient, which is the
// same convolution with flipped taps and transposed weights.
//
// Why a separate kernel: at 32x256 with Ci = 64 the implicit GEMM (conv.hip) has K = 576, so
// every 256 x 128 tile re-reads its 9x im2col rows and the whole 147 KB weight from L2 for only
// nine 64-deep K-steps — the launch runs at the L2 bandwidth, ~0.5 PFLOP/s. Here:
//   * one workgroup owns a BAND: one image, one 128-pixel half of the width, all H rows, and
//     walks it top to bottom (persistent over the band's H tiles);
//   * its weights live in VGPRs for the whole band (each wave holds the K x CO/4 slice it needs);
//   * the input rows y-1, y, y+1 (+ halo columns) sit in a 4-slot LDS ring; row y+2 is fetched
//     into registers while row y computes and written to the free slot afterwards, so each input
//     byte crosses HBM -> LDS once per band;
//   * A fragments come straight from the ring with ds_read_b128 (pixel pitch padded so the 16
//     pixels of each lane group land on distinct banks).
// Wave (pw, cw) of 8 (two per SIMD): 64 output pixels x CO/4 channels, MFMA 16x16x32 bf16, fp32
// accumulate; each wave's weight slice (CO/4 x 9*CI) is 144 VGPRs.
// The forward also emits BatchNorm partial statistics in conv.hip's (sum, M2) layout, one partial
// row per 64 output pixels (one wave's share of a tile), from the fp32 accumulators.
#include "gemm.hpp"
#include "crnn_internal.hpp"

using namespace gemm;

namespace {

constexpr int TW = 128;  // output pixels per tile: half of a 256-wide row

template <int CI> struct Ring {
  // bytes per halo pixel: (CI/8 + 2) 16-B slots, = 2 mod 4 slots, which keeps every ds_read_b128 lane
  // group of an A fragment (16 pixels, 2 channel chunks) on distinct banks (enumerated offline)
  // (CI = 8, the 3-channel input conv: one 16-B slot per pixel, taps packed along k instead)
  static constexpr int PITCH = CI >= 32 ? CI * 2 + 32 : CI * 2;
  static constexpr int SLOT = (TW + 2) * PITCH;  // one input row of the band + 2 halo columns
  static constexpr int CH = CI / 8;              // 16-B chunks per pixel
  static constexpr int NCHUNK = (TW + 2) * CH;
  static constexpr int PER_T = (NCHUNK + 511) / 512;
};

// FLIP = false: y = conv(x, W), W packed [CO][3][3][CI] (conv.hip's OHWI pack).
// FLIP = true : dx = conv(dy, W'), W'[o][t][c] = W[c][8 - t][o], read from the forward pack
//               [CI][3][3][CO] (CI = forward Co, CO = forward Ci).
// ROW16 (CRNN_OPT_HALO_ROW16, not with POOL): the output tile (128 pixels x CO, contiguous in NHWC) goes
// through LDS, so each lane stores whole 16-B chunks and a wave instruction covers full 128-B lines, instead of
// 8-B pieces of 16 pixels from the MFMA layout; staged in the ring slot the finished row frees when it is
// large enough, else in an array of its own. Used for the 3 (8) -> 64 input conv, whose rows are
// store-bound (130 -> 100 us at B = 256, profiles/r05u/); the 64 -> 128 forward spills with it (+2.5 %) and
// the input gradient does not move, so those keep the direct stores.
template <int CI, int CO, bool FLIP, bool POOL = false, bool ROW16 = false>
__global__ __launch_bounds__(512) void halo3x3_kernel(const bf16* __restrict__ x, const bf16* __restrict__ wp,
                                                      bf16* __restrict__ y, float* __restrict__ psum,
                                                      float* __restrict__ psq, int H, int W, int RB, uint32_t xbytes,
                                                      const float* __restrict__ esc = nullptr,
                                                      const float* __restrict__ esh = nullptr) {
  using R = Ring<CI>;
  // CI = 8 (TAPK): a 32-deep k-step holds 4 taps x 8 channels, lane group g takes tap 4ks + g
  // (taps 9..11 of the last step: zero weights, any finite data)
  constexpr bool TAPK = CI == 8;
  constexpr int KC = TAPK ? 1 : CI / 32;  // 32-deep k-steps per tap
  constexpr int KS = TAPK ? 3 : 9 * KC;   // k-steps
  constexpr int CW = CO / 4;        // output channels per wave
  constexpr int NJ = CW / 16;       // channel fragments per wave
  constexpr int MI = 4;             // 64 pixels per wave
  static_assert((CI % 32 == 0 || TAPK) && CO % 32 == 0 && !(TAPK && FLIP), "channels");
  __shared__ __attribute__((aligned(16))) char ring[4 * R::SLOT];

  const int lane = threadIdx.x & 63, c = lane & 15, g = lane >> 4;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int pw = wv & 1, cw = wv >> 1;
  // band = (image b, 128-column half xh, chunk of RB rows starting at r0)
  const int nxh = W / TW, nrc = H / RB;
  const int band = blockIdx.x;
  const int b = band / (nxh * nrc), xh = (band / nrc) % nxh, r0 = (band % nrc) * RB;
  const int x0 = xh * TW;

  // weights: slot ks of fragment j = output channel cw*CW + 16j + c, k = 32ks + 8g .. +7
  bf16x8 wf[NJ][KS];
  if constexpr (!FLIP) {
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int ks = 0; ks < KS; ++ks)
        if constexpr (TAPK) {
          const bf16x8 v = *reinterpret_cast<const bf16x8*>(wp + (size_t)(cw * CW + 16 * j + c) * 72 + 8 * min(4 * ks + g, 8));
          wf[j][ks] = 4 * ks + g < 9 ? v : bf16x8{};
        } else {
          wf[j][ks] = *reinterpret_cast<const bf16x8*>(wp + (size_t)(cw * CW + 16 * j + c) * 9 * CI + 32 * ks + 8 * g);
        }
  } else {
    // W' is a gather of the forward pack: build it in the (still unused) ring one half of the
    // output channels at a time, [CO/2][9*CI] rows
    static_assert((size_t)2 * CW * 9 * CI * 2 <= 4 * R::SLOT, "W' half fits the ring");
    bf16* wl = reinterpret_cast<bf16*>(ring);
#pragma unroll 1
    for (int hh = 0; hh < 2; ++hh) {
      // a thread moves 8 consecutive o of one kk = t * CI + cc: one 16-B global read, 8 LDS
      // writes whose lanes differ in kk (consecutive addresses, no bank conflicts)
      for (int e = threadIdx.x; e < 2 * CW / 8 * 9 * CI; e += 512) {
        const int kk = e % (9 * CI), o8 = e / (9 * CI), t = kk / CI, cc = kk % CI;
        const bf16x8 v = *reinterpret_cast<const bf16x8*>(wp + ((size_t)cc * 9 + (8 - t)) * CO + hh * 2 * CW + 8 * o8);
#pragma unroll
        for (int q = 0; q < 8; ++q) wl[(8 * o8 + q) * 9 * CI + kk] = v[q];
      }
      __syncthreads();
      if ((cw >> 1) == hh) {
#pragma unroll
        for (int j = 0; j < NJ; ++j)
#pragma unroll
          for (int ks = 0; ks < KS; ++ks)
            wf[j][ks] = *reinterpret_cast<const bf16x8*>(wl + ((cw & 1) * CW + 16 * j + c) * 9 * CI + 32 * ks + 8 * g);
      }
      __syncthreads();
    }
  }

  const __amdgpu_buffer_rsrc_t rx = mk_rsrc(x, xbytes);
  u32x4 pre[R::PER_T];
  // input row r of image b, columns x0-1 .. x0+TW, into registers (zeros outside the image:
  // out-of-range buffer offsets read 0, so the loads carry no branches)
  auto load_row = [&](int r) {
#pragma unroll
    for (int i = 0; i < R::PER_T; ++i) {
      const int q = threadIdx.x + 512 * i;
      const int px = q / R::CH, ch = q % R::CH;
      const int xc = x0 - 1 + px;
      const bool ok = q < R::NCHUNK && r >= 0 && r < H && xc >= 0 && xc < W;
      const uint32_t off = ok ? ((((uint32_t)b * H + r) * W + xc) * CI + ch * 8) * 2u : OOB;
      pre[i] = __builtin_amdgcn_raw_buffer_load_b128(rx, off, 0, 0);
    }
  };
  auto store_row = [&](int r) {
    char* s = ring + ((r + 1) & 3) * R::SLOT;
#pragma unroll
    for (int i = 0; i < R::PER_T; ++i) {
      const int q = threadIdx.x + 512 * i;
      const int px = q / R::CH, ch = q % R::CH;
      if (q < R::NCHUNK) *reinterpret_cast<u32x4*>(s + px * R::PITCH + ch * 16) = pre[i];
    }
  };
  load_row(r0 - 1);
  store_row(r0 - 1);
  load_row(r0);
  store_row(r0);
  load_row(r0 + 1);
  store_row(r0 + 1);
  __syncthreads();

  const uint32_t abase = (uint32_t)((pw * 64 + c) * R::PITCH + (TAPK ? 0 : 16 * g));
  // POOL: the even row's activations (bf16: rounding is monotonic, so max and rounding commute) in
  // this lane's slice of LDS, max-combined with the odd row's (same lane: no barrier)
  __shared__ __attribute__((aligned(16))) bf16 keep[POOL ? 512 * MI * NJ * 4 : 4];
  static_assert(!(ROW16 && POOL) && (!ROW16 || CO % 64 == 0), "row stores: CO multiple of 64, no pool");
  constexpr int STG = TW * CO * 2;                 // the staged output tile, bytes
  constexpr bool STG_IN_RING = STG <= R::SLOT;
  __shared__ __attribute__((aligned(16))) char stg_own[ROW16 && !STG_IN_RING ? STG : 16];
  for (int yy = r0; yy < r0 + RB; ++yy) {
    load_row(yy + 2);  // lands while this row computes; stored to the free slot below
    f32x4 acc[MI][NJ];
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    const char* rowp[3];  // input rows yy - 1 .. yy + 1 (TAPK: this lane's tap of k-step kh)
#pragma unroll
    for (int kh = 0; kh < 3; ++kh) {
      if constexpr (TAPK) {
        const int t = min(4 * kh + g, 8), th = t / 3;
        rowp[kh] = ring + ((yy + th) & 3) * R::SLOT + abase + (t - 3 * th) * R::PITCH;
      } else {
        rowp[kh] = ring + ((yy + kh) & 3) * R::SLOT + abase;
      }
    }
    // k-step ks = (kh, kw, kc): A fragments of step ks+1 are read while step ks multiplies
    // (software double buffer; the scheduling barrier keeps the compiler from sinking the reads
    // next to their MFMAs)
    bf16x8 af[2][MI];
    auto read_a = [&](int ks, bf16x8 (&a)[MI]) {
      const int kh = TAPK ? ks : ks / (3 * KC), kw = TAPK ? 0 : (ks / KC) % 3, kc = ks % KC;
#pragma unroll
      for (int i = 0; i < MI; ++i)
        a[i] = *reinterpret_cast<const bf16x8*>(rowp[kh] + (16 * i + kw) * R::PITCH + kc * 64);
    };
    read_a(0, af[0]);
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      if (ks + 1 < KS) read_a(ks + 1, af[(ks + 1) & 1]);
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j) mma<bf16>(acc[i][j], wf[j][ks], af[ks & 1][i]);
      if (ks + 1 < KS) __builtin_amdgcn_sched_group_barrier(0x100, MI, 0);  // the DS reads first,
      __builtin_amdgcn_sched_group_barrier(0x008, MI * NJ, 0);             // then the MFMAs
      __builtin_amdgcn_sched_barrier(0);
    }
    store_row(yy + 2);

    // outputs: lane (c, g) of fragment (i, j) = pixel pw*64 + 16i + c, channels co .. co+3
    const size_t m0 = ((size_t)b * H + yy) * W + x0;
    if (esc != nullptr) {  // eval-mode BN (running statistics) + ReLU on the accumulators
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int co = cw * CW + 16 * j + 4 * g;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float a = esc[co + r], h = esh[co + r];
#pragma unroll
          for (int i = 0; i < MI; ++i) acc[i][j][r] = fmaxf(fmaf(acc[i][j][r], a, h), 0.f);
        }
      }
    }
    if constexpr (POOL) {
      // eval inference (stem, model/seresnet31.py:81-89): BN -> ReLU -> 2x2 max-pool in the epilogue;
      // rows yy, yy+1 of a window are consecutive rows of this band (r0, RB even), pixels 2p, 2p+1
      // are lanes c, c^1 of one fragment row: y is the pooled [B][H/2][W/2][CO] map
      bf16* kp = keep + (size_t)threadIdx.x * (MI * NJ * 4);
      if ((yy & 1) == 0) {
#pragma unroll
        for (int i = 0; i < MI; ++i)
#pragma unroll
          for (int j = 0; j < NJ; ++j) st4<bf16>(kp + (i * NJ + j) * 4, acc[i][j]);
      } else {
        const size_t p0 = ((size_t)b * (H / 2) + (yy >> 1)) * (W / 2) + (x0 >> 1);
#pragma unroll
        for (int i = 0; i < MI; ++i)
#pragma unroll
          for (int j = 0; j < NJ; ++j) {
            f32x4 v;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const float a = fmaxf(acc[i][j][r], (float)kp[(i * NJ + j) * 4 + r]);
              v[r] = fmaxf(a, __shfl_xor(a, 1));
            }
            if ((c & 1) == 0)
              st4<bf16>(y + (p0 + ((pw * 64 + 16 * i + c) >> 1)) * CO + cw * CW + 16 * j + 4 * g, v);
          }
      }
    } else if constexpr (ROW16) {
      // [128 pixels][CO] bf16, 16-B chunk q of pixel p at chunk q ^ (p & 7)
      char* sg = STG_IN_RING ? ring + (yy & 3) * R::SLOT : stg_own;   // ring: the slot of row yy - 1
      if constexpr (STG_IN_RING) __syncthreads();   // every wave is done reading row yy - 1
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
          const int px = pw * 64 + 16 * i + c, ch = cw * CW + 16 * j + 4 * g;
          const bf16x4 v = {(bf16)acc[i][j][0], (bf16)acc[i][j][1], (bf16)acc[i][j][2], (bf16)acc[i][j][3]};
          *reinterpret_cast<bf16x4*>(sg + px * (CO * 2) + (((ch >> 3) ^ (px & 7)) << 4) + ((ch >> 2) & 1) * 8) = v;
        }
      __syncthreads();
      constexpr int QN = CO / 8;   // 16-B chunks per pixel
#pragma unroll
      for (int k = 0; k < TW * QN / 512; ++k) {
        const int e = threadIdx.x + 512 * k, px = e / QN, q = e % QN;
        const u32x4 v = *reinterpret_cast<const u32x4*>(sg + px * (CO * 2) + ((q ^ (px & 7)) << 4));
        *reinterpret_cast<u32x4*>(y + (m0 + px) * CO + 8 * q) = v;
      }
    } else {
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j)
          st4<bf16>(y + (m0 + pw * 64 + 16 * i + c) * CO + cw * CW + 16 * j + 4 * g, acc[i][j]);
    }

    if (psum != nullptr) {
      // BN partial statistics: (sum, M2 about the partial mean) of this wave's 64 pixels, one
      // partial row per 64 pixels (crnn_conv_stat_rows_per_partial), straight from the accumulators
      const size_t prow = (m0 + pw * 64) / 64;
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        f32x4 s = {0.f, 0.f, 0.f, 0.f}, q = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int i = 0; i < MI; ++i) s += acc[i][j];
#pragma unroll
        for (int r = 0; r < 4; ++r) s[r] = rowgroup_sum<16>(s[r]);
#pragma unroll
        for (int i = 0; i < MI; ++i)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float dv = acc[i][j][r] - s[r] * (1.f / 64.f);
            q[r] += dv * dv;
          }
#pragma unroll
        for (int r = 0; r < 4; ++r) q[r] = rowgroup_sum<16>(q[r]);
        if (c == 0) {
          const int co = cw * CW + 16 * j + 4 * g;
          *reinterpret_cast<f32x4*>(psum + prow * CO + co) = s;
          *reinterpret_cast<f32x4*>(psq + prow * CO + co) = q;
        }
      }
    }
    __syncthreads();
  }
}


// ------------------------------------------------------------------------------------------------
// Weight gradient of the same convolution, dW[co][t][ci] = sum_p dy[p][co] x[p + t][ci]: a GEMM
// with K = pixels, M = CO, N = 9*CI. A workgroup walks whole bands (as the forward does: x rows in
// a 4-slot ring, the band's dy row as a 128 x CO tile, both double-buffered through registers)
// and keeps its CO x 9*CI partial in accumulators across all of them; one fp32 slab per
// workgroup, summed by conv.hip's wgrad_reduce_kernel. Both operands stay pixel-major in LDS (NHWC
// rows as loaded) and are read with ds_read_b64_tr_b16. The k -> pixel map of a 32-deep k-step
// puts the two 16-lane groups of each 32-lane half on 8 CONSECUTIVE pixel rows
// (pixel = 16(g>>1) + 8h + 4(g&1) + q for lane group g, read h, block row q), and row pitches of
// 20 and 36 8-byte chunks (mod 32) spread any 8 consecutive rows over distinct banks — for every
// tap shift kw, so addresses are a per-lane base plus immediates (enumerated offline).
// Wave (mw, nw) of 8: CO/2 output channels x 9*CI/4 k' columns (144 accumulator VGPRs).
template <int CI, int CO>
__global__ __launch_bounds__(512) void halo3x3_wgrad_kernel(const bf16* __restrict__ dy, const bf16* __restrict__ x,
                                                            float* __restrict__ ws, int B, int H, int W,
                                                            uint32_t dybytes, uint32_t xbytes) {
  // TAPK (CI = 8, the input conv): a 16-column k' fragment spans two taps; each lane's tap comes
  // from its column quad, the 72 k' columns are padded to 5 fragments (extra columns not written)
  constexpr bool TAPK = CI == 8;
  constexpr int XROW = TAPK ? 32 : CI * 2 + 32, DROW = CO * 2 + 32;  // padded pixel rows (bytes)
  static_assert((XROW / 8) % 8 == 4 && (DROW / 8) % 8 == 4, "pitches of the conflict-free map");
  constexpr int XSLOT = (TW + 2) * XROW, DTILE = TW * DROW;
  constexpr int KP = 9 * CI;                      // k' = (tap, ci)
  constexpr int WVM = TAPK ? 4 : 2, WVN = 8 / WVM;  // waves along M (co) and N (k')
  constexpr int MW = CO / WVM;                    // per-wave co
  constexpr int NFT = (KP + 15) / 16;             // k' fragments in all
  constexpr int NF = (NFT + WVN - 1) / WVN, NW = 16 * NF;  // per wave
  constexpr int MF = MW / 16;
  constexpr int XCH = CI / 8, DCH = CO / 8;       // 16-B chunks per pixel
  constexpr int NT = 512;
  constexpr int XPER = ((TW + 2) * XCH + NT - 1) / NT, DPER = (TW * DCH + NT - 1) / NT;
  static_assert(MW % 16 == 0 && (CI % 16 == 0 || TAPK), "shape");
  __shared__ __attribute__((aligned(16))) char ring[4 * XSLOT];
  __shared__ __attribute__((aligned(16))) char dyt[2][DTILE];

  const int lane = threadIdx.x & 63, c = lane & 15, g = lane >> 4;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int mw = wv % WVM, nw = wv / WVM;
  const int nxh = W / TW, nbands = B * nxh;
  const __amdgpu_buffer_rsrc_t rx = mk_rsrc(x, xbytes), rd = mk_rsrc(dy, dybytes);
  // transposed-read lane roles: block row q, column quad p4; pixel of (h = 0, q) within a k-step
  const int q = c >> 2, p4 = c & 3;
  const int prow = 16 * (g >> 1) + 4 * (g & 1) + q;
  const uint32_t dbase = (uint32_t)(prow * DROW + (mw * MW + 4 * p4) * 2);
  const uint32_t xbase = (uint32_t)(prow * XROW + 4 * p4 * 2);

  f32x4 acc[MF][NF];
#pragma unroll
  for (int i = 0; i < MF; ++i)
#pragma unroll
    for (int j = 0; j < NF; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  u32x4 xpre[XPER], dpre[DPER];
  int b = 0, x0 = 0;
  auto load_x = [&](int r) {
#pragma unroll
    for (int i = 0; i < XPER; ++i) {
      const int e = threadIdx.x + NT * i, px = e / XCH, ch = e % XCH;
      const int xc = x0 - 1 + px;
      const bool ok = e < (TW + 2) * XCH && r >= 0 && r < H && xc >= 0 && xc < W;
      xpre[i] = __builtin_amdgcn_raw_buffer_load_b128(rx, ok ? ((((uint32_t)b * H + r) * W + xc) * CI + ch * 8) * 2u : OOB, 0, 0);
    }
  };
  auto store_x = [&](int r) {
    char* s = ring + ((r + 1) & 3) * XSLOT;
#pragma unroll
    for (int i = 0; i < XPER; ++i) {
      const int e = threadIdx.x + NT * i, px = e / XCH, ch = e % XCH;
      if (e < (TW + 2) * XCH) *reinterpret_cast<u32x4*>(s + px * XROW + ch * 16) = xpre[i];
    }
  };
  auto load_d = [&](int r) {
#pragma unroll
    for (int i = 0; i < DPER; ++i) {
      const int e = threadIdx.x + NT * i, px = e / DCH, ch = e % DCH;
      const bool ok = e < TW * DCH && r < H;
      dpre[i] = __builtin_amdgcn_raw_buffer_load_b128(rd, ok ? ((((uint32_t)b * H + r) * W + x0 + px) * CO + ch * 8) * 2u : OOB, 0, 0);
    }
  };
  auto store_d = [&](int r) {
    char* s = dyt[r & 1];
#pragma unroll
    for (int i = 0; i < DPER; ++i) {
      const int e = threadIdx.x + NT * i, px = e / DCH, ch = e % DCH;
      if (e < TW * DCH) *reinterpret_cast<u32x4*>(s + px * DROW + ch * 16) = dpre[i];
    }
  };
  typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

  for (int band = blockIdx.x; band < nbands; band += gridDim.x) {
    b = band / nxh;
    x0 = (band - b * nxh) * TW;
    load_x(-1);
    store_x(-1);
    load_x(0);
    store_x(0);
    load_x(1);
    store_x(1);
    load_d(0);
    store_d(0);
    __syncthreads();
    for (int yy = 0; yy < H; ++yy) {
      load_x(yy + 2);
      load_d(yy + 1);
      const char* dt = dyt[yy & 1] + dbase;
      const char* sl[3];
#pragma unroll
      for (int kh = 0; kh < 3; ++kh) sl[kh] = ring + ((yy + kh) & 3) * XSLOT + xbase;
#pragma unroll
      for (int ks = 0; ks < TW / 32; ++ks) {
        bf16x8 xa[MF];
#pragma unroll
        for (int i = 0; i < MF; ++i) {
          const char* pa = dt + ks * 32 * DROW + i * 32;
          s16x4 t2[2] = {__builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(pa)),
                         __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(pa + 8 * DROW))};
          xa[i] = *reinterpret_cast<const bf16x8*>(t2);
        }
#pragma unroll
        for (int j = 0; j < NF; ++j) {
          const int f = nw * NF + j;
          if (f >= NFT) break;  // wave-uniform
          const char* pb;
          if constexpr (TAPK) {
            // columns 16f + 4p4 .. +3: tap 2f + p4/2 (clamped: its columns are not written), ci 4(p4&1)
            const int t = min(2 * f + (p4 >> 1), 8), kh = t / 3, kw = t - 3 * kh;
            pb = ring + ((yy + kh) & 3) * XSLOT + prow * XROW + (ks * 32 + kw) * XROW + 8 * (p4 & 1);
          } else {
            const int t = f / (CI / 16), ci0 = (f % (CI / 16)) * 16;
            const int kh = t / 3, kw = t % 3;
            pb = sl[kh] + (ks * 32 + kw) * XROW + ci0 * 2;
          }
          s16x4 t2[2] = {__builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(pb)),
                         __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(pb + 8 * XROW))};
          const bf16x8 yb = *reinterpret_cast<const bf16x8*>(t2);
#pragma unroll
          for (int i = 0; i < MF; ++i) mma<bf16>(acc[i][j], xa[i], yb);
        }
      }
      store_x(yy + 2);
      store_d(yy + 1);
      __syncthreads();
    }
  }
  // slab [blockIdx.x][CO][KP]: lane (c, g) of fragment (i, j) holds rows co = 4g + r, column k' = c
  float* slab = ws + (size_t)blockIdx.x * CO * KP;
#pragma unroll
  for (int i = 0; i < MF; ++i)
#pragma unroll
    for (int j = 0; j < NF; ++j) {
      const int n = nw * NW + 16 * j + c;
      if (n < KP)
#pragma unroll
        for (int r = 0; r < 4; ++r) slab[(size_t)(mw * MW + 16 * i + 4 * g + r) * KP + n] = acc[i][j][r];
    }
}

}  // namespace

// conv.hip dispatch: the halo kernel covers 3x3 / stride 1 / pad 1 convolutions whose width is a
// multiple of 128 and whose (Ci, Co) has an instance — the stem's (8 = 3 padded, 64) and (64, 128);
// dgrad = the same kernel on the flipped weights (64, 128 only: the input conv needs no dx)
bool conv_halo_fits(const crnn_conv_desc* d, bool dgrad) {
  if (!(d->KH == 3 && d->KW == 3 && d->sh == 1 && d->sw == 1 && d->ph == 1 && d->pw == 1)) return false;
  if (d->Ho != d->Hi || d->Wo != d->Wi || d->Wi % TW || d->Hi < 1) return false;
  if (dgrad) return d->Ci == 64 && d->Co == 128;
  return (d->Ci == 64 && d->Co == 128) || (d->Ci == 8 && d->Co == 64);
}

// rows per band: the memory-bound input conv (few FLOPs per row, several workgroups per CU) takes
// short bands so more of them are in flight; the MFMA-bound ones walk the whole height
// (tuning: CRNN_OPT_HALO_CONV = n >= 2 sets n rows for every halo forward, when it divides H)
static int band_rows(int H, int ci) {
  const int opt = crnn_option(CRNN_OPT_HALO_CONV);
  if (opt >= 2 && H % opt == 0) return opt;
  if (ci == 8)
    for (int rb : {8, 4, 2})
      if (H % rb == 0 && H > rb) return rb;
  if (ci == 64 && H % 16 == 0 && H > 16) return 16;  // 4 bands per CU: measured 7 % faster than H
  return H;
}

int conv_halo_fwd(const crnn_conv_desc* d, const void* x, const void* w, void* y, float* psum, float* psq,
                  hipStream_t st, const float* esc, const float* esh) {
  const int rb = band_rows(d->Hi, d->Ci);
  const dim3 grid(d->B * (d->Wi / TW) * (d->Hi / rb));
  const uint32_t xbytes = (uint32_t)((size_t)d->B * d->Hi * d->Wi * d->Ci * 2);
  const bool row16 = crnn_option(CRNN_OPT_HALO_ROW16) != 0;
  if (d->Ci == 8 && row16)
    hipLaunchKernelGGL((halo3x3_kernel<8, 64, false, false, true>), grid, dim3(512), 0, st, (const bf16*)x,
                       (const bf16*)w, (bf16*)y, psum, psq, d->Hi, d->Wi, rb, xbytes, esc, esh);
  else if (d->Ci == 8)
    hipLaunchKernelGGL((halo3x3_kernel<8, 64, false>), grid, dim3(512), 0, st, (const bf16*)x, (const bf16*)w,
                       (bf16*)y, psum, psq, d->Hi, d->Wi, rb, xbytes, esc, esh);
  else
    hipLaunchKernelGGL((halo3x3_kernel<64, 128, false>), grid, dim3(512), 0, st, (const bf16*)x, (const bf16*)w,
                       (bf16*)y, psum, psq, d->Hi, d->Wi, rb, xbytes, esc, esh);
  return (int)hipGetLastError();
}

bool conv_halo_pool_fits(const crnn_conv_desc* d) {
  return d->Ci == 64 && d->Co == 128 && d->Hi % 2 == 0 && d->Wi % 2 == 0 && band_rows(d->Hi, d->Ci) % 2 == 0;
}

// eval stem: conv -> BN (running statistics) -> ReLU -> 2x2 max-pool in one launch, y = the pooled map
int conv_halo_fwd_pool(const crnn_conv_desc* d, const void* x, const void* w, void* y, const float* esc,
                       const float* esh, hipStream_t st) {
  const int rb = band_rows(d->Hi, d->Ci);
  if (d->Ci != 64 || d->Hi % 2 || d->Wi % 2 || rb % 2) return crnn_set_error(hipErrorInvalidValue, "halo pool: shape");
  const dim3 grid(d->B * (d->Wi / TW) * (d->Hi / rb));
  const uint32_t xbytes = (uint32_t)((size_t)d->B * d->Hi * d->Wi * d->Ci * 2);
  hipLaunchKernelGGL((halo3x3_kernel<64, 128, false, true>), grid, dim3(512), 0, st, (const bf16*)x,
                     (const bf16*)w, (bf16*)y, (float*)nullptr, (float*)nullptr, d->Hi, d->Wi, rb, xbytes, esc, esh);
  return (int)hipGetLastError();
}

int conv_halo_dgrad(const crnn_conv_desc* d, const void* dy, const void* w, void* dx, hipStream_t st) {
  const dim3 grid(d->B * (d->Wi / TW));
  const uint32_t dybytes = (uint32_t)((size_t)d->B * d->Ho * d->Wo * d->Co * 2);
  hipLaunchKernelGGL((halo3x3_kernel<128, 64, true>), grid, dim3(512), 0, st, (const bf16*)dy, (const bf16*)w,
                     (bf16*)dx, (float*)nullptr, (float*)nullptr, d->Hi, d->Wi, d->Hi, dybytes);
  return (int)hipGetLastError();
}

// stem wgrad on the halo kernel: grid = slabs = min(bands, CUs). The input conv's (CI = 8: 12 accumulator
// registers, 41 KB of LDS) streams dy with one row in flight per workgroup; CRNN_OPT_HALO_WG2 gives it one
// workgroup per band, up to two per CU, for twice the bytes in flight
int conv_halo_wgrad_slabs(const crnn_conv_desc* d) {
  const int bands = d->B * (d->Wi / TW);
  int ncu = crnn_cu_count();
  if (ncu <= 0) ncu = 256;
  const int cap = d->Ci == 8 && crnn_option(CRNN_OPT_HALO_WG2) ? 2 * ncu : ncu;
  return bands < cap ? bands : cap;
}

int conv_halo_wgrad(const crnn_conv_desc* d, const void* dy, const void* x, float* ws, hipStream_t st) {
  const int S = conv_halo_wgrad_slabs(d);
  const uint32_t dybytes = (uint32_t)((size_t)d->B * d->Ho * d->Wo * d->Co * 2);
  const uint32_t xbytes = (uint32_t)((size_t)d->B * d->Hi * d->Wi * d->Ci * 2);
  if (d->Ci == 8)
    hipLaunchKernelGGL((halo3x3_wgrad_kernel<8, 64>), dim3(S), dim3(512), 0, st, (const bf16*)dy, (const bf16*)x, ws,
                       d->B, d->Hi, d->Wi, dybytes, xbytes);
  else
    hipLaunchKernelGGL((halo3x3_wgrad_kernel<64, 128>), dim3(S), dim3(512), 0, st, (const bf16*)dy, (const bf16*)x,
                       ws, d->B, d->Hi, d->Wi, dybytes, xbytes);
  return (int)hipGetLastError();
}
