// 256-row bf16 conv GEMM with a W-halo A image (r04): 3x3 / stride 1 / pad 1 convolutions whose output
// width Wo is a power of two in [32, 256] (the forward conv and the stride-1 input gradient on the
// forward path, conv.hip). Same tiles, waves, phases, B operand, epilogue and stagger as gemm256_item
// (gemm256.hpp); only the A operand differs.
//
// gemm256_item stages A per K-tile: 256 output rows x 64 channels of ONE tap, so each input pixel
// crosses L2 -> LDS once per tap (9 times per channel block), and the A LDS-DMA is 1/2 of the DMA
// pieces a workgroup issues. Here the K-tiles run in (kh, channel block, kw) order, and ONE image per
// (kh, channel block) serves its three kw K-tiles: the tile's 256/Wo output rows, each widened by
// one pixel on both sides (Wo + 2 image rows per output row, zero where the column is padding), so
// output row r at tap kw reads image row r + 2 (r / Wo) + kw. The B operand's K order follows by
// remapping the K-tile's first k.
//
// Image layout: rows of 10 16-B slots (pitch 160 B; slots 8 and 9 are padding). A fragment read is then
// a per-lane base (row c16, chunk g4) plus a wave-uniform offset (first row, kw, buffer): one VALU add
// per fragment. With pitch 160 the 16 lanes of every ds_read_b128 lane group land on distinct banks at
// ANY first row (enumerated). An XOR-swizzled 128-B pitch needs ~5 VALU per fragment to rebuild the
// swizzle for each kw shift, which cost more than the DMA it saved (+24 % VALU, +7 % busy cycles,
// profiles/r04m_*). A DMA wave-instruction fills 64 consecutive slots (6.4 rows); its lanes on padding
// slots read zeros. <= 43 pieces per image (8 output rows of 32 + 2 columns = 272 rows); IA = 6 per
// wave, pieces past the image go to a dummy KB.
//
// LDS: two image buffers (43 KB each: image u+1 is filled while the three K-tiles of image u read the
// other), the dummy KB, and the two B stages of gemm256_item (32 KB each at BN = 256) = 151 KB.
//
// DMA schedule (per wave; vmcnt retires in issue order):
//   K-tile 3u   : P1 image u+1 pieces 0, 1; P2 piece 2     P3 / P4: B of K-tile t+2 (as gemm256_item)
//   K-tile 3u+1 : P1 pieces 3, 4;       P2 piece 5         P3 / P4: B of t+2
//   K-tile 3u+2 : -                                       P3 / P4: B of t+2
// The image buffer of u+1 was last read in P3 of K-tile 3u-1 (the distance gemm256_item keeps between
// a half-tile's last read and its re-fill). The P4 wait of K-tile t leaves outstanding only what was
// issued after the B of t+1 (tile t's image pieces and the B of t+2), so the image of K-tile 3u+3 is
// complete at the P4 wait of 3u+2.
#pragma once
#include "gemm256.hpp"

namespace gemm {

struct HaloWDesc {
  const bf16* x;      // NHWC input [B][Hi][Wi][Ci] (Hi = Ho, Wi = Wo)
  uint32_t bytes;     // of x (buffer descriptor range: out-of-range offsets read zero)
  int B, Ho, Wo, Ci;  // Ci % 64 == 0
  int lwo;            // log2(Wo)
  int ncb;            // Ci / 64
};

template <int BN, int SKIP, class LB, class EPI>
__global__ __launch_bounds__(512) void gemm256hw_kernel(HaloWDesc a, LB lb, EPI epi, int M, int N, int tiles_m,
                                                        int tiles_n, int stagger) {
  using T = bf16;
  constexpr int BM = 256;
  constexpr int WM = BM / 2, WN = BN / 4;
  constexpr int MI = WM / 16, NI = WN / 16;
  constexpr int MQ = MI / 2, NQ = NI / 2;
  constexpr int QN = WN / 2;
  using OB = Op256<LB, BN, QN>;
  constexpr int IA = 6;                    // image pieces (64 slots of 16 B) per wave
  constexpr int NPMAX = 43;                // pieces of the largest image (272 rows x 10 slots)
  constexpr int AIMG = NPMAX * 1024;       // one image buffer
  constexpr int PITCH = 160;               // image row pitch (10 slots)
  constexpr int VB = 2 * OB::I;            // B DMA instructions of one K-tile
  __shared__ __attribute__((aligned(1024))) char smem[2 * AIMG + 1024 + 2 * OB::TB];

  // ---- work item (as gemm256_kernel: XCD remap, grouped tile order)
  const int nwg = tiles_m * tiles_n;
  const int wg = xcd_remap(blockIdx.x, nwg);
  int n_tile = wg % tiles_n, m_tile = wg / tiles_n;
  if constexpr (GEMM_GROUP_M > 0) {
    const int per = GEMM_GROUP_M * tiles_n, g0 = (wg / per) * GEMM_GROUP_M;
    const int gs = min(tiles_m - g0, GEMM_GROUP_M);
    m_tile = g0 + (wg % per) % gs;
    n_tile = (wg % per) / gs;
  }
  const int m0 = m_tile * BM, n0 = n_tile * BN;

  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wid >> 2, wc = wid & 3;

  OB ob;
  ob.init(lb, n0, wid, lane, wc);
  const __amdgpu_buffer_rsrc_t rb = lb.rsrc();
  const __amdgpu_buffer_rsrc_t ra = mk_rsrc(a.x, a.bytes);
  char* const sA = smem;
  char* const sDummy = smem + 2 * AIMG;   // destination of the pieces past the image (zeros)
  char* const sB = smem + 2 * AIMG + 1024;

  // ---- image DMA contexts: lane l of piece q = IA wid + i fills slot 64 q + l = (row j, chunk c)
  const int W2 = a.Wo + 2, Wi = a.Wo, Hi = a.Ho;
  const int IR = (BM >> a.lwo) * W2;       // image rows in use
  const int NP = (IR * 10 + 63) >> 6;      // pieces in use (<= NPMAX)
  const int orow0 = m0 >> a.lwo;           // the tile's first output row (b Ho + ho)
  // per piece: element offset of (b, ho, wcol, chunk c) in bits 0-28 (host: x < 2^30 bytes), bit 29 + kh
  // set when that input row exists and the slot is a real chunk of a real column (one register per piece)
  uint32_t actx[IA];
#pragma unroll
  for (int i = 0; i < IA; ++i) {
    const int sl = (wid * IA + i) * 64 + lane;
    const int j = (sl * 0xCCCD) >> 19, c = sl - 10 * j;   // sl / 10 (sl < 2^14)
    const int q = j / W2, wcol = j - q * W2 - 1, orow = orow0 + q;
    const int b = orow / a.Ho, ho = orow - b * a.Ho;
    const bool ok = c < 8 && j < IR && orow < a.B * a.Ho && wcol >= 0 && wcol < Wi;
    uint32_t mk = 0;
#pragma unroll
    for (int kh = 0; kh < 3; ++kh)
      if (ok && (unsigned)(ho + kh - 1) < (unsigned)Hi) mk |= 1u << (29 + kh);
    // the kh = 1 row's offset: non-negative whenever a row bit is set
    actx[i] = mk | ((uint32_t)(((b * Hi + ho) * Wi + wcol) * a.Ci + c * 8) & 0x1fffffffu);
  }
  const int rowstride = Wi * a.Ci;
  auto issue_a = [&](int i, int buf, int kh, int cb) __attribute__((always_inline)) {
    const uint32_t cx = actx[i];
    const uint32_t voff = ((cx >> (29 + kh)) & 1u)
                              ? (uint32_t)((int)(cx & 0x1fffffffu) + (kh - 1) * rowstride + cb * 64) * 2u : OOB;
    const int pq = wid * IA + i;
    dma16(ra, pq < NP ? sA + buf * AIMG + pq * 1024 : sDummy, voff);
  };

  f32x4 acc[MI][NI];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // ---- prologue: image 0, B of K-tiles 0 and 1; wait for all but the last (B of 1)
#pragma unroll
  for (int i = 0; i < IA; ++i) issue_a(i, 0, 0, 0);
  {
    const int k0 = 0, k1 = a.Ci;             // K-tiles 0 and 1: (kh 0, cb 0, kw 0 / 1)
    ob.issue(lb, rb, sB, 0, k0);
    ob.issue(lb, rb, sB, 1, k0);
    ob.issue(lb, rb, sB + OB::TB, 0, k1);
    ob.issue(lb, rb, sB + OB::TB, 1, k1);
  }
  asm volatile("s_waitcnt vmcnt(%0)" ::"i"(VB) : "memory");
  raw_barrier();
  if (stagger && wr == 1) raw_barrier();

  bf16x8 af[MQ][2], bfr[NI][2];
  const uint32_t lbase = (uint32_t)((lane & 15) * PITCH + (lane >> 4) * 16);   // row c16, chunk g4
  // A fragments of quadrant H (rows wr*128 + H*64 + 16f + c16) at tap kw from image buffer ib
  auto read_a = [&](auto hc, auto fmc, int ib, int kw) __attribute__((always_inline)) {
    constexpr int H = decltype(hc)::value;
    constexpr uint32_t FM = decltype(fmc)::value;
    // the wave's row base, opaque here: every uniform offset below is rebuilt per call by a few SALU
    // ops instead of 24 loop-invariant SGPRs (which spill, through VGPR lanes, next to the accumulators)
    int wbase = wr * WM;
    asm volatile("" : "+s"(wbase));
#pragma unroll
    for (int f = 0; f < MQ; ++f)
      if ((FM >> (H * MQ + f)) & 1u) {
        const int rbf = wbase + H * (WM / 2) + f * 16;
        // wave-uniform byte offset of the fragment's first row
        int u0 = ib * AIMG + (rbf + ((rbf >> a.lwo) << 1) + kw) * PITCH;
        asm volatile("" : "+s"(u0));
        const char* p = sA + lbase + u0;
        af[f][0] = *reinterpret_cast<const bf16x8*>(p);
        af[f][1] = *reinterpret_cast<const bf16x8*>(p + 64);
      }
  };

  // K-tile t = 3u + P of image u = (kh, cb); the next image (khn, cbn) exists when nu
  auto ktile = [&](auto pc, auto fmc, int u, int kh, int cb, int khn, int cbn, bool nu)
                   __attribute__((always_inline)) {
    constexpr int P = decltype(pc)::value;   // position in the image's three K-tiles = kw
    constexpr uint32_t FM = decltype(fmc)::value;
    const int ib = u & 1, bs = (u + P) & 1;
    const char* Bs = sB + bs * OB::TB;
    const uint32_t lB = lds_addr(Bs);
    const bool n2 = P == 0 || nu;            // K-tile t + 2 exists
    // its first k in the reference order: (kh, kw = 2) of this image, or kw = P - 1 of the next
    const int kb2 = P == 0 ? (kh * 3 + 2) * a.Ci + cb * 64 : (khn * 3 + (P - 1)) * a.Ci + cbn * 64;
    // ---- P1: quadrant (0,0)
    read_a(std::integral_constant<int, 0>{}, fmc, ib, P);
    ob.template load<0, NQ>(*reinterpret_cast<bf16x8(*)[NQ][2]>(&bfr[0]), Bs, lB, wc * WN, lane);
    if constexpr (P == 0) {
      if (nu) {
        issue_a(0, ib ^ 1, khn, cbn);
        issue_a(1, ib ^ 1, khn, cbn);
      }
    } else if constexpr (P == 1) {
      if (nu) {
        issue_a(3, ib ^ 1, khn, cbn);
        issue_a(4, ib ^ 1, khn, cbn);
      }
    }
    lds_wait_all();
    raw_barrier();
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int i = 0; i < MQ; ++i)
        if ((FM >> i) & 1u)
#pragma unroll
          for (int j = 0; j < NQ; ++j) mma<T>(acc[i][j], bfr[j][kk], af[i][kk]);
    __builtin_amdgcn_s_setprio(0);
    raw_barrier();
    // ---- P2: quadrant (0,1)
    ob.template load<1, NQ>(*reinterpret_cast<bf16x8(*)[NQ][2]>(&bfr[NQ]), Bs, lB, wc * WN, lane);
    if constexpr (P == 0) {
      if (nu) issue_a(2, ib ^ 1, khn, cbn);
    } else if constexpr (P == 1) {
      if (nu) issue_a(5, ib ^ 1, khn, cbn);
    }
    lds_wait_all();
    raw_barrier();
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int i = 0; i < MQ; ++i)
        if ((FM >> i) & 1u)
#pragma unroll
          for (int j = NQ; j < NI; ++j) mma<T>(acc[i][j], bfr[j][kk], af[i][kk]);
    __builtin_amdgcn_s_setprio(0);
    raw_barrier();
    // ---- P3: quadrant (1,1)
    read_a(std::integral_constant<int, 1>{}, fmc, ib, P);
    if (n2) ob.issue(lb, rb, sB + bs * OB::TB, 0, kb2);
    lds_wait_all();
    raw_barrier();
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int i = 0; i < MQ; ++i)
        if ((FM >> (MQ + i)) & 1u)
#pragma unroll
          for (int j = NQ; j < NI; ++j) mma<T>(acc[MQ + i][j], bfr[j][kk], af[i][kk]);
    __builtin_amdgcn_s_setprio(0);
    raw_barrier();
    // ---- P4: quadrant (1,0); wait: all but what this tile issued after the B of t+1
    if (n2) {
      ob.issue(lb, rb, sB + bs * OB::TB, 1, kb2);
      if constexpr (P == 0) {
        if (nu) asm volatile("s_waitcnt vmcnt(%0)" ::"i"(VB + 3) : "memory");
        else asm volatile("s_waitcnt vmcnt(%0)" ::"i"(VB) : "memory");
      } else if constexpr (P == 1) {
        if (nu) asm volatile("s_waitcnt vmcnt(%0)" ::"i"(VB + 3) : "memory");
        else asm volatile("s_waitcnt vmcnt(%0)" ::"i"(VB) : "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(%0)" ::"i"(VB) : "memory");
      }
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    raw_barrier();
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int i = 0; i < MQ; ++i)
        if ((FM >> (MQ + i)) & 1u)
#pragma unroll
          for (int j = 0; j < NQ; ++j) mma<T>(acc[MQ + i][j], bfr[j][kk], af[i][kk]);
    __builtin_amdgcn_s_setprio(0);
    raw_barrier();
  };
  auto triple = [&](auto fmc, int u, int kh, int cb, int khn, int cbn, bool nu) __attribute__((always_inline)) {
    ktile(std::integral_constant<int, 0>{}, fmc, u, kh, cb, khn, cbn, nu);
    ktile(std::integral_constant<int, 1>{}, fmc, u, kh, cb, khn, cbn, nu);
    ktile(std::integral_constant<int, 2>{}, fmc, u, kh, cb, khn, cbn, nu);
  };
  // kernel row kh owns images [ncb kh, ncb (kh + 1)); SKIP as gemm256_item (4-row maps: the fragment
  // rows that read only padding at kh = 0 / 2)
  constexpr uint32_t M0 = SKIP == 1 ? 0xfcu : (SKIP == 2 ? 0x3fu : 0xffu);
  constexpr uint32_t M2 = SKIP == 1 ? 0x3fu : (SKIP == 2 ? 0xfcu : 0xffu);
  if constexpr (SKIP == 0) {
    int kh = 0, cb = 0;
    for (int u = 0; u < 3 * a.ncb; ++u) {
      const bool last = cb + 1 == a.ncb;
      const int khn = last ? kh + 1 : kh, cbn = last ? 0 : cb + 1;
      triple(std::integral_constant<uint32_t, 0xffu>{}, u, kh, cb, khn, cbn, khn < 3);
      kh = khn;
      cb = cbn;
    }
  } else {
    auto row = [&](auto fmc, int kh) __attribute__((always_inline)) {
      for (int cb = 0; cb < a.ncb; ++cb) {
        // kh opaque inside the loop: no per-lane kh-derived values hoisted per segment (register budget)
        asm volatile("" : "+s"(kh));
        const bool last = cb + 1 == a.ncb;
        const int khn = last ? kh + 1 : kh, cbn = last ? 0 : cb + 1;
        triple(fmc, kh * a.ncb + cb, kh, cb, khn, cbn, khn < 3);
      }
    };
    row(std::integral_constant<uint32_t, M0>{}, 0);
    row(std::integral_constant<uint32_t, 0xffu>{}, 1);
    row(std::integral_constant<uint32_t, M2>{}, 2);
  }
  if (stagger && wr == 0) raw_barrier();
  // nothing of the epilogue (per-column BN constants of the tile hooks) is computed before this point
  asm volatile("" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);

  // ---- epilogue (as gemm256_item)
  const int mr = lane & 15, nq = 4 * (lane >> 4);
  if constexpr (has_row8<EPI>::value && crnn_row8_on) {
    row8_epilogue<MI, NI, WM, WN>(acc, epi, smem, wid, lane, m0 + wr * WM, n0 + wc * WN, 0);
  } else {
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NI; ++j) epi.store(m0 + wr * WM + i * 16 + mr, n0 + wc * WN + j * 16 + nq, acc[i][j], 0);
  }
  if constexpr (EPI::kStats) wave_col_stats<MI, NI>(acc, epi, M, m0 + wr * WM, m_tile * 2 + wr, n0 + wc * WN, lane);
  if constexpr (has_tile_hook<EPI>::value) epi.template tile<MI, NI>(acc, M, m0 + wr * WM, m_tile * 2 + wr, n0 + wc * WN, lane);
}

// the W-halo kernel takes a 3x3 / stride-1 / pad-1 geometry with Ci % 64 == 0 and Wo a power of two in
// [32, 256] (then 256 output rows are whole output rows and the image fits NPMAX pieces)
inline int halo_w_log2(int Wo) {
  for (int l = 5; l <= 8; ++l)
    if (Wo == (1 << l)) return l;
  return -1;
}

template <int BN, int SKIP, class LB, class EPI>
inline int launch256hw(const HaloWDesc& a, const LB& lb, const EPI& epi, int M, int N, hipStream_t st) {
  if (M <= 0 || N <= 0) return 0;
  const int tm = (M + 255) / 256, tn = (N + BN - 1) / BN;
  hipLaunchKernelGGL((gemm256hw_kernel<BN, SKIP, LB, EPI>), dim3(tm * tn), dim3(512), 0, st, a, lb, epi, M, N, tm, tn,
                     crnn_option(CRNN_OPT_GEMM_STAGGER));
  return (int)hipGetLastError();
}

}  // namespace gemm
