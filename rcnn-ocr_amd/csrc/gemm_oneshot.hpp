// Latency-oriented bf16 GEMM for the LSTM recurrence (small M = batch, one step at a time).
//
//   C[m][n] = sum_{k in split} A(m,k) * B(n,k)      A, B K-contiguous (gemm.hpp loaders with offs())
//
// A 64 x 64 tile per block (4 waves, 2 x 2, each 32 x 32): the block's whole K chunk (<= KC = 512,
// i.e. 8 sub-tiles of 64) is staged by LDS-DMA in ONE burst — 32 buffer_load...lds per wave, one
// vmcnt(0), one barrier — then 64 MFMAs per wave run back to back. The step GEMMs have only
// ~8 K-stages of work, so a staged pipeline spends its time in per-stage round trips; the burst
// pays one. LDS: 8 x (64 + 64) rows x 128 B = 128 KB (1 block per CU, 256 blocks fill the chip).
// Sub-tile image = gemm256's K-contiguous layout: rows of 64 bf16, 16-B chunks XOR (row>>1)&7,
// swizzle applied on the DMA source side.
// nsplit: K split across blocks (each split <= KC); nbatch: independent problems selected by the
// loaders' / epilogue's set_batch (the two LSTM directions).
#pragma once
#include "gemm256.hpp"

namespace gemm {

template <int KC, class LA, class LB, class EPI>
__global__ __launch_bounds__(256) void gemm_oneshot_kernel(LA la, LB lb, EPI epi, int M, int N, int K, int klen,
                                                           int tiles_m, int tiles_n, int nsplit, int nbatch) {
  using T = bf16;
  static_assert(!LA::kRowVec && !LB::kRowVec, "K-contiguous operands");
  static_assert(KC % 64 == 0 && KC <= 512, "K chunk");
  constexpr int BM = 64, BN = 64, KT = KC / 64;
  constexpr int TA = BM * 128, TB = BN * 128, SUB = TA + TB;
  __shared__ __attribute__((aligned(1024))) char smem[KT * SUB];

  const int nwg = tiles_m * tiles_n * nsplit * nbatch;
  const int wg = xcd_remap(blockIdx.x, nwg);
  const int n_tile = wg % tiles_n;
  const int m_tile = (wg / tiles_n) % tiles_m;
  const int kz = (wg / (tiles_n * tiles_m)) % nsplit;
  const int bz = wg / (tiles_n * tiles_m * nsplit);
  if constexpr (has_set_batch<LA>::value) la.set_batch(bz);
  if constexpr (has_set_batch<LB>::value) lb.set_batch(bz);
  if constexpr (has_set_batch<EPI>::value) epi.set_batch(bz);
  const int m0 = m_tile * BM, n0 = n_tile * BN;
  const int kbeg = kz * klen;
  const int kend = min(K, kbeg + klen);
  const int nk = kend > kbeg ? min(KT, (kend - kbeg + 63) / 64) : 0;

  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wid >> 1, wc = wid & 1;

  // ---- one burst: every sub-tile, 8-row groups 2*wid, 2*wid+1 of A and of B per wave
  {
    typename LA::Ctx ca[2];
    typename LB::Ctx cb[2];
    int ka[2], kb[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int r = (2 * wid + i) * 8 + (lane >> 3);
      ca[i] = la.row_ctx(m0 + r);
      cb[i] = lb.row_ctx(n0 + r);
      ka[i] = kb[i] = ((lane & 7) ^ ((r >> 1) & 7)) * 8;
    }
    const __amdgpu_buffer_rsrc_t ra = la.rsrc(), rb = lb.rsrc();
    for (int kt = 0; kt < nk; ++kt) {
      const typename LA::Prep pa = la.prep(kbeg + kt * 64);
      const typename LB::Prep pb = lb.prep(kbeg + kt * 64);
      char* sub = smem + kt * SUB;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        dma16(ra, sub + (2 * wid + i) * 1024, la.offs(ca[i], pa, ka[i]));
        dma16(rb, sub + TA + (2 * wid + i) * 1024, lb.offs(cb[i], pb, kb[i]));
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int kt = 0; kt < nk; ++kt) {
    const T* As = reinterpret_cast<const T*>(smem + kt * SUB);
    const T* Bs = reinterpret_cast<const T*>(smem + kt * SUB + TA);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 af[2], bfr[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) af[i] = frag<T, BM, false, false, 64>(As, wr * 32 + i * 16, kk, lane);
#pragma unroll
      for (int j = 0; j < 2; ++j) bfr[j] = frag<T, BN, false, false, 64>(Bs, wc * 32 + j * 16, kk, lane);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) mma<T>(acc[i][j], bfr[j], af[i]);
    }
  }
  const int mr = lane & 15, nq = 4 * (lane >> 4);
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) epi.store(m0 + wr * 32 + i * 16 + mr, n0 + wc * 32 + j * 16 + nq, acc[i][j], kz);
}

// splits of <= KC over K (multiples of 64); returns the split count used
template <int KC, class LA, class LB, class EPI>
inline int launch_oneshot(const LA& la, const LB& lb, const EPI& epi, int M, int N, int K, int nsplit, hipStream_t st,
                          int nbatch = 1) {
  if (M <= 0 || N <= 0) return 0;
  const int tm = (M + 63) / 64, tn = (N + 63) / 64;
  int klen = (K + nsplit - 1) / nsplit;
  klen = (klen + 63) / 64 * 64;
  if (klen > KC) return -1;
  nsplit = K > 0 ? (K + klen - 1) / klen : 1;
  hipLaunchKernelGGL((gemm_oneshot_kernel<KC, LA, LB, EPI>), dim3(tm * tn * nsplit * nbatch), dim3(256), 0, st, la, lb,
                     epi, M, N, K, klen, tm, tn, nsplit, nbatch);
  return (int)hipGetLastError();
}

}  // namespace gemm
