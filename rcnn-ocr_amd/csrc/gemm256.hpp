// Deep-pipelined bf16 MFMA GEMM: BM x BN = 256 x {256,128} tiles, 512 threads (8 waves as
// 2(M) x 4(N)), K-tile 64, operands staged global -> LDS by LDS-DMA (buffer_load ... lds).
//
//   C[m][n] = sum_k A(m,k) * B(n,k)       (gemm.hpp loaders with offs()/rsrc(); either operand
//                                          K-contiguous or row-contiguous, split-K optional)
//
// Why this shape (cdna_hip_programming.md §5): a 128^2 tile with a barrier per K-step stalls on the
// vmcnt(0) that __syncthreads() emits while the next stage is in flight. Here the LDS-DMA
// prefetch stays in flight ACROSS raw s_barriers and is retired by a counted vmcnt once per
// K-tile, with 1 block per CU doing 64 MFMAs per wave per K-tile.
//
// Schedule of K-tile t (LDS buffer b = t & 1), four phases, one C quadrant (mh, nh) each:
//   P1 (0,0): read A[mh=0], B[nh=0] fragments     issue A-half1 of tile t+1 -> buffer b^1
//   P2 (0,1): read B[nh=1]                         issue A-half0 of tile t+2 -> buffer b
//   P3 (1,1): read A[mh=1]                         issue B-half0 of tile t+2 -> buffer b
//   P4 (1,0): (registers only)                     issue B-half1 of tile t+2 -> buffer b; vmcnt(VM)
// each phase: ds_reads, DMA issue, s_barrier, lgkmcnt(0), 16 MFMA, s_barrier. A half-tile slot is
// re-filled only after the phase that read it into registers has passed its second barrier (WAR),
// and tile t+1 is complete once P4 of tile t retires everything but tile t+2's last three
// half-tiles (RAW: read one phase after the wait).
//
// LDS image: rows of 64 bf16 (128 B), 16-B chunks XOR-swizzled by (row>>1)&7 (gemm::swz) — the
// DMA destination is lane-linear (1 KiB = 8 rows per wave-instruction), so the swizzle is applied
// on the SOURCE side: the lane that fills physical chunk c of row r loads logical chunk c^swz(r).
// A half h holds the quadrant row blocks {r : (r / QM) % 2 == h} (same for B with QN).
#pragma once
#include "gemm.hpp"

#include <type_traits>
#include <utility>
#include "crnn_hip.h"
int crnn_option(int key);  // capi.cpp (crnn_set_option)
int crnn_cu_count();       // capi.cpp: compute units of the current device (cached)
#ifndef GEMM_GROUP_M
#define GEMM_GROUP_M 8   // grouped tile order (launch kernels below); 0 = plain row-major tile order
#endif

namespace gemm {

typedef __attribute__((address_space(3))) void lds_void_t;

__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t r, char* lds_seg, uint32_t voff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void_t*)lds_seg, 16, voff, 0, 0, 0);
}

// Row-contiguous fragments are read with ds_read_b64_tr_b16 as inline asm (Op256::trd): the
// builtin makes hipcc drain every in-flight LDS-DMA (s_waitcnt vmcnt(0)) before it, which would
// de-pipeline the kernel; the asm read is not tracked by hipcc, so the kernel's own lgkmcnt(0)
// after each phase barrier retires it.

// after the explicit lgkmcnt(0): keep the scheduler from hoisting MFMAs that consume asm reads
__device__ __forceinline__ void lds_wait_all() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

// lgkmcnt(0) the compiler's waitcnt pass knows about (an inline-asm wait is opaque to it, so it
// would still count the waited reads as outstanding and add its own, later, waits)
__device__ __forceinline__ void lds_wait_all_known() {
  __builtin_amdgcn_s_waitcnt(0xC07F);   // gfx9 encoding: vmcnt 63, expcnt 7, lgkmcnt 0
  __builtin_amdgcn_sched_barrier(0);
}

// compile-time loop: f(integral_constant<int, i>) for i = 0 .. N-1
template <class F, int... I>
__device__ __forceinline__ void sfor_impl(F&& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, class F> __device__ __forceinline__ void sfor(F&& f) {
  sfor_impl(f, std::make_integer_sequence<int, N>{});
}

__device__ __forceinline__ void raw_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// optional epilogue hook: an EPI with `static constexpr bool kTileHook = true` gets
// epi.tile<MI, NI>(acc, M, first row, partial row, first column, lane) after its stores
template <class E, class = void> struct has_tile_hook : std::false_type {};
template <class E> struct has_tile_hook<E, std::void_t<decltype(E::kTileHook)>> : std::bool_constant<E::kTileHook> {};

// optional row-vector stores: an EPI with `static constexpr bool kRow8 = true` gets
// epi.store8(m, n, f32x4 lo, f32x4 hi, kz) for 8 consecutive columns n..n+7 of row m (one 16-B bf16
// store) instead of store() per 4 columns. The accumulators are transposed through LDS first (the
// MFMA layout gives a lane 4 columns of a row): a wave-instruction then stores whole 128-B row
// pieces with half the store instructions — the epilogue's store tail is issue-bound
// (MI355X_MICROARCH.md, epilogue store tail).
// an EPI with `static constexpr int kPrefer4W = bit` runs on the 4-wave form when CRNN_OPT_GEMM4W has that bit
// (2: the conv weight-gradient slabs, 4: the BN-fused conv input gradients, 8: the BiLSTM weight-gradient
// slabs; per-layer kbench, profiles/r05y/: the conv wgrads gain, the forwards lose); CRNN_OPT_GEMM4W = 1:
// every launch. Off by default: one unreproduced co-scheduled determinism failure with bit 2 on
template <class E, class = void> struct prefers_4w : std::integral_constant<int, 0> {};
template <class E> struct prefers_4w<E, std::void_t<decltype(E::kPrefer4W)>> : std::integral_constant<int, E::kPrefer4W> {};

template <class E, class = void> struct has_row8 : std::false_type {};
template <class E> struct has_row8<E, std::void_t<decltype(E::kRow8)>> : std::bool_constant<E::kRow8> {};

// per-wave, per-column partial statistics (sum, sum of squared deviations from the partial
// mean) over this wave's WM accumulator rows — the BN two-pass-in-registers epilogue
template <int MI, int NI, class EPI>
__device__ __forceinline__ void wave_col_stats(const f32x4 (&acc)[MI][NI], const EPI& epi, int M, int rbase,
                                               int prow, int ncol0, int lane) {
  constexpr int WM = MI * 16;
  const int mr = lane & 15, nq = 4 * (lane >> 4);
  const int nval = min(WM, max(0, M - rbase));
#pragma unroll
  for (int j = 0; j < NI; ++j) {
    f32x4 s = {0.f, 0.f, 0.f, 0.f}, q = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < MI; ++i) s += acc[i][j];
#pragma unroll
    for (int r = 0; r < 4; ++r) s[r] = rowgroup_sum<16>(s[r]);   // the 16 rows of a lane row (DPP)
    const float inv_n = nval > 0 ? 1.f / (float)nval : 0.f;
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      const bool ok = rbase + i * 16 + mr < M;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float dv = acc[i][j][r] - s[r] * inv_n;
        q[r] += ok ? dv * dv : 0.f;
      }
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) q[r] = rowgroup_sum<16>(q[r]);
    if (mr == 0) epi.stats(prow, ncol0 + j * 16 + nq, s, q);
  }
}

// One operand of the deep kernel: R rows (BM or BN), quadrant extent Q, staged by LDS-DMA.
//  K-contiguous (L::kRowVec false): image [R][64] (row pitch 128 B), chunk swizzle (row>>1)&7;
//    half h = rows {r : (r/Q) % 2 == h}, each wave-instruction fills 8 consecutive rows.
//  row-contiguous (L::kRowVec true): image [half][64 k][R/2 rows] (k-row pitch R bytes), 16-B chunk
//    swizzle fsw(k) on 32-B slots, read with ds_read_b64_tr_b16 from k-rows 8g+q (lo) and
//    8g+4+q (hi): a lane then holds k = 8g..8g+7 — the same k map as a K-contiguous ds_read_b128,
//    so mixed operands need no permuted (bank-conflicting) 8-byte reads. fsw keeps the 32 lanes
//    of each read pass on distinct banks for both R (checked by enumeration).
template <class L, int R, int Q, int NW = 8> struct Op256 {   // NW: waves of the workgroup
  static constexpr bool RV = L::kRowVec;
  static constexpr int I = R * 8 / (128 * NW);  // DMA wave-instructions per wave per half-tile
  static constexpr int kR = R, kQ = Q;
  static constexpr int TB = R * 64 * 2;    // tile bytes
  static constexpr int HB = TB / 2;
  typename L::Ctx ctx[2][I];
  int kofs[2][I], seg[2][I];
  uint32_t plo, phi;                       // RV: per-lane read offsets (half 0, kk 0, fragment 0)

  static __device__ __forceinline__ int fsw(int k) {
    return R == 256 ? 2 * ((k + 4 * (k >> 3)) & 7) : 2 * (((k >> 1) + 2 * (k >> 3)) & 3);
  }

  // base: first tile row of the block; blk: this wave's row block (wr or wc) of extent 2Q
  __device__ __forceinline__ void init(const L& l, int base, int wid, int lane, int blk) {
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int i = 0; i < I; ++i) {
        const int g = wid * I + i;
        if constexpr (!RV) {
          constexpr int per = Q / 8;
          const int r0 = (g / per) * 2 * Q + h * Q + (g % per) * 8;
          const int r = r0 + (lane >> 3);
          ctx[h][i] = l.row_ctx(base + r);
          kofs[h][i] = ((lane & 7) ^ ((r >> 1) & 7)) * 8;
          seg[h][i] = r0 * 128;
        } else {
          constexpr int CPR = R / 16, KPI = 64 / CPR;  // chunks per k-row, k-rows per instruction
          const int kr = g * KPI + lane / CPR;
          const int j = ((lane % CPR) ^ fsw(kr)) * 8;  // half-local row of this lane's 8 rows
          ctx[h][i] = l.row_ctx(base + (j / Q) * 2 * Q + h * Q + j % Q);
          kofs[h][i] = kr;
          seg[h][i] = h * HB + g * 1024;
        }
      }
    if constexpr (RV) {
      // fragment f of the wave's quadrant rows: half-local column blk*Q + 16f + 4p -> chunk
      // c0 + 2f with c0 = blk*Q/8 + (p>>1); c0 and 2f occupy disjoint bits, so chunk ^ fsw =
      // (c0 ^ fsw) ^ 2f and a fragment's offset is the lane offset XOR 32f.
      const int g = lane >> 4, c = lane & 15, q = c >> 2, p = c & 3;
      const int c0 = blk * (Q / 8) + (p >> 1);
      const int klo = 8 * g + q, khi = klo + 4;
      plo = (uint32_t)(klo * R + ((c0 ^ fsw(klo)) << 4) + (p & 1) * 8);
      phi = (uint32_t)(khi * R + ((c0 ^ fsw(khi)) << 4) + (p & 1) * 8);
    }
  }
  __device__ __forceinline__ void issue(const L& l, __amdgpu_buffer_rsrc_t rs, char* tile, int h,
                                        const typename L::Prep& p) const {
#pragma unroll
    for (int i = 0; i < I; ++i) dma16(rs, tile + seg[h][i], l.offs(ctx[h][i], p, kofs[h][i]));
  }

  template <int OFF> static __device__ __forceinline__ s16x4 trd(uint32_t a) {
    s16x4 v;
    asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(v) : "v"(a), "i"(OFF));
    return v;
  }
  static __device__ __forceinline__ bf16x8 cat(s16x4 lo, s16x4 hi) {
    s16x4 t[2] = {lo, hi};
    return *reinterpret_cast<const bf16x8*>(t);
  }
  // N fragments (rows rb0 + H*Q + 16f) x both 32-deep k sub-steps, from the operand tile at `tile`
  // (LDS address `lds` of the same tile for the row-contiguous asm reads)
  // FM (compile time): fragments to read, bit H * N + f (the A operand's padding-row skip)
  template <int H, int N, uint32_t FM = 0xffu>
  __device__ __forceinline__ void load(bf16x8 (&fr)[N][2], const char* tile, uint32_t lds, int rb0, int lane) const {
    if constexpr (!RV) {
#pragma unroll
      for (int f = 0; f < N; ++f)
        if ((FM >> (H * N + f)) & 1u)
#pragma unroll
          for (int kk = 0; kk < 2; ++kk)
            fr[f][kk] = gemm::frag<bf16, R, false, false, 64>(reinterpret_cast<const bf16*>(tile), rb0 + H * Q + f * 16, kk, lane);
    } else {
      const uint32_t bl = lds + plo, bh = lds + phi;
#pragma unroll
      for (int f = 0; f < N; ++f) {
        const uint32_t al = bl ^ (uint32_t)(32 * f), ah = bh ^ (uint32_t)(32 * f);
        fr[f][0] = cat(trd<H * HB>(al), trd<H * HB>(ah));
        fr[f][1] = cat(trd<H * HB + 32 * R>(al), trd<H * HB + 32 * R>(ah));
      }
    }
  }
};

__device__ __forceinline__ uint32_t lds_addr(const char* p) {
  return (uint32_t)(size_t)((const __attribute__((address_space(3))) char*)p);
}

#ifndef CRNN_ROW8_EPILOGUE
#define CRNN_ROW8_EPILOGUE 1
#endif
constexpr bool crnn_row8_on = CRNN_ROW8_EPILOGUE != 0;

// The wave's WM x WN accumulator block through its own LDS region (the pipeline's stage buffers are
// free once the K loop is done): two halves of 64 rows, fp32 row-major with the 16-B chunk index
// XOR-swizzled by the row (the 16 lanes of a write pass put one row each into distinct banks),
// then each lane reads 8 consecutive columns of a row and the epilogue stores them as one vector.
template <int MI, int NI, int WM, int WN, class EPI>
__device__ __forceinline__ void row8_epilogue(const f32x4 (&acc)[MI][NI], const EPI& epi, char* smem, int wid,
                                              int lane, int rbase, int cbase, int kz) {
  static_assert(WM == 128 && (WN == 64 || WN == 32), "row8 epilogue: 256-row tiles");
  constexpr int CH = WN / 4;            // 16-B chunks per row
  constexpr int LPR = WN / 8;           // lanes per row in the read-back
  constexpr int RPI = 64 / LPR;         // rows per read-back instruction
  float* stg = reinterpret_cast<float*>(smem) + wid * (64 * WN);
  const int mr = lane & 15, g = lane >> 4;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
#pragma unroll
    for (int ii = 0; ii < MI / 2; ++ii)
#pragma unroll
      for (int j = 0; j < NI; ++j) {
        const int r = ii * 16 + mr, q = (4 * j + g) ^ (r & (CH - 1));
        *reinterpret_cast<f32x4*>(stg + r * WN + 4 * q) = acc[h * (MI / 2) + ii][j];
      }
#pragma unroll
    for (int it = 0; it < 64 / RPI; ++it) {
      const int r = it * RPI + lane / LPR, c = (lane % LPR) * 8;
      const int q0 = (c / 4) ^ (r & (CH - 1)), q1 = (c / 4 + 1) ^ (r & (CH - 1));
      const f32x4 lo = *reinterpret_cast<const f32x4*>(stg + r * WN + 4 * q0);
      const f32x4 hi = *reinterpret_cast<const f32x4*>(stg + r * WN + 4 * q1);
      epi.store8(rbase + h * 64 + r, cbase + c, lo, hi, kz);
    }
  }
}

// Diagnostic build only (-DCRNN_GEMM_STAMPS=1, tools/gemm_stamps.py): per workgroup s_memrealtime
// stamps (10 ns) at entry, after the prologue, after the K loop, after the epilogue's stores are
// issued and after they completed, plus the XCC / hardware ids, into a per-TU device array read
// back by crnn_diag_gemm_stamps (defined in conv.hip). The stamps go to that array only.
#ifndef CRNN_GEMM_STAMPS
#define CRNN_GEMM_STAMPS 0
#endif
#if CRNN_GEMM_STAMPS
constexpr int GEMM_STAMP_SLOTS = 6;
constexpr int GEMM_STAMP_BLOCKS = 8192;
static __device__ unsigned long long g_gemm_stamps[GEMM_STAMP_BLOCKS * GEMM_STAMP_SLOTS];
__device__ __forceinline__ void gemm_stamp(int p) {
  if (threadIdx.x == 0 && blockIdx.x < GEMM_STAMP_BLOCKS)
    g_gemm_stamps[blockIdx.x * GEMM_STAMP_SLOTS + p] = __builtin_amdgcn_s_memrealtime();
}
__device__ __forceinline__ void gemm_stamp_ids() {
  if (threadIdx.x == 0 && blockIdx.x < GEMM_STAMP_BLOCKS) {
    unsigned x, h;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(h));
    g_gemm_stamps[blockIdx.x * GEMM_STAMP_SLOTS + 5] = ((unsigned long long)x << 32) | h;
  }
}
#define GEMM_STAMP(p) gemm_stamp(p)
#else
#define GEMM_STAMP(p)
#endif

// Diagnostic build only (-DCRNN_DIAG_A_ONCE=n, tools/build_variant.sh; results invalid): the A operand's
// LDS-DMA is issued for the first n K-tiles only, the later ones reuse whatever the buffers hold — the
// upper bound of a kernel that stages each conv input pixel once per channel chunk (halo tile) instead of
// once per tap
#ifndef CRNN_DIAG_A_ONCE
#define CRNN_DIAG_A_ONCE 0
#endif
__device__ __forceinline__ bool diag_a_issue(int t) { return CRNN_DIAG_A_ONCE == 0 || t < CRNN_DIAG_A_ONCE; }

// One work item of the grid kernel: tile (m_tile, n_tile), K range [kz*klen, min(K, (kz+1)*klen)).
template <int BM, int BN, int SKIP, class LA, class LB, class EPI>
__device__ __forceinline__ void gemm256_item(LA la, LB lb, EPI epi, int M, int K, int klen, int m_tile, int n_tile,
                                             int kz, int stagger, int ktk) {
  using T = bf16;
  static_assert(BM == 256 && (BN == 256 || BN == 128), "tile");
  constexpr int KS = 64;
  constexpr int WM = BM / 2, WN = BN / 4;        // per-wave output block
  constexpr int MI = WM / 16, NI = WN / 16;      // 16x16 fragments per wave
  constexpr int MQ = MI / 2, NQ = NI / 2;        // fragments per quadrant
  constexpr int QM = WM / 2, QN = WN / 2;        // quadrant extent
  using OA = Op256<LA, BM, QM>;
  using OB = Op256<LB, BN, QN>;
  constexpr int STAGE = OA::TB + OB::TB;
  constexpr int VM = OA::I + 2 * OB::I;          // DMA instructions of tile t+2 issued before the P4 wait
  __shared__ __attribute__((aligned(1024))) char smem[2 * STAGE];

  const int m0 = m_tile * BM, n0 = n_tile * BN;
  const int kbeg = kz * klen, kend = min(K, kbeg + klen);
  const int nk = kend > kbeg ? (kend - kbeg + KS - 1) / KS : 0;
  GEMM_STAMP(0);
#if CRNN_GEMM_STAMPS
  gemm_stamp_ids();
#endif

  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wid >> 2, wc = wid & 3;

  OA oa;
  OB ob;
  oa.init(la, m0, wid, lane, wr);
  ob.init(lb, n0, wid, lane, wc);
  const __amdgpu_buffer_rsrc_t ra = la.rsrc(), rb = lb.rsrc();
  char* const sA0 = smem;
  char* const sB0 = smem + OA::TB;

  f32x4 acc[MI][NI];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // ---- prologue: tile 0 whole, tile 1 except its A-half1 (issued in P1 of tile 0)
  typename LA::Prep pa2 = la.prep(kbeg);
  typename LB::Prep pb2 = lb.prep(kbeg);
  if (nk > 0) {
    oa.issue(la, ra, sA0, 0, pa2);
    ob.issue(lb, rb, sB0, 0, pb2);
    ob.issue(lb, rb, sB0, 1, pb2);
    oa.issue(la, ra, sA0, 1, pa2);
  }
  typename LA::Prep pa1 = pa2;  // prep of tile t+1 (for its A-half1)
  if (nk > 1) {
    pa1 = la.prep(kbeg + KS);
    const typename LB::Prep pb1 = lb.prep(kbeg + KS);
    oa.issue(la, ra, sA0 + STAGE, 0, pa1);
    ob.issue(lb, rb, sB0 + STAGE, 0, pb1);
    ob.issue(lb, rb, sB0 + STAGE, 1, pb1);
    asm volatile("s_waitcnt vmcnt(%0)" ::"i"(VM) : "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  raw_barrier();
  GEMM_STAMP(1);
  // ping-pong: waves 4-7 (wr == 1, one per SIMD) run one barrier behind waves 0-3, so each SIMD
  // alternates one wave's MFMA cluster with its partner's ds_read / LDS-DMA issue segment
  if (stagger && wr == 1) raw_barrier();

  bf16x8 af[MQ][2], bfr[NI][2];
  // one K-tile; FM (compile time): the fragment rows i whose MFMAs run (bit i). Fragment skipping
  // is only ever a compile-time property of a loop segment: a runtime mask test between the MFMAs
  // breaks the phase's MFMA cluster (measured 20-25 % slower, profiles/r02h_rowskip_regression.log)
  auto ktile = [&](auto fmc, int t) {
    constexpr uint32_t FM = decltype(fmc)::value;
    const int b = t & 1;
    const char* As = smem + b * STAGE;
    const char* Bs = As + OA::TB;
    const uint32_t lA = lds_addr(As), lB = lds_addr(Bs);
    const bool n1 = t + 1 < nk, n2 = t + 2 < nk;
    if (n2) {
      pa2 = la.prep(kbeg + (t + 2) * KS);
      pb2 = lb.prep(kbeg + (t + 2) * KS);
    }
    // ---- P1: quadrant (0,0)
    oa.template load<0, MQ, FM>(af, As, lA, wr * WM, lane);
    ob.template load<0, NQ>(*reinterpret_cast<bf16x8(*)[NQ][2]>(&bfr[0]), Bs, lB, wc * WN, lane);
    if (n1 && diag_a_issue(t + 1)) oa.issue(la, ra, sA0 + (b ^ 1) * STAGE, 1, pa1);
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
    if (n2 && diag_a_issue(t + 2)) oa.issue(la, ra, sA0 + b * STAGE, 0, pa2);
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
    oa.template load<1, MQ, FM>(af, As, lA, wr * WM, lane);
    if (n2) ob.issue(lb, rb, sB0 + b * STAGE, 0, pb2);
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
    // ---- P4: quadrant (1,0)
    if (n2) {
      ob.issue(lb, rb, sB0 + b * STAGE, 1, pb2);
      asm volatile("s_waitcnt vmcnt(%0)" ::"i"(VM) : "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    pa1 = pa2;
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
  if constexpr (SKIP == 0) {
    for (int t = 0; t < nk; ++t) ktile(std::integral_constant<uint32_t, 0xffu>{}, t);
  } else {
    // 3x3 conv over 4-row maps, one image per wave (128 rows = 4 rows x 32 columns): the K-tiles run
    // in tap order, kernel row kh owning [kh * ktk, (kh + 1) * ktk); for kh = 0 and kh = 2 one
    // image row (two fragment rows) reads only zero padding (SKIP 1: conv fwd, output row 0 / 3;
    // SKIP 2: dgrad, input row 3 / 0) — 1/6 of the MFMAs, skipped per segment at compile time
    constexpr uint32_t M0 = SKIP == 1 ? 0xfcu : 0x3fu, M2 = SKIP == 1 ? 0x3fu : 0xfcu;
    const int e0 = min(nk, ktk), e1 = min(nk, 2 * ktk);
    int t = 0;
    for (; t < e0; ++t) ktile(std::integral_constant<uint32_t, M0>{}, t);
    for (; t < e1; ++t) ktile(std::integral_constant<uint32_t, 0xffu>{}, t);
    for (; t < nk; ++t) ktile(std::integral_constant<uint32_t, M2>{}, t);
  }
  if (stagger && wr == 0) raw_barrier();
  GEMM_STAMP(2);

  const int mr = lane & 15, nq = 4 * (lane >> 4);
  if constexpr (has_row8<EPI>::value && crnn_row8_on) {
    row8_epilogue<MI, NI, WM, WN>(acc, epi, smem, wid, lane, m0 + wr * WM, n0 + wc * WN, kz);
  } else {
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NI; ++j) epi.store(m0 + wr * WM + i * 16 + mr, n0 + wc * WN + j * 16 + nq, acc[i][j], kz);
  }
  if constexpr (EPI::kStats) wave_col_stats<MI, NI>(acc, epi, M, m0 + wr * WM, m_tile * 2 + wr, n0 + wc * WN, lane);
  if constexpr (has_tile_hook<EPI>::value) epi.template tile<MI, NI>(acc, M, m0 + wr * WM, m_tile * 2 + wr, n0 + wc * WN, lane);
#if CRNN_GEMM_STAMPS
  GEMM_STAMP(3);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  GEMM_STAMP(4);
#endif
}

// One block per work item (the default): the K-loop above, block-level.
template <int BM, int BN, int SKIP, class LA, class LB, class EPI>
__global__ __launch_bounds__(512) void gemm256_kernel(LA la, LB lb, EPI epi, int M, int N, int K, int klen,
                                                      int tiles_m, int tiles_n, int nsplit, int stagger,
                                                      int nbatch, int ktk) {
  // one work item per block: ((batch * nsplit + split) * tiles_m + m_tile) * tiles_n + n_tile
  const int nwg = tiles_m * tiles_n * nsplit * nbatch;
  const int wg = xcd_remap(blockIdx.x, nwg);
  int n_tile = wg % tiles_n, m_tile = (wg / tiles_n) % tiles_m;
  const int kz = (wg / (tiles_n * tiles_m)) % nsplit;
  if constexpr (GEMM_GROUP_M > 0) {   // grouped tile order: GEMM_GROUP_M m-tiles share each n sweep (L2 reuse)
    const int pid = wg % (tiles_n * tiles_m), per = GEMM_GROUP_M * tiles_n, g0 = (pid / per) * GEMM_GROUP_M;
    const int gs = min(tiles_m - g0, GEMM_GROUP_M);
    m_tile = g0 + (pid % per) % gs;
    n_tile = (pid % per) / gs;
  }
  if (nbatch > 1) {
    const int bz = wg / (tiles_n * tiles_m * nsplit);
    if constexpr (has_set_batch<LA>::value) la.set_batch(bz);
    if constexpr (has_set_batch<LB>::value) lb.set_batch(bz);
    if constexpr (has_set_batch<EPI>::value) epi.set_batch(bz);
  }
  gemm256_item<BM, BN, SKIP>(la, lb, epi, M, K, klen, m_tile, n_tile, kz, stagger, ktk);
}

// 4-wave form helper: N fragments of one 32-deep k sub-step KK (see Op256::load), fragments
// F0 .. F0+N-1 of quadrant half H
template <class OP, int H, int N, int KK, int F0 = 0>
__device__ __forceinline__ void load_kk(const OP& op, bf16x8* fr, const char* tile, uint32_t lds, int rb0, int lane) {
  constexpr int R = OP::kR, Q = OP::kQ, HB = OP::HB;
  if constexpr (!OP::RV) {
#pragma unroll
    for (int f = 0; f < N; ++f)
      fr[f] = gemm::frag<bf16, R, false, false, 64>(reinterpret_cast<const bf16*>(tile), rb0 + H * Q + (F0 + f) * 16, KK, lane);
  } else {
    const uint32_t bl = lds + op.plo, bh = lds + op.phi;
#pragma unroll
    for (int f = 0; f < N; ++f) {
      const uint32_t al = bl ^ (uint32_t)(32 * (F0 + f)), ah = bh ^ (uint32_t)(32 * (F0 + f));
      fr[f] = OP::cat(OP::template trd<H * HB + KK * 32 * R>(al), OP::template trd<H * HB + KK * 32 * R>(ah));
    }
  }
}

// ---------------------------------------------------------------- 4-wave form (CRNN_OPT_GEMM4W)
// Same tile, K-tile, LDS image and operand loaders as gemm256_item, with ONE wave per SIMD: 4 waves
// as 2(M) x 2(N), each owning 128 x BN/2 (MI x NI = 8 x 8 fragments: all 256 AGPRs hold
// accumulators, so the MFMAs are asm tied to their AGPRs — the builtin's untied form would rotate
// them through VGPRs). The fragments of the two 32-deep k sub-steps live in two register sets
// (F0, F1), so every LDS read and LDS-DMA issue runs in the shadow of MFMAs of the other set. Per
// K-tile t (stage b = t & 1), S = 2 NM MFMA slots, one memory op after the MFMA of its slot:
//   slots [0, NR)            read F1(t) from b (one fragment per slot)
//   slot  B1 = NR + 8        lgkmcnt(0), s_barrier: every wave is done with stage b (WAR)
//   slots [B1, V)            LDS-DMA of tile t+2 -> b, spread evenly
//   slot  V = S - NR - 8     vmcnt(ND) [tile t+1, issued a K-tile earlier, landed], s_barrier (RAW)
//   slots [V, V + NR)        read F0(t+1) from b^1
// (r02j's 4-wave form read F1 and issued all DMA after one mid-tile barrier and waited for tile t+1
// half a tile after issuing it: the waves waited 21 % of their cycles.) Measured equal to the
// 8-wave form on this path (profiles/r02r_gemm4w_dma_study.log: the main-loop LDS-DMA issue stalls
// on the memory side in both), so it stays an option, off by default.
template <int BM, int BN, int SKIP, class LA, class LB, class EPI>
__device__ __forceinline__ void gemm4w_item(LA la, LB lb, EPI epi, int M, int K, int klen, int m_tile, int n_tile,
                                            int kz, int ktk) {
  static_assert(BM == 256 && (BN == 256 || BN == 128), "tile");
  constexpr int KS = 64, NW = 4;
  constexpr int WM = BM / 2, WN = BN / 2;        // per-wave output block (128 x 128 or 128 x 64)
  constexpr int MI = WM / 16, NI = WN / 16;      // fragments per wave
  constexpr int MQ = MI / 2, NQ = NI / 2;        // fragments per quadrant (LDS half)
  constexpr int QM = WM / 2, QN = WN / 2;
  using OA = Op256<LA, BM, QM, NW>;
  using OB = Op256<LB, BN, QN, NW>;
  constexpr int STAGE = OA::TB + OB::TB;
  constexpr int NM = MI * NI, NR = MI + NI, NDA = 2 * OA::I, ND = NDA + 2 * OB::I;
  constexpr int S = 2 * NM, B1 = NR + 8, V = S - NR - 8;
  static_assert(B1 + ND <= V && V + NR <= S, "schedule");
  __shared__ __attribute__((aligned(1024))) char smem[2 * STAGE];

  const int m0 = m_tile * BM, n0 = n_tile * BN;
  const int kbeg = kz * klen, kend = min(K, kbeg + klen);
  const int nk = kend > kbeg ? (kend - kbeg + KS - 1) / KS : 0;
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wid >> 1, wc = wid & 1;

  OA oa;
  OB ob;
  oa.init(la, m0, wid, lane, wr);
  ob.init(lb, n0, wid, lane, wc);
  const __amdgpu_buffer_rsrc_t ra = la.rsrc(), rb = lb.rsrc();

  f32x4 acc[MI][NI];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // DMA wave-instruction d (< ND) of a tile into the stage at `stg`
  auto dma = [&](auto dc, char* stg, const typename LA::Prep& pa, const typename LB::Prep& pb) {
    constexpr int d = decltype(dc)::value;
    if constexpr (d < NDA) {
      constexpr int h = d / OA::I, i = d % OA::I;
      dma16(ra, stg + oa.seg[h][i], la.offs(oa.ctx[h][i], pa, oa.kofs[h][i]));
    } else {
      constexpr int h = (d - NDA) / OB::I, i = (d - NDA) % OB::I;
      dma16(rb, stg + OA::TB + ob.seg[h][i], lb.offs(ob.ctx[h][i], pb, ob.kofs[h][i]));
    }
  };
  auto dma_tile = [&](int t, int buf) {
    const typename LA::Prep pa = la.prep(kbeg + t * KS);
    const typename LB::Prep pb = lb.prep(kbeg + t * KS);
    sfor<ND>([&](auto dc) { dma(dc, smem + buf * STAGE, pa, pb); });
  };
  // fragment r (< NR: A rows, then B columns) of k sub-step KK from the stage at As
  auto read_one = [&](auto rc, auto kkc, const char* As, bf16x8 (&af)[MI], bf16x8 (&bfr)[NI]) {
    constexpr int r = decltype(rc)::value, KK = decltype(kkc)::value;
    const char* Bs = As + OA::TB;
    if constexpr (r < MI) {
      load_kk<OA, r / MQ, 1, KK, r % MQ>(oa, af + r, As, lds_addr(As), wr * WM, lane);
    } else {
      constexpr int rr = r - MI;
      load_kk<OB, rr / NQ, 1, KK, rr % NQ>(ob, bfr + rr, Bs, lds_addr(Bs), wc * WN, lane);
    }
  };

  bf16x8 a0[MI], b0[NI], a1[MI], b1[NI];
  if (nk > 0) {
    dma_tile(0, 0);
    dma_tile(min(1, nk - 1), 1);
    asm volatile("s_waitcnt vmcnt(%0)" ::"i"(ND) : "memory");   // tile 0 landed
    raw_barrier();
    const char* As = smem;
    sfor<NR>([&](auto rc) { read_one(rc, std::integral_constant<int, 0>{}, As, a0, b0); });
  }
  // Past the last K-tile the DMA re-fetches tile nk-1 into the stage nobody reads again and the
  // reads of F0(nk) fill registers nobody uses: no runtime guard inside the MFMA stream.
  auto ktile = [&](auto fmc, int t) {
    constexpr uint32_t FM = decltype(fmc)::value;
    const int b = t & 1;
    lds_wait_all_known();                               // F0(t) in registers
    const int kn = kbeg + min(t + 2, nk - 1) * KS;
    const typename LA::Prep pa = la.prep(kn);
    const typename LB::Prep pb = lb.prep(kn);
    const char* As = smem + b * STAGE;
    const char* As1 = smem + (b ^ 1) * STAGE;
    char* st = smem + b * STAGE;
    __builtin_amdgcn_s_setprio(1);
    sfor<S>([&](auto mc) {
      constexpr int m = decltype(mc)::value;
      constexpr int mm = m < NM ? m : m - NM, i = mm / NI, j = mm % NI;
      if constexpr ((FM >> i) & 1u) {
        if constexpr (m < NM)
          asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc[i][j]) : "v"(b0[j]), "v"(a0[i]));
        else
          asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc[i][j]) : "v"(b1[j]), "v"(a1[i]));
      }
      if constexpr (m < NR) read_one(std::integral_constant<int, m>{}, std::integral_constant<int, 1>{}, As, a1, b1);
      if constexpr (m == B1) {
        lds_wait_all_known();                           // F1(t) in registers: done with stage b
        raw_barrier();
      }
      sfor<ND>([&](auto dc) {
        constexpr int d = decltype(dc)::value;
        if constexpr (m == B1 + d * (V - B1) / ND) dma(dc, st, pa, pb);
      });
      if constexpr (m == V) {
        asm volatile("s_waitcnt vmcnt(%0)" ::"i"(ND) : "memory");   // tile t+1 landed (this wave)
        raw_barrier();                                                // ... for every wave
      }
      if constexpr (m >= V && m < V + NR)
        read_one(std::integral_constant<int, m - V>{}, std::integral_constant<int, 0>{}, As1, a0, b0);
      __builtin_amdgcn_sched_barrier(0);
    });
    __builtin_amdgcn_s_setprio(0);
  };
  // asm MFMAs are invisible to hipcc's hazard padding: the accumulator zeroing must be 2+ wait
  // states ahead of the first MFMA reading it
  asm volatile("s_nop 4" ::);
  __builtin_amdgcn_sched_barrier(0);
  if constexpr (SKIP == 0) {
    for (int t = 0; t < nk; ++t) ktile(std::integral_constant<uint32_t, 0xffu>{}, t);
  } else {   // gemm256_item: compile-time padding-row segments of 4-row maps
    constexpr uint32_t M0 = SKIP == 1 ? 0xfcu : 0x3fu, M2 = SKIP == 1 ? 0x3fu : 0xfcu;
    const int e0 = min(nk, ktk), e1 = min(nk, 2 * ktk);
    int t = 0;
    for (; t < e0; ++t) ktile(std::integral_constant<uint32_t, M0>{}, t);
    for (; t < e1; ++t) ktile(std::integral_constant<uint32_t, 0xffu>{}, t);
    for (; t < nk; ++t) ktile(std::integral_constant<uint32_t, M2>{}, t);
  }
  // The F0(nk) reads past the last K-tile are asm LDS loads (trd / frag), which hipcc neither counts nor
  // keeps live: their registers are dead after the loop, so hipcc reused them for the epilogue's LDS
  // addresses while the reads were still in flight, and a late LDS return (a co-resident workgroup
  // slows the LDS) overwrote the address — the r05 co-scheduled wgrad mismatch (found by
  // tools/asm_hazard_scan.py "pending"). Wait for them here with every F0 register named as an operand,
  // so none is reused before the data has landed.
  asm volatile("s_waitcnt lgkmcnt(0)"
               : "+v"(a0[0]), "+v"(a0[1]), "+v"(a0[2]), "+v"(a0[3]), "+v"(a0[4]), "+v"(a0[5]), "+v"(a0[6]),
                 "+v"(a0[7]));
  if constexpr (NI == 8)
    asm volatile("" : "+v"(b0[0]), "+v"(b0[1]), "+v"(b0[2]), "+v"(b0[3]), "+v"(b0[4]), "+v"(b0[5]), "+v"(b0[6]),
                 "+v"(b0[7]));
  else
    asm volatile("" : "+v"(b0[0]), "+v"(b0[1]), "+v"(b0[2]), "+v"(b0[3]));
  // ... and the last MFMA's result 11+ wait states (8-pass XDL) ahead of its first VALU / LDS read
  asm volatile("s_nop 15\n\ts_nop 15" ::);
  __builtin_amdgcn_sched_barrier(0);

  const int mr = lane & 15, nq = 4 * (lane >> 4);
  if constexpr (!EPI::kStats && !has_tile_hook<EPI>::value) {
    // through wave-private LDS (MI/2 fragment rows at a time): a rolled store loop instead of an
    // unrolled epilogue over 64 register fragments, whose pressure would spill the accumulators
    constexpr int RH = MI / 2;
    static_assert(NW * RH * NI * 64 * 16 <= 2 * STAGE, "epilogue LDS");
    f32x4* ws = reinterpret_cast<f32x4*>(smem) + wid * RH * NI * 64 + lane;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the re-fetch DMA past the last K-tile
    lds_wait_all_known();
    raw_barrier();                                      // every wave is done with the operand tiles
#pragma unroll
    for (int h = 0; h < 2; ++h) {
#pragma unroll
      for (int i = 0; i < RH; ++i)
#pragma unroll
        for (int j = 0; j < NI; ++j) ws[(i * NI + j) * 64] = acc[h * RH + i][j];
#pragma unroll 1
      for (int f = 0; f < RH * NI; ++f) {
        const f32x4 v = ws[f * 64];
        const int i = h * RH + f / NI, j = f % NI;
        epi.store(m0 + wr * WM + i * 16 + mr, n0 + wc * WN + j * 16 + nq, v, kz);
      }
    }
    return;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j) epi.store(m0 + wr * WM + i * 16 + mr, n0 + wc * WN + j * 16 + nq, acc[i][j], kz);
  if constexpr (EPI::kStats) wave_col_stats<MI, NI>(acc, epi, M, m0 + wr * WM, m_tile * 2 + wr, n0 + wc * WN, lane);
  if constexpr (has_tile_hook<EPI>::value) epi.template tile<MI, NI>(acc, M, m0 + wr * WM, m_tile * 2 + wr, n0 + wc * WN, lane);
}

template <int BM, int BN, int SKIP, class LA, class LB, class EPI>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1))) void gemm4w_kernel(
    LA la, LB lb, EPI epi, int M, int N, int K, int klen, int tiles_m, int tiles_n, int nsplit, int nbatch, int ktk) {
  const int nwg = tiles_m * tiles_n * nsplit * nbatch;
  const int wg = xcd_remap(blockIdx.x, nwg);
  int n_tile = wg % tiles_n, m_tile = (wg / tiles_n) % tiles_m;
  const int kz = (wg / (tiles_n * tiles_m)) % nsplit;
  if constexpr (GEMM_GROUP_M > 0) {   // grouped tile order: GEMM_GROUP_M m-tiles share each n sweep (L2 reuse)
    const int pid = wg % (tiles_n * tiles_m), per = GEMM_GROUP_M * tiles_n, g0 = (pid / per) * GEMM_GROUP_M;
    const int gs = min(tiles_m - g0, GEMM_GROUP_M);
    m_tile = g0 + (pid % per) % gs;
    n_tile = (pid % per) / gs;
  }
  if (nbatch > 1) {
    const int bz = wg / (tiles_n * tiles_m * nsplit);
    if constexpr (has_set_batch<LA>::value) la.set_batch(bz);
    if constexpr (has_set_batch<LB>::value) lb.set_batch(bz);
    if constexpr (has_set_batch<EPI>::value) epi.set_batch(bz);
  }
  gemm4w_item<BM, BN, SKIP>(la, lb, epi, M, K, klen, m_tile, n_tile, kz, ktk);
}

// nsplit: split-K factor (K ranges of split_len(K, nsplit), multiples of 64)
// nbatch: independent GEMMs of one shape in one launch (loaders / epilogue with set_batch(int))
// SKIP (1: conv fwd, 2: stride-1 dgrad, 3x3 over 4-row maps of 128 pixels; nsplit 1): the
// padding-row fragment skip of gemm256_item, ktk = K-tiles per kernel row
template <int BM, int BN, int SKIP = 0, class LA, class LB, class EPI>
inline int launch256(const LA& la, const LB& lb, const EPI& epi, int M, int N, int K, hipStream_t st,
                     int nsplit = 1, int nbatch = 1, int ktk = 0) {
  if (M <= 0 || N <= 0) return 0;
  const int tm = (M + BM - 1) / BM, tn = (N + BN - 1) / BN;
  const int klen = split_len(K, nsplit);
  nsplit = K > 0 ? (K + klen - 1) / klen : 1;
  const int items = tm * tn * nsplit * nbatch;
  const int f4 = crnn_option(CRNN_OPT_GEMM4W);
  if (f4 == 1 || (f4 & ~1 & prefers_4w<EPI>::value) != 0) {
    hipLaunchKernelGGL((gemm4w_kernel<BM, BN, SKIP, LA, LB, EPI>), dim3(items), dim3(256), 0, st, la, lb, epi, M, N, K,
                       klen, tm, tn, nsplit, nbatch, ktk);
    return (int)hipGetLastError();
  }
    hipLaunchKernelGGL((gemm256_kernel<BM, BN, SKIP, LA, LB, EPI>), dim3(items), dim3(512), 0, st, la, lb, epi,
                       M, N, K, klen, tm, tn, nsplit, crnn_option(CRNN_OPT_GEMM_STAGGER), nbatch, ktk);
  return (int)hipGetLastError();
}

}  // namespace gemm
