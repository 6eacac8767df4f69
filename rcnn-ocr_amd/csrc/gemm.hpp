// MFMA GEMM core for the CRNN path (gfx950).
//
//   C[m][n] = sum_k A(m,k) * B(n,k)        fp32 accumulate, T in {float, bf16}
//
// A and B are produced by *loaders* that fetch 8 elements at a time from global
// memory in whichever direction is contiguous there:
//   kRowVec = false : elements (row, k..k+7)    ("K-contiguous")
//   kRowVec = true  : elements (row8..row8+7, k) ("row-contiguous")
// Loader interface: Ctx row_ctx(row) once per thread and staged row (row offsets, masks);
// Prep prep(k0) once per pipeline stage (wave-uniform: lands in SALU); and
// v8 load(ctx, prep, kofs) for k = k0 + kofs — a range-checked buffer load.
// and stage them to LDS in that same orientation. Fragments for the MFMA are
// then read K-contiguous (ds_read_b64/b128) or transposed (gfx950
// ds_read_b64_tr_b16), so implicit-GEMM conv fwd (im2col rows), conv dgrad
// (transposed weights read from OHWI without a copy), conv wgrad (reduction
// over output pixels) and the LSTM/linear products all share one kernel.
//
// Tiling: 256 threads = 4 waves as 2(M) x 2(N); a block owns BM x BN, each wave
// (BM/2) x (BN/2) as 16x16 MFMA tiles. BK = 32 (one bf16 16x16x32 MFMA, or
// eight exact-f32 16x16x4 MFMAs, per tile per K-step). LDS is double-buffered
// with one barrier per K-step; the global loads for step k+1 are issued before
// step k's MFMAs so their latency hides under them.
//
// The MFMA is issued "swapped" (B-fragment as the MFMA A operand), so each lane
// ends up holding 4 CONSECUTIVE output columns n..n+3 of one row m: epilogues
// store 8/16 B per lane and LSTM gate quadruples (i,f,g,o interleaved) land in
// one lane.
#pragma once
#include <type_traits>
#include <utility>
#include "common.hpp"

namespace gemm {

// optional batch hook: loaders / epilogues with set_batch(int) are re-targeted per batch entry
template <class X, class = void> struct has_set_batch : std::false_type {};
template <class X>
struct has_set_batch<X, std::void_t<decltype(std::declval<X&>().set_batch(0))>> : std::true_type {};

// two parameter sets (e.g. the two LSTM directions) of one loader type, selected per batch
template <class L> struct Pair {
  static constexpr bool kRowVec = L::kRowVec;
  using Ctx = typename L::Ctx;
  using Prep = decltype(std::declval<const L&>().prep(0));
  L a, b;
  __device__ __forceinline__ void set_batch(int bz) {
    if (bz) a = b;
  }
  __device__ __forceinline__ Ctx row_ctx(int r) const { return a.row_ctx(r); }
  __device__ __forceinline__ Prep prep(int k0) const { return a.prep(k0); }
  __device__ __forceinline__ auto load(const Ctx& c, const Prep& p, int kofs) const { return a.load(c, p, kofs); }
  __device__ __forceinline__ auto rsrc() const { return a.rsrc(); }
  __device__ __forceinline__ auto offs(const Ctx& c, const Prep& p, int kofs) const { return a.offs(c, p, kofs); }
};
template <class E> struct EpiPair {
  static constexpr bool kStats = E::kStats;
  E a, b;
  __device__ __forceinline__ void set_batch(int bz) {
    if (bz) a = b;
  }
  __device__ __forceinline__ void store(int m, int n, f32x4 v, int kz) const { a.store(m, n, v, kz); }
  __device__ __forceinline__ void stats(int r, int n, f32x4 s, f32x4 q) const { a.stats(r, n, s, q); }
};

constexpr int BK = 32;  // K per MFMA sub-step; a pipeline stage holds KS = 32 or 64 (128 / 256: linear.hip run_mix)
constexpr int NT = 256;

// K-contiguous tiles: bf16 rows are unpadded (KS elements) with the 16-byte chunks XOR-swizzled
// per row (swz below) so every ds_read_b128 lane group hits 16 distinct 16-B bank slots;
// f32 rows (parity mode) are padded by 16 B instead.
template <typename T, int KS = BK> constexpr int kpitch() { return sizeof(T) == 2 ? KS : KS + (int)(16 / sizeof(T)); }

// physical 16-byte chunk of logical chunk c in row r (bf16 K-contiguous tiles)
template <typename T, int KS> __device__ __forceinline__ int swz(int r, int c) {
  if constexpr (sizeof(T) != 2) return c;
  else if constexpr (KS >= 64) return c ^ ((r >> 1) & 7);
  else {
    const int q = (r >> 2) & 3;
    return c ^ (q == 1 ? 3 : (q == 3 ? 1 : q));  // h = {0,3,2,1}
  }
}
// row-contiguous pitch: 32*odd bytes for bf16 (conflict-free ds_read_b64_tr_b16
// over 8 k-rows), (R+4) floats for f32 (conflict-free strided ds_read_b32)
template <typename T, int R> constexpr int rpitch() { return sizeof(T) == 2 ? R + 16 : R + 4; }
template <typename T, int R, bool RowVec, int KS = BK> constexpr int tile_elems() {
  return RowVec ? KS * rpitch<T, R>() : R * kpitch<T, KS>();
}

// k index held by element j of a lane in 16-lane group g.
//  PERM=false: k = 8g + j (one 16-B K-contiguous read)
//  PERM=true : k = 4g + j (j<4) / 16 + 4g + (j-4) (j>=4) — two 4-row blocks a
//              transposed read can fetch; both operands must use the same map.
template <bool PERM> __device__ __forceinline__ int kmap(int g, int j) {
  if constexpr (PERM) return j < 4 ? 4 * g + j : 16 + 4 * g + (j - 4);
  else return 8 * g + j;
}

template <typename T, int R, int KS, class L> struct Stager {
  static constexpr bool RV = L::kRowVec;
  static constexpr int ITEMS = R * KS / 8;
  static constexpr int PT = ITEMS >= NT ? ITEMS / NT : 1;
  static constexpr bool PARTIAL = ITEMS < NT;  // small tiles: only the first ITEMS threads stage
  static_assert(ITEMS < NT || ITEMS % NT == 0, "tile/thread mismatch");
  typename L::Ctx ctx[PT];
  int lds_off[PT];
  int kofs[PT];
  bool act;
  typename VT<T>::v8 reg[PT];

  __device__ __forceinline__ void init(const L& l, int row0, int tid) {
    act = !PARTIAL || tid < ITEMS;
#pragma unroll
    for (int j = 0; j < PT; ++j) {
      int i = act ? tid + j * NT : 0;
      if constexpr (RV) {
        int k = i / (R / 8), r8 = (i % (R / 8)) * 8;
        ctx[j] = l.row_ctx(row0 + r8);
        lds_off[j] = k * rpitch<T, R>() + r8;
        kofs[j] = k;
      } else {
        int r = i / (KS / 8), kg = i % (KS / 8);
        ctx[j] = l.row_ctx(row0 + r);
        lds_off[j] = r * kpitch<T, KS>() + swz<T, KS>(r, kg) * 8;
        kofs[j] = kg * 8;
      }
    }
  }
  __device__ __forceinline__ void load(const L& l, int k0) {
    if (!act) return;
    const auto pr = l.prep(k0);
#pragma unroll
    for (int j = 0; j < PT; ++j) reg[j] = l.load(ctx[j], pr, kofs[j]);
  }
  __device__ __forceinline__ void store(T* tile) {
    if (!act) return;
#pragma unroll
    for (int j = 0; j < PT; ++j) st8<T>(tile + lds_off[j], reg[j]);
  }
};

// Fragment of 16 MFMA rows [rb, rb+16) x 32 k for this lane.
// kk: which 32-deep MFMA sub-step of the KS-deep stage
template <typename T, int R, bool RV, bool PERM, int KS>
__device__ __forceinline__ typename VT<T>::v8 frag(const T* tile, int rb, int kk, int lane) {
  typename VT<T>::v8 v;
  const int g = lane >> 4, c = lane & 15;
  if constexpr (!RV) {
    const int row = rb + c;
    const T* p = tile + row * kpitch<T, KS>();
    if constexpr (!PERM) {
      v = *reinterpret_cast<const typename VT<T>::v8*>(p + swz<T, KS>(row, kk * 4 + g) * 8);
    } else {
      // k = 4g..4g+3 and 16+4g..: halves of chunks kk*4 + g/2 and kk*4 + 2 + g/2
      const int h = (g & 1) * 4;
      typename VT<T>::v4 lo = *reinterpret_cast<const typename VT<T>::v4*>(p + swz<T, KS>(row, kk * 4 + (g >> 1)) * 8 + h);
      typename VT<T>::v4 hi = *reinterpret_cast<const typename VT<T>::v4*>(p + swz<T, KS>(row, kk * 4 + 2 + (g >> 1)) * 8 + h);
      v[0] = lo[0]; v[1] = lo[1]; v[2] = lo[2]; v[3] = lo[3];
      v[4] = hi[0]; v[5] = hi[1]; v[6] = hi[2]; v[7] = hi[3];
    }
  } else {
    static_assert(PERM, "row-contiguous tiles need the transposed-read k map");
    if constexpr (sizeof(T) == 2) {
      const int q = c >> 2, p = c & 3;
      typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
      const T* a0 = tile + (kk * BK + 4 * g + q) * rpitch<T, R>() + rb + 4 * p;
      const T* a1 = tile + (kk * BK + 16 + 4 * g + q) * rpitch<T, R>() + rb + 4 * p;
      s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a0));
      s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a1));
      s16x4 tmp[2] = {lo, hi};
      v = *reinterpret_cast<const bf16x8*>(tmp);
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = tile[(kk * BK + kmap<true>(g, j)) * rpitch<T, R>() + rb + c];
    }
  }
  return v;
}

template <typename T>
__device__ __forceinline__ void mma(f32x4& acc, const typename VT<T>::v8& a, const typename VT<T>::v8& b) {
  if constexpr (sizeof(T) == 2) {
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc, 0, 0, 0);
  } else {
#pragma unroll
    for (int j = 0; j < 8; ++j) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[j], b[j], acc, 0, 0, 0);
  }
}

template <typename T, int BM, int BN, int KS, class LA, class LB, class EPI>
__global__ __launch_bounds__(256) void gemm_kernel(LA la, LB lb, EPI epi, int M, int N, int K,
                                                   int klen, int tiles_m, int tiles_n, int nsplit, int nbatch) {
  constexpr bool PERM = LA::kRowVec || LB::kRowVec;
  constexpr int WM = BM / 2, WN = BN / 2, MI = WM / 16, NI = WN / 16;
  constexpr int AE = tile_elems<T, BM, LA::kRowVec, KS>();
  constexpr int BE = tile_elems<T, BN, LB::kRowVec, KS>();
  __shared__ __attribute__((aligned(16))) T smem[2 * (AE + BE)];

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
  const int nk = kend > kbeg ? (kend - kbeg + KS - 1) / KS : 0;

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;

  Stager<T, BM, KS, LA> sa;
  Stager<T, BN, KS, LB> sb;
  sa.init(la, m0, tid);
  sb.init(lb, n0, tid);

  f32x4 acc[MI][NI];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  T* As0 = smem;
  T* Bs0 = smem + AE;
  T* As1 = smem + AE + BE;
  T* Bs1 = smem + 2 * AE + BE;

  if (nk > 0) {
    sa.load(la, kbeg);
    sb.load(lb, kbeg);
    sa.store(As0);
    sb.store(Bs0);
  }
  __syncthreads();

  for (int kt = 0; kt < nk; ++kt) {
    const bool more = kt + 1 < nk;
    const T* Ac = (kt & 1) ? As1 : As0;
    const T* Bc = (kt & 1) ? Bs1 : Bs0;
    if (more) {
      sa.load(la, kbeg + (kt + 1) * KS);
      sb.load(lb, kbeg + (kt + 1) * KS);
    }
#pragma unroll
    for (int kk = 0; kk < KS / BK; ++kk) {
      typename VT<T>::v8 af[MI], bfr[NI];
#pragma unroll
      for (int i = 0; i < MI; ++i) af[i] = frag<T, BM, LA::kRowVec, PERM, KS>(Ac, wm * WM + i * 16, kk, lane);
#pragma unroll
      for (int j = 0; j < NI; ++j) bfr[j] = frag<T, BN, LB::kRowVec, PERM, KS>(Bc, wn * WN + j * 16, kk, lane);
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NI; ++j) mma<T>(acc[i][j], bfr[j], af[i]);
    }
    if (more) {
      sa.store((kt & 1) ? As0 : As1);
      sb.store((kt & 1) ? Bs0 : Bs1);
    }
    __syncthreads();
  }

  const int mr = lane & 15, nq = 4 * (lane >> 4);
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j)
      epi.store(m0 + wm * WM + i * 16 + mr, n0 + wn * WN + j * 16 + nq, acc[i][j], kz);

  if constexpr (EPI::kStats) {
    // per-column partial statistics over this wave's WM rows, two-pass in registers:
    // s = sum, q = sum (x - s/n)^2 over the n = rows < M (no E[x^2]-E[x]^2 cancellation);
    // crnn_bn_finalize combines the partials with Chan's formula in double.
    const int rbase = m0 + wm * WM;
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
      if (mr == 0) epi.stats(m_tile * 2 + wm, n0 + wn * WN + j * 16 + nq, s, q);
    }
  }
}

// K splits are whole multiples of 64 so that both stage depths tile them exactly
constexpr int KSPLIT_Q = 64;

inline int split_len(int K, int nsplit) {
  if (nsplit < 1) nsplit = 1;
  int klen = ((K + nsplit - 1) / nsplit + KSPLIT_Q - 1) / KSPLIT_Q * KSPLIT_Q;
  return klen < KSPLIT_Q ? KSPLIT_Q : klen;
}

// number of K splits the launcher will actually use
inline int eff_splits(int K, int nsplit) {
  int klen = split_len(K, nsplit);
  return K > 0 ? (K + klen - 1) / klen : 1;
}

// default pipeline stage depth: 64 for bf16 (one barrier per two MFMA K-steps), 32 for the
// f32 parity mode (its exact-f32 MFMA is 16x slower; LDS stays small)
template <typename T> constexpr int kstage() { return sizeof(T) == 2 ? 64 : 32; }

template <typename T, int BM, int BN, int KS = kstage<T>(), class LA, class LB, class EPI>
inline int launch(const LA& la, const LB& lb, const EPI& epi, int M, int N, int K, int nsplit,
                  hipStream_t st, int nbatch = 1) {
  if (M <= 0 || N <= 0) return 0;
  const int tm = (M + BM - 1) / BM, tn = (N + BN - 1) / BN;
  const int klen = split_len(K, nsplit);
  nsplit = K > 0 ? (K + klen - 1) / klen : 1;
  const int nwg = tm * tn * nsplit * nbatch;
  hipLaunchKernelGGL((gemm_kernel<T, BM, BN, KS, LA, LB, EPI>), dim3(nwg), dim3(NT), 0, st, la, lb, epi,
                     M, N, K, klen, tm, tn, nsplit, nbatch);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------- simple loaders
// Row-major matrix, K-contiguous: element (row, k) at p[row*ld + k]; rows, K bounds.
template <typename T> struct RowMajorK {
  static constexpr bool kRowVec = false;
  const T* p;
  int ld, rows, K;
  struct Ctx { uint32_t off; bool ok; };
  typedef int Prep;
  __device__ __forceinline__ Ctx row_ctx(int r) const { return Ctx{(uint32_t)r * (uint32_t)ld, r < rows}; }
  __device__ __forceinline__ Prep prep(int k0) const { return k0; }
  __device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc() const { return mk_rsrc(p, bytes()); }
  __device__ __forceinline__ uint32_t offs(const Ctx& c, Prep k0, int kofs) const {
    const int k = k0 + kofs;
    return boff<T>(c.off + k, c.ok && k < K);
  }
  __device__ __forceinline__ typename VT<T>::v8 load(const Ctx& c, Prep k0, int kofs) const {
    return bld8<T>(rsrc(), offs(c, k0, kofs));
  }
  __device__ __forceinline__ uint32_t bytes() const { return (uint32_t)((size_t)(rows > 0 ? rows : 1) * ld * sizeof(T)); }
};

// Row-contiguous view: element (row, k) at p[k*ld + row] (8 rows per vector); rows % 8 == 0.
template <typename T> struct ColMajorK {
  static constexpr bool kRowVec = true;
  const T* p;
  int ld, rows, K;
  struct Ctx { uint32_t off; bool ok; };
  typedef int Prep;
  __device__ __forceinline__ Ctx row_ctx(int r8) const { return Ctx{(uint32_t)r8, r8 < rows}; }
  __device__ __forceinline__ Prep prep(int k0) const { return k0; }
  __device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc() const {
    return mk_rsrc(p, (uint32_t)((size_t)K * ld * sizeof(T)));
  }
  __device__ __forceinline__ uint32_t offs(const Ctx& c, Prep k0, int kofs) const {
    const int k = k0 + kofs;
    return boff<T>((uint32_t)k * (uint32_t)ld + c.off, c.ok && k < K);
  }
  __device__ __forceinline__ typename VT<T>::v8 load(const Ctx& c, Prep k0, int kofs) const {
    return bld8<T>(rsrc(), offs(c, k0, kofs));
  }
};

// fp32 operands staged as bf16 (CRNN_F32_BF16MMA: the attention decoder's training GEMMs, fp32 in memory and
// bf16 MFMA with fp32 accumulation, as the reference's fp16 autocast computes them): the register-staged
// kernels' loaders convert 8 fp32 elements to bf16 on the way to LDS. No LDS-DMA form (nothing to convert
// with), so these views run only on gemm_kernel.
template <class L32> struct Bf16Of {
  static constexpr bool kRowVec = L32::kRowVec;
  using Ctx = typename L32::Ctx;
  typedef int Prep;
  L32 l;
  __device__ __forceinline__ Ctx row_ctx(int r) const { return l.row_ctx(r); }
  __device__ __forceinline__ Prep prep(int k0) const { return k0; }
  __device__ __forceinline__ bf16x8 load(const Ctx& c, Prep k0, int kofs) const {
    const f32x8 v = l.load(c, k0, kofs);
    return bf16x8{(bf16)v[0], (bf16)v[1], (bf16)v[2], (bf16)v[3], (bf16)v[4], (bf16)v[5], (bf16)v[6], (bf16)v[7]};
  }
};

}  // namespace gemm
