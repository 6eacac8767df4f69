// Persistent BiLSTM recurrence (bf16): the whole T-step sweep of one layer — forward recurrence
// or BPTT — in ONE launch, both directions, W_hh resident in registers for all T steps.
// Reference: nn.LSTM(in, H, bidirectional=True, batch_first=True), model/model.py:152-163
// (gate order i,f,g,o; h0 = c0 = 0); the per-step kernels in lstm.hip compute the same thing
// one launch per step (and remain the fp32 / unsupported-shape path).
//
// Decomposition (B = batch, H = hidden, T = steps): one workgroup per
//   (direction d, batch slice bs of S samples, unit slice ns of U units), S x U = 16 x 64,
// 16 x 32 or 32 x 32 (seq_config), 2 * (B/S) * (H/U) workgroups, 4 waves each, at most one per CU (all must be co-resident:
// the host checks the grid against the CU count). The step GEMM's K is split over the 4 waves
// (each wave holds its K-quarter of the W_hh slice as MFMA fragments in VGPRs, loaded once), the
// four partial tiles are summed through LDS, and the cell math runs on the summed tile.
//
//   forward  step: gates[b][4u+q] = xg[b][t][d][4u+q] + sum_k h_{t-1}[b][k] W_hh'[4u+q][k]
//                  (W_hh' = gate-interleaved packing, lstm.hip) -> c, h; saves gates, c for BPTT
//   BPTT     step: dh_rec[b][u]   = sum_g dgates_{t'}[b][g] W_hh'[g][u]   (t' = the step before)
//                  -> cell backward -> dgates_t (and the running dc, kept in registers)
//
// Per-step hand-off (cdna_hip_programming.md Guideline 16, MI355X_MICROARCH.md "Valid forms",
// first table row): the only data crossing workgroups are h_t (forward) / dgates_t (BPTT) of a
// batch slice, consumed by the 16..24 workgroups of the same (d, bs). Producers store them with
// write-through (sc1) 16-B stores, every storing wave drains vmcnt(0), the workgroup barriers,
// then ONE lane adds 1 (agent scope) to the slice's counter. A consumer's wave 0 polls that
// counter with sc1 loads until it reaches (unit slices) x (steps done), the workgroup barriers,
// and every load of the handed-off bytes is an sc1 buffer load to registers. Counters are zeroed
// by a memset in the launch function. Every spin is bounded: on time-out the kernel records an
// error word (ws[2*(B/16+1)], see include/crnn_hip.h) and the step's outputs carry NaN.
#include "gemm.hpp"
#include "crnn_internal.hpp"

using namespace gemm;

namespace {

typedef bf16 bf16x2_t __attribute__((ext_vector_type(2)));
typedef unsigned int u32x2_t __attribute__((ext_vector_type(2)));

constexpr unsigned long long SEQ_TIMEOUT_TICKS = 50000000ull;  // s_memrealtime @100 MHz: 0.5 s per wait

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc_of(const void* p) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, 0x7fffffff, 0x00020000);
}
// write-through (sc1) 16-B load / store: the hand-off's only access kinds for shared bytes
__device__ __forceinline__ bf16x8 ld_sc1(__amdgpu_buffer_rsrc_t r, uint32_t byteoff) {
  return __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(r, byteoff, 0, 16));
}
__device__ __forceinline__ void st_sc1(__amdgpu_buffer_rsrc_t r, uint32_t byteoff, bf16x8 v) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), r, byteoff, 0, 16);
}

// one lane: wait until *cnt >= target (relaxed agent-scope sc1 polls, s_sleep between polls)
__device__ __noinline__ bool seq_wait(unsigned* cnt, unsigned target, unsigned* err) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  while (__hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
    if (__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return false;
    if (__builtin_amdgcn_s_memrealtime() - t0 > SEQ_TIMEOUT_TICKS) {
      __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return false;
    }
    __builtin_amdgcn_s_sleep(2);
  }
  return true;
}

// every storing wave drains its stores, the workgroup joins, one lane signals
__device__ __forceinline__ void seq_publish(unsigned* cnt) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// optional per-phase timestamps (s_memrealtime, 10 ns) of workgroup `id`, step s: stamps[(id*T+s)*8+p]
#define SEQ_STAMP(p)                                                                              \
  if (stamps && threadIdx.x == 0) stamps[((size_t)blockIdx.x * Tn + s) * 8 + (p)] = __builtin_amdgcn_s_memrealtime()

__device__ __forceinline__ void seq_coords(int nsl, int nbs, int& d, int& bs, int& ns) {
  // logical id = (d * nbs + bs) * nsl + ns; xcd_remap keeps a (d, bs) group's workgroups together
  const int nwg = 2 * nbs * nsl;
  const int id = xcd_remap(blockIdx.x, nwg);
  ns = id % nsl;
  bs = (id / nsl) % nbs;
  d = id / (nsl * nbs);
}

// XCD-local hand-off (CRNN_OPT_LSTM_L2_HANDOFF = 1, default): true when every workgroup of this
// (d, bs) group runs on this workgroup's XCD. Each workgroup's lane 0 publishes its XCC id
// (HW_REG_XCC_ID + 1, relaxed agent-scope store) into a per-launch table (zeroed with the counters)
// and polls its group's entries. HIP promises no placement, so it is checked, never assumed: on one
// XCD the group's hand-off payload may be written with plain stores that keep the lines in that
// XCD's L2, where the consumers' sc1 loads (L1-bypassing, L2-served) find them — an sc1 store drops
// the line from L2 and makes every consumer read at the cross-XCD rate (MI355X_MICROARCH.md,
// inter-workgroup visibility). Split groups keep the sc1 stores. Bounded wait (error word).
__device__ __noinline__ bool seq_group_local(unsigned* tab, int gbase, int nsl, int ns, unsigned* err) {
  __shared__ int flag;
  if (threadIdx.x == 0) {
    unsigned x;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
    x = (x & 15u) + 1u;
    __hip_atomic_store(tab + gbase + ns, x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    bool same = true;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    for (int p = 0; p < nsl && same; ++p) {
      unsigned v;
      while ((v = __hip_atomic_load(tab + gbase + p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) == 0u) {
        if (__builtin_amdgcn_s_memrealtime() - t0 > SEQ_TIMEOUT_TICKS) {
          __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
      same = v == x;
    }
    flag = same ? 1 : 0;
  }
  __syncthreads();
  return flag != 0;
}

// ---------------------------------------------------------------- forward sweep
// Workgroup = (direction, S samples, U units = 4U gate rows); wave w holds the K-quarter
// [w*H/4, (w+1)*H/4) of the W_hh' slice (NJ = 4U/16 row fragments x KK k-steps) in VGPRs and
// computes an S x 4U partial tile; the partials are summed through LDS and wave w finalises the
// fragment blocks bi = w*QB .. w*QB+QB-1 (QB = MI*NJ/4), bi -> (i = bi / NJ, j = bi % NJ).
//
// TAG = true (the default, CRNN_OPT_LSTM_HANDOFF = 1): h_t travels as data-tagged 8-byte granules
// {2 bf16 of h, u32 tag = step + 1} in a 2-slot ring (slot = step & 1, zeroed per launch), written
// by 16-B sc1 stores (two granules each) and read by 16-B sc1 loads that each wave re-issues until
// every tag it loaded matches (MI355X_MICROARCH.md price list, handoff-1to1 vs handoff-flag: no
// vmcnt drain, barrier, counter add or poll on the critical path). Two slots suffice: a producer
// writes slot s & 1 again at step s + 2 only after it has read h_{s+1} of every workgroup of its
// group, each of which was computed after that workgroup's loads of h_s had returned.
// TAG = false: the write-through payload + drained counter hand-off described at the top.
template <int H, int S, int U, bool TAG>
__global__ __launch_bounds__(256) void lstm_seq_fwd_kernel(const bf16* __restrict__ xg, const bf16* __restrict__ whh,
                                                           bf16* hseq, bf16* __restrict__ gsv, float* __restrict__ csv,
                                                           unsigned* cnt, unsigned* err, uint2* ring, int B, int Tn,
                                                           unsigned long long* stamps, unsigned* xtab) {
  constexpr int KW = H / 4, KK = KW / 32;
  constexpr int GR = 4 * U, NJ = GR / 16, MI = S / 16;
  constexpr int QB = MI * NJ / 4;   // blocks finalised per wave
  constexpr int H4 = 4 * H;
  static_assert(H % 128 == 0 && S % 16 == 0 && U % 16 == 0 && (MI * NJ) % 4 == 0, "shape");
  static_assert(S * U / 8 <= 256 && S * U / 4 <= 256, "publish: one 16-B store per thread");
  __shared__ __attribute__((aligned(16))) f32x4 part[4][MI][NJ][64];
  __shared__ __attribute__((aligned(16))) bf16 htile[S][U];

  const int nsl = H / U, nbs = B / S;
  int d, bs, ns;
  seq_coords(nsl, nbs, d, bs, ns);
  const int lane = threadIdx.x & 63, c = lane & 15, g = lane >> 4;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int b0 = bs * S, n0 = ns * GR;
  unsigned* mycnt = cnt + d * nbs + bs;
  if (stamps && threadIdx.x == 0) stamps[(size_t)blockIdx.x * Tn * 8 + 7] = __builtin_amdgcn_s_memrealtime();

  // step 0's input rows first: vmcnt retires in order, so issued ahead of the 64 W_hh loads below
  // they let step 0 (no recurrent term) compute and publish while the slice is still arriving
  bf16x4 xv[QB];  // raw prefetch: converted at the step's use, not at the load
  auto load_xg = [&](int t) {
#pragma unroll
    for (int q = 0; q < QB; ++q) {
      const int bi = w * QB + q, i = bi / NJ, j = bi % NJ;
      const int b = b0 + 16 * i + c, n = n0 + 16 * j + 4 * g;
      xv[q] = *reinterpret_cast<const bf16x4*>(xg + ((size_t)b * Tn + t) * 2 * H4 + d * H4 + n);
    }
  };
  load_xg(d == 0 ? 0 : Tn - 1);

  // W_hh' slice fragments: rows n0 + 16j + c, k = w*KW + 32kc + 8g; register slot kk holds K-chunk
  // kc = (kk + rot) % KK: the workgroups of a (d, bs) group read the handed-off h in rotated chunk
  // order, spreading their simultaneous requests over memory channels
  const int rot = ns % KK;
  bf16x8 wf[NJ][KK];
  {
    const bf16* wb = whh + (size_t)d * H4 * H;
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int kk = 0; kk < KK; ++kk) {
        const int kc = kk + rot < KK ? kk + rot : kk + rot - KK;
        wf[j][kk] = *reinterpret_cast<const bf16x8*>(wb + (size_t)(n0 + 16 * j + c) * H + w * KW + 32 * kc + 8 * g);
      }
  }
  const __amdgpu_buffer_rsrc_t rh = rsrc_of(hseq);
  const __amdgpu_buffer_rsrc_t rr = rsrc_of(ring);
  const bool l2_handoff = TAG && xtab && seq_group_local(xtab, (d * nbs + bs) * nsl, nsl, ns, err);
  float cst[QB];
#pragma unroll
  for (int q = 0; q < QB; ++q) cst[q] = 0.f;

  for (int s = 0; s < Tn; ++s) {
    const int t = d == 0 ? s : Tn - 1 - s;
    const int tp = d == 0 ? t - 1 : t + 1;
    // the input rows xv are added after the hand-off (their load's latency hides under it)
    f32x4 sum[QB];
    bool ok = true;
    SEQ_STAMP(0);
    if (s > 0) {
      bf16x8 af[MI][KK];
      if constexpr (TAG) {
        // granules of h_{s-1}: row b0 + 16i + c, k = w*KW + 32kc + 8g .. +7 -> 4 granules (32 B)
        const uint32_t want = (uint32_t)s;
        const uint32_t gbase =
            (uint32_t)((((size_t)((s - 1) & 1) * B + b0 + c) * H + (d * H + w * KW + 8 * g) / 2) * 8u);
        unsigned long long t0 = 0;
        u32x4 gv[MI][KK][2];
        for (;;) {
#pragma unroll
          for (int kk = 0; kk < KK; ++kk)
#pragma unroll
            for (int i = 0; i < MI; ++i) {
              const int kc = kk + rot < KK ? kk + rot : kk + rot - KK;
              const uint32_t off = gbase + (uint32_t)(i * 16 * H * 8 + kc * 128);
              gv[i][kk][0] = __builtin_amdgcn_raw_buffer_load_b128(rr, off, 0, 16);
              gv[i][kk][1] = __builtin_amdgcn_raw_buffer_load_b128(rr, off + 16, 0, 16);
            }
          bool mine = true;
#pragma unroll
          for (int kk = 0; kk < KK; ++kk)
#pragma unroll
            for (int i = 0; i < MI; ++i)
#pragma unroll
              for (int h2 = 0; h2 < 2; ++h2) mine &= (gv[i][kk][h2][1] == want) & (gv[i][kk][h2][3] == want);
          if (__all(mine)) break;
          const unsigned long long now = __builtin_amdgcn_s_memrealtime();
          if (t0 == 0) t0 = now;
          if (now - t0 > SEQ_TIMEOUT_TICKS || __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
            __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            ok = false;
            break;
          }
          __builtin_amdgcn_s_sleep(1);
        }
        SEQ_STAMP(1);
#pragma unroll
        for (int kk = 0; kk < KK; ++kk)
#pragma unroll
          for (int i = 0; i < MI; ++i)
            af[i][kk] = __builtin_bit_cast(bf16x8, u32x4{gv[i][kk][0][0], gv[i][kk][0][2], gv[i][kk][1][0],
                                                         gv[i][kk][1][2]});
      } else {
        __shared__ int okflag;
        if (threadIdx.x == 0) okflag = seq_wait(mycnt, (unsigned)(nsl * s), err) ? 1 : 0;
        __syncthreads();
        SEQ_STAMP(1);
        ok = okflag != 0;
        // A fragments: h_{tp}[b0 + 16i + c][w*KW + 32kc + 8g] (sc1: handed-off bytes)
        const uint32_t abase = (uint32_t)((((size_t)b0 + c) * Tn + tp) * 2 * H + d * H + w * KW + 8 * g) * 2u;
#pragma unroll
        for (int kk = 0; kk < KK; ++kk)
#pragma unroll
          for (int i = 0; i < MI; ++i) {
            const int kc = kk + rot < KK ? kk + rot : kk + rot - KK;
            af[i][kk] = ld_sc1(rh, abase + (uint32_t)(i * 16 * Tn * 2 * H * 2 + kc * 64));
          }
        // every hand-off load in flight before the first MFMA (else the scheduler interleaves them
        // with the MFMAs one load at a time, each behind a vmcnt(0))
        __builtin_amdgcn_sched_barrier(0);
      }
      f32x4 acc[MI][NJ];
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < KK; ++kk)
#pragma unroll
        for (int i = 0; i < MI; ++i)
#pragma unroll
          for (int j = 0; j < NJ; ++j) mma<bf16>(acc[i][j], wf[j][kk], af[i][kk]);
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j) part[w][i][j][lane] = acc[i][j];
      SEQ_STAMP(2);
      __syncthreads();
      SEQ_STAMP(3);
#pragma unroll
      for (int q = 0; q < QB; ++q) {
        const int bi = w * QB + q, i = bi / NJ, j = bi % NJ;
        sum[q] = f32x4{(float)xv[q][0], (float)xv[q][1], (float)xv[q][2], (float)xv[q][3]};
#pragma unroll
        for (int ww = 0; ww < 4; ++ww) sum[q] += part[ww][i][j][lane];
      }
    } else {
#pragma unroll
      for (int q = 0; q < QB; ++q) sum[q] = f32x4{(float)xv[q][0], (float)xv[q][1], (float)xv[q][2], (float)xv[q][3]};
    }
    // next step's input rows, unconditionally (a load under a runtime branch gets a vmcnt(0) at
    // the join); the last step re-reads its own row. Granule form: issued as soon as xv is
    // consumed, a whole step ahead of its use (nothing drains vmcnt before the next poll); counter
    // form: after the publish's vmcnt(0) drain
    const int tn = s + 1 < Tn ? (d == 0 ? t + 1 : t - 1) : t;
    if constexpr (TAG) load_xg(tn);
    // cell update: lane holds gates (i,f,g,o) of unit n/4 for one sample, per block
    f32x4 gq[QB];
#pragma unroll
    for (int q = 0; q < QB; ++q) {
      const int bi = w * QB + q, i = bi / NJ, j = bi % NJ;
      f32x4 v = sum[q];
      const float ig = sigmoid_fast(v[0]), fg = sigmoid_fast(v[1]), gg = tanh_fast(v[2]), og = sigmoid_fast(v[3]);
      float cc = fg * cst[q] + ig * gg;
      float hh = og * tanh_fast(cc);
      if (!ok) hh = cc = __builtin_nanf("");
      cst[q] = cc;
      gq[q] = f32x4{ig, fg, gg, og};
      htile[16 * i + c][4 * j + g] = (bf16)hh;
    }
    SEQ_STAMP(4);
    __syncthreads();
    if constexpr (TAG) {
      // publish: S rows x U/2 granules into slot s & 1, two granules per 16-B sc1 store
      if (threadIdx.x < S * U / 4) {
        const int row = threadIdx.x / (U / 4), gp = threadIdx.x % (U / 4);
        const u32x4 hv = __builtin_bit_cast(u32x4, *reinterpret_cast<const bf16x8*>(&htile[row][8 * (gp >> 1)]));
        const uint32_t tag = (uint32_t)(s + 1);
        const u32x4 v = (gp & 1) ? u32x4{hv[2], tag, hv[3], tag} : u32x4{hv[0], tag, hv[1], tag};
        const uint32_t ro = (uint32_t)((((size_t)(s & 1) * B + b0 + row) * H + (d * H + ns * U + 4 * gp) / 2) * 8u);
        if (l2_handoff) __builtin_amdgcn_raw_buffer_store_b128(v, rr, ro, 0, 0);   // stays in the XCD's L2
        else __builtin_amdgcn_raw_buffer_store_b128(v, rr, ro, 0, 16);            // sc1: written through
      }
      SEQ_STAMP(5);
      // h_t for the next layer / BPTT: plain stores, off the critical path
      if (threadIdx.x < S * U / 8) {
        const int row = threadIdx.x / (U / 8), ch = threadIdx.x % (U / 8);
        *reinterpret_cast<bf16x8*>(hseq + ((size_t)(b0 + row) * Tn + t) * 2 * H + d * H + ns * U + 8 * ch) =
            *reinterpret_cast<const bf16x8*>(&htile[row][8 * ch]);
      }
      SEQ_STAMP(6);
    } else {
      // publish h_t of this (samples, units) tile: S rows x 2U bytes, one 16-B sc1 store per thread
      if (threadIdx.x < S * U / 8) {
        const int row = threadIdx.x / (U / 8), ch = threadIdx.x % (U / 8);
        const bf16x8 hv = *reinterpret_cast<const bf16x8*>(&htile[row][8 * ch]);
        st_sc1(rh, (uint32_t)((((size_t)(b0 + row) * Tn + t) * 2 * H + d * H + ns * U + 8 * ch) * sizeof(bf16)), hv);
      }
      SEQ_STAMP(5);
      seq_publish(mycnt);
      SEQ_STAMP(6);
    }
    // saved-forward stores for BPTT, off the hand-off's critical path (issued after the signal;
    // the next step's vmcnt(0) drains them long after they completed). gsv == nullptr: inference,
    // nothing saved (a uniform branch on a kernel argument)
    if (gsv != nullptr) {
#pragma unroll
      for (int q = 0; q < QB; ++q) {
        const int bi = w * QB + q, i = bi / NJ, j = bi % NJ;
        const int b = b0 + 16 * i + c;
        const int n = n0 + 16 * j + 4 * g, u = n >> 2;
        csv[((size_t)(d * Tn + t) * B + b) * H + u] = cst[q];
        st4<bf16>(gsv + ((size_t)(d * Tn + t) * B + b) * H4 + n, gq[q]);
      }
    }
    if constexpr (!TAG) load_xg(tn);
  }
  if constexpr (TAG) {  // steps completed (the counter-mode invariant: (H/U)*T per slice at the end)
    if (threadIdx.x == 0) __hip_atomic_fetch_add(mycnt, (unsigned)Tn, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}


// ---------------------------------------------------------------- forward sweep, unit-complete waves
// (CRNN_OPT_LSTM_HANDOFF = 2). Same workgroup tile (direction, S samples, U units) and the same
// granule ring as above, but the K split is gone: wave w OWNS NT * 4 = U/4 whole units over the full
// K = H (NT = U/16 gate-row fragments of 4 units x 4 gates, KK = H/32 k-steps in VGPRs/AGPRs: the same
// 64 KB of W_hh per wave and the same MFMA count per wave as the K-split form). What moves instead is
// h_{t-1}: each wave polls its K-quarter of the granules (as before) and writes it to a double-buffered
// LDS image of the whole h row block [S][H]; ONE barrier; then every wave reads all of it as MFMA B
// fragments. No fp32 partial tiles are exchanged (the K-split form wrote and re-read 64 KB of partials
// per workgroup per step plus a second barrier before the publish).
// Row order inside a wave: fragment jt, A row r -> unit NT*(r/4) + jt, gate r%4, so the accumulator
// rows 4g..4g+3 of lane (c, g) are the four gates of unit NT*g + jt of sample c: a lane ends the step
// with NT CONSECUTIVE units of one sample and publishes them straight from registers, NT/2 granules
// in one 8- or 16-B store (no h tile in LDS, no barrier before the publish).
// LDS image pitch H + 8 bf16 (16 B off a multiple of 256 B per row): the 16 lanes of a fragment read
// group land on distinct 16-B bank groups.
// Ring reuse (2 slots): a wave writes slot s & 1 at step s after its workgroup's step-s barrier, i.e.
// after all 4 waves' polls of h_{s-1} returned, from every producer wave of the group; each of those
// produced h_{s-1} after its own workgroup had read h_{s-2} (the slot's previous contents).
template <int H, int S, int U, int W>
__global__ __launch_bounds__(64 * W) void lstm_seq_fwd_uc_kernel(const bf16* __restrict__ xg,
                                                              const bf16* __restrict__ whh, bf16* hseq,
                                                              bf16* __restrict__ gsv, float* __restrict__ csv,
                                                              unsigned* cnt, unsigned* err, uint2* ring, int B,
                                                              int Tn, unsigned long long* stamps, unsigned* xtab) {
  constexpr int UW = U / W;           // units per wave
  constexpr int NT = UW / 4;          // fragments (and consecutive units per lane) per wave
  constexpr int KK = H / 32;          // k-steps over the full K
  constexpr int HW = H / W;           // one wave's poll slice of K
  constexpr int KQ = HW / 32;         // its k-steps
  constexpr int MI = S / 16, H4 = 4 * H, HP = H + 8;
  static_assert(HW % 32 == 0 && S % 16 == 0 && (NT == 2 || NT == 4), "shape");
  __shared__ __attribute__((aligned(16))) bf16 himg[2][S][HP];

  const int nsl = H / U, nbs = B / S;
  int d, bs, ns;
  seq_coords(nsl, nbs, d, bs, ns);
  const int lane = threadIdx.x & 63, c = lane & 15, g = lane >> 4;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int b0 = bs * S;
  const int ul = ns * U + w * UW + NT * g;   // this lane's first unit (NT consecutive)
  unsigned* mycnt = cnt + d * nbs + bs;
  if (stamps && threadIdx.x == 0) stamps[(size_t)blockIdx.x * Tn * 8 + 7] = __builtin_amdgcn_s_memrealtime();

  // x-gate rows of (sample b0 + 16i + c, units ul .. ul+NT-1): 4*NT consecutive packed gate rows
  bf16x8 xv[MI][NT / 2];
  auto load_xg = [&](int t) {
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int h2 = 0; h2 < NT / 2; ++h2)
        xv[i][h2] = *reinterpret_cast<const bf16x8*>(xg + ((size_t)(b0 + 16 * i + c) * Tn + t) * 2 * H4 + d * H4 +
                                                      4 * ul + 8 * h2);
  };
  load_xg(d == 0 ? 0 : Tn - 1);

  // W_hh' fragments: A row c of fragment jt = packed row 4 * (ns*U + w*UW + NT*(c>>2) + jt) + (c & 3)
  bf16x8 wf[NT][KK];
  {
    const bf16* wb = whh + (size_t)d * H4 * H;
#pragma unroll
    for (int jt = 0; jt < NT; ++jt) {
      const int row = 4 * (ns * U + w * UW + NT * (c >> 2) + jt) + (c & 3);
#pragma unroll
      for (int kk = 0; kk < KK; ++kk)
        wf[jt][kk] = *reinterpret_cast<const bf16x8*>(wb + (size_t)row * H + 32 * kk + 8 * g);
    }
  }
  const __amdgpu_buffer_rsrc_t rr = rsrc_of(ring);
  const bool l2_handoff = xtab && seq_group_local(xtab, (d * nbs + bs) * nsl, nsl, ns, err);
  const int rot = ns % KQ;   // rotated poll order: the group's workgroups spread their requests
  float cst[MI][NT];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int jt = 0; jt < NT; ++jt) cst[i][jt] = 0.f;

  for (int s = 0; s < Tn; ++s) {
    const int t = d == 0 ? s : Tn - 1 - s;
    const int buf = s & 1;
    bool ok = true;
    // accumulators start at the x-gate rows (the recurrent product accumulates onto them), initialised once the
    // hand-off has arrived (the rows' load then never holds up the poll's start; before the poll the step measured
    // 4.22-4.27 us inside the train step, after it 4.03, profiles/r06/r06u1_uc_variants_ab.log), which frees xv
    // for the next step's rows
    f32x4 acc[MI][NT];
    auto init_acc = [&]() {
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int jt = 0; jt < NT; ++jt) {
          const bf16x8& x8 = xv[i][jt >> 1];
          const int o = (jt & 1) * 4;
          acc[i][jt] = f32x4{(float)x8[o], (float)x8[o + 1], (float)x8[o + 2], (float)x8[o + 3]};
        }
    };
    const int tn = s + 1 < Tn ? (d == 0 ? t + 1 : t - 1) : t;
    bf16 hh[MI][NT];
    f32x4 gq[MI][NT];
    // cell update of fragment (i, jt): lane holds gates (i, f, g, o) of unit ul + jt of one sample
    auto cell = [&](int i, int jt) {
      const f32x4 v = acc[i][jt];
      const float ig = sigmoid_fast(v[0]), fg = sigmoid_fast(v[1]), gg = tanh_fast(v[2]), og = sigmoid_fast(v[3]);
      float cc = fg * cst[i][jt] + ig * gg;
      float h = og * tanh_fast(cc);
      if (!ok) h = cc = __builtin_nanf("");
      cst[i][jt] = cc;
      gq[i][jt] = f32x4{ig, fg, gg, og};
      hh[i][jt] = (bf16)h;
    };
    SEQ_STAMP(0);
    if (s > 0) {
      // poll this wave's K-slice of h_{s-1}: row b0 + 16i + c, k = w*H/4 + 32kc + 8g .. +7 (4 granules)
      const uint32_t want = (uint32_t)s;
      const uint32_t gbase =
          (uint32_t)((((size_t)((s - 1) & 1) * B + b0 + c) * H + (d * H + w * HW + 8 * g) / 2) * 8u);
      unsigned long long t0 = 0;
      u32x4 gv[MI][KQ][2];
      for (;;) {
#pragma unroll
        for (int kq = 0; kq < KQ; ++kq)
#pragma unroll
          for (int i = 0; i < MI; ++i) {
            const int kc = kq + rot < KQ ? kq + rot : kq + rot - KQ;
            const uint32_t off = gbase + (uint32_t)(i * 16 * H * 8 + kc * 128);
            gv[i][kq][0] = __builtin_amdgcn_raw_buffer_load_b128(rr, off, 0, 16);
            gv[i][kq][1] = __builtin_amdgcn_raw_buffer_load_b128(rr, off + 16, 0, 16);
          }
        bool mine = true;
#pragma unroll
        for (int kq = 0; kq < KQ; ++kq)
#pragma unroll
          for (int i = 0; i < MI; ++i)
#pragma unroll
            for (int h2 = 0; h2 < 2; ++h2) mine &= (gv[i][kq][h2][1] == want) & (gv[i][kq][h2][3] == want);
        if (__all(mine)) break;
        const unsigned long long now = __builtin_amdgcn_s_memrealtime();
        if (t0 == 0) t0 = now;
        if (now - t0 > SEQ_TIMEOUT_TICKS || __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
          __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          ok = false;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
      SEQ_STAMP(1);
      init_acc();
#pragma unroll
      for (int kq = 0; kq < KQ; ++kq)
#pragma unroll
        for (int i = 0; i < MI; ++i) {
          const int kc = kq + rot < KQ ? kq + rot : kq + rot - KQ;
          *reinterpret_cast<u32x4*>(&himg[buf][16 * i + c][w * HW + 32 * kc + 8 * g]) =
              u32x4{gv[i][kq][0][0], gv[i][kq][0][2], gv[i][kq][1][0], gv[i][kq][1][2]};
        }
      load_xg(tn);   // issued behind the hand-off loads, a whole step ahead of its use
      SEQ_STAMP(2);
      __syncthreads();
      SEQ_STAMP(3);
      if constexpr (MI == 1 && KK <= 16) {
        // all B fragments in flight first, then fragment after fragment: fragment jt's 4 cells run in the
        // shadow of fragment jt+1's MFMAs (an MFMA holds vector issue for 8 of its 16 cycles)
        bf16x8 hb[KK];
#pragma unroll
        for (int kk = 0; kk < KK; ++kk) hb[kk] = *reinterpret_cast<const bf16x8*>(&himg[buf][c][32 * kk + 8 * g]);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int jt = 0; jt < NT; ++jt) {
#pragma unroll
          for (int kk = 0; kk < KK; ++kk) mma<bf16>(acc[0][jt], wf[jt][kk], hb[kk]);
          if (jt > 0) {
            cell(0, jt - 1);
            // the scheduler keeps a fragment's MFMA chain together and the cell math after it: ask for
            // one MFMA then ~3 VALU (the cell's ~45 instructions spread over the 16 MFMA gaps)
#pragma unroll
            for (int q = 0; q < KK; ++q) {
              __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);   // MFMA
              __builtin_amdgcn_sched_group_barrier(0x002, 3, 0);   // VALU
            }
          }
          __builtin_amdgcn_sched_barrier(0);
        }
        cell(0, NT - 1);
      } else {
        // B fragments in batches of up to 16 reads, all issued before the batch's MFMAs (one
        // ds_read -> lgkmcnt(0) -> MFMA round trip per k-step would expose the LDS latency 16 times)
        constexpr int CH = MI * KK <= 16 ? KK : 16 / MI;
#pragma unroll
        for (int k0 = 0; k0 < KK; k0 += CH) {
          bf16x8 hb[MI][CH];
#pragma unroll
          for (int kk = 0; kk < CH; ++kk)
#pragma unroll
            for (int i = 0; i < MI; ++i)
              if (k0 + kk < KK)
                hb[i][kk] = *reinterpret_cast<const bf16x8*>(&himg[buf][16 * i + c][32 * (k0 + kk) + 8 * g]);
          __builtin_amdgcn_sched_barrier(0);   // every read of the batch in flight before its first MFMA
#pragma unroll
          for (int kk = 0; kk < CH; ++kk)
#pragma unroll
            for (int i = 0; i < MI; ++i)
#pragma unroll
              for (int jt = 0; jt < NT; ++jt)
                if (k0 + kk < KK) mma<bf16>(acc[i][jt], wf[jt][k0 + kk], hb[i][kk]);
        }
#pragma unroll
        for (int i = 0; i < MI; ++i)
#pragma unroll
          for (int jt = 0; jt < NT; ++jt) cell(i, jt);
      }
    } else {
      init_acc();
      load_xg(tn);
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int jt = 0; jt < NT; ++jt) cell(i, jt);
    }
    SEQ_STAMP(4);
    // publish: NT/2 granules {2 bf16, tag = s + 1} per (lane, sample tile), straight from registers
    const uint32_t tag = (uint32_t)(s + 1);
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      const uint32_t ro = (uint32_t)((((size_t)(s & 1) * B + b0 + 16 * i + c) * H + (d * H + ul) / 2) * 8u);
      const uint32_t h01 = __builtin_bit_cast(uint32_t, bf16x2_t{hh[i][0], hh[i][1]});
      if constexpr (NT == 4) {
        const uint32_t h23 = __builtin_bit_cast(uint32_t, bf16x2_t{hh[i][2], hh[i][3]});
        const u32x4 v = u32x4{h01, tag, h23, tag};
        if (l2_handoff) __builtin_amdgcn_raw_buffer_store_b128(v, rr, ro, 0, 0);   // stays in the XCD's L2
        else __builtin_amdgcn_raw_buffer_store_b128(v, rr, ro, 0, 16);            // sc1: written through
      } else {
        const u32x2_t v = u32x2_t{h01, tag};
        if (l2_handoff) __builtin_amdgcn_raw_buffer_store_b64(v, rr, ro, 0, 0);
        else __builtin_amdgcn_raw_buffer_store_b64(v, rr, ro, 0, 16);
      }
    }
    SEQ_STAMP(5);
    // h_t for the next layer / BPTT and the saved forward state: plain stores, off the critical path
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      const int b = b0 + 16 * i + c;
      bf16* hp = hseq + ((size_t)b * Tn + t) * 2 * H + d * H + ul;
      if constexpr (NT == 4) *reinterpret_cast<bf16x4*>(hp) = bf16x4{hh[i][0], hh[i][1], hh[i][2], hh[i][3]};
      else *reinterpret_cast<bf16x2_t*>(hp) = bf16x2_t{hh[i][0], hh[i][1]};
      if (gsv != nullptr) {
        float* cp = csv + ((size_t)(d * Tn + t) * B + b) * H + ul;
        bf16* gp = gsv + ((size_t)(d * Tn + t) * B + b) * H4 + 4 * ul;
#pragma unroll
        for (int h2 = 0; h2 < NT / 2; ++h2) {
          const f32x4 a = gq[i][2 * h2], e = gq[i][2 * h2 + 1];
          *reinterpret_cast<bf16x8*>(gp + 8 * h2) =
              bf16x8{(bf16)a[0], (bf16)a[1], (bf16)a[2], (bf16)a[3], (bf16)e[0], (bf16)e[1], (bf16)e[2], (bf16)e[3]};
        }
        if constexpr (NT == 4) *reinterpret_cast<f32x4*>(cp) = f32x4{cst[i][0], cst[i][1], cst[i][2], cst[i][3]};
        else *reinterpret_cast<float2*>(cp) = float2{cst[i][0], cst[i][1]};
      }
    }
    SEQ_STAMP(6);
  }
  if (threadIdx.x == 0) __hip_atomic_fetch_add(mycnt, (unsigned)Tn, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ---------------------------------------------------------------- BPTT sweep
// wave w: K-quarter [w*H, (w+1)*H) of the 4H gate columns; partial tile S samples x U units
// (MI x NU fragments); waves w < MI*NU finalise block (i, j) = (w % MI, w / MI): 16 samples x 16
// units, one sample and 4 consecutive units per lane.
template <int H, int S, int U>
__global__ __launch_bounds__(256) void lstm_seq_bwd_kernel(const bf16* __restrict__ dhseq, const bf16* __restrict__ whh_t,
                                                           const bf16* __restrict__ gsv, const float* __restrict__ csv,
                                                           bf16* dgates, unsigned* cnt, unsigned* err, int B, int Tn,
                                                           unsigned long long* stamps, unsigned* xtab) {
  constexpr int KW = H, KK = KW / 32;
  constexpr int H4 = 4 * H, MI = S / 16, NU = U / 16, NBLK = MI * NU;
  static_assert(H % 32 == 0 && NBLK <= 4 && S % 16 == 0 && U % 16 == 0, "shape");
  __shared__ __attribute__((aligned(16))) f32x4 part[4][MI][NU][64];

  const int nsl = H / U, nbs = B / S;
  int d, bs, ns;
  seq_coords(nsl, nbs, d, bs, ns);
  const int lane = threadIdx.x & 63, c = lane & 15, g = lane >> 4;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int b0 = bs * S, u0 = ns * U;
  unsigned* mycnt = cnt + d * nbs + bs;

  if (stamps && threadIdx.x == 0) stamps[(size_t)blockIdx.x * Tn * 8 + 7] = __builtin_amdgcn_s_memrealtime();
  // dgates payload: plain stores + the drained counter when the group is on one XCD (the
  // consumers' sc1 loads then hit the shared L2), sc1 stores otherwise (seq_group_local). Checked
  // BEFORE the prologue's loads: the check is a call, and a non-kernel function starts with a full
  // s_waitcnt, which after the W_hh slice loads held every workgroup ~8 us (r06 stamps: 11 us from
  // entry to step 0)
  const bool l2_handoff = xtab && seq_group_local(xtab, (d * nbs + bs) * nsl, nsl, ns, err);
  const bool fin = w < NBLK;
  const int fi = fin ? w % MI : 0, fj = fin ? w / MI : 0;
  const int bl = 16 * fi + c, b = b0 + bl;
  const int u = u0 + 16 * fj + 4 * g;  // this lane's 4 units u..u+3
  float dcs[4] = {0.f, 0.f, 0.f, 0.f};

  // per-step saved-forward inputs of this lane (independent of the recurrence: prefetched;
  // loads are unconditional — the t-1 of the first step reads a clamped row and is masked)
  bf16x8 gv0, gv1;
  f32x4 cv, cpv, dhv;
  float has_prev_f = 0.f;
  auto load_in = [&](int t) {
    const size_t gi = ((size_t)(d * Tn + t) * B + b) * H4 + 4 * u;
    gv0 = *reinterpret_cast<const bf16x8*>(gsv + gi);
    gv1 = *reinterpret_cast<const bf16x8*>(gsv + gi + 8);
    cv = *reinterpret_cast<const f32x4*>(csv + ((size_t)(d * Tn + t) * B + b) * H + u);
    const int tf = d == 0 ? t - 1 : t + 1;
    const bool has_prev = d == 0 ? t > 0 : t < Tn - 1;
    const int tfc = has_prev ? tf : t;
    cpv = *reinterpret_cast<const f32x4*>(csv + ((size_t)(d * Tn + tfc) * B + b) * H + u);
    has_prev_f = has_prev ? 1.f : 0.f;
    dhv = ld4f<bf16>(dhseq + ((size_t)b * Tn + t) * 2 * H + d * H + u);
  };
  load_in(d == 0 ? Tn - 1 : 0);   // ahead of the W_hh slice loads (forward sweep)

  // W_hh'^T slice fragments: rows u0 + 16j + c of whh_t[d] ([H][4H]), k = w*KW + 32kc + 8g
  const int rot = (ns * KK / nsl) % KK;   // rotated K-chunk order, as in the forward kernel
  bf16x8 wf[NU][KK];
  {
    const bf16* wb = whh_t + (size_t)d * H * H4;
#pragma unroll
    for (int j = 0; j < NU; ++j)
#pragma unroll
      for (int kk = 0; kk < KK; ++kk) {
        const int kc = kk + rot < KK ? kk + rot : kk + rot - KK;
        wf[j][kk] = *reinterpret_cast<const bf16x8*>(wb + (size_t)(u0 + 16 * j + c) * H4 + w * KW + 32 * kc + 8 * g);
      }
  }
  const __amdgpu_buffer_rsrc_t rg = rsrc_of(dgates);

  for (int s = 0; s < Tn; ++s) {
    const int t = d == 0 ? Tn - 1 - s : s;
    const int tn = d == 0 ? t + 1 : t - 1;  // time of the previous BPTT step
    f32x4 dh = dhv;
    bool ok = true;
    SEQ_STAMP(0);
    if (s > 0) {
      __shared__ int okflag;
      if (threadIdx.x == 0) okflag = seq_wait(mycnt, (unsigned)(nsl * s), err) ? 1 : 0;
      __syncthreads();
      SEQ_STAMP(1);
      ok = okflag != 0;
      bf16x8 af[MI][KK];
      const uint32_t abase = (uint32_t)((((size_t)(d * Tn + tn) * B + b0 + c) * H4 + w * KW + 8 * g) * 2u);
#pragma unroll
      for (int kk = 0; kk < KK; ++kk)
#pragma unroll
        for (int i = 0; i < MI; ++i) {
          const int kc = kk + rot < KK ? kk + rot : kk + rot - KK;
          af[i][kk] = ld_sc1(rg, abase + (uint32_t)(i * 16 * H4 * 2 + kc * 64));
        }
      __builtin_amdgcn_sched_barrier(0);  // all loads issued first (forward sweep)
      f32x4 acc[MI][NU];
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NU; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < KK; ++kk)
#pragma unroll
        for (int i = 0; i < MI; ++i)
#pragma unroll
          for (int j = 0; j < NU; ++j) mma<bf16>(acc[i][j], wf[j][kk], af[i][kk]);
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NU; ++j) part[w][i][j][lane] = acc[i][j];
      SEQ_STAMP(2);
      __syncthreads();
      SEQ_STAMP(3);
      if (fin)
#pragma unroll
        for (int ww = 0; ww < 4; ++ww) dh += part[ww][fi][fj][lane];
    }
    if (fin) {
      // cell backward of units u..u+3 (lstm.hip cell_bwd)
      bf16x8 out0, out1;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const bf16x8& gv = r < 2 ? gv0 : gv1;
        const int o = (r & 1) * 4;
        const float ig = (float)gv[o], fg = (float)gv[o + 1], gg = (float)gv[o + 2], og = (float)gv[o + 3];
        const float tc = tanh_fast(cv[r]);
        const float dcv = dcs[r] + dh[r] * og * (1.f - tc * tc);
        const float do_ = dh[r] * tc;
        const float di = dcv * gg, dg = dcv * ig, df = dcv * cpv[r] * has_prev_f;
        dcs[r] = dcv * fg;
        float q0 = di * ig * (1.f - ig), q1 = df * fg * (1.f - fg), q2 = dg * (1.f - gg * gg), q3 = do_ * og * (1.f - og);
        if (!ok) q0 = q1 = q2 = q3 = __builtin_nanf("");
        bf16x8& ov = r < 2 ? out0 : out1;
        ov[o] = (bf16)q0;
        ov[o + 1] = (bf16)q1;
        ov[o + 2] = (bf16)q2;
        ov[o + 3] = (bf16)q3;
      }
      SEQ_STAMP(4);
      const uint32_t go = (uint32_t)((((size_t)(d * Tn + t) * B + b) * H4 + 4 * u) * sizeof(bf16));
      if (l2_handoff) {   // the group is on one XCD: the lines stay in its L2
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, out0), rg, go, 0, 0);
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, out1), rg, go + 16, 0, 0);
      } else {
        st_sc1(rg, go, out0);
        st_sc1(rg, go + 16, out1);
      }
    }
    SEQ_STAMP(5);
    seq_publish(mycnt);
    SEQ_STAMP(6);
    // unconditional prefetch (see the forward sweep); non-finalising waves read valid rows unused
    load_in(s + 1 < Tn ? (d == 0 ? t - 1 : t + 1) : t);
  }
}

// ---------------------------------------------------------------- BPTT sweep, partial-sum form
// (CRNN_OPT_LSTM_BWD_PART = 1; measured against the counter form in one process: cfg2 6.42 vs
// 5.92 us per step, long config 6.24 vs 6.39 — so the counter form stays the default,
// profiles/r02l_lstm_bwd_partial_ab.log). Each workgroup multiplies its OWN dgates by its own
// packed W_hh' rows: partial[b][h] = sum over its 4U gate rows k of dgates_t[b][k] W_hh'[k][h]
// (wave w: the h quarter [w H/4, (w+1) H/4); W_hh'^T fragments resident in VGPRs), and publishes
// the partial as data-tagged granules {2 bf16, u32 tag = step + 1} (the forward's handoff-1to1
// form). The finalising lanes of the next step gather, for their 16 samples x 4 units, the
// partials of all H/U workgroups of their (d, bs) group and sum them in fp32: per step a
// workgroup gathers S x U x (H/U) partials (cfg2: 16 KB of bf16 + tags) instead of the S x 4H
// dgates the counter form needs (64 KB), the MFMA needs no remote data, and nothing drains,
// barriers or counts on the hand-off. Ring: [2 slots][2 d][B][H/U producers][H] granule
// positions (4 B per value), zeroed per launch; slot s & 1 is rewritten at step s + 2 only after
// its consumers' gathers of step s + 1 returned (they precede their step s + 1 publish, which the
// producer's own step s + 2 gather waited for).
template <int H, int S, int U>
__global__ __launch_bounds__(256) void lstm_seq_bwdp_kernel(const bf16* __restrict__ dhseq,
                                                            const bf16* __restrict__ whh_t,
                                                            const bf16* __restrict__ gsv,
                                                            const float* __restrict__ csv, bf16* dgates,
                                                            unsigned* cnt, unsigned* err, uint2* ring, int B,
                                                            int Tn, unsigned long long* stamps) {
  constexpr int GR = 4 * U, KK = GR / 32;   // MFMA k: the workgroup's packed gate rows
  constexpr int HQ = H / 4, NJ = HQ / 16;   // wave w: h in [w HQ, (w + 1) HQ)
  constexpr int H4 = 4 * H, MI = S / 16, NU = U / 16, NBLK = MI * NU;
  constexpr int DP = GR + 8;                // dgates tile pitch (bf16): rows 16 B off-bank
  static_assert(S % 16 == 0 && U % 16 == 0 && HQ % 16 == 0 && NBLK <= 4 && GR % 32 == 0, "shape");
  __shared__ __attribute__((aligned(16))) bf16 dgt[2][S][DP];

  const int nsl = H / U, nbs = B / S;
  int d, bs, ns;
  seq_coords(nsl, nbs, d, bs, ns);
  const int lane = threadIdx.x & 63, c = lane & 15, g = lane >> 4;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int b0 = bs * S, u0 = ns * U;
  unsigned* mycnt = cnt + d * nbs + bs;

  // W_hh'^T fragments (MFMA A operand): row h = w HQ + 16j + c of whh_t[d] ([H][4H]), k = the
  // packed gate rows 4 u0 + 32kk + 8g .. +7
  bf16x8 wf[NJ][KK];
  {
    const bf16* wb = whh_t + (size_t)d * H * H4;
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int kk = 0; kk < KK; ++kk)
        wf[j][kk] = *reinterpret_cast<const bf16x8*>(wb + (size_t)(w * HQ + 16 * j + c) * H4 + 4 * u0 + 32 * kk + 8 * g);
  }
  const __amdgpu_buffer_rsrc_t rr = rsrc_of(ring);
  // granule position of value (slot, b, producer p, h): 4 bytes per value, two values per granule
  auto gpos = [&](int slot, int b, int p, int h) -> uint32_t {
    return (uint32_t)(((((size_t)(slot * 2 + d) * B + b) * nsl + p) * H + h) * 4u);
  };
  const bool fin = w < NBLK;
  const int fi = fin ? w % MI : 0, fj = fin ? w / MI : 0;
  const int bl = 16 * fi + c, b = b0 + bl;
  const int u = u0 + 16 * fj + 4 * g;  // this lane's 4 units u..u+3
  float dcs[4] = {0.f, 0.f, 0.f, 0.f};

  bf16x8 gv0, gv1;
  f32x4 cv, cpv, dhv;
  float has_prev_f = 0.f;
  auto load_in = [&](int t) {
    const size_t gi = ((size_t)(d * Tn + t) * B + b) * H4 + 4 * u;
    gv0 = *reinterpret_cast<const bf16x8*>(gsv + gi);
    gv1 = *reinterpret_cast<const bf16x8*>(gsv + gi + 8);
    cv = *reinterpret_cast<const f32x4*>(csv + ((size_t)(d * Tn + t) * B + b) * H + u);
    const int tf = d == 0 ? t - 1 : t + 1;
    const bool has_prev = d == 0 ? t > 0 : t < Tn - 1;
    const int tfc = has_prev ? tf : t;
    cpv = *reinterpret_cast<const f32x4*>(csv + ((size_t)(d * Tn + tfc) * B + b) * H + u);
    has_prev_f = has_prev ? 1.f : 0.f;
    dhv = ld4f<bf16>(dhseq + ((size_t)b * Tn + t) * 2 * H + d * H + u);
  };
  load_in(d == 0 ? Tn - 1 : 0);

  bool ok = true;
  for (int s = 0; s < Tn; ++s) {
    const int t = d == 0 ? Tn - 1 - s : s;
    const int buf = s & 1;
    f32x4 dh = dhv;
    SEQ_STAMP(0);
    if (fin) {
      if (s > 0) {
        // the previous step's partials of this lane's (sample, 4 units) from every producer
        const uint32_t want = (uint32_t)s;
        unsigned long long t0 = 0;
        constexpr int NP = H / U;
        u32x4 pv[NP];
        for (;;) {
#pragma unroll
          for (int p = 0; p < NP; ++p) pv[p] = __builtin_amdgcn_raw_buffer_load_b128(rr, gpos((s - 1) & 1, b, p, u), 0, 16);
          bool mine = true;
#pragma unroll
          for (int p = 0; p < NP; ++p) mine &= (pv[p][1] == want) & (pv[p][3] == want);
          if (__all(mine)) break;
          const unsigned long long now = __builtin_amdgcn_s_memrealtime();
          if (t0 == 0) t0 = now;
          if (now - t0 > SEQ_TIMEOUT_TICKS || __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
            __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            ok = false;
            break;
          }
          __builtin_amdgcn_s_sleep(1);
        }
        SEQ_STAMP(1);
#pragma unroll
        for (int p = 0; p < NP; ++p) {
          const bf16x4 v = __builtin_bit_cast(bf16x4, uint2{pv[p][0], pv[p][2]});
          dh += f32x4{(float)v[0], (float)v[1], (float)v[2], (float)v[3]};
        }
      }
      // cell backward of units u..u+3 (lstm.hip cell_bwd)
      bf16x8 out0, out1;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const bf16x8& gv = r < 2 ? gv0 : gv1;
        const int o = (r & 1) * 4;
        const float ig = (float)gv[o], fg = (float)gv[o + 1], gg = (float)gv[o + 2], og = (float)gv[o + 3];
        const float tc = tanh_fast(cv[r]);
        const float dcv = dcs[r] + dh[r] * og * (1.f - tc * tc);
        const float do_ = dh[r] * tc;
        const float di = dcv * gg, dg = dcv * ig, df = dcv * cpv[r] * has_prev_f;
        dcs[r] = dcv * fg;
        float q0 = di * ig * (1.f - ig), q1 = df * fg * (1.f - fg), q2 = dg * (1.f - gg * gg), q3 = do_ * og * (1.f - og);
        if (!ok) q0 = q1 = q2 = q3 = __builtin_nanf("");
        bf16x8& ov = r < 2 ? out0 : out1;
        ov[o] = (bf16)q0;
        ov[o + 1] = (bf16)q1;
        ov[o + 2] = (bf16)q2;
        ov[o + 3] = (bf16)q3;
      }
      *reinterpret_cast<bf16x8*>(&dgt[buf][bl][4 * (u - u0)]) = out0;
      *reinterpret_cast<bf16x8*>(&dgt[buf][bl][4 * (u - u0) + 8]) = out1;
      // dgates for the weight gradients: plain stores, off the hand-off path
      bf16* go = dgates + ((size_t)(d * Tn + t) * B + b) * H4 + 4 * u;
      *reinterpret_cast<bf16x8*>(go) = out0;
      *reinterpret_cast<bf16x8*>(go + 8) = out1;
    }
    SEQ_STAMP(2);
    __syncthreads();  // the dgates tile of this step (double-buffered: see the ring note above)
    SEQ_STAMP(3);
    if (s + 1 < Tn) {
      bf16x8 af[MI][KK];
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int kk = 0; kk < KK; ++kk) af[i][kk] = *reinterpret_cast<const bf16x8*>(&dgt[buf][16 * i + c][32 * kk + 8 * g]);
      // one output tile at a time (a dependent MFMA chain costs no more than independent ones,
      // MI355X_MICROARCH.md), published as soon as it is complete: its stores overlap the next
      // tile's MFMAs. Lane: h = w HQ + 16j + 4g .. +3 of sample b0 + 16i + c -> two granules
      const uint32_t tag = (uint32_t)(s + 1);
#pragma unroll
      for (int j = 0; j < NJ; ++j)
#pragma unroll
        for (int i = 0; i < MI; ++i) {
          f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int kk = 0; kk < KK; ++kk) mma<bf16>(acc, wf[j][kk], af[i][kk]);
          const bf16x4 hv = {(bf16)acc[0], (bf16)acc[1], (bf16)acc[2], (bf16)acc[3]};
          const uint2 hp = __builtin_bit_cast(uint2, hv);
          __builtin_amdgcn_raw_buffer_store_b128(u32x4{hp.x, tag, hp.y, tag}, rr,
                                                 gpos(buf, b0 + 16 * i + c, ns, w * HQ + 16 * j + 4 * g), 0, 16);
        }
      SEQ_STAMP(4);
    }
    SEQ_STAMP(5);
    SEQ_STAMP(6);
    // unconditional prefetch of the next step's saved-forward inputs (the last step re-reads its own)
    load_in(s + 1 < Tn ? (d == 0 ? t - 1 : t + 1) : t);
  }
  // the counter-form invariant ((H/U) * T per slice at the end)
  if (threadIdx.x == 0) __hip_atomic_fetch_add(mycnt, (unsigned)Tn, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

int g_cus = -1;
unsigned long long* g_stamps = nullptr;  // crnn_lstm_seq_debug_stamps

int cu_count() {
  if (g_cus < 0) {
    int dev = 0;
    hipDeviceProp_t p;
    g_cus = (hipGetDevice(&dev) == hipSuccess && hipGetDeviceProperties(&p, dev) == hipSuccess) ? p.multiProcessorCount : 0;
  }
  return g_cus;
}

// (samples, units) per workgroup: 16 samples halve the per-step hand-off each workgroup gathers;
// 64 units (H <= 512: the W_hh slice still fits the VGPRs) keep the grid at <= one per CU
bool seq_config(int B, int H, bool bwd, int& S, int& U) {
  if (!(H == 256 || H == 512 || H == 768)) return false;
  const int ncu = cu_count();
  // preference order measured on MI355X (profiles/r01k_lstm_tiles.log): 16 samples halve the
  // hand-off bytes each workgroup gathers per step; 16 x 64 over 16 x 32 where both fit
  static const int order[2][3][2] = {{{16, 64}, {16, 32}, {32, 32}}, {{16, 64}, {16, 32}, {32, 32}}};
  const int force = crnn_option(CRNN_OPT_LSTM_TILE);  // 1: 32x32, 2: 16x32, 3: 16x64 only
  for (int k = 0; k < 3; ++k) {
    const int s = order[bwd][k][0], u = order[bwd][k][1];
    if (force >= 1 && force <= 3 && (s == 32 ? 1 : u == 32 ? 2 : 3) != force) continue;
    if (u == 64 && H > 512) continue;  // the 4U x H/4 W_hh slice must stay in VGPRs
    if (B % s || 2 * (B / s) * (H / u) > ncu) continue;
    S = s;
    U = u;
    return true;
  }
  return false;
}

template <int H, int S, int U>
void launch_fwd_tile(int form, dim3 grid, hipStream_t st, const bf16* xg, const bf16* whh, bf16* hseq, bf16* gsv,
                     float* csv, unsigned* cnt, unsigned* err, uint2* ring, int B, int T, unsigned* xtab) {
  if constexpr (U == 64) {
    if (form == 3) {   // 8 waves of 8 units: 2 waves per SIMD, weights without AGPR copies
      hipLaunchKernelGGL((lstm_seq_fwd_uc_kernel<H, S, U, 8>), grid, dim3(512), 0, st, xg, whh, hseq, gsv, csv, cnt,
                         err, ring, B, T, g_stamps, xtab);
      return;
    }
  }
  // form 3 on a 32-unit tile (H = 768): the K-split granule form, which measured faster there
  // (3.29 vs 4.11 us per step at B = 64, profiles/r06/r06a_lstm_forms_ab.log)
  if (form >= 3) form = 1;
  if (form == 2)
    hipLaunchKernelGGL((lstm_seq_fwd_uc_kernel<H, S, U, 4>), grid, dim3(256), 0, st, xg, whh, hseq, gsv, csv, cnt, err,
                       ring, B, T, g_stamps, xtab);
  else if (form == 1)
    hipLaunchKernelGGL((lstm_seq_fwd_kernel<H, S, U, true>), grid, dim3(256), 0, st, xg, whh, hseq, gsv, csv, cnt, err,
                       ring, B, T, g_stamps, xtab);
  else
    hipLaunchKernelGGL((lstm_seq_fwd_kernel<H, S, U, false>), grid, dim3(256), 0, st, xg, whh, hseq, gsv, csv, cnt,
                       err, ring, B, T, g_stamps, nullptr);
}

template <int H>
int launch_fwd(int S, int U, dim3 grid, hipStream_t st, const bf16* xg, const bf16* whh, bf16* hseq, bf16* gsv,
               float* csv, unsigned* cnt, unsigned* err, uint2* ring, int B, int T, unsigned* xtab) {
  const int tag = crnn_option(CRNN_OPT_LSTM_HANDOFF);
  if constexpr (H <= 512) {  // 16 x 64 would spill at H = 768 (seq_config never picks it)
    if (S == 16 && U == 64) {
      launch_fwd_tile<H, 16, 64>(tag, grid, st, xg, whh, hseq, gsv, csv, cnt, err, ring, B, T, xtab);
      return (int)hipGetLastError();
    }
  }
  if (S == 16)
    launch_fwd_tile<H, 16, 32>(tag, grid, st, xg, whh, hseq, gsv, csv, cnt, err, ring, B, T, xtab);
  else
    launch_fwd_tile<H, 32, 32>(tag, grid, st, xg, whh, hseq, gsv, csv, cnt, err, ring, B, T, xtab);
  return (int)hipGetLastError();
}

template <int H>
int launch_bwd(int S, int U, dim3 grid, hipStream_t st, const bf16* dhseq, const bf16* whh_t, const bf16* gsv,
               const float* csv, bf16* dg, unsigned* cnt, unsigned* err, uint2* ring, int B, int T, unsigned* xtab) {
  if (crnn_option(CRNN_OPT_LSTM_BWD_PART)) {
    if constexpr (H <= 512) {
      if (S == 16 && U == 64) {
        hipLaunchKernelGGL((lstm_seq_bwdp_kernel<H, 16, 64>), grid, dim3(256), 0, st, dhseq, whh_t, gsv, csv, dg, cnt,
                           err, ring, B, T, g_stamps);
        return (int)hipGetLastError();
      }
    }
    if (S == 16)
      hipLaunchKernelGGL((lstm_seq_bwdp_kernel<H, 16, 32>), grid, dim3(256), 0, st, dhseq, whh_t, gsv, csv, dg, cnt,
                         err, ring, B, T, g_stamps);
    else
      hipLaunchKernelGGL((lstm_seq_bwdp_kernel<H, 32, 32>), grid, dim3(256), 0, st, dhseq, whh_t, gsv, csv, dg, cnt,
                         err, ring, B, T, g_stamps);
    return (int)hipGetLastError();
  }
  if constexpr (H <= 512) {
    if (S == 16 && U == 64) {
      hipLaunchKernelGGL((lstm_seq_bwd_kernel<H, 16, 64>), grid, dim3(256), 0, st, dhseq, whh_t, gsv, csv, dg, cnt, err, B, T, g_stamps, xtab);
      return (int)hipGetLastError();
    }
  }
  if (S == 16)
    hipLaunchKernelGGL((lstm_seq_bwd_kernel<H, 16, 32>), grid, dim3(256), 0, st, dhseq, whh_t, gsv, csv, dg, cnt, err, B, T, g_stamps, xtab);
  else
    hipLaunchKernelGGL((lstm_seq_bwd_kernel<H, 32, 32>), grid, dim3(256), 0, st, dhseq, whh_t, gsv, csv, dg, cnt, err, B, T, g_stamps, xtab);
  return (int)hipGetLastError();
}

// sticky status: OR the launch's error word into a word no launch zeroes (read by the host
// asynchronously, crnn_hip/engine.py poll_status), so a timed-out wait cannot pass unnoticed
__global__ void seq_status_accum_kernel(const unsigned* err, unsigned* sticky) {
  const unsigned e = err[0];
  if (e) sticky[0] |= e;
}

}  // namespace

extern "C" {

int crnn_lstm_seq_supported(int dtype, int B, int H) {
  int S, U;
  return dtype == CRNN_BF16 && seq_config(B, H, false, S, U) && seq_config(B, H, true, S, U) ? 1 : 0;
}

int crnn_lstm_seq_config(int B, int H, int bwd, int* S, int* U) {
  int s = 0, u = 0;
  const int ok = seq_config(B, H, bwd != 0, s, u) ? 1 : 0;
  if (S) *S = ok ? s : 0;
  if (U) *U = ok ? u : 0;
  return ok;
}

// diagnostics: per-phase timestamps of the NEXT persistent launches into `buf` (device,
// grid * T * 8 u64), NULL to stop. Not for production paths.
int crnn_lstm_seq_debug_stamps(unsigned long long* buf) {
  g_stamps = buf;
  return 0;
}

// counters: one per (direction, batch slice) of the smallest slice (16 samples), then the error word;
// then (from byte seq_ring_offset) the granule ring shared by the sweeps (one runs at a time on the
// stream): the forward's 2 x B x H 8-byte granules, or the partial-sum BPTT's
// 2 slots x 2 d x B x (H/U) x H 4-byte value positions (sized for H = 768 with U = 32, the largest)
// then (from byte seq_tab_offset, zeroed with the counters) the XCC table of seq_group_local: one
// word per workgroup of the grid (<= the CU count; 1024 words)
static size_t seq_tab_offset(int B) { return (size_t)((2 * (B / 16 + 1) + 1 + 63) / 64 * 256); }
static size_t seq_ring_offset(int B) { return seq_tab_offset(B) + 4096; }
static size_t seq_ring_bytes_bwdp(int B, int H, int U) { return (size_t)2 * 2 * B * (H / U) * H * 4; }
static size_t seq_ring_bytes(int B) {
  const size_t f = (size_t)2 * B * 768 * 8, p = seq_ring_bytes_bwdp(B, 768, 32);
  return f > p ? f : p;
}
// after the ring: the sticky status word (zeroed once by the caller when it allocates ws)
size_t crnn_lstm_seq_status_offset(int B) { return seq_ring_offset(B) + seq_ring_bytes(B); }
size_t crnn_lstm_seq_workspace(int B) { return crnn_lstm_seq_status_offset(B) + 256; }

// crnn_lstm_seq_time_next: events recorded right before / after the NEXT sweep's kernel, so a caller's
// kernel time excludes the counter memset in front of it and the status kernel behind it
static hipEvent_t g_seq_ev[2] = {nullptr, nullptr};
static void seq_time_mark(hipStream_t st, int end) {
  if (g_seq_ev[end] == nullptr) return;
  (void)hipEventRecord(g_seq_ev[end], st);
  g_seq_ev[end] = nullptr;
}

static int seq_accum_status(unsigned* ws, int B, hipStream_t st, int rc) {
  if (rc != 0) return rc;
  hipLaunchKernelGGL(seq_status_accum_kernel, dim3(1), dim3(64), 0, st, ws + 2 * (B / 16 + 1),
                     (unsigned*)((char*)ws + crnn_lstm_seq_status_offset(B)));
  return (int)hipGetLastError();
}

// clears the one-shot events on every path out of a sweep call: an early return (validation, memset failure)
// must not leave handles armed that the caller may destroy before the next sweep records them
struct SeqEvGuard {
  ~SeqEvGuard() { g_seq_ev[0] = g_seq_ev[1] = nullptr; }
};

int crnn_lstm_seq_time_next(void* ev_start, void* ev_end) {
  g_seq_ev[0] = (hipEvent_t)ev_start;
  g_seq_ev[1] = (hipEvent_t)ev_end;
  return 0;
}

int crnn_lstm_seq_fwd(const void* xg, const void* whh, void* hseq, void* gsv, float* csv, unsigned* ws, int B, int T,
                      int H, void* stream) {
  const SeqEvGuard ev_guard;
  hipStream_t st = (hipStream_t)stream;
  int S, U;
  if (!seq_config(B, H, false, S, U)) return crnn_set_error(hipErrorInvalidValue, "lstm_seq: unsupported shape");
  if ((gsv == nullptr) != (csv == nullptr))
    return crnn_set_error(hipErrorInvalidValue, "lstm_seq_fwd: gates and cell are saved together or not at all");
  // counters + error word, and the ring slots this (B, H) uses (tag 0 = not yet written)
  const size_t zero = seq_ring_offset(B) + (crnn_option(CRNN_OPT_LSTM_HANDOFF) ? (size_t)2 * B * H * 8 : 0);
  hipError_t e = hipMemsetAsync(ws, 0, zero, st);
  if (e != hipSuccess) return (int)e;
  unsigned* cnt = ws;
  unsigned* err = ws + 2 * (B / 16 + 1);
  uint2* ring = (uint2*)((char*)ws + seq_ring_offset(B));
  const dim3 grid(2 * (B / S) * (H / U));
  if (grid.x > 1024) return crnn_set_error(hipErrorInvalidValue, "lstm_seq: grid exceeds the XCC table");
  // the forward's granule hand-off gains ~1 % from the XCD-local form, less than the check costs
  // (one extra group hand-off per launch): only the BPTT, whose gather is 4x larger, uses it
  unsigned* xtab = crnn_option(CRNN_OPT_LSTM_L2_HANDOFF) > 1 ? (unsigned*)((char*)ws + seq_tab_offset(B)) : nullptr;
  const bf16 *x = (const bf16*)xg, *w = (const bf16*)whh;
  int rc;
  seq_time_mark(st, 0);
  if (H == 256) rc = launch_fwd<256>(S, U, grid, st, x, w, (bf16*)hseq, (bf16*)gsv, csv, cnt, err, ring, B, T, xtab);
  else if (H == 512) rc = launch_fwd<512>(S, U, grid, st, x, w, (bf16*)hseq, (bf16*)gsv, csv, cnt, err, ring, B, T, xtab);
  else rc = launch_fwd<768>(S, U, grid, st, x, w, (bf16*)hseq, (bf16*)gsv, csv, cnt, err, ring, B, T, xtab);
  seq_time_mark(st, 1);
  return seq_accum_status(ws, B, st, rc);
}

int crnn_lstm_seq_bwd(const void* dhseq, const void* whh_t, const void* gsv, const float* csv, void* dgates,
                      unsigned* ws, int B, int T, int H, void* stream) {
  const SeqEvGuard ev_guard;
  hipStream_t st = (hipStream_t)stream;
  int S, U;
  if (!seq_config(B, H, true, S, U)) return crnn_set_error(hipErrorInvalidValue, "lstm_seq: unsupported shape");
  // counters + error word, and the partial ring this (B, H, U) uses (tag 0 = not yet written)
  const size_t zero = seq_ring_offset(B) + (crnn_option(CRNN_OPT_LSTM_BWD_PART) ? seq_ring_bytes_bwdp(B, H, U) : 0);
  hipError_t e = hipMemsetAsync(ws, 0, zero, st);
  if (e != hipSuccess) return (int)e;
  unsigned* cnt = ws;
  unsigned* err = ws + 2 * (B / 16 + 1);
  uint2* ring = (uint2*)((char*)ws + seq_ring_offset(B));
  const dim3 grid(2 * (B / S) * (H / U));
  if (grid.x > 1024) return crnn_set_error(hipErrorInvalidValue, "lstm_seq: grid exceeds the XCC table");
  unsigned* xtab = crnn_option(CRNN_OPT_LSTM_L2_HANDOFF) ? (unsigned*)((char*)ws + seq_tab_offset(B)) : nullptr;
  const bf16 *dh = (const bf16*)dhseq, *wt = (const bf16*)whh_t, *gv = (const bf16*)gsv;
  int rc;
  seq_time_mark(st, 0);
  if (H == 256) rc = launch_bwd<256>(S, U, grid, st, dh, wt, gv, csv, (bf16*)dgates, cnt, err, ring, B, T, xtab);
  else if (H == 512) rc = launch_bwd<512>(S, U, grid, st, dh, wt, gv, csv, (bf16*)dgates, cnt, err, ring, B, T, xtab);
  else rc = launch_bwd<768>(S, U, grid, st, dh, wt, gv, csv, (bf16*)dgates, cnt, err, ring, B, T, xtab);
  seq_time_mark(st, 1);
  return seq_accum_status(ws, B, st, rc);
}

}  // extern "C"
