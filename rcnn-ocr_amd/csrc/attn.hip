// Attention decoder step kernels (fp32): the reference's shipping head, model/model.py:23-148
// (AttentionCell + Attention._greedy_decode / teacher-forced forward), SURVEY §8(f) next-1.
// One decoder step is
//   proj_h   = h W_h2h^T + b_h2h                                   (crnn_gemm_nt)
//   e[b,t]   = score . tanh(proj_H[b,t] + proj_h[b]), alpha = softmax_t(e)
//   context  = sum_t alpha[b,t] enc[b,t]                           (attn_context_kernel)
//   gates    = [context, h] [W_ih[:, :C], W_hh]^T                  (crnn_gemm_nt, one GEMM)
//              + b_ih + b_hh + W_ih[:, C + char]                   (the one-hot input: a column gather)
//   (h, c)   = LSTMCell gates (i, f, g, o)                          (attn_cell_kernel)
//   logits   = h W_gen^T + b_gen, blank masked, argmax -> char      (attn_out_kernel)
// proj_H = enc W_i2h^T is step-invariant and computed once (the reference recomputes it per step).
#include "common.hpp"
#include "crnn_internal.hpp"

namespace {

__device__ __forceinline__ float ldf(const float* p) { return *p; }
__device__ __forceinline__ float ldf(const bf16* p) { return (float)*p; }
// the attention's tanh: libm's for the fp32 parity path, the exp / rcp form (tanh_fast, common.hpp) when the operands
// are bf16 (its ~1e-7 error is far below their 2^-9 rounding)
template <typename TE> __device__ __forceinline__ float att_tanh(float x) {
  if constexpr (sizeof(TE) == 2) return tanh_fast(x);
  else return tanhf(x);
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}
// the same sum without LDS round trips: DPP within each 16-lane row, then the four row sums read into a scalar
// (the per-step attention kernels; __shfl_xor is a ds_bpermute per level)
__device__ __forceinline__ float wave_sum_dpp(float v) {
  v = rowgroup_sum<16>(v);
  const int i = __float_as_int(v);
  return (__int_as_float(__builtin_amdgcn_readlane(i, 0)) + __int_as_float(__builtin_amdgcn_readlane(i, 16))) +
         (__int_as_float(__builtin_amdgcn_readlane(i, 32)) + __int_as_float(__builtin_amdgcn_readlane(i, 48)));
}

// block (1024 threads) per sample: e[t] (wave per t), softmax over t, then context with a thread per channel c
// summing over t from registers. The first 32 enc rows of every thread's channel are loaded before the scores, so
// their round trip hides under the score and softmax phases (the r05 form loaded them after, 4 channel groups in
// turn, 15 us per step at B = 256, T = 32, C = 1024). Loads use clamped indices and masked values (a load under
// a runtime condition costs a branch and a full vmcnt wait).
constexpr int ATT_NT = 1024;
constexpr int ATT_TC = 32;   // enc rows per register pass
// TE: how proj_H and enc are stored (fp32, or bf16 for the bf16 training pass: crnn_attn_context_bf16)
template <typename TE>
__global__ __launch_bounds__(ATT_NT) void attn_context_kernel(const TE* __restrict__ projH,
                                                              const float* __restrict__ projh,
                                                              const float* __restrict__ score,
                                                              const TE* __restrict__ enc, float* __restrict__ ctx,
                                                              int ldc, float* __restrict__ alpha_out, int T, int H,
                                                              int C, uint32_t thr, float scale,
                                                              unsigned long long seed) {
  extern __shared__ float sm[];  // [T] scores -> weights (after the training-mode dropout)
  const int b = blockIdx.x, lane = threadIdx.x & 63, w = threadIdx.x >> 6, tid = threadIdx.x;
  const TE* eb = enc + (size_t)b * T * C;
  float ev[ATT_TC];
  {
    const int cc = min(tid, C - 1);
#pragma unroll
    for (int u = 0; u < ATT_TC; ++u) ev[u] = ldf(eb + (size_t)min(u, T - 1) * C + cc);
  }
  const float* ph = projh + (size_t)b * H;
  for (int t = w; t < T; t += ATT_NT / 64) {
    const TE* pH = projH + ((size_t)b * T + t) * H;
    float s = 0.f;
#pragma unroll 4
    for (int k = lane; k < H; k += 64) s += score[k] * att_tanh<TE>(ldf(pH + k) + ph[k]);
    s = wave_sum_dpp(s);
    if (lane == 0) sm[t] = s;
  }
  __syncthreads();
  if (w == 0) {  // softmax over t (T <= a few hundred)
    float m = -INFINITY;
    for (int t = lane; t < T; t += 64) m = fmaxf(m, sm[t]);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
    float z = 0.f;
    for (int t = lane; t < T; t += 64) z += expf(sm[t] - m);
    z = wave_sum_dpp(z);
    const float rz = 1.f / z;
    for (int t = lane; t < T; t += 64) {
      const float a = expf(sm[t] - m) * rz;
      // F.dropout(alpha) (model/model.py:38): alpha_out keeps the softmax output for the backward
      sm[t] = thr == 0u ? a : (drop_hash(seed, (unsigned long long)b * T + t) >= thr ? a * scale : 0.f);
      if (alpha_out) alpha_out[(size_t)b * T + t] = a;
    }
  }
  __syncthreads();
  for (int c0 = 0; c0 < C; c0 += ATT_NT) {
    const int c = c0 + tid, cc = min(c, C - 1);
    float s = 0.f;
    for (int t0 = 0; t0 < T; t0 += ATT_TC) {
      if (c0 > 0 || t0 > 0) {
#pragma unroll
        for (int u = 0; u < ATT_TC; ++u) ev[u] = ldf(eb + (size_t)min(t0 + u, T - 1) * C + cc);
      }
#pragma unroll
      for (int u = 0; u < ATT_TC; ++u) s += (t0 + u < T ? sm[t0 + u] : 0.f) * ev[u];
    }
    if (c < C) ctx[(size_t)b * ldc + c] = s;
  }
}

__device__ __forceinline__ float sigm(float x) { return 1.f / (1.f + expf(-x)); }

// thread per (b, j): LSTMCell (gate rows i, f, g, o of H each, torch order) with the one-hot
// input folded in as a column of W_ih; h' also goes to the next GEMM's input row and to hs
__global__ void attn_cell_kernel(const float* __restrict__ gates, const float* __restrict__ b_ih,
                                 const float* __restrict__ b_hh, const float* __restrict__ w_ih, int ldw,
                                 const int* __restrict__ ch, int ch_stride, float* __restrict__ h,
                                 float* __restrict__ c, float* __restrict__ hx, int ldx, float* __restrict__ hs,
                                 int ld_hs, float* __restrict__ gact, float* __restrict__ cs, int B, int H, int C) {
  const long n = (long)B * H;
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < n; e += (long)gridDim.x * blockDim.x) {
    const int b = (int)(e / H), j = (int)(e - (long)b * H);
    const int col = C + ch[(size_t)b * ch_stride];
    const float* gr = gates + (size_t)b * 4 * H;
    float v[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int r = q * H + j;
      v[q] = gr[r] + b_ih[r] + b_hh[r] + w_ih[(size_t)r * ldw + col];
    }
    const float ig = sigm(v[0]), fg = sigm(v[1]), gg = tanhf(v[2]), og = sigm(v[3]);
    const float cn = fg * c[e] + ig * gg;
    const float hn = og * tanhf(cn);
    c[e] = cn;
    h[e] = hn;
    hx[(size_t)b * ldx + C + j] = hn;
    if (hs) hs[(size_t)b * ld_hs + j] = hn;
    if (gact) {  // saved for the backward: activated gates, cell state
      float* gr2 = gact + (size_t)b * 4 * H;
      gr2[j] = ig;
      gr2[H + j] = fg;
      gr2[2 * H + j] = gg;
      gr2[3 * H + j] = og;
      cs[e] = cn;
    }
  }
}

// ---- backward (teacher forcing, model/model.py:114-148)
// LSTM cell backward, thread per (b, j): dgates (pre-activation, torch order i f g o), dc_prev
__global__ void attn_cell_bwd_kernel(const float* __restrict__ gact, const float* __restrict__ c_t,
                                     const float* __restrict__ c_prev, const float* __restrict__ dh1, int ld1,
                                     const float* __restrict__ dh2, int ld2, const float* __restrict__ dc,
                                     float* __restrict__ dgates, float* __restrict__ dc_prev, int B, int H) {
  const long n = (long)B * H;
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < n; e += (long)gridDim.x * blockDim.x) {
    const int b = (int)(e / H), j = (int)(e - (long)b * H);
    const float* g = gact + (size_t)b * 4 * H;
    const float ig = g[j], fg = g[H + j], gg = g[2 * H + j], og = g[3 * H + j];
    const float tc = tanhf(c_t[e]);
    // dh = the recurrent gradient (dh1) + this step's output gradient (dh2), both row-strided
    const float dhv = (dh1 ? dh1[(size_t)b * ld1 + j] : 0.f) + (dh2 ? dh2[(size_t)b * ld2 + j] : 0.f);
    const float dcv = (dc ? dc[e] : 0.f) + dhv * og * (1.f - tc * tc);
    const float cp = c_prev ? c_prev[e] : 0.f;
    float* d = dgates + (size_t)b * 4 * H;
    d[j] = dcv * gg * ig * (1.f - ig);
    d[H + j] = dcv * cp * fg * (1.f - fg);
    d[2 * H + j] = dcv * ig * (1.f - gg * gg);
    d[3 * H + j] = dhv * tc * og * (1.f - og);
    dc_prev[e] = dcv * fg;
  }
}

// attention backward, split so that no step touches a [B][T][*] array read-modify-write:
//   context = sum_t' alpha'_t' enc_t', alpha = softmax(e), e_t' = score . tanh(u_t'),
//   u_t' = proj_H[b,t'] + proj_h[b]; alpha' = alpha * mask / (1 - p) (training, model/model.py:40)
// per decoder step (attn_step_bwd_kernel, block per sample):
//   dalpha_t' = mask_t'/(1-p) dctx . enc_t' ; de_t' = alpha_t' (dalpha_t' - sum alpha dalpha) -> de
//   dprojh[b] = sum_t' de_t' score (1 - tanh^2 u_t') ; dscore_part[b] += sum_t' de_t' tanh(u_t')
// after the step loop (all steps at once):
//   denc[b,t'] = sum_t alpha'_t[b,t'] dctx_t[b]                              (attn_denc_kernel)
//   dprojH[b,t',k] = score_k sum_t de_t[b,t'] (1 - tanh^2(proj_H[b,t',k] + proj_h_t[b,k]))
//                                                                            (attn_dprojH_kernel)
__device__ __forceinline__ float keep_scale(uint32_t thr, float scale, unsigned long long seed,
                                            unsigned long long i) {
  return thr == 0u ? 1.f : (drop_hash(seed, i) >= thr ? scale : 0.f);
}

template <typename TE>
__global__ __launch_bounds__(ATT_NT) void attn_step_bwd_kernel(const float* __restrict__ dctx, int lddc,
                                                               const float* __restrict__ alpha,
                                                               const TE* __restrict__ enc,
                                                               const TE* __restrict__ projH,
                                                               const float* __restrict__ projh,
                                                               const float* __restrict__ score,
                                                               float* __restrict__ de_out, float* __restrict__ dprojh,
                                                               float* __restrict__ dscore_part, int T, int H, int C,
                                                               uint32_t thr, float scale, unsigned long long seed) {
  extern __shared__ float sm[];  // [2][T]: dalpha, de
  __shared__ float red[2][4][256];
  float* da = sm;
  float* de = sm + T;
  const int b = blockIdx.x, lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const float* dc = dctx + (size_t)b * lddc;
  const TE* eb = enc + (size_t)b * T * C;
  const float* al = alpha + (size_t)b * T;
  // dalpha: wave w owns t = w, w + 16, ...; per pass over 512 channels a lane holds its 8 dctx values in
  // registers and issues the enc loads of TWO rows before any sum (clamped indices, masked values; 16 channels
  // per lane spilled at the 128-register budget of 1024-thread blocks)
  constexpr int KC = 8;
  for (int k0 = 0; k0 < C; k0 += 64 * KC) {
    float dcr[KC];
#pragma unroll
    for (int j = 0; j < KC; ++j) {
      const int k = k0 + lane + 64 * j;
      const float v = dc[min(k, C - 1)];
      dcr[j] = k < C ? v : 0.f;
    }
    for (int t = w; t < T; t += 2 * (ATT_NT / 64)) {
      const int t2 = t + ATT_NT / 64;
      const TE* e1 = eb + (size_t)t * C;
      const TE* e2 = eb + (size_t)min(t2, T - 1) * C;
      float x1[KC], x2[KC];
#pragma unroll
      for (int j = 0; j < KC; ++j) {
        const int k = min(k0 + lane + 64 * j, C - 1);
        x1[j] = ldf(e1 + k);
        x2[j] = ldf(e2 + k);
      }
      float s1 = 0.f, s2 = 0.f;
#pragma unroll
      for (int j = 0; j < KC; ++j) {
        s1 += dcr[j] * x1[j];
        s2 += dcr[j] * x2[j];
      }
      s1 = wave_sum_dpp(s1);
      s2 = wave_sum_dpp(s2);
      if (lane == 0) {
        da[t] = (k0 > 0 ? da[t] : 0.f) + s1;
        if (t2 < T) da[t2] = (k0 > 0 ? da[t2] : 0.f) + s2;
      }
    }
  }
  __syncthreads();
  if (w == 0)
    for (int t = lane; t < T; t += 64) da[t] *= keep_scale(thr, scale, seed, (unsigned long long)b * T + t);
  __syncthreads();
  if (w == 0) {
    float z = 0.f;
    for (int t = lane; t < T; t += 64) z += al[t] * da[t];
    z = wave_sum_dpp(z);
    for (int t = lane; t < T; t += 64) {
      const float v = al[t] * (da[t] - z);
      de[t] = v;
      de_out[(size_t)b * T + t] = v;
    }
  }
  __syncthreads();
  const float* ph = projh + (size_t)b * H;
  const TE* pH = projH + (size_t)b * T * H;
  const int kq = threadIdx.x & 255, tq = threadIdx.x >> 8;
  for (int k0 = 0; k0 < H; k0 += 256) {
    const int k = k0 + kq;
    float acc_h = 0.f, acc_s = 0.f;
    if (k < H) {
      const float pk = ph[k];
#pragma unroll 8
      for (int t = tq; t < T; t += 4) {
        const float th = att_tanh<TE>(ldf(pH + (size_t)t * H + k) + pk);
        acc_h += de[t] * (1.f - th * th);
        acc_s += de[t] * th;
      }
    }
    red[0][tq][kq] = acc_h;
    red[1][tq][kq] = acc_s;
    __syncthreads();
    if (tq == 0 && k < H) {
      dprojh[(size_t)b * H + k] = (((red[0][0][kq] + red[0][1][kq]) + red[0][2][kq]) + red[0][3][kq]) * score[k];
      dscore_part[(size_t)b * H + k] += ((red[1][0][kq] + red[1][1][kq]) + red[1][2][kq]) + red[1][3][kq];
    }
    __syncthreads();
  }
}

// block per (sample, 256 channels): dctx of every step and the step's alpha' staged in LDS
__global__ __launch_bounds__(256) void attn_denc_kernel(const float* __restrict__ dctx, int lddc,
                                                        const float* __restrict__ alpha, int steps, int B, int T,
                                                        int C, uint32_t thr, float scale,
                                                        unsigned long long seed, float* __restrict__ denc) {
  extern __shared__ float sm[];  // [steps][256] dctx, [steps][T] alpha'
  float* dcs = sm;
  float* as = sm + steps * 256;
  const int b = blockIdx.x, c0 = blockIdx.y * 256, c = c0 + threadIdx.x;
  for (int i = threadIdx.x; i < steps * T; i += blockDim.x) {
    const int t = i / T, tp = i - t * T;
    as[i] = alpha[((size_t)t * B + b) * T + tp] *
            keep_scale(thr, scale, seed + (unsigned long long)t, (unsigned long long)b * T + tp);
  }
  for (int t = 0; t < steps; ++t) dcs[t * 256 + threadIdx.x] = c < C ? dctx[((size_t)t * B + b) * lddc + c] : 0.f;
  __syncthreads();
  if (c >= C) return;
  float* out = denc + (size_t)b * T * C + c;
  for (int tp = 0; tp < T; ++tp) {
    float acc = 0.f;
    for (int t = 0; t < steps; ++t) acc += as[t * T + tp] * dcs[t * 256 + threadIdx.x];
    out[(size_t)tp * C] = acc;
  }
}

// block per (sample b, 256 k): the sample's de rows of every step staged in LDS; a thread holds proj_H[b, t', k]
// for 32 t' and proj_h[t][b][k] for 32 steps in registers (all loads issued before any tanh) and sums over the steps
// in step order. (The r05 form, a thread per (b, t', k) re-reading proj_h for every t', took 137 us at B = 256,
// T = 32.) TE = bf16: proj_H stored as bf16 and the exp / rcp tanh (the bf16 training pass).
template <typename TE>
__global__ __launch_bounds__(256) void attn_dprojH_kernel(const float* __restrict__ projh, const float* __restrict__ de,
                                                          const TE* __restrict__ projH,
                                                          const float* __restrict__ score, int steps, int B, int T,
                                                          int H, float* __restrict__ dprojH) {
  extern __shared__ float sde[];  // [steps][T]
  const int b = blockIdx.x, k = blockIdx.y * 256 + threadIdx.x;
  for (int i = threadIdx.x; i < steps * T; i += 256) {
    const int t = i / T, tp = i - t * T;
    sde[i] = de[((size_t)t * B + b) * T + tp];
  }
  __syncthreads();
  if (k >= H) return;
  for (int t0 = 0; t0 < T; t0 += 32) {
    float u[32], acc[32];
#pragma unroll
    for (int j = 0; j < 32; ++j) {
      u[j] = ldf(projH + ((size_t)b * T + min(t0 + j, T - 1)) * H + k);
      acc[j] = 0.f;
    }
    for (int s0 = 0; s0 < steps; s0 += 32) {
      float p[32];
#pragma unroll
      for (int q = 0; q < 32; ++q) p[q] = projh[((size_t)min(s0 + q, steps - 1) * B + b) * H + k];
      const int ns = min(32, steps - s0);
      for (int q = 0; q < ns; ++q) {
        const float* d = sde + (s0 + q) * T + t0;
#pragma unroll
        for (int j = 0; j < 32; ++j) {
          const float th = att_tanh<TE>(u[j] + p[q]);
          acc[j] += (t0 + j < T ? d[j] : 0.f) * (1.f - th * th);
        }
      }
    }
    const float sk = score[k];
#pragma unroll
    for (int j = 0; j < 32; ++j)
      if (t0 + j < T) dprojH[((size_t)b * T + t0 + j) * H + k] = acc[j] * sk;
  }
}

// teacher-forcing one-hot rows: X[t][b][col0 + text[b][t]] = 1 (X zeroed by the caller); the
// backward's gradient of W_ih's one-hot columns is then part of the [context | h | onehot] GEMM
__global__ void attn_onehot_rows_kernel(const int* __restrict__ text, int text_ld, int steps, int B, int V,
                                        float* __restrict__ X, int ldx, int col0) {
  const long n = (long)steps * B;
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < n; e += (long)gridDim.x * blockDim.x) {
    const int t = (int)(e / B), b = (int)(e - (long)t * B);
    const int v = text[(size_t)b * text_ld + t];
    if (v >= 0 && v < V) X[(size_t)e * ldx + col0 + v] = 1.f;
  }
}

// block per sample: blank masked to -1e4 (model/model.py:87-89), logits to probs[:, t], argmax
// (first maximum, as torch.argmax) -> next input char
__global__ __launch_bounds__(256) void attn_out_kernel(const float* __restrict__ logits, int ldl, int V, int blank,
                                                       float* __restrict__ probs_t, int ldp, int* __restrict__ ch) {
  __shared__ float bv[256];
  __shared__ int bi[256];
  const int b = blockIdx.x;
  float best = -INFINITY;
  int arg = 0x7fffffff;
  for (int v = threadIdx.x; v < V; v += blockDim.x) {
    float x = logits[(size_t)b * ldl + v];
    if (v == blank) x = -1e4f;
    if (probs_t) probs_t[(size_t)b * ldp + v] = x;
    if (x > best) {
      best = x;
      arg = v;
    }
  }
  bv[threadIdx.x] = best;
  bi[threadIdx.x] = arg;
  __syncthreads();
  for (int s = blockDim.x / 2; s > 0; s >>= 1) {
    if (threadIdx.x < s) {
      const float o = bv[threadIdx.x + s];
      const int oi = bi[threadIdx.x + s];
      if (o > bv[threadIdx.x] || (o == bv[threadIdx.x] && oi < bi[threadIdx.x])) {
        bv[threadIdx.x] = o;
        bi[threadIdx.x] = oi;
      }
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) ch[b] = bi[0];
}

// ---- the attention head's loss: nn.CrossEntropyLoss(ignore_index=PAD) over [M = B*steps][V]
// (training/train.py:289,503), mean over the rows whose target != ignore_index
__global__ __launch_bounds__(256) void xent_count_kernel(const int* __restrict__ tgt, int M, int ignore,
                                                         float* __restrict__ inv_n) {
  __shared__ int part[4];
  int n = 0;
  for (int r = threadIdx.x; r < M; r += blockDim.x) n += tgt[r] != ignore;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) n += __shfl_xor(n, o);
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = n;
  __syncthreads();
  if (threadIdx.x == 0) inv_n[0] = 1.f / (float)(part[0] + part[1] + part[2] + part[3]);
}

// wave per row: log-sum-exp, loss_row = (lse - x[tgt]) / n, d = (softmax - onehot) / n (0 if ignored)
__global__ __launch_bounds__(256) void xent_rows_kernel(const float* __restrict__ x, int ldx,
                                                        const int* __restrict__ tgt, int M, int V, int ignore,
                                                        const float* __restrict__ inv_n, float* __restrict__ lrow,
                                                        float* __restrict__ d, int ldd) {
  const int lane = threadIdx.x & 63;
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= M) return;
  const float* xr = x + (size_t)r * ldx;
  const int t = tgt[r];
  const bool on = t != ignore;
  const float sc = on ? inv_n[0] : 0.f;
  float m = -INFINITY;
  for (int v = lane; v < V; v += 64) m = fmaxf(m, xr[v]);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
  float z = 0.f;
  for (int v = lane; v < V; v += 64) z += expf(xr[v] - m);
  z = wave_sum(z);
  const float lse = m + logf(z), rz = 1.f / z;
  if (d)
    for (int v = lane; v < V; v += 64) d[(size_t)r * ldd + v] = (expf(xr[v] - m) * rz - (v == t ? 1.f : 0.f)) * sc;
  if (lane == 0) lrow[r] = on ? (lse - xr[t]) * sc : 0.f;
}

__global__ __launch_bounds__(256) void xent_sum_kernel(const float* __restrict__ lrow, int M,
                                                       float* __restrict__ loss) {
  __shared__ float part[4];
  float s = 0.f;
  for (int r = threadIdx.x; r < M; r += blockDim.x) s += lrow[r];
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) loss[0] = part[0] + part[1] + part[2] + part[3];
}

}  // namespace

extern "C" {

int crnn_attn_context(const float* projH, const float* projh, const float* score, const float* enc, float* ctx,
                      int ldc, float* alpha, int B, int T, int H, int C, float drop_p, unsigned long long seed,
                      void* stream) {
  if (T <= 0 || T > 4096) return crnn_set_error(hipErrorInvalidValue, "attn_context: T out of range");
  if (!(drop_p >= 0.f && drop_p < 1.f)) return crnn_set_error(hipErrorInvalidValue, "attn_context: p not in [0, 1)");
  hipLaunchKernelGGL(attn_context_kernel<float>, dim3(B), dim3(ATT_NT), (size_t)T * sizeof(float), (hipStream_t)stream,
                     projH, projh, score, enc, ctx, ldc, alpha, T, H, C, drop_threshold(drop_p), 1.f / (1.f - drop_p),
                     seed);
  return (int)hipGetLastError();
}

int crnn_attn_context_bf16(const void* projH, const float* projh, const float* score, const void* enc, float* ctx,
                           int ldc, float* alpha, int B, int T, int H, int C, float drop_p, unsigned long long seed,
                           void* stream) {
  if (T <= 0 || T > 4096) return crnn_set_error(hipErrorInvalidValue, "attn_context: T out of range");
  if (!(drop_p >= 0.f && drop_p < 1.f)) return crnn_set_error(hipErrorInvalidValue, "attn_context: p not in [0, 1)");
  hipLaunchKernelGGL(attn_context_kernel<bf16>, dim3(B), dim3(ATT_NT), (size_t)T * sizeof(float), (hipStream_t)stream,
                     (const bf16*)projH, projh, score, (const bf16*)enc, ctx, ldc, alpha, T, H, C,
                     drop_threshold(drop_p), 1.f / (1.f - drop_p), seed);
  return (int)hipGetLastError();
}

int crnn_attn_cell(const float* gates, const float* b_ih, const float* b_hh, const float* w_ih, int ldw, const int* ch,
                   int ch_stride, float* h, float* c, float* hx, int ldx, float* hs, int ld_hs, float* gact, float* cs,
                   int B, int H, int C, void* stream) {
  hipLaunchKernelGGL(attn_cell_kernel, dim3(grid_for((long)B * H)), dim3(256), 0, (hipStream_t)stream, gates, b_ih,
                     b_hh, w_ih, ldw, ch, ch_stride, h, c, hx, ldx, hs, ld_hs, gact, cs, B, H, C);
  return (int)hipGetLastError();
}

int crnn_attn_cell_bwd(const float* gact, const float* c_t, const float* c_prev, const float* dh1, int ld1,
                       const float* dh2, int ld2, const float* dc, float* dgates, float* dc_prev, int B, int H,
                       void* stream) {
  hipLaunchKernelGGL(attn_cell_bwd_kernel, dim3(grid_for((long)B * H)), dim3(256), 0, (hipStream_t)stream, gact, c_t,
                     c_prev, dh1, ld1, dh2, ld2, dc, dgates, dc_prev, B, H);
  return (int)hipGetLastError();
}

int crnn_attn_bwd(const float* dctx, int lddc, const float* alpha, const float* enc, const float* projH,
                  const float* projh, const float* score, float* de, float* dprojh, float* dscore_part, int B, int T,
                  int H, int C, float drop_p, unsigned long long seed, void* stream) {
  if (T <= 0 || T > 4096) return crnn_set_error(hipErrorInvalidValue, "attn_bwd: T out of range");
  if (!(drop_p >= 0.f && drop_p < 1.f)) return crnn_set_error(hipErrorInvalidValue, "attn_bwd: p not in [0, 1)");
  hipLaunchKernelGGL(attn_step_bwd_kernel<float>, dim3(B), dim3(ATT_NT), (size_t)2 * T * sizeof(float),
                     (hipStream_t)stream, dctx, lddc, alpha, enc, projH, projh, score, de, dprojh, dscore_part, T, H, C,
                     drop_threshold(drop_p), 1.f / (1.f - drop_p), seed);
  return (int)hipGetLastError();
}

int crnn_attn_bwd_bf16(const float* dctx, int lddc, const float* alpha, const void* enc, const void* projH,
                       const float* projh, const float* score, float* de, float* dprojh, float* dscore_part, int B,
                       int T, int H, int C, float drop_p, unsigned long long seed, void* stream) {
  if (T <= 0 || T > 4096) return crnn_set_error(hipErrorInvalidValue, "attn_bwd: T out of range");
  if (!(drop_p >= 0.f && drop_p < 1.f)) return crnn_set_error(hipErrorInvalidValue, "attn_bwd: p not in [0, 1)");
  hipLaunchKernelGGL(attn_step_bwd_kernel<bf16>, dim3(B), dim3(ATT_NT), (size_t)2 * T * sizeof(float),
                     (hipStream_t)stream, dctx, lddc, alpha, (const bf16*)enc, (const bf16*)projH, projh, score, de,
                     dprojh, dscore_part, T, H, C, drop_threshold(drop_p), 1.f / (1.f - drop_p), seed);
  return (int)hipGetLastError();
}

int crnn_attn_denc(const float* dctx, int lddc, const float* alpha, int steps, int B, int T, int C, float drop_p,
                   unsigned long long seed, float* denc, void* stream) {
  const size_t lds = (size_t)steps * (256 + T) * sizeof(float);
  if (steps <= 0 || T <= 0 || lds > 64 * 1024)
    return crnn_set_error(hipErrorInvalidValue, "attn_denc: steps * (256 + T) exceeds the LDS stage");
  if (!(drop_p >= 0.f && drop_p < 1.f)) return crnn_set_error(hipErrorInvalidValue, "attn_denc: p not in [0, 1)");
  hipLaunchKernelGGL(attn_denc_kernel, dim3(B, (C + 255) / 256), dim3(256), lds, (hipStream_t)stream, dctx, lddc,
                     alpha, steps, B, T, C, drop_threshold(drop_p), 1.f / (1.f - drop_p), seed, denc);
  return (int)hipGetLastError();
}

int crnn_attn_dproj_enc(const float* projh, const float* de, const float* projH, const float* score, int steps, int B,
                     int T, int H, float* dprojH, void* stream) {
  const size_t lds = (size_t)steps * T * sizeof(float);
  if (steps <= 0 || T <= 0 || lds > 64 * 1024)
    return crnn_set_error(hipErrorInvalidValue, "attn_dproj_enc: steps * T exceeds the LDS stage");
  hipLaunchKernelGGL(attn_dprojH_kernel<float>, dim3(B, (H + 255) / 256), dim3(256), lds, (hipStream_t)stream, projh,
                     de, projH, score, steps, B, T, H, dprojH);
  return (int)hipGetLastError();
}

int crnn_attn_dproj_enc_bf16(const float* projh, const float* de, const void* projH, const float* score, int steps,
                             int B, int T, int H, float* dprojH, void* stream) {
  const size_t lds = (size_t)steps * T * sizeof(float);
  if (steps <= 0 || T <= 0 || lds > 64 * 1024)
    return crnn_set_error(hipErrorInvalidValue, "attn_dproj_enc: steps * T exceeds the LDS stage");
  hipLaunchKernelGGL(attn_dprojH_kernel<bf16>, dim3(B, (H + 255) / 256), dim3(256), lds, (hipStream_t)stream, projh,
                     de, (const bf16*)projH, score, steps, B, T, H, dprojH);
  return (int)hipGetLastError();
}

int crnn_attn_onehot_rows(const int* text, int text_ld, int steps, int B, int V, float* X, int ldx, int col0,
                          void* stream) {
  hipLaunchKernelGGL(attn_onehot_rows_kernel, dim3(grid_for((long)steps * B)), dim3(256), 0, (hipStream_t)stream,
                     text, text_ld, steps, B, V, X, ldx, col0);
  return (int)hipGetLastError();
}

int crnn_attn_out(const float* logits, int ldl, int B, int V, int blank, float* probs_t, int ldp, int* ch,
                  void* stream) {
  hipLaunchKernelGGL(attn_out_kernel, dim3(B), dim3(256), 0, (hipStream_t)stream, logits, ldl, V, blank, probs_t, ldp,
                     ch);
  return (int)hipGetLastError();
}

int crnn_attn_xent(const float* logits, int ldl, const int* targets, int M, int V, int ignore_index, float* loss,
                   float* dlogits, int ldd, float* ws, void* stream) {
  if (M <= 0 || V <= 0) return crnn_set_error(hipErrorInvalidValue, "attn_xent: empty input");
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(xent_count_kernel, dim3(1), dim3(256), 0, st, targets, M, ignore_index, ws);
  hipLaunchKernelGGL(xent_rows_kernel, dim3((M + 3) / 4), dim3(256), 0, st, logits, ldl, targets, M, V, ignore_index,
                     ws, ws + 1, dlogits, ldd);
  hipLaunchKernelGGL(xent_sum_kernel, dim3(1), dim3(256), 0, st, ws + 1, M, loss);
  return (int)hipGetLastError();
}

}  // extern "C"
