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

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// block per sample: e[t] (wave per t), softmax over t, context over c
__global__ __launch_bounds__(256) void attn_context_kernel(const float* __restrict__ projH,
                                                           const float* __restrict__ projh,
                                                           const float* __restrict__ score,
                                                           const float* __restrict__ enc, float* __restrict__ ctx,
                                                           int ldc, float* __restrict__ alpha_out, int T, int H,
                                                           int C, uint32_t thr, float scale,
                                                           unsigned long long seed) {
  extern __shared__ float sm[];  // [T] scores -> weights (after the training-mode dropout)
  const int b = blockIdx.x, lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const float* ph = projh + (size_t)b * H;
  for (int t = w; t < T; t += 4) {
    const float* pH = projH + ((size_t)b * T + t) * H;
    float s = 0.f;
    for (int k = lane; k < H; k += 64) s += score[k] * tanhf(pH[k] + ph[k]);
    s = wave_sum(s);
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
    z = wave_sum(z);
    const float rz = 1.f / z;
    for (int t = lane; t < T; t += 64) {
      const float a = expf(sm[t] - m) * rz;
      // F.dropout(alpha) (model/model.py:38): alpha_out keeps the softmax output for the backward
      sm[t] = thr == 0u ? a : (drop_hash(seed, (unsigned long long)b * T + t) >= thr ? a * scale : 0.f);
      if (alpha_out) alpha_out[(size_t)b * T + t] = a;
    }
  }
  __syncthreads();
  const float* eb = enc + (size_t)b * T * C;
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    float s = 0.f;
    for (int t = 0; t < T; ++t) s += sm[t] * eb[(size_t)t * C + c];
    ctx[(size_t)b * ldc + c] = s;
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

// attention backward, block per sample: context = sum_t alpha_t enc_t, alpha = softmax(e),
// e_t = score . tanh(u_t), u_t = proj_H[b,t] + proj_h[b]:
//   (alpha' = alpha * mask / (1 - p) in training, model/model.py:38)
//   denc[b,t] += alpha'_t dctx ; dalpha_t = mask_t / (1-p) dctx . enc_t ;
//   de_t = alpha_t (dalpha_t - sum alpha dalpha)
//   du_t = de_t score (1 - tanh^2 u_t) -> dprojH[b,t] += du_t, dprojh[b] = sum_t du_t,
//   dscore_part[b] += sum_t de_t tanh(u_t)
__global__ __launch_bounds__(256) void attn_bwd_kernel(const float* __restrict__ dctx, int lddc,
                                                       const float* __restrict__ alpha,
                                                       const float* __restrict__ enc,
                                                       const float* __restrict__ projH,
                                                       const float* __restrict__ projh,
                                                       const float* __restrict__ score, float* __restrict__ denc,
                                                       float* __restrict__ dprojH, float* __restrict__ dprojh,
                                                       float* __restrict__ dscore_part, int T, int H, int C,
                                                       uint32_t thr, float scale, unsigned long long seed) {
  extern __shared__ float sm[];  // [3][T]: dalpha, de, dropped alpha
  float* da = sm;
  float* de = sm + T;
  float* ad = sm + 2 * T;
  const int b = blockIdx.x, lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const float* dc = dctx + (size_t)b * lddc;
  const float* eb = enc + (size_t)b * T * C;
  const float* al = alpha + (size_t)b * T;
  for (int t = threadIdx.x; t < T; t += blockDim.x)  // the forward's dropout mask, from its seed
    ad[t] = thr == 0u ? 1.f : (drop_hash(seed, (unsigned long long)b * T + t) >= thr ? scale : 0.f);
  __syncthreads();
  for (int t = w; t < T; t += 4) {
    float s = 0.f;
    for (int k = lane; k < C; k += 64) s += dc[k] * eb[(size_t)t * C + k];
    s = wave_sum(s);
    if (lane == 0) da[t] = s * ad[t];
  }
  __syncthreads();
  if (w == 0) {
    float z = 0.f;
    for (int t = lane; t < T; t += 64) z += al[t] * da[t];
    z = wave_sum(z);
    for (int t = lane; t < T; t += 64) de[t] = al[t] * (da[t] - z);
  }
  // denc += alpha'_t dctx (alpha' = the dropped weights the forward used)
  float* db_ = denc + (size_t)b * T * C;
  for (int k = threadIdx.x; k < C; k += blockDim.x) {
    const float dk = dc[k];
    for (int t = 0; t < T; ++t) db_[(size_t)t * C + k] += al[t] * ad[t] * dk;
  }
  __syncthreads();
  const float* ph = projh + (size_t)b * H;
  for (int k = threadIdx.x; k < H; k += blockDim.x) {
    float acc_h = 0.f, acc_s = 0.f;
    const float sk = score[k], pk = ph[k];
    for (int t = 0; t < T; ++t) {
      const size_t o = ((size_t)b * T + t) * H + k;
      const float th = tanhf(projH[o] + pk);
      const float du = de[t] * sk * (1.f - th * th);
      dprojH[o] += du;
      acc_h += du;
      acc_s += de[t] * th;
    }
    dprojh[(size_t)b * H + k] = acc_h;
    dscore_part[(size_t)b * H + k] += acc_s;
  }
}

// one-hot input columns of W_ih: dW_ih[r][C + char[b][t]] += dgates[t][b][r] (fp32 atomics)
__global__ void attn_onehot_wgrad_kernel(const float* __restrict__ dgates, const int* __restrict__ text,
                                         int text_ld, int steps, int B, int H4, float* __restrict__ dw_ih, int ldw,
                                         int C) {
  const long n = (long)steps * B * H4;
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < n; e += (long)gridDim.x * blockDim.x) {
    const int r = (int)(e % H4);
    const long tb = e / H4;
    const int b = (int)(tb % B), t = (int)(tb / B);
    const int col = C + text[(size_t)b * text_ld + t];
    atomicAdd(dw_ih + (size_t)r * ldw + col, dgates[e]);
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

}  // namespace

extern "C" {

int crnn_attn_context(const float* projH, const float* projh, const float* score, const float* enc, float* ctx,
                      int ldc, float* alpha, int B, int T, int H, int C, float drop_p, unsigned long long seed,
                      void* stream) {
  if (T <= 0 || T > 4096) return crnn_set_error(hipErrorInvalidValue, "attn_context: T out of range");
  if (!(drop_p >= 0.f && drop_p < 1.f)) return crnn_set_error(hipErrorInvalidValue, "attn_context: p not in [0, 1)");
  hipLaunchKernelGGL(attn_context_kernel, dim3(B), dim3(256), (size_t)T * sizeof(float), (hipStream_t)stream, projH,
                     projh, score, enc, ctx, ldc, alpha, T, H, C, drop_threshold(drop_p), 1.f / (1.f - drop_p), seed);
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
                  const float* projh, const float* score, float* denc, float* dprojH, float* dprojh,
                  float* dscore_part, int B, int T, int H, int C, float drop_p, unsigned long long seed,
                  void* stream) {
  if (T <= 0 || T > 4096) return crnn_set_error(hipErrorInvalidValue, "attn_bwd: T out of range");
  if (!(drop_p >= 0.f && drop_p < 1.f)) return crnn_set_error(hipErrorInvalidValue, "attn_bwd: p not in [0, 1)");
  hipLaunchKernelGGL(attn_bwd_kernel, dim3(B), dim3(256), (size_t)3 * T * sizeof(float), (hipStream_t)stream, dctx,
                     lddc, alpha, enc, projH, projh, score, denc, dprojH, dprojh, dscore_part, T, H, C,
                     drop_threshold(drop_p), 1.f / (1.f - drop_p), seed);
  return (int)hipGetLastError();
}

int crnn_attn_onehot_wgrad(const float* dgates, const int* text, int text_ld, int steps, int B, int H4, float* dw_ih,
                           int ldw, int C, void* stream) {
  hipLaunchKernelGGL(attn_onehot_wgrad_kernel, dim3(grid_for((long)steps * B * H4)), dim3(256), 0,
                     (hipStream_t)stream, dgates, text, text_ld, steps, B, H4, dw_ih, ldw, C);
  return (int)hipGetLastError();
}

int crnn_attn_out(const float* logits, int ldl, int B, int V, int blank, float* probs_t, int ldp, int* ch,
                  void* stream) {
  hipLaunchKernelGGL(attn_out_kernel, dim3(B), dim3(256), 0, (hipStream_t)stream, logits, ldl, V, blank, probs_t, ldp,
                     ch);
  return (int)hipGetLastError();
}

}  // extern "C"
