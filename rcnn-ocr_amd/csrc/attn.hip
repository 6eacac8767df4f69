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
                                                           int C) {
  extern __shared__ float sm[];  // [T] scores -> weights
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
      sm[t] = a;
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
                                 int ld_hs, int B, int H, int C) {
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
    const float cn = sigm(v[1]) * c[e] + sigm(v[0]) * tanhf(v[2]);
    const float hn = sigm(v[3]) * tanhf(cn);
    c[e] = cn;
    h[e] = hn;
    hx[(size_t)b * ldx + C + j] = hn;
    if (hs) hs[(size_t)b * ld_hs + j] = hn;
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
                      int ldc, float* alpha, int B, int T, int H, int C, void* stream) {
  if (T <= 0 || T > 4096) return crnn_set_error(hipErrorInvalidValue, "attn_context: T out of range");
  hipLaunchKernelGGL(attn_context_kernel, dim3(B), dim3(256), (size_t)T * sizeof(float), (hipStream_t)stream, projH,
                     projh, score, enc, ctx, ldc, alpha, T, H, C);
  return (int)hipGetLastError();
}

int crnn_attn_cell(const float* gates, const float* b_ih, const float* b_hh, const float* w_ih, int ldw, const int* ch,
                   int ch_stride, float* h, float* c, float* hx, int ldx, float* hs, int ld_hs, int B, int H, int C,
                   void* stream) {
  hipLaunchKernelGGL(attn_cell_kernel, dim3(grid_for((long)B * H)), dim3(256), 0, (hipStream_t)stream, gates, b_ih,
                     b_hh, w_ih, ldw, ch, ch_stride, h, c, hx, ldx, hs, ld_hs, B, H, C);
  return (int)hipGetLastError();
}

int crnn_attn_out(const float* logits, int ldl, int B, int V, int blank, float* probs_t, int ldp, int* ch,
                  void* stream) {
  hipLaunchKernelGGL(attn_out_kernel, dim3(B), dim3(256), 0, (hipStream_t)stream, logits, ldl, V, blank, probs_t, ldp,
                     ch);
  return (int)hipGetLastError();
}

}  // extern "C"
