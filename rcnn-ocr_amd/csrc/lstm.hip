// Bidirectional LSTM (nn.LSTM(in, H, bidirectional=True, batch_first=True),
// model/model.py:152-163; gate order i,f,g,o; h0 = c0 = 0) — recurrence and BPTT.
//
// The input projection x W_ih^T + b_ih + b_hh for all T and both directions is
// one GEMM (crnn_gemm_nt) done before the recurrence. Each recurrent step is
// one MFMA GEMM  h_{t-1} [B x H] . W_hh'^T [H x 4H]  whose epilogue finishes
// the cell: weights are packed with gate-interleaved rows (packed row 4j+q =
// reference row q*H+j) so the swapped-MFMA accumulator layout hands every lane
// the four gate pre-activations (i,f,g,o) of one (b, j) — sigmoid/tanh, the
// cell update and h are computed in registers with no extra pass.
// BPTT mirrors it: step s's GEMM dgates_{s-1} . W_hh' produces dh_rec and its
// epilogue runs the cell backward of step s (again one lane per (b, 4 units)).
#include "gemm.hpp"
#include "gemm_oneshot.hpp"
#include "gemm256.hpp"
#include "crnn_internal.hpp"

using namespace gemm;

namespace {

// ---------------------------------------------------------------- forward step
template <typename T> struct StepFwdEpi {
  static constexpr bool kStats = false;
  const T* xg;   // [B][T][2][4H]
  T* hseq;       // [B][T][2H]
  T* gsv;        // [2][T][B][4H]
  float* csv;    // [2][T][B][H]
  int B, Tn, H, d, t, tp, first;
  __device__ __forceinline__ void store(int b, int n, f32x4 v, int) const {
    if (b >= B || n >= 4 * H) return;
    const int j = n >> 2, H4 = 4 * H;
    f32x4 x = ld4f<T>(xg + ((size_t)b * Tn + t) * 2 * H4 + d * H4 + n);
    v += x;
    float ig = sigmoidf_(v[0]), fg = sigmoidf_(v[1]), gg = tanhf_(v[2]), og = sigmoidf_(v[3]);
    float cp = first ? 0.f : csv[((size_t)(d * Tn + tp) * B + b) * H + j];
    float c = fg * cp + ig * gg;
    float h = og * tanhf_(c);
    csv[((size_t)(d * Tn + t) * B + b) * H + j] = c;
    st4<T>(gsv + ((size_t)(d * Tn + t) * B + b) * H4 + n, f32x4{ig, fg, gg, og});
    hseq[((size_t)b * Tn + t) * 2 * H + d * H + j] = fromf<T>(h);
  }
  __device__ __forceinline__ void stats(int, int, f32x4, f32x4) const {}
};

// both directions in one launch (batch index = direction)
template <typename T>
int step_fwd_t(const void* xg, const void* whh, void* hseq, void* gsv, float* csv, int B, int Tn, int H, int s,
               hipStream_t st) {
  Pair<RowMajorK<T>> la, lb;
  EpiPair<StepFwdEpi<T>> ep;
  for (int d = 0; d < 2; ++d) {
    int t = d == 0 ? s : Tn - 1 - s;
    int tp = d == 0 ? t - 1 : t + 1;
    int first = s == 0;
    // A: h_{t-1} rows b, k = j  (all-zero rows at the first step)
    RowMajorK<T> a{(const T*)hseq + (size_t)(first ? 0 : tp) * 2 * H + d * H, Tn * 2 * H, first ? 0 : B, H};
    RowMajorK<T> b{(const T*)whh + (size_t)d * 4 * H * H, H, 4 * H, H};
    StepFwdEpi<T> e{(const T*)xg, (T*)hseq, (T*)gsv, csv, B, Tn, H, d, t, tp, first};
    (d ? la.b : la.a) = a;
    (d ? lb.b : lb.a) = b;
    (d ? ep.b : ep.a) = e;
  }
  if constexpr (sizeof(T) == 2) {
    if (H <= 512 && H % 16 == 0) return launch_oneshot<512>(la, lb, ep, B, 4 * H, H, 1, st, 2);  // one K burst
  }
  if ((long)B * 4 * H >= 64L * 64 * 256) return launch<T, 64, 64>(la, lb, ep, B, 4 * H, H, 1, st, 2);
  return launch<T, 32, 32>(la, lb, ep, B, 4 * H, H, 1, st, 2);
}

// ---------------------------------------------------------------- backward step
// cell backward for unit u of (d, t, b), given dh_rec (recurrent part of dh)
template <typename T>
__device__ __forceinline__ void cell_bwd(const T* dhseq, const T* gsv, const float* csv, T* dgates, float* dc, int B,
                                         int Tn, int H, int d, int t, int b, int u, float dh_rec) {
  const int H4 = 4 * H;
  const size_t gi = ((size_t)(d * Tn + t) * B + b) * H4 + 4 * u;
  f32x4 g = ld4f<T>(gsv + gi);
  float ig = g[0], fg = g[1], gg = g[2], og = g[3];
  float c = csv[((size_t)(d * Tn + t) * B + b) * H + u];
  int tf = d == 0 ? t - 1 : t + 1;  // previous time in the forward recurrence
  bool has_prev = d == 0 ? t > 0 : t < Tn - 1;
  float cp = has_prev ? csv[((size_t)(d * Tn + tf) * B + b) * H + u] : 0.f;
  float dh = dh_rec + tof(dhseq[((size_t)b * Tn + t) * 2 * H + d * H + u]);
  float tc = tanhf_(c);
  float* dcp = dc + ((size_t)d * B + b) * H + u;
  float dcv = *dcp + dh * og * (1.f - tc * tc);
  float do_ = dh * tc;
  float di = dcv * gg, dg = dcv * ig, df = dcv * cp;
  *dcp = dcv * fg;
  st4<T>(dgates + gi, f32x4{di * ig * (1.f - ig), df * fg * (1.f - fg), dg * (1.f - gg * gg), do_ * og * (1.f - og)});
}

template <typename T> struct StepBwdEpi {
  static constexpr bool kStats = false;
  const T* dhseq;
  const T* gsv;
  const float* csv;
  T* dgates;
  float* dc;
  int B, Tn, H, d, t;
  __device__ __forceinline__ void store(int b, int n, f32x4 v, int) const {
    if (b >= B || n >= H) return;
#pragma unroll
    for (int r = 0; r < 4; ++r) cell_bwd<T>(dhseq, gsv, csv, dgates, dc, B, Tn, H, d, t, b, n + r, v[r]);
  }
  __device__ __forceinline__ void stats(int, int, f32x4, f32x4) const {}
};

template <typename T>
__global__ void bptt_init_kernel(const T* dhseq, const T* gsv, const float* csv, T* dgates, float* dc, int B, int Tn,
                                 int H) {
  const long n = 2L * B * H;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    int u = (int)(i % H);
    long q = i / H;
    int b = (int)(q % B), d = (int)(q / B);
    dc[((size_t)d * B + b) * H + u] = 0.f;
    int t = d == 0 ? Tn - 1 : 0;
    cell_bwd<T>(dhseq, gsv, csv, dgates, dc, B, Tn, H, d, t, b, u, 0.f);
  }
}

// ---- bf16 BPTT step as split-K one-shot GEMM (dh_rec partials) + sum-and-cell-backward pass
constexpr int BPTT_KC = 512;
inline int bptt_splits(int H) { return (4 * H + BPTT_KC - 1) / BPTT_KC; }

struct BpttSlabEpi {
  static constexpr bool kStats = false;
  float* ws;  // [nsplit][2][B][H]
  int B, H, d;
  __device__ __forceinline__ void set_batch(int bz) { d = bz; }
  __device__ __forceinline__ void store(int b, int n, f32x4 v, int kz) const {
    if (b < B && n < H) *reinterpret_cast<f32x4*>(ws + (((size_t)kz * 2 + d) * B + b) * H + n) = v;
  }
  __device__ __forceinline__ void stats(int, int, f32x4, f32x4) const {}
};

template <typename T>
__global__ void bptt_cell_kernel(const float* __restrict__ ws, int nsplit, const T* dhseq, const T* gsv,
                                 const float* csv, T* dgates, float* dc, int B, int Tn, int H, int s) {
  const long n = 2L * B * H;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const int u = (int)(i % H);
    const long q = i / H;
    const int b = (int)(q % B), d = (int)(q / B);
    float dh = 0.f;
    for (int z = 0; z < nsplit; ++z) dh += ws[(((size_t)z * 2 + d) * B + b) * H + u];
    const int t = d == 0 ? Tn - 1 - s : s;
    cell_bwd<T>(dhseq, gsv, csv, dgates, dc, B, Tn, H, d, t, b, u, dh);
  }
}

int step_bwd_oneshot(const bf16* dhseq, const bf16* whh_t, const bf16* gsv, const float* csv, bf16* dgates, float* dc,
                     float* ws, int B, int Tn, int H, int s, hipStream_t st) {
  Pair<RowMajorK<bf16>> la, lb;
  for (int d = 0; d < 2; ++d) {
    const int t = d == 0 ? Tn - 1 - s : s;  // time processed now
    const int tn = d == 0 ? t + 1 : t - 1;  // time processed at step s-1
    RowMajorK<bf16> a{dgates + (size_t)(d * Tn + tn) * B * 4 * H, 4 * H, B, 4 * H};  // dgates of step s-1
    RowMajorK<bf16> b{whh_t + (size_t)d * H * 4 * H, 4 * H, H, 4 * H};               // W_hh'^T [H][4H]
    (d ? la.b : la.a) = a;
    (d ? lb.b : lb.a) = b;
  }
  const int ns = bptt_splits(H);
  BpttSlabEpi ep{ws, B, H, 0};
  int rc = launch_oneshot<BPTT_KC>(la, lb, ep, B, H, 4 * H, ns, st, 2);
  if (rc) return rc;
  const long n = 2L * B * H;
  hipLaunchKernelGGL(bptt_cell_kernel<bf16>, dim3(grid_for(n)), dim3(256), 0, st, ws, ns, dhseq, gsv, csv, dgates, dc,
                     B, Tn, H, s);
  return (int)hipGetLastError();
}

template <typename T>
int step_bwd_t(const void* dhseq, const void* whh, const void* gsv, const float* csv, void* dgates, float* dc, int B,
               int Tn, int H, int s, hipStream_t st) {
  if (s == 0) {
    long n = 2L * B * H;
    hipLaunchKernelGGL(bptt_init_kernel<T>, dim3(grid_for(n)), dim3(256), 0, st, (const T*)dhseq, (const T*)gsv, csv,
                       (T*)dgates, dc, B, Tn, H);
    return (int)hipGetLastError();
  }
  Pair<RowMajorK<T>> la;
  Pair<ColMajorK<T>> lb;
  EpiPair<StepBwdEpi<T>> ep;
  for (int d = 0; d < 2; ++d) {
    int t = d == 0 ? Tn - 1 - s : s;  // time processed now
    int tn = d == 0 ? t + 1 : t - 1;  // time processed at step s-1
    RowMajorK<T> a{(const T*)dgates + (size_t)(d * Tn + tn) * B * 4 * H, 4 * H, B, 4 * H};
    ColMajorK<T> b{(const T*)whh + (size_t)d * 4 * H * H, H, H, 4 * H};
    StepBwdEpi<T> e{(const T*)dhseq, (const T*)gsv, csv, (T*)dgates, dc, B, Tn, H, d, t};
    (d ? la.b : la.a) = a;
    (d ? lb.b : lb.a) = b;
    (d ? ep.b : ep.a) = e;
  }
  if ((long)B * H >= 64L * 64 * 256) return launch<T, 64, 64>(la, lb, ep, B, H, 4 * H, 1, st, 2);
  return launch<T, 32, 32>(la, lb, ep, B, H, 4 * H, 1, st, 2);
}

// ---------------------------------------------------------------- weight grads
// A: dgates as rows g' (packed), k = t*B + b : element at dg[k*4H + g']
// B (dW_hh): h_{t-1} rows j, k = t*B + b
template <typename T> struct HPrevB {
  static constexpr bool kRowVec = true;
  const T* hseq;
  int B, Tn, H, d;
  FastDiv dB;
  struct Ctx { int j; bool ok; };
  typedef int Prep;
  __device__ __forceinline__ Ctx row_ctx(int r8) const { return Ctx{r8, r8 < H}; }
  __device__ __forceinline__ Prep prep(int k0) const { return k0; }
  __device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc() const {
    return mk_rsrc(hseq, (uint32_t)((size_t)B * Tn * 2 * H * sizeof(T)));
  }
  __device__ __forceinline__ uint32_t offs(const Ctx& c, Prep k0, int kofs) const {
    const int k = k0 + kofs;
    uint32_t bu;
    const int t = (int)dB.divmod((uint32_t)k, bu), b = (int)bu;
    const int tp = d == 0 ? t - 1 : t + 1;
    const bool ok = c.ok && k < Tn * B && tp >= 0 && tp < Tn;
    return boff<T>((uint32_t)(((b * Tn + tp) * 2 * H) + d * H + c.j), ok);
  }
  __device__ __forceinline__ typename VT<T>::v8 load(const Ctx& c, Prep k0, int kofs) const {
    return bld8<T>(rsrc(), offs(c, k0, kofs));
  }
};
// B (dW_ih): x rows i, k = t*B + b : x[b][t][i]
template <typename T> struct XB {
  static constexpr bool kRowVec = true;
  const T* x;
  int B, Tn, In;
  FastDiv dB;
  struct Ctx { int i; bool ok; };
  typedef int Prep;
  __device__ __forceinline__ Ctx row_ctx(int r8) const { return Ctx{r8, r8 < In}; }
  __device__ __forceinline__ Prep prep(int k0) const { return k0; }
  __device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc() const {
    return mk_rsrc(x, (uint32_t)((size_t)B * Tn * In * sizeof(T)));
  }
  __device__ __forceinline__ uint32_t offs(const Ctx& c, Prep k0, int kofs) const {
    const int k = k0 + kofs;
    uint32_t bu;
    const int t = (int)dB.divmod((uint32_t)k, bu), b = (int)bu;
    return boff<T>((uint32_t)((b * Tn + t) * In + c.i), c.ok && k < Tn * B);
  }
  __device__ __forceinline__ typename VT<T>::v8 load(const Ctx& c, Prep k0, int kofs) const {
    return bld8<T>(rsrc(), offs(c, k0, kofs));
  }
};

// writes rows in reference gate order: packed row g' = 4j+q -> q*H + j
struct GateRowEpi {
  static constexpr bool kStats = false;
  float* out;  // [4H][N]
  int H, N, atomic, accumulate;
  __device__ __forceinline__ void store(int gp, int n, f32x4 v, int) const {
    if (gp >= 4 * H || n >= N) return;
    int row = (gp & 3) * H + (gp >> 2);
    float* p = out + (size_t)row * N + n;
    if (atomic) {
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (n + r < N) atomicAdd(p + r, v[r]);
    } else {
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (n + r < N) p[r] = accumulate ? p[r] + v[r] : v[r];
    }
  }
  __device__ __forceinline__ void stats(int, int, f32x4, f32x4) const {}
};

template <typename T, class LB>
int gate_wgrad(const T* dgates_d, const LB& lb, float* out, int B, int Tn, int H, int N, int accumulate, hipStream_t st) {
  const int K = Tn * B;
  ColMajorK<T> la{dgates_d, 4 * H, 4 * H, K};
  const int b = (4 * H >= 128 && N >= 128) ? 128 : 64;
  long tiles = (long)((4 * H + b - 1) / b) * ((N + b - 1) / b);
  long want = (256 + tiles - 1) / tiles;
  long maxs = (K + 4 * BK - 1) / (4 * BK);
  if (want > maxs) want = maxs;
  if (want < 1) want = 1;
  int splits = eff_splits(K, (int)want);
  if (splits > 1 && !accumulate) {
    hipError_t e = hipMemsetAsync(out, 0, (size_t)4 * H * N * sizeof(float), st);
    if (e != hipSuccess) return (int)e;
  }
  GateRowEpi ep{out, H, N, splits > 1 ? 1 : 0, accumulate};
  if (b == 128) return launch<T, 128, 128>(la, lb, ep, 4 * H, N, K, splits, st);
  return launch<T, 64, 64>(la, lb, ep, 4 * H, N, K, splits, st);
}

// db[d][q*H+j] = sum_k dgates[d][k][4j+q], two deterministic stages:
// partials ws[chunk][d][gp] over row chunks, then a fixed-order sum scattered to reference rows
constexpr int DB_CHUNKS = 64;
template <typename T>
__global__ void dbias_part_kernel(const T* __restrict__ dg, float* __restrict__ ws, int K, int H, long rpc) {
  __shared__ float red[4][64];
  const int c = threadIdx.x & 63, r = threadIdx.x >> 6;
  const int H4 = 4 * H, d = blockIdx.z;
  const int gp = blockIdx.x * 64 + c;
  const long k0 = blockIdx.y * rpc, k1 = min((long)K, k0 + rpc);
  const T* p = dg + (size_t)d * K * H4;
  float s = 0.f;
  if (gp < H4)
    for (long k = k0 + r; k < k1; k += 4) s += tof(p[k * H4 + gp]);
  red[r][c] = s;
  __syncthreads();
  if (r == 0 && gp < H4)
    ws[((size_t)blockIdx.y * 2 + d) * H4 + gp] = red[0][c] + red[1][c] + red[2][c] + red[3][c];
}

__global__ void dbias_fin_kernel(const float* __restrict__ ws, int chunks, int H, float* bf, float* b2f, float* br,
                                 float* b2r, int accumulate) {
  const int H4 = 4 * H;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= 2 * H4) return;
  const int d = i / H4, gp = i - d * H4;
  float s = 0.f;
  for (int c = 0; c < chunks; ++c) s += ws[((size_t)c * 2 + d) * H4 + gp];
  const int row = (gp & 3) * H + (gp >> 2);
  float* o1 = d ? br : bf;
  float* o2 = d ? b2r : b2f;
  o1[row] = accumulate ? o1[row] + s : s;
  if (o2) o2[row] = accumulate ? o2[row] + s : s;
}

// dx: A rows m = b*T + t, k = (d, g') -> dgates[(d*T + t)*B + b][g']
template <typename T> struct DgatesA {
  static constexpr bool kRowVec = false;
  const T* dg;
  int B, Tn, H;
  struct Ctx { int b, t; bool ok; };
  typedef int Prep;
  __device__ __forceinline__ Ctx row_ctx(int m) const {
    Ctx c;
    c.ok = m < B * Tn;
    int mm = c.ok ? m : 0;
    c.b = mm / Tn;
    c.t = mm - c.b * Tn;
    return c;
  }
  __device__ __forceinline__ Prep prep(int k0) const { return k0; }
  __device__ __forceinline__ typename VT<T>::v8 load(const Ctx& c, Prep k0, int kofs) const {
    const int H4 = 4 * H, k = k0 + kofs;
    const bool ok = c.ok && k < 2 * H4;
    const int d = k >= H4 ? 1 : 0, gp = k - d * H4;
    return bld8<T>(mk_rsrc(dg, (uint32_t)((size_t)2 * Tn * B * H4 * sizeof(T))),
                   boff<T>((uint32_t)(((d * Tn + c.t) * B + c.b) * H4 + gp), ok));
  }
};

template <typename T> struct StoreEpi {
  static constexpr bool kStats = false;
  T* y;
  int M, N;
  __device__ __forceinline__ void store(int m, int n, f32x4 v, int) const {
    if (m < M && n < N) st4<T>(y + (size_t)m * N + n, v);
  }
  __device__ __forceinline__ void stats(int, int, f32x4, f32x4) const {}
};

// ---- all four weight-gradient GEMMs of a layer in one launch (bf16):
//   batch bz = 2*d + kind:  kind 0  dW_ih[d] = dgates[d]^T x          ([4H][In])
//                           kind 1  dW_hh[d] = dgates[d]^T h_prev[d]  ([4H][H])
// split-K over ~one block per CU into fp32 slabs [bz][split][4H][N] (N = max(In, H)), then one
// reduce that sums the splits in fixed order and scatters packed gate rows (4j+q) to the
// reference rows (q*H + j). Four GEMMs share the grid, so each needs ~4x fewer splits than alone.
// batch-selectable loaders: the batch entry's parameters are derived arithmetically from bz
// (an array of per-batch loader copies indexed at run time would live in scratch memory)
template <typename T> struct GateWA {   // A rows g' (packed gate), k = t*B + b: dgates[d][k][g']
  static constexpr bool kRowVec = true;
  const T* dg;
  int H4, K, d;
  struct Ctx { uint32_t off; bool ok; };
  typedef int Prep;
  __device__ __forceinline__ void set_batch(int bz) { d = bz >> 1; }
  __device__ __forceinline__ Ctx row_ctx(int r8) const { return Ctx{(uint32_t)r8, r8 < H4}; }
  __device__ __forceinline__ Prep prep(int k0) const { return k0; }
  __device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc() const {
    return mk_rsrc(dg + (size_t)d * K * H4, (uint32_t)((size_t)K * H4 * sizeof(T)));
  }
  __device__ __forceinline__ uint32_t offs(const Ctx& c, Prep k0, int kofs) const {
    const int k = k0 + kofs;
    return boff<T>((uint32_t)k * (uint32_t)H4 + c.off, c.ok && k < K);
  }
};

template <typename T> struct GateWB {   // B rows n, k = t*B + b: x[b][t][n] (kind 0) or h_{t-1}[b][d][n] (kind 1)
  static constexpr bool kRowVec = true;
  const T* x;
  const T* hseq;
  int B, Tn, H, In, d, kind;
  FastDiv dB;
  struct Ctx { int j; bool ok; };
  typedef int Prep;
  __device__ __forceinline__ void set_batch(int bz) {
    d = bz >> 1;
    kind = bz & 1;
  }
  __device__ __forceinline__ Ctx row_ctx(int r8) const { return Ctx{r8, r8 < (kind ? H : In)}; }
  __device__ __forceinline__ Prep prep(int k0) const { return k0; }
  __device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc() const {
    return kind == 0 ? mk_rsrc(x, (uint32_t)((size_t)B * Tn * In * sizeof(T)))
                     : mk_rsrc(hseq, (uint32_t)((size_t)B * Tn * 2 * H * sizeof(T)));
  }
  __device__ __forceinline__ uint32_t offs(const Ctx& c, Prep k0, int kofs) const {
    const int k = k0 + kofs;
    uint32_t bu;
    const int t = (int)dB.divmod((uint32_t)k, bu), b = (int)bu;
    if (kind == 0) return boff<T>((uint32_t)((b * Tn + t) * In + c.j), c.ok && k < Tn * B);
    const int tp = d == 0 ? t - 1 : t + 1;
    const bool ok = c.ok && k < Tn * B && tp >= 0 && tp < Tn;
    return boff<T>((uint32_t)(((b * Tn + tp) * 2 * H) + d * H + c.j), ok);
  }
};

struct BatchSlabEpi {
  static constexpr bool kStats = false;
  static constexpr int kPrefer4W = 8;
  float* ws;  // [NB][nsplit][M][N]
  int M, N, nsplit, bz;
  __device__ __forceinline__ void set_batch(int b) { bz = b; }
  __device__ __forceinline__ void store(int m, int n, f32x4 v, int kz) const {
    if (m < M && n < N) *reinterpret_cast<f32x4*>(ws + (((size_t)bz * nsplit + kz) * M + m) * N + n) = v;
  }
  __device__ __forceinline__ void stats(int, int, f32x4, f32x4) const {}
};

struct GateOut {
  float* p[4];   // [bz] destination, [4H][cols] reference gate order
  int cols[4];
};

__global__ __launch_bounds__(256) void gate_slab_reduce_kernel(const float* __restrict__ ws, int S, int H, int N,
                                                               GateOut out, int accumulate) {
  const int bz = blockIdx.y, H4 = 4 * H, cols = out.cols[bz];
  const long total = (long)H4 * N;
  for (long i4 = blockIdx.x * (long)blockDim.x + threadIdx.x; 4 * i4 < total; i4 += (long)gridDim.x * blockDim.x) {
    const long i = 4 * i4;
    const int gp = (int)(i / N), n = (int)(i - (long)gp * N);
    if (n >= cols) continue;
    f32x4 s = {0.f, 0.f, 0.f, 0.f};
    const float* base = ws + (size_t)bz * S * total + i;
    int z = 0;
    for (; z + 4 <= S; z += 4) {
      f32x4 v[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) v[q] = *reinterpret_cast<const f32x4*>(base + (size_t)(z + q) * total);
#pragma unroll
      for (int q = 0; q < 4; ++q) s += v[q];
    }
    for (; z < S; ++z) s += *reinterpret_cast<const f32x4*>(base + (size_t)z * total);
    float* o = out.p[bz] + (size_t)((gp & 3) * H + (gp >> 2)) * cols + n;
    if (accumulate) s += *reinterpret_cast<const f32x4*>(o);
    *reinterpret_cast<f32x4*>(o) = s;
  }
}

inline int lstm_wgrad_splits(int B, int T, int H, int In) {
  const int N = In > H ? In : H, K = T * B;
  const long tiles = 4L * ((4 * H + 255) / 256) * ((N + 255) / 256);
  long s = (crnn_cu_count() + tiles - 1) / tiles;
  const long smax = K / (64 * 8);
  if (s > smax) s = smax;
  if (s < 1) s = 1;
  return eff_splits(K, (int)s);
}

}  // namespace

extern "C" {

int crnn_lstm_step_fwd(int dtype, const void* xg, const void* whh, void* hseq, void* gsv, float* csv, int B, int T,
                       int H, int step, void* stream) {
  if (H % 8) return crnn_set_error(hipErrorInvalidValue, "lstm: H must be a multiple of 8");
  hipStream_t st = (hipStream_t)stream;
  return dtype == CRNN_BF16 ? step_fwd_t<bf16>(xg, whh, hseq, gsv, csv, B, T, H, step, st)
                            : step_fwd_t<float>(xg, whh, hseq, gsv, csv, B, T, H, step, st);
}

size_t crnn_lstm_bptt_workspace(int B, int H) { return (size_t)bptt_splits(H) * 2 * B * H * sizeof(float); }

int crnn_lstm_step_bwd(int dtype, const void* dhseq, const void* whh, const void* whh_t, const void* gsv,
                       const float* csv, void* dgates, float* dc, float* ws, int B, int T, int H, int step,
                       void* stream) {
  if (H % 8) return crnn_set_error(hipErrorInvalidValue, "lstm: H must be a multiple of 8");
  hipStream_t st = (hipStream_t)stream;
  if (dtype == CRNN_BF16 && whh_t && ws && step > 0 && H % 16 == 0)
    return step_bwd_oneshot((const bf16*)dhseq, (const bf16*)whh_t, (const bf16*)gsv, csv, (bf16*)dgates, dc, ws, B, T,
                            H, step, st);
  return dtype == CRNN_BF16 ? step_bwd_t<bf16>(dhseq, whh, gsv, csv, dgates, dc, B, T, H, step, st)
                            : step_bwd_t<float>(dhseq, whh, gsv, csv, dgates, dc, B, T, H, step, st);
}

int crnn_lstm_dwhh(int dtype, const void* dgates, const void* hseq, float* dwhh_f, float* dwhh_r, int B, int T, int H,
                   int accumulate, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  for (int d = 0; d < 2; ++d) {
    size_t off = (size_t)d * T * B * 4 * H;
    float* out = d ? dwhh_r : dwhh_f;
    int rc = dtype == CRNN_BF16
                 ? gate_wgrad<bf16>((const bf16*)dgates + off, HPrevB<bf16>{(const bf16*)hseq, B, T, H, d, FastDiv(B)}, out, B, T,
                                    H, H, accumulate, st)
                 : gate_wgrad<float>((const float*)dgates + off, HPrevB<float>{(const float*)hseq, B, T, H, d, FastDiv(B)}, out, B,
                                     T, H, H, accumulate, st);
    if (rc) return rc;
  }
  return 0;
}

int crnn_lstm_dwih(int dtype, const void* dgates, const void* x, float* dwih_f, float* dwih_r, int B, int T, int H,
                   int In, int accumulate, void* stream) {
  if (In % 8) return crnn_set_error(hipErrorInvalidValue, "lstm: In must be a multiple of 8");
  hipStream_t st = (hipStream_t)stream;
  for (int d = 0; d < 2; ++d) {
    size_t off = (size_t)d * T * B * 4 * H;
    float* out = d ? dwih_r : dwih_f;
    int rc = dtype == CRNN_BF16
                 ? gate_wgrad<bf16>((const bf16*)dgates + off, XB<bf16>{(const bf16*)x, B, T, In, FastDiv(B)}, out, B, T, H, In,
                                    accumulate, st)
                 : gate_wgrad<float>((const float*)dgates + off, XB<float>{(const float*)x, B, T, In, FastDiv(B)}, out, B, T, H,
                                     In, accumulate, st);
    if (rc) return rc;
  }
  return 0;
}

size_t crnn_lstm_dbias_workspace(int H) { return (size_t)DB_CHUNKS * 2 * 4 * H * sizeof(float); }

int crnn_lstm_dbias(int dtype, const void* dgates, float* b_f, float* b2_f, float* b_r, float* b2_r, float* ws, int B,
                    int T, int H, int accumulate, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  const int K = T * B;
  const long rpc = (K + DB_CHUNKS - 1) / DB_CHUNKS;
  const int chunks = (int)((K + rpc - 1) / rpc);
  dim3 grid((4 * H + 63) / 64, (unsigned)chunks, 2);
  if (dtype == CRNN_BF16)
    hipLaunchKernelGGL(dbias_part_kernel<bf16>, grid, dim3(256), 0, st, (const bf16*)dgates, ws, K, H, rpc);
  else
    hipLaunchKernelGGL(dbias_part_kernel<float>, grid, dim3(256), 0, st, (const float*)dgates, ws, K, H, rpc);
  hipLaunchKernelGGL(dbias_fin_kernel, dim3((8 * H + 255) / 256), dim3(256), 0, st, ws, chunks, H, b_f, b2_f, b_r, b2_r,
                     accumulate);
  return (int)hipGetLastError();
}

int crnn_lstm_dx(int dtype, const void* dgates, const void* wih, void* dx, int B, int T, int H, int In, void* stream) {
  if (In % 8) return crnn_set_error(hipErrorInvalidValue, "lstm: In must be a multiple of 8");
  hipStream_t st = (hipStream_t)stream;
  const int M = B * T, K = 8 * H;
  if (dtype == CRNN_BF16) {
    DgatesA<bf16> la{(const bf16*)dgates, B, T, H};
    ColMajorK<bf16> lb{(const bf16*)wih, In, In, K};
    StoreEpi<bf16> ep{(bf16*)dx, M, In};
    return launch<bf16, 128, 128>(la, lb, ep, M, In, K, 1, st);
  }
  DgatesA<float> la{(const float*)dgates, B, T, H};
  ColMajorK<float> lb{(const float*)wih, In, In, K};
  StoreEpi<float> ep{(float*)dx, M, In};
  return launch<float, 64, 64>(la, lb, ep, M, In, K, 1, st);
}

size_t crnn_lstm_wgrad_workspace(int B, int T, int H, int In) {
  const int N = In > H ? In : H;
  return (size_t)4 * lstm_wgrad_splits(B, T, H, In) * 4 * H * N * sizeof(float);
}

int crnn_lstm_wgrad(const void* dgates, const void* x, const void* hseq, float* dwih_f, float* dwih_r, float* dwhh_f,
                    float* dwhh_r, float* ws, size_t ws_bytes, int B, int T, int H, int In, int accumulate,
                    void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (In % 8 || H % 8) return crnn_set_error(hipErrorInvalidValue, "lstm_wgrad: In, H must be multiples of 8");
  if (ws_bytes < crnn_lstm_wgrad_workspace(B, T, H, In))
    return crnn_set_error(hipErrorInvalidValue, "lstm_wgrad: workspace too small");
  const int N = In > H ? In : H, K = T * B, S = lstm_wgrad_splits(B, T, H, In);
  GateWA<bf16> la{(const bf16*)dgates, 4 * H, K, 0};
  GateWB<bf16> lb{(const bf16*)x, (const bf16*)hseq, B, T, H, In, 0, 0, FastDiv(B)};
  BatchSlabEpi ep{ws, 4 * H, N, S, 0};
  int rc = launch256<256, 256>(la, lb, ep, 4 * H, N, K, st, S, 4);
  if (rc) return rc;
  GateOut go{{dwih_f, dwhh_f, dwih_r, dwhh_r}, {In, H, In, H}};
  const long n4 = (long)4 * H * N / 4;
  int bx = (int)((n4 + 255) / 256);
  if (bx > 1024) bx = 1024;
  hipLaunchKernelGGL(gate_slab_reduce_kernel, dim3(bx, 4), dim3(256), 0, st, ws, S, H, N, go, accumulate);
  return (int)hipGetLastError();
}

}  // extern "C"
