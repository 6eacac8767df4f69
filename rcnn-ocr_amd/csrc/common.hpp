// Shared types and helpers for the CRNN HIP kernels (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stddef.h>

typedef __bf16 bf16;
typedef bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x8 __attribute__((ext_vector_type(8)));

// 8 elements of T, naturally the unit of a 16 B (bf16) / 32 B (f32) vector access.
template <typename T> struct VT;
template <> struct VT<float> { using v8 = f32x8; using v4 = f32x4; };
template <> struct VT<bf16> { using v8 = bf16x8; using v4 = bf16x4; };

__device__ __forceinline__ float tof(float x) { return x; }
__device__ __forceinline__ float tof(bf16 x) { return (float)x; }
template <typename T> __device__ __forceinline__ T fromf(float x);
template <> __device__ __forceinline__ float fromf<float>(float x) { return x; }
template <> __device__ __forceinline__ bf16 fromf<bf16>(float x) { return (bf16)x; }

template <typename T>
__device__ __forceinline__ typename VT<T>::v8 ld8(const T* p) {
  if constexpr (sizeof(T) == 2) {
    return *reinterpret_cast<const bf16x8*>(p);
  } else {
    f32x4 a = *reinterpret_cast<const f32x4*>(p);
    f32x4 b = *reinterpret_cast<const f32x4*>(p + 4);
    f32x8 r;
    r[0] = a[0]; r[1] = a[1]; r[2] = a[2]; r[3] = a[3];
    r[4] = b[0]; r[5] = b[1]; r[6] = b[2]; r[7] = b[3];
    return r;
  }
}

template <typename T>
__device__ __forceinline__ void st8(T* p, const typename VT<T>::v8& v) {
  if constexpr (sizeof(T) == 2) {
    *reinterpret_cast<bf16x8*>(p) = v;
  } else {
    f32x4 a, b;
    a[0] = v[0]; a[1] = v[1]; a[2] = v[2]; a[3] = v[3];
    b[0] = v[4]; b[1] = v[5]; b[2] = v[6]; b[3] = v[7];
    *reinterpret_cast<f32x4*>(p) = a;
    *reinterpret_cast<f32x4*>(p + 4) = b;
  }
}

template <typename T> __device__ __forceinline__ typename VT<T>::v8 zero8() {
  typename VT<T>::v8 z;
#pragma unroll
  for (int i = 0; i < 8; ++i) z[i] = fromf<T>(0.f);
  return z;
}

// 8 elements -> floats, and back
template <typename T>
__device__ __forceinline__ void unpack8(const typename VT<T>::v8& v, float* f) {
#pragma unroll
  for (int i = 0; i < 8; ++i) f[i] = tof(v[i]);
}
template <typename T>
__device__ __forceinline__ typename VT<T>::v8 pack8(const float* f) {
  typename VT<T>::v8 v;
#pragma unroll
  for (int i = 0; i < 8; ++i) v[i] = fromf<T>(f[i]);
  return v;
}

// store 4 consecutive values (n..n+3) of one row
template <typename T>
__device__ __forceinline__ void st4(T* p, f32x4 v) {
  if constexpr (sizeof(T) == 2) {
    bf16x4 b;
    b[0] = (bf16)v[0]; b[1] = (bf16)v[1]; b[2] = (bf16)v[2]; b[3] = (bf16)v[3];
    *reinterpret_cast<bf16x4*>(p) = b;
  } else {
    *reinterpret_cast<f32x4*>(p) = v;
  }
}
template <typename T>
__device__ __forceinline__ f32x4 ld4f(const T* p) {
  f32x4 r;
  if constexpr (sizeof(T) == 2) {
    bf16x4 b = *reinterpret_cast<const bf16x4*>(p);
    r[0] = (float)b[0]; r[1] = (float)b[1]; r[2] = (float)b[2]; r[3] = (float)b[3];
  } else {
    r = *reinterpret_cast<const f32x4*>(p);
  }
  return r;
}

__device__ __forceinline__ float sigmoidf_(float x) { return 1.f / (1.f + __expf(-x)); }
__device__ __forceinline__ float tanhf_(float x) {
  // tanh via exp, saturating for large |x|
  float e = __expf(-2.f * fabsf(x));
  float t = (1.f - e) / (1.f + e);
  return copysignf(t, x);
}

// bf16-path variants: hardware reciprocal (1 ulp) instead of the IEEE division sequence
__device__ __forceinline__ float sigmoid_fast(float x) { return __builtin_amdgcn_rcpf(1.f + __expf(-x)); }
__device__ __forceinline__ float tanh_fast(float x) {
  float e = __expf(-2.f * fabsf(x));
  return copysignf((1.f - e) * __builtin_amdgcn_rcpf(1.f + e), x);
}

// sum over aligned groups of G (2, 4, 8 or 16) lanes with DPP moves (no LDS round trip, unlike
// __shfl_xor's ds_bpermute); every lane of a group gets the same, lane-order-independent sum
template <int CTRL> __device__ __forceinline__ float dppf(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
template <int G> __device__ __forceinline__ float rowgroup_sum(float v) {
  static_assert(G == 2 || G == 4 || G == 8 || G == 16, "group");
  v += dppf<0xB1>(v);                          // quad_perm [1,0,3,2]
  if constexpr (G >= 4) v += dppf<0x4E>(v);    // quad_perm [2,3,0,1]
  if constexpr (G >= 8) v += dppf<0x141>(v);   // row_half_mirror: quads 0 <-> 1 of each 8
  if constexpr (G >= 16) v += dppf<0x140>(v);  // row_mirror: halves of each 16-lane row
  return v;
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Bijective XCD-aware remap (cdna_hip_programming.md §5 / T1): consecutive logical
// tiles land on the same XCD so their shared operand panels hit one L2.
__device__ __forceinline__ int xcd_remap(int b, int nwg) {
  const int nx = 8;
  int xcd = b % nx, q = nwg / nx, r = nwg % nx;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + b / nx;
}

// ---- range-checked buffer loads (CDNA raw buffer addressing)
// A lane whose byte offset is >= the descriptor's num_records reads zeros in hardware,
// so masked / out-of-bounds gathers need no exec-mask branches.
// counter-based dropout hash (enc_dropout in bn.hip, attention-weight dropout in attn.hip):
// splitmix64's finalizer on seed ^ (i * golden ratio); element i is kept iff hash >= p * 2^32
__device__ __forceinline__ uint32_t drop_hash(unsigned long long seed, unsigned long long i) {
  unsigned long long z = seed ^ (i * 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return (uint32_t)((z ^ (z >> 31)) >> 32);
}
__host__ inline uint32_t drop_threshold(float p) {
  const double t = (double)p * 4294967296.0;
  return t >= 4294967295.0 ? 0xffffffffu : (uint32_t)t;
}

constexpr uint32_t OOB = 0x80000000u;
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ __amdgpu_buffer_rsrc_t mk_rsrc(const void* p, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}

template <typename T>
__device__ __forceinline__ typename VT<T>::v8 bld8(__amdgpu_buffer_rsrc_t r, uint32_t byteoff) {
  if constexpr (sizeof(T) == 2) {
    u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, byteoff, 0, 0);
    return __builtin_bit_cast(bf16x8, v);
  } else {
    u32x4 a = __builtin_amdgcn_raw_buffer_load_b128(r, byteoff, 0, 0);
    u32x4 b = __builtin_amdgcn_raw_buffer_load_b128(r, byteoff + 16u, 0, 0);
    f32x4 fa = __builtin_bit_cast(f32x4, a), fb = __builtin_bit_cast(f32x4, b);
    f32x8 o;
    o[0] = fa[0]; o[1] = fa[1]; o[2] = fa[2]; o[3] = fa[3];
    o[4] = fb[0]; o[5] = fb[1]; o[6] = fb[2]; o[7] = fb[3];
    return o;
  }
}

// element offset -> byte offset, or OOB when !ok
template <typename T> __device__ __forceinline__ uint32_t boff(uint32_t elem, bool ok) {
  return ok ? elem * (uint32_t)sizeof(T) : OOB;
}

// Division by a runtime-invariant divisor via a precomputed magic number:
// n / d = (umulhi(n, mul) + n) >> shift, exact for 0 <= n < 2^31 (Granlund-Montgomery).
struct FastDiv {
  uint32_t d, mul, shift;
  FastDiv() = default;
  __host__ FastDiv(uint32_t div) : d(div) {
    uint32_t s = 0;
    while (s < 32 && (1ull << s) < div) ++s;
    uint64_t one = 1;
    uint64_t m = ((one << 32) * ((one << s) - div)) / div + 1;
    mul = (uint32_t)m;
    shift = s;
  }
  __device__ __forceinline__ uint32_t div(uint32_t n) const {
    uint32_t t = __umulhi(n, mul);
    return (t + n) >> shift;
  }
  // q = n / d, r = n - q*d
  __device__ __forceinline__ uint32_t divmod(uint32_t n, uint32_t& r) const {
    uint32_t q = div(n);
    r = n - q * d;
    return q;
  }
};

#define CRNN_CHECK_LAUNCH() return (int)hipGetLastError()
