// Diagnostics that ship in the library (not on any training / inference path).
//
// LDS sentinel (VERDICT r04 "next 1"): workgroups that fill their LDS allocation with a known
// pattern and re-check it for a while, so that a kernel running concurrently on another stream
// (this library's LDS-DMA GEMMs, the halo convs, hipBLASLt) can be checked for writes that land
// outside its own LDS allocation, i.e. inside a co-resident workgroup of another kernel. A
// mismatch is recorded with the victim's hardware ids (HW_ID: CU / SIMD / wave slot; LDS_ALLOC:
// base and size of its allocation) so that the corrupting pattern can be matched to its source.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "crnn_internal.hpp"
#include "common.hpp"

namespace {

constexpr int SENT_REC = 64;        // mismatch records kept
constexpr int SENT_REC_WORDS = 8;   // words per record

__device__ __forceinline__ uint32_t sentinel_word(uint32_t seed, uint32_t blk, uint32_t i) {
  return 0xA5000000u | ((seed * 0x9E3779B1u + blk * 7919u + i) & 0x00FFFFFFu);
}

// out: [0] mismatching words seen (summed over checks), [1] records taken, [2] waves that saw one,
//      [3] checks done; records from word 8: {index, got, expected, HW_ID, LDS_ALLOC, XCC_ID, check, block}
// mode bit 0: every check first REWRITES the whole allocation with a pattern of its own (16-B stores),
// barriers, then reads it back — a write lost or altered while other kernels' LDS traffic (LDS-DMA
// landings, transposing reads) shares the CU shows as a mismatch; bit 1: every check also folds a
// known per-lane value over the wave with __shfl_xor (ds_bpermute) and checks the sum
__global__ __launch_bounds__(256) void lds_sentinel_kernel(uint32_t* out, int words, int iters, uint32_t seed,
                                                           int sleep, int mode) {
  extern __shared__ uint32_t lds[];
  const uint32_t blk = blockIdx.x;
  for (int i = threadIdx.x; i < words; i += 256) lds[i] = sentinel_word(seed, blk, (uint32_t)i);
  __syncthreads();
  uint32_t hw, la, xcc;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_LDS_ALLOC)" : "=s"(la));
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
  uint32_t seen = 0;
  for (int it = 0; it < iters; ++it) {
    for (int s = 0; s < sleep; ++s) __builtin_amdgcn_s_sleep(127);
    const uint32_t sd = (mode & 1) ? seed + 0x1000193u * (uint32_t)(it + 1) : seed;
    if (mode & 1) {
      __syncthreads();   // every wave's reads of the previous pattern are done
      for (int i = 4 * threadIdx.x; i + 3 < words; i += 1024) {
        u32x4 v;
        for (int e = 0; e < 4; ++e) v[e] = sentinel_word(sd, blk, (uint32_t)(i + e));
        *reinterpret_cast<u32x4*>(lds + i) = v;
      }
      __syncthreads();
    }
    if (mode & 2) {
      float x = (float)((threadIdx.x & 63) + 1);
      for (int o = 1; o < 64; o <<= 1) x += __shfl_xor(x, o, 64);
      if (x != 2080.f) {   // 1 + ... + 64
        ++seen;
        const uint32_t slot = atomicAdd(out + 1, 1u);
        if (slot < (uint32_t)SENT_REC) {
          uint32_t* r = out + 8 + slot * SENT_REC_WORDS;
          r[0] = 0xFFFFFFFFu; r[1] = __float_as_uint(x); r[2] = __float_as_uint(2080.f); r[3] = hw;
          r[4] = la; r[5] = xcc; r[6] = (uint32_t)it; r[7] = blk;
        }
      }
    }
    for (int i = threadIdx.x; i < words; i += 256) {
      const uint32_t want = sentinel_word(sd, blk, (uint32_t)i);
      const uint32_t got = lds[i];
      if (got != want) {
        ++seen;
        const uint32_t slot = atomicAdd(out + 1, 1u);
        if (slot < (uint32_t)SENT_REC) {
          uint32_t* r = out + 8 + slot * SENT_REC_WORDS;
          r[0] = (uint32_t)i; r[1] = got; r[2] = want; r[3] = hw;
          r[4] = la; r[5] = xcc; r[6] = (uint32_t)it; r[7] = blk;
        }
        lds[i] = want;   // re-arm: count each later hit again
      }
    }
  }
  if (seen) atomicAdd(out, seen);
  __syncthreads();
  if (threadIdx.x == 0) atomicAdd(out + 3, (uint32_t)iters);
  // blocks that saw a mismatch (one lane per wave that saw one)
  const unsigned long long any = __ballot(seen != 0);
  if (any && (threadIdx.x & 63) == (uint32_t)__builtin_ctzll(any)) atomicAdd(out + 2, 1u);
}

}  // namespace

extern "C" int crnn_diag_lds_sentinel(unsigned* out, int blocks, int lds_bytes, int iters, unsigned seed, int sleep,
                                      int mode, void* stream) {
  if (!out || blocks <= 0 || lds_bytes < 1024 || lds_bytes > 160 * 1024 || (lds_bytes & 3) || iters < 0 || sleep < 0)
    return crnn_set_error((int)hipErrorInvalidValue, "crnn_diag_lds_sentinel: bad arguments");
  static bool attr = false;
  if (!attr) {   // dynamic LDS above 64 KB must be allowed explicitly
    (void)hipFuncSetAttribute((const void*)lds_sentinel_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr = true;
  }
  hipLaunchKernelGGL(lds_sentinel_kernel, dim3(blocks), dim3(256), lds_bytes, (hipStream_t)stream, (uint32_t*)out,
                     lds_bytes / 4, iters, (uint32_t)seed, sleep, mode);
  return (int)hipGetLastError();
}

extern "C" int crnn_diag_lds_sentinel_words(void) { return 8 + SENT_REC * SENT_REC_WORDS; }
