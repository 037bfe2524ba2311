// Shared device helpers for the gfx950 (CDNA4) Whisper kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef __bf16 bf16;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(4))) int i32x4;

#define WAVE 64
#define STAT_SLOTS 256   // profiler byte counters per kernel class (spread to avoid one hot atomic)

__device__ __forceinline__ float bf2f(bf16 x) { return (float)x; }
__device__ __forceinline__ bf16 f2bf(float x) { return (bf16)x; }

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

__device__ __forceinline__ float gelu_erf(float x) { return 0.5f * x * (1.0f + erff(x * 0.70710678118654752f)); }

// Float <-> order-preserving uint for atomicMax on floats of any sign.
__device__ __forceinline__ unsigned int float_to_ordered(float f) {
  unsigned int u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float ordered_to_float(unsigned int u) {
  u = (u & 0x80000000u) ? (u & 0x7fffffffu) : ~u;
  return __uint_as_float(u);
}

// Device error word of a decode (engine.cpp d_err): [0] = code, [1], [2] = where.  The first failure wins (the
// host reads the word at every poll of a decode and at its end, and raises).  Global atomics (vector memory).
#define WM_ERR_NONFINITE 1     // a logits row held NaN / inf among its allowed tokens
#define WM_ERR_NO_TOKEN 2      // the logit rules left no allowed token
#define WM_ERR_TOKEN_RANGE 3   // a decoder input token id / position outside its table
__device__ __forceinline__ void wm_report_error(int* err, int code, int a, int b) {
  if (!err) return;
  if (atomicCAS(err, 0, code) == 0) {
    atomicExch(err + 1, a);
    atomicExch(err + 2, b);
  }
}

// Cross-attention fusions (attn_dec.hip launch_cross_attn): read q as bf16(sum of split-K slabs + bias) and/or
// combine the key splits in-kernel (last arriver per item, counter words zero between launches).
struct CrossFuse {
  const float* q_part = nullptr;   // [q_splits][q_rows][ldq] f32 slabs of the cq projection (nullptr: read q)
  int q_splits = 0, q_rows = 0;
  const float* q_bias = nullptr;
  int* cnt = nullptr;              // >= rows*H zeroed ints (nullptr: separate combine kernel)
  int tf = 0;                      // teacher-forced pass (`group` contiguous rows per window): matrix-core kernel
  int mfma = 0;                    // decode pass: row groups of 2..32 rows per window on the matrix-core kernel
  int* tf_cnt = nullptr;           // matrix-core decode pass: >= rows*H zeroed ints, the key-split combine done by
                                   // the last-arriving split in-kernel (nullptr: separate combine kernel)
};

// The factored cross-attention's cut of a decoder pass (attn_xenc.hip xattn_plan): `slabs` partials per row (key splits,
// or at most that many LDS-DMA chunk pieces); sk_W > 0: the stream-K chunk cut of sk_W units into sk_P chunks.
struct XPlan {
  int slabs = 1;
  long long sk_W = 0;
  int sk_P = 0;
};

// Launch check used by every host-side launcher: converts an asynchronous launch failure into an
// exception the C-ABI layer turns into an error code + wm_last_error() text.
#define WM_LAUNCH_CHECK(what)                                                                  \
  do {                                                                                         \
    hipError_t e__ = hipGetLastError();                                                        \
    if (e__ != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e__)); \
  } while (0)
