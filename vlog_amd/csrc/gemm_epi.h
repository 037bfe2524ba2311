// Fused GEMM epilogues shared by the tiled (gemm.hip) and large-tile (gemm_big.hip) kernels: one output
// element (row, col) with its f32 accumulator -> bias / GELU / residual / positional add / KV-cache scatter.
#pragma once
#include "gemm.h"

template <int KIND>
__device__ __forceinline__ void apply_epi(const GemmEpi& epi, int row, int col, float acc) {
  float v = acc + (epi.bias ? epi.bias[col] : 0.f);
  switch (KIND) {
    case EPI_BF16: {
      if (epi.act == 1) v = gelu_erf(v);
      long long o = epi.rpb ? (long long)(row / epi.rpb) * epi.bstride + (long long)(row % epi.rpb + epi.roff) * epi.ldc
                            : (long long)row * epi.ldc;
      ((bf16*)epi.out)[o + col] = f2bf(v);
      break;
    }
    case EPI_RESID_F32: {
      float* p = (float*)epi.out + (long long)row * epi.ldc + col;
      *p += v;
      break;
    }
    case EPI_GELU_POS_F32: {
      const int t = row % epi.rpb;
      ((float*)epi.out)[(long long)row * epi.ldc + col] = gelu_erf(v) + epi.pos[(long long)t * epi.ldc + col];
      break;
    }
    case EPI_F32: {
      ((float*)epi.out)[(long long)row * epi.ldc + col] = v;
      break;
    }
    case EPI_DEC_QKV: {
      const int d = epi.d;
      if (col < d) {
        ((bf16*)epi.out)[(long long)row * epi.ldc + col] = f2bf(v);
      } else {
        const int c2 = col - d;
        const int kv = c2 >= d;
        const int cc = kv ? c2 - d : c2;
        const int h = cc / epi.head_dim, e2 = cc - h * epi.head_dim;
        const long long slot = (((long long)epi.row_hyp[row] * epi.n_head + h) * epi.n_ctx + epi.row_pos[row]) * epi.head_dim + e2;
        (kv ? epi.vcache : epi.kcache)[slot] = f2bf(v);
      }
      break;
    }
    case EPI_CROSS_KV: {
      // col = l*2d + kv*d + h*hd + e ; row = b*T + t  ->  [L*2][slots][H][T][hd]
      const int d = epi.d, hd = epi.head_dim;
      const int l2 = col / d, cc = col - l2 * d;
      const int h = cc / hd, e2 = cc - h * hd;
      const int b = row / epi.rpb, t = row - b * epi.rpb;
      const long long o = ((((long long)l2 * epi.n_slots + epi.slot0 + b) * epi.n_head + h) * epi.rpb + t) * hd + e2;
      ((bf16*)epi.out)[o] = f2bf(v);
      break;
    }
    default:   // EPI_RESID_LN never reaches a per-element epilogue (always split-K slabs + fused reduce)
      break;
  }
}

// Four consecutive output columns col0..col0+3 of one row (col0 % 4 == 0, col0 + 3 < N): the same
// arithmetic as four apply_epi calls, stored as one 8-B (bf16) or 16-B (f32) access.  Used by kernels whose
// MFMA operands are swapped (C^T fragments: each lane holds 4 consecutive columns of one row).
template <int KIND>
__device__ __forceinline__ void apply_epi4(const GemmEpi& epi, int row, int col0, f32x4 acc) {
  f32x4 v = acc;
  if (epi.bias) {
    const f32x4 b = *(const f32x4*)(epi.bias + col0);
    v += b;
  }
  switch (KIND) {
    case EPI_BF16: {
      if (epi.act == 1) {
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = gelu_erf(v[e]);
      }
      long long o = epi.rpb ? (long long)(row / epi.rpb) * epi.bstride + (long long)(row % epi.rpb + epi.roff) * epi.ldc
                            : (long long)row * epi.ldc;
      bf16x4 r;
#pragma unroll
      for (int e = 0; e < 4; ++e) r[e] = f2bf(v[e]);
      *(bf16x4*)((bf16*)epi.out + o + col0) = r;
      break;
    }
    case EPI_RESID_F32: {
      f32x4* p = (f32x4*)((float*)epi.out + (long long)row * epi.ldc + col0);
      *p = *p + v;
      break;
    }
    case EPI_GELU_POS_F32: {
      const int t = row % epi.rpb;
      const f32x4 pe = *(const f32x4*)(epi.pos + (long long)t * epi.ldc + col0);
      f32x4 r;
#pragma unroll
      for (int e = 0; e < 4; ++e) r[e] = gelu_erf(v[e]) + pe[e];
      *(f32x4*)((float*)epi.out + (long long)row * epi.ldc + col0) = r;
      break;
    }
    case EPI_F32: {
      *(f32x4*)((float*)epi.out + (long long)row * epi.ldc + col0) = v;
      break;
    }
    case EPI_DEC_QKV: {
      const int d = epi.d;
      bf16x4 r;
#pragma unroll
      for (int e = 0; e < 4; ++e) r[e] = f2bf(v[e]);
      if (col0 < d) {
        *(bf16x4*)((bf16*)epi.out + (long long)row * epi.ldc + col0) = r;
      } else {
        const int c2 = col0 - d;
        const int kv = c2 >= d;
        const int cc = kv ? c2 - d : c2;
        const int h = cc / epi.head_dim, e2 = cc - h * epi.head_dim;
        const long long slot = (((long long)epi.row_hyp[row] * epi.n_head + h) * epi.n_ctx + epi.row_pos[row]) * epi.head_dim + e2;
        *(bf16x4*)((kv ? epi.vcache : epi.kcache) + slot) = r;
      }
      break;
    }
    case EPI_CROSS_KV: {
      const int d = epi.d, hd = epi.head_dim;
      const int l2 = col0 / d, cc = col0 - l2 * d;
      const int h = cc / hd, e2 = cc - h * hd;
      const int b = row / epi.rpb, t = row - b * epi.rpb;
      const long long o = ((((long long)l2 * epi.n_slots + epi.slot0 + b) * epi.n_head + h) * epi.rpb + t) * hd + e2;
      bf16x4 r;
#pragma unroll
      for (int e = 0; e < 4; ++e) r[e] = f2bf(v[e]);
      *(bf16x4*)((bf16*)epi.out + o) = r;
      break;
    }
    default:
      break;
  }
}

// apply_epi4 with its loaded operands passed in: the bias chunk `b` (used only when epi.bias is set) and, for
// EPI_DEC_QKV, the row's hypothesis and position.  A kernel that stores several fragments requests these for all of
// them before the first store (inside the fragment loop each load waited for its own round trip); the arithmetic is
// apply_epi4's.
template <int KIND>
__device__ __forceinline__ void apply_epi4_pre(const GemmEpi& epi, int row, int col0, f32x4 acc, f32x4 b, int hyp,
                                               int pos) {
  if constexpr (KIND == EPI_BF16 || KIND == EPI_DEC_QKV) {
    f32x4 v = acc;
    if (epi.bias) v += b;
    if constexpr (KIND == EPI_BF16) {
      if (epi.act == 1) {
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = gelu_erf(v[e]);
      }
      long long o = epi.rpb ? (long long)(row / epi.rpb) * epi.bstride + (long long)(row % epi.rpb + epi.roff) * epi.ldc
                            : (long long)row * epi.ldc;
      bf16x4 r;
#pragma unroll
      for (int e = 0; e < 4; ++e) r[e] = f2bf(v[e]);
      *(bf16x4*)((bf16*)epi.out + o + col0) = r;
    } else {
      const int d = epi.d;
      bf16x4 r;
#pragma unroll
      for (int e = 0; e < 4; ++e) r[e] = f2bf(v[e]);
      if (col0 < d) {
        *(bf16x4*)((bf16*)epi.out + (long long)row * epi.ldc + col0) = r;
      } else {
        const int c2 = col0 - d;
        const int kv = c2 >= d;
        const int cc = kv ? c2 - d : c2;
        const int h = cc / epi.head_dim, e2 = cc - h * epi.head_dim;
        const long long slot = (((long long)hyp * epi.n_head + h) * epi.n_ctx + pos) * epi.head_dim + e2;
        *(bf16x4*)((kv ? epi.vcache : epi.kcache) + slot) = r;
      }
    }
  } else {
    apply_epi4<KIND>(epi, row, col0, acc);
  }
}

// ---- Staged epilogue helpers (gemm_8p.hip): the value of 4 consecutive outputs (bias / activation /
// positional add folded in, same arithmetic as apply_epi4), and whole 16-B chunk stores of it.
template <int KIND>
__device__ __forceinline__ f32x4 epi_value4(const GemmEpi& epi, int row, int col0, f32x4 acc) {
  f32x4 v = acc;
  if (epi.bias) {
    const f32x4 b = *(const f32x4*)(epi.bias + col0);
    v += b;
  }
  if (KIND == EPI_BF16 && epi.act == 1) {
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = gelu_erf(v[e]);
  }
  if (KIND == EPI_GELU_POS_F32) {
    const int t = row % epi.rpb;
    const f32x4 pe = *(const f32x4*)(epi.pos + (long long)t * epi.ldc + col0);
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = gelu_erf(v[e]) + pe[e];
  }
  return v;
}

// epi_value4 with the bias chunk `b` loaded ahead (used only when epi.bias is set): a kernel whose fragments share
// a few columns requests those chunks once, before its fragment loop (loaded per fragment, each load waited for its
// own round trip).  GELU_POS still loads its positional row per fragment.
template <int KIND>
__device__ __forceinline__ f32x4 epi_value4_pre(const GemmEpi& epi, int row, int col0, f32x4 acc, f32x4 b) {
  if constexpr (KIND == EPI_GELU_POS_F32) {
    return epi_value4<KIND>(epi, row, col0, acc);
  } else {
    f32x4 v = acc;
    if (epi.bias) v += b;
    if (KIND == EPI_BF16 && epi.act == 1) {
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = gelu_erf(v[e]);
    }
    return v;
  }
}

// 8 consecutive bf16 outputs (col0 % 8 == 0) of a bf16-output kind
template <int KIND>
__device__ __forceinline__ void epi_store8_bf16(const GemmEpi& epi, int row, int col0, bf16x8 v) {
  if (KIND == EPI_BF16) {
    const long long o = epi.rpb ? (long long)(row / epi.rpb) * epi.bstride + (long long)(row % epi.rpb + epi.roff) * epi.ldc
                                : (long long)row * epi.ldc;
    *(bf16x8*)((bf16*)epi.out + o + col0) = v;
  } else if (KIND == EPI_CROSS_KV) {
    const int d = epi.d, hd = epi.head_dim;
    const int l2 = col0 / d, cc = col0 - l2 * d;
    const int h = cc / hd, e2 = cc - h * hd;
    const int b = row / epi.rpb, t = row - b * epi.rpb;
    const long long o = ((((long long)l2 * epi.n_slots + epi.slot0 + b) * epi.n_head + h) * epi.rpb + t) * hd + e2;
    *(bf16x8*)((bf16*)epi.out + o) = v;
  }
}

// 4 consecutive f32 outputs of an f32-output kind (RESID_F32 adds into the residual)
template <int KIND>
__device__ __forceinline__ void epi_store4_f32(const GemmEpi& epi, int row, int col0, f32x4 v) {
  f32x4* p = (f32x4*)((float*)epi.out + (long long)row * epi.ldc + col0);
  if (KIND == EPI_RESID_F32) *p = *p + v;
  else *p = v;
}
