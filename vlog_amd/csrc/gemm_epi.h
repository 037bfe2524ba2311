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
