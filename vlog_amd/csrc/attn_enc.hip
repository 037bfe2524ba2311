// Encoder self-attention (non-causal, T = 1500, head_dim 64) as a flash-style MFMA kernel for gfx950.
//
// One workgroup = 4 waves = 64 queries of one (window, head); each wave owns 16 queries.  Per 64-key tile:
//   S^T = K . Q^T   (v_mfma_f32_16x16x32_bf16, K tile from LDS as the A operand, Q held in registers as
//                    the B operand) -> each lane holds 16 scores of ONE query (query = lane & 15), so the
//                    online-softmax state (m, l) is lane-local and the row reductions are 2 shuffles;
//   O^T += V^T . P^T (the S^T accumulator IS the P^T operand: the k slots of lane group g are keys
//                    {4g..4g+3} U {16+4g..16+4g+3} of each 32-key step, and the V^T operand is read
//                    from LDS in the same permuted order — cdna_hip_programming.md §3 "an accumulator tile
//                    as the next MFMA's operand").
// K is staged with the GEMM's 128-B-row XOR swizzle; V is staged transposed ([hd][key], 136-B rows) so the
// A-operand reads are two ds_read_b64 per lane.  Next tile's global loads are issued before the current
// tile's MFMAs (register double buffer).
#include "common.h"
#include <stdexcept>
#include <string>

#define HD 64
#define KT 64        // keys per tile
#define VT_LD 68     // V^T row stride (elements)

__device__ __forceinline__ int kswz(int row, int ch) { return row * HD + ((ch ^ ((row >> 1) & 7)) << 3); }

__global__ __launch_bounds__(256) void attn_enc_kernel(const bf16* __restrict__ qkv, bf16* __restrict__ out, int T,
                                                       int d, float scale_log2) {
  __shared__ __attribute__((aligned(16))) bf16 sK[KT * HD];
  __shared__ __attribute__((aligned(16))) bf16 sVt[HD * VT_LD];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int g = lane >> 4, ql = lane & 15;
  const int h = blockIdx.y, b = blockIdx.z;
  const long long ld = 3LL * d;
  const bf16* base = qkv + (long long)b * T * ld;
  const int q0 = blockIdx.x * 64 + wv * 16;

  // Q fragments (B operand): Q[q0 + ql][kk*32 + 8g .. +7]
  bf16x8 qf[2];
  {
    const int q = q0 + ql;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      if (q < T) qf[kk] = *(const bf16x8*)(base + (long long)q * ld + h * HD + kk * 32 + 8 * g);
      else qf[kk] = bf16x8{};
    }
  }

  f32x4 o[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) o[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m_run = -INFINITY, l_run = 0.f;

  // staging: each thread moves 2 x 16 B of K and 2 x 16 B of V per tile
  i32x4 rk[2], rv[2];
  const int nt = (T + KT - 1) / KT;
#define LOAD_TILE(t_)                                                                       \
  {                                                                                         \
    _Pragma("unroll") for (int i = 0; i < 2; ++i) {                                         \
      const int c = tid + i * 256, key = (t_) * KT + (c >> 3), ch = c & 7;                  \
      if (key < T) {                                                                        \
        const bf16* p = base + (long long)key * ld + h * HD + ch * 8;                        \
        rk[i] = *(const i32x4*)(p + d);                                                     \
        rv[i] = *(const i32x4*)(p + 2 * d);                                                 \
      } else {                                                                              \
        rk[i] = i32x4{0, 0, 0, 0};                                                          \
        rv[i] = i32x4{0, 0, 0, 0};                                                          \
      }                                                                                     \
    }                                                                                       \
  }
  LOAD_TILE(0);
  for (int t = 0; t < nt; ++t) {
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int c = tid + i * 256, key = c >> 3, ch = c & 7;
      *(i32x4*)(&sK[kswz(key, ch)]) = rk[i];
      bf16x8 vv = __builtin_bit_cast(bf16x8, rv[i]);
#pragma unroll
      for (int e = 0; e < 8; ++e) sVt[(ch * 8 + e) * VT_LD + key] = vv[e];
    }
    __syncthreads();
    if (t + 1 < nt) LOAD_TILE(t + 1);

    // ---- S^T = K . Q^T : 4 key blocks x 2 k-steps
    f32x4 s[4];
#pragma unroll
    for (int mi = 0; mi < 4; ++mi) {
      s[mi] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        const bf16x8 ka = *(const bf16x8*)(&sK[kswz(mi * 16 + ql, kk * 4 + g)]);
        s[mi] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ka, qf[kk], s[mi], 0, 0, 0);
      }
    }
    // ---- online softmax (lane = one query; keys mi*16 + 4g + e)
    float tmax = -INFINITY;
    const int kbase = t * KT;
#pragma unroll
    for (int mi = 0; mi < 4; ++mi)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int key = kbase + mi * 16 + 4 * g + e;
        float v = s[mi][e] * scale_log2;
        if (key >= T) v = -INFINITY;
        s[mi][e] = v;
        tmax = fmaxf(tmax, v);
      }
    tmax = fmaxf(tmax, __shfl_xor(tmax, 16, 64));
    tmax = fmaxf(tmax, __shfl_xor(tmax, 32, 64));
    const float m_new = fmaxf(m_run, tmax);
    const float alpha = exp2f(m_run - m_new);
    float psum = 0.f;
#pragma unroll
    for (int mi = 0; mi < 4; ++mi)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float p = exp2f(s[mi][e] - m_new);
        s[mi][e] = p;
        psum += p;
      }
    psum += __shfl_xor(psum, 16, 64);
    psum += __shfl_xor(psum, 32, 64);
    l_run = l_run * alpha + psum;
    m_run = m_new;
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) o[ni] *= alpha;

    // ---- O^T += V^T . P^T : 4 hd blocks x 2 key steps
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 pb;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        pb[e] = f2bf(s[2 * ks][e]);
        pb[4 + e] = f2bf(s[2 * ks + 1][e]);
      }
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) {
        const bf16* vr = &sVt[(ni * 16 + ql) * VT_LD + ks * 32 + 4 * g];
        const bf16x4 lo = *(const bf16x4*)(vr);
        const bf16x4 hi = *(const bf16x4*)(vr + 16);
        bf16x8 va;
#pragma unroll
        for (int e = 0; e < 4; ++e) { va[e] = lo[e]; va[4 + e] = hi[e]; }
        o[ni] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(va, pb, o[ni], 0, 0, 0);
      }
    }
  }
#undef LOAD_TILE

  const int q = q0 + ql;
  if (q < T) {
    const float inv = 1.0f / l_run;
    bf16* orow = out + ((long long)b * T + q) * d + h * HD;
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) {
      bf16x4 w;
#pragma unroll
      for (int e = 0; e < 4; ++e) w[e] = f2bf(o[ni][e] * inv);
      *(bf16x4*)(orow + ni * 16 + 4 * g) = w;
    }
  }
}

void launch_attn_enc(const bf16* qkv, bf16* out, int B, int T, int d, int n_head, hipStream_t st) {
  if (B <= 0) return;
  if (d != n_head * HD) throw std::runtime_error("attn_enc: head_dim must be 64");
  dim3 grid((T + 63) / 64, n_head, B);
  const float scale_log2 = 0.125f * 1.4426950408889634f;
  hipLaunchKernelGGL(attn_enc_kernel, grid, dim3(256), 0, st, qkv, out, T, d, scale_log2);
  WM_LAUNCH_CHECK("attn_enc_kernel");
}
