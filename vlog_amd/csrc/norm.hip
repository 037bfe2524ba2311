// Row kernels for gfx950: LayerNorm (f32 residual -> bf16 GEMM operand), decoder token+position embedding,
// conv1 im2col straight from the whole-file log-mel (window slicing + pad_or_trim zero fill fused), and the
// zero pad row conv2's implicit im2col reads.
#include "common.h"
#include <stdexcept>
#include <string>

// One wave per row; each lane owns NP float2 pairs (d = 128 * NP).
template <int NP>
__global__ __launch_bounds__(256) void layernorm_kernel(const float* __restrict__ x, long long ldx,
                                                        const int* __restrict__ row_idx, int rows,
                                                        const float* __restrict__ g, const float* __restrict__ b,
                                                        bf16* __restrict__ y, long long ldy, float eps) {
  const int lane = threadIdx.x & 63;
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= rows) return;
  const int src = row_idx ? row_idx[r] : r;
  const float2* xr = (const float2*)(x + (long long)src * ldx);
  constexpr int D = 128 * NP;
  float2 v[NP];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NP; ++i) {
    v[i] = xr[lane + 64 * i];
    s += v[i].x + v[i].y;
  }
  const float mean = wave_sum(s) * (1.0f / D);
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < NP; ++i) {
    const float a = v[i].x - mean, c = v[i].y - mean;
    q += a * a + c * c;
  }
  const float rstd = rsqrtf(wave_sum(q) * (1.0f / D) + eps);
  bf16x2* yr = (bf16x2*)(y + (long long)r * ldy);
  const float2* g2 = (const float2*)g;
  const float2* b2 = (const float2*)b;
#pragma unroll
  for (int i = 0; i < NP; ++i) {
    const int c = lane + 64 * i;
    const float2 gg = g2[c], bb = b2[c];
    bf16x2 o;
    o[0] = f2bf((v[i].x - mean) * rstd * gg.x + bb.x);
    o[1] = f2bf((v[i].y - mean) * rstd * gg.y + bb.y);
    yr[c] = o;
  }
}

void launch_layernorm(const float* x, long long ldx, const int* row_idx, int rows, int d, const float* g,
                      const float* b, bf16* y, long long ldy, hipStream_t st) {
  if (rows <= 0) return;
  dim3 grid((rows + 3) / 4), block(256);
  const float eps = 1e-5f;
  switch (d) {
    case 256: hipLaunchKernelGGL(layernorm_kernel<2>, grid, block, 0, st, x, ldx, row_idx, rows, g, b, y, ldy, eps); break;
    case 384: hipLaunchKernelGGL(layernorm_kernel<3>, grid, block, 0, st, x, ldx, row_idx, rows, g, b, y, ldy, eps); break;
    case 512: hipLaunchKernelGGL(layernorm_kernel<4>, grid, block, 0, st, x, ldx, row_idx, rows, g, b, y, ldy, eps); break;
    case 640: hipLaunchKernelGGL(layernorm_kernel<5>, grid, block, 0, st, x, ldx, row_idx, rows, g, b, y, ldy, eps); break;
    case 768: hipLaunchKernelGGL(layernorm_kernel<6>, grid, block, 0, st, x, ldx, row_idx, rows, g, b, y, ldy, eps); break;
    case 1024: hipLaunchKernelGGL(layernorm_kernel<8>, grid, block, 0, st, x, ldx, row_idx, rows, g, b, y, ldy, eps); break;
    case 1280: hipLaunchKernelGGL(layernorm_kernel<10>, grid, block, 0, st, x, ldx, row_idx, rows, g, b, y, ldy, eps); break;
    case 128: hipLaunchKernelGGL(layernorm_kernel<1>, grid, block, 0, st, x, ldx, row_idx, rows, g, b, y, ldy, eps); break;
    default: throw std::runtime_error("layernorm: unsupported width " + std::to_string(d));
  }
  WM_LAUNCH_CHECK("layernorm_kernel");
}

// x[r, :] = E[tok[r], :] + P[pos[r], :]
// A token id or position outside its table is an error (reported through the decode's device error word, which
// the host raises on); the index is also clamped, purely as a memory guard, so the broken row never reads out of
// bounds before the host sees the error.
__global__ void embed_kernel(const int* __restrict__ tok, const int* __restrict__ pos, const bf16* __restrict__ E,
                             const float* __restrict__ P, float* __restrict__ x, int d, int n_vocab, int n_pos,
                             int* __restrict__ err) {
  const int r = blockIdx.x;
  const int t0 = tok[r], p0 = pos[r];
  if ((t0 < 0 || t0 >= n_vocab || p0 < 0 || p0 >= n_pos) && threadIdx.x == 0) wm_report_error(err, WM_ERR_TOKEN_RANGE, t0, p0);
  const long long t = min(max(t0, 0), n_vocab - 1), p = min(max(p0, 0), n_pos - 1);
  for (int c = threadIdx.x; c < d; c += blockDim.x) x[(long long)r * d + c] = bf2f(E[t * d + c]) + P[p * d + c];
}

void launch_embed(const int* tok, const int* pos, const bf16* E, const float* P, float* x, int rows, int d, int n_vocab,
                  int n_pos, hipStream_t st, int* err) {
  if (rows <= 0) return;
  hipLaunchKernelGGL(embed_kernel, dim3(rows), dim3(256), 0, st, tok, pos, E, P, x, d, n_vocab, n_pos, err);
  WM_LAUNCH_CHECK("embed_kernel");
}

// conv1 implicit-GEMM operand: A[b*3000 + t, k*n_mels + c] = win_b(c, t + k - 1), zero outside
// [0, len_b) (conv padding and pad_or_trim), zero for padded columns >= 3*n_mels.
__global__ void im2col_conv1_kernel(const float* __restrict__ mel, long long ld, const int* __restrict__ seek,
                                    const int* __restrict__ len, int n_mels, int kp, bf16* __restrict__ out) {
  const int row = blockIdx.x;               // b*3000 + t
  const int b = row / 3000, t = row - b * 3000;
  const int s0 = seek[b], L = len[b];
  for (int col = threadIdx.x; col < kp; col += blockDim.x) {
    float v = 0.f;
    if (col < 3 * n_mels) {
      const int k = col / n_mels, c = col - k * n_mels;
      const int f = t + k - 1;
      if (f >= 0 && f < L) v = mel[(long long)c * ld + s0 + f];
    }
    out[(long long)row * kp + col] = f2bf(v);
  }
}

void launch_im2col_conv1(const float* mel, long long ld, const int* seek, const int* len, int B, int n_mels, int kp,
                         bf16* out, hipStream_t st) {
  if (B <= 0) return;
  hipLaunchKernelGGL(im2col_conv1_kernel, dim3(B * 3000), dim3(256), 0, st, mel, ld, seek, len, n_mels, kp, out);
  WM_LAUNCH_CHECK("im2col_conv1_kernel");
}

// zero row 0 of every [3001][d] conv1-output block (conv2's left padding)
__global__ void zero_rows_kernel(bf16* __restrict__ h, long long bstride, int d) {
  bf16* p = h + (long long)blockIdx.x * bstride;
  for (int c = threadIdx.x; c < d; c += blockDim.x) p[c] = f2bf(0.f);
}

void launch_zero_pad_rows(bf16* h, int B, long long bstride, int d, hipStream_t st) {
  if (B <= 0) return;
  hipLaunchKernelGGL(zero_rows_kernel, dim3(B), dim3(256), 0, st, h, bstride, d);
  WM_LAUNCH_CHECK("zero_rows_kernel");
}
