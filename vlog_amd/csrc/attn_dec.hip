// Decoder attention for gfx950 — HBM-bound single-query attention ("flash decoding").
//
// Self-attention: one wave per (row, head).  A row is one hypothesis at one position; its keys are
// positions 0..pos, each read from the physical cache slot lin[hyp][p] (beam search reorders hypotheses by
// copying the small lineage table instead of the KV cache; greedy uses lin == identity).
//
// Cross-attention: keys are the 1500 encoder positions of the row's window, cache layout
// [L][2][slot][H][1500][64] so one (slot, head) is a contiguous 192 KB K panel and 192 KB V panel.  The
// 1500 keys are split over `splits` workgroups when there are few rows (parity mode: one window), each
// workgroup streams its K range (scores to LDS), then its V range, and a combine kernel merges the
// (max, sum, o) partials.  8 lanes cover one 128-B key row (16 B per lane), 8 keys per wave-instruction:
// fully coalesced 1 KiB per wave load.  Finished hypotheses are skipped (their rows still flow through
// the weight-bound GEMMs, which read the weights once per step regardless).
#include "common.h"
#include <stdexcept>
#include <string>

#define HD 64
#define MAX_CTX 448

__device__ __forceinline__ void load8(const bf16* p, float* f) {
  const bf16x8 v = *(const bf16x8*)p;
#pragma unroll
  for (int i = 0; i < 8; ++i) f[i] = bf2f(v[i]);
}

__global__ __launch_bounds__(256) void self_attn_kernel(const bf16* __restrict__ q, long long ldq,
                                                        const bf16* __restrict__ kc, const bf16* __restrict__ vc,
                                                        const int* __restrict__ lin, const int* __restrict__ row_hyp,
                                                        const int* __restrict__ row_pos, const int* __restrict__ done,
                                                        bf16* __restrict__ out, long long ldo, int rows, int H,
                                                        int n_ctx, float scale_log2, unsigned long long* stat) {
  __shared__ float s_sc[4][MAX_CTX];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int idx = blockIdx.x * 4 + wv;
  if (idx >= rows * H) return;
  const int row = idx / H, h = idx - row * H;
  const int hyp = row_hyp[row];
  if (done && done[hyp]) return;
  const int pos = row_pos[row];
  const int nk = pos + 1;
  const int sub = lane & 7, g = lane >> 3;
  if (stat && lane == 0) atomicAdd(stat, (unsigned long long)(nk * 2 * HD * 2 + 2 * HD * 2));
  float qf[8];
  load8(q + (long long)row * ldq + h * HD + sub * 8, qf);
#pragma unroll
  for (int i = 0; i < 8; ++i) qf[i] *= scale_log2;
  float* sc = s_sc[wv];
  const int* lrow = lin ? lin + (long long)hyp * n_ctx : nullptr;
  for (int kb = 0; kb < nk; kb += 8) {
    const int p = kb + g;
    float part = 0.f;
    if (p < nk) {
      const int ph = lrow ? lrow[p] : hyp;
      float kf[8];
      load8(kc + (((long long)ph * H + h) * n_ctx + p) * HD + sub * 8, kf);
#pragma unroll
      for (int i = 0; i < 8; ++i) part = fmaf(qf[i], kf[i], part);
    }
    part += __shfl_xor(part, 1, 64);
    part += __shfl_xor(part, 2, 64);
    part += __shfl_xor(part, 4, 64);
    if (sub == 0 && p < nk) sc[p] = part;
  }
  __builtin_amdgcn_s_waitcnt(0);
  __builtin_amdgcn_wave_barrier();
  float mx = -INFINITY;
  for (int p = lane; p < nk; p += 64) mx = fmaxf(mx, sc[p]);
  mx = wave_max(mx);
  float sum = 0.f;
  for (int p = lane; p < nk; p += 64) {
    const float e = exp2f(sc[p] - mx);
    sc[p] = e;
    sum += e;
  }
  sum = wave_sum(sum);
  __builtin_amdgcn_wave_barrier();
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  for (int p = g; p < nk; p += 8) {
    const int ph = lrow ? lrow[p] : hyp;
    const float w = sc[p];
    float vf[8];
    load8(vc + (((long long)ph * H + h) * n_ctx + p) * HD + sub * 8, vf);
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[i] = fmaf(w, vf[i], acc[i]);
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    acc[i] += __shfl_xor(acc[i], 8, 64);
    acc[i] += __shfl_xor(acc[i], 16, 64);
    acc[i] += __shfl_xor(acc[i], 32, 64);
  }
  if (g == 0) {
    const float inv = 1.0f / sum;
    bf16x8 o;
#pragma unroll
    for (int i = 0; i < 8; ++i) o[i] = f2bf(acc[i] * inv);
    *(bf16x8*)(out + (long long)row * ldo + h * HD + sub * 8) = o;
  }
}

void launch_self_attn(const bf16* q, long long ldq, const bf16* kc, const bf16* vc, const int* lin, const int* row_hyp,
                      const int* row_pos, const int* done, bf16* out, long long ldo, int rows, int H, int n_ctx,
                      unsigned long long* stat, hipStream_t st) {
  if (rows <= 0) return;
  if (n_ctx > MAX_CTX) throw std::runtime_error("self_attn: n_ctx > 448");
  const float scale_log2 = 0.125f * 1.4426950408889634f;
  dim3 grid((rows * H + 3) / 4);
  hipLaunchKernelGGL(self_attn_kernel, grid, dim3(256), 0, st, q, ldq, kc, vc, lin, row_hyp, row_pos, done, out, ldo,
                     rows, H, n_ctx, scale_log2, stat);
  WM_LAUNCH_CHECK("self_attn_kernel");
}

// ------------------------------------------------------------------------------------------ cross
#define CT_MAX 1536

__global__ __launch_bounds__(256) void cross_attn_kernel(
    const bf16* __restrict__ q, long long ldq, const bf16* __restrict__ kbase, const bf16* __restrict__ vbase,
    long long panel, const int* __restrict__ hyp_slot, const int* __restrict__ row_hyp, const int* __restrict__ done,
    bf16* __restrict__ out, long long ldo, int H, int T, int splits, float* __restrict__ part_m,
    float* __restrict__ part_l, float* __restrict__ part_o, float* __restrict__ probs, const int* __restrict__ head_map,
    int n_align, float scale_log2, unsigned long long* stat) {
  __shared__ float s_sc[CT_MAX];
  __shared__ float s_red[4];
  __shared__ float s_acc[4][HD];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int pair = blockIdx.x;              // row * H + h
  const int split = blockIdx.y;
  const int row = pair / H, h = pair - row * H;
  const int hyp = row_hyp[row];
  if (done && done[hyp]) return;
  const int slot = hyp_slot[hyp];
  const int chunk = (T + splits - 1) / splits;
  const int k0 = split * chunk, k1 = min(T, k0 + chunk), nk = k1 - k0;
  if (stat && tid == 0) atomicAdd(stat, (unsigned long long)(nk * 2 * HD * 2 + 2 * HD * 2));
  const long long off = ((long long)slot * H + h) * panel;       // panel = T * HD
  const bf16* K = kbase + off;
  const bf16* V = vbase + off;
  const int sub = lane & 7, g = lane >> 3;
  float qf[8];
  load8(q + (long long)row * ldq + h * HD + sub * 8, qf);
#pragma unroll
  for (int i = 0; i < 8; ++i) qf[i] *= scale_log2;

  for (int kb = 0; kb < nk; kb += 32) {
    const int p = kb + wv * 8 + g;
    float part = 0.f;
    if (p < nk) {
      float kf[8];
      load8(K + (long long)(k0 + p) * HD + sub * 8, kf);
#pragma unroll
      for (int i = 0; i < 8; ++i) part = fmaf(qf[i], kf[i], part);
    }
    part += __shfl_xor(part, 1, 64);
    part += __shfl_xor(part, 2, 64);
    part += __shfl_xor(part, 4, 64);
    if (sub == 0 && p < nk) s_sc[p] = part;
  }
  __syncthreads();
  float mx = -INFINITY;
  for (int p = tid; p < nk; p += 256) mx = fmaxf(mx, s_sc[p]);
  mx = wave_max(mx);
  if (lane == 0) s_red[wv] = mx;
  __syncthreads();
  mx = fmaxf(fmaxf(s_red[0], s_red[1]), fmaxf(s_red[2], s_red[3]));
  __syncthreads();
  float sum = 0.f;
  for (int p = tid; p < nk; p += 256) {
    const float e = exp2f(s_sc[p] - mx);
    s_sc[p] = e;
    sum += e;
  }
  sum = wave_sum(sum);
  if (lane == 0) s_red[wv] = sum;
  __syncthreads();
  sum = s_red[0] + s_red[1] + s_red[2] + s_red[3];

  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  for (int kb = 0; kb < nk; kb += 32) {
    const int p = kb + wv * 8 + g;
    if (p < nk) {
      const float w = s_sc[p];
      float vf[8];
      load8(V + (long long)(k0 + p) * HD + sub * 8, vf);
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[i] = fmaf(w, vf[i], acc[i]);
    }
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    acc[i] += __shfl_xor(acc[i], 8, 64);
    acc[i] += __shfl_xor(acc[i], 16, 64);
    acc[i] += __shfl_xor(acc[i], 32, 64);
  }
  if (g == 0) {
#pragma unroll
    for (int i = 0; i < 8; ++i) s_acc[wv][sub * 8 + i] = acc[i];
  }
  if (probs && head_map[h] >= 0) {
    const float inv = 1.0f / sum;
    float* pr = probs + ((long long)row * n_align + head_map[h]) * T;
    for (int p = tid; p < nk; p += 256) pr[k0 + p] = s_sc[p] * inv;
  }
  __syncthreads();
  if (tid < HD) {
    const float a = s_acc[0][tid] + s_acc[1][tid] + s_acc[2][tid] + s_acc[3][tid];
    if (splits == 1) {
      out[(long long)row * ldo + h * HD + tid] = f2bf(a / sum);
    } else {
      const long long pi = (long long)pair * splits + split;
      part_o[pi * HD + tid] = a;
      if (tid == 0) { part_m[pi] = mx; part_l[pi] = sum; }
    }
  }
}

__global__ void cross_combine_kernel(const float* __restrict__ part_m, const float* __restrict__ part_l,
                                     const float* __restrict__ part_o, const int* __restrict__ row_hyp,
                                     const int* __restrict__ done, bf16* __restrict__ out, long long ldo, int H,
                                     int splits) {
  const int pair = blockIdx.x;
  const int row = pair / H, h = pair - row * H;
  if (done && done[row_hyp[row]]) return;
  const int e = threadIdx.x;
  const long long pb = (long long)pair * splits;
  float M = -INFINITY;
  for (int s = 0; s < splits; ++s) M = fmaxf(M, part_m[pb + s]);
  float L = 0.f, o = 0.f;
  for (int s = 0; s < splits; ++s) {
    const float w = exp2f(part_m[pb + s] - M);
    L += part_l[pb + s] * w;
    o += part_o[(pb + s) * HD + e] * w;
  }
  out[(long long)row * ldo + h * HD + e] = f2bf(o / L);
}

void launch_cross_attn(const bf16* q, long long ldq, const bf16* kbase, const bf16* vbase, int T, const int* hyp_slot,
                       const int* row_hyp, const int* done, bf16* out, long long ldo, int rows, int H, int splits,
                       float* part_m, float* part_l, float* part_o, float* probs, const int* head_map, int n_align,
                       unsigned long long* stat, hipStream_t st) {
  if (rows <= 0) return;
  if (T > CT_MAX * splits) throw std::runtime_error("cross_attn: too many keys per split");
  if (probs && splits != 1) throw std::runtime_error("cross_attn: attention capture needs splits == 1");
  const float scale_log2 = 0.125f * 1.4426950408889634f;
  dim3 grid(rows * H, splits);
  hipLaunchKernelGGL(cross_attn_kernel, grid, dim3(256), 0, st, q, ldq, kbase, vbase, (long long)T * HD, hyp_slot,
                     row_hyp, done, out, ldo, H, T, splits, part_m, part_l, part_o, probs, head_map, n_align,
                     scale_log2, stat);
  WM_LAUNCH_CHECK("cross_attn_kernel");
  if (splits > 1) {
    hipLaunchKernelGGL(cross_combine_kernel, dim3(rows * H), dim3(HD), 0, st, part_m, part_l, part_o, row_hyp, done,
                       out, ldo, H, splits);
    WM_LAUNCH_CHECK("cross_combine_kernel");
  }
}
