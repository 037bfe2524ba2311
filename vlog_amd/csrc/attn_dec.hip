// Decoder attention for gfx950 — HBM-bound single-query attention ("flash decoding").
//
// Self-attention: a row is one hypothesis at one position; its keys are positions 0..pos, each read from
// the physical cache slot lin[hyp][p] (beam search reorders hypotheses by copying the small lineage table
// instead of the KV cache; greedy uses lin == identity).
//
// Cross-attention: keys are the 1500 encoder positions of the row's window, cache layout
// [L][2][slot][H][1500][64] so one (slot, head) is a contiguous 192 KB K panel and 192 KB V panel.  The
// 1500 keys are split over `splits` workgroups when there are few rows (parity mode: one window), each
// workgroup streams its K range (scores to LDS), then its V range, and a combine kernel merges the
// (max, sum, o) partials.  8 lanes cover one 128-B key row (16 B per lane), 8 keys per wave-instruction:
// fully coalesced 1 KiB per wave load.  Finished hypotheses are skipped (their rows still flow through
// the weight-bound GEMMs, which read the weights once per step regardless).
#include "common.h"
#include <hip/hip_ext.h>
#include <stdexcept>
#include <string>

#define HD 64
#define MAX_CTX 448

__device__ __forceinline__ void load8(const bf16* p, float* f) {
  const bf16x8 v = *(const bf16x8*)p;
#pragma unroll
  for (int i = 0; i < 8; ++i) f[i] = bf2f(v[i]);
}

struct DecAttnArgs {
  const bf16* q; long long ldq;
  const bf16* kbase; const bf16* vbase;   // cross: [slot][H][T][64] panels; self: [n_hyp][H][n_ctx][64]
  const int* hyp_slot; const int* row_hyp; const int* row_pos; const int* done; const int* lin;
  bf16* out; long long ldo;
  int H, T, n_ctx, splits;
  float* part_m; float* part_l; float* part_o;
  float* probs; const int* head_map; int n_align;
  float scale_log2;
  unsigned long long* stat;
};

#define CT_MAX 1536

// One 256-thread workgroup per (row, head[, key split]); 4 waves x 8 keys per step, 8 lanes x 16 B per key row.
// SELF: keys are positions 0..row_pos of the row's hypothesis, each from physical slot lin[hyp][p].
// CROSS: keys are the 1500 encoder positions of the hypothesis's window slot.
template <bool SELF>
__global__ __launch_bounds__(256) void dec_attn_kernel(DecAttnArgs a) {
  __shared__ float s_sc[CT_MAX];
  __shared__ float s_red[4];
  __shared__ float s_acc[4][HD];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int pair = blockIdx.x;              // row * H + h
  const int split = blockIdx.y;
  const int H = a.H;
  const int row = pair / H, h = pair - row * H;
  const int hyp = a.row_hyp[row];
  if (a.done && a.done[hyp]) return;
  int k0, nk;
  const bf16* K;
  const bf16* V;
  const int* lrow = nullptr;
  if (SELF) {
    k0 = 0;
    nk = a.row_pos[row] + 1;
    lrow = a.lin ? a.lin + (long long)hyp * a.n_ctx : nullptr;
    K = a.kbase + (long long)h * a.n_ctx * HD;
    V = a.vbase + (long long)h * a.n_ctx * HD;
  } else {
    const int chunk = (a.T + a.splits - 1) / a.splits;
    k0 = split * chunk;
    nk = min(a.T, k0 + chunk) - k0;
    const long long off = ((long long)a.hyp_slot[hyp] * H + h) * ((long long)a.T * HD);
    K = a.kbase + off;
    V = a.vbase + off;
  }
  if (a.stat && tid == 0) atomicAdd(a.stat, (unsigned long long)(nk * 2 * HD * 2 + 2 * HD * 2));
  const long long hstride = (long long)H * a.n_ctx * HD;    // SELF: elements per physical hypothesis
  const int sub = lane & 7, g = lane >> 3;
  float qf[8];
  load8(a.q + (long long)row * a.ldq + h * HD + sub * 8, qf);
#pragma unroll
  for (int i = 0; i < 8; ++i) qf[i] *= a.scale_log2;

  auto krow = [&](const bf16* base, int p) -> const bf16* {
    if (SELF) {
      const int ph = lrow ? lrow[p] : hyp;
      return base + ph * hstride + (long long)p * HD;
    }
    return base + (long long)(k0 + p) * HD;
  };

  for (int kb = 0; kb < nk; kb += 64) {
    float part[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int p = kb + u * 32 + wv * 8 + g;
      part[u] = 0.f;
      if (p < nk) {
        float kf[8];
        load8(krow(K, p) + sub * 8, kf);
#pragma unroll
        for (int i = 0; i < 8; ++i) part[u] = fmaf(qf[i], kf[i], part[u]);
      }
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      float v = part[u];
      v += __shfl_xor(v, 1, 64);
      v += __shfl_xor(v, 2, 64);
      v += __shfl_xor(v, 4, 64);
      const int p = kb + u * 32 + wv * 8 + g;
      if (sub == 0 && p < nk) s_sc[p] = v;
    }
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
  for (int kb = 0; kb < nk; kb += 64) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int p = kb + u * 32 + wv * 8 + g;
      if (p < nk) {
        const float w = s_sc[p];
        float vf[8];
        load8(krow(V, p) + sub * 8, vf);
#pragma unroll
        for (int i = 0; i < 8; ++i) acc[i] = fmaf(w, vf[i], acc[i]);
      }
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
  if (!SELF && a.probs && a.head_map[h] >= 0) {
    const float inv = 1.0f / sum;
    float* pr = a.probs + ((long long)row * a.n_align + a.head_map[h]) * a.T;
    for (int p = tid; p < nk; p += 256) pr[k0 + p] = s_sc[p] * inv;
  }
  __syncthreads();
  if (tid < HD) {
    const float v = s_acc[0][tid] + s_acc[1][tid] + s_acc[2][tid] + s_acc[3][tid];
    if (SELF || a.splits == 1) {
      a.out[(long long)row * a.ldo + h * HD + tid] = f2bf(v / sum);
    } else {
      const long long pi = (long long)pair * a.splits + split;
      a.part_o[pi * HD + tid] = v;
      if (tid == 0) { a.part_m[pi] = mx; a.part_l[pi] = sum; }
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

static void launch_k(bool self, dim3 grid, const DecAttnArgs& a, hipStream_t st, hipEvent_t ev0, hipEvent_t ev1) {
  if (ev0) {
    if (self) hipExtLaunchKernelGGL(dec_attn_kernel<true>, grid, dim3(256), 0, st, ev0, ev1, 0, a);
    else hipExtLaunchKernelGGL(dec_attn_kernel<false>, grid, dim3(256), 0, st, ev0, ev1, 0, a);
  } else {
    if (self) hipLaunchKernelGGL(dec_attn_kernel<true>, grid, dim3(256), 0, st, a);
    else hipLaunchKernelGGL(dec_attn_kernel<false>, grid, dim3(256), 0, st, a);
  }
}

void launch_self_attn(const bf16* q, long long ldq, const bf16* kc, const bf16* vc, const int* lin, const int* row_hyp,
                      const int* row_pos, const int* done, bf16* out, long long ldo, int rows, int H, int n_ctx,
                      unsigned long long* stat, hipStream_t st, hipEvent_t ev0, hipEvent_t ev1) {
  if (rows <= 0) return;
  if (n_ctx > CT_MAX) throw std::runtime_error("self_attn: n_ctx too large");
  DecAttnArgs a{};
  a.q = q; a.ldq = ldq; a.kbase = kc; a.vbase = vc; a.row_hyp = row_hyp; a.row_pos = row_pos; a.done = done; a.lin = lin;
  a.out = out; a.ldo = ldo; a.H = H; a.T = n_ctx; a.n_ctx = n_ctx; a.splits = 1;
  a.scale_log2 = 0.125f * 1.4426950408889634f; a.stat = stat;
  launch_k(true, dim3(rows * H, 1), a, st, ev0, ev1);
  WM_LAUNCH_CHECK("dec_attn_kernel<self>");
}

void launch_cross_attn(const bf16* q, long long ldq, const bf16* kbase, const bf16* vbase, int T, const int* hyp_slot,
                       const int* row_hyp, const int* done, bf16* out, long long ldo, int rows, int H, int splits,
                       float* part_m, float* part_l, float* part_o, float* probs, const int* head_map, int n_align,
                       unsigned long long* stat, hipStream_t st, hipEvent_t ev0, hipEvent_t ev1) {
  if (rows <= 0) return;
  if (T > CT_MAX * splits) throw std::runtime_error("cross_attn: too many keys per split");
  if (probs && splits != 1) throw std::runtime_error("cross_attn: attention capture needs splits == 1");
  DecAttnArgs a{};
  a.q = q; a.ldq = ldq; a.kbase = kbase; a.vbase = vbase; a.hyp_slot = hyp_slot; a.row_hyp = row_hyp; a.done = done;
  a.out = out; a.ldo = ldo; a.H = H; a.T = T; a.n_ctx = T; a.splits = splits;
  a.part_m = part_m; a.part_l = part_l; a.part_o = part_o; a.probs = probs; a.head_map = head_map; a.n_align = n_align;
  a.scale_log2 = 0.125f * 1.4426950408889634f; a.stat = stat;
  launch_k(false, dim3(rows * H, splits), a, st, ev0, ev1);
  WM_LAUNCH_CHECK("dec_attn_kernel<cross>");
  if (splits > 1) {
    hipLaunchKernelGGL(cross_combine_kernel, dim3(rows * H), dim3(HD), 0, st, part_m, part_l, part_o, row_hyp, done,
                       out, ldo, H, splits);
    WM_LAUNCH_CHECK("cross_combine_kernel");
  }
}
