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
#include <type_traits>
#include <hip/hip_ext.h>
#include <algorithm>
#include <stdexcept>
#include <string>

#define HD 64
#define MAX_CTX 448

__device__ __forceinline__ void load8(const bf16* p, float* f) {
  const bf16x8 v = *(const bf16x8*)p;
#pragma unroll
  for (int i = 0; i < 8; ++i) f[i] = bf2f(v[i]);
}

// Cross-KV panels are read once per decode step (36.9 GB per step for 150 large-v3 windows, far past the
// 256 MB MALL): non-temporal loads keep them from evicting the weights and activations that are re-read.
__device__ __forceinline__ bf16x8 ld_stream(const bf16* p) {
  return __builtin_bit_cast(bf16x8, __builtin_nontemporal_load((const i32x4*)p));
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
  unsigned long long* stat;   // profiler byte counter: STAT_SLOTS slots, summed on read (no hot atomic)
  // cross, fused forms: (1) q = bf16(sum of q_splits split-K slabs [s][q_rows][ldq] + q_bias) instead of
  // reading a.q (the cq projection's combine folded in, same summation order as splitk_reduce_kernel);
  // (2) key splits combined in-kernel by the last-arriving split of each (group, head), counted in cnt
  // (zero between launches: the last arriver resets its word).
  const float* q_part; int q_splits, q_rows; const float* q_bias;
  int* cnt;
  // self-attention of beam groups (sgroup = hypotheses per window > 1): the (row, head) pairs are walked as (window,
  // head, hypothesis) in XCD-contiguous block order, so one head's waves of a window's beams run together on one XCD
  // and the history rows the beams share (the lineage) are fetched from HBM once and served by its L1 / L2
  int sgroup;
};

#define CT_MAX 1536
#define QMAXS 16               // max cq split-K slabs summed in the cross-attention q load

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
  if (a.stat && tid == 0) atomicAdd(a.stat + (blockIdx.x & (STAT_SLOTS - 1)), (unsigned long long)(nk * 2 * HD * 2 + 2 * HD * 2));
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
  const int e = threadIdx.x;
  const long long pb = (long long)pair * splits;
  // every load requested before any is used (a runtime loop over the splits paid one dependent round trip per split
  // and operand: ~6 us per launch at 12 splits); sums in split order as before.  The done flag (row -> hypothesis ->
  // flag) goes out around the partials instead of two round trips ahead of them (a finished row's partials are read
  // and dropped).  All as vector loads from an opaque zero offset, so the compiler can neither turn the uniform
  // ones into scalar loads waited one batch later nor hoist the flag's branch above the partials.
  int z = 0;
  asm volatile("" : "+v"(z));
  // (branch-free: without a done table both loads read part_m's first word and are ignored)
  const int hyp = *((done ? row_hyp + row : (const int*)part_m) + z);
  constexpr int SMAX = 16;
  float pm[SMAX], pl[SMAX], po[SMAX];
#pragma unroll
  for (int s = 0; s < SMAX; ++s) {
    const long long q = pb + (s < splits ? s : 0) + z;
    pm[s] = part_m[q];
    pl[s] = part_l[q];
    po[s] = part_o[q * HD + e];
  }
  const int flag = *(done ? done + hyp : (const int*)part_m);
  const bool dead = done && flag;
  float M = -INFINITY;
#pragma unroll
  for (int s = 0; s < SMAX; ++s)
    if (s < splits) M = fmaxf(M, pm[s]);
  float L = 0.f, o = 0.f;
#pragma unroll
  for (int s = 0; s < SMAX; ++s)
    if (s < splits) {
      const float w = exp2f(pm[s] - M);
      L += pl[s] * w;
      o += po[s] * w;
    }
  if (!dead) out[(long long)row * ldo + h * HD + e] = f2bf(o / L);
}

// The key-split merge of one (row, head, element) from partials another block wrote through to L2 (agent-scope
// loads): cross_combine_kernel's arithmetic and order, every load requested before any is used (clamped indices,
// no per-split branch: a branch per split made each load wait for the previous one, ~16 round trips at 16 splits)
__device__ __forceinline__ float combine_l2(const float* part_m, const float* part_l, const float* part_o,
                                            long long pb, int splits, int e) {
  constexpr int SMAX = 16;
  float pm[SMAX], pl[SMAX], po[SMAX];
#pragma unroll
  for (int s = 0; s < SMAX; ++s) {
    const long long q = pb + (s < splits ? s : 0);
    pm[s] = __hip_atomic_load(part_m + q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    pl[s] = __hip_atomic_load(part_l + q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    po[s] = __hip_atomic_load(part_o + q * HD + e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  float M = -INFINITY;
#pragma unroll
  for (int s = 0; s < SMAX; ++s)
    if (s < splits) M = fmaxf(M, pm[s]);
  float L = 0.f, o = 0.f;
#pragma unroll
  for (int s = 0; s < SMAX; ++s)
    if (s < splits) {
      const float w = exp2f(pm[s] - M);
      L += pl[s] * w;
      o += po[s] * w;
    }
  return o / L;
}

// ------------------------------------------------------------------------------------------------------
// Cross-attention, single pass (flash decoding) over RG query rows that share one window slot — the
// beam hypotheses of a window, or the prompt positions of a prefill — so each (slot, head) K/V panel is
// streamed from HBM once per group instead of once per row.  One 256-thread block per (group, head[, key
// split]); 8 lanes x 16 B cover one 128-B key row, each lane group of 8 lanes takes every 8th key of its
// wave, and every lane issues the K AND V rows of 4 keys before using any (8 x 16 B in flight per lane).
// Per (row, lane group) an online softmax keeps (m, l, o[8]); groups merge by xor-shuffles, waves through
// LDS.  With splits > 1 the (m, l, o) partials go to cross_combine_kernel (per row, as the legacy path).
template <int RG>
__device__ __forceinline__ void cross_item(const DecAttnArgs& a, int bx, int split, float (&s_m)[4][RG],
                                           float (&s_l)[4][RG], float (&s_o)[4][RG][HD], float (&s_q)[RG][HD]) {
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int sub = lane & 7, g = lane >> 3;
  const int H = a.H;
  const int grp = bx / H, h = bx - grp * H;
  const int row0 = grp * RG;
  bool live[RG];
  bool any = false;
#pragma unroll
  for (int r = 0; r < RG; ++r) {
    live[r] = !(a.done && a.done[a.row_hyp[row0 + r]]);
    any |= live[r];
  }
  if (!any) return;
  const int chunk = (a.T + a.splits - 1) / a.splits;
  const int k0 = split * chunk;
  const int nk = min(a.T, k0 + chunk) - k0;
  const long long off = ((long long)a.hyp_slot[a.row_hyp[row0]] * H + h) * ((long long)a.T * HD) + (long long)k0 * HD;
  const bf16* K = a.kbase + off + sub * 8;
  const bf16* V = a.vbase + off + sub * 8;
  if (a.stat && tid == 0)
    atomicAdd(a.stat + ((bx + split) & (STAT_SLOTS - 1)), (unsigned long long)(nk * 2 * HD * 2 + RG * 2 * HD * 2));

  // the first 128-key chunk's K and V rows are requested before the q load (they do not depend on it): one
  // memory round trip for both instead of two in sequence
  bf16x8 kr[4], vr[4];
  bool ok[4];
  auto load_chunk = [&](int kb) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int p = kb + u * 32 + wv * 8 + g;
      ok[u] = p < nk;
      const int pc = ok[u] ? p : 0;
      kr[u] = ld_stream(K + (long long)pc * HD);
      vr[u] = ld_stream(V + (long long)pc * HD);
    }
  };
  load_chunk(0);
  float qf[RG][8];
  if (a.q_part) {
    // the cq split-K slabs summed into q by the whole block in ONE memory round trip (every slab load of a
    // value issued before any add), in slab order plus the bias as splitk_reduce_kernel does (bit-identical
    // to the unfused bf16 q); the rows go through LDS.  (Per lane and row, a runtime loop over the slabs paid
    // one dependent round trip per slab and row: ~18 us per launch at 5 rows x 4 slabs.)
    // (a thread's NIT values are unrolled too: their loads go out together, not one round trip per value)
    const long long slab = (long long)a.q_rows * a.ldq;
    constexpr int NIT = (RG * HD + 255) / 256;
    float pv[NIT][QMAXS], bq[NIT];
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
      const int idx = min(tid + 256 * it, RG * HD - 1);
      const int r = idx / HD, e = idx - r * HD;
      const float* pq = a.q_part + (long long)(row0 + r) * a.ldq + h * HD + e;
#pragma unroll
      for (int sp = 0; sp < QMAXS; ++sp)
        if (sp < a.q_splits) pv[it][sp] = pq[sp * slab];
      bq[it] = a.q_bias[h * HD + e];
    }
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
      const int idx = tid + 256 * it;
      if (idx >= RG * HD) break;
      const int r = idx / HD, e = idx - r * HD;
      float v = 0.f;
#pragma unroll
      for (int sp = 0; sp < QMAXS; ++sp)
        if (sp < a.q_splits) v += pv[it][sp];
      s_q[r][e] = bf2f(f2bf(v + bq[it]));
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < RG; ++r)
#pragma unroll
      for (int i = 0; i < 8; ++i) qf[r][i] = s_q[r][sub * 8 + i] * a.scale_log2;
  } else {
#pragma unroll
    for (int r = 0; r < RG; ++r) {
      load8(a.q + (long long)(row0 + r) * a.ldq + h * HD + sub * 8, qf[r]);
#pragma unroll
      for (int i = 0; i < 8; ++i) qf[r][i] *= a.scale_log2;
    }
  }
  float m[RG], l[RG], o[RG][8];
#pragma unroll
  for (int r = 0; r < RG; ++r) {
    m[r] = -INFINITY;
    l[r] = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) o[r][i] = 0.f;
  }
  for (int kb = 0; kb < nk; kb += 128) {
    if (kb > 0) load_chunk(kb);
#pragma unroll
    for (int r = 0; r < RG; ++r) {
      float sc[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        float d = 0.f;
#pragma unroll
        for (int i = 0; i < 8; ++i) d = fmaf(qf[r][i], bf2f(kr[u][i]), d);
        d += __shfl_xor(d, 1, 64);
        d += __shfl_xor(d, 2, 64);
        d += __shfl_xor(d, 4, 64);
        sc[u] = ok[u] ? d : -INFINITY;
      }
      const float mx = fmaxf(fmaxf(m[r], fmaxf(sc[0], sc[1])), fmaxf(sc[2], sc[3]));
      const float ms = mx == -INFINITY ? 0.f : mx;
      const float corr = exp2f(m[r] - ms);
      float pu[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) pu[u] = exp2f(sc[u] - ms);
      l[r] = l[r] * corr + ((pu[0] + pu[1]) + (pu[2] + pu[3]));
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        float x = o[r][i] * corr;
#pragma unroll
        for (int u = 0; u < 4; ++u) x = fmaf(pu[u], bf2f(vr[u][i]), x);
        o[r][i] = x;
      }
      m[r] = mx;
    }
  }
  // merge the 8 lane groups of the wave (same sub, different keys)
#pragma unroll
  for (int r = 0; r < RG; ++r) {
#pragma unroll
    for (int off2 = 8; off2 < 64; off2 <<= 1) {
      const float mo = __shfl_xor(m[r], off2, 64);
      const float lo = __shfl_xor(l[r], off2, 64);
      const float M = fmaxf(m[r], mo);
      const float Ms = M == -INFINITY ? 0.f : M;
      const float ca = exp2f(m[r] - Ms), cb = exp2f(mo - Ms);
      l[r] = l[r] * ca + lo * cb;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const float oo = __shfl_xor(o[r][i], off2, 64);
        o[r][i] = o[r][i] * ca + oo * cb;
      }
      m[r] = M;
    }
    if (g == 0) {
#pragma unroll
      for (int i = 0; i < 8; ++i) s_o[wv][r][sub * 8 + i] = o[r][i];
      if (sub == 0) {
        s_m[wv][r] = m[r];
        s_l[wv][r] = l[r];
      }
    }
  }
  __syncthreads();
  for (int idx = tid; idx < RG * HD; idx += 256) {
    const int r = idx / HD, e = idx - r * HD;
    float M = -INFINITY;
#pragma unroll
    for (int w = 0; w < 4; ++w) M = fmaxf(M, s_m[w][r]);
    const float Ms = M == -INFINITY ? 0.f : M;
    float L = 0.f, O = 0.f;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      const float c = exp2f(s_m[w][r] - Ms);
      L += s_l[w][r] * c;
      O += s_o[w][r][e] * c;
    }
    const int row = row0 + r;
    if (a.splits == 1) {
      if (!(a.done && a.done[a.row_hyp[row]])) a.out[(long long)row * a.ldo + h * HD + e] = f2bf(O / L);
    } else if (a.cnt) {
      // hand-off to the last-arriving split: write-through (sc1) stores of the partial, drained, then one
      // agent-scope ticket per item (cdna_hip_programming.md §6 Guideline 16, R1 / counter form)
      const long long pi = ((long long)row * H + h) * a.splits + split;
      __hip_atomic_store(a.part_o + pi * HD + e, O, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (e == 0) {
        __hip_atomic_store(a.part_m + pi, M, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(a.part_l + pi, L, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    } else {
      const long long pi = ((long long)row * H + h) * a.splits + split;
      a.part_o[pi * HD + e] = O;
      if (e == 0) { a.part_m[pi] = M; a.part_l[pi] = L; }
    }
  }
  if (a.splits > 1 && a.cnt) {
    __shared__ int s_last;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every storing wave's partial has left
    __syncthreads();
    if (tid == 0) {
      int* c = a.cnt + bx;
      const int old = __hip_atomic_fetch_add(c, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const int last = old == a.splits - 1;
      if (last) __hip_atomic_store(c, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      s_last = last;
    }
    __syncthreads();
    if (s_last) {
      // same arithmetic and order as cross_combine_kernel (combine_l2)
      for (int idx = tid; idx < RG * HD; idx += 256) {
        const int r = idx / HD, e = idx - r * HD;
        const int row = row0 + r;
        if (a.done && a.done[a.row_hyp[row]]) continue;
        const long long pb = ((long long)row * H + h) * a.splits;
        a.out[(long long)row * a.ldo + h * HD + e] = f2bf(combine_l2(a.part_m, a.part_l, a.part_o, pb, a.splits, e));
      }
    }
  }
}

// Items (group x head x key split) are walked with a grid stride: launched with one block per item this is
// the plain grid; launched with a capped grid (persistent form) each block takes every gridDim.x-th item, so
// the kernel holds a bounded number of wave slots per CU and kernels on other streams (the decoder's weight
// GEMMs) always find room beside it.
template <int RG>
__global__ __launch_bounds__(256) void cross_attn_group_kernel(DecAttnArgs a, int n_items) {
  __shared__ float s_m[4][RG], s_l[4][RG];
  __shared__ float s_o[4][RG][HD];
  __shared__ float s_q[RG][HD];
  for (int it = blockIdx.x; it < n_items; it += gridDim.x) {
    cross_item<RG>(a, it / a.splits, it % a.splits, s_m, s_l, s_o, s_q);
    __syncthreads();
  }
}

template <int RG>
static void launch_group(int n_items, int cap, const DecAttnArgs& a, hipStream_t st, hipEvent_t ev0, hipEvent_t ev1) {
  const dim3 grid(cap > 0 ? std::min(n_items, cap) : n_items);
  if (ev0) hipExtLaunchKernelGGL(cross_attn_group_kernel<RG>, grid, dim3(256), 0, st, ev0, ev1, 0, a, n_items);
  else hipLaunchKernelGGL(cross_attn_group_kernel<RG>, grid, dim3(256), 0, st, a, n_items);
}

// ------------------------------------------------------------------------------------------------------
// Self-attention, single pass: one WAVE per (row, head), 4 per block, no LDS and no barriers.  A row's
// keys are positions 0..pos of its hypothesis, key p read from physical slot lin[hyp][p] (beam lineage).
// Per chunk (128 keys while more than 64 remain, else 64) each lane fetches one lineage index per 64 keys and the 8
// lane groups get theirs by shuffle; every lane then issues the K and V rows of all its keys of the chunk (16 or 32
// x 16 B in flight) before using them.  Online softmax
// per lane group, merged by xor-shuffles; lanes 0-7 store the 64 outputs (16 B each).
// KSPLIT (few pairs: one window's beam): one BLOCK per (row, head), its 4 waves take contiguous quarters of the
// keys and merge (m, l, o) through LDS in wave order, so a long history costs one chunk per wave instead of a
// chain of dependent chunks in one wave.
template <bool KSPLIT>
__global__ __launch_bounds__(256) void self_attn_wave_kernel(DecAttnArgs a, int n_pairs) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int H = a.H;
  int pair, row, h;
  if (a.sgroup > 1) {
    const int nwg = gridDim.x, bid = blockIdx.x, xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
    const int wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
    pair = KSPLIT ? wgid : wgid * 4 + wv;
    const int K = a.sgroup, j = pair % K, t = pair / K;
    h = t % H;
    row = (t / H) * K + j;
  } else {
    pair = KSPLIT ? (int)blockIdx.x : (int)blockIdx.x * 4 + wv;
    row = pair / H;
    h = pair - row * H;
  }
  if (pair >= n_pairs) return;                         // KSPLIT: uniform over the block
  const int sub = lane & 7, g = lane >> 3;
  // the row's hypothesis, position and q go out together; the done flag (a second dependent load) is only read at
  // the store, so a live row's K/V requests no longer wait for it (a finished row's loads stay in bounds: its
  // position is clamped to the context and its lineage row is valid, and nothing of it is stored)
  const int hyp = a.row_hyp[row];
  const int nk = min(a.row_pos[row] + 1, a.n_ctx);
  float qf[8];
  load8(a.q + (long long)row * a.ldq + h * HD + sub * 8, qf);
  const int kbeg = KSPLIT ? wv * nk / 4 : 0, kend = KSPLIT ? (wv + 1) * nk / 4 : nk;
  const int* lrow = a.lin ? a.lin + (long long)hyp * a.n_ctx : nullptr;
  // the done flag is requested here, with the first keys (read at the store: loaded there, it was one more round trip)
  // (branch-free: without a done table the load reads the row's own hypothesis entry and is ignored)
  const int done_v = *(a.done ? a.done + hyp : a.row_hyp + row);
  const long long hstride = (long long)H * a.n_ctx * HD;
  const bf16* K = a.kbase + (long long)h * a.n_ctx * HD + sub * 8;
  const bf16* V = a.vbase + (long long)h * a.n_ctx * HD + sub * 8;
#pragma unroll
  for (int i = 0; i < 8; ++i) qf[i] *= a.scale_log2;
  float m = -INFINITY, l = 0.f, o[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) o[i] = 0.f;
  // one chunk of 8 U keys: lane group g takes keys kb + 8 u + g, u < U; every K and V row of the chunk is
  // requested before any is used (2 U x 16 B in flight per lane)
  auto chunk = [&](auto uc, int kb) {
    constexpr int U = decltype(uc)::value, NL = U / 8;
    int phl[NL];
#pragma unroll
    for (int j = 0; j < NL; ++j) {
      const int pl = kb + 64 * j + lane;
      phl[j] = (lrow && pl < kend) ? lrow[pl] : hyp;
    }
    bf16x8 kr[U], vr[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int p = kb + u * 8 + g;
      const int ph = __shfl(phl[u >> 3], (u & 7) * 8 + g, 64);
      const int pc = p < kend ? p : 0;
      const long long ro = (long long)ph * hstride + (long long)pc * HD;
      kr[u] = *(const bf16x8*)(K + ro);
      vr[u] = *(const bf16x8*)(V + ro);
    }
    float sc[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      float d = 0.f;
#pragma unroll
      for (int i = 0; i < 8; ++i) d = fmaf(qf[i], bf2f(kr[u][i]), d);
      d += __shfl_xor(d, 1, 64);
      d += __shfl_xor(d, 2, 64);
      d += __shfl_xor(d, 4, 64);
      sc[u] = (kb + u * 8 + g) < kend ? d : -INFINITY;
    }
    float mx = m;
#pragma unroll
    for (int u = 0; u < U; ++u) mx = fmaxf(mx, sc[u]);
    const float ms = mx == -INFINITY ? 0.f : mx;
    const float corr = exp2f(m - ms);
    float pu[U], ps = 0.f;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      pu[u] = exp2f(sc[u] - ms);
      ps += pu[u];
    }
    l = l * corr + ps;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      float x = o[i] * corr;
#pragma unroll
      for (int u = 0; u < U; ++u) x = fmaf(pu[u], bf2f(vr[u][i]), x);
      o[i] = x;
    }
    m = mx;
  };
  // 128-key chunks while more than 64 keys remain (one memory round trip per 128 keys), a 64-key chunk for the rest
  for (int kb = kbeg; kb < kend;) {
    if (kend - kb > 64) {
      chunk(std::integral_constant<int, 16>{}, kb);
      kb += 128;
    } else {
      chunk(std::integral_constant<int, 8>{}, kb);
      kb += 64;
    }
  }
#pragma unroll
  for (int off2 = 8; off2 < 64; off2 <<= 1) {
    const float mo = __shfl_xor(m, off2, 64);
    const float lo = __shfl_xor(l, off2, 64);
    const float M = fmaxf(m, mo);
    const float Ms = M == -INFINITY ? 0.f : M;
    const float ca = exp2f(m - Ms), cb = exp2f(mo - Ms);
    l = l * ca + lo * cb;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const float oo = __shfl_xor(o[i], off2, 64);
      o[i] = o[i] * ca + oo * cb;
    }
    m = M;
  }
  const bool dead = a.done && done_v != 0;
  if (a.stat && !dead && lane == 0 && (!KSPLIT || wv == 0))
    atomicAdd(a.stat + (pair & (STAT_SLOTS - 1)), (unsigned long long)(nk * 2 * HD * 2 + 2 * HD * 2));
  if constexpr (KSPLIT) {
    // the 4 waves' (m, l, o) merged in wave order (a wave with no keys has m = -inf, l = 0, o = 0)
    __shared__ float s_o[4][HD], s_ml[4][2];
    if (g == 0) {
#pragma unroll
      for (int i = 0; i < 8; ++i) s_o[wv][sub * 8 + i] = o[i];
      if (sub == 0) { s_ml[wv][0] = m; s_ml[wv][1] = l; }
    }
    __syncthreads();
    if (wv != 0) return;
    float M = -INFINITY;
#pragma unroll
    for (int w = 0; w < 4; ++w) M = fmaxf(M, s_ml[w][0]);
    float L = 0.f, O[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      const float c = exp2f(s_ml[w][0] - M);
      L += s_ml[w][1] * c;
#pragma unroll
      for (int i = 0; i < 8; ++i) O[i] += s_o[w][sub * 8 + i] * c;
    }
    if (g == 0 && !dead) {
      const float inv = 1.0f / L;
      bf16x8 r;
#pragma unroll
      for (int i = 0; i < 8; ++i) r[i] = f2bf(O[i] * inv);
      *(bf16x8*)(a.out + (long long)row * a.ldo + h * HD + sub * 8) = r;
    }
  } else if (g == 0 && !dead) {
    const float inv = 1.0f / l;
    bf16x8 r;
#pragma unroll
    for (int i = 0; i < 8; ++i) r[i] = f2bf(o[i] * inv);
    *(bf16x8*)(a.out + (long long)row * a.ldo + h * HD + sub * 8) = r;
  }
}

// Cross-attention WITH capture (word alignment, wm_align_batch's teacher-forced pass): one block per (up to RG
// rows of one window, head).  The window's K panel is streamed ONCE for the block's rows (pass 1: each 8-lane group
// takes one key and forms all RG dot products, scores to LDS), each row's softmax is formed in LDS and written out
// for a captured head, then the V panel streams once (pass 3: every row's weighted sum at once).  The per-(row, head)
// form (dec_attn_kernel) streamed both panels per row: ~2 TB of L2/MALL reads per 150-window large-v3 alignment.
template <int RG>
__global__ __launch_bounds__(256) void cross_capture_kernel(DecAttnArgs a, int group, int bpg) {
  __shared__ float s_sc[RG][CT_MAX];
  __shared__ float s_sum[RG];
  __shared__ float s_acc[4][RG][HD];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, sub = lane & 7, kg = tid >> 3;
  const int H = a.H, T = a.T;
  const int h = blockIdx.x % H, rb = blockIdx.x / H;
  const int g = rb / bpg, j = rb - g * bpg;
  const int r0 = g * group + j * RG, nr = min(RG, group - j * RG);
  const int hyp0 = a.row_hyp[r0];
  if (a.done && a.done[hyp0]) return;
  const long long off = ((long long)a.hyp_slot[hyp0] * H + h) * ((long long)T * HD);
  const bf16* K = a.kbase + off;
  const bf16* V = a.vbase + off;
  if (a.stat && tid == 0) atomicAdd(a.stat + (blockIdx.x & (STAT_SLOTS - 1)), (unsigned long long)(T * 2 * HD * 2 + nr * 2 * HD * 2));
  float qf[RG][8];
#pragma unroll
  for (int r = 0; r < RG; ++r) {
    if (r < nr) {
      load8(a.q + (long long)(r0 + r) * a.ldq + h * HD + sub * 8, qf[r]);
#pragma unroll
      for (int i = 0; i < 8; ++i) qf[r][i] *= a.scale_log2;
    } else {
#pragma unroll
      for (int i = 0; i < 8; ++i) qf[r][i] = 0.f;
    }
  }
  // pass 1: scores, 32 keys per iteration (one per 8-lane group)
  for (int kb = 0; kb < T; kb += 32) {
    const int p = kb + kg;
    float kf[8];
    if (p < T) load8(K + (long long)p * HD + sub * 8, kf);
    else {
#pragma unroll
      for (int i = 0; i < 8; ++i) kf[i] = 0.f;
    }
#pragma unroll
    for (int r = 0; r < RG; ++r) {
      float d = 0.f;
#pragma unroll
      for (int i = 0; i < 8; ++i) d = fmaf(qf[r][i], kf[i], d);
      d += __shfl_xor(d, 1, 64);
      d += __shfl_xor(d, 2, 64);
      d += __shfl_xor(d, 4, 64);
      if (sub == 0 && p < T && r < nr) s_sc[r][p] = d;
    }
  }
  __syncthreads();
  // softmax per row: wave w takes rows w, w + 4, ...
  for (int r = wv; r < nr; r += 4) {
    float mx = -INFINITY;
    for (int p = lane; p < T; p += 64) mx = fmaxf(mx, s_sc[r][p]);
    mx = wave_max(mx);
    float sum = 0.f;
    for (int p = lane; p < T; p += 64) {
      const float e = exp2f(s_sc[r][p] - mx);
      s_sc[r][p] = e;
      sum += e;
    }
    sum = wave_sum(sum);
    if (lane == 0) s_sum[r] = sum;
  }
  __syncthreads();
  if (a.probs && a.head_map[h] >= 0) {
    const int hm = a.head_map[h];
    for (int r = 0; r < nr; ++r) {
      const float inv = 1.0f / s_sum[r];
      float* pr = a.probs + ((long long)(r0 + r) * a.n_align + hm) * T;
      for (int p = tid; p < T; p += 256) pr[p] = s_sc[r][p] * inv;
    }
  }
  // pass 3: V, every row at once
  float acc[RG][8];
#pragma unroll
  for (int r = 0; r < RG; ++r)
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[r][i] = 0.f;
  for (int kb = 0; kb < T; kb += 32) {
    const int p = kb + kg;
    if (p < T) {
      float vf[8];
      load8(V + (long long)p * HD + sub * 8, vf);
#pragma unroll
      for (int r = 0; r < RG; ++r) {
        const float w = s_sc[r][p];
#pragma unroll
        for (int i = 0; i < 8; ++i) acc[r][i] = fmaf(w, vf[i], acc[r][i]);
      }
    }
  }
#pragma unroll
  for (int r = 0; r < RG; ++r)
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      acc[r][i] += __shfl_xor(acc[r][i], 8, 64);
      acc[r][i] += __shfl_xor(acc[r][i], 16, 64);
      acc[r][i] += __shfl_xor(acc[r][i], 32, 64);
    }
  if (lane < 8) {
#pragma unroll
    for (int r = 0; r < RG; ++r)
#pragma unroll
      for (int i = 0; i < 8; ++i) s_acc[wv][r][sub * 8 + i] = acc[r][i];
  }
  __syncthreads();
  for (int idx = tid; idx < nr * HD; idx += 256) {
    const int r = idx / HD, e = idx - r * HD;
    const float v = s_acc[0][r][e] + s_acc[1][r][e] + s_acc[2][r][e] + s_acc[3][r][e];
    a.out[(long long)(r0 + r) * a.ldo + h * HD + e] = f2bf(v / s_sum[r]);
  }
}

// ------------------------------------------------------------------------------------------------------
// Cross-attention of a TEACHER-FORCED pass (wm_align_batch / wm_forward with capture: `group` rows of one window,
// up to ~220, against its 1500 keys) on the matrix cores.  The VALU kernels above do ~2 x 64 FMAs per (row, key)
// per head: at 150 windows x ~100 rows x 32 layers that is ~3.7 TFLOP of f32 FMA (~260 ms), while the K/V panels
// are only 1.15 GB per layer.  Here one block = 128 rows (4 waves x 32) of one (window, head): the window's K/V
// panels stream through LDS once per block, S^T = K . Q^T and O^T += V^T . P^T on 32x32x16 bf16 MFMA with the
// encoder kernel's fragment layouts and LDS swizzles (attn_enc.hip attn_enc_v2_kernel).  Differences from it:
// q is used as stored (exact bf16) and the f32 scores are scaled after the MFMA; for a CAPTURED head (head_map >= 0)
// a first pass over K alone forms each row's exact max and sum, so the second pass writes the normalised f32
// probabilities (p = exp2(s - m) / l, as the VALU capture kernel) and accumulates O with the final max (no rescale).
// Uncaptured heads take one pass with the online softmax and deferred rescale.
typedef __attribute__((ext_vector_type(4))) short tf_i16x4;
typedef __attribute__((ext_vector_type(2))) int tf_i32x2;
#define TF_KT 64
#define TF_THR 8.0f
__device__ __forceinline__ int tf_kslot(int r, int c) { return r * 64 + ((c ^ ((r >> 1) & 7)) << 3); }
__device__ __forceinline__ int tf_vslot(int r, int c) { return r * 64 + ((c ^ (((r >> 1) & 1) << 2)) << 3); }

// Key splits (a.splits > 1, no capture): block (window, head, row tile, split) takes tiles [split nt / S, (split+1) nt / S)
// and writes its (m, l, unnormalised o) partial for cross_combine_kernel, as the VALU kernels do.  This is also the
// decode path of beam groups (`group` = the window's hypotheses, 2..32 rows padded to one 32-row wave tile).
__global__ __launch_bounds__(256, 2) void cross_tf_kernel(DecAttnArgs a, int group, int nqt) {
  __shared__ __attribute__((aligned(16))) bf16 smem[2 * 2 * TF_KT * HD];     // [buf][K | V][64 keys][64]
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int ql = lane & 31, hh = lane >> 5;
  const int H = a.H, T = a.T;
  int qt, h, g, sp;
  {
    // XCD-aware: the row tiles of one (window, head) get consecutive remapped ids (one XCD's L2 holds the panels)
    const int nwg = gridDim.x, bid = blockIdx.x, xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
    const int wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
    qt = wgid % nqt;
    int rest = wgid / nqt;
    sp = rest % a.splits;
    rest /= a.splits;
    h = rest % H;
    g = rest / H;
  }
  const int row0 = g * group;
  const int rr = qt * 128 + tid;                 // this thread's row of the liveness vote
  const int r = qt * 128 + wv * 32 + ql;         // this lane's row of the tile
  // The index loads in two dependent batches (row -> hypothesis -> slot / done flag), every load of a batch issued
  // before any of them is used (loaded one at a time, between branches and the vote, they were six round trips)
  int z = 0;                                     // opaque zero: the uniform index loads go out as vector loads
  asm volatile("" : "+v"(z));                    // with their batch (as scalar loads they were sunk to their uses)
  const int hyp0v = a.row_hyp[row0 + z];
  const int hyp_t = a.row_hyp[row0 + min(rr, group - 1)];
  const int hyp_r = a.row_hyp[row0 + min(r, group - 1)];
  const int hmv = a.probs ? a.head_map[h + z] : -1;
  // panels by window slot; without a slot table (the factored form's per-layer projection of the pass's windows)
  // by the pass's window index
  const int slotv = a.hyp_slot ? a.hyp_slot[hyp0v] : hyp0v;
  int done_t = 0, done_r = 0;
  if (a.done) {                                  // one branch: both flags requested together
    done_t = a.done[hyp_t];
    done_r = a.done[hyp_r];
  }
  const int slot = __builtin_amdgcn_readfirstlane(slotv), hm = __builtin_amdgcn_readfirstlane(hmv);
  // Liveness per ROW: the hypotheses of a sampling group (best_of > 1) end at different steps, so the block runs
  // while any row of its tile is live and writes only live rows (the VALU group kernel's rule)
  if (a.done) {
    const bool live = tid < 128 && rr < group && !done_t;
    if (!__syncthreads_or(live)) return;
  }
  const long long off = ((long long)slot * H + h) * ((long long)T * HD);
  const bf16* K = a.kbase + off;
  const bf16* V = a.vbase + off;
  const bool cap = hm >= 0;
  if (a.stat && tid == 0)
    atomicAdd(a.stat + (blockIdx.x & (STAT_SLOTS - 1)), (unsigned long long)((cap ? 3 : 2) * T * HD * 2));
  const bool valid = r < group;
  const bool live = valid && !done_r;            // output writes only for live rows
  const bool wave_on = qt * 128 + wv * 32 < group;     // wave-uniform: a wave with no row only stages tiles
  const float sl2 = a.scale_log2;
  const int ntt = (T + TF_KT - 1) / TF_KT;
  const int tb = sp * ntt / a.splits, te = (sp + 1) * ntt / a.splits;   // this split's key tiles
  const int nt = te - tb;
  i32x4 rk[2], rv[2];
  auto load_tile = [&](int t, bool withv) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int c = tid + i * 256, key = min((tb + t) * TF_KT + (c >> 3), T - 1), ch = c & 7;
      rk[i] = __builtin_nontemporal_load((const i32x4*)(K + (long long)key * HD + ch * 8));
      if (withv) rv[i] = __builtin_nontemporal_load((const i32x4*)(V + (long long)key * HD + ch * 8));
    }
  };
  auto store_tile = [&](int buf, bool withv) {
    bf16* sK = smem + buf * (2 * TF_KT * HD);
    bf16* sV = sK + TF_KT * HD;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int c = tid + i * 256, rr = c >> 3, ch = c & 7;
      *(i32x4*)(sK + tf_kslot(rr, ch)) = rk[i];
      if (withv) *(i32x4*)(sV + tf_vslot(rr, ch)) = rv[i];
    }
  };
  // (requesting the first tile's K and V before the q load, as cross_item does, measured 2 % slower here: 111.5 vs
  // 109.5 ms of cross-attention per 60 s beam-5 call, alternating arms on one box)
  bf16x8 qf[4];
  if (a.q_part) {
    // q = bf16(sum of the cq split-K slabs in slab order + bias), as splitk_reduce_kernel forms it (bit-identical
    // to the unfused bf16 q).  Slabs in chunks of QC, every load of a chunk issued before its adds, indices clamped
    // instead of branched (a runtime loop per slab waited one round trip per slab and 16-column group: 16 at 4 slabs)
    const long long slab = (long long)a.q_rows * a.ldq;
    const float* qp = a.q_part + (long long)(row0 + min(r, group - 1)) * a.ldq + h * HD + 8 * hh;
    constexpr int QC = 4;
    f32x4 v0[4], v1[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) v0[s] = v1[s] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int k0 = 0; k0 < a.q_splits; k0 += QC) {
      f32x4 t0[QC][4], t1[QC][4];
#pragma unroll
      for (int j = 0; j < QC; ++j) {
        const float* pk = qp + (long long)min(k0 + j, a.q_splits - 1) * slab;
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          t0[j][s] = *(const f32x4*)(pk + 16 * s);
          t1[j][s] = *(const f32x4*)(pk + 16 * s + 4);
        }
      }
#pragma unroll
      for (int j = 0; j < QC; ++j) {
        const bool use = k0 + j < a.q_splits;
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          v0[s] = use ? v0[s] + t0[j][s] : v0[s];
          v1[s] = use ? v1[s] + t1[j][s] : v1[s];
        }
      }
    }
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const float* bq = a.q_bias + h * HD + 8 * hh + 16 * s;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        qf[s][j] = f2bf(v0[s][j] + bq[j]);
        qf[s][4 + j] = f2bf(v1[s][j] + bq[4 + j]);
      }
    }
  } else {
    const bf16* qp = a.q + (long long)(row0 + min(r, group - 1)) * a.ldq + h * HD + 8 * hh;
#pragma unroll
    for (int s = 0; s < 4; ++s) qf[s] = *(const bf16x8*)(qp + 16 * s);
  }
  // S^T of the tile's two 32-key blocks, scaled to log2 units, keys past T masked
  auto scores = [&](const bf16* sK, int t, f32x16 (&sc)[2]) {
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
#pragma unroll
      for (int e = 0; e < 16; ++e) sc[kb][e] = 0.f;
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const bf16x8 ka = *(const bf16x8*)(sK + tf_kslot(kb * 32 + ql, 2 * s + hh));
        sc[kb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ka, qf[s], sc[kb], 0, 0, 0);
      }
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int key = (tb + t) * TF_KT + kb * 32 + 8 * (e >> 2) + 4 * hh + (e & 3);
        sc[kb][e] = key < T ? sc[kb][e] * sl2 : -INFINITY;
      }
    }
  };

  float m_run = -INFINITY, l_run = 0.f;
  if (cap) {
    // pass 1: exact row max and sum from K alone (lane-local partials over the lane's half of the keys)
    load_tile(0, false);
    store_tile(0, false);
    __syncthreads();
    for (int t = 0; t < nt; ++t) {
      const bf16* sK = smem + (t & 1) * (2 * TF_KT * HD);
      if (t + 1 < nt) load_tile(t + 1, false);
      if (wave_on) {
        f32x16 sc[2];
        scores(sK, t, sc);
        float mx = m_run;
#pragma unroll
        for (int kb = 0; kb < 2; ++kb)
#pragma unroll
          for (int e = 0; e < 16; ++e) mx = fmaxf(mx, sc[kb][e]);
        float acc = 0.f;
#pragma unroll
        for (int kb = 0; kb < 2; ++kb)
#pragma unroll
          for (int e = 0; e < 16; ++e) acc += exp2f(sc[kb][e] - mx);
        l_run = l_run * exp2f(m_run - mx) + acc;   // mx is finite: every tile holds a key < T
        m_run = mx;
      }
      if (t + 1 < nt) store_tile((t + 1) & 1, false);
      __syncthreads();
    }
    const float mo = __shfl_xor(m_run, 32, 64), lo = __shfl_xor(l_run, 32, 64);
    const float M = fmaxf(m_run, mo);
    l_run = l_run * exp2f(m_run - M) + lo * exp2f(mo - M);
    m_run = M;
  }
  const float inv_cap = cap ? 1.0f / l_run : 0.f;
  float* prow = cap && valid ? a.probs + ((long long)(row0 + r) * a.n_align + hm) * T : nullptr;

  f32x16 o[2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int e = 0; e < 16; ++e) o[i][e] = 0.f;
  load_tile(0, true);
  store_tile(0, true);
  __syncthreads();
  const int G = lane >> 4, gi = lane & 15, gq = gi >> 2, gp = gi & 3;    // tr_b16: group, row q, col block p
  for (int t = 0; t < nt; ++t) {
    const bf16* sK = smem + (t & 1) * (2 * TF_KT * HD);
    const bf16* sV = sK + TF_KT * HD;
    if (t + 1 < nt) load_tile(t + 1, true);
    if (wave_on) {
    f32x16 sc[2];
    scores(sK, t, sc);
    if (!cap) {
      float mx = sc[0][0];
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int e = 0; e < 16; ++e) mx = fmaxf(mx, sc[kb][e]);
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      if (__any(mx > m_run + TF_THR)) {
        const float mn = fmaxf(m_run, mx);
        const float alpha = exp2f(m_run - mn);
        l_run *= alpha;
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int e = 0; e < 16; ++e) o[i][e] *= alpha;
        m_run = mn;
      }
    }
    bf16x8 pf[2][2];                                    // [key block][k-step]
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
      float pv[16];
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        pv[e] = exp2f(sc[kb][e] - m_run);
        if (!cap) l_run += pv[e];
        pf[kb][e >> 3][e & 7] = f2bf(pv[e]);
      }
      if (prow) {
#pragma unroll
        for (int gg = 0; gg < 4; ++gg) {
          const int key = (tb + t) * TF_KT + kb * 32 + 8 * gg + 4 * hh;
          if (key < T)
            *(f32x4*)(prow + key) = f32x4{pv[4 * gg] * inv_cap, pv[4 * gg + 1] * inv_cap, pv[4 * gg + 2] * inv_cap,
                                          pv[4 * gg + 3] * inv_cap};
        }
      }
    }
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int hb = 0; hb < 2; ++hb) {
          tf_i32x2 vw[2];
#pragma unroll
          for (int jh = 0; jh < 2; ++jh) {
            const int row = kb * 32 + 16 * s + 8 * jh + 4 * (G >> 1) + gq;
            const int col = 32 * hb + 16 * (G & 1) + 4 * gp;
            const bf16* ad = sV + tf_vslot(row, col >> 3) + (col & 7);
            // (whole-register bit casts, as attn_enc.hip: an element-wise insert miscompiles on ROCm 7.2)
            vw[jh] = __builtin_bit_cast(tf_i32x2, __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                                                      (__attribute__((address_space(3))) tf_i16x4*)(ad)));
          }
          const bf16x8 va = __builtin_bit_cast(bf16x8, i32x4{vw[0][0], vw[0][1], vw[1][0], vw[1][1]});
          o[hb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(va, pf[kb][s], o[hb], 0, 0, 0);
        }
    }
    if (t + 1 < nt) store_tile((t + 1) & 1, true);
    __syncthreads();
  }
  if (!cap) l_run += __shfl_xor(l_run, 32, 64);
  if (a.splits > 1 && a.cnt) {
    // the combine folded in: every split writes its partial through to L2 (agent-scope stores), drains, and takes
    // one ticket per (group, head, row tile); the last arriver combines with cross_combine_kernel's arithmetic and
    // order (bit-identical to the separate kernel) and re-arms the counter (cdna_hip_programming.md §6 Guideline 16)
    if (valid) {
      const long long pi = ((long long)(row0 + r) * H + h) * a.splits + sp;
#pragma unroll
      for (int hb = 0; hb < 2; ++hb)
#pragma unroll
        for (int gg = 0; gg < 4; ++gg)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            __hip_atomic_store(a.part_o + pi * HD + 32 * hb + 8 * gg + 4 * hh + j, o[hb][4 * gg + j],
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (hh == 0) {
        __hip_atomic_store(a.part_m + pi, m_run, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(a.part_l + pi, l_run, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    __shared__ int s_last;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
      int* c = a.cnt + (g * H + h) * nqt + qt;
      const int old = __hip_atomic_fetch_add(c, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const int last = old == a.splits - 1;
      if (last) __hip_atomic_store(c, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      s_last = last;
    }
    __syncthreads();
    if (!s_last) return;
    const int nr = min(128, group - qt * 128);
    for (int idx = tid; idx < nr * HD; idx += 256) {
      const int rr = idx / HD, e = idx - rr * HD;
      const int row = row0 + qt * 128 + rr;
      if (a.done && a.done[a.row_hyp[row]]) continue;
      const long long pb = ((long long)row * H + h) * a.splits;
      a.out[(long long)row * a.ldo + h * HD + e] = f2bf(combine_l2(a.part_m, a.part_l, a.part_o, pb, a.splits, e));
    }
    return;
  }
  if (valid && a.splits > 1) {
    // partial of this key split (unnormalised o, its max and sum in log2 units) for cross_combine_kernel
    const long long pi = ((long long)(row0 + r) * H + h) * a.splits + sp;
#pragma unroll
    for (int hb = 0; hb < 2; ++hb)
#pragma unroll
      for (int gg = 0; gg < 4; ++gg)
        *(f32x4*)(a.part_o + pi * HD + 32 * hb + 8 * gg + 4 * hh) =
            f32x4{o[hb][4 * gg], o[hb][4 * gg + 1], o[hb][4 * gg + 2], o[hb][4 * gg + 3]};
    if (hh == 0) {
      a.part_m[pi] = m_run;
      a.part_l[pi] = l_run;
    }
    return;
  }
  if (live) {
    const float inv = cap ? inv_cap : 1.0f / l_run;
    bf16* orow = a.out + (long long)(row0 + r) * a.ldo + h * HD;
#pragma unroll
    for (int hb = 0; hb < 2; ++hb)
#pragma unroll
      for (int gg = 0; gg < 4; ++gg) {
        bf16x4 w;
#pragma unroll
        for (int e = 0; e < 4; ++e) w[e] = f2bf(o[hb][4 * gg + e] * inv);
        *(bf16x4*)(orow + 32 * hb + 8 * gg + 4 * hh) = w;
      }
  }
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
                      unsigned long long* stat, hipStream_t st, hipEvent_t ev0, hipEvent_t ev1, int plan_rows, int group) {
  if (rows <= 0) return;
  if (plan_rows < rows) plan_rows = rows;
  DecAttnArgs a{};
  a.sgroup = group > 1 && rows % group == 0 ? group : 0;   // (the pair order only: results are the same either way)
  a.q = q; a.ldq = ldq; a.kbase = kc; a.vbase = vc; a.row_hyp = row_hyp; a.row_pos = row_pos; a.done = done; a.lin = lin;
  a.out = out; a.ldo = ldo; a.H = H; a.T = n_ctx; a.n_ctx = n_ctx; a.splits = 1;
  a.scale_log2 = 0.125f * 1.4426950408889634f; a.stat = stat;
  const int n_pairs = rows * H;
  // few (row, head) pairs (one window's beam, a few windows): a block per pair, keys split over its 4 waves.  A
  // function of the whole PASS's rows (plan_rows), not this launch's slice, so a row's summation order — and so
  // its result, bit for bit — does not depend on how the pass is sliced (decode_split)
  const bool ksplit = plan_rows * H <= 256;
  const dim3 grid(ksplit ? n_pairs : (n_pairs + 3) / 4);
  if (ksplit) {
    if (ev0) hipExtLaunchKernelGGL(self_attn_wave_kernel<true>, grid, dim3(256), 0, st, ev0, ev1, 0, a, n_pairs);
    else hipLaunchKernelGGL(self_attn_wave_kernel<true>, grid, dim3(256), 0, st, a, n_pairs);
  } else {
    if (ev0) hipExtLaunchKernelGGL(self_attn_wave_kernel<false>, grid, dim3(256), 0, st, ev0, ev1, 0, a, n_pairs);
    else hipLaunchKernelGGL(self_attn_wave_kernel<false>, grid, dim3(256), 0, st, a, n_pairs);
  }
  WM_LAUNCH_CHECK("self_attn_wave_kernel");
}

void launch_cross_attn(const bf16* q, long long ldq, const bf16* kbase, const bf16* vbase, int T, const int* hyp_slot,
                       const int* row_hyp, const int* done, bf16* out, long long ldo, int rows, int H, int group,
                       float* part_m, float* part_l, float* part_o, float* probs, const int* head_map, int n_align,
                       int plan_rows, int cap, const CrossFuse& fz, unsigned long long* stat, hipStream_t st,
                       hipEvent_t ev0, hipEvent_t ev1) {
  if (rows <= 0) return;
  if (plan_rows < rows) plan_rows = rows;
  if (fz.q_part && fz.q_splits > QMAXS) throw std::runtime_error("cross_attn: too many cq split-K slabs");
  DecAttnArgs a{};
  a.q_part = fz.q_part; a.q_splits = fz.q_splits; a.q_rows = fz.q_rows; a.q_bias = fz.q_bias; a.cnt = fz.cnt;
  a.q = q; a.ldq = ldq; a.kbase = kbase; a.vbase = vbase; a.hyp_slot = hyp_slot; a.row_hyp = row_hyp; a.done = done;
  a.out = out; a.ldo = ldo; a.H = H; a.T = T; a.n_ctx = T;
  a.part_m = part_m; a.part_l = part_l; a.part_o = part_o; a.probs = probs; a.head_map = head_map; a.n_align = n_align;
  a.scale_log2 = 0.125f * 1.4426950408889634f; a.stat = stat;
  // matrix-core form: teacher-forced passes (>= 16 rows per window), and with fz.mfma the decode passes of row groups
  // (beam hypotheses / prefill rows of a window; 2..32 rows)
  const bool mf_tf = fz.tf && group >= 16;
  const bool mf_dec = !fz.tf && fz.mfma && group >= 2 && group <= 32 && !probs;
  if ((mf_tf || mf_dec) && rows % group == 0) {
    if (probs && !head_map) throw std::runtime_error("cross_attn: capture without a head map");
    const int nqt = (group + 127) / 128;
    const int ntt = (T + 63) / 64;
    int splits = 1;
    if (mf_dec) {
      // key splits until ~one round of blocks fills the chip (256 blocks: at one window, 13 splits of ~2 tiles; a
      // 512-block target, 16 splits, measured 4 % slower: 109 vs 104-105 ms of cross-attention per 60 s beam-5 call,
      // `prof_worker_seq_r04_tf_target_ab.jsonl`); a function of the whole pass (plan_rows), so a row's summation
      // order does not depend on how the pass is sliced
      const int plan_blocks = plan_rows / group * H * nqt;
      splits = std::max(1, std::min(std::min(16, ntt), (256 + plan_blocks - 1) / plan_blocks));
    }
    a.splits = splits;
    // in-kernel combine only for decode key splits (one row tile per group: the counters are rows/group x H)
    a.cnt = mf_dec && nqt == 1 ? fz.tf_cnt : nullptr;
    const long long nblk = (long long)(rows / group) * H * nqt * splits;
    if (nblk > (1LL << 31) - 1) throw std::runtime_error("cross_attn: grid too large");
    if (splits > 1 && (!part_m || !part_l || !part_o)) throw std::runtime_error("cross_attn: no split scratch");
    hipEvent_t e1 = (splits == 1 || a.cnt) ? ev1 : nullptr;
    if (ev0) hipExtLaunchKernelGGL(cross_tf_kernel, dim3((unsigned)nblk), dim3(256), 0, st, ev0, e1, 0, a, group, nqt);
    else hipLaunchKernelGGL(cross_tf_kernel, dim3((unsigned)nblk), dim3(256), 0, st, a, group, nqt);
    WM_LAUNCH_CHECK("cross_tf_kernel");
    if (splits > 1 && !a.cnt) {
      if (ev1)
        hipExtLaunchKernelGGL(cross_combine_kernel, dim3(rows * H), dim3(HD), 0, st, nullptr, ev1, 0, part_m, part_l,
                              part_o, row_hyp, done, out, ldo, H, splits);
      else
        hipLaunchKernelGGL(cross_combine_kernel, dim3(rows * H), dim3(HD), 0, st, part_m, part_l, part_o, row_hyp, done,
                           out, ldo, H, splits);
      WM_LAUNCH_CHECK("cross_combine_kernel");
    }
    return;
  }
  if (!hyp_slot) throw std::runtime_error("cross_attn: no slot table outside the teacher-forced kernel");
  if (probs) {        // attention capture (word alignment): the two-pass kernel keeps the probabilities
    if (T > CT_MAX) throw std::runtime_error("cross_attn: too many keys for capture");
    if (fz.q_part) throw std::runtime_error("cross_attn: fused q slabs unsupported with capture");
    a.splits = 1;
    if (group > 1 && rows % group == 0) {
      constexpr int RG = 8;
      const int bpg = (group + RG - 1) / RG;
      const dim3 grid((rows / group) * bpg * H);
      if (ev0) hipExtLaunchKernelGGL(cross_capture_kernel<RG>, grid, dim3(256), 0, st, ev0, ev1, 0, a, group, bpg);
      else hipLaunchKernelGGL(cross_capture_kernel<RG>, grid, dim3(256), 0, st, a, group, bpg);
      WM_LAUNCH_CHECK("cross_capture_kernel");
      return;
    }
    launch_k(false, dim3(rows * H, 1), a, st, ev0, ev1);
    WM_LAUNCH_CHECK("dec_attn_kernel<cross>");
    return;
  }
  // rows [k RG, (k+1) RG) share a slot: RG = the largest divisor of `group` (rows sharing a slot,
  // contiguous) that is <= 8 and divides rows
  int rg = 1;
  for (int c = 8; c >= 1; --c)
    if (group % c == 0 && rows % c == 0) { rg = c; break; }
  const int blocks = rows / rg * H;
  // RG = 1 is HBM-bound: split keys until the last round of resident blocks (~1280 at RG = 1) is a small
  // fraction; RG > 1 does RG x the VALU work per byte, so only fill the chip (~2048 blocks).  The split count
  // follows `plan_rows` (the whole pass), not this launch's rows, so a row's summation order — and so its
  // result, bit for bit — does not depend on how the pass was sliced into launches.
  const int plan_blocks = plan_rows / rg * H;
  int splits = ((rg == 1 ? 10240 : 2048) + plan_blocks - 1) / plan_blocks;
  // at most one 128-key pass per block when the grid is small (a 1500-key window: 12 splits of 125 keys, not
  // 11 of 137, which took a second, nearly empty pass through the dependent load loop)
  splits = std::max(1, std::min(splits, std::min(16, (T + 127) / 128)));
  a.splits = splits;
  const int n_items = blocks * splits;
  // events (profiler): start on the attention kernel, stop on the last kernel of the pair
  hipEvent_t e0 = ev0, e1 = (splits == 1 || fz.cnt) ? ev1 : nullptr;
  switch (rg) {
    case 1: launch_group<1>(n_items, cap, a, st, e0, e1); break;
    case 2: launch_group<2>(n_items, cap, a, st, e0, e1); break;
    case 3: launch_group<3>(n_items, cap, a, st, e0, e1); break;
    case 4: launch_group<4>(n_items, cap, a, st, e0, e1); break;
    case 5: launch_group<5>(n_items, cap, a, st, e0, e1); break;
    case 6: launch_group<6>(n_items, cap, a, st, e0, e1); break;
    case 7: launch_group<7>(n_items, cap, a, st, e0, e1); break;
    default: launch_group<8>(n_items, cap, a, st, e0, e1); break;
  }
  WM_LAUNCH_CHECK("cross_attn_group_kernel");
  if (splits > 1 && !fz.cnt) {
    if (ev1)
      hipExtLaunchKernelGGL(cross_combine_kernel, dim3(rows * H), dim3(HD), 0, st, nullptr, ev1, 0, part_m, part_l,
                            part_o, row_hyp, done, out, ldo, H, splits);
    else
      hipLaunchKernelGGL(cross_combine_kernel, dim3(rows * H), dim3(HD), 0, st, part_m, part_l, part_o, row_hyp, done,
                         out, ldo, H, splits);
    WM_LAUNCH_CHECK("cross_combine_kernel");
  }
}
