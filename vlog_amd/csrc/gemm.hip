// bf16 MFMA GEMM for gfx950:  C[M,N] = A[M,K] . W[N,K]^T, both operands K-contiguous (PyTorch / HF
// Linear layout), f32 accumulation, fused epilogues (bias, GELU, residual add, positional add, KV-cache
// scatter).  Used for the encoder projections/MLP, the conv stem (implicit im2col through the strided A
// descriptor), the cross-KV projection, the decoder projections and the tied-embedding logits.
//
// Structure (cdna_hip_programming.md §5 "standard MFMA GEMM main loop"): BK = 64 tiles staged
// global -> registers -> LDS (double-buffered LDS, one barrier per K-tile, next tile's global loads issued
// before the current tile's MFMAs), v_mfma_f32_16x16x32_bf16, 64-wide waves each owning a
// (BM/WM) x (BN/WN) sub-tile.  LDS rows are 128 B; 16-B chunks are XOR-swizzled with (row>>1)&7 so the
// ds_read_b128 lane groups hit 16 distinct bank slots.  Grid is XCD-remapped (T1) so consecutive N-tiles
// of one M-panel share an XCD's L2.
#include "gemm.h"
#include "gemm_epi.h"
#include <cstdlib>
#include <algorithm>
#include <stdexcept>
#include <string>

#define BK 64

void launch_layernorm(const float*, long long, const int*, int, int, const float*, const float*, bf16*, long long, hipStream_t);

__device__ __forceinline__ int swz(int row, int ch) { return row * BK + ((ch ^ ((row >> 1) & 7)) << 3); }

template <int BM, int BN, int WM, int WN, int KIND>
__global__ __launch_bounds__(WM * WN * 64) void gemm_kernel(GemmA a, const bf16* __restrict__ w, long long ldw,
                                                            int M, int N, int K, GemmEpi epi, int tiles_n,
                                                            int splitk, int kt_per_split, float* __restrict__ part) {
  constexpr int NT = WM * WN * 64;
  constexpr int TM = BM / WM, TN = BN / WN;        // per-wave tile
  constexpr int FM = TM / 16, FN = TN / 16;        // 16x16 fragments per wave
  constexpr int CA = (BM * 8 + NT - 1) / NT, CB = (BN * 8 + NT - 1) / NT;  // 16-B chunks per thread per operand
  __shared__ __attribute__((aligned(16))) bf16 sA[2][BM * BK];
  __shared__ __attribute__((aligned(16))) bf16 sB[2][BN * BK];

  // XCD-aware remap of the linear block id (bijective for any grid size); consecutive ids share an XCD.
  const int nwg = gridDim.x;
  const int bid = blockIdx.x;
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  const int wgid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  const int split = wgid % splitk, tile = wgid / splitk;
  const int tm = tile / tiles_n, tn = tile - tm * tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  const int nk_total = K / BK;
  const int kt0 = split * kt_per_split;
  const int nk = min(nk_total - kt0, kt_per_split);
  const int kbase = kt0 * BK;

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid - wm * WN;

  const bf16* pa[CA];
  const bf16* pb[CB];
  bool va[CA], vb[CB], sa[CA], sb[CB];
#pragma unroll
  for (int i = 0; i < CA; ++i) {
    const int c = tid + i * NT, row = c >> 3, ch = c & 7;
    sa[i] = c < BM * 8;
    const int gr = m0 + row;
    va[i] = sa[i] && gr < M;
    const int rr = va[i] ? gr : 0;
    long long off = a.rpb ? (long long)(rr / a.rpb) * a.bstride + (long long)(rr % a.rpb) * a.ld : (long long)rr * a.ld;
    pa[i] = a.ptr + off + ch * 8 + kbase;
  }
#pragma unroll
  for (int i = 0; i < CB; ++i) {
    const int c = tid + i * NT, row = c >> 3, ch = c & 7;
    sb[i] = c < BN * 8;
    const int gn = n0 + row;
    vb[i] = sb[i] && gn < N;
    pb[i] = w + (long long)(vb[i] ? gn : 0) * ldw + ch * 8 + kbase;
  }

  i32x4 ra[CA], rb[CB];
#define GLOAD(k0)                                                                                   \
  {                                                                                                 \
    _Pragma("unroll") for (int i = 0; i < CA; ++i) ra[i] = va[i] ? *(const i32x4*)(pa[i] + (k0)) : i32x4{0, 0, 0, 0}; \
    _Pragma("unroll") for (int i = 0; i < CB; ++i) rb[i] = vb[i] ? *(const i32x4*)(pb[i] + (k0)) : i32x4{0, 0, 0, 0}; \
  }
#define SSTORE(s_)                                                                                  \
  {                                                                                                 \
    _Pragma("unroll") for (int i = 0; i < CA; ++i) {                                                \
      const int c = tid + i * NT;                                                                   \
      if (sa[i]) *(i32x4*)(&sA[s_][swz(c >> 3, c & 7)]) = ra[i];                                    \
    }                                                                                               \
    _Pragma("unroll") for (int i = 0; i < CB; ++i) {                                                \
      const int c = tid + i * NT;                                                                   \
      if (sb[i]) *(i32x4*)(&sB[s_][swz(c >> 3, c & 7)]) = rb[i];                                    \
    }                                                                                               \
  }

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  GLOAD(0);
  SSTORE(0);
  __syncthreads();
  for (int t = 0; t < nk; ++t) {
    const int s = t & 1;
    if (t + 1 < nk) GLOAD((t + 1) * BK);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 fa[FM], fb[FN];
      const int ch = kk * 4 + (lane >> 4);
#pragma unroll
      for (int i = 0; i < FM; ++i) fa[i] = *(const bf16x8*)(&sA[s][swz(wm * TM + i * 16 + (lane & 15), ch)]);
#pragma unroll
      for (int j = 0; j < FN; ++j) fb[j] = *(const bf16x8*)(&sB[s][swz(wn * TN + j * 16 + (lane & 15), ch)]);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
    }
    if (t + 1 < nk) SSTORE(s ^ 1);
    __syncthreads();
  }

  // ---------------------------------------------------------------- epilogue
#pragma unroll
  for (int i = 0; i < FM; ++i) {
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int col = n0 + wn * TN + j * 16 + (lane & 15);
      if (col >= N) continue;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int row = m0 + wm * TM + i * 16 + (lane >> 4) * 4 + e;
        if (row >= M) continue;
        if (splitk > 1)
          part[((long long)split * M + row) * N + col] = acc[i][j][e];
        else
          apply_epi<KIND>(epi, row, col, acc[i][j][e]);
      }
    }
  }
}

// deterministic split-K combine: sum the partial slabs in split order, then the real epilogue
template <int KIND>
__global__ __launch_bounds__(256) void splitk_reduce_kernel(const float* __restrict__ part, int splitk, int M, int N,
                                                            GemmEpi epi) {
  const long long total = (long long)M * N;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long long)gridDim.x * blockDim.x) {
    float v = 0.f;
#pragma unroll 4
    for (int s = 0; s < splitk; ++s) v += part[s * total + i];
    const int row = (int)(i / N), col = (int)(i - (long long)row * N);
    apply_epi<KIND>(epi, row, col, v);
  }
}

// ------------------------------------------------------------------------------------------------------
// Skinny path (decoder rows, M <= 256): the weight stream is the whole cost, so nothing about W touches LDS.
// A block = 4 waves x 16 output columns (64 columns) over a K range [kb, kb + kr); each wave loads its
// B fragments (W rows n, 16 B at k = 32kk + 8(lane>>4)) for a whole KS chunk straight into registers —
// all KS/32 loads issued back to back, so every CU keeps its share of W in flight at once — while the
// block's A rows [0, 16 MF) x chunk are DMA'd into LDS (global_load_lds, 128-B panel rows, XOR swizzle on
// the source address) and shared by the 4 waves.  K is split across blocks until the grid covers the chip;
// partial slabs are combined in split order by the reduce kernels below (deterministic).
template <int MF, int KS, int KIND>
__global__ __launch_bounds__(256) void skinny_kernel(GemmA a, const bf16* __restrict__ w, long long ldw, int M, int N,
                                                     int K, GemmEpi epi, int tiles_n, int splitk, int kr,
                                                     float* __restrict__ part) {
  constexpr int ROWS = MF * 16, PANEL = ROWS * 64, NF = KS / 32;
  __shared__ __attribute__((aligned(16))) bf16 sA[(KS / 64) * PANEL];
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  const int wgid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  const int split = wgid % splitk, tile = wgid / splitk;
  const int n0 = tile * 64;
  const int kb = split * kr, kend = min(K, kb + kr);
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int ncol = n0 + wid * 16 + (lane & 15);
  const bf16* wrow = w + (long long)min(ncol, N - 1) * ldw + 8 * (lane >> 4);

  f32x4 acc[MF];
#pragma unroll
  for (int i = 0; i < MF; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};

  for (int c0 = kb; c0 < kend; c0 += KS) {
    const int clen = min(KS, kend - c0);
    bf16x8 fb[NF];
#pragma unroll
    for (int kk = 0; kk < NF; ++kk) fb[kk] = *(const bf16x8*)(wrow + c0 + min(32 * kk, clen - 32));
    const int ngrp = (clen / 64) * (2 * MF);
    for (int g = wid; g < ngrp; g += 4) {
      const int panel = g / (2 * MF), rg = g - panel * (2 * MF);
      const int row = rg * 8 + (lane >> 3), ch = (lane & 7) ^ ((row >> 1) & 7);
      const int gr = min(row, M - 1);
      const long long off = a.rpb ? (long long)(gr / a.rpb) * a.bstride + (long long)(gr % a.rpb) * a.ld : (long long)gr * a.ld;
      __builtin_amdgcn_global_load_lds((const void*)(a.ptr + off + c0 + panel * 64 + ch * 8),
                                       (__attribute__((address_space(3))) void*)(sA + panel * PANEL + rg * 8 * 64), 16, 0, 0);
    }
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < NF; ++kk) {
      if (32 * kk < clen) {
        const int ch = (kk & 1) * 4 + (lane >> 4);
        const bf16* pa = sA + (kk >> 1) * PANEL;
        bf16x8 fa[MF];
#pragma unroll
        for (int i = 0; i < MF; ++i) fa[i] = *(const bf16x8*)(pa + swz(i * 16 + (lane & 15), ch));
#pragma unroll
        for (int i = 0; i < MF; ++i) acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[kk], fa[i], acc[i], 0, 0, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, MF, 0);   // all MF ds_reads of this k-step first,
        __builtin_amdgcn_sched_group_barrier(0x008, MF, 0);   // then the MF MFMAs
      }
    }
    __syncthreads();
  }

  // operands are swapped (W fragment as the MFMA A operand): acc[i] holds C^T, lane l has row
  // m = 16 i + (l & 15) and the 4 consecutive columns n = col0 + e -> one 16-B slab store per fragment
  const bool to_slab = splitk > 1 || KIND == EPI_RESID_LN;
  const int col0 = n0 + wid * 16 + 4 * (lane >> 4);
  const bool vec = (N % 4 == 0) && (to_slab || (epi.ldc % 4 == 0 && (epi.rpb == 0 || epi.bstride % 4 == 0)));
#pragma unroll
  for (int i = 0; i < MF; ++i) {
    const int row = i * 16 + (lane & 15);
    if (row >= M) continue;
    if (vec && col0 < N) {
      if (to_slab)
        *(f32x4*)(part + ((long long)split * M + row) * N + col0) = acc[i];
      else
        apply_epi4<KIND>(epi, row, col0, acc[i]);
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        if (col0 + e >= N) continue;
        if (to_slab)
          part[((long long)split * M + row) * N + col0 + e] = acc[i][e];
        else
          apply_epi<KIND>(epi, row, col0 + e, acc[i][e]);
      }
    }
  }
}

// Split-K combine fused with the residual add and the LayerNorm that consumes it: one block per row, one
// thread per float2 pair (N/2 threads, up to 16 waves), the slab loop unrolled 8-deep so a thread has 8
// loads in flight (150 decoder rows cannot fill the chip, so latency, not bandwidth, is the cost).
// x[r] += sum_s part[s][r] + bias;  ln_out[r] = LN(x[r]) (two-pass mean / variance, eps 1e-5).  Summation
// order per element = splitk_reduce_kernel's.
// FOLD (a folded-LayerNorm consumer follows, GemmEpi.xg_out): instead of the LayerNorm, the row's sums (sum x,
// sum x^2) go to stat_out[r] (one tile per row) and xg_out[r] = bf16(x[r] * xg_g).
template <bool FOLD>
__global__ __launch_bounds__(1024) void resid_ln_reduce_kernel(const float* __restrict__ part, int splitk, int M, int N,
                                                               GemmEpi epi) {
  __shared__ float red[2][16];
  const int r = blockIdx.x, c = threadIdx.x, lane = c & 63, wid = c >> 6, nw = blockDim.x >> 6;
  const int np = N >> 1;
  const bool act = c < np;
  const long long slab2 = ((long long)M * N) >> 1;
  const float2* pr = (const float2*)(part + (long long)r * N) + (act ? c : 0);
  // every operand this thread needs (residual, bias, LayerNorm affine) is requested with the slabs, so the
  // kernel pays one memory round trip instead of one before the sums and another after the statistics
  const int cc = act ? c : 0;
  float2* xr = (float2*)((float*)epi.out + (long long)r * epi.ldc);
  const float2 x0 = xr[cc];
  const float2 bias2 = epi.bias ? ((const float2*)epi.bias)[cc] : make_float2(0.f, 0.f);
  const float2 gg = ((const float2*)(FOLD ? epi.xg_g : epi.ln_g))[cc];
  const float2 lb = FOLD ? make_float2(0.f, 0.f) : ((const float2*)epi.ln_b)[cc];
  float2 acc = make_float2(0.f, 0.f);
#pragma unroll 8
  for (int sp = 0; sp < splitk; ++sp) {
    const float2 v = pr[sp * slab2];
    acc.x += v.x;
    acc.y += v.y;
  }
  float s = 0.f;
  if (act) {
    if (epi.bias) {
      acc.x += bias2.x;
      acc.y += bias2.y;
    }
    float2 xv = x0;
    xv.x += acc.x;
    xv.y += acc.y;
    xr[c] = xv;
    acc = xv;
    s = xv.x + xv.y;
  }
  if constexpr (FOLD) {
    float q2 = act ? acc.x * acc.x + acc.y * acc.y : 0.f;
    s = wave_sum(s);
    q2 = wave_sum(q2);
    if (lane == 0) {
      red[0][wid] = s;
      red[1][wid] = q2;
    }
    if (act) {
      bf16x2 o;
      o[0] = f2bf(acc.x * gg.x);
      o[1] = f2bf(acc.y * gg.y);
      ((bf16x2*)(epi.xg_out + (long long)r * epi.xg_ld))[c] = o;
    }
    __syncthreads();
    if (c == 0) {
      float t1 = 0.f, t2 = 0.f;
      for (int i = 0; i < nw; ++i) {
        t1 += red[0][i];
        t2 += red[1][i];
      }
      *(float2*)(epi.stat_out + 2LL * r) = make_float2(t1, t2);
    }
    return;
  }
  s = wave_sum(s);
  if (lane == 0) red[0][wid] = s;
  __syncthreads();
  float tot = 0.f;
  for (int i = 0; i < nw; ++i) tot += red[0][i];
  const float mean = tot / (float)N;
  float q = 0.f;
  if (act) {
    const float a = acc.x - mean, b = acc.y - mean;
    q = a * a + b * b;
  }
  q = wave_sum(q);
  if (lane == 0) red[1][wid] = q;
  __syncthreads();
  float qt = 0.f;
  for (int i = 0; i < nw; ++i) qt += red[1][i];
  const float rstd = rsqrtf(qt / (float)N + 1e-5f);
  if (act) {
    bf16x2 o;
    o[0] = f2bf((acc.x - mean) * rstd * gg.x + lb.x);
    o[1] = f2bf((acc.y - mean) * rstd * gg.y + lb.y);
    ((bf16x2*)(epi.ln_out + (long long)r * epi.ln_ld))[c] = o;
  }
}

static void launch_resid_ln_reduce(const float* part, int splitk, int M, int N, const GemmEpi& epi, hipStream_t st) {
  if (N % 2 != 0 || N > 2048) throw std::runtime_error("resid_ln_reduce: unsupported width " + std::to_string(N));
  const int threads = ((N / 2 + 63) / 64) * 64;
  if (epi.kind == EPI_RESID_F32) hipLaunchKernelGGL((resid_ln_reduce_kernel<true>), dim3(M), dim3(threads), 0, st, part, splitk, M, N, epi);
  else hipLaunchKernelGGL((resid_ln_reduce_kernel<false>), dim3(M), dim3(threads), 0, st, part, splitk, M, N, epi);
  WM_LAUNCH_CHECK("resid_ln_reduce_kernel");
}

// Deterministic combine of `splitk` partial slabs [splitk][M][N] + the epilogue (used by gemm_dec.hip).
void launch_splitk_combine(const float* part, int splitk, int M, int N, const GemmEpi& epi, hipStream_t st) {
  if (epi.kind == EPI_RESID_LN || (epi.kind == EPI_RESID_F32 && epi.xg_out)) {
    launch_resid_ln_reduce(part, splitk, M, N, epi, st);
    return;
  }
  const long long total = (long long)M * N;
  const int blocks = (int)std::min<long long>((total + 255) / 256, 2048);
  switch (epi.kind) {
    case EPI_BF16: hipLaunchKernelGGL((splitk_reduce_kernel<EPI_BF16>), dim3(blocks), dim3(256), 0, st, part, splitk, M, N, epi); break;
    case EPI_RESID_F32: hipLaunchKernelGGL((splitk_reduce_kernel<EPI_RESID_F32>), dim3(blocks), dim3(256), 0, st, part, splitk, M, N, epi); break;
    case EPI_F32: hipLaunchKernelGGL((splitk_reduce_kernel<EPI_F32>), dim3(blocks), dim3(256), 0, st, part, splitk, M, N, epi); break;
    case EPI_DEC_QKV: hipLaunchKernelGGL((splitk_reduce_kernel<EPI_DEC_QKV>), dim3(blocks), dim3(256), 0, st, part, splitk, M, N, epi); break;
    default: throw std::runtime_error("splitk_combine: bad epilogue kind");
  }
  WM_LAUNCH_CHECK("splitk_reduce_kernel");
}

// Skinny-path geometry: split K so the grid reaches ~256 blocks, each split at least 128 deep (partial
// slabs cost 8 B per output per split); returns false when the slabs do not fit the scratch.
static bool skinny_plan(int M, int N, int K, size_t ws_bytes, int* splitk, int* kr) {
  const int tiles_n = (N + 63) / 64;
  int s = std::max(1, (256 + tiles_n / 2) / tiles_n);
  s = std::min(s, std::max(1, K / 128));
  int k = ((K + s - 1) / s + 63) / 64 * 64;
  s = (K + k - 1) / k;
  while (s > 1 && (size_t)s * M * N * 4 > ws_bytes) {
    --s;
    k = ((K + s - 1) / s + 63) / 64 * 64;
    s = (K + k - 1) / k;
  }
  *splitk = s;
  *kr = k;
  return (size_t)s * M * N * 4 <= ws_bytes;
}

template <int MF, int KS, int KIND>
static void run_skinny(const GemmA& a, const bf16* w, long long ldw, int M, int N, int K, const GemmEpi& epi, float* ws,
                       int splitk, int kr, hipStream_t st) {
  const int tiles_n = (N + 63) / 64;
  hipLaunchKernelGGL((skinny_kernel<MF, KS, KIND>), dim3(tiles_n * splitk), dim3(256), 0, st, a, w, ldw, M, N, K, epi,
                     tiles_n, splitk, kr, ws);
  WM_LAUNCH_CHECK("skinny_kernel");
  if (KIND == EPI_RESID_LN) {
    launch_resid_ln_reduce(ws, splitk, M, N, epi, st);
  } else if (splitk > 1 && !epi.defer_combine) {
    const long long total = (long long)M * N;
    int blocks = (int)std::min<long long>((total + 255) / 256, 2048);
    hipLaunchKernelGGL((splitk_reduce_kernel<KIND>), dim3(blocks), dim3(256), 0, st, ws, splitk, M, N, epi);
    WM_LAUNCH_CHECK("splitk_reduce_kernel");
  }
}

template <int KIND>
static void dispatch_skinny(const GemmA& a, const bf16* w, long long ldw, int M, int N, int K, const GemmEpi& epi,
                            float* ws, int splitk, int kr, hipStream_t st) {
  if (M <= 16) run_skinny<1, 512, KIND>(a, w, ldw, M, N, K, epi, ws, splitk, kr, st);
  else if (M <= 32) run_skinny<2, 512, KIND>(a, w, ldw, M, N, K, epi, ws, splitk, kr, st);
  else if (M <= 64) run_skinny<4, 512, KIND>(a, w, ldw, M, N, K, epi, ws, splitk, kr, st);
  else if (M <= 128) run_skinny<8, 256, KIND>(a, w, ldw, M, N, K, epi, ws, splitk, kr, st);
  else if (M <= 160) run_skinny<10, 256, KIND>(a, w, ldw, M, N, K, epi, ws, splitk, kr, st);
  else if (M <= 256) run_skinny<16, 128, KIND>(a, w, ldw, M, N, K, epi, ws, splitk, kr, st);
  else if (M <= 320) run_skinny<20, 128, KIND>(a, w, ldw, M, N, K, epi, ws, splitk, kr, st);
  else run_skinny<32, 64, KIND>(a, w, ldw, M, N, K, epi, ws, splitk, kr, st);
}

int skinny_splits(int M, int N, int K, size_t ws_bytes) {
  static const bool skinny_enabled = [] {
    const char* e = std::getenv("VLOG_AMD_GEMM_SKINNY");
    return !(e && e[0] == '0');
  }();
  int splitk, kr;
  if (!skinny_enabled || M <= 0 || M > 512 || K % BK != 0 || !skinny_plan(M, N, K, ws_bytes, &splitk, &kr)) return 0;
  return splitk;
}

static bool try_skinny(const GemmA& a, const bf16* w, long long ldw, int M, int N, int K, const GemmEpi& epi, float* ws,
                       size_t ws_bytes, hipStream_t st) {
  if (M > 512 || !ws) return false;
  int splitk, kr;
  if (!skinny_plan(M, N, K, ws_bytes, &splitk, &kr)) return false;
  switch (epi.kind) {
    case EPI_BF16: dispatch_skinny<EPI_BF16>(a, w, ldw, M, N, K, epi, ws, splitk, kr, st); break;
    case EPI_RESID_F32: dispatch_skinny<EPI_RESID_F32>(a, w, ldw, M, N, K, epi, ws, splitk, kr, st); break;
    case EPI_F32: dispatch_skinny<EPI_F32>(a, w, ldw, M, N, K, epi, ws, splitk, kr, st); break;
    case EPI_DEC_QKV: dispatch_skinny<EPI_DEC_QKV>(a, w, ldw, M, N, K, epi, ws, splitk, kr, st); break;
    case EPI_RESID_LN: dispatch_skinny<EPI_RESID_LN>(a, w, ldw, M, N, K, epi, ws, splitk, kr, st); break;
    default: return false;
  }
  return true;
}

template <int BM, int BN, int WM, int WN, int KIND>
static void run(const GemmA& a, const bf16* w, long long ldw, int M, int N, int K, const GemmEpi& epi, float* ws,
                size_t ws_bytes, hipStream_t st) {
  const int tiles_m = (M + BM - 1) / BM, tiles_n = (N + BN - 1) / BN;
  const int tiles = tiles_m * tiles_n;
  const int nk = K / BK;
  // split K until the grid covers the chip ~4x (weight-streaming skinny GEMMs), deterministic combine
  int splitk = 1;
  if (ws && tiles < 1024) {
    splitk = std::min(std::max(1, 1024 / tiles), std::max(1, nk / 4));
    while (splitk > 1 && (size_t)splitk * M * N * 4 > ws_bytes) --splitk;
  }
  const int kps = (nk + splitk - 1) / splitk;
  splitk = (nk + kps - 1) / kps;
  dim3 grid(tiles * splitk);
  hipLaunchKernelGGL((gemm_kernel<BM, BN, WM, WN, KIND>), grid, dim3(WM * WN * 64), 0, st, a, w, ldw, M, N, K, epi,
                     tiles_n, splitk, kps, ws);
  WM_LAUNCH_CHECK("gemm_kernel");
  if (splitk > 1) {
    const long long total = (long long)M * N;
    int blocks = (int)std::min<long long>((total + 255) / 256, 2048);
    hipLaunchKernelGGL((splitk_reduce_kernel<KIND>), dim3(blocks), dim3(256), 0, st, ws, splitk, M, N, epi);
    WM_LAUNCH_CHECK("splitk_reduce_kernel");
  }
}

template <int KIND>
static void dispatch(const GemmA& a, const bf16* w, long long ldw, int M, int N, int K, const GemmEpi& epi, float* ws,
                     size_t wsb, hipStream_t st) {
  if (M <= 16)
    run<16, 64, 1, 4, KIND>(a, w, ldw, M, N, K, epi, ws, wsb, st);
  else if (M <= 32)
    run<32, 64, 1, 4, KIND>(a, w, ldw, M, N, K, epi, ws, wsb, st);
  else if (M <= 64)
    run<64, 64, 1, 4, KIND>(a, w, ldw, M, N, K, epi, ws, wsb, st);
  else if (M <= 128)
    run<128, 64, 2, 2, KIND>(a, w, ldw, M, N, K, epi, ws, wsb, st);
  else if (M <= 256)
    run<256, 64, 4, 1, KIND>(a, w, ldw, M, N, K, epi, ws, wsb, st);
  else
    run<128, 128, 2, 2, KIND>(a, w, ldw, M, N, K, epi, ws, wsb, st);
}

void launch_gemm(const GemmA& a, const bf16* w, long long ldw, int M, int N, int K, const GemmEpi& epi, float* ws,
                 size_t ws_bytes, hipStream_t st) {
  if (M <= 0 || N <= 0) return;
  if (K % BK != 0) throw std::runtime_error("launch_gemm: K must be a multiple of 64 (got " + std::to_string(K) + ")");
  static const bool big_enabled = [] {
    const char* e = std::getenv("VLOG_AMD_GEMM_BIG");
    return !(e && e[0] == '0');
  }();
  static const bool p8_enabled = [] {
    const char* e = std::getenv("VLOG_AMD_GEMM_8P");
    return !(e && e[0] == '0');
  }();
  static const bool skinny_enabled = [] {
    const char* e = std::getenv("VLOG_AMD_GEMM_SKINNY");
    return !(e && e[0] == '0');
  }();
  if (skinny_enabled && try_skinny(a, w, ldw, M, N, K, epi, ws, ws_bytes, st)) return;
  if (epi.kind == EPI_RESID_LN) {        // unfused form: residual epilogue, then the LayerNorm
    GemmEpi r = epi;
    r.kind = EPI_RESID_F32;
    launch_gemm(a, w, ldw, M, N, K, r, ws, ws_bytes, st);
    launch_layernorm((const float*)epi.out, epi.ldc, nullptr, M, N, epi.ln_g, epi.ln_b, epi.ln_out, epi.ln_ld, st);
    return;
  }
  const bool vec4 = epi.ldc % 4 == 0 && (epi.rpb == 0 || epi.bstride % 4 == 0);   // 4-column vector epilogue
  // large-tile kernels need enough 256 x 256 tiles to occupy the CUs (one window's encoder is 6 row tiles:
  // 30-120 tiles for 256 CUs); below VLOG_AMD_GEMM_MIN_TILES of them the 128 x 128 kernel runs instead
  static const int min_tiles = [] {
    const char* e = std::getenv("VLOG_AMD_GEMM_MIN_TILES");
    return e ? std::atoi(e) : 0;
  }();
  const long long tiles256 = (long long)((M + 255) / 256) * ((N + 255) / 256);
  if (tiles256 < min_tiles) {
    switch (epi.kind) {
      case EPI_BF16: run<128, 128, 2, 2, EPI_BF16>(a, w, ldw, M, N, K, epi, nullptr, 0, st); return;
      case EPI_RESID_F32: run<128, 128, 2, 2, EPI_RESID_F32>(a, w, ldw, M, N, K, epi, nullptr, 0, st); return;
      case EPI_GELU_POS_F32: run<128, 128, 2, 2, EPI_GELU_POS_F32>(a, w, ldw, M, N, K, epi, nullptr, 0, st); return;
      default: break;
    }
  }
  if (p8_enabled && vec4 && gemm_8p_applicable(M, N, K)) {
    launch_gemm_8p(a, w, ldw, M, N, K, epi, st);
    return;
  }
  if (big_enabled && vec4 && gemm_big_applicable(M, N, K)) {
    launch_gemm_big(a, w, ldw, M, N, K, epi, st);
    return;
  }
  switch (epi.kind) {
    case EPI_BF16: dispatch<EPI_BF16>(a, w, ldw, M, N, K, epi, ws, ws_bytes, st); break;
    case EPI_RESID_F32: dispatch<EPI_RESID_F32>(a, w, ldw, M, N, K, epi, ws, ws_bytes, st); break;
    case EPI_GELU_POS_F32: dispatch<EPI_GELU_POS_F32>(a, w, ldw, M, N, K, epi, ws, ws_bytes, st); break;
    case EPI_F32: dispatch<EPI_F32>(a, w, ldw, M, N, K, epi, ws, ws_bytes, st); break;
    case EPI_DEC_QKV: dispatch<EPI_DEC_QKV>(a, w, ldw, M, N, K, epi, ws, ws_bytes, st); break;
    case EPI_CROSS_KV: dispatch<EPI_CROSS_KV>(a, w, ldw, M, N, K, epi, ws, ws_bytes, st); break;
    default: throw std::runtime_error("launch_gemm: bad epilogue kind");
  }
}
