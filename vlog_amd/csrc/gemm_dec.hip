// Decoder-row GEMM for gfx950 (M <= 256 rows: one row per live hypothesis; C = A . W^T, W [N][K] bf16).
//
// The weight stream is the cost (1.6 GB per decode step for large-v3, ~46 MB per layer); the activations
// A [M][K] (<= 1.3 MB) sit in L2.  One 256-thread block = 64 output columns (4 waves x 16) x all rows x a
// K range of KR (split-K over blocks).  The block issues EVERY load of its K range up front — its W
// fragments straight into registers (16 B per lane, v_mfma B layout) and its A rows into LDS by LDS-DMA
// (128-B panel rows, XOR swizzle on the source address) — then waits once and runs KR/32 x MF MFMAs per
// wave.  One round trip per block instead of one per K chunk: the per-block latency, not bandwidth, is
// what a 150-row decoder GEMM pays (cdna_hip_programming.md §5 "Projection GEMM at M = 256").
// Split-K partial slabs are combined by the existing deterministic reduce kernels (gemm.hip), so a row's
// summation order is a function of (N, K, KR) only.
#include "gemm.h"
#include "gemm_epi.h"
#include <cstring>
#include <stdexcept>
#include <string>

__device__ __forceinline__ int dswz(int row, int ch) { return row * 64 + ((ch ^ ((row >> 1) & 7)) << 3); }

// ABL (microbenchmark ablations only; the product uses 0): bit 0 skips the A DMA, bit 1 the MFMAs, bit 2 the
// output stores — each skipped part's inputs are kept live so nothing else is eliminated.
template <int MF, int KR, int KIND, int ABL = 0>
__global__ __launch_bounds__(256) void dec_gemm_kernel(GemmA a, const bf16* __restrict__ w, long long ldw, int M, int N,
                                                       int K, GemmEpi epi, int tiles_n, int splitk,
                                                       float* __restrict__ part) {
  constexpr int ROWS = MF * 16, PANEL = ROWS * 64, NP = KR / 64, NF = KR / 32;
  __shared__ __attribute__((aligned(16))) bf16 sA[NP * PANEL];
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  const int wgid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  const int split = wgid % splitk, tile = wgid / splitk;
  const int n0 = tile * 64;
  const int kb = split * KR, klen = min(KR, K - kb);
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int ncol = n0 + wid * 16 + (lane & 15);
  const bf16* wrow = w + (long long)min(ncol, N - 1) * ldw + kb + 8 * (lane >> 4);

  // W fragments: all of this block's K range, issued first (the HBM stream)
  bf16x8 fb[NF];
#pragma unroll
  for (int kk = 0; kk < NF; ++kk) fb[kk] = *(const bf16x8*)(wrow + min(32 * kk, klen - 32));
  // A rows [0, ROWS) x [kb, kb + klen) -> LDS panels of 64 k (8 rows x 128 B per wave-instruction)
  const int ngrp = (ABL & 1) ? 0 : (klen / 64) * (ROWS / 8);
  for (int g = wid; g < ngrp; g += 4) {
    const int panel = g / (ROWS / 8), rg = g - panel * (ROWS / 8);
    const int row = rg * 8 + (lane >> 3), ch = (lane & 7) ^ ((row >> 1) & 7);
    const int gr = min(row, M - 1);
    const long long off = a.rpb ? (long long)(gr / a.rpb) * a.bstride + (long long)(gr % a.rpb) * a.ld : (long long)gr * a.ld;
    __builtin_amdgcn_global_load_lds((const void*)(a.ptr + off + kb + panel * 64 + ch * 8),
                                     (__attribute__((address_space(3))) void*)(sA + panel * PANEL + rg * 8 * 64), 16, 0, 0);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  f32x4 acc[MF];
#pragma unroll
  for (int i = 0; i < MF; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int kk = 0; kk < NF; ++kk) {
    if (32 * kk < klen) {
      const int ch = (kk & 1) * 4 + (lane >> 4);
      const bf16* pa = sA + (kk >> 1) * PANEL;
      bf16x8 fa[MF];
#pragma unroll
      for (int i = 0; i < MF; ++i) fa[i] = *(const bf16x8*)(pa + dswz(i * 16 + (lane & 15), ch));
      if (ABL & 2) {
#pragma unroll
        for (int i = 0; i < MF; ++i) asm volatile("" :: "v"(fa[i]), "v"(fb[kk]));
      } else {
#pragma unroll
        for (int i = 0; i < MF; ++i) acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[kk], fa[i], acc[i], 0, 0, 0);
      }
    }
  }
  if (ABL & 4) {
#pragma unroll
    for (int i = 0; i < MF; ++i) asm volatile("" :: "v"(acc[i]));
    return;
  }

  // operands swapped (W fragment as the MFMA A operand): acc[i] holds C^T, lane l has row m = 16 i + (l & 15)
  // and the 4 consecutive columns n = col0 + e
  const bool to_slab = splitk > 1 || KIND == EPI_RESID_LN;
  const int col0 = n0 + wid * 16 + 4 * (lane >> 4);
  if (col0 >= N) return;
#pragma unroll
  for (int i = 0; i < MF; ++i) {
    const int row = i * 16 + (lane & 15);
    if (row >= M) continue;
    if (to_slab)
      *(f32x4*)(part + ((long long)split * M + row) * N + col0) = acc[i];
    else
      apply_epi4<KIND>(epi, row, col0, acc[i]);
  }
}

// Plan: split count for a K range of KR (multiple of 64); returns false if the shape is not supported.
bool dec_gemm_plan(int M, int N, int K, int KR, size_t ws_bytes, int* splitk) {
  if (M > 256 || N % 64 != 0 || K % 64 != 0 || KR % 64 != 0) return false;
  const int s = (K + KR - 1) / KR;
  if ((K - (s - 1) * KR) % 64 != 0) return false;
  *splitk = s;
  return true;
}

template <int MF, int KR, int KIND>
static void run_dec(const GemmA& a, const bf16* w, long long ldw, int M, int N, int K, const GemmEpi& epi, float* ws,
                    int splitk, hipStream_t st) {
  const int tiles_n = N / 64;
  hipLaunchKernelGGL((dec_gemm_kernel<MF, KR, KIND>), dim3(tiles_n * splitk), dim3(256), 0, st, a, w, ldw, M, N, K, epi,
                     tiles_n, splitk, ws);
  WM_LAUNCH_CHECK("dec_gemm_kernel");
}

// launch_splitk_combine (gemm.hip): the deterministic slab reduce + epilogue (RESID_LN: fused residual+LayerNorm)
void launch_splitk_combine(const float* part, int splitk, int M, int N, const GemmEpi& epi, hipStream_t st);

template <int MF, int KIND>
static void dispatch_kr(const GemmA& a, const bf16* w, long long ldw, int M, int N, int K, const GemmEpi& epi,
                        float* ws, int KR, int splitk, hipStream_t st) {
  switch (KR) {
    case 128: run_dec<MF, 128, KIND>(a, w, ldw, M, N, K, epi, ws, splitk, st); break;
    case 192: run_dec<MF, 192, KIND>(a, w, ldw, M, N, K, epi, ws, splitk, st); break;
    case 256: run_dec<MF, 256, KIND>(a, w, ldw, M, N, K, epi, ws, splitk, st); break;
    case 320: run_dec<MF, 320, KIND>(a, w, ldw, M, N, K, epi, ws, splitk, st); break;
    case 448: run_dec<MF, 448, KIND>(a, w, ldw, M, N, K, epi, ws, splitk, st); break;
    default: throw std::runtime_error("dec_gemm: unsupported KR " + std::to_string(KR));
  }
}

template <int KIND>
static void dispatch_mf(const GemmA& a, const bf16* w, long long ldw, int M, int N, int K, const GemmEpi& epi,
                        float* ws, int KR, int splitk, hipStream_t st) {
  if (M <= 32) dispatch_kr<2, KIND>(a, w, ldw, M, N, K, epi, ws, KR, splitk, st);
  else if (M <= 64) dispatch_kr<4, KIND>(a, w, ldw, M, N, K, epi, ws, KR, splitk, st);
  else if (M <= 96) dispatch_kr<6, KIND>(a, w, ldw, M, N, K, epi, ws, KR, splitk, st);
  else if (M <= 128) dispatch_kr<8, KIND>(a, w, ldw, M, N, K, epi, ws, KR, splitk, st);
  else if (M <= 160) dispatch_kr<10, KIND>(a, w, ldw, M, N, K, epi, ws, KR, splitk, st);
  else throw std::runtime_error("dec_gemm: M > 160 not instantiated");
}

// Returns false when the shape / KR is not supported (caller falls back to the skinny path).
bool launch_dec_gemm(const GemmA& a, const bf16* w, long long ldw, int M, int N, int K, const GemmEpi& epi, float* ws,
                     size_t ws_bytes, int KR, hipStream_t st) {
  int splitk = 1;
  if (M > 160 || !dec_gemm_plan(M, N, K, KR, ws_bytes, &splitk)) return false;
  const int mf = M <= 32 ? 2 : M <= 64 ? 4 : M <= 96 ? 6 : M <= 128 ? 8 : 10;
  if ((size_t)mf * 16 * KR * 2 > 150 * 1024) return false;      // A panels must fit in LDS
  const bool slab = splitk > 1 || epi.kind == EPI_RESID_LN;
  if (slab && (!ws || (size_t)splitk * M * N * 4 > ws_bytes)) return false;
  switch (epi.kind) {
    case EPI_BF16: dispatch_mf<EPI_BF16>(a, w, ldw, M, N, K, epi, ws, KR, splitk, st); break;
    case EPI_RESID_F32: dispatch_mf<EPI_RESID_F32>(a, w, ldw, M, N, K, epi, ws, KR, splitk, st); break;
    case EPI_F32: dispatch_mf<EPI_F32>(a, w, ldw, M, N, K, epi, ws, KR, splitk, st); break;
    case EPI_DEC_QKV: dispatch_mf<EPI_DEC_QKV>(a, w, ldw, M, N, K, epi, ws, KR, splitk, st); break;
    case EPI_RESID_LN: dispatch_mf<EPI_RESID_LN>(a, w, ldw, M, N, K, epi, ws, KR, splitk, st); break;
    default: return false;
  }
  if (slab) launch_splitk_combine(ws, splitk, M, N, epi, st);
  return true;
}

// microbenchmark entry (tools/dec_gemm_bench): the GEMM body alone (no combine), with ablation bits
void launch_dec_gemm_body(const GemmA& a, const bf16* w, long long ldw, int M, int N, int K, float* ws, int KR, int abl,
                          hipStream_t st) {
  GemmEpi epi;
  memset(&epi, 0, sizeof(epi));
  epi.kind = EPI_BF16;
  const int splitk = (K + KR - 1) / KR;
  const dim3 grid(N / 64 * splitk);
#define DG_CASE(KRV, AB)                                                                                        \
  if (KR == KRV && abl == AB) {                                                                                 \
    hipLaunchKernelGGL((dec_gemm_kernel<10, KRV, EPI_BF16, AB>), grid, dim3(256), 0, st, a, w, ldw, M, N, K, epi, \
                       N / 64, splitk, ws);                                                                     \
    return;                                                                                                     \
  }
#define DG_KR(KRV) DG_CASE(KRV, 0) DG_CASE(KRV, 1) DG_CASE(KRV, 2) DG_CASE(KRV, 4) DG_CASE(KRV, 7)
  DG_KR(128) DG_KR(256) DG_KR(448)
#undef DG_KR
#undef DG_CASE
  throw std::runtime_error("launch_dec_gemm_body: unsupported KR/abl");
}
