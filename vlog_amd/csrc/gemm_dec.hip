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
#include <algorithm>
#include <cstdlib>
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
  // folded LayerNorm: a consumer needs the stat rows of its pass; a producer writes whole 16-column tiles
  if (a.fold_stat && (!(a.fold_tiles == 1 || (a.fold_tiles % 2 == 0 && a.fold_tiles <= 80)) || a.fold_rows < M || epi.bias ||
                      !epi.fold_s || !epi.fold_c || slab)) return false;
  if (epi.xg_out && (epi.kind != EPI_RESID_F32 || N % 16 != 0 || !epi.stat_out || !epi.bias || !epi.xg_g)) return false;
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

// ------------------------------------------------------------------------------------------------------
// Ring-pipelined decoder GEMM: one block = 32 output columns x all rows (MF fragments of 16, MF even) x a
// K range of kr (the whole K when the activations are <= 1280 wide: no split-K, no partial slabs, no
// combine launch).  A-row panels and W-row panels of 64 k (128-B rows, XOR-swizzled chunks on the DMA
// source) stream through an R-slot LDS ring by LDS-DMA, R-1 panels in flight; every wave waits for its own
// DMAs of panel p with a counted vmcnt, and the raw barrier after it both publishes panel p to all waves and
// frees the slot of panel p-1 (whose readers' ds_reads retired before their MFMAs) for panel p+R-1.
// Waves: 2 (16 columns each) x 2 (row halves of MF/2 fragments).
__device__ __forceinline__ void vm_wait(int n) {
  switch (n) {
#define VMW(k) case k: asm volatile("s_waitcnt vmcnt(" #k ")" ::: "memory"); break;
    VMW(0) VMW(1) VMW(2) VMW(3) VMW(4) VMW(5) VMW(6) VMW(7) VMW(8) VMW(9) VMW(10) VMW(11) VMW(12) VMW(13)
    VMW(14) VMW(15) VMW(16) VMW(17) VMW(18) VMW(19) VMW(20) VMW(21) VMW(22) VMW(23) VMW(24) VMW(25) VMW(26)
    VMW(27) VMW(28) VMW(29) VMW(30) VMW(31) VMW(32) VMW(33) VMW(34) VMW(35) VMW(36)
#undef VMW
    default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
  }
}

// LNF: the folded-LayerNorm consumer (GemmA.fold_*): its row-sum loads are issued before the ring's first panels and
// reduced after the last one (the epilogue is their only reader), in a separate instantiation so the plain kernel's
// pipeline is untouched (a runtime-gated prologue made the compiler drain the DMA queue: 1.6x slower at 750 rows).
// NW = 4 or 8 waves: 2 column halves x NW / 2 row slices.  Eight waves halve each wave's LDS-DMA issue and fragment
// reads per sub-panel and put two waves on every SIMD, so one wave's DMA issue and barrier wait overlap the other's
// MFMAs (at 750 rows the 4-wave block was bound by its own per-wave DMA issue, not by the L2).
template <int MF, int KIND, int R, int PK = 1, int NC = 1, bool LNF = false, int NW = 4>
__global__ __launch_bounds__(NW * 64) void dec_ring_kernel(GemmA a, const bf16* __restrict__ w, long long ldw, int M, int N,
                                                           int K, GemmEpi epi, int tiles_n, int splitk, int kr,
                                                           float* __restrict__ part, int rgroups) {
  static_assert(NW == 4 || NW == 8, "4 or 8 waves");
  static_assert(!LNF || NW == 4, "the folded-LayerNorm statistics split assumes 256 threads");
  // a ring slot holds PK consecutive 64-k sub-panels (one barrier per PK x 64 of K); a block covers WR = 32 NC
  // output columns (each wave NC fragments of 16) and ROWS rows (each wave HALF fragments of 16: its row slice)
  constexpr int WRS = NW / 2, ROWS = MF * 16, HALF = MF / WRS, WR = 32 * NC, SUB = (ROWS + WR) * 64, SLOT = PK * SUB,
                DA = ROWS / (8 * NW), NCW = NC * 4 / NW, DPP = PK * (DA + NCW);
  static_assert(MF % WRS == 0 && ROWS % (8 * NW) == 0 && (NC * 4) % NW == 0, "tile does not split over the waves");
  __shared__ __attribute__((aligned(16))) bf16 smem[R * SLOT];
  __shared__ float sMR[2][LNF ? ROWS : 1];              // folded LayerNorm: rstd and rstd * mean per row
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  const int wgid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  // consecutive ids (one XCD) = the K splits and row groups of one column tile: its weight panel is read from
  // HBM once and served to the other row groups from that XCD's L2
  const int split = wgid % splitk, rg = (wgid / splitk) % rgroups, tile = wgid / (splitk * rgroups);
  const int n0 = tile * WR, m0 = rg * ROWS;
  const int kb = split * kr, klen = min(kr, K - kb), NS = klen / 64, NP = (NS + PK - 1) / PK;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wc = wid & 1, wr = wid >> 1;
  // folded LayerNorm (a.fold_stat): the row sums [M][tiles][2] of the block's rows are requested BEFORE the ring's
  // first panels and reduced after them, so their round trip overlaps the DMA latency; 8 threads per row, thread p
  // summing 16-B pairs of tiles p, p + 8, ... in order, then a fixed xor tree (every block forms the same bits)
  constexpr int FCH = LNF ? (ROWS + 31) / 32 : 1, FT = LNF ? 10 : 1;  // 32-row chunks; up to 80 tiles = 8 x 10
  // every load unconditional (clamped address, masked at the reduction): a select on a loaded value made the
  // compiler wait for it (vmcnt(0)) before the ring's first DMAs
  float2 fq[FCH][FT];
  f32x4 pfs[LNF ? NC : 1], pfc[LNF ? NC : 1];
  if constexpr (LNF) {
    const int T = a.fold_tiles, part = tid & 7;
#pragma unroll
    for (int ch = 0; ch < FCH; ++ch) {
      const int gr = min(m0 + ch * 32 + (tid >> 3), M - 1);
      const float* sr = a.fold_stat + (long long)gr * T * 2;
#pragma unroll
      for (int j = 0; j < FT; ++j) fq[ch][j] = *(const float2*)(sr + 2 * min(part + 8 * j, T - 1));
    }
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const int col0 = min(n0 + (wc * NC + c) * 16 + 4 * (lane >> 4), N - 4);
      pfs[c] = *(const f32x4*)(epi.fold_s + col0);
      pfc[c] = *(const f32x4*)(epi.fold_c + col0);
    }
  }
  // DMA sources: wave `wid` moves A rows [wid*ROWS/NW, +ROWS/NW) (DA instructions of 8 rows) and W rows
  // [8 NCW wid, +8 NCW) (NCW instructions)
  const bf16* srcA[DA];
#pragma unroll
  for (int j = 0; j < DA; ++j) {
    const int row = wid * (ROWS / NW) + j * 8 + (lane >> 3);
    const int ch = (lane & 7) ^ ((row >> 1) & 7);
    const int gr = min(m0 + row, M - 1);
    const long long off = a.rpb ? (long long)(gr / a.rpb) * a.bstride + (long long)(gr % a.rpb) * a.ld : (long long)gr * a.ld;
    srcA[j] = a.ptr + off + kb + ch * 8;
  }
  const bf16* srcW[NCW];
#pragma unroll
  for (int j = 0; j < NCW; ++j) {
    const int row = (wid * NCW + j) * 8 + (lane >> 3);
    const int ch = (lane & 7) ^ ((row >> 1) & 7);
    srcW[j] = w + (long long)min(n0 + row, N - 1) * ldw + kb + ch * 8;
  }
  // super-panel p = sub-panels [p PK, p PK + PK) (clamped to the last one: duplicates are never read)
  auto issue = [&](int p) {
#pragma unroll
    for (int u = 0; u < PK; ++u) {
      const int sp = min(p * PK + u, NS - 1);
      bf16* s = smem + (p % R) * SLOT + u * SUB;
#pragma unroll
      for (int j = 0; j < DA; ++j)
        __builtin_amdgcn_global_load_lds((const void*)(srcA[j] + sp * 64),
                                         (__attribute__((address_space(3))) void*)(s + (wid * (ROWS / NW) + j * 8) * 64), 16, 0, 0);
#pragma unroll
      for (int j = 0; j < NCW; ++j)
        __builtin_amdgcn_global_load_lds((const void*)(srcW[j] + sp * 64),
                                         (__attribute__((address_space(3))) void*)(s + (ROWS + (wid * NCW + j) * 8) * 64), 16, 0, 0);
    }
  };

  f32x4 acc[NC][HALF];
#pragma unroll
  for (int c = 0; c < NC; ++c)
#pragma unroll
    for (int i = 0; i < HALF; ++i) acc[c][i] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int pre = min(R - 1, NP);
  for (int p = 0; p < pre; ++p) issue(p);
  for (int p = 0; p < NP; ++p) {
    vm_wait(min(NP - 1 - p, R - 2) * DPP);            // this wave's DMAs of super-panel p have landed
    asm volatile("s_barrier" ::: "memory");           // ... everyone's; slot of super-panel p-1 is free
    __builtin_amdgcn_sched_barrier(0);
    if (p + R - 1 < NP) issue(p + R - 1);
    auto sub = [&](int u) {
      const bf16* sA = smem + (p % R) * SLOT + u * SUB;
      const bf16* sW = sA + ROWS * 64;
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        const int ch = kk * 4 + (lane >> 4);
        bf16x8 fb[NC];
#pragma unroll
        for (int c = 0; c < NC; ++c) fb[c] = *(const bf16x8*)(sW + dswz((wc * NC + c) * 16 + (lane & 15), ch));
        bf16x8 fa[HALF];
#pragma unroll
        for (int i = 0; i < HALF; ++i) fa[i] = *(const bf16x8*)(sA + dswz((wr * HALF + i) * 16 + (lane & 15), ch));
#pragma unroll
        for (int c = 0; c < NC; ++c)
#pragma unroll
          for (int i = 0; i < HALF; ++i) acc[c][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[c], fa[i], acc[c][i], 0, 0, 0);
      }
    };
    if (p * PK + PK <= NS) {              // a whole super-panel: no per-sub-panel branch in the MFMA stream
#pragma unroll
      for (int u = 0; u < PK; ++u) sub(u);
    } else {
      for (int u = 0; u < NS - p * PK; ++u) sub(u);
    }
  }

  if constexpr (LNF) {
    const int T = a.fold_tiles, part = tid & 7;
#pragma unroll
    for (int ch = 0; ch < FCH; ++ch) {
      float s1 = 0.f, s2 = 0.f;
#pragma unroll
      for (int j = 0; j < FT; ++j) {
        const bool in = part + 8 * j < T;
        s1 += in ? fq[ch][j].x : 0.f;
        s2 += in ? fq[ch][j].y : 0.f;
      }
#pragma unroll
      for (int o = 1; o < 8; o <<= 1) {
        s1 += __shfl_xor(s1, o, 64);
        s2 += __shfl_xor(s2, o, 64);
      }
      const int rr = ch * 32 + (tid >> 3);
      if ((tid & 7) == 0 && rr < ROWS) {
        const float mean = s1 / (float)K, var = fmaxf(s2 / (float)K - mean * mean, 0.f);
        const float rs = rsqrtf(var + 1e-5f);
        sMR[0][rr] = rs;
        sMR[1][rr] = rs * mean;
      }
    }
    __syncthreads();
  }
  const bool to_slab = splitk > 1 || KIND == EPI_RESID_LN;
  // the epilogue's operands (bias chunks; DEC_QKV: each row's hypothesis and position) requested before the first
  // store, at clamped in-bounds addresses (loaded in the fragment loop, each took its own round trip)
  constexpr bool PRE = KIND == EPI_BF16 || KIND == EPI_DEC_QKV;
  f32x4 bpre[NC];
  int hpre[HALF], ppre[HALF];
  if constexpr (PRE) {
    if (!to_slab) {
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        const int col0 = n0 + (wc * NC + c) * 16 + 4 * (lane >> 4);
        bpre[c] = epi.bias ? *(const f32x4*)(epi.bias + (col0 < N ? col0 : 0)) : f32x4{0.f, 0.f, 0.f, 0.f};
      }
      if constexpr (KIND == EPI_DEC_QKV) {
#pragma unroll
        for (int i = 0; i < HALF; ++i) {
          const int row = min(m0 + (wr * HALF + i) * 16 + (lane & 15), M - 1);
          hpre[i] = epi.row_hyp[row];
          ppre[i] = epi.row_pos[row];
        }
      }
      // one wait for all of them here, before any store: each value re-emerges from an empty asm, so no later use
      // carries a wait (the compiler put a vmcnt(0) at every fragment, i.e. waited for the previous one's stores)
#pragma unroll
      for (int c = 0; c < NC; ++c) asm volatile("" : "+v"(bpre[c]));
      if constexpr (KIND == EPI_DEC_QKV) {
#pragma unroll
        for (int i = 0; i < HALF; ++i) asm volatile("" : "+v"(hpre[i]), "+v"(ppre[i]));
      }
    }
  }
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int col0 = n0 + (wc * NC + c) * 16 + 4 * (lane >> 4);
#pragma unroll
    for (int i = 0; i < HALF; ++i) {
      const int lr = (wr * HALF + i) * 16 + (lane & 15), row = m0 + lr;
      // residual producer for a folded LayerNorm (uniform over the block; N % 16 == 0): the updated residual, its
      // bf16(x * g) operand image and the per-(16-column tile, row) sums, the tile's 4 lanes of a row reduced by a
      // fixed xor tree (every lane takes part: the 4 lanes of a row share its validity)
      if (KIND == EPI_RESID_F32 && !to_slab && epi.xg_out) {
        const bool ok = row < M && col0 < N;
        f32x4 xn = f32x4{0.f, 0.f, 0.f, 0.f};
        if (ok) {
          f32x4* px = (f32x4*)((float*)epi.out + (long long)row * epi.ldc + col0);
          xn = *px + acc[c][i] + *(const f32x4*)(epi.bias + col0);
          *px = xn;
          const f32x4 g = *(const f32x4*)(epi.xg_g + col0);
          bf16x4 xg;
#pragma unroll
          for (int e = 0; e < 4; ++e) xg[e] = f2bf(xn[e] * g[e]);
          *(bf16x4*)(epi.xg_out + (long long)row * epi.xg_ld + col0) = xg;
        }
        float s1 = (xn[0] + xn[1]) + (xn[2] + xn[3]);
        float s2 = (xn[0] * xn[0] + xn[1] * xn[1]) + (xn[2] * xn[2] + xn[3] * xn[3]);
        s1 += __shfl_xor(s1, 16, 64);
        s2 += __shfl_xor(s2, 16, 64);
        s1 += __shfl_xor(s1, 32, 64);
        s2 += __shfl_xor(s2, 32, 64);
        if (ok && (lane >> 4) == 0)
          *(float2*)(epi.stat_out + ((long long)row * (N >> 4) + (col0 >> 4)) * 2) = make_float2(s1, s2);
        continue;
      }
      if (col0 >= N || row >= M) continue;
      if (to_slab) {
        *(f32x4*)(part + ((long long)split * M + row) * N + col0) = acc[c][i];
      } else if (LNF) {
        // folded LayerNorm consumer: rstd (W . gx) - rstd mean (W g) + (W b + bias), then the epilogue kind
        const float rs = sMR[0][lr], rm = sMR[1][lr];
        f32x4 v;
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = fmaf(acc[c][i][e], rs, pfc[c][e] - rm * pfs[c][e]);
        if constexpr (PRE) apply_epi4_pre<KIND>(epi, row, col0, v, bpre[c], hpre[KIND == EPI_DEC_QKV ? i : 0],
                                                ppre[KIND == EPI_DEC_QKV ? i : 0]);
        else apply_epi4<KIND>(epi, row, col0, v);
      } else {
        if constexpr (PRE) apply_epi4_pre<KIND>(epi, row, col0, acc[c][i], bpre[c], hpre[KIND == EPI_DEC_QKV ? i : 0],
                                                ppre[KIND == EPI_DEC_QKV ? i : 0]);
        else apply_epi4<KIND>(epi, row, col0, acc[c][i]);
      }
    }
  }
}

// Sub-panels of 64 k per ring slot: one barrier per PK x 64 of K, fewer slots to stay within 144 KiB.  Default
// 4 where 3+ such slots fit (32/64-row blocks), else 2 (VLOG_AMD_RING_PK=1|2|4 overrides).  Measured on the
// 150-row large-v3 decode: dec_gemm 405.6 (PK 1) / 391.2 (2) / 380.1 (4) ms per step, identical tokens.
static int ring_pk() {
  static const int v = [] {
    const char* e = std::getenv("VLOG_AMD_RING_PK");
    return e ? std::atoi(e) : 4;
  }();
  return v;
}

// LDS budget of a ring block: 144 KiB (one block per CU: the deepest ring) or 72 KiB (VLOG_AMD_RING_LDS=72: two
// resident blocks per CU, twice the DMA requests in flight per CU with half the ring depth each).
static int ring_lds_kb() {
  static const int v = [] {
    const char* e = std::getenv("VLOG_AMD_RING_LDS");
    return e && std::atoi(e) == 72 ? 72 : 144;
  }();
  return v;
}

template <int MF, int KIND, int NC, int CAPKB, bool LNF, int NW = 4>
static void run_ring_cap_f(const GemmA& a, const bf16* w, long long ldw, int M, int N, int K, const GemmEpi& epi, float* ws,
                         int splitk, int kr, hipStream_t st) {
  constexpr int SUBB = (MF * 16 + 32 * NC) * 128;      // bytes of one 64-k sub-panel
  constexpr int CAP = CAPKB * 1024;
  constexpr int R = std::max(2, NC == 1 ? std::min(MF <= 4 ? 8 : MF <= 8 ? 7 : 6, CAP / SUBB) : std::min(8, CAP / SUBB));
  constexpr int R2 = std::min(8, CAP / (2 * SUBB)), R4 = std::min(8, CAP / (4 * SUBB));
  const int tiles_n = (N + 32 * NC - 1) / (32 * NC);
  const int rgroups = (M + MF * 16 - 1) / (MF * 16);
  const dim3 grid(tiles_n * rgroups * splitk);
  const int pk = ring_pk();
  if constexpr (R4 >= 3) {
    if (pk == 4) {
      hipLaunchKernelGGL((dec_ring_kernel<MF, KIND, R4, 4, NC, LNF, NW>), grid, dim3(NW * 64), 0, st, a, w, ldw, M, N, K, epi, tiles_n,
                         splitk, kr, ws, rgroups);
      WM_LAUNCH_CHECK("dec_ring_kernel");
      return;
    }
  }
  if constexpr (R2 >= 3) {
    if (pk >= 2) {
      hipLaunchKernelGGL((dec_ring_kernel<MF, KIND, R2, 2, NC, LNF, NW>), grid, dim3(NW * 64), 0, st, a, w, ldw, M, N, K, epi, tiles_n,
                         splitk, kr, ws, rgroups);
      WM_LAUNCH_CHECK("dec_ring_kernel");
      return;
    }
  }
  static_assert(R * SUBB <= 160 * 1024, "ring exceeds the LDS");
  hipLaunchKernelGGL((dec_ring_kernel<MF, KIND, R, 1, NC, LNF, NW>), grid, dim3(NW * 64), 0, st, a, w, ldw, M, N, K, epi, tiles_n, splitk,
                     kr, ws, rgroups);
  WM_LAUNCH_CHECK("dec_ring_kernel");
}

template <int MF, int KIND, int NC, int CAPKB>
static void run_ring_cap(const GemmA& a, const bf16* w, long long ldw, int M, int N, int K, const GemmEpi& epi, float* ws,
                         int splitk, int kr, hipStream_t st, int waves) {
  if constexpr (MF % 4 == 0 && MF * 16 % 64 == 0 && NC % 2 == 0) {
    if (waves == 8 && !a.fold_stat) {
      run_ring_cap_f<MF, KIND, NC, CAPKB, false, 8>(a, w, ldw, M, N, K, epi, ws, splitk, kr, st);
      return;
    }
  }
  if (waves == 8) throw std::runtime_error("dec_ring: 8 waves need 64 or 128 rows x 64 or 128 columns, no folded LayerNorm");
  if constexpr (KIND == EPI_BF16 || KIND == EPI_DEC_QKV) {
    if (a.fold_stat) {
      run_ring_cap_f<MF, KIND, NC, CAPKB, true>(a, w, ldw, M, N, K, epi, ws, splitk, kr, st);
      return;
    }
  }
  run_ring_cap_f<MF, KIND, NC, CAPKB, false>(a, w, ldw, M, N, K, epi, ws, splitk, kr, st);
}

template <int MF, int KIND, int NC>
static void run_ring(const GemmA& a, const bf16* w, long long ldw, int M, int N, int K, const GemmEpi& epi, float* ws,
                     int splitk, int kr, hipStream_t st, int lds_kb, int waves) {
  if ((lds_kb > 0 ? lds_kb : ring_lds_kb()) == 72) run_ring_cap<MF, KIND, NC, 72>(a, w, ldw, M, N, K, epi, ws, splitk, kr, st, waves);
  else run_ring_cap<MF, KIND, NC, 144>(a, w, ldw, M, N, K, epi, ws, splitk, kr, st, waves);
}

// rows_per_block 0: one row group covering every row (MF from M); else 32 / 64 / 96 / 128 / 160 rows per block
// and ceil(M / rows) row groups.
template <int KIND>
static void dispatch_ring(const GemmA& a, const bf16* w, long long ldw, int M, int N, int K, const GemmEpi& epi,
                          float* ws, int splitk, int kr, int rows_per_block, int cols, hipStream_t st, int lds_kb, int waves) {
  const int rows = rows_per_block > 0 ? std::min(rows_per_block, ((M + 31) / 32) * 32) : M;
  if (cols == 128) {                     // 128-column tiles (waves of 64 columns): row groups of 64 or 128
    if (rows <= 64) run_ring<4, KIND, 4>(a, w, ldw, M, N, K, epi, ws, splitk, kr, st, lds_kb, waves);
    else if (rows <= 128) run_ring<8, KIND, 4>(a, w, ldw, M, N, K, epi, ws, splitk, kr, st, lds_kb, waves);
    else throw std::runtime_error("dec_ring: 128-column tiles take at most 128 rows per block");
    return;
  }
  if (cols == 64) {                      // 64-column tiles: row groups of 32, 64 or 128
    if (rows <= 32) run_ring<2, KIND, 2>(a, w, ldw, M, N, K, epi, ws, splitk, kr, st, lds_kb, waves);
    else if (rows <= 64) run_ring<4, KIND, 2>(a, w, ldw, M, N, K, epi, ws, splitk, kr, st, lds_kb, waves);
    else if (rows <= 128) run_ring<8, KIND, 2>(a, w, ldw, M, N, K, epi, ws, splitk, kr, st, lds_kb, waves);
    else throw std::runtime_error("dec_ring: 64-column tiles take at most 128 rows per block");
    return;
  }
  if (rows <= 32) run_ring<2, KIND, 1>(a, w, ldw, M, N, K, epi, ws, splitk, kr, st, lds_kb, waves);
  else if (rows <= 64) run_ring<4, KIND, 1>(a, w, ldw, M, N, K, epi, ws, splitk, kr, st, lds_kb, waves);
  else if (rows <= 96) run_ring<6, KIND, 1>(a, w, ldw, M, N, K, epi, ws, splitk, kr, st, lds_kb, waves);
  else if (rows <= 128) run_ring<8, KIND, 1>(a, w, ldw, M, N, K, epi, ws, splitk, kr, st, lds_kb, waves);
  else run_ring<10, KIND, 1>(a, w, ldw, M, N, K, epi, ws, splitk, kr, st, lds_kb, waves);
}

// Ring path: N % 4 == 0, K % 64 == 0; M <= 160 for one row group, any M with rows_per_block > 0.  kr = K range
// per block (0: the whole K up to 1280, else split into ceil(K / 1280) ranges).  cols = output columns per block,
// 32 or 64 (64: at most 64 rows per block).  A column tile's width never changes a row's K summation order, so
// both widths give bit-identical results.  Returns false when unsupported.
bool launch_dec_ring(const GemmA& a, const bf16* w, long long ldw, int M, int N, int K, const GemmEpi& epi, float* ws,
                     size_t ws_bytes, int kr, hipStream_t st, int rows_per_block, int cols, int lds_kb, int waves) {
  if (lds_kb != 0 && lds_kb != 72 && lds_kb != 144) return false;
  if (waves != 4 && waves != 8) return false;
  if (waves == 8) {                      // 8 waves: 64 / 128 rows per block x 64 / 128 columns, no folded LayerNorm
    const int rows = rows_per_block > 0 ? std::min(rows_per_block, ((M + 31) / 32) * 32) : M;
    if (cols < 64 || !(rows > 32 && rows <= 128) || a.fold_stat) return false;
  }
  if ((rows_per_block <= 0 && M > 160) || rows_per_block > 160 || N % 4 != 0 || K % 64 != 0) return false;
  if (cols != 32 && cols != 64 && cols != 128) return false;
  if (cols >= 64 && (rows_per_block <= 0 ? M : std::min(rows_per_block, ((M + 31) / 32) * 32)) > 128) return false;
  if (cols == 128 && lds_kb == 72) return false;        // a 128 x 128 sub-panel is 32 KiB: two slots would be all of it
  if (kr <= 0) kr = K <= 1280 ? K : ((K + (K + 1279) / 1280 - 1) / ((K + 1279) / 1280) + 63) / 64 * 64;
  if (kr % 64 != 0) return false;
  const int splitk = (K + kr - 1) / kr;
  if ((K - (splitk - 1) * kr) % 64 != 0) return false;
  const bool slab = splitk > 1 || epi.kind == EPI_RESID_LN;
  if (slab && (!ws || (size_t)splitk * M * N * 4 > ws_bytes)) return false;
  // folded LayerNorm: a consumer needs the stat rows of its pass; a producer writes whole 16-column tiles
  if (a.fold_stat && (!(a.fold_tiles == 1 || (a.fold_tiles % 2 == 0 && a.fold_tiles <= 80)) || a.fold_rows < M || epi.bias ||
                      !epi.fold_s || !epi.fold_c || slab)) return false;
  if (epi.xg_out && (epi.kind != EPI_RESID_F32 || N % 16 != 0 || !epi.stat_out || !epi.bias || !epi.xg_g)) return false;
  if (!slab && (epi.ldc % 4 != 0 || (epi.rpb != 0 && epi.bstride % 4 != 0))) return false;
  switch (epi.kind) {
    case EPI_BF16: dispatch_ring<EPI_BF16>(a, w, ldw, M, N, K, epi, ws, splitk, kr, rows_per_block, cols, st, lds_kb, waves); break;
    case EPI_RESID_F32: dispatch_ring<EPI_RESID_F32>(a, w, ldw, M, N, K, epi, ws, splitk, kr, rows_per_block, cols, st, lds_kb, waves); break;
    case EPI_F32: dispatch_ring<EPI_F32>(a, w, ldw, M, N, K, epi, ws, splitk, kr, rows_per_block, cols, st, lds_kb, waves); break;
    case EPI_DEC_QKV: dispatch_ring<EPI_DEC_QKV>(a, w, ldw, M, N, K, epi, ws, splitk, kr, rows_per_block, cols, st, lds_kb, waves); break;
    case EPI_RESID_LN: dispatch_ring<EPI_RESID_LN>(a, w, ldw, M, N, K, epi, ws, splitk, kr, rows_per_block, cols, st, lds_kb, waves); break;
    default: return false;
  }
  if (slab && !epi.defer_combine) launch_splitk_combine(ws, splitk, M, N, epi, st);
  return true;
}

// (A register-streaming variant — every wave loading its own fragments from L2/HBM, no LDS — measured 2x
// slower than the ring on these shapes: ~30-35 GB/s per CU either way, the A re-reads dominate.)

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

// ------------------------------------------------------------------------------------------------------
// One-shot decoder GEMM (the default decoder projection path): one 512-thread block = 32 rows x NC*16 output
// columns x a K range of <= 1280.  The K range is split over the 8 waves (up to 5 k-steps of 32 each); every
// wave issues ALL its loads at once — its W fragments (the HBM stream) and its A fragments (L2-resident
// activations), 16 B per lane straight into MFMA operand registers, no LDS staging — so a block pays one
// memory round trip, with up to 160 KB in flight per block.  The 8 per-wave partial tiles are summed through
// LDS in wave order (deterministic), then the epilogue is applied in place (or a split-K slab is written when
// K > 1280).  Row groups of one column tile get consecutive ids (one XCD): the weight panel is fetched from HBM
// once and served to the other row groups by that XCD's L2.  Replaces, at decoder row counts, split-K slabs
// whose write + re-read cost more than the weight stream itself (tools/dec_gemm_bench: slab stores were ~half
// of the skinny kernel's time at M = 150).
template <int NC, int KIND>
__global__ __launch_bounds__(512) void dec_oneshot_kernel(GemmA a, const bf16* __restrict__ w, long long ldw, int M,
                                                          int N, int K, GemmEpi epi, int rgroups, int splitk, int kr,
                                                          float* __restrict__ part) {
  constexpr int KSMAX = 5;
  __shared__ __attribute__((aligned(16))) f32x4 sred[8][2 * NC][64];
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  const int wgid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  const int split = wgid % splitk, rg = (wgid / splitk) % rgroups, tile = wgid / (splitk * rgroups);
  const int n0 = tile * (NC * 16), m0 = rg * 32;
  const int kb = split * kr, klen = min(kr, K - kb);
  // the wave index through readfirstlane: the k-step guards below are then scalar (wave-uniform) branches.
  // MFMAs ignore EXEC, so an MFMA behind a guard the compiler treats as divergent would still run, on the
  // (uninitialised) operand registers of a skipped step (tools/gemv_check found NaN outputs that way)
  const int tid = threadIdx.x, lane = tid & 63, wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nks = klen / 32;                                    // k-steps of this block
  const int s0 = wv * nks / 8, s1 = (wv + 1) * nks / 8;         // this wave's k-steps [s0, s1)
  const int kl = kb + 8 * (lane >> 4);
  bf16x8 fw[KSMAX][NC], fa[KSMAX][2];
#pragma unroll
  for (int s = 0; s < KSMAX; ++s) {
    if (s0 + s < s1) {
      const int k = kl + 32 * (s0 + s);
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        const int n = min(n0 + c * 16 + (lane & 15), N - 1);
        fw[s][c] = *(const bf16x8*)(w + (long long)n * ldw + k);
      }
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int m = min(m0 + i * 16 + (lane & 15), M - 1);
        const long long off = a.rpb ? (long long)(m / a.rpb) * a.bstride + (long long)(m % a.rpb) * a.ld : (long long)m * a.ld;
        fa[s][i] = *(const bf16x8*)(a.ptr + off + k);
      }
    }
  }
  f32x4 acc[NC][2];
#pragma unroll
  for (int c = 0; c < NC; ++c)
#pragma unroll
    for (int i = 0; i < 2; ++i) acc[c][i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < KSMAX; ++s) {
    if (s0 + s < s1) {
#pragma unroll
      for (int c = 0; c < NC; ++c)
#pragma unroll
        for (int i = 0; i < 2; ++i) acc[c][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fw[s][c], fa[s][i], acc[c][i], 0, 0, 0);
    }
  }
  // W fragment as the MFMA A operand: acc[c][i] holds C^T, lane l has row m0 + 16 i + (l & 15) and the 4
  // consecutive columns n0 + 16 c + 4 (l >> 4) + e
#pragma unroll
  for (int c = 0; c < NC; ++c)
#pragma unroll
    for (int i = 0; i < 2; ++i) sred[wv][c * 2 + i][lane] = acc[c][i];
  __syncthreads();
  const bool to_slab = splitk > 1 || KIND == EPI_RESID_LN;
  for (int idx = tid; idx < 2 * NC * 64; idx += 512) {
    const int f = idx >> 6, ln = idx & 63;
    f32x4 v = sred[0][f][ln];
#pragma unroll
    for (int w2 = 1; w2 < 8; ++w2) v += sred[w2][f][ln];
    const int c = f >> 1, i = f & 1;
    const int row = m0 + i * 16 + (ln & 15), col0 = n0 + c * 16 + 4 * (ln >> 4);
    if (row >= M || col0 >= N) continue;
    if (to_slab)
      *(f32x4*)(part + ((long long)split * M + row) * N + col0) = v;
    else
      apply_epi4<KIND>(epi, row, col0, v);
  }
}

template <int NC, int KIND>
static void run_oneshot(const GemmA& a, const bf16* w, long long ldw, int M, int N, int K, const GemmEpi& epi, float* ws,
                        int splitk, int kr, hipStream_t st) {
  const int tiles_n = (N + NC * 16 - 1) / (NC * 16), rgroups = (M + 31) / 32;
  hipLaunchKernelGGL((dec_oneshot_kernel<NC, KIND>), dim3(tiles_n * rgroups * splitk), dim3(512), 0, st, a, w, ldw, M, N,
                     K, epi, rgroups, splitk, kr, ws);
  WM_LAUNCH_CHECK("dec_oneshot_kernel");
}

template <int KIND>
static void dispatch_oneshot(const GemmA& a, const bf16* w, long long ldw, int M, int N, int K, const GemmEpi& epi,
                             float* ws, int splitk, int kr, int nc, hipStream_t st) {
  if (nc == 4) run_oneshot<4, KIND>(a, w, ldw, M, N, K, epi, ws, splitk, kr, st);
  else run_oneshot<2, KIND>(a, w, ldw, M, N, K, epi, ws, splitk, kr, st);
}

// One-shot path: K % 32 == 0, N % 4 == 0, any M (rows in groups of 32).  K ranges of at most 1280 (8 waves x 5
// k-steps): K <= 1280 in one range, else split into equal ranges (multiples of 32) with slabs combined by
// launch_splitk_combine.  nc = 16-column fragments per block (2 or 4).  Returns false when unsupported.
bool launch_dec_oneshot(const GemmA& a, const bf16* w, long long ldw, int M, int N, int K, const GemmEpi& epi, float* ws,
                        size_t ws_bytes, int nc, hipStream_t st) {
  if (M <= 0 || N % 4 != 0 || K % 32 != 0 || (nc != 2 && nc != 4)) return false;
  const int ks = K / 32;
  const int splitk = (ks + 39) / 40;                       // ranges of <= 40 k-steps (1280)
  if (ks % splitk != 0) return false;
  const int kr = K / splitk;
  const bool slab = splitk > 1 || epi.kind == EPI_RESID_LN;
  if (slab && (!ws || (size_t)splitk * M * N * 4 > ws_bytes)) return false;
  // folded LayerNorm: a consumer needs the stat rows of its pass; a producer writes whole 16-column tiles
  if (a.fold_stat && (!(a.fold_tiles == 1 || (a.fold_tiles % 2 == 0 && a.fold_tiles <= 80)) || a.fold_rows < M || epi.bias ||
                      !epi.fold_s || !epi.fold_c || slab)) return false;
  if (epi.xg_out && (epi.kind != EPI_RESID_F32 || N % 16 != 0 || !epi.stat_out || !epi.bias || !epi.xg_g)) return false;
  if (!slab && (epi.ldc % 4 != 0 || (epi.rpb != 0 && epi.bstride % 4 != 0))) return false;
  switch (epi.kind) {
    case EPI_BF16: dispatch_oneshot<EPI_BF16>(a, w, ldw, M, N, K, epi, ws, splitk, kr, nc, st); break;
    case EPI_RESID_F32: dispatch_oneshot<EPI_RESID_F32>(a, w, ldw, M, N, K, epi, ws, splitk, kr, nc, st); break;
    case EPI_F32: dispatch_oneshot<EPI_F32>(a, w, ldw, M, N, K, epi, ws, splitk, kr, nc, st); break;
    case EPI_DEC_QKV: dispatch_oneshot<EPI_DEC_QKV>(a, w, ldw, M, N, K, epi, ws, splitk, kr, nc, st); break;
    case EPI_RESID_LN: dispatch_oneshot<EPI_RESID_LN>(a, w, ldw, M, N, K, epi, ws, splitk, kr, nc, st); break;
    default: return false;
  }
  if (slab && !epi.defer_combine) launch_splitk_combine(ws, splitk, M, N, epi, st);
  return true;
}

// ------------------------------------------------------------------------------------------------------
// Small-M weight-streaming decoder GEMM (M <= 32 rows: one window's beam, a few windows): at these row counts
// a projection is a GEMV over the weight matrix, and the cost is how many weight bytes each CU has in
// flight and how many CUs stream.  One 256-thread block = 16 output columns x a K range of kr (a multiple of
// 128); wave w owns an equal share of its 32-deep k-steps and issues ALL of them at once: the weight
// fragments (16 B per lane, non-temporal: each weight byte is read once per step, MI355X_MICROARCH
// nt-weights) and the activation fragments (rows clamped to M - 1, L2/L1-resident), then its MFMAs
// (16x16x32: the weight fragment is the A operand, 16 columns x 32 k; the activations the B operand, 32 k x
// 16 rows, MF fragments of 16 rows).  The 4 wave partials are summed through LDS in wave order, then the
// epilogue runs in place (or a split-K slab is written: RESID_LN always, other kinds when kr < K).  Grid =
// 16-column tiles x K splits, >= ~256 blocks (gemv_plan).  NWV = 16 waves (1024 threads): a K range up to 5120 in
// one block (fc2 as a residual producer with row statistics, no split-K), the 16 partials summed in wave order.
template <int MF, int KSW, int KIND, bool LNA, int NWV = 4>
__global__ __launch_bounds__(NWV * 64) void gemv_dec_kernel(GemmA a, const bf16* __restrict__ w, long long ldw, int M,
                                                            int N, int K, GemmEpi epi, int splitk, int kr,
                                                            float* __restrict__ part, int abl) {
  static_assert(!LNA || NWV == 4, "the LayerNorm operand's statistics split assumes 256 threads");
  __shared__ __attribute__((aligned(16))) f32x4 sred[NWV][MF][64];
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  const int wgid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  const int split = wgid % splitk, tile = wgid / splitk;
  const int n0 = tile * 16;
  const int kb = split * kr, klen = min(kr, K - kb), nks = klen / 32;
  // wave index through readfirstlane: the k-step guards are scalar branches (MFMAs ignore EXEC, so an MFMA behind a
  // guard the compiler treats as divergent runs anyway, on a skipped step's uninitialised operands: NaN outputs,
  // found by tools/gemv_check).  (Zeroing the operands instead costs a memory wait at the first guarded load.)
  const int tid = threadIdx.x, lane = tid & 63, wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int s0 = wv * nks / NWV, s1 = (wv + 1) * nks / NWV;
  const bf16* wr = w + (long long)min(n0 + (lane & 15), N - 1) * ldw + kb + 8 * (lane >> 4);
  bf16x8 fw[KSW], fa[KSW][MF];
  // (LNA: every step's load issued unconditionally, the step clamped into the block's range, so the load count is
  // static and the statistics merge waits for its own loads only; the MFMAs keep their scalar step guards)
  auto load_w = [&]() {
#pragma unroll
    for (int s = 0; s < KSW; ++s) {
      if (LNA) {
        const int sc = min(s0 + s, nks - 1);
        fw[s] = __builtin_bit_cast(bf16x8, __builtin_nontemporal_load((const i32x4*)(wr + 32 * sc)));
      } else if (s0 + s < s1) {
        fw[s] = __builtin_bit_cast(bf16x8, __builtin_nontemporal_load((const i32x4*)(wr + 32 * (s0 + s))));
      }
    }
  };
  if constexpr (!LNA) {
    load_w();
    const bf16* ar[MF];
#pragma unroll
    for (int i = 0; i < MF; ++i) {
      const int m = min(i * 16 + (lane & 15), M - 1);
      const long long off = a.rpb ? (long long)(m / a.rpb) * a.bstride + (long long)(m % a.rpb) * a.ld : (long long)m * a.ld;
      ar[i] = a.ptr + off + kb + 8 * (lane >> 4);
    }
#pragma unroll
    for (int s = 0; s < KSW; ++s)
      if (s0 + s < s1) {
#pragma unroll
        for (int i = 0; i < MF; ++i) fa[s][i] = *(const bf16x8*)(ar[i] + 32 * (s0 + s));
      }
  } else {
    // LayerNorm-consuming operand (MF == 1: M <= 16).  Issued together with the weight stream: this wave's f32
    // activation chunks, the block's affine range (into LDS) and the producer's per-tile row statistics (sum and
    // sum of squares about the tile's own mean); then A = bf16((x - mean) * rstd * g + b).  The variance is
    // two-pass-equivalent: within-tile M2 plus 16 (tile mean - mean)^2 per tile, after the mean (no E[x^2] - mean^2
    // cancellation), so it agrees with resid_ln_reduce_kernel's two-pass statistics to f32 rounding.
    // Load order: the statistics and the affine range first, then the weight stream, then the activations, and the
    // barriers of the statistics merge are raw (LDS only: `s_waitcnt lgkmcnt(0); s_barrier`), so only the first
    // loads must have landed when the merge runs; the weight and activation loads stay in flight behind it and
    // each k-step waits for its own operands.  (With the loads issued weights-first and __syncthreads, whose
    // workgroup fence waits for every outstanding load, the operand cost 2.1-3.1 us per launch over a bf16 one.)
    __shared__ __attribute__((aligned(16))) float sg[1280], sb[1280];
    // thread t sums tiles [g T / 16, (g + 1) T / 16) of row t & 15 (g = t >> 4, at most 8 tiles); the 16 group
    // partials go through LDS and each lane adds them in group order (so every lane of a row, and every block,
    // gets the same bits)
    __shared__ float sst[16][16][2];
    constexpr int TG = 8;                                    // T <= 128 tiles (N <= 2048)
    const int T = a.ln_tiles, g = tid >> 4, r16 = tid & 15, mr = min(r16, M - 1);
    const int t0 = g * T / 16, t1 = (g + 1) * T / 16;
    float2 sv[TG];
#pragma unroll
    for (int j = 0; j < TG; ++j)
      sv[j] = (abl & 1) ? make_float2(0.f, 1.f) : *(const float2*)(a.ln_stat + ((long long)min(t0 + j, T - 1) * M + mr) * 2);
    float gv[5], bv[5];                                      // klen <= 1280 = 5 x 256
#pragma unroll
    for (int j = 0; j < 5; ++j) {
      const int i = min(tid + 256 * j, klen - 1);
      gv[j] = (abl & 4) ? 1.f : a.ln_g[kb + i];
      bv[j] = (abl & 4) ? 0.f : a.ln_b[kb + i];
    }
    load_w();
    const int m = min(lane & 15, M - 1);
    const float* xr = a.lnx + (long long)m * a.ld + kb + 8 * (lane >> 4);
    f32x4 xv[KSW][2];
#pragma unroll
    for (int s = 0; s < KSW; ++s) {
      const int sc = min(s0 + s, nks - 1);
      xv[s][0] = *(const f32x4*)(xr + 32 * sc);
      xv[s][1] = *(const f32x4*)(xr + 32 * sc + 4);
    }
    {
      float q1 = 0.f;
#pragma unroll
      for (int j = 0; j < TG; ++j)
        if (t0 + j < t1) q1 += sv[j].x;
      sst[g][r16][0] = q1;
    }
#pragma unroll
    for (int j = 0; j < 5; ++j)
      if (tid + 256 * j < klen) {
        sg[tid + 256 * j] = gv[j];
        sb[tid + 256 * j] = bv[j];
      }
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    float p1 = 0.f;
    if (!(abl & 8)) {
#pragma unroll
      for (int g2 = 0; g2 < 16; ++g2) p1 += sst[g2][lane & 15][0];
    }
    const float invn = 1.0f / (float)(a.ln_tiles * 16);
    const float mean = p1 * invn;                            // row lane & 15 == row tid & 15 (this thread's tiles)
    if (!(abl & 8)) {
      float q2 = 0.f;
#pragma unroll
      for (int j = 0; j < TG; ++j)
        if (t0 + j < t1) {
          const float dm = sv[j].x * (1.0f / 16.0f) - mean;
          q2 += sv[j].y + 16.0f * dm * dm;
        }
      sst[g][r16][1] = q2;
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    }
    float p2 = (abl & 8) ? 1.f : 0.f;
    if (!(abl & 8)) {
#pragma unroll
      for (int g2 = 0; g2 < 16; ++g2) p2 += sst[g2][lane & 15][1];
    }
    const float rstd = rsqrtf(p2 * invn + 1e-5f);
#pragma unroll
    for (int s = 0; s < KSW; ++s)
      if (s0 + s < s1) {
        const int k0 = 32 * (s0 + s) + 8 * (lane >> 4);
        const f32x4 g0 = *(const f32x4*)(sg + k0), g1 = *(const f32x4*)(sg + k0 + 4);
        const f32x4 b0 = *(const f32x4*)(sb + k0), b1 = *(const f32x4*)(sb + k0 + 4);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          fa[s][0][e] = f2bf((xv[s][0][e] - mean) * rstd * g0[e] + b0[e]);
          fa[s][0][4 + e] = f2bf((xv[s][1][e] - mean) * rstd * g1[e] + b1[e]);
        }
      }
  }
  // the epilogue's operands (bias chunk; DEC_QKV: each row's hypothesis and position), requested behind the operand
  // loads instead of after the reduction (there they cost one or two more round trips per launch)
  constexpr bool PRE = KIND == EPI_BF16 || KIND == EPI_DEC_QKV;
  f32x4 bpre = f32x4{0.f, 0.f, 0.f, 0.f};
  int hpre[MF], ppre[MF];
  if constexpr (PRE) {
    if (splitk == 1 && wv == 0) {
      const int c0 = n0 + 4 * (lane >> 4);
      if (epi.bias) bpre = *(const f32x4*)(epi.bias + (c0 < N ? c0 : 0));
      if constexpr (KIND == EPI_DEC_QKV) {
#pragma unroll
        for (int i = 0; i < MF; ++i) {
          const int row = min(i * 16 + (lane & 15), M - 1);
          hpre[i] = epi.row_hyp[row];
          ppre[i] = epi.row_pos[row];
        }
      }
    }
  }
  f32x4 acc[MF];
#pragma unroll
  for (int i = 0; i < MF; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < KSW; ++s)
    if (s0 + s < s1) {
#pragma unroll
      for (int i = 0; i < MF; ++i) acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fw[s], fa[s][i], acc[i], 0, 0, 0);
    }
#pragma unroll
  for (int i = 0; i < MF; ++i) sred[wv][i][lane] = acc[i];
  __syncthreads();
  if (wv != 0) return;
  // acc holds C^T: lane l has row m = 16 i + (l & 15) and the 4 consecutive columns n0 + 4 (l >> 4) + e
  const bool to_slab = splitk > 1 || KIND == EPI_RESID_LN;
  const int col0 = n0 + 4 * (lane >> 4);
  if (KIND == EPI_RESID_F32 && epi.stat_out) {
    // residual producer for a LayerNorm-consuming GEMM (no split-K): x += acc + bias in place, and this tile's
    // row statistics of the new x: the sum, then the sum of squares about the tile mean (columns in a fixed order:
    // the 4 of a lane, then the 4 lanes)
#pragma unroll
    for (int i = 0; i < MF; ++i) {
      f32x4 v = sred[0][i][lane];
#pragma unroll
      for (int w2 = 1; w2 < NWV; ++w2) v += sred[w2][i][lane];
      const int row = i * 16 + (lane & 15);
      const bool ok = row < M && col0 < N;
      float q1 = 0.f, q2 = 0.f;
      f32x4 xs = f32x4{0.f, 0.f, 0.f, 0.f};
      if (ok) {
        f32x4 u = v;
        if (epi.bias) u += *(const f32x4*)(epi.bias + col0);
        f32x4* xp = (f32x4*)((float*)epi.out + (long long)row * epi.ldc + col0);
        const f32x4 xn = *xp + u;
        *xp = xn;
        xs = xn;
        q1 = (xn[0] + xn[1]) + (xn[2] + xn[3]);
      }
      q1 += __shfl_xor(q1, 16, 64);
      q1 += __shfl_xor(q1, 32, 64);
      if (ok) {
        const float mt = q1 * (1.0f / 16.0f);
        const float d0 = xs[0] - mt, d1 = xs[1] - mt, d2 = xs[2] - mt, d3 = xs[3] - mt;
        q2 = (d0 * d0 + d1 * d1) + (d2 * d2 + d3 * d3);
      }
      q2 += __shfl_xor(q2, 16, 64);
      q2 += __shfl_xor(q2, 32, 64);
      if (ok && lane < 16) *(float2*)(epi.stat_out + ((long long)tile * M + row) * 2) = make_float2(q1, q2);
    }
    return;
  }
  if constexpr (PRE) {                   // one wait for the prefetched operands, none at the fragments' stores
    if (!to_slab) {
      asm volatile("" : "+v"(bpre));
      if constexpr (KIND == EPI_DEC_QKV) {
#pragma unroll
        for (int i = 0; i < MF; ++i) asm volatile("" : "+v"(hpre[i]), "+v"(ppre[i]));
      }
    }
  }
#pragma unroll
  for (int i = 0; i < MF; ++i) {
    f32x4 v = sred[0][i][lane];
#pragma unroll
    for (int w2 = 1; w2 < NWV; ++w2) v += sred[w2][i][lane];
    const int row = i * 16 + (lane & 15);
    if (row >= M || col0 >= N) continue;
    if (to_slab)
      *(f32x4*)(part + ((long long)split * M + row) * N + col0) = v;
    else if constexpr (PRE)
      apply_epi4_pre<KIND>(epi, row, col0, v, bpre, hpre[KIND == EPI_DEC_QKV ? i : 0], ppre[KIND == EPI_DEC_QKV ? i : 0]);
    else
      apply_epi4<KIND>(epi, row, col0, v);
  }
}

// K range per block for the small-M path: no split when the 16-column tiles alone reach 3/4 of the CUs;
// otherwise split K (ranges of a multiple of 128, <= 1280) until the grid reaches ~256 blocks.
static int g_gemv_blocks = 256;          // target grid (tools/gemv_bench sweeps it: gemv_set_target_blocks)
void gemv_set_target_blocks(int b) { g_gemv_blocks = b > 0 ? b : 256; }
static int g_gemv_abl = 0;               // microbenchmark ablations of the LayerNorm operand (tools/gemv_bench only)
void gemv_set_ablation(int b) { g_gemv_abl = b; }

int gemv_splits(int M, int N, int K, int* kr_out) {
  if (M <= 0 || M > 32 || N % 16 != 0 || K % 128 != 0) return 0;
  const int tiles = N / 16;
  int s = tiles >= (3 * g_gemv_blocks) / 4 ? 1 : (g_gemv_blocks + tiles - 1) / tiles;
  s = std::max(s, (K + 1279) / 1280);                     // <= 10 k-steps per wave
  int kr = ((K + s - 1) / s + 127) / 128 * 128;
  s = (K + kr - 1) / kr;
  if (kr_out) *kr_out = kr;
  return s;
}

template <int MF, int KIND, bool LNA = false, int NWV = 4, int KSW = 10>
static void run_gemv(const GemmA& a, const bf16* w, long long ldw, int M, int N, int K, const GemmEpi& epi, float* ws,
                     int splitk, int kr, hipStream_t st) {
  hipLaunchKernelGGL((gemv_dec_kernel<MF, KSW, KIND, LNA, NWV>), dim3((N / 16) * splitk), dim3(NWV * 64), 0, st, a, w,
                     ldw, M, N, K, epi, splitk, kr, ws, g_gemv_abl);
  WM_LAUNCH_CHECK("gemv_dec_kernel");
}

// The LayerNorm-operand form issues every one of its KSW steps' loads (clamped, so the count is static): KSW is
// the per-wave step count of this K range rounded up to 3, 5 or 10 (cq at 4 K splits: 3 steps, not 10 loads)
template <int KIND>
static void run_gemv_lna(const GemmA& a, const bf16* w, long long ldw, int M, int N, int K, const GemmEpi& epi, float* ws,
                         int splitk, int kr, hipStream_t st) {
  const int per_wave = (kr / 32 + 3) / 4;
  if (per_wave <= 3) run_gemv<1, KIND, true, 4, 3>(a, w, ldw, M, N, K, epi, ws, splitk, kr, st);
  else if (per_wave <= 5) run_gemv<1, KIND, true, 4, 5>(a, w, ldw, M, N, K, epi, ws, splitk, kr, st);
  else run_gemv<1, KIND, true, 4, 10>(a, w, ldw, M, N, K, epi, ws, splitk, kr, st);
}

template <int KIND>
static void dispatch_gemv(const GemmA& a, const bf16* w, long long ldw, int M, int N, int K, const GemmEpi& epi,
                          float* ws, int splitk, int kr, hipStream_t st) {
  if (M <= 16) run_gemv<1, KIND>(a, w, ldw, M, N, K, epi, ws, splitk, kr, st);
  else run_gemv<2, KIND>(a, w, ldw, M, N, K, epi, ws, splitk, kr, st);
}

bool gemv_ln_fusable(int M, int N_prod, int K_prod, int K_cons) {
  return M >= 1 && M <= 16 && N_prod % 16 == 0 && N_prod / 16 <= 128 && K_prod % 128 == 0 && K_prod <= 5120 &&
         K_cons == N_prod && K_cons % 128 == 0;
}

// Small-M path: M <= 32, N % 16 == 0, K % 128 == 0.  Returns false when unsupported.  A residual producer with
// row statistics (EPI_RESID_F32 + stat_out) runs without split-K (K > 1280, up to 5120: 16-wave blocks); a
// LayerNorm-consuming operand (a.lnx) is supported for bf16 outputs and the self-attention qkv epilogue at M <= 16.
bool launch_dec_gemv(const GemmA& a, const bf16* w, long long ldw, int M, int N, int K, const GemmEpi& epi, float* ws,
                     size_t ws_bytes, hipStream_t st) {
  int kr = 0;
  int splitk = gemv_splits(M, N, K, &kr);
  if (splitk <= 0) return false;
  const bool stat = epi.kind == EPI_RESID_F32 && epi.stat_out;
  if (stat) {
    if (M > 16 || K > 5120 || N / 16 > 128) return false;
    splitk = 1;
    kr = K;
  }
  if (a.lnx) {
    if ((epi.kind != EPI_BF16 && epi.kind != EPI_DEC_QKV) || M > 16 || kr > 1280 || a.ln_tiles < 1 ||
        a.ln_tiles > 128 || a.ld % 4 != 0 || a.ln_tiles * 16 != K)
      return false;
  }
  const bool slab = splitk > 1 || epi.kind == EPI_RESID_LN;
  if (slab && (!ws || (size_t)splitk * M * N * 4 > ws_bytes)) return false;
  // folded LayerNorm: a consumer needs the stat rows of its pass; a producer writes whole 16-column tiles
  if (a.fold_stat && (!(a.fold_tiles == 1 || (a.fold_tiles % 2 == 0 && a.fold_tiles <= 80)) || a.fold_rows < M || epi.bias ||
                      !epi.fold_s || !epi.fold_c || slab)) return false;
  if (epi.xg_out && (epi.kind != EPI_RESID_F32 || N % 16 != 0 || !epi.stat_out || !epi.bias || !epi.xg_g)) return false;
  if (!slab && (epi.ldc % 4 != 0 || (epi.rpb != 0 && epi.bstride % 4 != 0))) return false;
  if (a.lnx) {
    if (epi.kind == EPI_DEC_QKV) run_gemv_lna<EPI_DEC_QKV>(a, w, ldw, M, N, K, epi, ws, splitk, kr, st);
    else run_gemv_lna<EPI_BF16>(a, w, ldw, M, N, K, epi, ws, splitk, kr, st);
    if (slab && !epi.defer_combine) launch_splitk_combine(ws, splitk, M, N, epi, st);
    return true;
  }
  if (stat && K > 1280) {
    run_gemv<1, EPI_RESID_F32, false, 16>(a, w, ldw, M, N, K, epi, ws, splitk, kr, st);
    return true;
  }
  switch (epi.kind) {
    case EPI_BF16: dispatch_gemv<EPI_BF16>(a, w, ldw, M, N, K, epi, ws, splitk, kr, st); break;
    case EPI_RESID_F32: dispatch_gemv<EPI_RESID_F32>(a, w, ldw, M, N, K, epi, ws, splitk, kr, st); break;
    case EPI_F32: dispatch_gemv<EPI_F32>(a, w, ldw, M, N, K, epi, ws, splitk, kr, st); break;
    case EPI_DEC_QKV: dispatch_gemv<EPI_DEC_QKV>(a, w, ldw, M, N, K, epi, ws, splitk, kr, st); break;
    case EPI_RESID_LN: dispatch_gemv<EPI_RESID_LN>(a, w, ldw, M, N, K, epi, ws, splitk, kr, st); break;
    default: return false;
  }
  if (slab && !epi.defer_combine) launch_splitk_combine(ws, splitk, M, N, epi, st);
  return true;
}

// ------------------------------------------------------------------------------------------------------
// Folded-LayerNorm vectors of a consumer projection W [N][K] (bf16, as the GEMM reads it) behind a LayerNorm with
// affine (g, b): s[n] = sum_k W[n][k] g[k] and c[n] = sum_k W[n][k] b[k] + bias[n], accumulated in f64 in a fixed
// order (one wave per output column), rounded once to f32.  Run once per weight upload (engine.cpp fold_vectors).
__global__ __launch_bounds__(256) void fold_vec_kernel(const bf16* __restrict__ w, int N, int K, const float* __restrict__ g,
                                                       const float* __restrict__ b, const float* __restrict__ bias,
                                                       float* __restrict__ s_out, float* __restrict__ c_out) {
  const int n = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (n >= N) return;
  double s = 0.0, c = 0.0;
  for (int k = lane; k < K; k += 64) {
    const double wv = (double)bf2f(w[(long long)n * K + k]);
    s += wv * (double)g[k];
    c += wv * (double)b[k];
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    s += __shfl_xor(s, o, 64);
    c += __shfl_xor(c, o, 64);
  }
  if (lane == 0) {
    s_out[n] = (float)s;
    c_out[n] = (float)(c + (double)bias[n]);
  }
}

void launch_fold_vectors(const bf16* w, int N, int K, const float* g, const float* b, const float* bias, float* s_out,
                         float* c_out, hipStream_t st) {
  hipLaunchKernelGGL(fold_vec_kernel, dim3((N + 3) / 4), dim3(256), 0, st, w, N, K, g, b, bias, s_out, c_out);
  WM_LAUNCH_CHECK("fold_vec_kernel");
}
