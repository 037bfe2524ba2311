// Large-M bf16 GEMM for gfx950 (encoder projections/MLP, conv2, cross-KV projection): C = A . W^T.
//
// 256 x 128 x 64 tiles, 8 waves (4 along M x 2 along N, 64 x 64 per wave, v_mfma_f32_16x16x32_bf16).
// Operands move HBM/L2 -> LDS by LDS-DMA (`global_load_lds_dwordx4`, 16 B per lane, 1 KiB per wave
// instruction) into a 3-slot ring: tile t+2 is issued while tile t is computed, and the loop waits with a
// COUNTED `s_waitcnt vmcnt(6)` (the 6 DMAs of tile t+1 stay in flight) before a raw `s_barrier`
// (cdna_hip_programming.md §5 "Pipelining across barriers": __syncthreads would drain vmcnt to 0).  The LDS
// image is lane-linear, so the bank-conflict XOR swizzle (16-B chunk c of row r stored at slot
// c ^ ((r >> 1) & 7)) is applied to the per-lane SOURCE address and undone on the ds_read (rule 21).  All
// LDS is one __shared__ array (trap 4(a)).  Rows past M re-load row M-1 (results discarded) so every lane
// issues its DMA with EXEC full.
#include "gemm.h"
#include "gemm_epi.h"
#include <stdexcept>
#include <string>

#define BBM 256
#define BBN 128
#define BBK 64
#define NSTAGE 3
#define A_BYTES (BBM * BBK * 2)
#define B_BYTES (BBN * BBK * 2)
#define STAGE_BYTES (A_BYTES + B_BYTES)

__device__ __forceinline__ int swz_off(int row, int ch) { return row * BBK + ((ch ^ ((row >> 1) & 7)) << 3); }

template <int KIND>
__global__ __launch_bounds__(512, 1) void gemm_big_kernel(GemmA a, const bf16* __restrict__ w, long long ldw, int M,
                                                          int N, int K, GemmEpi epi, int tiles_n) {
  __shared__ __attribute__((aligned(16))) char smem[NSTAGE * STAGE_BYTES];
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  const int wgid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  const int tm = wgid / tiles_n, tn = wgid - tm * tiles_n;
  const int m0 = tm * BBM, n0 = tn * BBN;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;            // 4 x 2 waves

  // Per-lane DMA sources.  Wave-instruction j of a stage covers 8 rows (1 KiB): lane -> (row, slot),
  // source chunk = slot ^ ((row >> 1) & 7).  A: 32 rows per wave (4 instrs), B: 16 rows per wave (2 instrs).
  const bf16* srcA[4];
  const bf16* srcB[2];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int row = wid * 32 + j * 8 + (lane >> 3), slot = lane & 7;
    const int ch = slot ^ ((row >> 1) & 7);
    int gr = m0 + row;
    if (gr >= M) gr = M - 1;
    const long long off = a.rpb ? (long long)(gr / a.rpb) * a.bstride + (long long)(gr % a.rpb) * a.ld : (long long)gr * a.ld;
    srcA[j] = a.ptr + off + ch * 8;
  }
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int row = wid * 16 + j * 8 + (lane >> 3), slot = lane & 7;
    const int ch = slot ^ ((row >> 1) & 7);
    int gn = n0 + row;
    if (gn >= N) gn = N - 1;
    srcB[j] = w + (long long)gn * ldw + ch * 8;
  }
  auto issue = [&](int t) {
    char* st = smem + (t % NSTAGE) * STAGE_BYTES;
    const int k0 = t * BBK;
#pragma unroll
    for (int j = 0; j < 4; ++j)
      __builtin_amdgcn_global_load_lds((const void*)(srcA[j] + k0), (__attribute__((address_space(3))) void*)(st + (wid * 32 + j * 8) * 128), 16, 0, 0);
#pragma unroll
    for (int j = 0; j < 2; ++j)
      __builtin_amdgcn_global_load_lds((const void*)(srcB[j] + k0), (__attribute__((address_space(3))) void*)(st + A_BYTES + (wid * 16 + j * 8) * 128), 16, 0, 0);
  };

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = K / BBK;
  issue(0);
  if (nk > 1) issue(1);
  for (int t = 0; t < nk; ++t) {
    if (t + 1 < nk) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (t + 2 < nk) issue(t + 2);
    const bf16* sA = (const bf16*)(smem + (t % NSTAGE) * STAGE_BYTES);
    const bf16* sB = (const bf16*)(smem + (t % NSTAGE) * STAGE_BYTES + A_BYTES);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 fa[4], fb[4];
      const int ch = kk * 4 + (lane >> 4);
#pragma unroll
      for (int i = 0; i < 4; ++i) fa[i] = *(const bf16x8*)(sA + swz_off(wm * 64 + i * 16 + (lane & 15), ch));
#pragma unroll
      for (int j = 0; j < 4; ++j) fb[j] = *(const bf16x8*)(sB + swz_off(wn * 64 + j * 16 + (lane & 15), ch));
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
    }
  }

#pragma unroll
  for (int i = 0; i < 4; ++i) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int col = n0 + wn * 64 + j * 16 + (lane & 15);
      if (col >= N) continue;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int row = m0 + wm * 64 + i * 16 + (lane >> 4) * 4 + e;
        if (row >= M) continue;
        apply_epi<KIND>(epi, row, col, acc[i][j][e]);
      }
    }
  }
}

template <int KIND>
static void run_big(const GemmA& a, const bf16* w, long long ldw, int M, int N, int K, const GemmEpi& epi, hipStream_t st) {
  const int tiles_m = (M + BBM - 1) / BBM, tiles_n = (N + BBN - 1) / BBN;
  hipLaunchKernelGGL((gemm_big_kernel<KIND>), dim3(tiles_m * tiles_n), dim3(512), 0, st, a, w, ldw, M, N, K, epi, tiles_n);
  WM_LAUNCH_CHECK("gemm_big_kernel");
}

bool gemm_big_applicable(int M, int N, int K) { return M >= 1024 && N >= 128 && K % BBK == 0 && K >= 2 * BBK; }

void launch_gemm_big(const GemmA& a, const bf16* w, long long ldw, int M, int N, int K, const GemmEpi& epi, hipStream_t st) {
  switch (epi.kind) {
    case EPI_BF16: run_big<EPI_BF16>(a, w, ldw, M, N, K, epi, st); break;
    case EPI_RESID_F32: run_big<EPI_RESID_F32>(a, w, ldw, M, N, K, epi, st); break;
    case EPI_GELU_POS_F32: run_big<EPI_GELU_POS_F32>(a, w, ldw, M, N, K, epi, st); break;
    case EPI_F32: run_big<EPI_F32>(a, w, ldw, M, N, K, epi, st); break;
    case EPI_DEC_QKV: run_big<EPI_DEC_QKV>(a, w, ldw, M, N, K, epi, st); break;
    case EPI_CROSS_KV: run_big<EPI_CROSS_KV>(a, w, ldw, M, N, K, epi, st); break;
    default: throw std::runtime_error("launch_gemm_big: bad epilogue kind");
  }
}
