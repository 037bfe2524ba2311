// Large-M bf16 GEMM for gfx950 (encoder projections/MLP, conv stem, cross-KV projection): C = A . W^T.
//
// 256 x 256 output tile per block, 8 waves as 2 (M) x 4 (N), each wave 128 x 64 = 8 x 4 fragments of
// v_mfma_f32_16x16x32_bf16 (64 flop per LDS byte read — a 64 x 64 wave tile is half that and runs into the
// LDS/L2 feed).  K advances in BK = 32 tiles through a 4-slot LDS ring filled by LDS-DMA
// (`global_load_lds_dwordx4`: 16 B per lane, one 1-KiB 16-row block per wave instruction, 4 per thread per
// tile).  Tile t+3 is issued right after the barrier that opens tile t, into the slot tile t-1 vacated;
// the barrier is preceded by a COUNTED `s_waitcnt vmcnt(8)` (tiles t+1, t+2 stay in flight) and is a raw
// `s_barrier`, so DMA stays in flight across it (cdna_hip_programming.md §5 "Pipelining across barriers").
// One __shared__ array (trap 4(a)).  LDS rows are 64 B; chunk c of row r sits in slot c ^ g(r) with
// g = [0,3,2,1][(r >> 2) & 3], which spreads every ds_read_b128 lane group (MI355X_MICROARCH.md §LDS) over
// 16 distinct 16-B bank slots; the swizzle is applied to the DMA SOURCE address (lane-linear LDS image,
// rule 21).  Rows/cols past M/N re-load row M-1 / N-1 (results discarded), so every DMA runs with EXEC full.
#include "gemm.h"
#include "gemm_epi.h"
#include <stdexcept>
#include <string>

#define BBM 256
#define BBN 256
#define BBK 32
#define NSLOT 4
#define TILE_A (BBM * BBK)            // elements
#define TILE_B (BBN * BBK)
#define SLOT_ELEMS (TILE_A + TILE_B)  // 16384 bf16 = 32 KiB

__device__ __forceinline__ int g_swz(int row) { return (4 - ((row >> 2) & 3)) & 3; }
__device__ __forceinline__ int swz32(int row, int ch) { return row * BBK + ((ch ^ g_swz(row)) << 3); }

template <int KIND>
__global__ __launch_bounds__(512, 1) void gemm_big_kernel(GemmA a, const bf16* __restrict__ w, long long ldw, int M,
                                                          int N, int K, GemmEpi epi, int tiles_n) {
  __shared__ __attribute__((aligned(16))) bf16 smem[NSLOT * SLOT_ELEMS];
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  const int wgid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  const int tm = wgid / tiles_n, tn = wgid - tm * tiles_n;
  const int m0 = tm * BBM, n0 = tn * BBN;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 2, wn = wid & 3;                 // 2 x 4 waves

  // DMA sources: wave `wid` fills rows [32 wid, 32 wid + 32) of A and of B, 16 rows per instruction;
  // lane -> (row = base + lane/4, slot = lane%4), source chunk = slot ^ g(row).
  const bf16* srcA[2];
  const bf16* srcB[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int row = wid * 32 + j * 16 + (lane >> 2);
    const int ch = (lane & 3) ^ g_swz(row);
    int gr = m0 + row;
    if (gr >= M) gr = M - 1;
    const long long off = a.rpb ? (long long)(gr / a.rpb) * a.bstride + (long long)(gr % a.rpb) * a.ld : (long long)gr * a.ld;
    srcA[j] = a.ptr + off + ch * 8;
    int gn = n0 + row;
    if (gn >= N) gn = N - 1;
    srcB[j] = w + (long long)gn * ldw + ch * 8;
  }
  auto issue = [&](int t) {
    bf16* st = smem + (t & (NSLOT - 1)) * SLOT_ELEMS;
    const int k0 = t * BBK;
#pragma unroll
    for (int j = 0; j < 2; ++j)
      __builtin_amdgcn_global_load_lds((const void*)(srcA[j] + k0),
                                       (__attribute__((address_space(3))) void*)(st + (wid * 32 + j * 16) * BBK), 16, 0, 0);
#pragma unroll
    for (int j = 0; j < 2; ++j)
      __builtin_amdgcn_global_load_lds((const void*)(srcB[j] + k0),
                                       (__attribute__((address_space(3))) void*)(st + TILE_A + (wid * 32 + j * 16) * BBK), 16, 0, 0);
  };

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = K / BBK;                 // >= 3 (gemm_big_applicable)
  issue(0);
  issue(1);
  issue(2);
  const int ch = lane >> 4, fr = lane & 15;
  for (int t = 0; t < nk; ++t) {
    // tile t's 4 DMAs retired for this wave once at most the later tiles' DMAs are outstanding
    if (t + 2 < nk) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else if (t + 1 < nk) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (t + 3 < nk) issue(t + 3);
    const bf16* sA = smem + (t & (NSLOT - 1)) * SLOT_ELEMS;
    const bf16* sB = sA + TILE_A;
    bf16x8 fb[4], fa[8];
#pragma unroll
    for (int j = 0; j < 4; ++j) fb[j] = *(const bf16x8*)(sB + swz32(wn * 64 + j * 16 + fr, ch));
#pragma unroll
    for (int i = 0; i < 8; ++i) fa[i] = *(const bf16x8*)(sA + swz32(wm * 128 + i * 16 + fr, ch));
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[j], fa[i], acc[i][j], 0, 0, 0);
    __builtin_amdgcn_sched_group_barrier(0x100, 12, 0);   // the 12 fragment reads first, then the 32 MFMAs
    __builtin_amdgcn_sched_group_barrier(0x008, 32, 0);   // (waits become counted lgkmcnt(N), reads overlap MFMAs)
  }

  // operands are swapped (W fragment as the MFMA A operand), so acc[i][j] holds C^T: lane l has row
  // m = ... + (l & 15) and the 4 consecutive columns n = ... + 4 (l >> 4) + e -> one vector store per fragment
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int row = m0 + wm * 128 + i * 16 + fr;
    if (row >= M) continue;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int col0 = n0 + wn * 64 + j * 16 + 4 * (lane >> 4);
      if (col0 < N) apply_epi4<KIND>(epi, row, col0, acc[i][j]);
    }
  }
}

template <int KIND>
static void run_big(const GemmA& a, const bf16* w, long long ldw, int M, int N, int K, const GemmEpi& epi, hipStream_t st) {
  const int tiles_m = (M + BBM - 1) / BBM, tiles_n = (N + BBN - 1) / BBN;
  hipLaunchKernelGGL((gemm_big_kernel<KIND>), dim3(tiles_m * tiles_n), dim3(512), 0, st, a, w, ldw, M, N, K, epi, tiles_n);
  WM_LAUNCH_CHECK("gemm_big_kernel");
}

bool gemm_big_applicable(int M, int N, int K) { return M >= 1024 && N >= 256 && N % 4 == 0 && K % BBK == 0 && K >= 3 * BBK; }

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
