// Large-M bf16 GEMM for gfx950 (encoder projections/MLP, conv stem, cross-KV projection): C = A . W^T, both
// operands K-contiguous.  256 x 256 output tile per 512-thread block, 8 waves as 2 (M) x 4 (N), each wave
// 128 x 64 = 8 x 4 fragments of v_mfma_f32_16x16x32_bf16 (operands swapped: the W fragment is the MFMA A
// operand, so a lane's accumulator holds 4 consecutive output columns of one row -> vector epilogue).
//
// Schedule (cdna_hip_programming.md §5 "The 256² 8-phase template", restated for this layout):
//  * BK = 64 K-tiles, LDS double buffer: [2][A 256 x 64 | W 256 x 64] bf16 = 128 KiB in ONE __shared__ array.
//    Rows are 128 B; 16-B chunk c of row r sits in slot c ^ ((r >> 1) & 7) (applied to the LDS-DMA source
//    address; the image itself is lane-linear).
//  * Each K-tile is 4 phases, one per 64 x 32 quadrant of the wave's output (Q00, Q01, Q11, Q10: each step
//    reloads ONE operand set).  A phase = [ds_read the new operand fragments, issue part of the NEXT tile's
//    LDS-DMA] lgkmcnt(0) s_barrier [setprio 1, 16 MFMAs, setprio 0] s_barrier.
//  * The two wave groups (wm = 0 / 1; one wave of each on every SIMD) run one barrier apart: group 1 takes
//    an extra barrier at entry (group 0 one at exit), so on every SIMD one wave's MFMAs overlap the other
//    wave's LDS reads and DMA issue.
//  * Tile t+1 is DMA'd into the other buffer during tile t's phases 0-1 (its last readers retired their
//    reads with lgkmcnt(0) before the barrier that opened tile t) and waited (vmcnt(0)) in phase 3 before
//    the barrier that ends that wave's read slot, so every reader of tile t+1 is past a barrier that follows
//    every issuing wave's wait (RAW), and no DMA targets a buffer a wave may still read (WAR).
#include "gemm.h"
#include "gemm_epi.h"
#include <algorithm>
#include <cstdlib>
#include <stdexcept>
#include <string>

#define P8_BM 256
#define P8_BN 256
#define P8_BK 64
#define P8_TILE (P8_BM * P8_BK)          // elements of one operand tile (A or W)
#define P8_BUF (2 * P8_TILE)             // A + W of one K-tile
#define P8_SR16 (P8_BN + 16)             // staged bf16 epilogue: LDS row stride (elements)
#define P8_SR32 (P8_BN + 4)              // staged f32 epilogue (128-row halves): LDS row stride (floats)
#define P8_SMEM (P8_BM * P8_SR16 > 2 * P8_BUF ? P8_BM * P8_SR16 : 2 * P8_BUF)   // bf16 elements

__device__ __forceinline__ int p8_swz(int row, int ch) { return row * P8_BK + ((ch ^ ((row >> 1) & 7)) << 3); }

// ABL (microbenchmark ablations only; the product uses 0): bit 0 skips the epilogue stores, bit 1 the MFMAs,
// bit 2 the LDS-DMA of tiles 1.. (the LDS keeps tile 0), each skipped part's inputs kept live.
// (A variant that retired the LDS reads after the slot barrier, with the DMA one phase later, measured
// 2-8 % slower on the encoder shapes and was dropped.)
template <int KIND, int ABL = 0, bool EARLY = true>
__global__ __launch_bounds__(512, 1) void gemm_8p_kernel(GemmA a, const bf16* __restrict__ w, long long ldw, int M,
                                                         int N, int K, GemmEpi epi, int tiles_n, int gm) {
  __shared__ __attribute__((aligned(16))) bf16 smem[P8_SMEM];
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  const int wgid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  // tile order: each XCD walks a contiguous wgid range.  gm = 0: row tiles in order, all column tiles of a
  // row tile together (A panel reused from L2, every W panel re-fetched per row tile).  gm > 0: groups of gm row
  // tiles walked column by column, so ~32 co-resident blocks of one XCD share gm A panels and 32 / gm W panels.
  int tm, tn;
  if (gm > 0) {
    const int per = gm * tiles_n, g = wgid / per, tiles_m = nwg / tiles_n;
    const int gsz = min(gm, tiles_m - g * gm), j = wgid - g * per;
    tm = g * gm + j % gsz;
    tn = j / gsz;
  } else {
    tm = wgid / tiles_n;
    tn = wgid - tm * tiles_n;
  }
  const int m0 = tm * P8_BM, n0 = tn * P8_BN;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 2, wn = wid & 3;
  const int fr = lane & 15, fq = lane >> 4;

  // DMA sources.  Quarter qq of a K-tile = A rows [0,128) | A rows [128,256) | W rows [0,128) | W rows [128,256);
  // wave `wid` moves rows [qq*128 + 16 wid, +16) of each quarter as two 8-row x 128-B wave-instructions.
  const bf16* src[4][2];
#pragma unroll
  for (int qq = 0; qq < 4; ++qq)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int row = (qq & 1) * 128 + wid * 16 + j * 8 + (lane >> 3);
      const int ch = (lane & 7) ^ ((row >> 1) & 7);
      if (qq < 2) {
        int gr = m0 + row;
        if (gr >= M) gr = M - 1;
        const long long off = a.rpb ? (long long)(gr / a.rpb) * a.bstride + (long long)(gr % a.rpb) * a.ld : (long long)gr * a.ld;
        src[qq][j] = a.ptr + off + ch * 8;
      } else {
        int gn = n0 + row;
        if (gn >= N) gn = N - 1;
        src[qq][j] = w + (long long)gn * ldw + ch * 8;
      }
    }
  auto dma = [&](int qq, int t) {
    if ((ABL & 4) && t > 0) return;
    bf16* dst = smem + (t & 1) * P8_BUF + (qq >> 1) * P8_TILE + ((qq & 1) * 128 + wid * 16) * P8_BK;
    const int k0 = t * P8_BK;
#pragma unroll
    for (int j = 0; j < 2; ++j)
      __builtin_amdgcn_global_load_lds((const void*)(src[qq][j] + k0),
                                       (__attribute__((address_space(3))) void*)(dst + j * 8 * P8_BK), 16, 0, 0);
  };

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = K / P8_BK;
#pragma unroll
  for (int qq = 0; qq < 4; ++qq) dma(qq, 0);
  if (EARLY && nk > 1) {
#pragma unroll
    for (int qq = 0; qq < 4; ++qq) dma(qq, 1);
    asm volatile("s_waitcnt vmcnt(8)\n\ts_barrier" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
  }
  if (wm == 1) asm volatile("s_barrier" ::: "memory");   // stagger: group 1 runs one barrier behind

  bf16x8 fa[4][2], fb[2][2], fb2[2][2];               // [frag][k-step]; fb2: W half 1 (EARLY schedule)
  auto read_a = [&](const bf16* sA, int half) {       // wave rows wm*128 + half*64 + 16 i
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
        fa[i][kk] = *(const bf16x8*)(sA + p8_swz(wm * 128 + half * 64 + i * 16 + fr, kk * 4 + fq));
  };
  auto read_b = [&](const bf16* sB, int half, bf16x8 (&dst)[2][2]) {   // wave cols wn*64 + half*32 + 16 j
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
        dst[j][kk] = *(const bf16x8*)(sB + p8_swz(wn * 64 + half * 32 + j * 16 + fr, kk * 4 + fq));
  };
  auto mfma_q = [&](int ha, int hb, const bf16x8 (&fb)[2][2]) {
    if (ABL & 2) {
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
#pragma unroll
        for (int i = 0; i < 4; ++i) asm volatile("" :: "v"(fa[i][kk]));
#pragma unroll
        for (int j = 0; j < 2; ++j) asm volatile("" :: "v"(fb[j][kk]));
      }
      return;
    }
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[ha * 4 + i][hb * 2 + j] =
              __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[j][kk], fa[i][kk], acc[ha * 4 + i][hb * 2 + j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };
  // end of a read slot: this wave's LDS reads retired, then the barrier; MFMAs stay below it
#define P8_READ_DONE()                                          \
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); \
  __builtin_amdgcn_sched_barrier(0);
#define P8_MFMA_DONE()                                          \
  __builtin_amdgcn_sched_barrier(0);                            \
  asm volatile("s_barrier" ::: "memory");

  for (int t = 0; t < nk; ++t) {
    const bf16* sA = smem + (t & 1) * P8_BUF;
    const bf16* sB = sA + P8_TILE;
    if (EARLY) {
      // Both W halves stay in registers (fb, fb2), so W is read in phases 0-1 and A in phases 0 and 2:
      // the W region of this buffer is free from phase 2 and the A region from phase 3, and tile t+2 is
      // DMA'd into them there (its readers are >= 4 phases away).  The wait in phase 3 leaves exactly those
      // 8 DMAs in flight and retires tile t+1's (issued in phases 2-3 of tile t-1).
      const bool more2 = t + 2 < nk;
      read_b(sB, 0, fb);                                // phase 0: Q00
      read_a(sA, 0);
      P8_READ_DONE();
      mfma_q(0, 0, fb);
      P8_MFMA_DONE();
      read_b(sB, 1, fb2);                               // phase 1: Q01
      P8_READ_DONE();
      mfma_q(0, 1, fb2);
      P8_MFMA_DONE();
      read_a(sA, 1);                                    // phase 2: Q11 + W of tile t+2
      if (more2) { dma(2, t + 2); dma(3, t + 2); }
      P8_READ_DONE();
      mfma_q(1, 1, fb2);
      P8_MFMA_DONE();
      if (more2) {                                      // phase 3: Q10 + A of tile t+2
        dma(0, t + 2);
        dma(1, t + 2);
        asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      P8_READ_DONE();
      mfma_q(1, 0, fb);
      P8_MFMA_DONE();
      continue;
    }
    const bool more = t + 1 < nk;
    // phase 0: Q00 (A half 0, W half 0) + DMA quarters 0, 1 of tile t+1
    read_b(sB, 0, fb);
    read_a(sA, 0);
    if (more) { dma(0, t + 1); dma(1, t + 1); }
    P8_READ_DONE();
    mfma_q(0, 0, fb);
    P8_MFMA_DONE();
    // phase 1: Q01 (W half 1) + DMA quarters 2, 3
    read_b(sB, 1, fb);
    if (more) { dma(2, t + 1); dma(3, t + 1); }
    P8_READ_DONE();
    mfma_q(0, 1, fb);
    P8_MFMA_DONE();
    // phase 2: Q11 (A half 1)
    read_a(sA, 1);
    P8_READ_DONE();
    mfma_q(1, 1, fb);
    P8_MFMA_DONE();
    // phase 3: Q10 (W half 0); tile t+1 has landed (this wave's share) before this read slot ends
    read_b(sB, 0, fb);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    P8_READ_DONE();
    mfma_q(1, 0, fb);
    P8_MFMA_DONE();
  }
  if (wm == 0) asm volatile("s_barrier" ::: "memory");   // balance the stagger
#undef P8_READ_DONE
#undef P8_MFMA_DONE

  if (ABL & 1) {
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) asm volatile("" :: "v"(acc[i][j]));
    return;
  }
  // acc[i][j] holds C^T: lane l has row m = m0 + wm*128 + 16 i + (l & 15), columns n = ... + 4 (l >> 4) + e.
  // Staged epilogue: the tile goes through LDS (free once the balancing barrier above has passed: every
  // wave's last reads retired before it, and the last tile issues no DMA) and leaves as whole 512-B (bf16)
  // or 1-KiB (f32) row segments, 16 B per lane, instead of 16 rows x 8-16 B per store instruction.
  constexpr bool BF16_OUT = KIND == EPI_BF16 || KIND == EPI_CROSS_KV;
  constexpr bool F32_OUT = KIND == EPI_RESID_F32 || KIND == EPI_F32 || KIND == EPI_GELU_POS_F32;
  if (BF16_OUT && N % 8 == 0 && epi.ldc % 8 == 0 && (epi.rpb == 0 || epi.bstride % 8 == 0 || KIND == EPI_CROSS_KV)) {
    // this lane's 4 bias chunks (one per column fragment j), requested together and waited once: epi_value4 loaded
    // the chunk for each of the 32 fragments and waited for it (32 dependent L2 round trips per tile epilogue)
    f32x4 bj[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int col0 = min(n0 + wn * 64 + j * 16 + 4 * fq, N - 4);
      bj[j] = epi.bias ? *(const f32x4*)(epi.bias + col0) : f32x4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) asm volatile("" : "+v"(bj[j]));
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int rl = wm * 128 + i * 16 + fr;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int cl = wn * 64 + j * 16 + 4 * fq;
        const int col0 = min(n0 + cl, N - 4);
        const f32x4 v = epi_value4_pre<KIND>(epi, m0 + rl, col0, acc[i][j], bj[j]);
        bf16x4 o;
#pragma unroll
        for (int e = 0; e < 4; ++e) o[e] = f2bf(v[e]);
        *(bf16x4*)(smem + rl * P8_SR16 + cl) = o;
      }
    }
    __syncthreads();
#pragma unroll 4
    for (int k = 0; k < 16; ++k) {
      const int c = tid + 512 * k, rl = c >> 5, cc = (c & 31) * 8;
      const int row = m0 + rl, col0 = n0 + cc;
      if (row < M && col0 < N) epi_store8_bf16<KIND>(epi, row, col0, *(const bf16x8*)(smem + rl * P8_SR16 + cc));
    }
    return;
  }
  if (F32_OUT && epi.ldc % 4 == 0) {
    float* sf = (float*)smem;
    // RESID_F32 / F32: the bias is added in the store loop, where a thread's column is the same for every k and
    // both halves (c & 63 = tid & 63): one chunk, requested here, instead of loads between the staging writes
    // (half 1's waited for half 0's store acknowledgements: vmcnt counts stores).  v = acc + b as epi_value4.
    constexpr bool BIAS_AT_STORE = KIND == EPI_RESID_F32 || KIND == EPI_F32;
    f32x4 bS = f32x4{0.f, 0.f, 0.f, 0.f};
    if (BIAS_AT_STORE && epi.bias) bS = *(const f32x4*)(epi.bias + min(n0 + (tid & 63) * 4, N - 4));
#pragma unroll
    for (int half = 0; half < 2; ++half) {
      // RESID_F32: this thread's 16 residual chunks of the half are loaded before the staging (one memory round
      // trip, overlapping the LDS writes and the barrier) instead of four dependent batches in the store loop;
      // the accumulators of half 0 are dead by then, so the 64 registers are free
      f32x4 res[16];
      if (KIND == EPI_RESID_F32) {
#pragma unroll
        for (int k = 0; k < 16; ++k) {
          const int c = tid + 512 * k, rl = c >> 6, cc = (c & 63) * 4;
          const int row = min(m0 + half * 128 + rl, M - 1), col0 = min(n0 + cc, N - 4);
          res[k] = *(const f32x4*)((const float*)epi.out + (long long)row * epi.ldc + col0);
        }
      }
      if (wm == half) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int cl = wn * 64 + j * 16 + 4 * fq;
          const int col0 = min(n0 + cl, N - 4);
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            const int rl = i * 16 + fr;
            *(f32x4*)(sf + rl * P8_SR32 + cl) =
                BIAS_AT_STORE ? acc[i][j] : epi_value4<KIND>(epi, m0 + half * 128 + rl, col0, acc[i][j]);
          }
        }
      }
      __syncthreads();
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        const int c = tid + 512 * k, rl = c >> 6, cc = (c & 63) * 4;
        const int row = m0 + half * 128 + rl, col0 = n0 + cc;
        if (row < M && col0 < N) {
          f32x4 v = *(const f32x4*)(sf + rl * P8_SR32 + cc);
          if (BIAS_AT_STORE && epi.bias) v += bS;
          if (KIND == EPI_RESID_F32) *(f32x4*)((float*)epi.out + (long long)row * epi.ldc + col0) = res[k] + v;
          else epi_store4_f32<KIND>(epi, row, col0, v);
        }
      }
      __syncthreads();
    }
    return;
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int row = m0 + wm * 128 + i * 16 + fr;
    if (row >= M) continue;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int col0 = n0 + wn * 64 + j * 16 + 4 * fq;
      if (col0 < N) apply_epi4<KIND>(epi, row, col0, acc[i][j]);
    }
  }
}

// ------------------------------------------------------------------------------------------------------
// Persistent form (opt-in, gemm_persistent; large GEMMs with contiguous A): one block per CU walks a sequence of
// output tiles.  The K-step stream runs on across tile seams: in the last two K-steps of a tile, the slots that
// would prefetch K-tiles t+2 instead take the NEXT tile's K-tiles 0 and 1 (same buffers, same phases, same
// counted waits as inside a tile), so a new tile starts with its operands already in LDS instead of paying a
// DMA round trip.  The epilogue stages through a 32 KiB region beside the two 64 KiB operand buffers (64-row
// passes for bf16, 32-row passes for f32, 16-B chunks XOR-swizzled by row & 15: conflict-free for the fragment
// writes and the whole-row reads), so it runs while the next tile's operands land, and its stores drain behind
// the next tile's first K-step (the counted vmcnt there retires them with the K-tile-1 DMA).  RESID_F32 loads
// the residual of pass p + 1 while pass p is stored.  Every output's arithmetic is the non-persistent kernel's.
#define PP_STAGE (2 * P8_BUF)                      // bf16-element offset of the staging region (128 KiB)
#define PP_SMEM (PP_STAGE + 16384)                 // + 32 KiB = 160 KiB

template <int KIND>
__global__ __launch_bounds__(512, 1) void gemm_8pp_kernel(GemmA a, const bf16* __restrict__ w, long long ldw, int M,
                                                          int N, int K, GemmEpi epi, int tiles_n, int n_tiles) {
  __shared__ __attribute__((aligned(16))) bf16 smem[PP_SMEM];
  const int bid = blockIdx.x, npx = gridDim.x >> 3;
  const int xcd = bid & 7, jb = bid >> 3;
  // this XCD's contiguous tile range (row tiles in order, all column tiles of a row tile together), walked by
  // the XCD's npx blocks in lockstep rounds: co-resident blocks share A panels in the XCD's L2
  const int q = n_tiles >> 3, r8 = n_tiles & 7;
  const int start = xcd < r8 ? xcd * (q + 1) : r8 * (q + 1) + (xcd - r8) * q;
  const int size = q + (xcd < r8 ? 1 : 0);
  const int cnt = jb < size ? (size - jb + npx - 1) / npx : 0;
  if (cnt == 0) return;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 2, wn = wid & 3;
  const int fr = lane & 15, fq = lane >> 4;
  const int nk = K / P8_BK;

  // DMA sources of the tile being streamed: uniform 64-bit bases (scalar registers) + per-lane 32-bit offsets
  // (rows clamped to the matrix), switched to the next tile once, when the K-step stream crosses the seam.
  // quarter qq of K-tile kt -> buffer buf: the same row/chunk mapping as gemm_8p_kernel.
  const bf16* baseA = a.ptr;
  const bf16* baseW = w;
  int offA[2][2], offW[2][2];
  auto set_src = [&](int tm0, int tn0) {
    int lo = lane;
    asm volatile("" : "+v"(lo));
    baseA = a.ptr + (long long)tm0 * a.ld;
    baseW = w + (long long)tn0 * ldw;
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int row = h * 128 + wid * 16 + j * 8 + (lo >> 3);
        const int ch = (lo & 7) ^ ((row >> 1) & 7);
        offA[h][j] = (min(tm0 + row, M - 1) - tm0) * (int)a.ld + ch * 8;
        offW[h][j] = (min(tn0 + row, N - 1) - tn0) * (int)ldw + ch * 8;
      }
  };
  auto dma = [&](int qq, int kt, int buf) {
    bf16* dst = smem + buf * P8_BUF + (qq >> 1) * P8_TILE + ((qq & 1) * 128 + wid * 16) * P8_BK;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const bf16* src = (qq < 2 ? baseA + offA[qq & 1][j] : baseW + offW[qq & 1][j]) + kt * P8_BK;
      __builtin_amdgcn_global_load_lds((const void*)src, (__attribute__((address_space(3))) void*)(dst + j * 8 * P8_BK), 16,
                                       0, 0);
    }
  };
  auto tile_mn = [&](int i, int& m0, int& n0) {
    const int t = start + jb + npx * i;
    const int tm = t / tiles_n;
    m0 = tm * P8_BM;
    n0 = (t - tm * tiles_n) * P8_BN;
  };

  int m0, n0;
  tile_mn(0, m0, n0);
  set_src(m0, n0);
#pragma unroll
  for (int qq = 0; qq < 4; ++qq) dma(qq, 0, 0);
  if (nk > 1) {
#pragma unroll
    for (int qq = 0; qq < 4; ++qq) dma(qq, 1, 1);
    asm volatile("s_waitcnt vmcnt(8)\n\ts_barrier" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
  }
  int g = 0;                                        // K-steps done by this block (buffer parity)
  for (int i = 0; i < cnt; ++i) {
    if (i > 0) tile_mn(i, m0, n0);
    int m1 = 0, n1 = 0;
    const bool has_next = i + 1 < cnt;
    if (has_next) tile_mn(i + 1, m1, n1);
    if (wm == 1) asm volatile("s_barrier" ::: "memory");   // stagger: group 1 runs one barrier behind
    f32x4 acc[8][4];
#pragma unroll
    for (int ii = 0; ii < 8; ++ii)
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) acc[ii][jj] = f32x4{0.f, 0.f, 0.f, 0.f};
    bf16x8 fa[4][2], fb[2][2], fb2[2][2];
    auto read_a = [&](const bf16* sA, int half) {
#pragma unroll
      for (int ii = 0; ii < 4; ++ii)
#pragma unroll
        for (int kk = 0; kk < 2; ++kk)
          fa[ii][kk] = *(const bf16x8*)(sA + p8_swz(wm * 128 + half * 64 + ii * 16 + fr, kk * 4 + fq));
    };
    auto read_b = [&](const bf16* sB, int half, bf16x8 (&dst)[2][2]) {
#pragma unroll
      for (int jj = 0; jj < 2; ++jj)
#pragma unroll
        for (int kk = 0; kk < 2; ++kk)
          dst[jj][kk] = *(const bf16x8*)(sB + p8_swz(wn * 64 + half * 32 + jj * 16 + fr, kk * 4 + fq));
    };
    auto mfma_q = [&](int ha, int hb, const bf16x8 (&fbx)[2][2]) {
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int ii = 0; ii < 4; ++ii)
#pragma unroll
          for (int jj = 0; jj < 2; ++jj)
            acc[ha * 4 + ii][hb * 2 + jj] =
                __builtin_amdgcn_mfma_f32_16x16x32_bf16(fbx[jj][kk], fa[ii][kk], acc[ha * 4 + ii][hb * 2 + jj], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
    };
#define PP_READ_DONE()                                          \
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); \
  __builtin_amdgcn_sched_barrier(0);
#define PP_MFMA_DONE()                                          \
  __builtin_amdgcn_sched_barrier(0);                            \
  asm volatile("s_barrier" ::: "memory");
    for (int t = 0; t < nk; ++t, ++g) {
      const bf16* sA = smem + (g & 1) * P8_BUF;
      const bf16* sB = sA + P8_TILE;
      // the K-tile two steps ahead: this tile's t + 2, else the next tile's t + 2 - nk (0 or 1)
      const bool in_tile = t + 2 < nk;
      const bool more2 = in_tile || has_next;
      const int tk = in_tile ? t + 2 : t + 2 - nk;
      if (t + 2 == nk && has_next) set_src(m1, n1);     // the stream crosses into the next tile
      read_b(sB, 0, fb);                                // phase 0: Q00
      read_a(sA, 0);
      PP_READ_DONE();
      mfma_q(0, 0, fb);
      PP_MFMA_DONE();
      read_b(sB, 1, fb2);                               // phase 1: Q01
      PP_READ_DONE();
      mfma_q(0, 1, fb2);
      PP_MFMA_DONE();
      read_a(sA, 1);                                    // phase 2: Q11 + W of the K-tile two steps ahead
      if (more2) { dma(2, tk, g & 1); dma(3, tk, g & 1); }
      PP_READ_DONE();
      mfma_q(1, 1, fb2);
      PP_MFMA_DONE();
      if (more2) {                                      // phase 3: Q10 + its A
        dma(0, tk, g & 1);
        dma(1, tk, g & 1);
        asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      PP_READ_DONE();
      mfma_q(1, 0, fb);
      PP_MFMA_DONE();
    }
#undef PP_READ_DONE
#undef PP_MFMA_DONE
    if (wm == 0) asm volatile("s_barrier" ::: "memory");   // balance the stagger

    // ---- epilogue: raw f32 accumulators staged 32 rows at a time through the 32 KiB region; the bias (and
    // GELU, and the residual) are applied on the store side, where each thread's output columns are the same in
    // every pass, so the bias is loaded once per tile and no load sits between one pass's stores and the next
    // (a load there would wait for those stores: vmcnt counts them).  Same f32 arithmetic as epi_value4.
    char* stg = (char*)(smem + PP_STAGE);
    constexpr bool BF16_OUT = KIND == EPI_BF16;
    const int cq = BF16_OUT ? (tid & 31) * 8 : (tid & 63) * 4;      // this thread's first output column
    f32x4 bias0 = f32x4{0.f, 0.f, 0.f, 0.f}, bias1 = bias0;
    if (epi.bias) {
      bias0 = *(const f32x4*)(epi.bias + min(n0 + cq, N - 4));
      if (BF16_OUT) bias1 = *(const f32x4*)(epi.bias + min(n0 + cq + 4, N - 4));
    }
    f32x4 rn[4];                                        // RESID_F32: the next pass's residual chunks
    auto load_res = [&](int p, f32x4 (&dst)[4]) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int row = min(m0 + p * 32 + (tid >> 6) + 8 * k, M - 1), col0 = min(n0 + cq, N - 4);
        dst[k] = *(const f32x4*)((const float*)epi.out + (long long)row * epi.ldc + col0);
      }
    };
    if (KIND == EPI_RESID_F32) load_res(0, rn);
#pragma unroll
    for (int p = 0; p < 8; ++p) {                       // rows [32 p, 32 p + 32): wave group p >> 2, fragments 2 (p & 3) ..
      f32x4 rc[4];
      if (KIND == EPI_RESID_F32) {
#pragma unroll
        for (int k = 0; k < 4; ++k) rc[k] = rn[k];
        if (p + 1 < 8) load_res(p + 1, rn);
      }
      if (wm == (p >> 2)) {
#pragma unroll
        for (int ii = 0; ii < 2; ++ii) {
          const int rl = ii * 16 + fr;
#pragma unroll
          for (int jj = 0; jj < 4; ++jj) {
            const int cl = wn * 64 + jj * 16 + 4 * fq;
            *(f32x4*)(stg + rl * 1024 + (((cl >> 2) ^ (rl & 15)) << 4)) = acc[(p & 3) * 2 + ii][jj];
          }
        }
      }
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");   // LDS only: no vmcnt(0)
      if (BF16_OUT) {
#pragma unroll
        for (int k = 0; k < 2; ++k) {
          const int rl = (tid >> 5) + 16 * k, row = m0 + p * 32 + rl, col0 = n0 + cq;
          const int c4 = cq >> 2;                       // first of the two f32 chunks
          f32x4 v0 = *(const f32x4*)(stg + rl * 1024 + ((c4 ^ (rl & 15)) << 4)) + bias0;
          f32x4 v1 = *(const f32x4*)(stg + rl * 1024 + (((c4 + 1) ^ (rl & 15)) << 4)) + bias1;
          if (epi.act == 1) {
#pragma unroll
            for (int e = 0; e < 4; ++e) { v0[e] = gelu_erf(v0[e]); v1[e] = gelu_erf(v1[e]); }
          }
          bf16x8 o;
#pragma unroll
          for (int e = 0; e < 4; ++e) { o[e] = f2bf(v0[e]); o[4 + e] = f2bf(v1[e]); }
          if (row < M && col0 < N) epi_store8_bf16<KIND>(epi, row, col0, o);
        }
      } else {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int rl = (tid >> 6) + 8 * k, row = m0 + p * 32 + rl, col0 = n0 + cq;
          const f32x4 v = *(const f32x4*)(stg + rl * 1024 + (((cq >> 2) ^ (rl & 15)) << 4)) + bias0;
          if (row < M && col0 < N) {
            if (KIND == EPI_RESID_F32) *(f32x4*)((float*)epi.out + (long long)row * epi.ldc + col0) = rc[k] + v;
            else *(f32x4*)((float*)epi.out + (long long)row * epi.ldc + col0) = v;
          }
        }
      }
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    }
  }
}

// Process-wide (the GEMM launchers carry no engine): VLOG_AMD_GEMM_PERSIST=1 or wm_set_option("gemm_persistent", 1)
// selects the persistent kernel.  Bit-identical either way.  Off by default: measured equal in bench.py (encoder
// GEMM 296.9-298.7 vs 296.1-296.2 ms per step) and 3-7 % slower in tools/gemm_bench on the 16-window shapes, so
// a tile's fixed cost is not its prologue round trip (profiles/ab_r02_persist.txt).
static int g_gemm_persist = [] {
  const char* e = std::getenv("VLOG_AMD_GEMM_PERSIST");
  return e ? std::atoi(e) : 0;
}();
static int gemm_8p_persistent() { return g_gemm_persist; }
void gemm_8p_set_persistent(int on) { g_gemm_persist = on != 0; }
int gemm_8p_get_persistent() { return g_gemm_persist; }

static int device_cus() {
  static const int v = [] {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      return 256;
    return n > 0 ? n : 256;
  }();
  return v;
}

// Row tiles per group of the tile order (VLOG_AMD_GEMM_GROUP; 0 = row-major order).  Schedule only: every tile's
// arithmetic is the same in any order.
static int gemm_8p_group() {
  static const int v = [] {
    const char* e = std::getenv("VLOG_AMD_GEMM_GROUP");
    return e ? std::max(0, std::atoi(e)) : 0;
  }();
  return v;
}

template <int KIND>
static void run_8p(const GemmA& a, const bf16* w, long long ldw, int M, int N, int K, const GemmEpi& epi, hipStream_t st) {
  {
    constexpr bool PK = KIND == EPI_BF16 || KIND == EPI_RESID_F32 || KIND == EPI_F32;
    const int tiles_m = (M + P8_BM - 1) / P8_BM, tiles_n = (N + P8_BN - 1) / P8_BN;
    const int n_tiles = tiles_m * tiles_n, cus = device_cus();
    const bool out_ok = KIND == EPI_BF16 ? (N % 8 == 0 && epi.ldc % 8 == 0 && (epi.rpb == 0 || epi.bstride % 8 == 0))
                                         : epi.ldc % 4 == 0;
    if (PK && gemm_8p_persistent() && a.rpb == 0 && out_ok && cus % 8 == 0 && n_tiles >= 2 * cus && K >= 2 * P8_BK && gemm_8p_group() == 0) {
      hipLaunchKernelGGL((gemm_8pp_kernel<KIND>), dim3(cus), dim3(512), 0, st, a, w, ldw, M, N, K, epi, tiles_n, n_tiles);
      WM_LAUNCH_CHECK("gemm_8pp_kernel");
      return;
    }
  }
  static const bool early = [] {
    const char* e = std::getenv("VLOG_AMD_GEMM_8P");
    return !(e && e[0] == '2');
  }();
  const int tiles_m = (M + P8_BM - 1) / P8_BM, tiles_n = (N + P8_BN - 1) / P8_BN;
  const int gm = gemm_8p_group();
  if (early)
    hipLaunchKernelGGL((gemm_8p_kernel<KIND, 0, true>), dim3(tiles_m * tiles_n), dim3(512), 0, st, a, w, ldw, M, N, K, epi, tiles_n, gm);
  else
    hipLaunchKernelGGL((gemm_8p_kernel<KIND, 0, false>), dim3(tiles_m * tiles_n), dim3(512), 0, st, a, w, ldw, M, N, K, epi, tiles_n, gm);
  WM_LAUNCH_CHECK("gemm_8p_kernel");
}

bool gemm_8p_applicable(int M, int N, int K) { return M >= 1024 && N >= 256 && N % 4 == 0 && K % P8_BK == 0 && K >= P8_BK; }

void launch_gemm_8p(const GemmA& a, const bf16* w, long long ldw, int M, int N, int K, const GemmEpi& epi, hipStream_t st) {
  switch (epi.kind) {
    case EPI_BF16: run_8p<EPI_BF16>(a, w, ldw, M, N, K, epi, st); break;
    case EPI_RESID_F32: run_8p<EPI_RESID_F32>(a, w, ldw, M, N, K, epi, st); break;
    case EPI_GELU_POS_F32: run_8p<EPI_GELU_POS_F32>(a, w, ldw, M, N, K, epi, st); break;
    case EPI_F32: run_8p<EPI_F32>(a, w, ldw, M, N, K, epi, st); break;
    case EPI_DEC_QKV: run_8p<EPI_DEC_QKV>(a, w, ldw, M, N, K, epi, st); break;
    case EPI_CROSS_KV: run_8p<EPI_CROSS_KV>(a, w, ldw, M, N, K, epi, st); break;
    default: throw std::runtime_error("launch_gemm_8p: bad epilogue kind");
  }
}

// microbenchmark entry (tools/gemm_bench): EPI_BF16 body with ablation bits
void launch_gemm_8p_abl(const GemmA& a, const bf16* w, long long ldw, int M, int N, int K, const GemmEpi& epi, int abl,
                        hipStream_t st) {
  const int tiles_m = (M + P8_BM - 1) / P8_BM, tiles_n = (N + P8_BN - 1) / P8_BN;
  const dim3 g(tiles_m * tiles_n);
  switch (abl) {
    case 0: hipLaunchKernelGGL((gemm_8p_kernel<EPI_BF16, 0>), g, dim3(512), 0, st, a, w, ldw, M, N, K, epi, tiles_n, gemm_8p_group()); break;
    case 1: hipLaunchKernelGGL((gemm_8p_kernel<EPI_BF16, 1>), g, dim3(512), 0, st, a, w, ldw, M, N, K, epi, tiles_n, gemm_8p_group()); break;
    case 2: hipLaunchKernelGGL((gemm_8p_kernel<EPI_BF16, 2>), g, dim3(512), 0, st, a, w, ldw, M, N, K, epi, tiles_n, gemm_8p_group()); break;
    case 3: hipLaunchKernelGGL((gemm_8p_kernel<EPI_BF16, 3>), g, dim3(512), 0, st, a, w, ldw, M, N, K, epi, tiles_n, gemm_8p_group()); break;
    case 4: hipLaunchKernelGGL((gemm_8p_kernel<EPI_BF16, 4>), g, dim3(512), 0, st, a, w, ldw, M, N, K, epi, tiles_n, gemm_8p_group()); break;
    case 5: hipLaunchKernelGGL((gemm_8p_kernel<EPI_BF16, 5>), g, dim3(512), 0, st, a, w, ldw, M, N, K, epi, tiles_n, gemm_8p_group()); break;
    case 7: hipLaunchKernelGGL((gemm_8p_kernel<EPI_BF16, 7>), g, dim3(512), 0, st, a, w, ldw, M, N, K, epi, tiles_n, gemm_8p_group()); break;
    default: throw std::runtime_error("launch_gemm_8p_abl: bad ablation");
  }
}
