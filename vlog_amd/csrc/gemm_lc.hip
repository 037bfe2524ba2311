// Loader/consumer ring GEMM for decoder passes (gfx950): C = A . W^T over BM rows x BN columns per workgroup, the
// operand panels streamed through an LDS ring by DEDICATED loader waves (the guide's ring-gemm structure,
// MI355X_MICROARCH.md 'ring-gemm').
//
// Why: the ring of gemm_dec.hip (dec_ring_kernel) has every wave both issue its share of a sub-panel's LDS-DMA and
// run its MFMAs, with one workgroup barrier per sub-panel, so the next panels are requested only after the slowest
// wave reached the barrier; at beam-group row counts it takes in 30-50 GB/s per CU in the decode step
// (profiles/dgb_r06_*.txt).  Here 4 loader waves only issue LDS-DMA and 4 consumer waves only read fragments and run
// MFMAs; they meet through per-slot counters in LDS instead of barriers:
//   full[s]: every loader adds 1 once ITS LDS-DMA of the slot's current K-step has landed (counted vmcnt);
//            a consumer reads the slot for generation g once full[s] >= 4 (g + 1);
//   free[s]: every consumer adds 1 once its fragment reads of the slot returned (lgkmcnt(0)), before its MFMAs;
//            a loader refills the slot for generation g once free[s] >= 4 g.
// A slot holds one 64-deep K-step of both panels ((BM + BN) x 128 B), in the dec_ring layout (128-B rows, 16-B chunk
// c of row r at chunk c ^ ((r >> 1) & 7), applied on the DMA source address), NSLOT slots, D K-steps in flight per
// loader beyond the one being issued.  Every output's K order is the ring's (64-deep steps in order, two MFMA k-steps
// of 32 each), so results are bit-identical to dec_ring_kernel for the same K range.
// Counter polls and adds are inline-asm LDS ops (the compiler would otherwise drain the loader's DMA queue with
// vmcnt(0) before an LDS read it cannot prove independent of the pending LDS-DMA writes); every spin is bounded.
#include "gemm.h"
#include "gemm_epi.h"
#include <stdexcept>
#include <string>

__device__ __forceinline__ int lc_swz(int row, int ch) { return row * 64 + ((ch ^ ((row >> 1) & 7)) << 3); }

__device__ __forceinline__ unsigned lc_poll(unsigned addr) {
  unsigned v;
  asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(addr) : "memory");
  return v;
}
__device__ __forceinline__ void lc_add1(unsigned addr) {
  const unsigned one = 1;
  asm volatile("ds_add_u32 %0, %1" ::"v"(addr), "v"(one) : "memory");
}
// wait until the counter reaches target (bounded: ~1 s; a miss gives wrong results, never a hang)
__device__ __forceinline__ void lc_wait(unsigned addr, unsigned target) {
  for (int it = 0; it < (1 << 23); ++it) {
    if (lc_poll(addr) >= target) return;
    __builtin_amdgcn_s_sleep(1);
  }
}
__device__ __forceinline__ void lc_vm_wait(int n) {
  switch (n) {
#define LVW(k) case k: asm volatile("s_waitcnt vmcnt(" #k ")" ::: "memory"); break;
    LVW(0) LVW(1) LVW(2) LVW(3) LVW(4) LVW(5) LVW(6) LVW(7) LVW(8) LVW(9) LVW(10) LVW(11) LVW(12) LVW(13) LVW(14)
    LVW(15) LVW(16) LVW(17) LVW(18) LVW(19) LVW(20) LVW(21) LVW(22) LVW(23) LVW(24) LVW(25) LVW(26) LVW(27)
    LVW(28) LVW(29) LVW(30) LVW(31) LVW(32) LVW(33) LVW(34) LVW(35) LVW(36) LVW(37) LVW(38) LVW(39) LVW(40)
#undef LVW
    default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
  }
}

// BM rows (consumer waves 2 x 2: BM/2 rows x BN/2 columns each), BN columns, NSLOT ring slots, D steps in flight.
// WBLK: W stored panel-blocked, [N / BN][K / 64][BN][64] (every (column tile, K-step) piece one contiguous (BN x 128 B)
// run) instead of row-major [N][K] (the piece is BN row segments of 128 B at the K stride).
template <int BM, int BN, int NSLOT, int D, int KIND, bool WBLK = false>
__global__ __launch_bounds__(512, 1) void dec_lc_kernel(GemmA a, const bf16* __restrict__ w, long long ldw, int M, int N,
                                                        int K, GemmEpi epi, int splitk, int kr, float* __restrict__ part,
                                                        int rgroups) {
  constexpr int MFI = BM / 32, NFC = BN / 32;             // 16-row / 16-column fragments per consumer wave
  constexpr int SUB = (BM + BN) * 64;                     // elements of one slot
  constexpr int DA = BM / 32, DW = BN / 32;               // DMA instructions (8 rows x 128 B) per loader per step
  constexpr int DPS = DA + DW;
  static_assert(BM % 32 == 0 && BN % 32 == 0 && D >= 1 && D < NSLOT, "tile / ring");
  static_assert(DPS * (D - 1) <= 40, "vmcnt table");
  __shared__ __attribute__((aligned(16))) bf16 smem[NSLOT * SUB + 2 * NSLOT * 2];   // ring + full[] + free[] (u32)
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  const int wgid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  const int split = wgid % splitk, rg = (wgid / splitk) % rgroups, tile = wgid / (splitk * rgroups);
  const int n0 = tile * BN, m0 = rg * BM;
  const int kb = split * kr, klen = min(kr, K - kb), NS = klen / 64;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  unsigned* cnt = (unsigned*)(smem + NSLOT * SUB);        // full[NSLOT], free[NSLOT]
  const unsigned full0 = (unsigned)(uintptr_t)(__attribute__((address_space(3))) void*)cnt;
  if (tid < 2 * NSLOT) cnt[tid] = 0;
  __syncthreads();

  if (wv >= 4) {
    // ---------------- loader wave lw: A rows [lw BM/4, +BM/4), W rows [lw BN/4, +BN/4) of every step
    const int lw = wv - 4;
    const bf16* srcA[DA];
    const bf16* srcW[DW];
#pragma unroll
    for (int j = 0; j < DA; ++j) {
      const int row = lw * (BM / 4) + j * 8 + (lane >> 3);
      const int ch = (lane & 7) ^ ((row >> 1) & 7);
      const int gr = min(m0 + row, M - 1);
      const long long off = a.rpb ? (long long)(gr / a.rpb) * a.bstride + (long long)(gr % a.rpb) * a.ld : (long long)gr * a.ld;
      srcA[j] = a.ptr + off + kb + ch * 8;
    }
#pragma unroll
    for (int j = 0; j < DW; ++j) {
      const int row = lw * (BN / 4) + j * 8 + (lane >> 3);
      const int ch = (lane & 7) ^ ((row >> 1) & 7);
      if constexpr (WBLK) srcW[j] = w + (((long long)tile * (K / 64) + kb / 64) * BN + row) * 64 + ch * 8;
      else srcW[j] = w + (long long)min(n0 + row, N - 1) * ldw + kb + ch * 8;
    }
    constexpr int WSTEP = WBLK ? BN * 64 : 64;             // elements between consecutive K-steps of a W row piece
    for (int p = 0; p < NS; ++p) {
      const int s = p % NSLOT;
      if (p >= NSLOT) lc_wait(full0 + 4 * (NSLOT + s), 4u * (unsigned)(p / NSLOT));
      bf16* dst = smem + s * SUB;
#pragma unroll
      for (int j = 0; j < DA; ++j)
        __builtin_amdgcn_global_load_lds((const void*)(srcA[j] + p * 64),
                                         (__attribute__((address_space(3))) void*)(dst + (lw * (BM / 4) + j * 8) * 64), 16, 0, 0);
#pragma unroll
      for (int j = 0; j < DW; ++j)
        __builtin_amdgcn_global_load_lds((const void*)(srcW[j] + (long long)p * WSTEP),
                                         (__attribute__((address_space(3))) void*)(dst + (BM + lw * (BN / 4) + j * 8) * 64), 16, 0, 0);
      if (p >= D - 1) {                                    // step p - (D - 1) has landed for this wave
        lc_vm_wait(DPS * (D - 1));
        if (lane == 0) lc_add1(full0 + 4 * ((p - (D - 1)) % NSLOT));
      }
    }
    for (int p = (NS > D - 1 ? NS - (D - 1) : 0); p < NS; ++p) {   // the last D - 1 steps
      lc_vm_wait(DPS * (NS - 1 - p));
      if (lane == 0) lc_add1(full0 + 4 * (p % NSLOT));
    }
    return;
  }

  // ---------------- consumer wave (wr, wc): rows wr BM/2 + 16 i, columns wc BN/2 + 16 c
  const int wc = wv & 1, wr = wv >> 1;
  f32x4 acc[NFC][MFI];
#pragma unroll
  for (int c = 0; c < NFC; ++c)
#pragma unroll
    for (int i = 0; i < MFI; ++i) acc[c][i] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int p = 0; p < NS; ++p) {
    const int s = p % NSLOT;
    lc_wait(full0 + 4 * s, 4u * (unsigned)(p / NSLOT + 1));
    const bf16* sA = smem + s * SUB;
    const bf16* sW = sA + BM * 64;
    bf16x8 fa[2][MFI], fb[2][NFC];
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int ch = kk * 4 + (lane >> 4);
#pragma unroll
      for (int c = 0; c < NFC; ++c) fb[kk][c] = *(const bf16x8*)(sW + lc_swz(wc * (BN / 2) + c * 16 + (lane & 15), ch));
#pragma unroll
      for (int i = 0; i < MFI; ++i) fa[kk][i] = *(const bf16x8*)(sA + lc_swz(wr * (BM / 2) + i * 16 + (lane & 15), ch));
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // this wave's reads of the slot returned
    if (lane == 0) lc_add1(full0 + 4 * (NSLOT + s));
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int c = 0; c < NFC; ++c)
#pragma unroll
        for (int i = 0; i < MFI; ++i) acc[c][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[kk][c], fa[kk][i], acc[c][i], 0, 0, 0);
  }

  // W fragment as the MFMA A operand: acc[c][i] holds C^T, lane l has row 16 i + (l & 15) and 4 consecutive columns
  const bool to_slab = splitk > 1 || KIND == EPI_RESID_LN;
#pragma unroll
  for (int c = 0; c < NFC; ++c) {
    const int col0 = n0 + wc * (BN / 2) + c * 16 + 4 * (lane >> 4);
#pragma unroll
    for (int i = 0; i < MFI; ++i) {
      const int row = m0 + wr * (BM / 2) + i * 16 + (lane & 15);
      if (col0 >= N || row >= M) continue;
      if (to_slab) *(f32x4*)(part + ((long long)split * M + row) * N + col0) = acc[c][i];
      else apply_epi4<KIND>(epi, row, col0, acc[c][i]);
    }
  }
}

void launch_splitk_combine(const float* part, int splitk, int M, int N, const GemmEpi& epi, hipStream_t st);

static bool g_lc_wblk = false;     // microbenchmark: W given panel-blocked (dec_lc_kernel WBLK)
void dec_lc_set_wblk(bool on) { g_lc_wblk = on; }

template <int BM, int BN, int KIND>
static void run_lc(const GemmA& a, const bf16* w, long long ldw, int M, int N, int K, const GemmEpi& epi, float* ws,
                   int splitk, int kr, hipStream_t st) {
  // 4 slots of 64-deep steps, 2 steps in flight per loader (the guide: a ring at least three slots deeper than the
  // steps in flight beyond the one issued: 1 issued + 2 published for the consumers)
  constexpr int NSLOT = (BM + BN) * 128 * 4 <= 150 * 1024 ? 4 : 3;
  constexpr int D = 2;
  const int tiles_n = (N + BN - 1) / BN, rgroups = (M + BM - 1) / BM;
  if (g_lc_wblk)
    hipLaunchKernelGGL((dec_lc_kernel<BM, BN, NSLOT, D, KIND, true>), dim3(tiles_n * rgroups * splitk), dim3(512), 0, st, a,
                       w, ldw, M, N, K, epi, splitk, kr, ws, rgroups);
  else
    hipLaunchKernelGGL((dec_lc_kernel<BM, BN, NSLOT, D, KIND>), dim3(tiles_n * rgroups * splitk), dim3(512), 0, st, a, w,
                       ldw, M, N, K, epi, splitk, kr, ws, rgroups);
  WM_LAUNCH_CHECK("dec_lc_kernel");
}

template <int KIND>
static bool dispatch_lc(const GemmA& a, const bf16* w, long long ldw, int M, int N, int K, const GemmEpi& epi, float* ws,
                        int splitk, int kr, int bm, int bn, hipStream_t st) {
#define LC_CASE(BMV, BNV) \
  if (bm == BMV && bn == BNV) { run_lc<BMV, BNV, KIND>(a, w, ldw, M, N, K, epi, ws, splitk, kr, st); return true; }
  LC_CASE(128, 128) LC_CASE(128, 64) LC_CASE(64, 128) LC_CASE(64, 64) LC_CASE(96, 32) LC_CASE(64, 32) LC_CASE(160, 32)
  LC_CASE(160, 64) LC_CASE(32, 64) LC_CASE(32, 32)
#undef LC_CASE
  return false;
}

// Loader/consumer ring path: K % 64 == 0, N % 4 == 0; kr = K range per block (0: the whole K), a multiple of 64.
// bm x bn: 128x128, 128x64, 64x128, 64x64, 96x32, 64x32, 160x32, 160x64, 32x64, 32x32.  Returns false when unsupported.
bool launch_dec_lc(const GemmA& a, const bf16* w, long long ldw, int M, int N, int K, const GemmEpi& epi, float* ws,
                   size_t ws_bytes, int kr, hipStream_t st, int bm, int bn) {
  if (M <= 0 || N % 4 != 0 || K % 64 != 0) return false;
  if (a.fold_stat || a.lnx || epi.xg_out || epi.stat_out) return false;
  if (kr <= 0 || kr > K) kr = K;
  if (kr % 64 != 0) return false;
  const int splitk = (K + kr - 1) / kr;
  const bool slab = splitk > 1 || epi.kind == EPI_RESID_LN;
  if (slab && (!ws || (size_t)splitk * M * N * 4 > ws_bytes)) return false;
  if (!slab && (epi.ldc % 4 != 0 || (epi.rpb != 0 && epi.bstride % 4 != 0))) return false;
  bool ok = false;
  switch (epi.kind) {
    case EPI_BF16: ok = dispatch_lc<EPI_BF16>(a, w, ldw, M, N, K, epi, ws, splitk, kr, bm, bn, st); break;
    case EPI_RESID_F32: ok = dispatch_lc<EPI_RESID_F32>(a, w, ldw, M, N, K, epi, ws, splitk, kr, bm, bn, st); break;
    case EPI_F32: ok = dispatch_lc<EPI_F32>(a, w, ldw, M, N, K, epi, ws, splitk, kr, bm, bn, st); break;
    case EPI_DEC_QKV: ok = dispatch_lc<EPI_DEC_QKV>(a, w, ldw, M, N, K, epi, ws, splitk, kr, bm, bn, st); break;
    case EPI_RESID_LN: ok = dispatch_lc<EPI_RESID_LN>(a, w, ldw, M, N, K, epi, ws, splitk, kr, bm, bn, st); break;
    default: return false;
  }
  if (!ok) return false;
  if (slab && !epi.defer_combine) launch_splitk_combine(ws, splitk, M, N, epi, st);
  return true;
}
