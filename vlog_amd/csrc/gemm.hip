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
#include <algorithm>
#include <stdexcept>
#include <string>

#define BK 64

__device__ __forceinline__ int swz(int row, int ch) { return row * BK + ((ch ^ ((row >> 1) & 7)) << 3); }

template <int KIND>
__device__ __forceinline__ void apply_epi(const GemmEpi& epi, int row, int col, float acc) {
  float v = acc + (epi.bias ? epi.bias[col] : 0.f);
  switch (KIND) {
    case EPI_BF16: {
      if (epi.act == 1) v = gelu_erf(v);
      long long o = epi.rpb ? (long long)(row / epi.rpb) * epi.bstride + (long long)(row % epi.rpb + epi.roff) * epi.ldc
                            : (long long)row * epi.ldc;
      ((bf16*)epi.out)[o + col] = f2bf(v);
      break;
    }
    case EPI_RESID_F32: {
      float* p = (float*)epi.out + (long long)row * epi.ldc + col;
      *p += v;
      break;
    }
    case EPI_GELU_POS_F32: {
      const int t = row % epi.rpb;
      ((float*)epi.out)[(long long)row * epi.ldc + col] = gelu_erf(v) + epi.pos[(long long)t * epi.ldc + col];
      break;
    }
    case EPI_F32: {
      ((float*)epi.out)[(long long)row * epi.ldc + col] = v;
      break;
    }
    case EPI_DEC_QKV: {
      const int d = epi.d;
      if (col < d) {
        ((bf16*)epi.out)[(long long)row * epi.ldc + col] = f2bf(v);
      } else {
        const int c2 = col - d;
        const int kv = c2 >= d;
        const int cc = kv ? c2 - d : c2;
        const int h = cc / epi.head_dim, e2 = cc - h * epi.head_dim;
        const long long slot = (((long long)epi.row_hyp[row] * epi.n_head + h) * epi.n_ctx + epi.row_pos[row]) * epi.head_dim + e2;
        (kv ? epi.vcache : epi.kcache)[slot] = f2bf(v);
      }
      break;
    }
    case EPI_CROSS_KV: {
      // col = l*2d + kv*d + h*hd + e ; row = b*T + t  ->  [L*2][slots][H][T][hd]
      const int d = epi.d, hd = epi.head_dim;
      const int l2 = col / d, cc = col - l2 * d;
      const int h = cc / hd, e2 = cc - h * hd;
      const int b = row / epi.rpb, t = row - b * epi.rpb;
      const long long o = ((((long long)l2 * epi.n_slots + epi.slot0 + b) * epi.n_head + h) * epi.rpb + t) * hd + e2;
      ((bf16*)epi.out)[o] = f2bf(v);
      break;
    }
  }
}

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
    for (int s = 0; s < splitk; ++s) v += part[s * total + i];
    const int row = (int)(i / N), col = (int)(i - (long long)row * N);
    apply_epi<KIND>(epi, row, col, v);
  }
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
