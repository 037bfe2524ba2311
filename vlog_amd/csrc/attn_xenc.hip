// Factored cross-attention for the decoder (gfx950): attend over the encoder output itself, not over a
// projected cross-KV cache.
//
// For head h, Whisper's cross-attention reads K_h = E Wk_h^T and V_h = E Wv_h^T + bv_h, where E is the
// window's encoder output [1500][d] and Wk_h, Wv_h are rows h*64 .. h*64+63 of the k/v projections
// (modeling_whisper.py:241-356 [TF]; CTranslate2 projects them once per window [FW↑]).  Reassociated:
//   s_h[t] = q_h . K_h[t]          = (Wk_h^T q_h) . E[t]             q'_h = Wk_h^T q_h   (a d-vector)
//   o_h    = sum_t p_h[t] V_h[t]   = Wv_h (sum_t p_h[t] E[t]) + bv_h  u_h  = P_h E         (a d-vector)
// (the softmax row sums to 1, so the v bias passes through unchanged).  Per decoder step and layer, a
// window's attention then streams E ONCE for every head and every row of the window: 1500 x d bf16 =
// 3.84 MB for large-v3, against 2 x 3.84 MB of K and V panels.  The per-window cross-KV projection
// disappears too (314.6 GFLOP and 245.8 MB of HBM per large-v3 window).  The price is H x the attention
// FLOPs: a (H R) x 1500 x d GEMM pair per window and layer (R = rows sharing the window), which MFMA
// absorbs.  At R = 1 the kernel executes 64 FLOP per streamed byte (20 of its 32 MFMA rows used), far
// under the ~312 FLOP/B ridge of MI355X, so it stays HBM-bound.
//
// Three kernels per layer:
//   xq_kernel       q' = (1/8 log2 e) Wk_h^T q_h, bf16 [rows][H][d] (MFMA, K = 64).  Optionally sums the cq
//                   projection's split-K slabs while loading q, in the order splitk_reduce_kernel uses.
//   xattn_kernel    one workgroup per (window group, key split, m-tile of 32 (row, head) pairs).  NW waves
//                   (8, or 4 when d/8 is not a multiple of 32), wave w owns the QW = d/NW columns
//                   [w QW, (w+1) QW) of E.  Per 32-position tile:
//                     S^T partial = E[t][wave cols] . q'^T  (v_mfma_f32_32x32x16_bf16, E from LDS as the A
//                                   operand, q' register-resident as the B operand);
//                     the NW partials are summed through LDS in a fixed order (two barriers per tile), so
//                     every wave holds the same S^T and runs the same online softmax (deferred rescale,
//                     log2 units);
//                     U^T[wave cols] += E^T . P^T  (the S^T accumulator IS the P^T operand; E^T fragments
//                                   come from the same LDS image through ds_read_b64_tr_b16).
//                   E is streamed with coalesced 16-B non-temporal loads, register-staged one tile ahead,
//                   into a wave-private LDS image, so no barrier guards it.  Output per split: (m, l) and
//                   u / l as bf16.  (Tried: each wave streaming whole contiguous rows into a block-shared
//                   image reads faster alone, 5.1-5.5 vs 4.7-4.8 TB/s loads-only in tools/xattn_bench, but
//                   the two extra barriers per tile cost more than that with the compute in: 3181 vs 3217.)
//   xcomb_vo_kernel merges the key splits (weights l_s 2^(m_s - M) / L) and applies Wv_h and bv_h (MFMA,
//                   K = d) -> the attention output ao [rows][d].  With capture on, it also turns the raw
//                   scores that xattn wrote for the alignment heads into probabilities.
#include "common.h"
#include <hip/hip_ext.h>
#include <algorithm>
#include <cstdlib>
#include <stdexcept>
#include <string>
#include <type_traits>

#define XTHR 8.0f              // deferred-rescale threshold (log2 units)
#define XMAXS 16               // max key splits

typedef __attribute__((ext_vector_type(4))) short xi16x4;
typedef __attribute__((ext_vector_type(2))) int xi32x2;

__device__ __forceinline__ f32x16 xzero16() {
  f32x16 z;
#pragma unroll
  for (int r = 0; r < 16; ++r) z[r] = 0.f;
  return z;
}

// E image in LDS: rows of LDR elements with LDR / 8 = 4 (mod 16) 16-B slots, and 16-B chunk c of row r
// stored at chunk c ^ ((r >> 2) & 3) (a permutation inside each aligned quad of chunks).  Row r then starts
// on slot 4r (mod 16) of the 256-B bank row, and both reads are conflict-free: ds_read_b128 of one chunk
// over the 16 rows of a lane group (rows of equal r mod 4 differ in (r >> 2) & 3 inside every group of the
// b128 lane-group table), and ds_read_b64_tr_b16 of 4 rows (4k..4k+3) x 64 B (slots 4i + quad).
__device__ __forceinline__ int xchunk(int r, int c) { return c ^ ((r >> 2) & 3); }

// The cross-wave S reduction's barrier.  RAW: the LDS writes before it are retired by lgkmcnt(0).  With LDS-DMA in
// flight (the split-staging form) __syncthreads would also drain vmcnt (the compiler orders the pending DMA's LDS
// writes before a workgroup fence), i.e. wait for the next tiles' loads at every barrier; the wave-private DMA
// images are ordered for their own wave by the counted vmcnt at each tile instead (MI355X_MICROARCH.md item 7).
template <bool RAW>
__device__ __forceinline__ void xbarrier() {
  if constexpr (RAW) {
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  } else {
    __syncthreads();
  }
}
// swap bits 2 and 3 of a column's position in its 16-column block (the u record order: xstore_u)
__host__ __device__ constexpr int xswap23(int x) { return (x & 3) | ((x >> 1) & 4) | ((x << 1) & 8); }
__host__ __device__ constexpr int xldr(int qw) { return (qw / 8 + ((4 - qw / 8) % 16 + 16) % 16) * 8; }

// ------------------------------------------------------------------------------------------------------
// Weight packing, from the fused [L][K|V][d][d] cross projection (engine weight "dec.ckv.w"); runs once per
// weight upload:
//   wkt[l][h][c][j]            = Wk_l[h*64 + j][c]   (xq's A operand: 64 contiguous j per c)
//   wvb[l][h][c/16][j][p]      = Wv_l[h*64 + j][16 (c/16) + xswap23(p)]   (xcomb's B operand: one k-step of 32 j = 1 KB
//                                contiguous; within a 16-column block in the order xstore_u writes u)
__global__ void xpack_kernel(const bf16* __restrict__ ckv_w, bf16* __restrict__ wkt, bf16* __restrict__ wvb, int L,
                             int H, int d) {
  const long long total = (long long)L * H * d * 64;
  for (long long idx = blockIdx.x * 256LL + threadIdx.x; idx < total; idx += (long long)gridDim.x * 256) {
    {
      const int j = (int)(idx & 63);
      const long long rest = idx >> 6;
      const int c = (int)(rest % d);
      const long long lh = rest / d;
      const int h = (int)(lh % H), l = (int)(lh / H);
      wkt[idx] = ckv_w[((long long)l * 2 * d + h * 64 + j) * d + c];
    }
    {
      const int c16 = (int)(idx & 15);
      const long long r1 = idx >> 4;
      const int j = (int)(r1 & 63);
      const long long r2 = r1 >> 6;
      const int kb = (int)(r2 % (d / 16));
      const long long lh = r2 / (d / 16);
      const int h = (int)(lh % H), l = (int)(lh / H);
      wvb[idx] = ckv_w[((long long)l * 2 * d + d + h * 64 + j) * d + kb * 16 + xswap23(c16)];
    }
  }
}

// XCD-aware flattening of a (gx, gy) grid launched as gx * gy one-dimensional blocks: blocks with consecutive
// remapped ids (the gx blocks of one y) run on one XCD, so what they share (a head's weight slice) is fetched
// into that XCD's L2 once instead of by every XCD (speed only: any placement gives the same results).
__device__ __forceinline__ void xcd_block(int gx, int& bx, int& by) {
  const int nwg = gridDim.x, bid = blockIdx.x, xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  const int wgid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  by = wgid / gx;
  bx = wgid - by * gx;
}

// ------------------------------------------------------------------------------------------------------
struct XQArgs {
  const bf16* q; long long ldq;          // q rows [rows][ldq] (unused when q_part is set)
  const float* q_part; int q_splits, q_rows; const float* q_bias;   // cq split-K slabs [s][q_rows][ldq] + bias
  const bf16* wkt;                       // this layer's Wk^T [H][d][64]
  bf16* qp;                              // [rows][H][d]
  int rows, H, d;
  float scale;
};

// grid ceil(rows / 32) x H x ceil(d / 256) flattened (xcd_block); wave w computes c-tiles 8z + 2w and 8z + 2w + 1
// of head y for 32 rows.  D[c][r] = sum_j Wk^T[c][j] q[r][h*64 + j]: A = Wk^T rows (16-B loads), B = q rows.  The block
// first builds its 32 x 64 q tile in LDS: 8 elements per thread, every slab load issued before any add
// (the slab sum is then one memory round trip, not one per slab), summed in slab order plus the bias as
// splitk_reduce_kernel does, so the value is bit-identical to the unfused projection's bf16 q.
__global__ __launch_bounds__(256) void xq_kernel(XQArgs a) {
  __shared__ __attribute__((aligned(16))) bf16 sq[32 * 72];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, hh = lane >> 5, l32 = lane & 31;
  const int n_ct = a.d / 32, gz = (n_ct + 7) / 8;
  int bx, hz;
  xcd_block((a.rows + 31) / 32, bx, hz);              // the row tiles of one (head, column group) on one XCD
  const int h = hz / gz, bz = hz - h * gz;
  // this wave's Wk^T fragments first (independent of q: one memory round trip with the q loads)
  bf16x8 wf[2][4];
#pragma unroll
  for (int ci = 0; ci < 2; ++ci) {
    const int ct = min(bz * 8 + wv * 2 + ci, n_ct - 1);
    const bf16* wr = a.wkt + ((long long)h * a.d + ct * 32 + l32) * 64 + 8 * hh;
#pragma unroll
    for (int s = 0; s < 4; ++s) wf[ci][s] = *(const bf16x8*)(wr + 16 * s);
  }
  {
    const int rr = tid >> 3, c8 = (tid & 7) * 8, r = min(bx * 32 + rr, a.rows - 1);
    bf16x8 qv;
    const int col = h * 64 + c8;
    if (a.q_part) {
      // the bias first: requested with the slabs, not one more round trip after their sum
      const f32x4 bq0 = *(const f32x4*)(a.q_bias + col), bq1 = *(const f32x4*)(a.q_bias + col + 4);
      const long long slab = (long long)a.q_rows * a.ldq;
      const float* pq = a.q_part + (long long)r * a.ldq + col;
      f32x4 lo[XMAXS], hi[XMAXS];
#pragma unroll
      for (int sp = 0; sp < XMAXS; ++sp)
        if (sp < a.q_splits) {
          lo[sp] = *(const f32x4*)(pq + sp * slab);
          hi[sp] = *(const f32x4*)(pq + sp * slab + 4);
        }
      float v[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int sp = 0; sp < XMAXS; ++sp)
        if (sp < a.q_splits) {
#pragma unroll
          for (int i = 0; i < 4; ++i) { v[i] += lo[sp][i]; v[4 + i] += hi[sp][i]; }
        }
#pragma unroll
      for (int i = 0; i < 8; ++i) qv[i] = f2bf(v[i] + (i < 4 ? bq0[i] : bq1[i - 4]));
    } else {
      qv = *(const bf16x8*)(a.q + (long long)r * a.ldq + col);
    }
    *(bf16x8*)(sq + rr * 72 + c8) = qv;
  }
  __syncthreads();
  const int r = bx * 32 + l32;
  bf16x8 qb[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) qb[s] = *(const bf16x8*)(sq + l32 * 72 + 16 * s + 8 * hh);
#pragma unroll
  for (int ci = 0; ci < 2; ++ci) {
    const int ct = bz * 8 + wv * 2 + ci;
    if (ct >= n_ct) break;
    f32x16 acc = xzero16();
#pragma unroll
    for (int s = 0; s < 4; ++s) acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wf[ci][s], qb[s], acc, 0, 0, 0);
    if (r < a.rows) {
      bf16* op = a.qp + ((long long)r * a.H + h) * a.d + ct * 32 + 4 * hh;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        bf16x4 w;
#pragma unroll
        for (int e = 0; e < 4; ++e) w[e] = f2bf(acc[4 * g + e] * a.scale);
        *(bf16x4*)(op + 8 * g) = w;
      }
    }
  }
}

// ------------------------------------------------------------------------------------------------------
struct XAttnArgs {
  const bf16* qp;                        // [rows][H][d], pre-scaled (log2 units)
  const bf16* enc;                       // [slots][T][d] bf16, or (F8) [slots][T][d] OCP e4m3 bytes
  const float* escale;                   // F8: [slots][T] per-position scale (E[t] = e4m3[t] * escale[t])
  const int* hyp_slot; const int* row_hyp; const int* done;
  int H, T, d, G, n_mt, splits, n_items, per_xcd;
  int rev;                               // 1: each XCD walks its items in reverse (see launch_xattn)
  int keep;                              // window groups < keep load E with the default cache policy (else nt)
  long long slab_rows;                   // rows of the whole pass: partial slab stride
  bf16* part_u;                          // [splits][H][d/16][slab_rows][16]   u_s / l_s
  float* part_ml;                        // [splits][slab_rows][H][2]   (m_s, l_s)
  float* probs; const int* head_map; int n_align;   // capture: raw scores [row][n_align][T]
  unsigned long long* stat;
  long long sk_W; int sk_P, sk_lane0, sk_lanes, sk_c0, sk_nch, sk_map;   // LDS-DMA chunks (stream-K): units of the whole pass, chunk count,
                                         // this launch's first lane (of the pass) and lane count, its first chunk; sk_W = 0: items
  int abl;                               // microbenchmark ablations (tools/xattn_bench; product: 0, and the
                                         // product kernel is compiled without them: template ABL): bit 0 skips
                                         // the S MFMAs, bit 1 the cross-wave sum, bit 2 the U phase, bit 3
                                         // loads E with plain loads (same-box bench: 1 % slower than
                                         // non-temporal ones; tools/gpu_ablib.sh), bit 4 skips the E loads
};

// A split partial u / l of one (row, head) column as bf16 (up = its 16-element record in column block 0 of the wave's
// columns; kstride = elements per column block).  Accumulator register 4 g + e of column tile c holds column
// 32 c + 8 g + 4 hh + e (relative to the wave's first), i.e. 16-column block 2 c + (g >> 1) at column 8 (g & 1) + 4 hh + e.
// The record stores position 8 hh + 4 (g & 1) + e (bits 2 and 3 of the column swapped, xswap23): each lane writes its
// 8 values of a block as one 16-B store, so one store instruction covers 32 rows x 32 B = 1 KB contiguous (8-B pieces
// half-filled every line per instruction).  xpack_kernel packs Wv's columns in the same order, so the merge's MFMA
// pairs position p of u with position p of Wv.
template <int CT>
__device__ __forceinline__ void xstore_u(bf16* up, long long kstride, const f32x16 (&o)[CT], float inv, int hh) {
#pragma unroll
  for (int c = 0; c < CT; ++c)
#pragma unroll
    for (int gp = 0; gp < 2; ++gp) {
      bf16x8 w;
#pragma unroll
      for (int e = 0; e < 8; ++e) w[e] = f2bf(o[c][8 * gp + e] * inv);
      *(bf16x8*)(up + (2 * c + gp) * kstride + 8 * hh) = w;
    }
}

// One work item: rows of group `grp` x (row, head) m-tile `mt`, key tiles [tb, te) written as partial `split`.
template <int QW, int NW, int DEPTH, bool F8, int ABL, bool CAP>
__device__ __forceinline__ void xattn_segment(const XAttnArgs& a, char* smem, int grp, int mt, int split, int tb,
                                              int te) {
  constexpr int KS = QW / 16, CT = QW / 32, LDR = xldr(QW), CPR = F8 ? QW / 16 : QW / 8, LS = F8 ? KS / 2 : KS;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, hh = lane >> 5, l32 = lane & 31;
  const int M = a.G * a.H;
  const int m = mt * 32 + l32;
  const int row0 = grp * a.G;
  int row = row0, hd = 0;
  bool valid = m < M;
  if (valid) {
    const int ri = m / a.H;
    row = row0 + ri;
    hd = m - ri * a.H;
    valid = !(a.done && a.done[a.row_hyp[row]]);
  }
  if (!__any(valid)) return;             // identical in all waves: uniform exit before any barrier
  const int slot = a.hyp_slot[a.row_hyp[row0]];
  const int cb = wv * QW;
  constexpr int EB = F8 ? 1 : 2;                         // bytes per stored E element
  const char* E = (const char*)a.enc + ((long long)slot * a.T * a.d + cb) * EB;
  const float* Es = F8 ? a.escale + (long long)slot * a.T : nullptr;
  // bf16: the slot is stored tile-blocked (xblock_kernel): [tile][wave][32 rows][QW], so one wave's 32 x QW slice of a
  // tile is ONE contiguous, 128-B-aligned 10 KB run and every load is whole cache lines (row-major, each 320-B wave
  // row slice straddled three 128-B lines: 1.2-1.3x the line requests).  F8 keeps the row-major e4m3 image.
  const int n_tiles = (a.T + 31) / 32;
  const char* EB16 = (const char*)a.enc + ((long long)slot * n_tiles * NW + wv) * (32LL * QW * 2);
  constexpr int IMGR = 32;                                // image rows per wave
  bf16* sE = (bf16*)smem + wv * IMGR * LDR;
  bf16* sER = sE + 16 * LDR;                              // rows 16-31
  float* sX = (float*)(smem + NW * IMGR * LDR * 2);      // [NW][16][64] S^T partials
  float* sRed = sX + NW * 16 * 64;                       // [16][64] their sums
  {
    const unsigned long long nq = __popcll(__ballot(valid && hh == 0));
    if (a.stat && tid == 0) {
      const long long npos = (long long)min(te * 32, a.T) - tb * 32;
      unsigned long long by = nq * (unsigned long long)a.d * 2;
      if (mt == 0) by += (unsigned long long)(npos * a.d * EB + (F8 ? npos * 4 : 0));
      atomicAdd(a.stat + (blockIdx.x & (STAT_SLOTS - 1)), by);
    }
  }

  bf16x8 qf[KS];
  {
    const bf16* qr = a.qp + ((long long)row * a.H + hd) * a.d + cb + 8 * hh;
#pragma unroll
    for (int s = 0; s < KS; ++s) qf[s] = valid ? *(const bf16x8*)(qr + 16 * s) : bf16x8{};
  }
  f32x16 o[CT];
#pragma unroll
  for (int c = 0; c < CT; ++c) o[c] = xzero16();
  float m_run = -INFINITY, l_run = 0.f;

  // Address arithmetic is recomputed from an opaque copy of the lane id inside the loop (`lo`), so the
  // compiler does not hoist ~40 loop-invariant addresses into registers the accumulators need.
  i32x4 stgA[LS];
  float scA = 1.f;                       // F8: lane l (< 32) stages the scale of position tile*32 + l
  auto load = [&](i32x4 (&stg)[LS], float& scl, int tile, int lo) {
    if (ABL & 16) {                    // ablation: no E loads (compute-only timing)
#pragma unroll
      for (int i = 0; i < LS; ++i) stg[i] = i32x4{0x3c003c00 + lo, 0x3c003c00, 0x3c003c00, 0x3c003c00 + tile};
      scl = 1.f;
      return;
    }
#pragma unroll
    for (int i = 0; i < LS; ++i) {
      const int idx = i * 64 + lo;
      const i32x4* src;
      if constexpr (F8) {
        const int r = idx / CPR, ch = idx - r * CPR;
        const int t = min(tile * 32 + r, a.T - 1);
        src = (const i32x4*)(E + ((long long)t * a.d) * EB + ch * 16);
      } else {
        // chunk idx = (r, ch) of the wave's slice, stored at byte 16 idx of its tile block (rows past T are zeros)
        src = (const i32x4*)(EB16 + (long long)tile * NW * (32LL * QW * 2) + idx * 16);
      }
      if (ABL & 8) stg[i] = *src;
      else stg[i] = __builtin_nontemporal_load(src);
    }
    if (F8) scl = Es[min(tile * 32 + (lo & 31), a.T - 1)];
  };
  float* sScale = nullptr;
  if (F8) sScale = (float*)(smem + NW * IMGR * LDR * 2 + (NW + 1) * 16 * 64 * 4) + wv * 32;
  float* pr_row = nullptr;
  if (a.probs && wv == 0 && valid) {
    const int hm = a.head_map[hd];
    if (hm >= 0) pr_row = a.probs + ((long long)row * a.n_align + hm) * a.T;
  }
  // one tile: its staged registers -> the wave's LDS image, the loads of the next tile into the same
  // registers, then S^T, the cross-wave sum, the online softmax and U^T
  auto tile_step = [&](int tile, auto& stg, float& scl, int ahead) {
    int lo = lane;
    asm volatile("" : "+v"(lo));
    bf16* sEA = sE;                                       // rows 0-15 of this tile
    // wave-private LDS image of this tile (this wave's earlier reads of it are complete: LDS is in order);
    // F8: each 16-B chunk of 16 e4m3 values becomes two bf16 chunks (exact: e4m3 is a subset of bf16)
    int r = lo / CPR, ch = lo % CPR;     // chunk (r, ch) of load i, stepped like the global offsets
#pragma unroll
    for (int i = 0; i < LS; ++i) {
      if (i) {
        ch += 64 % CPR;
        r += 64 / CPR;
        if (ch >= CPR) { ch -= CPR; ++r; }
      }
      if (F8) {
#pragma unroll
        for (int hf = 0; hf < 2; ++hf) {
          bf16x8 v;
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            const int word = stg[i][2 * hf + j];
            const auto f01 = __builtin_amdgcn_cvt_pk_f32_fp8(word, false);
            const auto f23 = __builtin_amdgcn_cvt_pk_f32_fp8(word, true);
            v[4 * j] = f2bf(f01[0]); v[4 * j + 1] = f2bf(f01[1]);
            v[4 * j + 2] = f2bf(f23[0]); v[4 * j + 3] = f2bf(f23[1]);
          }
          *(bf16x8*)(sE + r * LDR + 8 * xchunk(r, 2 * ch + hf)) = v;
        }
      } else {
        *(i32x4*)(sE + r * LDR + 8 * xchunk(r, ch)) = stg[i];
      }
    }
    if (F8 && lo < 32) sScale[lo] = scl;
    if (tile + ahead < te) load(stg, scl, tile + ahead, lo);
    // ---- S^T partial over this wave's columns
    f32x16 sc = xzero16();
    {
      // A fragment of k-step s: row l32, chunk 2s + hh -> stored at 4 (s >> 1) + ((2 (s & 1) + hh) ^ g)
      const int l32o = lo & 31, g = (l32o >> 2) & 3;
      const bf16* rb = l32o < 16 ? sEA + l32o * LDR : sER + (l32o - 16) * LDR;
      const bf16* s0 = rb + 8 * (hh ^ g);
      const bf16* s1 = rb + 8 * ((2 + hh) ^ g);
      if (!(ABL & 1)) {
#pragma unroll
        for (int s = 0; s < KS; ++s) {
          const bf16x8 ea = *(const bf16x8*)(((s & 1) ? s1 : s0) + 32 * (s >> 1));
          sc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ea, qf[s], sc, 0, 0, 0);
        }
      }
    }
    // the NW partials -> the full S^T in every wave: partials to LDS; wave w sums registers
    // [w RPW, (w+1) RPW) over the waves in a fixed order (0..NW-1); every wave reads the 16 sums back
    if (!(ABL & 2)) {
#pragma unroll
      for (int r = 0; r < 16; ++r) sX[(wv * 16 + r) * 64 + lane] = sc[r];
      xbarrier<false>();
      // wave w sums registers r = w, w + NW, ... over the waves in order 0..NW-1 (any NW)
#pragma unroll
      for (int k = 0; k < (16 + NW - 1) / NW; ++k) {
        const int r = wv + k * NW;
        if (r >= 16) break;
        float v = sX[r * 64 + lane];
#pragma unroll
        for (int w2 = 1; w2 < NW; ++w2) v += sX[(w2 * 16 + r) * 64 + lane];
        sRed[r * 64 + lane] = v;
      }
      xbarrier<false>();
#pragma unroll
      for (int r = 0; r < 16; ++r) sc[r] = sRed[r * 64 + lane];
    }
    const int t0 = tile * 32;
    float ps[16];                        // F8: the scale of each S^T row this lane holds (U uses p * scale)
    if (F8) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const f32x4 sv = *(const f32x4*)(sScale + 8 * g + 4 * hh);
#pragma unroll
        for (int e2 = 0; e2 < 4; ++e2) {
          ps[4 * g + e2] = sv[e2];
          sc[4 * g + e2] *= sv[e2];
        }
      }
    }
    if (t0 + 32 > a.T) {
#pragma unroll
      for (int r = 0; r < 16; ++r)
        if (t0 + 8 * (r >> 2) + 4 * hh + (r & 3) >= a.T) sc[r] = -INFINITY;
    }
    if (CAP && pr_row) {                 // alignment capture: a separate instantiation (CAP)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int t = t0 + 8 * (r >> 2) + 4 * hh + (r & 3);
        if (t < a.T) pr_row[t] = sc[r];
      }
    }
    // ---- online softmax (lane = one (row, head) column), deferred rescale
    float mx = sc[0];
#pragma unroll
    for (int r = 1; r < 16; ++r) mx = fmaxf(mx, sc[r]);
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    if (__any(mx > m_run + XTHR)) {
      const float mn = fmaxf(m_run, mx);
      const float alpha = __builtin_amdgcn_exp2f(m_run - mn);
      l_run *= alpha;
#pragma unroll
      for (int c = 0; c < CT; ++c)
#pragma unroll
        for (int r = 0; r < 16; ++r) o[c][r] *= alpha;
      m_run = mn;
    }
    bf16x8 pf[2];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float p = __builtin_amdgcn_exp2f(sc[r] - m_run);
      l_run += p;
      pf[r >> 3][r & 7] = f2bf(F8 ? p * ps[r] : p);
    }
    // ---- U^T (wave cols) += E^T . P^T.  Transposed read of rows 16 ks + 8 jh + 4 hh + gq, columns
    // 32 c + 16 (G4 & 1) + 4 gp: chunk 4 c + lowc (lowc = 2 (G4 & 1) + (gp >> 1)) is stored at
    // 4 c + (lowc ^ (2 jh + hh)), so each jh has one base address and (ks, c) are immediate offsets.
    if (!(ABL & 4)) {
      const int G4 = (lo >> 4) & 3, gi = lo & 15, gq = gi >> 2, gp = gi & 3;
      const int lowc = 2 * (G4 & 1) + (gp >> 1);
      const int o0 = (4 * hh + gq) * LDR + 8 * (lowc ^ hh) + 4 * (gp & 1);
      const int o1 = (8 + 4 * hh + gq) * LDR + 8 * (lowc ^ (2 + hh)) + 4 * (gp & 1);
#pragma unroll
      for (int c = 0; c < CT; ++c)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
          // rows 16 ks .. 16 ks + 15: image of rows 0-15 or of rows 16-31 (same swizzle: (r >> 2) & 3 repeats)
          const bf16* tb0 = (ks ? sER : sEA) + o0;
          const bf16* tb1 = (ks ? sER : sEA) + o1;
          const int off = 32 * c;
          const xi32x2 v0 = __builtin_bit_cast(xi32x2, __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                                                            (__attribute__((address_space(3))) xi16x4*)(tb0 + off)));
          const xi32x2 v1 = __builtin_bit_cast(xi32x2, __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                                                            (__attribute__((address_space(3))) xi16x4*)(tb1 + off)));
          const bf16x8 va = __builtin_bit_cast(bf16x8, i32x4{v0[0], v0[1], v1[0], v1[1]});
          o[c] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(va, pf[ks], o[c], 0, 0, 0);
        }
    }
  };
  if constexpr ((ABL & 32) != 0) {
    // microbenchmark only (bit 5): two register staging sets, each tile's loads issued two tiles ahead -- does
    // the load path stream faster with twice the bytes in flight per wave?  (Loads-only: ABL 39.)
    i32x4 stgB[LS];
    float scB = 1.f;
    if (tb < te) load(stgA, scA, tb, lane);
    if (tb + 1 < te) load(stgB, scB, tb + 1, lane);
    for (int tile = tb; tile < te; tile += 2) {
      tile_step(tile, stgA, scA, 2);
      if (tile + 1 < te) tile_step(tile + 1, stgB, scB, 2);
    }
  } else {
    if (tb < te) load(stgA, scA, tb, lane);
    for (int tile = tb; tile < te; ++tile) tile_step(tile, stgA, scA, 1);
  }
  l_run += __shfl_xor(l_run, 32, 64);
  if (valid) {
    const float inv = 1.0f / l_run;
    const long long pi = ((long long)split * a.slab_rows + row) * a.H + hd;
    if (wv == 0 && hh == 0) {
      a.part_ml[2 * pi] = m_run;
      a.part_ml[2 * pi + 1] = l_run;
    }
    xstore_u(a.part_u + (((long long)split * a.H + hd) * (a.d / 16) + cb / 16) * (a.slab_rows * 16) + (long long)row * 16,
             a.slab_rows * 16, o, inv, hh);
  }
}

// stream-K cut of W units into P chunks: chunk c = units [xsk_begin(c), xsk_begin(c + 1)); xsk_chunk(g) holds unit g
__host__ __device__ __forceinline__ long long xsk_begin(long long c, long long W, int P) { return c * W / P; }
__host__ __device__ __forceinline__ int xsk_chunk(long long g, long long W, int P) { return (int)(((g + 1) * P - 1) / W); }

// The chunk cut's segments as separate work items (the register form; xattn_dma_kernel walks a chunk in one
// workgroup instead).  XCD x (block id & 7) takes the contiguous chunk range [c_x, c_x + n_x) of the launch: its items
// j < n_x are those chunks' first segments (from the chunk's start to the end of its lane or of the chunk), then one
// item per lane start strictly inside the range (that lane's first piece, to the end of the chunk or of the lane;
// an item whose lane start opens a chunk is empty).  The hardware hands an XCD's items to its CUs in block order, so
// the CUs that finish a short first segment first take the second segments: per CU about one chunk of units and at
// most two item start-ups, instead of ceil(items / CUs) rounds of equal items.  Segments, pieces and their order
// per lane are those of xattn_dma_kernel's chunks, so the two forms give the same bits.  -> false: empty item.
__device__ __forceinline__ bool xsk_item(const XAttnArgs& a, int n_tiles, int& lane, int& tb, int& te, int& piece) {
  const int x = blockIdx.x & 7, j = blockIdx.x >> 3;
  const int q = a.sk_nch >> 3, r = a.sk_nch & 7;
  const int cx0 = a.sk_c0 + (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q), ncx = q + (x < r ? 1 : 0);
  const long long L0 = (long long)a.sk_lane0 * n_tiles, L1 = L0 + (long long)a.sk_lanes * n_tiles;
  long long g0, g1;
  if (j < ncx) {
    const int c = cx0 + j;
    g0 = max(xsk_begin(c, a.sk_W, a.sk_P), L0);
    g1 = min(xsk_begin(c + 1, a.sk_W, a.sk_P), L1);
    if (g0 >= g1) return false;
    const long long la = g0 / n_tiles;
    g1 = min(g1, (la + 1) * n_tiles);
  } else {
    const long long lo = max(xsk_begin(cx0, a.sk_W, a.sk_P), L0 + 1), hi = min(xsk_begin(cx0 + ncx, a.sk_W, a.sk_P), L1);
    const long long la = (lo + n_tiles - 1) / n_tiles + (j - ncx);
    g0 = la * n_tiles;
    if (g0 >= hi) return false;
    const int c = xsk_chunk(g0, a.sk_W, a.sk_P);
    if (xsk_begin(c, a.sk_W, a.sk_P) == g0) return false;          // the chunk's own first segment covers it
    g1 = min(min(xsk_begin(c + 1, a.sk_W, a.sk_P), L1), g0 + n_tiles);
  }
  const long long la = g0 / n_tiles;
  lane = (int)(la - a.sk_lane0);
  tb = (int)(g0 - la * n_tiles);
  te = (int)(g1 - la * n_tiles);
  piece = xsk_chunk(g0, a.sk_W, a.sk_P) - xsk_chunk(la * n_tiles, a.sk_W, a.sk_P);
  return true;
}

// Blocks of a chunk-cut launch of the register form: 8 x the largest XCD item list (chunks + lane starts inside them).
int xsk_item_blocks(long long W, int P, int c0, int nch, int lane0, int lanes, int n_tiles) {
  const int q = nch >> 3, r = nch & 7;
  const long long L0 = (long long)lane0 * n_tiles, L1 = L0 + (long long)lanes * n_tiles;
  long long most = 0;
  for (int x = 0; x < 8; ++x) {
    const int cx0 = c0 + (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q), ncx = q + (x < r ? 1 : 0);
    if (ncx == 0) continue;
    const long long lo = std::max(xsk_begin(cx0, W, P), L0 + 1), hi = std::min(xsk_begin(cx0 + ncx, W, P), L1);
    const long long starts = hi > lo ? (hi + n_tiles - 1) / n_tiles - (lo + n_tiles - 1) / n_tiles : 0;
    most = std::max(most, (long long)ncx + std::max(0LL, starts));
  }
  return (int)(8 * most);
}

template <int QW, int NW, int DEPTH, bool F8 = false, int ABL = 0, bool CAP = false>
__global__ __launch_bounds__(NW * 64) void xattn_kernel(XAttnArgs a) {
  static_assert(DEPTH == 1, "one tile staged ahead (the other staging forms are retired: DESIGN.md §6)");
  constexpr int LDR = xldr(QW);
  constexpr int IMGR = 32;
  __shared__ __attribute__((aligned(16))) char smem[NW * IMGR * LDR * 2 + (NW + 1) * 16 * 64 * 4 + (F8 ? NW * 32 * 4 : 0)];
  const int n_tiles = (a.T + 31) / 32;
  if (a.sk_W) {                                  // the chunk cut (greedy passes: one m-tile per window group)
    int ln, tb, te, piece;
    if (!xsk_item(a, n_tiles, ln, tb, te, piece)) return;
    xattn_segment<QW, NW, DEPTH, F8, ABL, CAP>(a, smem, ln / a.n_mt, ln % a.n_mt, piece, tb, te);
    return;
  }
  // XCD-aware item order: the blocks of one (group, split), i.e. its m-tiles, run on one XCD at about the
  // same time, so the 2nd..n-th reads of an E tile hit that XCD's L2
  const int j = blockIdx.x >> 3;
  const int item = (blockIdx.x & 7) * a.per_xcd + (a.rev ? a.per_xcd - 1 - j : j);
  if (item >= a.n_items) return;
  const int mt = item % a.n_mt;
  const int rest = item / a.n_mt;
  const int split = rest % a.splits, grp = rest / a.splits;
  const int tb = split * n_tiles / a.splits, te = (split + 1) * n_tiles / a.splits;
  // a uniform choice per workgroup between two instantiations (no branch inside the tile loop): the first
  // `keep` window groups stream E with default-policy loads, which may stay in the Infinity Cache for the next
  // layer, the rest with non-temporal loads, which should not evict them
  if (ABL == 0 && grp < a.keep) xattn_segment<QW, NW, DEPTH, F8, 8, CAP>(a, smem, grp, mt, split, tb, te);
  else xattn_segment<QW, NW, DEPTH, F8, ABL, CAP>(a, smem, grp, mt, split, tb, te);
}

// ------------------------------------------------------------------------------------------------------
// LDS-DMA form (opt-in, cross_attn_dma; bf16 cross memory, d = 1280: 8 waves x 160 columns; measured slower than the
// register form in the bench step).  Per tile the same per-wave
// MFMAs and the same fixed-order cross-wave sum as xattn_segment; what changes is how E reaches LDS, where the S
// partials live, and how the work is cut:
//   - each wave streams its 10 KB slice of a tile straight into LDS (10 global_load_lds_dwordx4 of 1 KiB; the
//     image's chunk swizzle goes on the per-lane SOURCE address), two tiles ahead, into a ring of two 80 KB slots
//     that fills the whole 160 KB LDS -- no staging registers, no ds_write of E;
//   - after a wave has read its slice of the current tile (the S operand, and the U operand of rows 0-15), that part
//     of the slice is dead, and the S partials (4 KB) and their sums (512 B) are written there;
//   - a third barrier per tile (after every wave has read the sums) frees the slot, and each wave then issues its
//     DMAs of tile + 2 into it: a tile's loads are in flight for about one and a half tiles of compute;
//   - the work: a "lane" is a (window group, m-tile) pair, a "unit" one 32-position tile of a lane, units numbered
//     lane-major (lane x n_tiles + tile).  A workgroup walks a contiguous range of units -- one segment per lane it
//     touches, each segment one partial of its lane, merged by xcomb like a key split:
//       items:  the ranges of xattn_kernel's work items (window group, key split, m-tile): one segment each;
//       chunks (stream-K; greedy passes, one m-tile per window): the pass's units cut into P equal contiguous ranges,
//               P = the CU count (one 160 KB workgroup per CU), so every CU streams for the whole launch.  Items left
//               the last round part-empty (150 windows x 3 splits = 450 items on 256 CUs) and paid each item's
//               start-up (~7 us, tools/xattn_bench); a chunk pays it once and crosses one or two window boundaries.
//               Its pieces are a function of the whole pass (the window count), not of how the pass is sliced into
//               launches; a window's pieces add in a different order than its key splits, so the two cuts agree to
//               f32 rounding, not bit for bit.  A mid-chunk window boundary costs ~10 us (the finished segment's
//               partial stores are acknowledged late while every CU streams, and later DMA waits count them).
// Waits are counted vmcnt + raw s_barrier (no barrier drains the DMA queue: MI355X_MICROARCH.md item 7).  q' is an
// ordinary load whose first use sits where a full wait costs nothing extra: hipcc waits vmcnt(0) at the first use of
// an ordinary load's result while LDS-DMA is in flight (cdna_hip_programming.md §5, "Pipelining across barriers").
#define XD_QW 160
#define XD_NW 8
#define XD_IMG (32 * XD_QW * 2)            // bytes of one wave's slice of a tile
#define XD_LS (XD_IMG / 1024)              // its LDS-DMA instructions
#define XD_SLOT (XD_NW * XD_IMG)

template <int ABL = 0, bool CAP = false>
__global__ __launch_bounds__(XD_NW * 64) void xattn_dma_kernel(XAttnArgs a) {
  constexpr int QW = XD_QW, NW = XD_NW, KS = QW / 16, CT = QW / 32, LDR = xldr(QW), CPR = QW / 8, IMG = XD_IMG,
                LS = XD_LS, SLOT = XD_SLOT;
  static_assert(LDR == QW && IMG % 1024 == 0, "unpadded image rows, whole DMA instructions");
  static_assert(16 * 64 * 4 + 64 * 8 <= 16 * LDR * 2, "the S partials and sums fit in rows 0-15 of the slice");
  static_assert(KS == 10 && LS == 10 && CT == 5, "the asm blocks and vmcnt immediates below are written for d = 1280");
  __shared__ __attribute__((aligned(1024))) char smem[2 * XD_SLOT];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, hh = lane >> 5, l32 = lane & 31;
  const int n_tiles = (a.T + 31) / 32;
  const int M = a.G * a.H;
  const int cb = wv * QW;
  // this workgroup's units [gb, ge), launch-relative
  int gb, ge, chunk = 0, item_split = 0;
  if (a.sk_W) {
    int b = blockIdx.x;
    if (a.sk_map) {                              // XCD-contiguous: XCD x walks chunks [x n / 8, (x + 1) n / 8)
      const int n = gridDim.x, xcd = b & 7, q = n >> 3, r = n & 7;
      b = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (b >> 3);
    }
    chunk = a.sk_c0 + b;
    const long long L0 = (long long)a.sk_lane0 * n_tiles;
    gb = (int)(max(xsk_begin(chunk, a.sk_W, a.sk_P), L0) - L0);
    ge = (int)(min(xsk_begin(chunk + 1, a.sk_W, a.sk_P), L0 + (long long)a.sk_lanes * n_tiles) - L0);
    if (gb >= ge) return;
  } else {
    const int j = blockIdx.x >> 3;
    const int item = (blockIdx.x & 7) * a.per_xcd + (a.rev ? a.per_xcd - 1 - j : j);
    if (item >= a.n_items) return;
    const int mt = item % a.n_mt, rest = item / a.n_mt;
    item_split = rest % a.splits;
    const int ln = (rest / a.splits) * a.n_mt + mt;
    gb = ln * n_tiles + item_split * n_tiles / a.splits;
    ge = ln * n_tiles + (item_split + 1) * n_tiles / a.splits;
  }
  // DMA i of a tile fills LDS bytes [1024 i, 1024 i + 1024) of the wave's slice: lane l writes image granule
  // p = 64 i + l = (row r, slot s), which holds chunk c = s ^ ((r >> 2) & 3) of row r (xchunk is an involution).
  // CPR = 20 is a multiple of 4, so that source granule r CPR + c is p ^ ((r >> 2) & 3), r >> 2 = p / 80.  Computed
  // at each issue from an opaque lane id (ten persistent offsets cost the registers the accumulators need).
  static_assert(CPR == 20, "granule = p ^ ((p / 80) & 3) needs 20 chunks per row");
  // the wave's slice of tile 0 of a lane's window (the slot is tile-blocked: xblock_kernel)
  auto ebase = [&](int ln) -> const char* {
    const int slot = a.hyp_slot[a.row_hyp[(ln / a.n_mt) * a.G]];
    return (const char*)a.enc + ((long long)slot * n_tiles * NW + wv) * (long long)IMG;
  };
  int lane_c = gb / n_tiles;                     // the current segment's lane
  const char* base_c = ebase(lane_c);
  const char* base_n = (lane_c + 1) * n_tiles < ge ? ebase(lane_c + 1) : base_c;
  auto issue = [&](int g) {                      // unit g is in lane_c or lane_c + 1 (n_tiles >= 2)
    const int lg = g / n_tiles;
    const char* src = (lg == lane_c ? base_c : base_n) + (long long)(g - lg * n_tiles) * SLOT;
    char* dst = smem + ((g - gb) & 1) * SLOT + wv * IMG;
    int lo = lane;
    asm volatile("" : "+v"(lo));
#pragma unroll
    for (int i = 0; i < LS; ++i) {
      const int p = 64 * i + lo;
      __builtin_amdgcn_global_load_lds((const void*)(src + 16 * (p ^ ((p / 80) & 3))),
                                       (__attribute__((address_space(3))) void*)(dst + 1024 * i), 16, 0, 2 /* nt */);
    }
  };
  // Segment state.  Chunks: every (row, head) column below M counts as valid whether its row is finished or not (its
  // partial is stored and never merged: xcomb skips finished rows), so a segment's setup loads nothing but q'.
  struct Seg {
    int row, hd, piece;
    bool valid;
  };
  auto seg_of = [&](int ln) -> Seg {
    const int grp = ln / a.n_mt, mt = ln - grp * a.n_mt;
    const int m = mt * 32 + l32, row0 = grp * a.G;
    Seg sg{row0, 0, a.sk_W ? chunk - xsk_chunk((long long)(a.sk_lane0 + ln) * n_tiles, a.sk_W, a.sk_P) : item_split, m < M};
    if (sg.valid) {
      const int ri = m / a.H;
      sg.row = row0 + ri;
      sg.hd = m - ri * a.H;
    }
    return sg;
  };
  unsigned long long stat_bytes = 0;             // profiler bytes of this workgroup, one atomic at its end
  auto count = [&](int ln, const Seg& sg, int g) {
    const int tb = g - ln * n_tiles, te = min(n_tiles, ge - ln * n_tiles);
    const unsigned long long nq = __popcll(__ballot(sg.valid && hh == 0));
    const long long npos = (long long)min(te * 32, a.T) - tb * 32;
    stat_bytes += nq * (unsigned long long)a.d * 2;
    if (ln % a.n_mt == 0) stat_bytes += (unsigned long long)(npos * a.d * 2);
  };
  bf16x8 qf[KS];
  auto load_q = [&](const Seg& sg) {             // unconditional: row, hd are clamped
    const bf16* qr = a.qp + ((long long)sg.row * a.H + sg.hd) * a.d + cb + 8 * hh;
#pragma unroll
    for (int s = 0; s < KS; ++s) qf[s] = *(const bf16x8*)(qr + 16 * s);
  };
  // a use of q': the compiler waits vmcnt(0) here, and no later use of q' waits
  auto q_landed = [&](const Seg& sg) {
    asm volatile("" ::"v"(qf[0]), "v"(qf[1]), "v"(qf[2]), "v"(qf[3]), "v"(qf[4]), "v"(qf[5]), "v"(qf[6]), "v"(qf[7]),
                 "v"(qf[8]), "v"(qf[9]));
    if (!sg.valid) {
#pragma unroll
      for (int s = 0; s < KS; ++s) qf[s] = bf16x8{};
    }
  };
  float* pr_row = nullptr;
  auto cap_row = [&](const Seg& sg) {            // alignment capture: the row's raw-score row (wave 0)
    pr_row = nullptr;
    if (CAP && a.probs && wv == 0 && sg.valid) {
      const int hm = a.head_map[sg.hd];
      if (hm >= 0) pr_row = a.probs + ((long long)sg.row * a.n_align + hm) * a.T;
    }
  };
  f32x16 o[CT];
  float m_run, l_run;
  auto reset = [&] {
#pragma unroll
    for (int c = 0; c < CT; ++c) o[c] = xzero16();
    m_run = -INFINITY;
    l_run = 0.f;
  };
  // the segment's partial: (m, l) and u / l as bf16.  Every wave holds the same m, l (the same S after the cross-wave
  // sum), so every valid lane stores its column's pair (equal values); the wave issues 11 stores or none.
  auto flush = [&](const Seg& sg) {
    l_run += __shfl_xor(l_run, 32, 64);
    if (sg.valid) {
      const float inv = 1.0f / l_run;
      const long long pi = ((long long)sg.piece * a.slab_rows + sg.row) * a.H + sg.hd;
      *(float2*)(a.part_ml + 2 * pi) = float2{m_run, l_run};
      xstore_u(a.part_u + (((long long)sg.piece * a.H + sg.hd) * (a.d / 16) + cb / 16) * (a.slab_rows * 16) +
                   (long long)sg.row * 16,
               a.slab_rows * 16, o, inv, hh);
    }
  };

  Seg cur = seg_of(lane_c);
  if (!a.sk_W) {                                 // items: finished rows skip, and a finished m-tile exits
    if (cur.valid) cur.valid = !(a.done && a.done[a.row_hyp[cur.row]]);
    if (!__any(cur.valid)) return;               // uniform in the workgroup
  }
  count(lane_c, cur, gb);
  load_q(cur);
  if constexpr ((ABL & 16) != 0) {               // compute-only ablation: finite constant images instead of loads
#pragma unroll
    for (int i = 0; i < 2 * LS; ++i)
      *(i32x4*)(smem + (i / LS) * SLOT + wv * IMG + 1024 * (i % LS) + 16 * lane) = i32x4{0x3c003c00, 0x3c003c00, 0x3c003c00, 0x3c003c00};
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  } else {
    issue(gb);
  }
  q_landed(cur);                                 // with the first tile, which the first tile needs anyway
  cap_row(cur);
  if constexpr ((ABL & 16) == 0) {
    if (gb + 1 < ge) issue(gb + 1);              // a whole tile of compute ahead of its use
  }
  reset();
  // A mid-chunk boundary (chunks only) after unit g, the last of segment A:
  //   tile g:     no DMA after barrier 3; after A's U MFMAs, B's q' loads and their wait (vmcnt(0): B's q' and the
  //               DMA of g + 1, which tile g + 1 needs anyway), then the DMA of g + 2;
  //   tile g + 1: after its barrier 3 and the DMA of g + 3, A's partial stores (A's o, m, l are still live: B's first
  //               U MFMAs come after), then reset for B.
  // Store acknowledgements are slow while the loads stream (tools/xattn_bench: ~12 us when waited for at once), so
  // the stores are issued after two DMAs that the next two tile waits count past them: vmcnt(10 + 10) at g + 2 and
  // g + 3 (every vector-memory operation retires in issue order: MI355X_MICROARCH.md, vmcnt), and only the wait at
  // g + 4 covers them.
  int flushed = -8, f_ops = 0;                   // unit whose barrier-3 point issued A's stores; their count (>= 10)
  bool f_pending = false;
  Seg fseg = cur;
  // LDS reads and writes that the DMA's destination may alias are inline asm: the compiler gives the tr16 intrinsic
  // no alias information and cannot tell the other accesses from the DMA's destination, and would wait vmcnt(0) --
  // drain the DMA of the next tile -- before them.  Each asm block that loads waits for its own loads (lgkmcnt(0)) and
  // marks its outputs early-clobber: an asm output that returns after the statement could be copied by the compiler
  // before it arrives.
  auto lds_addr = [](const void* p) -> unsigned {
    return (unsigned)(size_t)(__attribute__((address_space(3))) const char*)p;
  };
  for (int g = gb;; ++g) {
    int lo = lane;
    asm volatile("" : "+v"(lo));
    const int tile = g - lane_c * n_tiles;
    const bool more = g + 1 < ge, last = !more || tile == n_tiles - 1;    // last unit of this segment
    char* base = smem + ((g - gb) & 1) * SLOT;
    bf16* sE = (bf16*)(base + wv * IMG);
    bf16* sER = sE + 16 * LDR;
    if constexpr ((ABL & 16) == 0) {             // this wave's DMAs of the tile have landed: all but the younger ones
      // (the DMA of g + 1, and a boundary's partial stores issued after this tile's DMA)
      const int younger = (more ? 10 : 0) + (g == flushed + 1 || g == flushed + 2 ? f_ops : 0);
      if (younger >= 20) asm volatile("s_waitcnt vmcnt(20)" ::: "memory");
      else if (younger >= 10) asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    f32x16 sc = xzero16();
    // transposed U operand reads (see xattn_segment): rows 16 ks .. 16 ks + 15
    const int G4 = (lo >> 4) & 3, gi = lo & 15, gq = gi >> 2, gp = gi & 3;
    const int lowc = 2 * (G4 & 1) + (gp >> 1);
    const int o0 = (4 * hh + gq) * LDR + 8 * (lowc ^ hh) + 4 * (gp & 1);
    const int o1 = (8 + 4 * hh + gq) * LDR + 8 * (lowc ^ (2 + hh)) + 4 * (gp & 1);
    // the 5 column tiles' transposed fragments of one 16-row half image (two ds_read_b64_tr_b16 each, 64 B apart per c)
    auto ufrags = [&](const bf16* img, bf16x8 (&u)[CT]) {
      xi32x2 v[10];
      asm volatile(
          "ds_read_b64_tr_b16 %0, %10\n\tds_read_b64_tr_b16 %1, %11\n\t"
          "ds_read_b64_tr_b16 %2, %10 offset:64\n\tds_read_b64_tr_b16 %3, %11 offset:64\n\t"
          "ds_read_b64_tr_b16 %4, %10 offset:128\n\tds_read_b64_tr_b16 %5, %11 offset:128\n\t"
          "ds_read_b64_tr_b16 %6, %10 offset:192\n\tds_read_b64_tr_b16 %7, %11 offset:192\n\t"
          "ds_read_b64_tr_b16 %8, %10 offset:256\n\tds_read_b64_tr_b16 %9, %11 offset:256\n\t"
          "s_waitcnt lgkmcnt(0)"
          : "=&v"(v[0]), "=&v"(v[1]), "=&v"(v[2]), "=&v"(v[3]), "=&v"(v[4]), "=&v"(v[5]), "=&v"(v[6]), "=&v"(v[7]),
            "=&v"(v[8]), "=&v"(v[9])
          : "v"(lds_addr(img + o0)), "v"(lds_addr(img + o1))
          : "memory");
#pragma unroll
      for (int c = 0; c < CT; ++c) u[c] = __builtin_bit_cast(bf16x8, i32x4{v[2 * c][0], v[2 * c][1], v[2 * c + 1][0], v[2 * c + 1][1]});
    };
    // the 8 waves' float2 at byte offset `off` of their slices (slices 0-3 from pr, 4-7 from pr + 4 IMG), waited
    static_assert(IMG * 3 + 4096 + 512 <= 65536, "4 slices within one 16-bit LDS offset");
    auto read8 = [&](unsigned pr, auto offc, float2 (&t)[NW]) {
      constexpr int off = decltype(offc)::value;
      asm volatile(
          "ds_read_b64 %0, %8 offset:%10\n\tds_read_b64 %1, %8 offset:%11\n\t"
          "ds_read_b64 %2, %8 offset:%12\n\tds_read_b64 %3, %8 offset:%13\n\t"
          "ds_read_b64 %4, %9 offset:%10\n\tds_read_b64 %5, %9 offset:%11\n\t"
          "ds_read_b64 %6, %9 offset:%12\n\tds_read_b64 %7, %9 offset:%13\n\t"
          "s_waitcnt lgkmcnt(0)"
          : "=&v"(t[0]), "=&v"(t[1]), "=&v"(t[2]), "=&v"(t[3]), "=&v"(t[4]), "=&v"(t[5]), "=&v"(t[6]), "=&v"(t[7])
          : "v"(pr), "v"(pr + 4 * IMG), "i"(off), "i"(off + IMG), "i"(off + 2 * IMG), "i"(off + 3 * IMG)
          : "memory");
    };
    bf16x8 u0[CT], u1[CT];
    if constexpr ((ABL & 7) != 7) {
      const int l32o = lo & 31, gg = (l32o >> 2) & 3;
      const bf16* rb = l32o < 16 ? sE + l32o * LDR : sER + (l32o - 16) * LDR;
      const bf16* s0 = rb + 8 * (hh ^ gg);
      const bf16* s1 = rb + 8 * ((2 + hh) ^ gg);
      bf16x8 ea[KS];
#pragma unroll
      for (int s = 0; s < KS; ++s) ea[s] = *(const bf16x8*)(((s & 1) ? s1 : s0) + 32 * (s >> 1));
      ufrags(sE, u0);                            // rows 0-15: their bytes are reused below
#pragma unroll
      for (int s = 0; s < KS; ++s) sc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ea[s], qf[s], sc, 0, 0, 0);
      // the partials into the dead rows 0-15 of this wave's slice (LDS is in order: after the reads above).  The
      // compiler's hazard recognizer does not look into inline asm: the wait states between the last S MFMA writing
      // sc and the first store reading it (a 16-pass MFMA's result read by a non-MFMA: 18) are spelled out.
      const unsigned px = lds_addr(sE) + 8 * lane;
      asm volatile("s_nop 15\n\ts_nop 3" : "+v"(sc)::"memory");
#define XD_W2(k_) asm volatile("ds_write_b64 %0, %1 offset:%2" ::"v"(px), "v"(float2{sc[2 * k_], sc[2 * k_ + 1]}), "i"(512 * k_) : "memory")
      XD_W2(0); XD_W2(1); XD_W2(2); XD_W2(3); XD_W2(4); XD_W2(5); XD_W2(6); XD_W2(7);
#undef XD_W2
      xbarrier<true>();
      // wave w sums registers 2w, 2w + 1 over the waves in order 0..7 (xattn_segment's order)
      float2 t[NW];
      read8(lds_addr(base) + 8 * (wv * 64 + lane), std::integral_constant<int, 0>{}, t);
      float2 v = t[0];
#pragma unroll
      for (int w2 = 1; w2 < NW; ++w2) {
        v.x += t[w2].x;
        v.y += t[w2].y;
      }
      asm volatile("ds_write_b64 %0, %1 offset:4096" ::"v"(px), "v"(v) : "memory");
      xbarrier<true>();
      read8(lds_addr(base) + 8 * lane, std::integral_constant<int, 4096>{}, t);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        sc[2 * k] = t[k].x;
        sc[2 * k + 1] = t[k].y;
      }
      ufrags(sER, u1);                           // rows 16-31: untouched by the partials
    }
    const int t0 = tile * 32;
    if (t0 + 32 > a.T) {
#pragma unroll
      for (int r = 0; r < 16; ++r)
        if (t0 + 8 * (r >> 2) + 4 * hh + (r & 3) >= a.T) sc[r] = -INFINITY;
    }
    if (CAP && pr_row) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int t = t0 + 8 * (r >> 2) + 4 * hh + (r & 3);
        if (t < a.T) pr_row[t] = sc[r];
      }
    }
    // every wave's reads of this slot are complete: its slices take unit g + 2 (the CAP stores above are older than
    // these DMAs, so the next tile's counted wait covers them).  At a segment's end that waits for the next q'.
    if constexpr ((ABL & 7) != 7) xbarrier<true>();
    if constexpr ((ABL & 16) == 0) {
      if (!(last && more) && g + 2 < ge) issue(g + 2);
    }
    if (f_pending) {                             // the previous segment's partial, after this tile's DMA (see above)
      flush(fseg);
      f_ops = __any(fseg.valid) ? 10 : 0;        // a lower bound of the store instructions issued (11 or 0)
      flushed = g;
      f_pending = false;
      reset();
    }
    if constexpr ((ABL & 7) != 7) {
      float mx = sc[0];
#pragma unroll
      for (int r = 1; r < 16; ++r) mx = fmaxf(mx, sc[r]);
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      if (__any(mx > m_run + XTHR)) {
        const float mn = fmaxf(m_run, mx);
        const float alpha = __builtin_amdgcn_exp2f(m_run - mn);
        l_run *= alpha;
#pragma unroll
        for (int c = 0; c < CT; ++c)
#pragma unroll
          for (int r = 0; r < 16; ++r) o[c][r] *= alpha;
        m_run = mn;
      }
      bf16x8 pf[2];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float p = __builtin_amdgcn_exp2f(sc[r] - m_run);
        l_run += p;
        pf[r >> 3][r & 7] = f2bf(p);
      }
#pragma unroll
      for (int c = 0; c < CT; ++c) {
        o[c] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(u0[c], pf[0], o[c], 0, 0, 0);
        o[c] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(u1[c], pf[1], o[c], 0, 0, 0);
      }
    }
    if (last) {
      if (!more) {
        flush(cur);
        break;
      }
      // the next lane's segment (chunks only): A's partial waits for tile g + 1 (no partial is pending here: a
      // pending one is stored at the first tile of its successor, before that tile's end); B's q' lands with the DMA
      // of g + 1
      fseg = cur;
      f_pending = true;
      cur = seg_of(lane_c + 1);
      load_q(cur);                               // loaded and waited for in one block: a load whose wait the compiler
                                                 // could not place before the loop's next use of q' would be waited
                                                 // for (vmcnt(0)) at every tile
      ++lane_c;
      base_c = base_n;
      base_n = (lane_c + 1) * n_tiles < ge ? ebase(lane_c + 1) : base_c;
      count(lane_c, cur, g + 1);
      q_landed(cur);
      cap_row(cur);
      if constexpr ((ABL & 16) == 0) {
        if (g + 2 < ge) issue(g + 2);
      }
    }
  }
  if (a.stat && tid == 0) atomicAdd(a.stat + (blockIdx.x & (STAT_SLOTS - 1)), stat_bytes);
}

// ------------------------------------------------------------------------------------------------------
struct XCombArgs {
  const bf16* part_u; const float* part_ml; int splits; long long slab_rows;
  long long sk_W; int sk_P, sk_lane0, n_tiles, G;   // LDS-DMA chunks: a row's piece count follows from its lane
  const bf16* wvb; const float* bv;      // this layer's V projection packed [H][d/16][64][16], bias [d]
  const int* row_hyp; const int* done;
  bf16* out; long long ldo;
  int rows, H, d, T;
  float* probs; const int* head_map; int n_align;
};

// grid ceil(rows / RT) x H flattened (xcd_block), 8 waves.  D[r][j] = sum_c u[r][h][c] Wv[h*64 + j][c]: A = merged u rows (built
// from the bf16 split partials while loading), B = Wv rows.  Wave w reduces c in [w d/8, (w+1) d/8): its
// partial and weight loads are issued KB k-steps at a time (one memory round trip per batch, not per
// k-step).  The merged u is split into bf16 hi + lo parts (two MFMAs), so the V projection sees u to
// ~16 bits instead of 8.  The 8 partial products are summed through LDS in a fixed order.
// RT = rows per block, 32 or 16.  With 16, MFMA rows 16..31 repeat rows 0..15 (same addresses: no extra bytes)
// and are not stored, so every output keeps the 32-row form's arithmetic bit for bit while the grid doubles
// (a block's partial bytes halve; the Wv_h panel is the same).
// EXACT (opt-in, see launch_xcomb_vo): the launch's split count is MAXS itself, so no load carries a per-split guard.  The
// guarded form branches around every (m, l) load and waits for each in turn (9 round trips before the first partial
// load at 4 splits); unguarded, the compiler issues them together and interleaves the partial loads with the MFMAs.
// A load batch also holds 20 / ns k-steps instead of 20 / (the next power of two): 5 splits in 3 batches, not 5.
template <int KS8, int MAXS, int RT = 32, bool EXACT = false>
__global__ __launch_bounds__(512) void xcomb_vo_kernel(XCombArgs a) {
  constexpr int KB = (20 / MAXS) < KS8 ? (20 / MAXS) : KS8;   // k-steps per load batch (<= 20 partial loads)
  __shared__ float sR[8][2][16][64];
  __shared__ float sML[32][2];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, hh = lane >> 5, l32 = lane & 31;
  int bx, h;
  xcd_block((a.rows + RT - 1) / RT, bx, h);
  const int r = bx * RT + (l32 & (RT - 1));
  const int rc = min(r, a.rows - 1);
  const long long sstride = a.slab_rows * a.H;          // (row, head) pairs per split slab
  float w[MAXS];
  float Mx = -INFINITY, L = 0.f;
  int ns = EXACT ? MAXS : a.splits;
  if (!EXACT && a.sk_W) {                // the chunks this row's window spans (xattn_dma_kernel)
    const long long f = (long long)(a.sk_lane0 + rc / a.G) * a.n_tiles;
    ns = xsk_chunk(f + a.n_tiles - 1, a.sk_W, a.sk_P) - xsk_chunk(f, a.sk_W, a.sk_P) + 1;
  }
#pragma unroll
  for (int s = 0; s < MAXS; ++s) w[s] = 0.f;
  {
    // every load is issued regardless of the row's state (rows past the end clamped; a finished row's
    // partials are stale but finite, and its output is never stored), so nothing waits on `done`
    const float* ml = a.part_ml + 2 * ((long long)rc * a.H + h);
    // every (m, l) pair requested before any is used, at a clamped split index (loaded behind the per-split guards,
    // each waited for the one before it: up to 9 round trips); the arithmetic below keeps its guards and order
    float pm[MAXS], pl[MAXS];
#pragma unroll
    for (int s = 0; s < MAXS; ++s) {
      const int sc = min(s, ns - 1);
      pm[s] = ml[2 * sc * sstride];
      pl[s] = ml[2 * sc * sstride + 1];
    }
#pragma unroll
    for (int s = 0; s < MAXS; ++s)
      if (s < ns) Mx = fmaxf(Mx, pm[s]);
#pragma unroll
    for (int s = 0; s < MAXS; ++s)
      if (s < ns) {
        w[s] = pl[s] * __builtin_amdgcn_exp2f(pm[s] - Mx);
        L += w[s];
      }
    const float inv = 1.0f / L;
#pragma unroll
    for (int s = 0; s < MAXS; ++s) w[s] *= inv;
  }
  f32x16 acc[2] = {xzero16(), xzero16()};
  const int kb0 = wv * KS8;               // this wave's first 16-column block
  const long long kstride = a.slab_rows * 16;
  const bf16* pu = a.part_u + ((long long)h * (a.d / 16) + kb0) * kstride + (long long)rc * 16 + 8 * hh;
  const bf16* w0 = a.wvb + (((long long)h * (a.d / 16) + kb0) * 64 + l32) * 16 + 8 * hh;
  const bf16* w1 = w0 + 32 * 16;
  const long long pstride = (long long)a.H * a.d * a.slab_rows;   // one split slab
#pragma unroll
  for (int s0 = 0; s0 < KS8; s0 += KB) {
    bf16x8 pv[KB][MAXS], wa[KB], wb[KB];
#pragma unroll
    for (int k = 0; k < KB; ++k) {
      if (s0 + k >= KS8) break;
      wa[k] = *(const bf16x8*)(w0 + (s0 + k) * 64 * 16);
      wb[k] = *(const bf16x8*)(w1 + (s0 + k) * 64 * 16);
#pragma unroll
      for (int sp = 0; sp < MAXS; ++sp)
        if (sp < ns) pv[k][sp] = *(const bf16x8*)(pu + sp * pstride + (s0 + k) * kstride);
        else pv[k][sp] = bf16x8{};
    }
#pragma unroll
    for (int k = 0; k < KB; ++k) {
      if (s0 + k >= KS8) break;
      float u[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int sp = 0; sp < MAXS; ++sp)
        if (sp < ns) {
#pragma unroll
          for (int i = 0; i < 8; ++i) u[i] = fmaf(w[sp], bf2f(pv[k][sp][i]), u[i]);
        }
      bf16x8 uh, ul;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        uh[i] = f2bf(u[i]);
        ul[i] = f2bf(u[i] - bf2f(uh[i]));
      }
      acc[0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(uh, wa[k], acc[0], 0, 0, 0);
      acc[0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ul, wa[k], acc[0], 0, 0, 0);
      acc[1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(uh, wb[k], acc[1], 0, 0, 0);
      acc[1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ul, wb[k], acc[1], 0, 0, 0);
    }
  }
#pragma unroll
  for (int jt = 0; jt < 2; ++jt)
#pragma unroll
    for (int i = 0; i < 16; ++i) sR[wv][jt][i][lane] = acc[jt][i];
  if (wv == 0 && hh == 0) {
    sML[l32][0] = Mx;
    sML[l32][1] = L;
  }
  __syncthreads();
  for (int idx = tid; idx < 2 * 16 * 64; idx += 512) {
    const int jt = idx >> 10, i = (idx >> 6) & 15, ln = idx & 63;
    float v = sR[0][jt][i][ln];
#pragma unroll
    for (int w2 = 1; w2 < 8; ++w2) v += sR[w2][jt][i][ln];
    const int j = 32 * jt + (ln & 31);
    const int tr = 8 * (i >> 2) + 4 * (ln >> 5) + (i & 3);
    if (tr >= RT) continue;
    const int rr = bx * RT + tr;
    if (rr < a.rows && !(a.done && a.done[a.row_hyp[rr]]))
      a.out[(long long)rr * a.ldo + h * 64 + j] = f2bf(v + a.bv[h * 64 + j]);
  }
  if (a.probs) {
    const int hm = a.head_map[h];
    if (hm >= 0) {
      for (int idx = tid; idx < RT * a.T; idx += 512) {
        const int ri = idx / a.T, t = idx - ri * a.T;
        const int rr = bx * RT + ri;
        if (rr >= a.rows) continue;
        float* p = a.probs + ((long long)rr * a.n_align + hm) * a.T + t;
        *p = __builtin_amdgcn_exp2f(*p - sML[ri][0]) / sML[ri][1];
      }
    }
  }
}

// ------------------------------------------------------------------------------------------------------
// fp8 cross memory (opt-in, engine option cross_fp8): a window's encoder output stored as OCP e4m3 with one
// scale per position, E[t] ~= e4m3(E[t] * 448 / amax_t) * (amax_t / 448), amax_t = max_c |E[t][c]| (an all-zero
// row stores zeros with scale 0).  Halves the bytes xattn streams per layer and step.  One wave per position;
// lane j converts groups of 4 consecutive columns (v_cvt_pk_fp8_f32, round to nearest even).
__global__ __launch_bounds__(256) void xquant8_kernel(const bf16* __restrict__ enc, long long rows, int d,
                                                      unsigned char* __restrict__ out, float* __restrict__ scale) {
  constexpr int MAXG = 5;                // d <= 1280 = 5 x 64 lanes x 4 columns
  const long long row = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  const bf16* x = enc + row * d;
  float v[MAXG][4];
  float amax = 0.f;
#pragma unroll
  for (int g = 0; g < MAXG; ++g) {
    const int c = (g * 64 + lane) * 4;
    if (c < d) {
      const bf16x4 q = *(const bf16x4*)(x + c);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        v[g][e] = bf2f(q[e]);
        amax = fmaxf(amax, fabsf(v[g][e]));
      }
    }
  }
  amax = wave_max(amax);
  const float inv = amax > 0.f ? 448.0f / amax : 0.f;
#pragma unroll
  for (int g = 0; g < MAXG; ++g) {
    const int c = (g * 64 + lane) * 4;
    if (c < d) {
      int w = __builtin_amdgcn_cvt_pk_fp8_f32(v[g][0] * inv, v[g][1] * inv, 0, false);
      w = __builtin_amdgcn_cvt_pk_fp8_f32(v[g][2] * inv, v[g][3] * inv, w, true);
      *(int*)(out + row * d + c) = w;
    }
  }
  if (lane == 0) scale[row] = amax / 448.0f;
}

void launch_xquant8(const bf16* enc, long long rows, int d, unsigned char* out, float* scale, hipStream_t st) {
  if (rows <= 0) return;
  if (d % 4 != 0 || d > 1280) throw std::runtime_error("xquant8: n_state must be a multiple of 4, <= 1280");
  hipLaunchKernelGGL(xquant8_kernel, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, st, enc, rows, d, out, scale);
  WM_LAUNCH_CHECK("xquant8_kernel");
}

// ------------------------------------------------------------------------------------------------------
// Tile-blocked encoder-output slots (the bf16 factored form): slot s holds [n_tiles][NW][32][QW] bf16, n_tiles =
// ceil(T / 32), rows past T zero; tile t, wave w's block is rows 32 t .. 32 t + 31, columns w QW .. w QW + QW - 1 of
// the window's [T][d] encoder output, row-major inside the block.  xblock_kernel writes it from row-major windows,
// xunblock_kernel reads windows back out (the alignment pass's K/V projection).  One thread per 16-B chunk.
void xattn_geometry(int d, int& qw, int& nw) {
  switch (d) {
    case 384: qw = 96; nw = 4; return;
    case 512: qw = 64; nw = 8; return;
    case 768: qw = 96; nw = 8; return;
    case 1024: qw = 128; nw = 8; return;
    case 1280: qw = 160; nw = 8; return;
    default: throw std::runtime_error("xattn: unsupported n_state " + std::to_string(d));
  }
}

long long xblock_slot_elems(int T, int d) { return (long long)((T + 31) / 32) * 32 * d; }

__global__ __launch_bounds__(256) void xblock_kernel(const bf16* __restrict__ src, int B, int T, int d, int qw, int nw,
                                                     bf16* __restrict__ dst, int to_blocked) {
  const int cpr = qw / 8, nt = (T + 31) / 32;
  const long long per = (long long)nt * 32 * d / 8;         // 16-B chunks per blocked slot
  const long long n = per * B;
  for (long long q = (long long)blockIdx.x * 256 + threadIdx.x; q < n; q += (long long)gridDim.x * 256) {
    const long long b = q / per;
    long long rem = q - b * per;
    const int c = (int)(rem % cpr);
    rem /= cpr;
    const int r = (int)(rem % 32);
    rem /= 32;
    const int w = (int)(rem % nw);
    const int t = (int)(rem / nw) * 32 + r;
    const long long rm = ((long long)b * T + t) * d + w * qw + c * 8;     // row-major element offset
    if (to_blocked) {
      i32x4 v = i32x4{0, 0, 0, 0};
      if (t < T) v = *(const i32x4*)(src + rm);
      *(i32x4*)(dst + q * 8) = v;
    } else if (t < T) {
      *(i32x4*)(dst + rm) = *(const i32x4*)(src + q * 8);
    }
  }
}

// B row-major windows [B][T][d] -> B blocked slots starting at dst (to_blocked), or back (from blocked slots)
void launch_xblock(const bf16* src, int B, int T, int d, bf16* dst, bool to_blocked, hipStream_t st) {
  if (B <= 0) return;
  int qw = 0, nw = 0;
  xattn_geometry(d, qw, nw);
  const long long n = (long long)B * xblock_slot_elems(T, d) / 8;
  const int blocks = (int)std::min<long long>((n + 255) / 256, 1 << 16);
  hipLaunchKernelGGL(xblock_kernel, dim3(blocks), dim3(256), 0, st, src, B, T, d, qw, nw, dst, to_blocked ? 1 : 0);
  WM_LAUNCH_CHECK("xblock_kernel");
}

// ------------------------------------------------------------------------------------------------------
// host launchers

void launch_xpack(const bf16* ckv_w, bf16* wkt, bf16* wvb, int L, int H, int d, hipStream_t st) {
  const long long total = (long long)L * H * d * 64;
  const int blocks = (int)std::min<long long>((total + 255) / 256, 65536);
  hipLaunchKernelGGL(xpack_kernel, dim3(blocks), dim3(256), 0, st, ckv_w, wkt, wvb, L, H, d);
  WM_LAUNCH_CHECK("xpack_kernel");
}

void launch_xq(const bf16* q, long long ldq, const CrossFuse& fz, const bf16* wkt, bf16* qp, int rows, int H, int d,
               hipStream_t st) {
  if (rows <= 0) return;
  if (d != H * 64) throw std::runtime_error("xq: n_state must be n_head * 64");
  if (fz.q_part && fz.q_splits > XMAXS) throw std::runtime_error("xq: too many cq split-K slabs");
  XQArgs a{};
  a.q = q; a.ldq = ldq; a.q_part = fz.q_part; a.q_splits = fz.q_splits; a.q_rows = fz.q_rows; a.q_bias = fz.q_bias;
  a.wkt = wkt; a.qp = qp; a.rows = rows; a.H = H; a.d = d;
  a.scale = 0.125f * 1.4426950408889634f;
  const dim3 grid((rows + 31) / 32 * H * ((d / 32 + 7) / 8));   // flattened (row tile, head, column group)
  hipLaunchKernelGGL(xq_kernel, grid, dim3(256), 0, st, a);
  WM_LAUNCH_CHECK("xq_kernel");
}

// CUs of the current device (one item per CU at a time: the kernels' LDS allows one workgroup per CU)
static int xattn_cus() {
  static const int n = [] {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      v = 256;
    return std::max(1, v);
  }();
  return n;
}

// Key splits of a pass.  A function of the whole pass, so slicing a pass into launches never changes a
// row's arithmetic: the count that minimises the launch model below (round 5: about 1.75 rounds of 256
// one-workgroup CUs; measured on the 150-window large-v3 decode: 1 / 2 / 3 / 4 / 5 splits -> 522 / 564 / 450 /
// 510 / 483 ms of attention per bench step), at most 8, at least one 32-position tile per split, and the bf16
// partial slabs capped at 256 MB.
int xattn_splits(int plan_rows, int group, int H, int T, int d) {
  static const int forced = [] {
    const char* e = std::getenv("VLOG_AMD_XSPLITS");
    return e ? std::atoi(e) : 0;
  }();
  // At most 8 splits: the split merge (xcomb) takes 9-16 splits in 10 dependent load batches (5 for 5-8), and the
  // row set's small tail passes (16 splits by the rule below) paid more there than the attention gained (variable
  // workload: 2657-2680 RTFx uncapped, 2698-2711 capped at 4-8, profiles/ab_r05_xsplits_max.txt).
  // VLOG_AMD_XSPLITS_MAX overrides the cap (A/B).
  static const int cap_env = [] {
    const char* e = std::getenv("VLOG_AMD_XSPLITS_MAX");
    return e ? std::max(0, std::atoi(e)) : 0;    // 0: the rule
  }();
  const int cap = cap_env > 0 ? cap_env : 8;
  const int groups = std::max(1, plan_rows / std::max(group, 1));
  const long long n_mt = ((long long)group * H + 31) / 32;
  const long long items = groups * n_mt;
  const int n_tiles = (T + 31) / 32;
  // Round 6: the split count minimises a measured model of the launch (tools/xattn_bench key-split sweep over 16-200
  // windows, profiles/xattn_bench_r06_split_sweep.txt): the items run in rounds of one per CU, an item of n tiles
  // takes 5.7 + n t us (t = 3.2 with the chip full, 2.87 with fewer than 94 % of the CUs busy), and the merge reads
  // one partial per row and split (0.017 us each).  It fills ONE round where it can (64 windows: 4 splits, 45.0 us
  // against 57.9 for the round-5 rule's 7; 128: 2, 80.5 against 96.9) and keeps 3 at the headline's 150.
  // VLOG_AMD_XSPLITS_RULE=0: the round-5 rule (about 1.75 rounds, A/B).
  static const int rule_env = [] {
    const char* e = std::getenv("VLOG_AMD_XSPLITS_RULE");
    return e ? std::atoi(e) : 1;
  }();
  const int s_max = std::max(1, std::min(std::min(cap, XMAXS), n_tiles));
  int s = (int)((448 + items / 2) / items);
  if (rule_env && n_mt == 1) {                  // greedy decode passes (the model was measured on one m-tile per window;
                                                // a prompt pass's m-tiles share E in L2: 3 splits instead of 1 at 150
                                                // windows x 3 rows cost the uniform bench 0.7 %, ab_r06_xsplits_rule)
    const long long cus = xattn_cus();
    double best = 1e300;
    for (int c = 1; c <= s_max; ++c) {
      const double tiles = (double)n_tiles / c;
      double t = 0.017 * plan_rows * c;
      for (long long left = items * c; left > 0; left -= cus) {
        const long long busy = std::min(left, cus);
        t += 5.7 + tiles * (busy * 100 >= cus * 94 ? 3.2 : 2.87);
      }
      if (t < best - 1e-9) {
        best = t;
        s = c;
      }
    }
  }
  if (forced > 0) s = forced;
  s = std::max(1, std::min(s, s_max));
  const long long slab = (long long)plan_rows * H * d * 2;
  while (s > 1 && slab * s > (256LL << 20)) --s;
  return s;
}

// The factored attention's plan for a pass: the LDS-DMA chunk cut (stream-K, xattn_dma_kernel) where it applies --
// `chunks_ok` (the engine: LDS-DMA form, bf16 cross memory, no cache-policy / walk-order experiment) and one m-tile
// per window group -- else xattn_splits' key splits.  `slabs` = partial slabs the pass writes (scratch sizing, and
// the merge's bound).  P = the CU count (one 160 KB workgroup per CU), at most one chunk per 7th of a window's tiles
// so a window spans at most 8 chunks.
XPlan xattn_plan(int plan_rows, int group, int H, int T, int d, bool chunks_ok) {
  XPlan p;
  p.slabs = xattn_splits(plan_rows, group, H, T, d);
  if (!chunks_ok || d != XD_NW * XD_QW || group * H > 32 || plan_rows < group) return p;
  const int ncu = xattn_cus();
  const int n_tiles = (T + 31) / 32;
  const long long W = (long long)(plan_rows / group) * n_tiles;
  const int min_chunk = std::max(2, (n_tiles + 6) / 7);
  static const int p_env = [] {                         // VLOG_AMD_XCHUNK_P: chunk count override (A/B)
    const char* e = std::getenv("VLOG_AMD_XCHUNK_P");
    return e ? std::atoi(e) : 0;
  }();
  const int P = (int)std::max<long long>(1, std::min<long long>(p_env > 0 ? p_env : ncu, W / min_chunk));
  const long long per = W / P;                           // >= min_chunk unless W < min_chunk (one chunk)
  p.slabs = (int)std::min<long long>(XMAXS, (n_tiles + per - 1) / per + 1);
  p.sk_W = W;
  p.sk_P = P;
  return p;
}

static int g_xattn_abl = [] {            // ablation / load-policy experiments (VLOG_AMD_XABL); product: 0
  const char* e = std::getenv("VLOG_AMD_XABL");
  return e ? std::atoi(e) : 0;
}();
void xattn_set_ablation(int abl) { g_xattn_abl = abl; }

void launch_xattn(const bf16* qp, const void* enc, const float* escale, const int* hyp_slot, const int* row_hyp,
                  const int* done, int rows, long long slab_rows, int group, int H, int T, int d, const XPlan& plan, int rev,
                  int keep, int dma, int lane0, bf16* part_u,
                  float* part_ml, float* probs, const int* head_map, int n_align, unsigned long long* stat,
                  hipStream_t st, hipEvent_t ev0, hipEvent_t ev1) {
  if (rows <= 0) return;
  if (group <= 0 || rows % group != 0) throw std::runtime_error("xattn: rows must be a multiple of the group");
  const int splits = plan.slabs, n_tiles = (T + 31) / 32;
  if (splits < 1 || splits > XMAXS || (!plan.sk_W && splits > n_tiles)) throw std::runtime_error("xattn: bad key splits");
  const bool dma_form = dma && !escale && d == XD_NW * XD_QW && keep == 0;
  if (plan.sk_W && (keep != 0 || rev != 0 || group * H > 32 || lane0 < 0 ||
                    (long long)(lane0 + rows / group) * n_tiles > plan.sk_W))
    throw std::runtime_error("xattn: chunk plan does not match the launch");
  XAttnArgs a{};
  a.qp = qp; a.enc = (const bf16*)enc; a.escale = escale; a.hyp_slot = hyp_slot; a.row_hyp = row_hyp; a.done = done;
  a.H = H; a.T = T; a.d = d; a.G = group; a.n_mt = (group * H + 31) / 32; a.splits = splits; a.rev = rev; a.keep = keep;
  const long long items = (long long)(rows / group) * a.n_mt * splits;
  if (items > (1LL << 30)) throw std::runtime_error("xattn: too many work items");
  a.n_items = (int)items;
  a.per_xcd = (a.n_items + 7) / 8;
  a.slab_rows = slab_rows; a.part_u = part_u; a.part_ml = part_ml;
  a.probs = probs; a.head_map = head_map; a.n_align = n_align; a.stat = stat; a.abl = g_xattn_abl;
  dim3 grid(a.per_xcd * 8);
  if (plan.sk_W) {                       // the chunks that hold this launch's lanes (a sliced pass: the same pieces)
    a.sk_W = plan.sk_W; a.sk_P = plan.sk_P; a.sk_lane0 = lane0; a.sk_lanes = rows / group;
    const long long g0 = (long long)lane0 * n_tiles, g1 = (long long)(lane0 + a.sk_lanes) * n_tiles;
    a.sk_c0 = xsk_chunk(g0, plan.sk_W, plan.sk_P);
    a.sk_nch = xsk_chunk(g1 - 1, plan.sk_W, plan.sk_P) + 1 - a.sk_c0;
    static const int map_env = [] {       // XCD-contiguous chunks (default; 0: chunk = block id): 3-7 % faster in
      const char* e = std::getenv("VLOG_AMD_XCHUNK_MAP");   // tools/xattn_bench at 128-256 windows
      return e ? std::atoi(e) : 1;
    }();
    a.sk_map = map_env;
    // the LDS-DMA kernel walks a chunk per workgroup; the register form takes its segments as items (xsk_item)
    grid = dma_form ? dim3(a.sk_nch)
                    : dim3(xsk_item_blocks(plan.sk_W, plan.sk_P, a.sk_c0, a.sk_nch, lane0, a.sk_lanes, n_tiles));
  }
#define XA_LAUNCH_C(QW_, NW_, DP_, F8_, CAP_)                                                                      \
  if (ev0) hipExtLaunchKernelGGL((xattn_kernel<QW_, NW_, DP_, F8_, 0, CAP_>), grid, dim3(NW_ * 64), 0, st, ev0, ev1, 0, a); \
  else hipLaunchKernelGGL((xattn_kernel<QW_, NW_, DP_, F8_, 0, CAP_>), grid, dim3(NW_ * 64), 0, st, a);
#define XA_LAUNCH_F(QW_, NW_, DP_, F8_)                                                                            \
  if (probs) { XA_LAUNCH_C(QW_, NW_, DP_, F8_, true) } else { XA_LAUNCH_C(QW_, NW_, DP_, F8_, false) }
#define XA_LAUNCH(QW_, NW_, DP_) XA_LAUNCH_F(QW_, NW_, DP_, false)
  if (a.abl) {                           // microbenchmark ablations (tools/xattn_bench): d = 1280, default form only
    if (d != 1280) throw std::runtime_error("xattn: ablations are built for n_state 1280 only");
    if (dma_form) {                      // LDS-DMA form: loads only (7) or compute only (16)
      switch (a.abl) {
        case 7: hipLaunchKernelGGL((xattn_dma_kernel<7>), grid, dim3(XD_NW * 64), 0, st, a); break;
        case 16: hipLaunchKernelGGL((xattn_dma_kernel<16>), grid, dim3(XD_NW * 64), 0, st, a); break;
        default: throw std::runtime_error("xattn: unsupported ablation of the LDS-DMA form");
      }
      WM_LAUNCH_CHECK("xattn_dma_kernel");
      return;
    }
#define XA_ABL(F8_, AB_) \
    case AB_: hipLaunchKernelGGL((xattn_kernel<160, 8, 1, F8_, AB_>), grid, dim3(512), 0, st, a); break;
    if (escale) {
      switch (a.abl) { XA_ABL(true, 1) XA_ABL(true, 2) XA_ABL(true, 4) XA_ABL(true, 7) XA_ABL(true, 8) XA_ABL(true, 16)
                       XA_ABL(true, 23) XA_ABL(true, 39) default: throw std::runtime_error("xattn: unsupported ablation"); }
    } else {
      switch (a.abl) { XA_ABL(false, 1) XA_ABL(false, 2) XA_ABL(false, 4) XA_ABL(false, 7) XA_ABL(false, 8)
                       XA_ABL(false, 16) XA_ABL(false, 23) XA_ABL(false, 39) default: throw std::runtime_error("xattn: unsupported ablation"); }
    }
#undef XA_ABL
    WM_LAUNCH_CHECK("xattn_kernel");
    return;
  }
  if (escale) {                          // fp8 cross memory: the default forms only
    switch (d) {
      case 384: XA_LAUNCH_F(96, 4, 1, true); break;
      case 512: XA_LAUNCH_F(64, 8, 1, true); break;
      case 768: XA_LAUNCH_F(96, 8, 1, true); break;
      case 1024: XA_LAUNCH_F(128, 8, 1, true); break;
      case 1280: XA_LAUNCH_F(160, 8, 1, true); break;
      default: throw std::runtime_error("xattn: unsupported n_state " + std::to_string(d));
    }
    WM_LAUNCH_CHECK("xattn_kernel");
    return;
  }
  if (dma_form) {
    if (probs) {
      if (ev0) hipExtLaunchKernelGGL((xattn_dma_kernel<0, true>), grid, dim3(XD_NW * 64), 0, st, ev0, ev1, 0, a);
      else hipLaunchKernelGGL((xattn_dma_kernel<0, true>), grid, dim3(XD_NW * 64), 0, st, a);
    } else {
      if (ev0) hipExtLaunchKernelGGL((xattn_dma_kernel<0, false>), grid, dim3(XD_NW * 64), 0, st, ev0, ev1, 0, a);
      else hipLaunchKernelGGL((xattn_dma_kernel<0, false>), grid, dim3(XD_NW * 64), 0, st, a);
    }
    WM_LAUNCH_CHECK("xattn_dma_kernel");
    return;
  }
  // 8 waves x d/8 columns (4 x d/4 at d = 384), one tile staged ahead: 80 KB of E in flight per CU at d = 1280
  // (retired forms, DESIGN.md §6: 4 waves two tiles ahead, 10 waves x 128 columns, LDS-DMA split staging, and
  // block-shared images fed by whole-row loads: each slower in the step)
  switch (d) {
    case 384: XA_LAUNCH(96, 4, 1); break;
    case 512: XA_LAUNCH(64, 8, 1); break;
    case 768: XA_LAUNCH(96, 8, 1); break;
    case 1024: XA_LAUNCH(128, 8, 1); break;
    case 1280: XA_LAUNCH(160, 8, 1); break;
    default: throw std::runtime_error("xattn: unsupported n_state " + std::to_string(d));
  }
#undef XA_LAUNCH
#undef XA_LAUNCH_F
#undef XA_LAUNCH_C
  WM_LAUNCH_CHECK("xattn_kernel");
}

void launch_xcomb_vo(const bf16* part_u, const float* part_ml, const XPlan& plan, int lane0, long long slab_rows,
                     const bf16* wvb, const float* bv, const int* row_hyp, const int* done, bf16* out, long long ldo, int rows,
                     int group, int H, int d, int T, float* probs, const int* head_map, int n_align, hipStream_t st) {
  if (rows <= 0) return;
  const int splits = plan.slabs;
  XCombArgs a{};
  a.part_u = part_u; a.part_ml = part_ml; a.splits = splits; a.slab_rows = slab_rows; a.wvb = wvb; a.bv = bv;
  a.sk_W = plan.sk_W; a.sk_P = plan.sk_P; a.sk_lane0 = lane0; a.n_tiles = (T + 31) / 32; a.G = group;
  a.row_hyp = row_hyp; a.done = done; a.out = out; a.ldo = ldo; a.rows = rows; a.H = H; a.d = d; a.T = T;
  a.probs = probs; a.head_map = head_map; a.n_align = n_align;
  // 16-row blocks unless the grid already fills the chip with 32-row ones (VLOG_AMD_XCOMB_RT=32|16 forces)
  static const int rt_forced = [] {
    const char* e = std::getenv("VLOG_AMD_XCOMB_RT");
    return e ? std::atoi(e) : 0;
  }();
  const int rt = rt_forced == 16 || rt_forced == 32 ? rt_forced : ((rows + 31) / 32 * H >= 256 ? 32 : 16);
  const dim3 grid((rows + rt - 1) / rt * H);           // flattened (row tile, head): xcd_block
#define XC_RT(KS8_, MS_)                                                                                          \
  if (rt == 16) hipLaunchKernelGGL((xcomb_vo_kernel<KS8_, MS_, 16>), grid, dim3(512), 0, st, a);                  \
  else hipLaunchKernelGGL((xcomb_vo_kernel<KS8_, MS_, 32>), grid, dim3(512), 0, st, a);
#define XC_RTX(KS8_, MS_)                                                                                         \
  if (rt == 16) hipLaunchKernelGGL((xcomb_vo_kernel<KS8_, MS_, 16, true>), grid, dim3(512), 0, st, a);            \
  else hipLaunchKernelGGL((xcomb_vo_kernel<KS8_, MS_, 32, true>), grid, dim3(512), 0, st, a);
  // uniform key splits (at most 8): the exact-count instantiations, opt-in (VLOG_AMD_XCOMB_EXACT=1).  5-13 % faster
  // merges (profiles/ab_r06_xcomb_exact.jsonl), same tokens on the bench workloads, but NOT the same bits: without
  // the per-split guards the compiler fuses the weight products differently, so the alignment heads' probabilities
  // move in the last bits, and tests/test_gpu_words.py's batched-vs-single-window near-ties flipped (7 of 8 words).
  static const int exact_env = [] {
    const char* e = std::getenv("VLOG_AMD_XCOMB_EXACT");
    return e ? std::atoi(e) : 0;
  }();
  const bool exact = exact_env && !plan.sk_W && splits >= 1 && splits <= 8;
#define XC_EXACT(KS8_)                                                                                   \
  switch (splits) {                                                                                      \
    case 1: XC_RTX(KS8_, 1) break;                                                                       \
    case 2: XC_RTX(KS8_, 2) break;                                                                       \
    case 3: XC_RTX(KS8_, 3) break;                                                                       \
    case 4: XC_RTX(KS8_, 4) break;                                                                       \
    case 5: XC_RTX(KS8_, 5) break;                                                                       \
    case 6: XC_RTX(KS8_, 6) break;                                                                       \
    case 7: XC_RTX(KS8_, 7) break;                                                                       \
    default: XC_RTX(KS8_, 8) break;                                                                      \
  }
#define XC_LAUNCH(KS8_)                                                                                  \
  if (exact) { XC_EXACT(KS8_) }                                                                          \
  else if (splits <= 1) { XC_RT(KS8_, 1) }                                                               \
  else if (splits <= 2) { XC_RT(KS8_, 2) }                                                               \
  else if (splits <= 4) { XC_RT(KS8_, 4) }                                                               \
  else if (splits <= 8) { XC_RT(KS8_, 8) }                                                               \
  else { XC_RT(KS8_, XMAXS) }
  switch (d) {                           // 8 waves x d/8 columns of the reduction: d/128 k-steps each
    case 384: XC_LAUNCH(3); break;
    case 512: XC_LAUNCH(4); break;
    case 768: XC_LAUNCH(6); break;
    case 1024: XC_LAUNCH(8); break;
    case 1280: XC_LAUNCH(10); break;
    default: throw std::runtime_error("xcomb_vo: unsupported n_state " + std::to_string(d));
  }
#undef XC_LAUNCH
#undef XC_EXACT
#undef XC_RTX
#undef XC_RT
  WM_LAUNCH_CHECK("xcomb_vo_kernel");
}
