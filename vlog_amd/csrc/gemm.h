// bf16 MFMA GEMM  C[M,N] = A[M,K] . W[N,K]^T  with fused epilogues (gfx950).
#pragma once
#include "common.h"

struct GemmA {
  const bf16* ptr;
  long long ld;        // elements between consecutive rows
  int rpb;             // rows per batch (0: plain 2-D)
  long long bstride;   // elements between batches
  // small-M path only (launch_dec_gemv, M <= 16): the operand is LayerNorm(lnx) rounded to bf16, computed in the
  // kernel from the f32 rows lnx (row stride ld), the affine ln_g / ln_b and the row statistics summed from the
  // producing GEMM's per-(16-column tile, row) partial sums ln_stat [ln_tiles][M][2] (GemmEpi.stat_out)
  const float* lnx;
  const float* ln_g;
  const float* ln_b;
  const float* ln_stat;
  int ln_tiles;
  // ring path only (launch_dec_ring), the folded LayerNorm: the operand rows hold bf16(x * g) (written by the
  // residual producer, GemmEpi.xg_out) and the row statistics are the producer's partial sums fold_stat
  // (sum x, sum x^2 per tile).  The kernel forms mean and rstd per row and its epilogue
  // applies y = rstd * acc - rstd * mean * fold_s[n] + fold_c[n] (GemmEpi) before the epilogue kind (fold_stat is
  // [fold_rows][fold_tiles][2]: 1 tile, or an even count <= 80):
  // W . LN(x) + bias = rstd (W . (g x)) - rstd mean (W g) + (W b + bias).
  const float* fold_stat;
  int fold_tiles;
  long long fold_rows;
};

// Epilogue kinds (see gemm.hip for the exact formulas)
enum EpiKind {
  EPI_BF16 = 0,        // C_bf16[r,c] = act(acc + bias[c]); row r -> (r/rpb)*bstride + (r%rpb + roff)*ldc
  EPI_RESID_F32 = 1,   // X_f32[r,c] += acc + bias[c]
  EPI_GELU_POS_F32 = 2,// X_f32[r,c]  = gelu(acc + bias[c]) + pos[r % rpb, c]
  EPI_F32 = 3,         // C_f32[r,c]  = acc (+ bias)
  EPI_DEC_QKV = 4,     // decoder self-attn: q -> C_bf16, k/v -> self-KV cache at (row_hyp[r], row_pos[r])
  EPI_CROSS_KV = 5,    // cross-KV projection -> [L][2][slots][H][T][hd]
  EPI_RESID_LN = 6,    // X_f32[r,c] += acc + bias[c], then ln_out[r] = LayerNorm(X[r]) (bf16) — N == row width
};

struct GemmEpi {
  int kind;
  int act;                 // EPI_BF16: 0 none, 1 gelu
  const float* bias;       // [N] or nullptr
  void* out;               // bf16* or float*
  long long ldc;
  int rpb;                 // output rows per batch (EPI_BF16, EPI_GELU_POS_F32, EPI_CROSS_KV: T)
  long long bstride;
  int roff;
  const float* pos;        // EPI_GELU_POS_F32
  // EPI_DEC_QKV
  bf16* kcache; bf16* vcache;       // layer base of the self-KV cache, [n_hyp_max][H][n_ctx][hd]
  const int* row_hyp; const int* row_pos;
  int d, n_head, head_dim, n_ctx;
  // EPI_CROSS_KV
  int n_slots, slot0;
  // EPI_RESID_LN: the LayerNorm that consumes the updated residual
  const float* ln_g; const float* ln_b; bf16* ln_out; long long ln_ld;
  // skinny split-K path only: leave the partial slabs in the scratch (no combine launch) for a consumer
  // that sums them itself (see skinny_splits)
  int defer_combine;
  // small-M path only, EPI_RESID_F32 without split-K: per (16-column tile, row) sums of the updated residual
  // (sum x, sum x^2) [N/16][M][2] for a LayerNorm-consuming GEMM (GemmA.lnx).  Ring path / split-K combine of an
  // EPI_RESID_F32 producer with xg_out set: the sums as [M][N/16][2] (ring) or [M][1][2] (the split-K combine)
  // plus xg_out[r][c] = bf16(x[r][c] * xg_g[c]) (the next LayerNorm's gamma) for a folded consumer (GemmA.fold_*)
  float* stat_out;
  bf16* xg_out; const float* xg_g; long long xg_ld;
  // folded-LayerNorm consumer (GemmA.fold_stat): W g and W b + bias per output column (bias is then nullptr)
  const float* fold_s; const float* fold_c;
};

// Split count the skinny path would use for this shape (>= 1), or 0 when launch_gemm would not take it.
int skinny_splits(int M, int N, int K, size_t ws_bytes);

// ws: f32 scratch for split-K partial slabs (nullptr disables split-K)
void launch_gemm(const GemmA& a, const bf16* w, long long ldw, int M, int N, int K, const GemmEpi& epi, float* ws,
                 size_t ws_bytes, hipStream_t st);

// Large-M path, staggered 4-phase-per-K-tile schedule (gemm_8p.hip): used by launch_gemm when applicable.
bool gemm_8p_applicable(int M, int N, int K);
void gemm_8p_set_persistent(int on);
int gemm_8p_get_persistent();
void launch_gemm_8p(const GemmA& a, const bf16* w, long long ldw, int M, int N, int K, const GemmEpi& epi, hipStream_t st);

// Large-M path (gemm_big.hip): 256x128 tiles, LDS-DMA ring; used by launch_gemm when applicable.
bool gemm_big_applicable(int M, int N, int K);
void launch_gemm_big(const GemmA& a, const bf16* w, long long ldw, int M, int N, int K, const GemmEpi& epi, hipStream_t st);

// Decoder-row path (gemm_dec.hip): M <= 160, N % 64 == 0, every load of a block's K range (KR, a multiple of
// 64) issued up front; split-K slabs combined by launch_splitk_combine.  Returns false if unsupported.
bool launch_dec_gemm(const GemmA& a, const bf16* w, long long ldw, int M, int N, int K, const GemmEpi& epi, float* ws,
                     size_t ws_bytes, int KR, hipStream_t st);
void launch_splitk_combine(const float* part, int splitk, int M, int N, const GemmEpi& epi, hipStream_t st);
// Ring-pipelined decoder-row path (gemm_dec.hip): M <= 160; kr = K range per block (0 = whole K up to 1280).
// rows_per_block > 0: the rows are split into groups of that many (32..160) — one block per (32-column tile, row
// group, K split); the row groups of a tile share its weight panel through one XCD's L2 (any M).  lds_kb: the ring's
// LDS budget, 144 (one block per CU) or 72 (two resident blocks per CU); 0 = the process default (VLOG_AMD_RING_LDS).
// waves: 4, or 8 (64 / 128 rows x 64 / 128 columns per block: two waves per SIMD).
bool launch_dec_ring(const GemmA& a, const bf16* w, long long ldw, int M, int N, int K, const GemmEpi& epi, float* ws,
                     size_t ws_bytes, int kr, hipStream_t st, int rows_per_block = 0, int cols = 32, int lds_kb = 0,
                     int waves = 4);
// Folded-LayerNorm vectors of a consumer projection (gemm_dec.hip): s = W g, c = W b + bias (f64 sums, f32 out).
void launch_fold_vectors(const bf16* w, int N, int K, const float* g, const float* b, const float* bias, float* s_out,
                         float* c_out, hipStream_t st);
// One-shot decoder-row path (gemm_dec.hip): 32 rows x nc*16 columns per 512-thread block, every load of a
// <= 1280-deep K range issued at once into MFMA operand registers, per-wave K split summed through LDS.
bool launch_dec_oneshot(const GemmA& a, const bf16* w, long long ldw, int M, int N, int K, const GemmEpi& epi, float* ws,
                        size_t ws_bytes, int nc, hipStream_t st);
// Small-M decoder path (gemm_dec.hip): M <= 32 rows, 16 output columns x a K range per 256-thread block, every
// weight fragment of the range issued at once (non-temporal), split-K where the tiles alone do not fill the chip.
// gemv_splits: the split count it would use (0: unsupported), kr_out = K range per block.
int gemv_splits(int M, int N, int K, int* kr_out);
void gemv_set_target_blocks(int blocks);   // microbenchmark knob (default 256)
void gemv_set_ablation(int bits);          // microbenchmark knob: LayerNorm-operand ablations (default 0)
bool launch_dec_gemv(const GemmA& a, const bf16* w, long long ldw, int M, int N, int K, const GemmEpi& epi, float* ws,
                     size_t ws_bytes, hipStream_t st);
// Whether the small-M path can run this shape as a residual producer with row statistics (EPI_RESID_F32 +
// stat_out, no split-K) and as a LayerNorm-consuming GEMM (GemmA.lnx).
bool gemv_ln_fusable(int M, int N_prod, int K_prod, int K_cons);
