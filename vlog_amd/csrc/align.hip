// Word alignment (word_timestamps=True) for gfx950: CTranslate2 Whisper.align's post-processing [FW↑]
// (oracle: oracle/align.py; DTW and median filter pinned against transformers).
//   token_probs_kernel  : softmax over the text vocabulary [0, eot) at each position -> prob of the next token
//   align_norm_kernel   : per (head, frame) column: crop to num_frames/2 keys + renormalise each row,
//                         z-score over the token axis                       -> z[h][r][f]
//   align_median_kernel : per (row, frame): width-w reflect median along time, mean over heads, negate
//   dtw_kernel          : one workgroup per matrix, anti-diagonal wavefront over the (N+1) x (F+1) cost grid
//                         (cells of one diagonal are independent), then a single-lane backtrace.
#include "common.h"
#include <algorithm>
#include <cstdlib>
#include <stdexcept>
#include <string>

__global__ __launch_bounds__(256) void token_probs_kernel(const float* __restrict__ logits, int V, int eot,
                                                          const int* __restrict__ next_tok, float* __restrict__ out) {
  __shared__ float red[4];
  const int r = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const float* lg = logits + (long long)r * V;
  float m = -INFINITY;
  for (int i = tid; i < eot; i += 256) m = fmaxf(m, lg[i]);
  m = wave_max(m);
  if (lane == 0) red[wv] = m;
  __syncthreads();
  m = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  __syncthreads();
  float s = 0.f;
  for (int i = tid; i < eot; i += 256) s += expf(lg[i] - m);
  s = wave_sum(s);
  if (lane == 0) red[wv] = s;
  __syncthreads();
  if (tid == 0) {
    s = red[0] + red[1] + red[2] + red[3];
    out[r] = expf(lg[next_tok[r]] - m) / s;
  }
}

// attn layout [S][n_heads][T]; rows r in [0, S); z layout [n_heads][S][F]
__global__ void align_norm_kernel(const float* __restrict__ attn, int S, int nh, int T, int F, float* __restrict__ rowsum,
                                  float* __restrict__ z) {
  const int h = blockIdx.y;
  const int f = blockIdx.x * blockDim.x + threadIdx.x;
  if (f >= F) return;
  double mean = 0.0, m2 = 0.0;
  for (int r = 0; r < S; ++r) {
    const double w = (double)attn[((long long)r * nh + h) * T + f] / (double)rowsum[r * nh + h];
    mean += w;
    m2 += w * w;
  }
  mean /= S;
  const double var = fmax(m2 / S - mean * mean, 0.0);
  const double inv = 1.0 / sqrt(var);
  for (int r = 0; r < S; ++r) {
    const double w = (double)attn[((long long)r * nh + h) * T + f] / (double)rowsum[r * nh + h];
    z[((long long)h * S + r) * F + f] = (float)((w - mean) * inv);
  }
}

// blockIdx.y = window k of a batch (tS / tF: per-window rows and frames; null: one window of S rows, F frames);
// window k's attention at attn + k astr, its row sums at rowsum + k rstr
__global__ void align_rowsum_kernel(const float* __restrict__ attn, int S, int nh, int T, int F, float* __restrict__ rowsum,
                                    const int* __restrict__ tS, const int* __restrict__ tF, long long astr, long long rstr) {
  const int k = blockIdx.y;
  if (tS) { S = tS[k]; F = tF[k]; }
  const int rh = blockIdx.x;     // r * nh + h
  if (rh >= S * nh) return;
  attn += k * astr;
  rowsum += k * rstr;
  float s = 0.f;
  for (int f = threadIdx.x; f < F; f += 64) s += attn[(long long)rh * T + f];
  s = wave_sum(s);
  if (threadIdx.x == 0) rowsum[rh] = s;
}

#define MEDW_MAX 15
// Per (output row, frame): the width-W median along time of every head's z row (reflect padding, as
// transformers' _median_filter), averaged over the heads and negated.  The median is an odd-even transposition
// sort of the W values in registers (W rounds of compare-exchanges with compile-time indices: no scratch, no
// divergent branches; the earlier insertion sort indexed a private array dynamically, which the compiler spills to
// scratch) — an exact selection, so the result is unchanged.
template <int WIDTH>
__global__ __launch_bounds__(128) void align_median_kernel(const float* __restrict__ z, int S, int nh, int F, int r0,
                                                           int nrows, float* __restrict__ mat) {
  const int r = blockIdx.y;          // output row: token row r0 + r
  const int f = blockIdx.x * blockDim.x + threadIdx.x;
  if (f >= F || r >= nrows) return;
  constexpr int PAD = WIDTH / 2;
  int idx[WIDTH];
#pragma unroll
  for (int k = 0; k < WIDTH; ++k) {
    int i = f - PAD + k;
    if (i < 0) i = -i;
    if (i >= F) i = 2 * (F - 1) - i;
    idx[k] = min(max(i, 0), F - 1);
  }
  float acc = 0.f;
  for (int h = 0; h < nh; ++h) {
    const float* row = z + ((long long)h * S + r0 + r) * F;
    float v;
    if (F <= PAD) {
      v = row[f];
    } else {
      float w[WIDTH];
#pragma unroll
      for (int k = 0; k < WIDTH; ++k) w[k] = row[idx[k]];
#pragma unroll
      for (int round = 0; round < WIDTH; ++round)
#pragma unroll
        for (int k = round & 1; k + 1 < WIDTH; k += 2) {
          const float lo = fminf(w[k], w[k + 1]), hi = fmaxf(w[k], w[k + 1]);
          w[k] = lo;
          w[k + 1] = hi;
        }
      v = w[PAD];
    }
    acc += v;
  }
  mat[(long long)r * F + f] = -(acc / nh);
}

// Fused form of align_norm_kernel + align_median_kernel (the default since round 5): the z-score statistics
// first (align_stats_kernel: per (head, frame) mean and 1/std over the token rows, f64, rows in order: the same
// loop as align_norm_kernel's first pass), then one WAVE per (output row, 64 - 2 PAD frames) recomputes each z from
// attn / rowsum with those statistics (the same f64 expression, so the same float) and takes the width-W median
// from its neighbours' lanes (shuffles; the reflect padding maps to lanes the wave holds), summing the heads in
// order.  z is never written: each attention value is read twice (statistics, median) instead of three times plus
// a z write and its W-tap re-reads.  Bit-identical to the two-kernel form.
__global__ __launch_bounds__(256) void align_stats_kernel(const float* __restrict__ attn, int S, int nh, int T, int F,
                                                          const float* __restrict__ rowsum, double* __restrict__ stats,
                                                          const int* __restrict__ tS, const int* __restrict__ tF,
                                                          long long astr, long long rstr, long long sstr) {
  const int h = blockIdx.y, k = blockIdx.z;
  if (tS) { S = tS[k]; F = tF[k]; }
  const int f = blockIdx.x * blockDim.x + threadIdx.x;
  if (f >= F) return;
  attn += k * astr;
  rowsum += k * rstr;
  stats += k * sstr;
  double mean = 0.0, m2 = 0.0;
  constexpr int U = 8;                                // rows in batches: loads first, then the sums in row order
  for (int r0 = 0; r0 < S; r0 += U) {
    float av[U], rs[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int r = min(r0 + u, S - 1);
      av[u] = attn[((long long)r * nh + h) * T + f];
      rs[u] = rowsum[r * nh + h];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (r0 + u >= S) break;
      const double w = (double)av[u] / (double)rs[u];
      mean += w;
      m2 += w * w;
    }
  }
  mean /= S;
  const double var = fmax(m2 / S - mean * mean, 0.0);
  stats[2 * ((long long)h * F + f)] = mean;
  stats[2 * ((long long)h * F + f) + 1] = 1.0 / sqrt(var);
}

template <int WIDTH>
__global__ __launch_bounds__(256) void align_zmed_kernel(const float* __restrict__ attn, int nh, int T, int F,
                                                         const float* __restrict__ rowsum, const double* __restrict__ stats,
                                                         int r0, int nrows, float* __restrict__ mat,
                                                         const int* __restrict__ tF, const int* __restrict__ trows,
                                                         const long long* __restrict__ tmat, long long astr, long long rstr,
                                                         long long sstr) {
  constexpr int PAD = WIDTH / 2, OUT = 64 - 2 * PAD;   // output frames per wave
  const int lane = threadIdx.x & 63;
  {
    const int k = blockIdx.y;                          // window k of a batch (tables; null: one window)
    if (tF) { F = tF[k]; nrows = trows[k]; mat += tmat[k]; }
    attn += k * astr;
    rowsum += k * rstr;
    stats += k * sstr;
  }
  const int nc = (F + OUT - 1) / OUT;
  const int gw = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int r = gw / nc, c = gw - r * nc;
  if (r >= nrows) return;                             // whole waves: the shuffles below see no exited lane
  const int f0 = c * OUT;
  const int ii = min(max(f0 - PAD + lane, 0), F - 1); // the frame whose z this lane computes
  const int f = f0 + lane - PAD;                       // the frame this lane outputs (lanes PAD .. 63 - PAD)
  int src[WIDTH];
#pragma unroll
  for (int k = 0; k < WIDTH; ++k) {
    int i = f - PAD + k;
    if (i < 0) i = -i;
    if (i >= F) i = 2 * (F - 1) - i;
    i = min(max(i, 0), F - 1);
    src[k] = min(max(i - (f0 - PAD), 0), 63);
  }
  const int self = min(max(min(max(f, 0), F - 1) - (f0 - PAD), 0), 63);
  const long long row = (long long)(r0 + r) * nh;
  float acc = 0.f;
  // heads in batches of U: every load of a batch issued before its first use (one memory round trip per batch,
  // not per head); the heads are still summed one by one in order
  constexpr int U = 8;
  for (int h0 = 0; h0 < nh; h0 += U) {
    float av[U], rs[U];
    double mu[U], iv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int h = min(h0 + u, nh - 1);
      av[u] = attn[(row + h) * T + ii];
      rs[u] = rowsum[row + h];
      mu[u] = stats[2 * ((long long)h * F + ii)];
      iv[u] = stats[2 * ((long long)h * F + ii) + 1];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
    if (h0 + u >= nh) break;
    const double w = (double)av[u] / (double)rs[u];
    const float z = (float)((w - mu[u]) * iv[u]);
    float v;
    if (F <= PAD) {
      v = __shfl(z, self, 64);
    } else {
      float t[WIDTH];
#pragma unroll
      for (int k = 0; k < WIDTH; ++k) t[k] = __shfl(z, src[k], 64);
#pragma unroll
      for (int round = 0; round < WIDTH; ++round)
#pragma unroll
        for (int k = round & 1; k + 1 < WIDTH; k += 2) {
          const float lo = fminf(t[k], t[k + 1]), hi = fmaxf(t[k], t[k + 1]);
          t[k] = lo;
          t[k + 1] = hi;
        }
      v = t[PAD];
    }
    acc += v;
    }
  }
  if (lane >= PAD && lane < 64 - PAD && f < F) mat[(long long)r * F + f] = -(acc / nh);
}

// cost [(N+1)][(M+1)] f32, trace [(N+1)][(M+1)] int8 scratch; x [N][M]; out path (text, time) reversed order fixed
__device__ __forceinline__ void dtw_kernel_body(const float* __restrict__ x, int N, int M, float* __restrict__ cost,
                                                signed char* __restrict__ trace, int* __restrict__ out_i,
                                                int* __restrict__ out_j, int* __restrict__ out_len) {
  const int tid = threadIdx.x;
  const long long W = M + 1;
  for (long long k = tid; k < (long long)(N + 1) * W; k += 256) {
    cost[k] = INFINITY;
    trace[k] = -1;
  }
  __syncthreads();
  if (tid == 0) cost[0] = 0.f;
  __syncthreads();
  // anti-diagonals d = i + j, i in [1, N], j in [1, M]
  for (int d = 2; d <= N + M; ++d) {
    const int i_lo = max(1, d - M), i_hi = min(N, d - 1);
    for (int i = i_lo + tid; i <= i_hi; i += 256) {
      const int j = d - i;
      const float c0 = cost[(i - 1) * W + (j - 1)], c1 = cost[(i - 1) * W + j], c2 = cost[i * W + (j - 1)];
      float c;
      signed char t;
      if (c0 < c1 && c0 < c2) { c = c0; t = 0; }
      else if (c1 < c0 && c1 < c2) { c = c1; t = 1; }
      else { c = c2; t = 2; }
      cost[i * W + j] = x[(long long)(i - 1) * M + (j - 1)] + c;
      trace[i * W + j] = t;
    }
    __syncthreads();
  }
  if (tid == 0) {
    int i = N, j = M, n = 0;
    while (i > 0 || j > 0) {
      out_i[n] = i - 1;
      out_j[n] = j - 1;
      ++n;
      const signed char t = (i == 0) ? 2 : (j == 0) ? 1 : trace[i * W + j];
      if (t == 0) { --i; --j; }
      else if (t == 1) { --i; }
      else { --j; }
    }
    // reverse in place
    for (int a = 0, b = n - 1; a < b; ++a, --b) {
      int ti = out_i[a]; out_i[a] = out_i[b]; out_i[b] = ti;
      int tj = out_j[a]; out_j[a] = out_j[b]; out_j[b] = tj;
    }
    *out_len = n;
  }
}

__global__ __launch_bounds__(256) void dtw_kernel(const float* __restrict__ x, int N, int M, float* __restrict__ cost,
                                                  signed char* __restrict__ trace, int* __restrict__ out_i,
                                                  int* __restrict__ out_j, int* __restrict__ out_len) {
  dtw_kernel_body(x, N, M, cost, trace, out_i, out_j, out_len);
}

void launch_token_probs(const float* logits, int rows, int V, int eot, const int* next_tok, float* out, hipStream_t st) {
  if (rows <= 0) return;
  hipLaunchKernelGGL(token_probs_kernel, dim3(rows), dim3(256), 0, st, logits, V, eot, next_tok, out);
  WM_LAUNCH_CHECK("token_probs_kernel");
}

// Process-wide (wm_set_option "align_fused"; VLOG_AMD_ALIGN_FUSED): 0 runs the round-4 two-kernel form (A/B, tests)
static int g_align_fused = [] {
  const char* e = std::getenv("VLOG_AMD_ALIGN_FUSED");
  return e ? std::atoi(e) : 1;
}();
static int align_fused() { return g_align_fused; }
void align_set_fused(int on) { g_align_fused = on != 0; }
int align_get_fused() { return g_align_fused; }

// z: scratch of n_heads x S x F floats (the two-kernel form's z; the fused form keeps its f64 statistics there,
// 4 floats per (head, frame): S >= 4 always holds for an aligned window, which has its sot prompt + text + eot)
void launch_align_matrix(const float* attn, int S, int nh, int T, int F, int width, int r0, int nrows, float* rowsum,
                         float* z, float* mat, hipStream_t st) {
  if (width > MEDW_MAX || width % 2 != 1) throw std::runtime_error("median filter width must be odd and <= 15");
  hipLaunchKernelGGL(align_rowsum_kernel, dim3(S * nh), dim3(64), 0, st, attn, S, nh, T, F, rowsum, nullptr, nullptr, 0LL, 0LL);
  WM_LAUNCH_CHECK("align_rowsum_kernel");
  if (align_fused() && S >= 4 && nrows > 0) {
    double* stats = (double*)z;
    hipLaunchKernelGGL(align_stats_kernel, dim3((F + 255) / 256, nh, 1), dim3(256), 0, st, attn, S, nh, T, F, rowsum, stats,
                       nullptr, nullptr, 0LL, 0LL, 0LL);
    WM_LAUNCH_CHECK("align_stats_kernel");
    const int out = 64 - 2 * (width / 2), waves = nrows * ((F + out - 1) / out);
    const dim3 g((waves + 3) / 4), b(256);
    switch (width) {
#define ZMED(W_) case W_: hipLaunchKernelGGL(align_zmed_kernel<W_>, g, b, 0, st, attn, nh, T, F, rowsum, stats, r0, nrows, mat, \
                                             nullptr, nullptr, nullptr, 0LL, 0LL, 0LL); break;
      ZMED(1) ZMED(3) ZMED(5) ZMED(7) ZMED(9) ZMED(11) ZMED(13) ZMED(15)
#undef ZMED
    }
    WM_LAUNCH_CHECK("align_zmed_kernel");
    return;
  }
  hipLaunchKernelGGL(align_norm_kernel, dim3((F + 127) / 128, nh), dim3(128), 0, st, attn, S, nh, T, F, rowsum, z);
  WM_LAUNCH_CHECK("align_norm_kernel");
  const dim3 g((F + 127) / 128, nrows), b(128);
  switch (width) {
#define MEDW(W_) case W_: hipLaunchKernelGGL(align_median_kernel<W_>, g, b, 0, st, z, S, nh, F, r0, nrows, mat); break;
    MEDW(1) MEDW(3) MEDW(5) MEDW(7) MEDW(9) MEDW(11) MEDW(13) MEDW(15)
#undef MEDW
  }
  WM_LAUNCH_CHECK("align_median_kernel");
}

// Every window of an alignment chunk at once (the fused form): window k's attention at attn + k smax nh T
// ([S_k][nh][T]), rows S_k (tS), frames F_k (tF), output rows rows_k (trows) written at mat + tmat[k]; scratch:
// rowsum [c][smax][nh] f32, stats [c][nh][fmax][2] f64.  One launch per kernel for the chunk instead of three per
// window (each window's launch alone was ~1.5 workgroups per CU: the median's head loop ran latency-bound).
void launch_align_matrix_batch(const float* attn, int c, int smax, int nh, int T, int fmax, int rows_max, int width,
                               int r0, const int* tS, const int* tF, const int* trows, const long long* tmat,
                               float* rowsum, double* stats, float* mat, hipStream_t st) {
  if (width > MEDW_MAX || width % 2 != 1) throw std::runtime_error("median filter width must be odd and <= 15");
  if (c <= 0) return;
  const long long astr = (long long)smax * nh * T, rstr = (long long)smax * nh, sstr = 2LL * nh * fmax;
  // windows on grid.y / grid.z: at most 65535 per launch
  for (int k0 = 0; k0 < c; k0 += 65535) {
    const int cc = std::min(c - k0, 65535);
    const float* at = attn + k0 * astr;
    float* rs = rowsum + k0 * rstr;
    double* sts = stats + k0 * sstr;
    hipLaunchKernelGGL(align_rowsum_kernel, dim3(smax * nh, cc), dim3(64), 0, st, at, smax, nh, T, fmax, rs, tS + k0,
                       tF + k0, astr, rstr);
    WM_LAUNCH_CHECK("align_rowsum_kernel");
    hipLaunchKernelGGL(align_stats_kernel, dim3((fmax + 255) / 256, nh, cc), dim3(256), 0, st, at, smax, nh, T, fmax, rs,
                       sts, tS + k0, tF + k0, astr, rstr, sstr);
    WM_LAUNCH_CHECK("align_stats_kernel");
    const int out = 64 - 2 * (width / 2), waves = rows_max * ((fmax + out - 1) / out);
    const dim3 g((waves + 3) / 4, cc), b(256);
    switch (width) {
#define ZMED(W_) case W_: hipLaunchKernelGGL(align_zmed_kernel<W_>, g, b, 0, st, at, nh, T, fmax, rs, sts, r0, rows_max, \
                                             mat, tF + k0, trows + k0, tmat + k0, astr, rstr, sstr); break;
      ZMED(1) ZMED(3) ZMED(5) ZMED(7) ZMED(9) ZMED(11) ZMED(13) ZMED(15)
#undef ZMED
    }
    WM_LAUNCH_CHECK("align_zmed_kernel");
  }
}

void launch_dtw(const float* x, int N, int M, float* cost, signed char* trace, int* out_i, int* out_j, int* out_len,
                hipStream_t st) {
  hipLaunchKernelGGL(dtw_kernel, dim3(1), dim3(256), 0, st, x, N, M, cost, trace, out_i, out_j, out_len);
  WM_LAUNCH_CHECK("dtw_kernel");
}

// Batched DTW: one workgroup per matrix (item b reads x + x_off[b], an N[b] x M[b] matrix; its cost / trace
// scratch starts at c_off[b], (N+1) x (M+1) cells; its path goes to out + p_off[b], capacity N + M).  The same
// wavefront and backtrace as dtw_kernel, so every item's path is bit-identical to a dtw_kernel launch on it.
__global__ __launch_bounds__(256) void dtw_batch_kernel(const float* __restrict__ x, const long long* __restrict__ x_off,
                                                        const int* __restrict__ Ns, const int* __restrict__ Ms,
                                                        float* __restrict__ cost_all, signed char* __restrict__ trace_all,
                                                        const long long* __restrict__ c_off, int* __restrict__ out_i,
                                                        int* __restrict__ out_j, const long long* __restrict__ p_off,
                                                        int* __restrict__ out_len) {
  const int b = blockIdx.x;
  dtw_kernel_body(x + x_off[b], Ns[b], Ms[b], cost_all + c_off[b], trace_all + c_off[b], out_i + p_off[b],
                  out_j + p_off[b], out_len + b);
}

void launch_dtw_batch(const float* x, const long long* x_off, const int* Ns, const int* Ms, float* cost,
                      signed char* trace, const long long* c_off, int* out_i, int* out_j, const long long* p_off,
                      int* out_len, int n, hipStream_t st) {
  if (n <= 0) return;
  hipLaunchKernelGGL(dtw_batch_kernel, dim3(n), dim3(256), 0, st, x, x_off, Ns, Ms, cost, trace, c_off, out_i, out_j,
                     p_off, out_len);
  WM_LAUNCH_CHECK("dtw_batch_kernel");
}
