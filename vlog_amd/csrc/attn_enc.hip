// Encoder self-attention (non-causal, T = 1500, head_dim 64) as a flash-style MFMA kernel for gfx950.
//
// One workgroup = 4 waves = 64 queries of one (window, head); each wave owns 16 queries.  Per 64-key tile:
//   S^T = K . Q^T   (v_mfma_f32_16x16x32_bf16, K tile from LDS as the A operand, Q held in registers as
//                    the B operand) -> each lane holds 16 scores of ONE query (query = lane & 15), so the
//                    online-softmax state (m, l) is lane-local and the row reductions are 2 shuffles;
//   O^T += V^T . P^T (the S^T accumulator IS the P^T operand: the k slots of lane group g are keys
//                    {4g..4g+3} U {16+4g..16+4g+3} of each 32-key step, and the V^T operand is read
//                    from LDS in the same permuted order — cdna_hip_programming.md §3 "an accumulator tile
//                    as the next MFMA's operand").
// K is staged with the GEMM's 128-B-row XOR swizzle; V is staged transposed ([hd][key], 136-B rows) so the
// A-operand reads are two ds_read_b64 per lane.  Next tile's global loads are issued before the current
// tile's MFMAs (register double buffer).
#include "common.h"
#include <cstdlib>
#include <stdexcept>
#include <string>
#include <type_traits>

#define HD 64
#define KT 64        // keys per tile
#define VT_LD 68     // V^T row stride (elements)

__device__ __forceinline__ int kswz(int row, int ch) { return row * HD + ((ch ^ ((row >> 1) & 7)) << 3); }

__global__ __launch_bounds__(256) void attn_enc_kernel(const bf16* __restrict__ qkv, bf16* __restrict__ out, int T,
                                                       int d, float scale_log2) {
  __shared__ __attribute__((aligned(16))) bf16 sK[KT * HD];
  __shared__ __attribute__((aligned(16))) bf16 sVt[HD * VT_LD];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int g = lane >> 4, ql = lane & 15;
  const int h = blockIdx.y, b = blockIdx.z;
  const long long ld = 3LL * d;
  const bf16* base = qkv + (long long)b * T * ld;
  const int q0 = blockIdx.x * 64 + wv * 16;

  // Q fragments (B operand): Q[q0 + ql][kk*32 + 8g .. +7]
  bf16x8 qf[2];
  {
    const int q = q0 + ql;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      if (q < T) qf[kk] = *(const bf16x8*)(base + (long long)q * ld + h * HD + kk * 32 + 8 * g);
      else qf[kk] = bf16x8{};
    }
  }

  f32x4 o[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) o[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m_run = -INFINITY, l_run = 0.f;

  // staging: each thread moves 2 x 16 B of K and 2 x 16 B of V per tile
  i32x4 rk[2], rv[2];
  const int nt = (T + KT - 1) / KT;
#define LOAD_TILE(t_)                                                                       \
  {                                                                                         \
    _Pragma("unroll") for (int i = 0; i < 2; ++i) {                                         \
      const int c = tid + i * 256, key = (t_) * KT + (c >> 3), ch = c & 7;                  \
      if (key < T) {                                                                        \
        const bf16* p = base + (long long)key * ld + h * HD + ch * 8;                        \
        rk[i] = *(const i32x4*)(p + d);                                                     \
        rv[i] = *(const i32x4*)(p + 2 * d);                                                 \
      } else {                                                                              \
        rk[i] = i32x4{0, 0, 0, 0};                                                          \
        rv[i] = i32x4{0, 0, 0, 0};                                                          \
      }                                                                                     \
    }                                                                                       \
  }
  LOAD_TILE(0);
  for (int t = 0; t < nt; ++t) {
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int c = tid + i * 256, key = c >> 3, ch = c & 7;
      *(i32x4*)(&sK[kswz(key, ch)]) = rk[i];
      bf16x8 vv = __builtin_bit_cast(bf16x8, rv[i]);
#pragma unroll
      for (int e = 0; e < 8; ++e) sVt[(ch * 8 + e) * VT_LD + key] = vv[e];
    }
    __syncthreads();
    if (t + 1 < nt) LOAD_TILE(t + 1);

    // ---- S^T = K . Q^T : 4 key blocks x 2 k-steps
    f32x4 s[4];
#pragma unroll
    for (int mi = 0; mi < 4; ++mi) {
      s[mi] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        const bf16x8 ka = *(const bf16x8*)(&sK[kswz(mi * 16 + ql, kk * 4 + g)]);
        s[mi] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ka, qf[kk], s[mi], 0, 0, 0);
      }
    }
    // ---- online softmax (lane = one query; keys mi*16 + 4g + e)
    float tmax = -INFINITY;
    const int kbase = t * KT;
#pragma unroll
    for (int mi = 0; mi < 4; ++mi)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int key = kbase + mi * 16 + 4 * g + e;
        float v = s[mi][e] * scale_log2;
        if (key >= T) v = -INFINITY;
        s[mi][e] = v;
        tmax = fmaxf(tmax, v);
      }
    tmax = fmaxf(tmax, __shfl_xor(tmax, 16, 64));
    tmax = fmaxf(tmax, __shfl_xor(tmax, 32, 64));
    const float m_new = fmaxf(m_run, tmax);
    const float alpha = exp2f(m_run - m_new);
    float psum = 0.f;
#pragma unroll
    for (int mi = 0; mi < 4; ++mi)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float p = exp2f(s[mi][e] - m_new);
        s[mi][e] = p;
        psum += p;
      }
    psum += __shfl_xor(psum, 16, 64);
    psum += __shfl_xor(psum, 32, 64);
    l_run = l_run * alpha + psum;
    m_run = m_new;
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) o[ni] *= alpha;

    // ---- O^T += V^T . P^T : 4 hd blocks x 2 key steps
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 pb;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        pb[e] = f2bf(s[2 * ks][e]);
        pb[4 + e] = f2bf(s[2 * ks + 1][e]);
      }
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) {
        const bf16* vr = &sVt[(ni * 16 + ql) * VT_LD + ks * 32 + 4 * g];
        const bf16x4 lo = *(const bf16x4*)(vr);
        const bf16x4 hi = *(const bf16x4*)(vr + 16);
        bf16x8 va;
#pragma unroll
        for (int e = 0; e < 4; ++e) { va[e] = lo[e]; va[4 + e] = hi[e]; }
        o[ni] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(va, pb, o[ni], 0, 0, 0);
      }
    }
  }
#undef LOAD_TILE

  const int q = q0 + ql;
  if (q < T) {
    const float inv = 1.0f / l_run;
    bf16* orow = out + ((long long)b * T + q) * d + h * HD;
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) {
      bf16x4 w;
#pragma unroll
      for (int e = 0; e < 4; ++e) w[e] = f2bf(o[ni][e] * inv);
      *(bf16x4*)(orow + ni * 16 + 4 * g) = w;
    }
  }
}

// ------------------------------------------------------------------------------------------------------
// v2: 32x32x16 MFMA flash attention, one wave = 32 queries, 4 waves = 128 queries of one (window, head).
//   S^T (32 keys x 32 queries) = K . Q^T with Q pre-scaled by scale*log2(e) (bf16) held as the B operand,
//   K row fragments (ds_read_b128) as the A operand -> lane (q = l&31, h = l>>5) holds 16 scores of query
//   q, keys 8g + 4h + e (g, e < 4): the row max is 16 in-lane max + one xor-32 shuffle, the row sum stays
//   lane-local until the end.
//   O^T (32 hd x 32 q) += V^T . P^T: the S^T accumulator converted pairwise to bf16 IS the B operand
//   (k-step s takes registers 8s..8s+7 = keys 16s + 8(j>>2) + 4h + (j&3)); the V^T A operand comes from
//   row-major V in LDS through ds_read_b64_tr_b16 (cdna_hip_programming.md §3, T10), two reads per k-step.
//   Online softmax with deferred rescale (T13, THR = 8 in log2 units: P <= 256, exact in the normalised
//   result); K/V register-staged one tile ahead (T14) into a double-buffered LDS image, one barrier/tile.
//   LDS images (128-B rows): K chunk c of row r at slot c ^ ((r >> 1) & 7) (conflict-free 32-row b128
//   reads); V chunk c of row r at slot c ^ (((r >> 1) & 1) << 2) (conflict-free 4-row tr_b16 reads).
#define A2_KT 64
#define A2_THR 8.0f
typedef __attribute__((ext_vector_type(4))) short i16x4;
typedef __attribute__((ext_vector_type(2))) int i32x2;

__device__ __forceinline__ int a2_kslot(int r, int c) { return r * 64 + ((c ^ ((r >> 1) & 7)) << 3); }
__device__ __forceinline__ int a2_vslot(int r, int c) { return r * 64 + ((c ^ (((r >> 1) & 1) << 2)) << 3); }

// Grid: (query tiles x heads x windows) flattened, XCD-aware: the query tiles of one (window, head) get
// consecutive remapped ids, i.e. one XCD, so that head's K/V (1500 x 64 x 2 x 2 B) is read into that XCD's L2
// once instead of by every XCD (placement only: results do not depend on it).
__global__ __launch_bounds__(256, 2) void attn_enc_v2_kernel(const bf16* __restrict__ qkv, bf16* __restrict__ out,
                                                             int T, int d, float scale_log2, int n_head) {
  __shared__ __attribute__((aligned(16))) bf16 smem[2 * 2 * A2_KT * HD];     // [buf][K | V][64 keys][64]
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int ql = lane & 31, hh = lane >> 5;
  const int nqt = (T + 127) / 128;
  int qt, h, b;
  {
    const int nwg = gridDim.x, bid = blockIdx.x, xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
    const int wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
    qt = wgid % nqt;
    const int rest = wgid / nqt;
    h = rest % n_head;
    b = rest / n_head;
  }
  const long long ld = 3LL * d;
  const bf16* base = qkv + (long long)b * T * ld + h * HD;
  const int q = qt * 128 + wv * 32 + ql;

  // Q (B operand of S^T): k-step s holds Q[q][16 s + 8 hh + j], pre-scaled
  bf16x8 qf[4];
  {
    const int qc = min(q, T - 1);
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const bf16x8 v = *(const bf16x8*)(base + (long long)qc * ld + 16 * s + 8 * hh);
#pragma unroll
      for (int j = 0; j < 8; ++j) qf[s][j] = f2bf(bf2f(v[j]) * scale_log2);
    }
  }
  f32x16 o[2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) o[i][r] = 0.f;
  float m_run = -INFINITY, l_run = 0.f;

  // staging: thread moves 16-B chunks (row = c >> 3, chunk = c & 7) for c = tid, tid + 256 of K and of V
  i32x4 rk[2], rv[2];
  const int nt = (T + A2_KT - 1) / A2_KT;
  auto load_tile = [&](int t) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int c = tid + i * 256, key = min(t * A2_KT + (c >> 3), T - 1), ch = c & 7;
      const bf16* p = base + (long long)key * ld + ch * 8;
      rk[i] = *(const i32x4*)(p + d);
      rv[i] = *(const i32x4*)(p + 2 * d);
    }
  };
  auto store_tile = [&](int buf) {
    bf16* sK = smem + buf * (2 * A2_KT * HD);
    bf16* sV = sK + A2_KT * HD;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int c = tid + i * 256, r = c >> 3, ch = c & 7;
      *(i32x4*)(sK + a2_kslot(r, ch)) = rk[i];
      *(i32x4*)(sV + a2_vslot(r, ch)) = rv[i];
    }
  };
  load_tile(0);
  store_tile(0);
  __syncthreads();

  const int G = lane >> 4, gi = lane & 15, gq = gi >> 2, gp = gi & 3;    // tr_b16: group, row q, col block p
  for (int t = 0; t < nt; ++t) {
    const bf16* sK = smem + (t & 1) * (2 * A2_KT * HD);
    const bf16* sV = sK + A2_KT * HD;
    if (t + 1 < nt) load_tile(t + 1);

    // ---- S^T for the two 32-key blocks
    f32x16 sc[2];
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
#pragma unroll
      for (int r = 0; r < 16; ++r) sc[kb][r] = 0.f;
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const bf16x8 ka = *(const bf16x8*)(sK + a2_kslot(kb * 32 + ql, 2 * s + hh));
        sc[kb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ka, qf[s], sc[kb], 0, 0, 0);
      }
    }
    if (t == nt - 1) {                                   // keys past T (last tile only)
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int key = t * A2_KT + kb * 32 + 8 * (r >> 2) + 4 * hh + (r & 3);
          if (key >= T) sc[kb][r] = -INFINITY;
        }
    }
    // ---- online softmax, deferred rescale
    float mx = sc[0][0];
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int r = 0; r < 16; ++r) mx = fmaxf(mx, sc[kb][r]);
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    if (__any(mx > m_run + A2_THR)) {
      const float mn = fmaxf(m_run, mx);
      const float alpha = __builtin_amdgcn_exp2f(m_run - mn);
      l_run *= alpha;
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) o[i][r] *= alpha;
      m_run = mn;
    }
    bf16x8 pf[2][2];                                    // [key block][k-step]
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float pv = __builtin_amdgcn_exp2f(sc[kb][r] - m_run);
        l_run += pv;
        pf[kb][r >> 3][r & 7] = f2bf(pv);
      }
    // ---- O^T += V^T . P^T
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int hb = 0; hb < 2; ++hb) {
          bf16x8 va;
#ifndef A2_SCALAR_V
          i32x2 vw[2];
#endif
#pragma unroll
          for (int jh = 0; jh < 2; ++jh) {
            const int row = kb * 32 + 16 * s + 8 * jh + 4 * (G >> 1) + gq;
            const int col = 32 * hb + 16 * (G & 1) + 4 * gp;             // hd element
#ifdef A2_SCALAR_V
            const int rowb = row - gq, hdc = 32 * hb + 16 * (G & 1) + gi;
#pragma unroll
            for (int e = 0; e < 4; ++e) va[4 * jh + e] = sV[a2_vslot(rowb + e, hdc >> 3) + (hdc & 7)];
#else
            const bf16* ad = sV + a2_vslot(row, col >> 3) + (col & 7);
            // (whole-register bit casts: an element-wise short -> bf16 insert here miscompiles on ROCm 7.2,
            //  duplicating one half of the fragment)
            vw[jh] = __builtin_bit_cast(i32x2, __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                                                   (__attribute__((address_space(3))) i16x4*)(ad)));
#endif
          }
#ifndef A2_SCALAR_V
          va = __builtin_bit_cast(bf16x8, i32x4{vw[0][0], vw[0][1], vw[1][0], vw[1][1]});
#endif
          o[hb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(va, pf[kb][s], o[hb], 0, 0, 0);
        }
    if (t + 1 < nt) store_tile((t + 1) & 1);
    __syncthreads();
  }

  l_run += __shfl_xor(l_run, 32, 64);
  if (q < T) {
    const float inv = 1.0f / l_run;
    bf16* orow = out + ((long long)b * T + q) * d + h * HD;
#pragma unroll
    for (int hb = 0; hb < 2; ++hb)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        bf16x4 w;
#pragma unroll
        for (int e = 0; e < 4; ++e) w[e] = f2bf(o[hb][4 * g + e] * inv);
        *(bf16x4*)(orow + 32 * hb + 8 * g + 4 * hh) = w;
      }
  }
}

// ------------------------------------------------------------------------------------------------------
// v3: v2's tile arithmetic (same MFMAs, same per-tile softmax, so the same result bit for bit), software-
// pipelined by one tile: S^T of tile t+1 is issued to the matrix pipe before tile t's exps (after its row max
// and rescale branch), so the exp / convert VALU of tile t can run while the pipe works on the next tile's
// scores (within one wave every phase of v2 waits on the one before it).  Measured slower (see attn_enc_form).  Needs a 3-slot LDS ring (K/V of tile t for
// PV, of t+1 for S, t+2 being written): 48 KB per workgroup, two workgroups per CU.  The ring slot written at
// the end of iteration t held tile t-1, whose last reader (PV, iteration t-1) is behind the barrier of t-1.
__device__ __forceinline__ void a3_scores(const bf16* sK, const bf16x8 (&qf)[4], int ql, int hh, f32x16 (&sc)[2]) {
#pragma unroll
  for (int kb = 0; kb < 2; ++kb)
#pragma unroll
    for (int r = 0; r < 16; ++r) sc[kb][r] = 0.f;
#pragma unroll
  for (int s = 0; s < 4; ++s)                           // the two key blocks' chains alternate (same sums)
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
      const bf16x8 ka = *(const bf16x8*)(sK + a2_kslot(kb * 32 + ql, 2 * s + hh));
      sc[kb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ka, qf[s], sc[kb], 0, 0, 0);
    }
}

__global__ __launch_bounds__(256, 2) void attn_enc_v3_kernel(const bf16* __restrict__ qkv, bf16* __restrict__ out,
                                                             int T, int d, float scale_log2, int n_head) {
  __shared__ __attribute__((aligned(16))) bf16 smem[3 * 2 * A2_KT * HD];     // [slot][K | V][64 keys][64]
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int ql = lane & 31, hh = lane >> 5;
  const int nqt = (T + 127) / 128;
  int qt, h, b;
  {
    const int nwg = gridDim.x, bid = blockIdx.x, xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
    const int wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
    qt = wgid % nqt;
    const int rest = wgid / nqt;
    h = rest % n_head;
    b = rest / n_head;
  }
  const long long ld = 3LL * d;
  const bf16* base = qkv + (long long)b * T * ld + h * HD;
  const int q = qt * 128 + wv * 32 + ql;

  bf16x8 qf[4];
  {
    const int qc = min(q, T - 1);
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const bf16x8 v = *(const bf16x8*)(base + (long long)qc * ld + 16 * s + 8 * hh);
#pragma unroll
      for (int j = 0; j < 8; ++j) qf[s][j] = f2bf(bf2f(v[j]) * scale_log2);
    }
  }
  f32x16 o[2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) o[i][r] = 0.f;
  float m_run = -INFINITY, l_run = 0.f;

  i32x4 rk[2], rv[2];
  const int nt = (T + A2_KT - 1) / A2_KT;
  auto load_tile = [&](int t) {                         // rows clamped to T - 1 (a tile past the end is harmless)
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int c = tid + i * 256, key = min(t * A2_KT + (c >> 3), T - 1), ch = c & 7;
      const bf16* p = base + (long long)key * ld + ch * 8;
      rk[i] = *(const i32x4*)(p + d);
      rv[i] = *(const i32x4*)(p + 2 * d);
    }
  };
  auto store_tile = [&](int slot) {
    bf16* sK = smem + slot * (2 * A2_KT * HD);
    bf16* sV = sK + A2_KT * HD;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int c = tid + i * 256, r = c >> 3, ch = c & 7;
      *(i32x4*)(sK + a2_kslot(r, ch)) = rk[i];
      *(i32x4*)(sV + a2_vslot(r, ch)) = rv[i];
    }
  };
  load_tile(0);
  store_tile(0);
  if (nt > 1) {
    load_tile(1);
    store_tile(1);
  }
  __syncthreads();

  const int G = lane >> 4, gi = lane & 15, gq = gi >> 2, gp = gi & 3;
  f32x16 sc[2];
  a3_scores(smem, qf, ql, hh, sc);

  // one tile: S^T(t+1) issued first (unless LAST), then tile t's softmax and PV
  auto tile = [&](int t, int slot, auto last_tag) {
    constexpr bool LAST = decltype(last_tag)::value;
    const bf16* sV = smem + slot * (2 * A2_KT * HD) + A2_KT * HD;
    f32x16 sn[2];
    if constexpr (!LAST) load_tile(t + 2);
    if constexpr (LAST) {
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int key = t * A2_KT + kb * 32 + 8 * (r >> 2) + 4 * hh + (r & 3);
          if (key >= T) sc[kb][r] = -INFINITY;
        }
    }
    float mx = sc[0][0];
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int r = 0; r < 16; ++r) mx = fmaxf(mx, sc[kb][r]);
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    if (__any(mx > m_run + A2_THR)) {
      const float mn = fmaxf(m_run, mx);
      const float alpha = __builtin_amdgcn_exp2f(m_run - mn);
      l_run *= alpha;
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) o[i][r] *= alpha;
      m_run = mn;
    }
    // S^T(t+1) after the rescale branch, in the same scheduling region as tile t's exps, interleaved with them
    if constexpr (!LAST) a3_scores(smem + (slot == 2 ? 0 : slot + 1) * (2 * A2_KT * HD), qf, ql, hh, sn);
    bf16x8 pf[2][2];
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float pv = __builtin_amdgcn_exp2f(sc[kb][r] - m_run);
        l_run += pv;
        pf[kb][r >> 3][r & 7] = f2bf(pv);
      }
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int hb = 0; hb < 2; ++hb) {
          i32x2 vw[2];
#pragma unroll
          for (int jh = 0; jh < 2; ++jh) {
            const int row = kb * 32 + 16 * s + 8 * jh + 4 * (G >> 1) + gq;
            const int col = 32 * hb + 16 * (G & 1) + 4 * gp;
            const bf16* ad = sV + a2_vslot(row, col >> 3) + (col & 7);
            vw[jh] = __builtin_bit_cast(i32x2, __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                                                   (__attribute__((address_space(3))) i16x4*)(ad)));
          }
          const bf16x8 va = __builtin_bit_cast(bf16x8, i32x4{vw[0][0], vw[0][1], vw[1][0], vw[1][1]});
          o[hb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(va, pf[kb][s], o[hb], 0, 0, 0);
        }
    if constexpr (!LAST) {
      store_tile(slot == 0 ? 2 : slot - 1);             // (slot + 2) % 3: the slot tile t-1 used
      __syncthreads();
#pragma unroll
      for (int kb = 0; kb < 2; ++kb) sc[kb] = sn[kb];
    }
  };
  int slot = 0;
  for (int t = 0; t < nt - 1; ++t) {
    tile(t, slot, std::false_type{});
    slot = slot == 2 ? 0 : slot + 1;
  }
  tile(nt - 1, slot, std::true_type{});

  l_run += __shfl_xor(l_run, 32, 64);
  if (q < T) {
    const float inv = 1.0f / l_run;
    bf16* orow = out + ((long long)b * T + q) * d + h * HD;
#pragma unroll
    for (int hb = 0; hb < 2; ++hb)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        bf16x4 w;
#pragma unroll
        for (int e = 0; e < 4; ++e) w[e] = f2bf(o[hb][4 * g + e] * inv);
        *(bf16x4*)(orow + 32 * hb + 8 * g + 4 * hh) = w;
      }
  }
}

// Kernel form: VLOG_AMD_ATTN_V = 1 | 2 | 3 (VLOG_AMD_ATTN_V1=1 is the old spelling of 1); default 2.  v3 measured
// slower than v2 at the bench's shape, bit-identical (tools/attn_enc_ab.py, profiles/ab_r04_attn_enc_pipelined.jsonl:
// 2.34 vs 2.52 ms per 3000 (window, head) pairs; with an interleave directive of 1 K read + 1 MFMA + 6 or 12 VALU
// 2.74-2.82 ms at 170-172 VGPRs; v2 forced to 4 waves per SIMD spills 84 B and takes 3.85-3.89 ms), kept opt-in.
static int attn_enc_form() {
  static const int v = [] {
    const char* e1 = std::getenv("VLOG_AMD_ATTN_V1");
    if (e1 && e1[0] == '1') return 1;
    const char* e = std::getenv("VLOG_AMD_ATTN_V");
    const int f = e ? std::atoi(e) : 2;
    return (f >= 1 && f <= 3) ? f : 2;
  }();
  return v;
}

void launch_attn_enc(const bf16* qkv, bf16* out, int B, int T, int d, int n_head, hipStream_t st) {
  if (B <= 0) return;
  if (d != n_head * HD) throw std::runtime_error("attn_enc: head_dim must be 64");
  const float scale_log2 = 0.125f * 1.4426950408889634f;
  const int form = attn_enc_form();
  if (form == 1) {
    dim3 grid((T + 63) / 64, n_head, B);
    hipLaunchKernelGGL(attn_enc_kernel, grid, dim3(256), 0, st, qkv, out, T, d, scale_log2);
  } else {
    const long long nblk = (long long)((T + 127) / 128) * n_head * B;
    if (nblk > (1LL << 31) - 1) throw std::runtime_error("attn_enc: grid too large");
    if (form == 3)
      hipLaunchKernelGGL(attn_enc_v3_kernel, dim3((unsigned)nblk), dim3(256), 0, st, qkv, out, T, d, scale_log2, n_head);
    else
      hipLaunchKernelGGL(attn_enc_v2_kernel, dim3((unsigned)nblk), dim3(256), 0, st, qkv, out, T, d, scale_log2, n_head);
  }
  WM_LAUNCH_CHECK("attn_enc_kernel");
}
