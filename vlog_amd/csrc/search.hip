// On-device decoding search for gfx950: Whisper logit rules + log-softmax + greedy / sampling / beam
// candidate selection, and per-window beam bookkeeping.  Restates what CTranslate2's Whisper generate does
// on the host side of each step [FW↑] (oracle: oracle/decode.py; timestamp rules pinned against
// transformers WhisperTimeStampLogitsProcessor):
//   1. SuppressBlank (first sampled step: " " and <|endoftext|>), 2. SuppressTokens (mask), 3. timestamp
//   rules (no <|notimestamps|>; pairs; monotonic; first token a timestamp <= max_initial; if the timestamp
//   log-mass beats the best text token, only timestamps remain).
// One 1024-thread workgroup per hypothesis row streams the 51,866-wide logits row twice (max, then
// sum-exp) per segment (text / timestamps), so the forcing rule and the final normaliser come out of two
// segment log-sum-exps without a third pass.  Greedy and sampling (Gumbel-max over logits / T) update the
// sequence state in the same kernel; beam search emits each hypothesis's top beam+1 candidates and a
// per-window kernel ranks them (openai BeamSearchDecoder semantics, patience, finished list).
#include "search.h"
#include <stdexcept>
#include <string>

#define SB SEARCH_SB
#define NW (SB / 64)
#define KMAX 9

struct Cand { float v; int i; };
__device__ __forceinline__ bool better(float v1, int i1, float v2, int i2) { return v1 > v2 || (v1 == v2 && i1 < i2); }

__device__ __forceinline__ unsigned long long mix64(unsigned long long x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}
__device__ __forceinline__ float gumbel(unsigned long long seed, int hyp, int step, int i) {
  unsigned long long h = mix64(seed ^ mix64(((unsigned long long)hyp << 40) ^ ((unsigned long long)step << 20) ^ (unsigned long long)i));
  // 23 random bits: (k + 0.5) / 2^23 is exact in float32 and lies in (0, 1) for every k.  (With 24 bits, k = 2^24 - 1
  // rounded u up to exactly 1.0f and the key to +inf: that token was drawn with certainty, ~0.3 % of steps.)
  const float u = ((float)(h >> 41) + 0.5f) * (1.0f / 8388608.0f);
  return -logf(-logf(u));
}

// block-wide (max, argmax) reduce; returns result in all threads
__device__ Cand block_argmax(Cand c, Cand* sh) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float v2 = __shfl_xor(c.v, o, 64);
    const int i2 = __shfl_xor(c.i, o, 64);
    if (better(v2, i2, c.v, c.i)) { c.v = v2; c.i = i2; }
  }
  __syncthreads();
  if (lane == 0) sh[wv] = c;
  __syncthreads();
  Cand r = sh[0];
  for (int w = 1; w < NW; ++w)
    if (better(sh[w].v, sh[w].i, r.v, r.i)) r = sh[w];
  return r;
}
__device__ float block_sum(float v, float* sh) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  v = wave_sum(v);
  __syncthreads();
  if (lane == 0) sh[wv] = v;
  __syncthreads();
  float r = 0.f;
  for (int w = 0; w < NW; ++w) r += sh[w];
  return r;
}

// MODE = p.mode as a template parameter (0 greedy, 1 beam top-k, 2 sampling): each instantiation only holds
// the registers its mode needs next to the register-resident row.
// REC: also write the per-step records (p.tok_lp / p.tok_lp_other; an extra register pass for the best other
// token), instantiated only when a caller asks for them.
template <int MODE, bool REC>
__global__ __launch_bounds__(SB) void logits_select_kernel(SearchParams p) {
  __shared__ Cand sh_c[NW];
  __shared__ float sh_f[NW];
  __shared__ int s_info[4];
  __shared__ Cand s_top[NW * KMAX];
  __shared__ int s_last_ts;
  const int row = blockIdx.x, tid = threadIdx.x;
  const int h = p.row_hyp ? p.row_hyp[row] : row;
  if (p.done[h]) return;
  const int len = p.seq_len[h];
  const int* seq = p.tokens + (long long)h * p.n_ctx;
  const int tb = p.ts_begin;
  // position of the last sampled timestamp: a block-wide max instead of a serial backward scan (a text-only
  // history made thread 0 walk the whole sequence one dependent load at a time)
  if (tid == 0) s_last_ts = -1;
  __syncthreads();
  for (int i = p.sample_begin + tid; i < len; i += SB)
    if (seq[i] >= tb) atomicMax(&s_last_ts, i);
  __syncthreads();
  if (tid == 0) {
    const int ns = len - p.sample_begin;
    const int last = ns >= 1 ? seq[len - 1] : -1;
    const int last_ts = ns >= 1 && last >= tb;
    const int pen_ts = ns < 2 || seq[len - 2] >= tb;
    const int lastv = s_last_ts >= 0 ? seq[s_last_ts] : -1;
    int bound = tb;                          // timestamps in [tb, bound) are masked
    if (lastv >= 0) bound = (last_ts && !pen_ts) ? lastv : lastv + 1;
    s_info[0] = ns == 0;
    s_info[1] = (last_ts && pen_ts) ? 1 : ((last_ts && !pen_ts) ? 2 : 0);
    s_info[2] = bound;
  }
  __syncthreads();
  const int first = s_info[0], pair_rule = s_info[1], bound = s_info[2];
  const float* lg = p.logits + (long long)row * p.ldl;
  const int V = p.V;
  const bool ts_on = p.with_ts != 0;
  const unsigned long long sup = p.suppress_bits[tid];
  // The rules as 64-bit masks over this thread's ids i = tid + k SB (bit k): every rule is a range or a single
  // id, so each costs O(1) instead of a branch chain per element (the per-element form was most of the
  // kernel's 11-17 k instructions of straight-line code)
  auto ge_mask = [&](long long x) -> unsigned long long {   // ids >= x
    const long long d = x - tid;
    if (d <= 0) return ~0ull;
    const long long k0 = (d + SB - 1) / SB;
    return k0 >= 64 ? 0ull : (~0ull << k0);
  };
  auto id_bit = [&](long long x) -> unsigned long long {    // the single id x
    const long long d = x - tid;
    return (d >= 0 && d % SB == 0 && d / SB < 64) ? (1ull << (d / SB)) : 0ull;
  };
  const unsigned long long ts_mask = ge_mask(tb);
  unsigned long long rule = 0;
  if (first && p.suppress_blank) rule |= id_bit(p.blank) | id_bit(p.eot);
  if (ts_on) {
    rule |= id_bit(p.no_timestamps);
    if (pair_rule == 1) rule |= ts_mask;
    rule |= ts_mask & ~ge_mask(bound);                                     // timestamps below the bound
    if (first && p.max_initial >= 0) rule |= ts_mask & ge_mask((long long)tb + p.max_initial + 1);
    if (pair_rule == 2) rule |= ~ts_mask & ~ge_mask(p.eot);                 // text below <|endoftext|>
    if (first) rule |= ~ts_mask;
  }
  // The row is loaded ONCE into registers (PER values per thread, every load issued before any is used),
  // masked entries recorded in a bitmask; both passes then run on registers.  (The earlier form looped
  // over the row twice with one dependent global load per iteration: ~90 us per launch of exposed latency.)
  // Beam (MODE 1) extracts its top-k in a third pass over the same registers, once `forced` is known.
  constexpr int PER = SEARCH_PER;                          // vocab <= 53248
  constexpr bool RES = true;
  float xv[RES ? PER : 1];
  unsigned long long live = 0;
  auto xat = [&](int k) -> float { return RES ? xv[k] : lg[tid + k * SB]; };
  if (RES) {
    // 32-bit byte offsets from the row base (global_load_dword v, v_off, s_base): one offset register per
    // load in flight instead of a 64-bit address each (that form spilled and waited on its spills), no
    // branches; ids >= V re-read the last id (never live: suppress_bits)
#pragma unroll
    for (int k = 0; k < PER; ++k)
      xv[RES ? k : 0] = *(const float*)((const char*)lg + (unsigned)(min(tid + k * SB, V - 1) * 4));
  }
  live = ~(sup | rule) & ((1ull << PER) - 1);
  // pass 1: per-segment max / argmax (and Gumbel keys for sampling, local top-k for beam)
  Cand mt{-INFINITY, 0x7fffffff}, ms{-INFINITY, 0x7fffffff};
  Cand gt{-INFINITY, 0x7fffffff}, gs{-INFINITY, 0x7fffffff};
  const int K = MODE == 1 ? p.topk : 0;
  // Gumbel noise keyed on the WINDOW's hypothesis id, not the slot: the row-set decode reuses slots, and a window's
  // draws must not depend on which slot it got (hyp_out[h] = w there, one hypothesis per window; h = w*nh + j else)
  const int gkey = MODE == 2 && p.hyp_out ? p.hyp_out[h] : h;
  // (explicit branches, not a reference chosen per element: a `Cand& m = is_ts ? ms : mt` put both in scratch;
  // a select-only form of this pass spilled)
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    if (!((live >> k) & 1)) continue;
    const int i = tid + k * SB;
    const float x = xat(k);
    const bool is_ts = (ts_mask >> k) & 1;
    if (is_ts) {
      if (better(x, i, ms.v, ms.i)) { ms.v = x; ms.i = i; }
    } else {
      if (better(x, i, mt.v, mt.i)) { mt.v = x; mt.i = i; }
    }
    if (MODE == 2) {
      // the decode step of this hypothesis = tokens it has sampled so far (equal to the host's step counter
      // for every live hypothesis; read from the device so a captured step graph replays unchanged)
      const float key = x * p.inv_temperature + gumbel(p.seed, gkey, len - p.sample_begin, i);
      if (is_ts) {
        if (better(key, i, gs.v, gs.i)) { gs.v = key; gs.i = i; }
      } else {
        if (better(key, i, gt.v, gt.i)) { gt.v = key; gt.i = i; }
      }
    }
  }
  mt = block_argmax(mt, sh_c);
  ms = block_argmax(ms, sh_c);
  // pass 2: sum-exp per segment
  float st = 0.f, ss = 0.f;
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    if (!((live >> k) & 1)) continue;
    if ((ts_mask >> k) & 1) ss += expf(xat(k) - ms.v);
    else st += expf(xat(k) - mt.v);
  }
  st = block_sum(st, sh_f);
  ss = block_sum(ss, sh_f);
  // Numeric breakage is an error, never a token: a NaN or +inf among the allowed logits makes its segment's
  // exp-sum NaN (NaN, and inf - inf, propagate through the sums), and a row whose rules allow nothing leaves both
  // maxima at -inf.  The hypothesis ends, the device error word records it, and the host raises at its next poll
  // (the worker turns that into FAILED, worker/transcription.py:436-443).  All tested values are block-uniform.
  if (isnan(st) || isnan(ss) || (mt.v == -INFINITY && ms.v == -INFINITY)) {
    if (tid == 0) {
      wm_report_error(p.err, (isnan(st) || isnan(ss)) ? WM_ERR_NONFINITE : WM_ERR_NO_TOKEN, h, len - p.sample_begin);
      if (MODE == 1) {
        for (int r = 0; r < p.topk; ++r) {
          p.cand_tok[(long long)h * p.topk + r] = -1;
          p.cand_lp[(long long)h * p.topk + r] = -INFINITY;
        }
      } else {
        p.done[h] = 1;
        atomicSub(p.n_active, 1);
      }
    }
    return;
  }
  const float lse_t = mt.v > -INFINITY ? mt.v + logf(st) : -INFINITY;
  const float lse_s = ms.v > -INFINITY ? ms.v + logf(ss) : -INFINITY;
  const bool forced = ts_on && lse_s > mt.v;
  float Z;
  if (forced) Z = lse_s;
  else if (lse_t == -INFINITY) Z = lse_s;
  else if (lse_s == -INFINITY) Z = lse_t;
  else Z = fmaxf(lse_t, lse_s) + log1pf(expf(-fabsf(lse_t - lse_s)));

  if (MODE == 1) {
    // pass 3: the top-K of the allowed set (timestamps only when forced), in `better` order.  A threshold
    // first: tau = the K-th best of the per-thread maxima (K distinct elements are >= tau, so every top-K
    // element is too); the few elements >= tau are appended to an LDS list and wave 0 ranks them.  (The
    // earlier form ran K rounds of a wave argmax over the whole register-resident row: K x 52 compare-selects
    // per thread, ~79 us per launch at beam 5, one CU per hypothesis.)  A list that overflows (ties) falls
    // back to that form, so the result is the exact top-K either way.
    unsigned long long avail = live;
    if (forced) avail &= ts_mask;
    const int wv = tid >> 6, lane = tid & 63;
    constexpr int LCAP = 256;
    __shared__ Cand s_list[LCAP];
    __shared__ int s_n;
    __shared__ Cand s_tau;
    {
      Cand lb{-INFINITY, 0x7fffffff};        // this thread's best allowed element
#pragma unroll
      for (int k = 0; k < PER; ++k) {
        const int i = tid + k * SB;
        if (((avail >> k) & 1) && better(xat(k), i, lb.v, lb.i)) { lb.v = xat(k); lb.i = i; }
      }
      for (int r = 0; r < K; ++r) {          // the wave's K best per-thread maxima
        Cand best = lb;
        int owner = lane;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
          const float v2 = __shfl_xor(best.v, o, 64);
          const int i2 = __shfl_xor(best.i, o, 64);
          const int ow2 = __shfl_xor(owner, o, 64);
          if (better(v2, i2, best.v, best.i) || (v2 == best.v && i2 == best.i && ow2 < owner)) {
            best.v = v2; best.i = i2; owner = ow2;
          }
        }
        if (lane == 0) s_top[wv * KMAX + r] = best;
        if (lane == owner) lb = Cand{-INFINITY, 0x7fffffff};
      }
    }
    __shared__ int s_ptr[NW];
    if (tid < NW) s_ptr[tid] = 0;
    if (tid == 0) s_n = 0;
    __syncthreads();
    if (tid == 0) {                          // tau: the K-th of the merged per-wave lists
      Cand tau{-INFINITY, 0x7fffffff};
      for (int r = 0; r < K; ++r) {
        Cand best{-INFINITY, 0x7fffffff};
        int bw = -1;
        for (int w = 0; w < NW; ++w) {
          const int pp = s_ptr[w];
          if (pp >= K) continue;
          const Cand c = s_top[w * KMAX + pp];
          if (better(c.v, c.i, best.v, best.i)) { best = c; bw = w; }
        }
        if (bw < 0) { tau = Cand{-INFINITY, 0x7fffffff}; break; }
        ++s_ptr[bw];
        tau = best;
      }
      s_tau = tau;
    }
    __syncthreads();
    const Cand tau = s_tau;
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      const int i = tid + k * SB;
      if (((avail >> k) & 1) && (better(xat(k), i, tau.v, tau.i) || (xat(k) == tau.v && i == tau.i))) {
        const int at = atomicAdd(&s_n, 1);
        if (at < LCAP) s_list[at] = Cand{xat(k), i};
      }
    }
    __syncthreads();
    const int n_list = s_n;
    if (n_list <= LCAP && !(p.abl & 2)) {
      if (wv == 0) {
        Cand c[LCAP / 64];
#pragma unroll
        for (int j = 0; j < LCAP / 64; ++j)
          c[j] = lane + 64 * j < n_list ? s_list[lane + 64 * j] : Cand{-INFINITY, 0x7fffffff};
        for (int r = 0; r < K; ++r) {
          Cand best = c[0];
          int bj = 0;
#pragma unroll
          for (int j = 1; j < LCAP / 64; ++j)
            if (better(c[j].v, c[j].i, best.v, best.i)) { best = c[j]; bj = j; }
          int owner = lane;
#pragma unroll
          for (int o = 32; o > 0; o >>= 1) {
            const float v2 = __shfl_xor(best.v, o, 64);
            const int i2 = __shfl_xor(best.i, o, 64);
            const int ow2 = __shfl_xor(owner, o, 64);
            if (better(v2, i2, best.v, best.i) || (v2 == best.v && i2 == best.i && ow2 < owner)) {
              best.v = v2; best.i = i2; owner = ow2;
            }
          }
          if (lane == owner) {
#pragma unroll
            for (int j = 0; j < LCAP / 64; ++j)
              if (j == bj) c[j] = Cand{-INFINITY, 0x7fffffff};
          }
          if (lane == 0) {
            const bool none = best.v == -INFINITY;
            p.cand_tok[(long long)h * p.topk + r] = none ? -1 : best.i;
            p.cand_lp[(long long)h * p.topk + r] = none ? -INFINITY : best.v - Z;
          }
        }
      }
      return;
    }
    // overflow (many tied values): K rounds over the whole row
    for (int r = 0; r < K; ++r) {
      Cand best{-INFINITY, 0x7fffffff};
      int bk = -1;
#pragma unroll
      for (int k = 0; k < PER; ++k) {
        const int i = tid + k * SB;
        if (((avail >> k) & 1) && better(xat(k), i, best.v, best.i)) { best.v = xat(k); best.i = i; bk = k; }
      }
      int owner = lane;
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
        const float v2 = __shfl_xor(best.v, o, 64);
        const int i2 = __shfl_xor(best.i, o, 64);
        const int ow2 = __shfl_xor(owner, o, 64);
        if (better(v2, i2, best.v, best.i) || (v2 == best.v && i2 == best.i && ow2 < owner)) {
          best.v = v2; best.i = i2; owner = ow2;
        }
      }
      if (lane == 0) s_top[wv * KMAX + r] = best;
      if (lane == owner && bk >= 0) avail &= ~(1ull << bk);
    }
    if (tid < NW) s_ptr[tid] = 0;
    __syncthreads();
    if (tid == 0) {
      for (int r = 0; r < K; ++r) {
        Cand best{-INFINITY, 0x7fffffff};
        int bw = -1;
        for (int w = 0; w < NW; ++w) {
          const int pp = s_ptr[w];
          if (pp >= K) continue;
          const Cand c = s_top[w * KMAX + pp];
          if (better(c.v, c.i, best.v, best.i)) { best = c; bw = w; }
        }
        if (bw < 0 || best.v == -INFINITY) {
          p.cand_tok[(long long)h * p.topk + r] = -1;
          p.cand_lp[(long long)h * p.topk + r] = -INFINITY;
        } else {
          ++s_ptr[bw];
          p.cand_tok[(long long)h * p.topk + r] = best.i;
          p.cand_lp[(long long)h * p.topk + r] = best.v - Z;
        }
      }
    }
    return;
  }

  if (MODE == 2) {
    gt = block_argmax(gt, sh_c);
    gs = block_argmax(gs, sh_c);
  }
  // the chosen token: every thread holds the block-reduced candidates and `forced`, so it is block-uniform
  int tok;
  if (MODE == 2) tok = forced ? gs.i : (better(gt.v, gt.i, gs.v, gs.i) ? gt.i : gs.i);
  else tok = forced ? ms.i : (better(mt.v, mt.i, ms.v, ms.i) ? mt.i : ms.i);
  float lp_other = -INFINITY;
  if (REC) {
    // the best allowed token other than the chosen one (the per-step margin of the records)
    const unsigned long long avail = forced ? (live & ts_mask) : live;
    Cand b{-INFINITY, 0x7fffffff};
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      const int i = tid + k * SB;
      if (((avail >> k) & 1) && i != tok && better(xat(k), i, b.v, b.i)) { b.v = xat(k); b.i = i; }
    }
    b = block_argmax(b, sh_c);
    lp_other = b.v - Z;
  }
  __shared__ int s_fin;
  if (tid == 0) {
    const float lp = lg[tok] - Z;
    const float cum = p.cum[h] + lp;
    p.cum[h] = cum;
    if (REC && p.tok_lp) {
      p.tok_lp[(long long)h * p.n_ctx + len] = lp;
      if (p.tok_lp_other) p.tok_lp_other[(long long)h * p.n_ctx + len] = lp_other;
    }
    bool fin = false;
    if (tok == p.eot) {
      fin = true;
    } else {
      p.tokens[(long long)h * p.n_ctx + len] = tok;
      p.seq_len[h] = len + 1;
      p.row_tok[row] = tok;
      p.row_pos[row] = len;
      if (len + 1 >= p.max_length) fin = true;
    }
    if (fin) {
      p.done[h] = 1;
      atomicSub(p.n_active, 1);
      if (p.res_tok) {
        const int o = p.hyp_out[h];
        p.res_len[o] = len + (tok == p.eot ? 0 : 1) - p.sample_begin;
        p.res_cum[o] = cum;
      }
    }
    s_fin = fin;
  }
  if (p.res_tok) {
    // row-set decode: the hypothesis' slot is reused once it ends, so its tokens (and records) move to the
    // output tables now, copied by the whole block
    __syncthreads();
    if (s_fin) {
      const int o = p.hyp_out[h];
      const int n = len + (tok == p.eot ? 0 : 1) - p.sample_begin;     // generated tokens, <|endoftext|> excluded
      const int* src = p.tokens + (long long)h * p.n_ctx + p.sample_begin;
      for (int t = tid; t < n; t += SB) p.res_tok[(long long)o * p.n_ctx + t] = src[t];
      if (REC && p.tok_lp && p.res_lp) {
        const int nr = len + 1 - p.sample_begin;                       // records up to position len
        const float* a = p.tok_lp + (long long)h * p.n_ctx + p.sample_begin;
        const float* b = p.tok_lp_other ? p.tok_lp_other + (long long)h * p.n_ctx + p.sample_begin : nullptr;
        for (int t = tid; t < nr; t += SB) {
          p.res_lp[(long long)o * p.n_ctx + t] = a[t];
          if (b && p.res_lp_other) p.res_lp_other[(long long)o * p.n_ctx + t] = b[t];
        }
      }
    }
  }
}

void search_suppress_bits(const unsigned char* sup, int V, unsigned long long* bits) {
  for (int t = 0; t < SB; ++t) {
    unsigned long long w = 0;
    for (int k = 0; k < 64; ++k) {
      const long long i = t + (long long)k * SB;
      if (i >= V || sup[i]) w |= 1ull << k;
    }
    bits[t] = w;
  }
}

void launch_logits_select(const SearchParams& p, int n_rows, hipStream_t st) {
  if (n_rows <= 0) return;
  if (p.V > 53248) throw std::runtime_error("logits_select: vocabulary larger than 53248");
  if (p.mode == 1 && (p.topk < 1 || p.topk > KMAX)) throw std::runtime_error("beam size must be <= 8");
  if (p.res_tok && (!p.hyp_out || !p.res_len || !p.res_cum || p.mode == 1))
    throw std::runtime_error("logits_select: incomplete output tables");
  const bool rec = p.tok_lp != nullptr && p.mode != 1;     // beam: beam_select_kernel keeps the records
  const dim3 g(n_rows), b(SB);
  switch (p.mode * 2 + (rec ? 1 : 0)) {
    case 0: hipLaunchKernelGGL((logits_select_kernel<0, false>), g, b, 0, st, p); break;
    case 1: hipLaunchKernelGGL((logits_select_kernel<0, true>), g, b, 0, st, p); break;
    case 2: case 3: hipLaunchKernelGGL((logits_select_kernel<1, false>), g, b, 0, st, p); break;
    case 4: hipLaunchKernelGGL((logits_select_kernel<2, false>), g, b, 0, st, p); break;
    default: hipLaunchKernelGGL((logits_select_kernel<2, true>), g, b, 0, st, p); break;
  }
  WM_LAUNCH_CHECK("logits_select_kernel");
}

// ------------------------------------------------------------------------------------ row-set bookkeeping
__global__ __launch_bounds__(256) void hyp_start_kernel(const int* __restrict__ hs, const int* __restrict__ ws,
                                                        const int* __restrict__ win_prompt, int P,
                                                        const int* __restrict__ win_slot, int n_ctx, int* tokens,
                                                        int* seq_len, int* done, float* cum, int* hyp_slot, int* hyp_out) {
  const int h = hs[blockIdx.x], w = ws[blockIdx.x];
  for (int p = threadIdx.x; p < P; p += blockDim.x) tokens[(long long)h * n_ctx + p] = win_prompt[(long long)w * P + p];
  if (threadIdx.x == 0) {
    seq_len[h] = P;
    done[h] = 0;
    cum[h] = 0.f;
    hyp_slot[h] = win_slot[w];
    hyp_out[h] = w;
  }
}

void launch_hyp_start(int n, const int* hs, const int* ws, const int* win_prompt, int P, const int* win_slot, int n_ctx,
                      int* tokens, int* seq_len, int* done, float* cum, int* hyp_slot, int* hyp_out, hipStream_t st) {
  if (n <= 0) return;
  hipLaunchKernelGGL(hyp_start_kernel, dim3(n), dim3(64), 0, st, hs, ws, win_prompt, P, win_slot, n_ctx, tokens, seq_len,
                     done, cum, hyp_slot, hyp_out);
  WM_LAUNCH_CHECK("hyp_start_kernel");
}

// Beam row-set decode: group gs[i] of K hypothesis slots starts window ws[i]: every hypothesis gets the window's
// prompt, its lineage points the prompt positions at the group's first slot (whose self-KV the pass prefills), the
// first slot carries the score (the others start dead, as the one-pass beam prefill), and the group's finished list
// is emptied.
__global__ __launch_bounds__(256) void beam_start_kernel(const int* __restrict__ gs, const int* __restrict__ ws, int K,
                                                         const int* __restrict__ win_prompt, int P,
                                                         const int* __restrict__ win_slot, int n_ctx, int* tokens,
                                                         int* lin, int* seq_len, int* done, float* cum, int* hyp_slot,
                                                         int* n_fin) {
  const int g = gs[blockIdx.x], w = ws[blockIdx.x], h0 = g * K;
  for (int i = threadIdx.x; i < K * P; i += blockDim.x) {
    const int b = i / P, p = i - b * P;
    tokens[(long long)(h0 + b) * n_ctx + p] = win_prompt[(long long)w * P + p];
    lin[(long long)(h0 + b) * n_ctx + p] = h0;
  }
  if (threadIdx.x < K) {
    const int h = h0 + threadIdx.x;
    seq_len[h] = P;
    done[h] = 0;
    cum[h] = threadIdx.x == 0 ? 0.f : -INFINITY;
    hyp_slot[h] = win_slot[w];
  }
  if (threadIdx.x == 0) n_fin[g] = 0;
}

void launch_beam_start(int n, const int* gs, const int* ws, int K, const int* win_prompt, int P, const int* win_slot,
                       int n_ctx, int* tokens, int* lin, int* seq_len, int* done, float* cum, int* hyp_slot, int* n_fin,
                       hipStream_t st) {
  if (n <= 0) return;
  hipLaunchKernelGGL(beam_start_kernel, dim3(n), dim3(256), 0, st, gs, ws, K, win_prompt, P, win_slot, n_ctx, tokens,
                     lin, seq_len, done, cum, hyp_slot, n_fin);
  WM_LAUNCH_CHECK("beam_start_kernel");
}

__global__ __launch_bounds__(256) void rows_fill_kernel(int n, const int* __restrict__ src, int* __restrict__ tok,
                                                        int* __restrict__ pos, const int* __restrict__ row_tok,
                                                        const int* __restrict__ row_pos) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int s = src[i];
  if (s >= 0) {
    tok[i] = row_tok[s];
    pos[i] = row_pos[s];
  }
}

void launch_rows_fill(int n, const int* src, int* tok, int* pos, const int* row_tok, const int* row_pos, hipStream_t st) {
  if (n <= 0) return;
  hipLaunchKernelGGL(rows_fill_kernel, dim3((n + 255) / 256), dim3(256), 0, st, n, src, tok, pos, row_tok, row_pos);
  WM_LAUNCH_CHECK("rows_fill_kernel");
}

// ------------------------------------------------------------------------------------ beam bookkeeping
#define BMAX 8
#define CMAX 16

// One workgroup per window.  The K x (K+1) candidates are ranked in parallel (rank = number of candidates
// that precede it in a stable descending sort of (beam, rank)-ordered candidates), and the ranked list lives in
// LDS, so the one serial walk (live beams / finished list, <= K (K+1) steps) touches no scratch memory; the
// finished hypotheses' tokens are copied by the whole workgroup.  (The earlier form ran an insertion sort and
// the copies in thread 0 over scratch arrays: ~0.2 ms per decode step of the sequential beam-5 call.)
__global__ __launch_bounds__(256) void beam_select_kernel(BeamParams p) {
  constexpr int NC = BMAX * (BMAX + 1);
  __shared__ int s_tok[BMAX][448];
  __shared__ int s_lin[BMAX][448];
  __shared__ float s_lp[BMAX][448];          // per-step records (p.tok_lp)
  __shared__ float c_sc[NC], o_sc[NC];
  __shared__ int c_ok[NC], o_src[NC], o_tk[NC];
  __shared__ int s_par[BMAX], s_new[BMAX];
  __shared__ float s_sc[BMAX], s_cum[BMAX];
  __shared__ int f_src[CMAX], f_slot[CMAX];
  __shared__ float f_sc[CMAX];
  __shared__ int s_nlive, s_nf_new;
  const int w = blockIdx.x, tid = threadIdx.x;
  const int K = p.beam, h0 = w * K, T = K + 1, NK = K * T;
  if (p.done[h0]) return;
  const int len = p.seq_len[h0];
  const bool rec = p.tok_lp != nullptr;
  for (int i = tid; i < K * len; i += blockDim.x) {
    const int b = i / len, t = i - b * len;
    s_tok[b][t] = p.tokens[(long long)(h0 + b) * p.n_ctx + t];
    s_lin[b][t] = p.lin[(long long)(h0 + b) * p.n_ctx + t];
    if (rec) s_lp[b][t] = p.tok_lp[(long long)(h0 + b) * p.n_ctx + t];
  }
  // candidate i = (beam j, rank r) in (beam, rank) order
  float sc_i = -INFINITY;
  int tk_i = -1;
  if (tid < NK) {
    const int j = tid / T;
    const float c = p.cum[h0 + j];
    if (tid % T == 0) s_cum[j] = c;
    tk_i = p.cand_tok[(long long)h0 * T + tid];
    const float s = c + p.cand_lp[(long long)h0 * T + tid];
    // a NaN score would compare false against every other and break the ranks' total order (the select kernel
    // already reports non-finite rows and emits no candidate for them; this keeps the ranking well-formed)
    const bool ok = c != -INFINITY && tk_i >= 0 && !isnan(s);
    if (ok) sc_i = s;
    c_ok[tid] = ok;
    c_sc[tid] = sc_i;
  }
  __syncthreads();
  if (tid < NK && c_ok[tid]) {
    int rank = 0;
    for (int j = 0; j < NK; ++j)
      if (c_ok[j] && (c_sc[j] > sc_i || (c_sc[j] == sc_i && j < tid))) ++rank;
    o_sc[rank] = sc_i; o_src[rank] = tid / T; o_tk[rank] = tk_i;
  }
  __syncthreads();
  if (tid == 0) {
    int n = 0;
    for (int j = 0; j < NK; ++j) n += c_ok[j];
    int nlive = 0, nf = p.n_fin[w], nnew = 0;
    for (int c = 0; c < n && nlive < K; ++c) {
      if (o_tk[c] == p.eot) {
        if (nf < p.max_cand) {
          f_src[nnew] = o_src[c]; f_slot[nnew] = nf; f_sc[nnew] = o_sc[c];
          ++nnew;
          ++nf;
        }
      } else {
        s_par[nlive] = o_src[c]; s_new[nlive] = o_tk[c]; s_sc[nlive] = o_sc[c]; ++nlive;
      }
    }
    if (nlive == 0) {
      // no live candidate (every candidate non-finite or finished): the dead beams below copy beam 0's lineage and a
      // valid token, so no later pass reads a hypothesis index or token from uninitialised LDS
      s_par[0] = 0; s_new[0] = p.eot; s_sc[0] = -INFINITY;
    }
    p.n_fin[w] = nf;
    s_nlive = nlive;
    s_nf_new = nnew;
    const bool fin = nf >= p.max_cand || len + 1 >= p.max_length || nlive == 0;
    if (fin) {
      for (int j = 0; j < K; ++j) p.done[h0 + j] = 1;
      atomicSub(p.n_active, K);
    }
  }
  __syncthreads();
  {
    const int nnew = s_nf_new, ng = len - p.sample_begin;
    for (int i = tid; i < nnew * ng; i += blockDim.x) {
      const int f = i / ng, t = i - f * ng;
      p.fin_tok[((long long)w * p.max_cand + f_slot[f]) * p.n_ctx + t] = s_tok[f_src[f]][p.sample_begin + t];
      if (rec) p.fin_lp[((long long)w * p.max_cand + f_slot[f]) * p.n_ctx + t] = s_lp[f_src[f]][p.sample_begin + t];
    }
    if (tid < nnew) {
      p.fin_len[w * p.max_cand + f_slot[tid]] = ng;
      p.fin_cum[w * p.max_cand + f_slot[tid]] = f_sc[tid];
      if (rec) p.fin_lp[((long long)w * p.max_cand + f_slot[tid]) * p.n_ctx + ng] = f_sc[tid] - s_cum[f_src[tid]];
    }
  }
  const int nlive = s_nlive;
  // write the new beams (beams beyond nlive are marked dead with cum = -inf)
  for (int i = tid; i < K * len; i += blockDim.x) {
    const int b = i / len, t = i - b * len;
    const int par = b < nlive ? s_par[b] : s_par[0];
    p.tokens[(long long)(h0 + b) * p.n_ctx + t] = s_tok[par][t];
    p.lin[(long long)(h0 + b) * p.n_ctx + t] = s_lin[par][t];
    if (rec) p.tok_lp[(long long)(h0 + b) * p.n_ctx + t] = s_lp[par][t];
  }
  __syncthreads();
  if (tid < K) {
    const int b = tid;
    const int par = b < nlive ? s_par[b] : s_par[0];
    const int tok = b < nlive ? s_new[b] : s_new[0];
    if (rec) p.tok_lp[(long long)(h0 + b) * p.n_ctx + len] = b < nlive ? s_sc[b] - s_cum[par] : -INFINITY;
    p.tokens[(long long)(h0 + b) * p.n_ctx + len] = tok;
    p.lin[(long long)(h0 + b) * p.n_ctx + len] = h0 + b;      // the next step writes KV at (hyp, len)
    p.seq_len[h0 + b] = len + 1;
    p.cum[h0 + b] = b < nlive ? s_sc[b] : -INFINITY;
    p.row_tok[h0 + b] = tok;
    p.row_pos[h0 + b] = len;
    (void)par;
  }
}

void launch_beam_select(const BeamParams& p, int n_win, hipStream_t st) {
  if (n_win <= 0) return;
  if (p.beam > BMAX || p.max_cand > CMAX || p.n_ctx > 448) throw std::runtime_error("beam_select: limits exceeded");
  hipLaunchKernelGGL(beam_select_kernel, dim3(n_win), dim3(256), 0, st, p);
  WM_LAUNCH_CHECK("beam_select_kernel");
}

// Language detection: out[r][j] = softmax over logits[r][lang_begin .. lang_begin + n_langs) (ctranslate2
// Whisper.detect_language's probabilities [FW↑]), f32 with an f32 max / sum
__global__ __launch_bounds__(256) void lang_probs_kernel(const float* __restrict__ logits, long long ldl, int lang_begin,
                                                         int n_langs, float* __restrict__ out) {
  __shared__ float sh[4];
  const float* lg = logits + (long long)blockIdx.x * ldl + lang_begin;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  float m = -INFINITY;
  for (int j = tid; j < n_langs; j += 256) m = fmaxf(m, lg[j]);
  m = wave_max(m);
  if (lane == 0) sh[wv] = m;
  __syncthreads();
  m = fmaxf(fmaxf(sh[0], sh[1]), fmaxf(sh[2], sh[3]));
  __syncthreads();
  float s = 0.f;
  for (int j = tid; j < n_langs; j += 256) s += expf(lg[j] - m);
  s = wave_sum(s);
  if (lane == 0) sh[wv] = s;
  __syncthreads();
  s = sh[0] + sh[1] + sh[2] + sh[3];
  for (int j = tid; j < n_langs; j += 256) out[(long long)blockIdx.x * n_langs + j] = expf(lg[j] - m) / s;
}

void launch_lang_probs(const float* logits, long long ldl, int rows, int lang_begin, int n_langs, float* out, hipStream_t st) {
  if (rows <= 0 || n_langs <= 0) return;
  hipLaunchKernelGGL(lang_probs_kernel, dim3(rows), dim3(256), 0, st, logits, ldl, lang_begin, n_langs, out);
  WM_LAUNCH_CHECK("lang_probs_kernel");
}

// softmax(logits[r])[no_speech]
__global__ __launch_bounds__(SB) void no_speech_kernel(const float* __restrict__ logits, long long ldl, int V, int ns,
                                                        float* __restrict__ out, const int* __restrict__ out_idx) {
  __shared__ Cand sh_c[NW];
  __shared__ float sh_f[NW];
  const float* lg = logits + (long long)blockIdx.x * ldl;
  Cand m{-INFINITY, 0};
  for (int i = threadIdx.x; i < V; i += SB)
    if (lg[i] > m.v) { m.v = lg[i]; m.i = i; }
  m = block_argmax(m, sh_c);
  float s = 0.f;
  for (int i = threadIdx.x; i < V; i += SB) s += expf(lg[i] - m.v);
  s = block_sum(s, sh_f);
  if (threadIdx.x == 0) out[out_idx ? out_idx[blockIdx.x] : blockIdx.x] = expf(lg[ns] - m.v) / s;
}

void launch_no_speech(const float* logits, long long ldl, int V, int rows, int no_speech, float* out, hipStream_t st,
                      const int* out_idx) {
  if (rows <= 0) return;
  hipLaunchKernelGGL(no_speech_kernel, dim3(rows), dim3(SB), 0, st, logits, ldl, V, no_speech, out, out_idx);
  WM_LAUNCH_CHECK("no_speech_kernel");
}
