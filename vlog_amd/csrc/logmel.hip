// Log-mel frontend for gfx950: reflect-centred STFT (n_fft 400, hop 160, periodic Hann) -> |X|^2 ->
// slaney mel filterbank -> log10(max(., 1e-10)), plus a global max for the max-8 clamp.
//
// Replaces faster-whisper's numpy FeatureExtractor.__call__ [FW↑] (reference call site
// worker/transcription.py:105-111; restated in oracle/mel.py).  n_fft = 400 = 4 * 4 * 5 * 5: the STFT is a
// mixed-radix Stockham FFT in LDS (two radix-4 then two radix-5 stages, natural-order output, twiddles from
// an LDS table), two real frames per complex transform (frame 2p as the real part, 2p+1 as the imaginary
// part, separated with X_a[k] = (Z[k] + conj Z[-k]) / 2, X_b[k] = (Z[k] - conj Z[-k]) / 2i).  The earlier
// direct DFT (one 400-term fmaf chain per bin) stays as logmel_dft_kernel (VLOG_AMD_LOGMEL_DFT=1).
//
// Frames are indexed GLOBALLY over the file so a shard (one GPU's window range) computes exactly the
// frames the whole-file spectrogram would: global padded sample i maps to file sample s = i - 200 with
// numpy "reflect" at the file edges over x_pad = pcm ++ zeros(pad_tail).
#include "common.h"
#include <cstdlib>
#include <stdexcept>
#include <string>

#define NFFT 400
#define NBIN 201
#define HOP 160
#define FPB 8          // frames per block

__global__ __launch_bounds__(256) void logmel_dft_kernel(
    const float* __restrict__ pcm, long long pcm_offset, long long n_samples, long long n_padded,
    long long frame0, int n_frames, const float* __restrict__ window, const float* __restrict__ twc,
    const float* __restrict__ tws, const float* __restrict__ filt, const int* __restrict__ flo,
    const int* __restrict__ fhi, int n_mels, float* __restrict__ out, long long ld,
    unsigned int* __restrict__ gmax) {
  __shared__ float s_x[FPB][NFFT];
  __shared__ float s_c[NFFT];
  __shared__ float s_s[NFFT];
  __shared__ float s_p[FPB][NBIN + 3];
  __shared__ float s_red[4];
  const int tid = threadIdx.x;
  const long long fb = (long long)blockIdx.x * FPB;   // first local frame of this block

  for (int i = tid; i < NFFT; i += 256) { s_c[i] = twc[i]; s_s[i] = tws[i]; }
  for (int i = tid; i < FPB * NFFT; i += 256) {
    const int f = i / NFFT, n = i - f * NFFT;
    float v = 0.f;
    const long long lf = fb + f;
    if (lf < n_frames) {
      long long s = (frame0 + lf) * HOP + n - NFFT / 2;      // file sample index before reflection
      if (s < 0) s = -s;
      if (s >= n_padded) s = 2 * (n_padded - 1) - s;
      if (s < n_samples) v = pcm[s - pcm_offset];
      v *= window[n];
    }
    s_x[f][n] = v;
  }
  __syncthreads();

  // Direct DFT: one (frame, bin) per work item; twiddle index (k*n) mod 400 advanced incrementally.
  for (int it = tid; it < FPB * NBIN; it += 256) {
    const int f = it / NBIN, k = it - f * NBIN;
    float re = 0.f, im = 0.f;
    int idx = 0;
    const float* x = s_x[f];
#pragma unroll 4
    for (int n = 0; n < NFFT; ++n) {
      const float xv = x[n];
      re = fmaf(xv, s_c[idx], re);
      im = fmaf(xv, s_s[idx], im);
      idx += k;
      if (idx >= NFFT) idx -= NFFT;
    }
    s_p[f][k] = fmaf(re, re, im * im);
  }
  __syncthreads();

  float lmax = -INFINITY;
  for (int it = tid; it < FPB * n_mels; it += 256) {
    const int m = it / FPB, f = it - m * FPB;
    const long long lf = fb + f;
    if (lf >= n_frames) continue;
    const float* w = filt + (long long)m * NBIN;
    float acc = 0.f;
    for (int k = flo[m]; k < fhi[m]; ++k) acc = fmaf(w[k], s_p[f][k], acc);
    const float lv = log10f(fmaxf(acc, 1e-10f));
    out[(long long)m * ld + lf] = lv;
    lmax = fmaxf(lmax, lv);
  }
  lmax = wave_max(lmax);
  if ((tid & 63) == 0) s_red[tid >> 6] = lmax;
  __syncthreads();
  if (tid == 0) {
    float m = fmaxf(fmaxf(s_red[0], s_red[1]), fmaxf(s_red[2], s_red[3]));
    if (m > -INFINITY) atomicMax(gmax, float_to_ordered(m));
  }
}

// one radix-R Stockham pass over NP complex transforms of 400 points: x -> y, Ns = product of earlier radices
template <int R>
__device__ __forceinline__ void fft_pass(const float2 (*x)[NFFT], float2 (*y)[NFFT], const float2* W, int Ns, int np) {
  constexpr int NR = NFFT / R;
  const float c1 = 0.30901699437494742f, c2 = -0.80901699437494742f;   // cos(2 pi / 5), cos(4 pi / 5)
  const float s1 = 0.95105651629515357f, s2 = 0.58778525229247313f;    // sin(2 pi / 5), sin(4 pi / 5)
  for (int it = threadIdx.x; it < np * NR; it += blockDim.x) {
    const int p = it / NR, j = it - p * NR;
    const int jm = j % Ns, tw = jm * (NFFT / (Ns * R));
    float2 v[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const float2 a = x[p][j + r * NR];
      if (r == 0) {
        v[r] = a;
      } else {
        const float2 w = W[(tw * r) % NFFT];
        v[r] = make_float2(a.x * w.x - a.y * w.y, a.x * w.y + a.y * w.x);
      }
    }
    float2 X[R];
    if constexpr (R == 4) {
      const float2 s02 = make_float2(v[0].x + v[2].x, v[0].y + v[2].y), d02 = make_float2(v[0].x - v[2].x, v[0].y - v[2].y);
      const float2 s13 = make_float2(v[1].x + v[3].x, v[1].y + v[3].y), d13 = make_float2(v[1].x - v[3].x, v[1].y - v[3].y);
      X[0] = make_float2(s02.x + s13.x, s02.y + s13.y);
      X[2] = make_float2(s02.x - s13.x, s02.y - s13.y);
      X[1] = make_float2(d02.x + d13.y, d02.y - d13.x);        // d02 - i d13
      X[3] = make_float2(d02.x - d13.y, d02.y + d13.x);        // d02 + i d13
    } else {
      const float2 t1 = make_float2(v[1].x + v[4].x, v[1].y + v[4].y), t2 = make_float2(v[2].x + v[3].x, v[2].y + v[3].y);
      const float2 t3 = make_float2(v[1].x - v[4].x, v[1].y - v[4].y), t4 = make_float2(v[2].x - v[3].x, v[2].y - v[3].y);
      X[0] = make_float2(v[0].x + t1.x + t2.x, v[0].y + t1.y + t2.y);
      const float2 a1 = make_float2(v[0].x + c1 * t1.x + c2 * t2.x, v[0].y + c1 * t1.y + c2 * t2.y);
      const float2 a2 = make_float2(v[0].x + c2 * t1.x + c1 * t2.x, v[0].y + c2 * t1.y + c1 * t2.y);
      const float2 b1 = make_float2(s1 * t3.x + s2 * t4.x, s1 * t3.y + s2 * t4.y);
      const float2 b2 = make_float2(s2 * t3.x - s1 * t4.x, s2 * t3.y - s1 * t4.y);
      X[1] = make_float2(a1.x + b1.y, a1.y - b1.x);            // a1 - i b1
      X[4] = make_float2(a1.x - b1.y, a1.y + b1.x);            // a1 + i b1
      X[2] = make_float2(a2.x + b2.y, a2.y - b2.x);
      X[3] = make_float2(a2.x - b2.y, a2.y + b2.x);
    }
    const int base = (j / Ns) * Ns * R + jm;
#pragma unroll
    for (int r = 0; r < R; ++r) y[p][base + r * Ns] = X[r];
  }
  __syncthreads();
}

__global__ __launch_bounds__(256) void logmel_kernel(
    const float* __restrict__ pcm, long long pcm_offset, long long n_samples, long long n_padded,
    long long frame0, int n_frames, const float* __restrict__ window, const float* __restrict__ twc,
    const float* __restrict__ tws, const float* __restrict__ filt, const int* __restrict__ flo,
    const int* __restrict__ fhi, int n_mels, float* __restrict__ out, long long ld,
    unsigned int* __restrict__ gmax) {
  constexpr int NP = FPB / 2;                          // complex transforms per block
  __shared__ float2 s_a[NP][NFFT];
  __shared__ float2 s_b[NP][NFFT];
  __shared__ float2 s_w[NFFT];
  __shared__ float s_p[FPB][NBIN + 3];
  __shared__ float s_red[4];
  const int tid = threadIdx.x;
  const long long fb = (long long)blockIdx.x * FPB;   // first local frame of this block

  for (int i = tid; i < NFFT; i += 256) s_w[i] = make_float2(twc[i], -tws[i]);   // e^{-2 pi i t / 400}
  for (int i = tid; i < NP * NFFT; i += 256) {
    const int p = i / NFFT, n = i - p * NFFT;
    float v2[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      float v = 0.f;
      const long long lf = fb + 2 * p + h;
      if (lf < n_frames) {
        long long sidx = (frame0 + lf) * HOP + n - NFFT / 2;      // file sample index before reflection
        if (sidx < 0) sidx = -sidx;
        if (sidx >= n_padded) sidx = 2 * (n_padded - 1) - sidx;
        if (sidx < n_samples) v = pcm[sidx - pcm_offset];
        v *= window[n];
      }
      v2[h] = v;
    }
    s_a[p][n] = make_float2(v2[0], v2[1]);
  }
  __syncthreads();
  fft_pass<4>(s_a, s_b, s_w, 1, NP);
  fft_pass<4>(s_b, s_a, s_w, 4, NP);
  fft_pass<5>(s_a, s_b, s_w, 16, NP);
  fft_pass<5>(s_b, s_a, s_w, 80, NP);
  // separate the two real frames and take |X|^2 for bins 0..200
  for (int it = tid; it < NP * NBIN; it += 256) {
    const int p = it / NBIN, k = it - p * NBIN;
    const float2 z = s_a[p][k], zc = s_a[p][(NFFT - k) % NFFT];
    const float ar = 0.5f * (z.x + zc.x), ai = 0.5f * (z.y - zc.y);          // (Z[k] + conj Z[-k]) / 2
    const float br = 0.5f * (z.y + zc.y), bi = -0.5f * (z.x - zc.x);         // (Z[k] - conj Z[-k]) / 2i
    s_p[2 * p][k] = fmaf(ar, ar, ai * ai);
    s_p[2 * p + 1][k] = fmaf(br, br, bi * bi);
  }
  __syncthreads();

  float lmax = -INFINITY;
  for (int it = tid; it < FPB * n_mels; it += 256) {
    const int m = it / FPB, f = it - m * FPB;
    const long long lf = fb + f;
    if (lf >= n_frames) continue;
    const float* w = filt + (long long)m * NBIN;
    float acc = 0.f;
    for (int k = flo[m]; k < fhi[m]; ++k) acc = fmaf(w[k], s_p[f][k], acc);
    const float lv = log10f(fmaxf(acc, 1e-10f));
    out[(long long)m * ld + lf] = lv;
    lmax = fmaxf(lmax, lv);
  }
  lmax = wave_max(lmax);
  if ((tid & 63) == 0) s_red[tid >> 6] = lmax;
  __syncthreads();
  if (tid == 0) {
    float m = fmaxf(fmaxf(s_red[0], s_red[1]), fmaxf(s_red[2], s_red[3]));
    if (m > -INFINITY) atomicMax(gmax, float_to_ordered(m));
  }
}

__global__ void logmel_clamp_kernel(float* __restrict__ mel, long long rows, long long cols, long long ld,
                                    const unsigned int* __restrict__ gmax, const float* __restrict__ gmax_f) {
  const float g = gmax_f ? gmax_f[0] : ordered_to_float(gmax[0]);
  const float lo = g - 8.0f;
  const long long n = rows * cols;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    const long long r = i / cols, c = i - r * cols;
    float* p = mel + r * ld + c;
    *p = (fmaxf(*p, lo) + 4.0f) * 0.25f;
  }
}

__global__ void ordered_to_float_kernel(const unsigned int* __restrict__ in, float* __restrict__ out) {
  out[0] = ordered_to_float(in[0]);
}

void launch_logmel(const float* pcm, long long pcm_offset, long long n_samples, long long n_padded,
                   long long frame0, int n_frames, const float* window, const float* twc, const float* tws,
                   const float* filt, const int* flo, const int* fhi, int n_mels, float* out, long long ld,
                   unsigned int* gmax, hipStream_t st) {
  if (n_frames <= 0) return;
  dim3 grid((n_frames + FPB - 1) / FPB);
  static const bool dft = [] {
    const char* e = std::getenv("VLOG_AMD_LOGMEL_DFT");
    return e && std::atoi(e) != 0;
  }();
  if (dft)
    hipLaunchKernelGGL(logmel_dft_kernel, grid, dim3(256), 0, st, pcm, pcm_offset, n_samples, n_padded, frame0,
                       n_frames, window, twc, tws, filt, flo, fhi, n_mels, out, ld, gmax);
  else
    hipLaunchKernelGGL(logmel_kernel, grid, dim3(256), 0, st, pcm, pcm_offset, n_samples, n_padded, frame0,
                       n_frames, window, twc, tws, filt, flo, fhi, n_mels, out, ld, gmax);
  WM_LAUNCH_CHECK("logmel_kernel");
}

void launch_logmel_clamp(float* mel, long long rows, long long cols, long long ld, const unsigned int* gmax,
                         const float* gmax_f, hipStream_t st) {
  long long n = rows * cols;
  if (n <= 0) return;
  int blocks = (int)((n + 255) / 256);
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(logmel_clamp_kernel, dim3(blocks), dim3(256), 0, st, mel, rows, cols, ld, gmax, gmax_f);
  WM_LAUNCH_CHECK("logmel_clamp_kernel");
}

void launch_ordered_to_float(const unsigned int* in, float* out, hipStream_t st) {
  hipLaunchKernelGGL(ordered_to_float_kernel, dim3(1), dim3(1), 0, st, in, out);
  WM_LAUNCH_CHECK("ordered_to_float_kernel");
}

// Per-frame log energy for the VAD stand-in: db[i] = 10*log10(mean(x^2) + 1e-12) over samples [i*W, i*W+W)
// (zero-padded tail), one wave per frame.
__global__ void frame_energy_kernel(const float* __restrict__ pcm, long long n, int W, int frames, float* __restrict__ db) {
  const int f = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (f >= frames) return;
  float s = 0.f;
  for (int i = lane; i < W; i += 64) {
    const long long k = (long long)f * W + i;
    const float v = k < n ? pcm[k] : 0.f;
    s = fmaf(v, v, s);
  }
  s = wave_sum(s);
  if (lane == 0) db[f] = 10.0f * log10f(s / W + 1e-12f);
}

void launch_frame_energy(const float* pcm, long long n, int W, int frames, float* db, hipStream_t st) {
  if (frames <= 0) return;
  hipLaunchKernelGGL(frame_energy_kernel, dim3((frames + 3) / 4), dim3(256), 0, st, pcm, n, W, frames, db);
  WM_LAUNCH_CHECK("frame_energy_kernel");
}

// Streaming ingest: s16le PCM (as the worker's ffmpeg extraction produces it) -> f32 x / 32768, the
// conversion faster-whisper's decode_audio applies.  8 samples per thread, 16-B loads.
__global__ void pcm_s16_kernel(const short* __restrict__ src, long long n, float* __restrict__ dst) {
  const long long i8 = ((long long)blockIdx.x * 256 + threadIdx.x) * 8;
  if (i8 + 8 <= n && ((reinterpret_cast<uintptr_t>(src + i8) & 15) == 0) && ((reinterpret_cast<uintptr_t>(dst + i8) & 15) == 0)) {
    const i32x4 v = *(const i32x4*)(src + i8);
    f32x4 lo, hi;
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      lo[2 * k] = (float)(short)(v[k] & 0xffff) * (1.0f / 32768.0f);
      lo[2 * k + 1] = (float)(short)((unsigned)v[k] >> 16) * (1.0f / 32768.0f);
      hi[2 * k] = (float)(short)(v[2 + k] & 0xffff) * (1.0f / 32768.0f);
      hi[2 * k + 1] = (float)(short)((unsigned)v[2 + k] >> 16) * (1.0f / 32768.0f);
    }
    *(f32x4*)(dst + i8) = lo;
    *(f32x4*)(dst + i8 + 4) = hi;
  } else {
    for (long long i = i8; i < i8 + 8 && i < n; ++i) dst[i] = (float)src[i] * (1.0f / 32768.0f);
  }
}

void launch_pcm_s16(const short* src, long long n, float* dst, hipStream_t st) {
  if (n <= 0) return;
  const long long threads = (n + 7) / 8;
  hipLaunchKernelGGL(pcm_s16_kernel, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, st, src, n, dst);
  WM_LAUNCH_CHECK("pcm_s16_kernel");
}
