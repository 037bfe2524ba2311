// Silero VAD v5 (16 kHz) speech probabilities on gfx950 — faster-whisper's vad_filter=True model [FW↑
// vad.py SileroVADModel], reached from the worker's call (reference worker/transcription.py:110).
//
// faster-whisper 1.1 runs Silero as two ONNX graphs: an encoder batched over every 512-sample window (each
// prefixed with the previous window's last 64 samples) and an LSTM decoder over the window sequence.  The
// same split maps onto the GPU:
//   vad_encoder_kernel : one workgroup per VAD_WB windows, f32 throughout —
//       x (576 samples) reflect-padded by 64 on the right -> STFT by a learned-basis conv (258 x 256, stride
//       128: 4 frames) -> magnitude (129 bins) -> conv(129->128,k3,p1)+ReLU -> conv(128->64,k3,s2,p1)+ReLU ->
//       conv(64->64,k3,s2,p1)+ReLU -> conv(64->128,k3,p1)+ReLU (1 frame) -> the LSTM input projection
//       W_ih x + b_ih + b_hh (512 gate pre-activations), written per window.
//   vad_lstm_kernel    : ONE 512-thread workgroup walks the windows in order: gates = pre[t] + W_hh h, LSTMCell
//       (i, f, g, o), one barrier per window;
//   vad_head_kernel    : sigmoid(w . relu(h_t) + b) for every window in parallel.
// Weight layouts are PyTorch's (conv [out][in][k], LSTM [4*128][128]); see include/whisper_mi355.h.
#include "common.h"
#include "vad.h"
#include <stdexcept>
#include <string>


// VAD_WB windows per workgroup: every weight fetched from L2 feeds VAD_WB windows.
#define VAD_WB 4

// conv1d over a short time axis held in LDS, for VAD_WB windows (in/out [VAD_WB][c][t]):
// out[o][f] = relu(b[o] + sum_{i,k} w[o][i][k] in[i][f*s + k - 1])
__device__ __forceinline__ void vad_conv(const float* __restrict__ w, const float* __restrict__ b, const float* in,
                                         int cin, int tin, float* out, int cout, int tout, int stride) {
  for (int idx = threadIdx.x; idx < cout * tout; idx += blockDim.x) {
    const int o = idx / tout, f = idx - o * tout;
    float acc[VAD_WB];
#pragma unroll
    for (int v = 0; v < VAD_WB; ++v) acc[v] = b[o];
    const float* wr = w + (long long)o * cin * 3;
#pragma unroll 2
    for (int i = 0; i < cin; ++i) {
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        const int t = f * stride + k - 1;
        if (t >= 0 && t < tin) {
          const float wv = wr[i * 3 + k];
#pragma unroll
          for (int v = 0; v < VAD_WB; ++v) acc[v] = fmaf(wv, in[(v * cin + i) * tin + t], acc[v]);
        }
      }
    }
#pragma unroll
    for (int v = 0; v < VAD_WB; ++v) out[(v * cout + o) * tout + f] = fmaxf(acc[v], 0.f);
  }
  __syncthreads();
}

__global__ __launch_bounds__(256) void vad_encoder_kernel(VadW w, const float* __restrict__ pcm, long long n_win,
                                                          float* __restrict__ pre) {
  __shared__ float xs[VAD_WB][640];
  __shared__ float spec[VAD_WB][258 * 4];
  __shared__ float mag[VAD_WB * 129 * 4];
  __shared__ float a1[VAD_WB * 128 * 4];
  __shared__ float a2[VAD_WB * 64 * 2];
  __shared__ float a3[VAD_WB * 64];
  __shared__ float a4[VAD_WB][128];
  const long long t0 = (long long)blockIdx.x * VAD_WB;
  const int tid = threadIdx.x;
  // window t = [64 context samples (previous window's tail; zeros before the first)] + 512 samples, then a
  // reflection of 64 on the right (x[576 + j] = x[574 - j]); windows past n_win read zeros and are not stored
  for (int j = tid; j < VAD_WB * 576; j += 256) {
    const int v = j / 576, jj = j - v * 576;
    const long long s = (t0 + v) * 512 + jj - 64;
    xs[v][jj] = (s >= 0 && t0 + v < n_win) ? pcm[s] : 0.f;
  }
  __syncthreads();
  if (tid < VAD_WB * 64) xs[tid >> 6][576 + (tid & 63)] = xs[tid >> 6][574 - (tid & 63)];
  __syncthreads();
  for (int r = tid; r < 258; r += 256) {
    const float4* br = (const float4*)(w.basis + (long long)r * 256);
    float acc[VAD_WB][4] = {};
#pragma unroll 2
    for (int k4 = 0; k4 < 64; ++k4) {
      const float4 bv = br[k4];
#pragma unroll
      for (int v = 0; v < VAD_WB; ++v)
#pragma unroll
        for (int f = 0; f < 4; ++f) {
          const float4 xv = *(const float4*)&xs[v][f * 128 + 4 * k4];
          acc[v][f] = fmaf(bv.x, xv.x, acc[v][f]);
          acc[v][f] = fmaf(bv.y, xv.y, acc[v][f]);
          acc[v][f] = fmaf(bv.z, xv.z, acc[v][f]);
          acc[v][f] = fmaf(bv.w, xv.w, acc[v][f]);
        }
    }
#pragma unroll
    for (int v = 0; v < VAD_WB; ++v)
#pragma unroll
      for (int f = 0; f < 4; ++f) spec[v][r * 4 + f] = acc[v][f];
  }
  __syncthreads();
  for (int idx = tid; idx < VAD_WB * 129 * 4; idx += 256) {
    const int v = idx / (129 * 4), e = idx - v * 129 * 4;
    const float re = spec[v][e], im = spec[v][129 * 4 + e];
    mag[idx] = sqrtf(re * re + im * im);
  }
  __syncthreads();
  vad_conv(w.cw[0], w.cb[0], mag, 129, 4, a1, 128, 4, 1);
  vad_conv(w.cw[1], w.cb[1], a1, 128, 4, a2, 64, 2, 2);
  vad_conv(w.cw[2], w.cb[2], a2, 64, 2, a3, 64, 1, 2);
  vad_conv(w.cw[3], w.cb[3], a3, 64, 1, &a4[0][0], 128, 1, 1);
  // LSTM input projection for these windows
  for (int j = tid; j < 512; j += 256) {
    const float4* wr = (const float4*)(w.w_ih + (long long)j * 128);
    float acc[VAD_WB];
#pragma unroll
    for (int v = 0; v < VAD_WB; ++v) acc[v] = w.b_ih[j] + w.b_hh[j];
#pragma unroll 2
    for (int k4 = 0; k4 < 32; ++k4) {
      const float4 wv = wr[k4];
#pragma unroll
      for (int v = 0; v < VAD_WB; ++v) {
        const float4 xv = *(const float4*)&a4[v][4 * k4];
        acc[v] = fmaf(wv.x, xv.x, acc[v]);
        acc[v] = fmaf(wv.y, xv.y, acc[v]);
        acc[v] = fmaf(wv.z, xv.z, acc[v]);
        acc[v] = fmaf(wv.w, xv.w, acc[v]);
      }
    }
#pragma unroll
    for (int v = 0; v < VAD_WB; ++v)
      if (t0 + v < n_win) pre[(t0 + v) * 512 + j] = acc[v];
  }
}

// Sequential LSTMCell over the windows.  512 threads: thread (k, q) = (tid / 4, tid % 4) owns unit k and the
// quarter q of h, keeping W_hh[g*128 + k][32q .. 32q+31] for the four gates g in registers; the four quarter
// sums of each gate meet by two lane shuffles (the quad is inside one wave), every thread of the quad then runs
// the cell for unit k, and ONE barrier per step publishes h (double-buffered in LDS).  Gate pre-activations are
// loaded VAD_DEPTH steps ahead (thread (k, q) loads gate q of unit k); h_t overwrites the already-consumed
// pre[t][0..127] and the sigmoid head runs afterwards over all windows in parallel (vad_head_kernel).
#define VAD_DEPTH 8
__device__ __forceinline__ float fsig(float x) { return __builtin_amdgcn_rcpf(1.0f + __expf(-x)); }
// quad exchange by DPP (no LDS round trip): 0xB1 = quad_perm(1,0,3,2), 0x4E = quad_perm(2,3,0,1)
template <int CTRL>
__device__ __forceinline__ float quad_swap(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float ftanh(float x) { return 2.0f * fsig(2.0f * x) - 1.0f; }

__global__ __launch_bounds__(512) void vad_lstm_kernel(VadW w, float* __restrict__ pre, long long n_win) {
  __shared__ float hs[2][128];
  const int tid = threadIdx.x, k = tid >> 2, q = tid & 3;
  typedef __attribute__((ext_vector_type(2))) float f32x2;
  f32x2 wr[4][16];                                 // packed pairs: the products run as v_pk_fma_f32
#pragma unroll
  for (int g = 0; g < 4; ++g)
#pragma unroll
    for (int i = 0; i < 32; i += 4) {
      const float4 v = *(const float4*)(w.w_hh + (long long)(g * 128 + k) * 128 + q * 32 + i);
      wr[g][i / 2] = f32x2{v.x, v.y};
      wr[g][i / 2 + 1] = f32x2{v.z, v.w};
    }
  float c = 0.f;
  if (tid < 128) hs[0][tid] = 0.f;
  float ring[VAD_DEPTH];
#pragma unroll
  for (int d = 0; d < VAD_DEPTH; ++d) ring[d] = d < n_win ? pre[(long long)d * 512 + q * 128 + k] : 0.f;
  __syncthreads();
  for (long long t = 0; t < n_win; t += VAD_DEPTH) {
#pragma unroll
    for (int d = 0; d < VAD_DEPTH; ++d) {
      const long long tt = t + d;
      if (tt >= n_win) break;                      // uniform over the block
      const int cur = d & 1;                       // VAD_DEPTH is even: buffer parity follows tt
      f32x2 a[4][2];
#pragma unroll
      for (int g = 0; g < 4; ++g) { a[g][0] = f32x2{g == q ? ring[d] : 0.f, 0.f}; a[g][1] = f32x2{0.f, 0.f}; }
      const long long nx = tt + VAD_DEPTH;
      ring[d] = nx < n_win ? pre[nx * 512 + q * 128 + k] : 0.f;
      const float4* hq = (const float4*)&hs[cur][q * 32];
#pragma unroll
      for (int i4 = 0; i4 < 8; ++i4) {
        const float4 hv = hq[i4];
        const f32x2 h01 = f32x2{hv.x, hv.y}, h23 = f32x2{hv.z, hv.w};
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          a[g][0] = __builtin_elementwise_fma(wr[g][2 * i4], h01, a[g][0]);
          a[g][1] = __builtin_elementwise_fma(wr[g][2 * i4 + 1], h23, a[g][1]);
        }
      }
      float s[4];
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const f32x2 p = a[g][0] + a[g][1];
        s[g] = p.x + p.y;
        s[g] += quad_swap<0xB1>(s[g]);
        s[g] += quad_swap<0x4E>(s[g]);
      }
      const float ig = fsig(s[0]), fg = fsig(s[1]), gg = ftanh(s[2]), og = fsig(s[3]);
      c = fg * c + ig * gg;
      const float h = og * ftanh(c);
      if (q == 0) {
        hs[cur ^ 1][k] = h;
        pre[tt * 512 + k] = h;                     // consumed by this thread VAD_DEPTH steps ago
      }
      __syncthreads();
    }
  }
}

// probs[t] = sigmoid(head_w . relu(h_t) + head_b), h_t in pre[t][0..127]; one wave per window
__global__ __launch_bounds__(256) void vad_head_kernel(VadW w, const float* __restrict__ pre, long long n_win,
                                                       float* __restrict__ probs) {
  const long long t = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (t >= n_win) return;
  const float* h = pre + t * 512;
  float y = fmaxf(h[lane], 0.f) * w.dec_w[lane] + fmaxf(h[lane + 64], 0.f) * w.dec_w[lane + 64];
  y = wave_sum(y);
  if (lane == 0) probs[t] = 1.0f / (1.0f + expf(-(y + w.dec_b[0])));
}

void launch_vad(const VadW& w, const float* pcm, long long n_win, float* pre, float* probs, hipStream_t st) {
  if (n_win <= 0) return;
  hipLaunchKernelGGL(vad_encoder_kernel, dim3((unsigned)((n_win + VAD_WB - 1) / VAD_WB)), dim3(256), 0, st, w, pcm,
                     n_win, pre);
  WM_LAUNCH_CHECK("vad_encoder_kernel");
  hipLaunchKernelGGL(vad_lstm_kernel, dim3(1), dim3(512), 0, st, w, pre, n_win);
  WM_LAUNCH_CHECK("vad_lstm_kernel");
  hipLaunchKernelGGL(vad_head_kernel, dim3((unsigned)((n_win + 3) / 4)), dim3(256), 0, st, w, pre, n_win, probs);
  WM_LAUNCH_CHECK("vad_head_kernel");
}
