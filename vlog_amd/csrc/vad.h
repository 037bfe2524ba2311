// Silero VAD v5 network on the device (vad.hip): weight pointers (f32, PyTorch layouts) and the launcher.
#pragma once
#include <hip/hip_runtime.h>

struct VadW {
  const float* basis;                 // STFT basis [258][256] (129 real rows, then 129 imaginary rows)
  const float* cw[4]; const float* cb[4];   // encoder convs [out][in][3], [out]
  const float* w_ih; const float* w_hh; const float* b_ih; const float* b_hh;   // LSTMCell [512][128], [512]
  const float* dec_w; const float* dec_b;                                       // head conv1x1 [128], [1]
};

// probs[t] for n_win windows of 512 samples of pcm; pre = n_win x 512 f32 scratch (gate pre-activations)
void launch_vad(const VadW& w, const float* pcm, long long n_win, float* pre, float* probs, hipStream_t st);
