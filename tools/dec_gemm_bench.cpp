// Decoder GEMM microbenchmark (tools only; not part of the product): the six per-layer decoder projections of
// large-v3 at M = 150 rows, timed back to back (a chain, as in a decode step) with HIP events, for
//   - the library's launch_gemm (skinny path + reduce),
//   - launch_dec_gemm at each K range KR (up-front loads, one wait),
//   - floors: an empty kernel, and a pure W stream (same grid, same bytes, no math).
// Outputs of every variant are compared with the launch_gemm output (max abs diff).
//   usage: dec_gemm_bench [reps] [M]
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>
#include "../vlog_amd/csrc/gemm.h"

void launch_dec_gemm_body(const GemmA& a, const bf16* w, long long ldw, int M, int N, int K, float* ws, int KR, int abl,
                          hipStream_t st);

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                                  \
    }                                                                                \
  } while (0)

static uint16_t f2b(float f) {
  uint32_t u;
  std::memcpy(&u, &f, 4);
  u += 0x7FFF + ((u >> 16) & 1);
  return (uint16_t)(u >> 16);
}
static float b2f(uint16_t b) {
  uint32_t u = (uint32_t)b << 16;
  float f;
  std::memcpy(&f, &u, 4);
  return f;
}

__global__ void empty_kernel(int x) {
  if (x == 12345) asm volatile("s_nop 0");
}

// pure weight stream: block (tile, split) reads 64 rows x kr of W with 16-B loads, no math beyond an xor
__global__ __launch_bounds__(256) void wstream_kernel(const bf16* __restrict__ w, int N, int K, int kr, int splitk,
                                                      unsigned* sink) {
  const int tile = blockIdx.x / splitk, split = blockIdx.x % splitk;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int n = tile * 64 + wid * 16 + (lane & 15);
  const int kb = split * kr, ke = min(K, kb + kr);
  const bf16* p = w + (long long)n * K + 8 * (lane >> 4);
  unsigned x = 0;
  for (int k = kb; k < ke; k += 32) {
    const i32x4 v = *(const i32x4*)(p + k);
    x ^= v[0] ^ v[1] ^ v[2] ^ v[3];
  }
  if (x == 0x9e3779b9u) sink[0] = x;
}

struct Shape {
  const char* name;
  int N, K, kind;
};

int main(int argc, char** argv) {
  const int reps = argc > 1 ? std::atoi(argv[1]) : 200;
  const int M = argc > 2 ? std::atoi(argv[2]) : 150;
  const Shape shapes[] = {
      {"qkv ", 3840, 1280, EPI_BF16}, {"out ", 1280, 1280, EPI_RESID_F32}, {"cq  ", 1280, 1280, EPI_BF16},
      {"fc1 ", 5120, 1280, EPI_BF16}, {"fc2 ", 1280, 5120, EPI_RESID_F32},
  };
  const int krs[] = {128, 192, 256, 320, 448};
  size_t maxW = 0;
  for (auto& s : shapes) maxW = std::max(maxW, (size_t)s.N * s.K);
  const size_t maxA = (size_t)M * (5120 + 64), maxC = (size_t)M * 5120;
  std::mt19937 rng(1);
  std::uniform_real_distribution<float> U(-1.f, 1.f);
  std::vector<uint16_t> hA(maxA), hW(maxW);
  for (auto& v : hA) v = f2b(U(rng));
  for (auto& v : hW) v = f2b(U(rng) * 0.05f);
  // distinct W copies rotated over the launches: 8 (default) stream from the 256 MB MALL; DGB_COPIES=40 puts every
  // launch's weights beyond it (cold, from HBM, as in a decode step, where 1.5 GB of weights cycle per pass)
  const int NCOPY = std::getenv("DGB_COPIES") ? std::max(1, std::atoi(std::getenv("DGB_COPIES"))) : 8;
  bf16 *dA, *dW;
  void *dC, *dRef;
  float* ws;
  unsigned* sink;
  const size_t wsb = 64ull << 20;
  // DGB_ACOPIES=n: n activation copies rotated with the weights (the big-rows sweep): each launch's A is then cold in
  // L2 and served from the MALL, as in a decode step where the previous kernel wrote it from every XCD
  const int ACOPY = std::getenv("DGB_ACOPIES") ? std::max(1, std::atoi(std::getenv("DGB_ACOPIES"))) : 1;
  CK(hipMalloc(&dA, maxA * 2 * ACOPY));
  CK(hipMalloc(&dW, maxW * 2 * NCOPY));
  CK(hipMalloc(&dC, maxC * 4));
  CK(hipMalloc(&dRef, maxC * 4));
  CK(hipMalloc(&ws, wsb));
  CK(hipMalloc(&sink, 16));
  for (int c = 0; c < ACOPY; ++c) CK(hipMemcpy(dA + maxA * c, hA.data(), maxA * 2, hipMemcpyHostToDevice));
  for (int c = 0; c < NCOPY; ++c) CK(hipMemcpy(dW + maxW * c, hW.data(), maxW * 2, hipMemcpyHostToDevice));
  hipStream_t st;
  CK(hipStreamCreate(&st));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto timeit = [&](auto&& fn) {
    for (int r = 0; r < 3; ++r) fn(r);
    CK(hipEventRecord(e0, st));
    for (int r = 0; r < reps; ++r) fn(r);
    CK(hipEventRecord(e1, st));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    return 1000.0 * ms / reps;
  };
  {
    const double us = timeit([&](int) { hipLaunchKernelGGL(empty_kernel, dim3(240), dim3(256), 0, st, 0); });
    std::printf("empty kernel (240 x 256)             %7.2f us\n", us);
  }
  // DGB_BIG=1: the large-pass ring plans only (beam-group row counts): rows per block x columns x LDS budget x K range
  // DGB_BIG=2: the same sweep over the 150-row plan's tiles and their 8-wave alternatives
  const int big_mode = std::getenv("DGB_BIG") ? std::atoi(std::getenv("DGB_BIG")) : 0;
  const bool big_only = big_mode == 1 || big_mode == 2;
  for (auto& s : shapes) {
    const double wbytes = 2.0 * s.N * s.K;
    GemmEpi ep;
    std::memset(&ep, 0, sizeof(ep));
    ep.kind = s.kind;
    ep.ldc = s.N;
    GemmA a{dA, (long long)s.K, 0, 0};
    const bool f32 = s.kind == EPI_RESID_F32;
    const size_t cbytes = (size_t)M * s.N * (f32 ? 4 : 2);
    ep.out = dRef;
    CK(hipMemsetAsync(dRef, 0, cbytes, st));
    launch_gemm(a, dW, s.K, M, s.N, s.K, ep, ws, wsb, st);
    std::vector<char> ref(cbytes), got(cbytes);
    CK(hipMemcpyAsync(ref.data(), dRef, cbytes, hipMemcpyDeviceToHost, st));
    CK(hipStreamSynchronize(st));
    auto maxdiff = [&]() {
      CK(hipMemcpy(got.data(), dC, cbytes, hipMemcpyDeviceToHost));
      double md = 0, mx = 0;
      for (size_t i = 0; i < (size_t)M * s.N; ++i) {
        const double x = f32 ? ((float*)ref.data())[i] : b2f(((uint16_t*)ref.data())[i]);
        const double y = f32 ? ((float*)got.data())[i] : b2f(((uint16_t*)got.data())[i]);
        md = std::max(md, std::fabs(x - y));
        mx = std::max(mx, std::fabs(x));
      }
      return md / (mx + 1e-30);
    };
    ep.out = dC;
    // the library path (times include its split-K reduce)
    {
      const double us = timeit([&](int r) {
        launch_gemm(a, dW + maxW * (r % NCOPY), s.K, M, s.N, s.K, ep, ws, wsb, st);
      });
      std::printf("%s N=%5d K=%5d  launch_gemm        %7.2f us  %7.1f GB/s(W)\n", s.name, s.N, s.K, us, wbytes / us / 1e3);
    }
    if (big_only) {
      struct BigCfg { int rpb, cols, lds, kr, waves; };
      const BigCfg cfgs[] = {{64, 64, 72, 0, 4},    {128, 64, 72, 0, 4},   {64, 32, 144, 0, 4},   {128, 128, 144, 0, 4},
                             {128, 128, 144, 0, 8}, {128, 64, 144, 0, 8},  {128, 64, 72, 0, 8},   {64, 128, 144, 0, 8},
                             {64, 64, 144, 0, 8},   {64, 64, 72, 0, 8},    {128, 128, 144, 640, 8}, {128, 128, 144, 1280, 8},
                             {128, 128, 144, 2560, 8}, {128, 64, 144, 2560, 8}, {64, 128, 144, 640, 8},
                             {64, 64, 72, 2560, 4},  {64, 64, 72, 1280, 4},  {64, 64, 72, 2560, 8}, {128, 64, 72, 1280, 8},
                             {128, 64, 72, 2560, 8}};
      const BigCfg cfgs150[] = {{96, 32, 144, 0, 4}, {32, 32, 144, 0, 4}, {64, 64, 144, 0, 4}, {64, 64, 144, 1280, 4},
                                {64, 64, 144, 0, 8}, {64, 64, 72, 0, 8}, {64, 64, 72, 0, 4}, {128, 64, 144, 0, 8},
                                {128, 64, 72, 0, 8}, {64, 128, 144, 0, 8}, {64, 64, 144, 1280, 8}, {64, 64, 72, 1280, 8},
                                {128, 64, 72, 1280, 8}, {32, 64, 144, 0, 4}, {64, 32, 144, 0, 4}};
      const int ncfg = big_mode == 2 ? (int)(sizeof(cfgs150) / sizeof(cfgs150[0])) : (int)(sizeof(cfgs) / sizeof(cfgs[0]));
      for (int ci = 0; ci < ncfg; ++ci) {
        const BigCfg& c = big_mode == 2 ? cfgs150[ci] : cfgs[ci];
        const int kr = c.kr >= s.K ? 0 : c.kr;
        if (c.kr && !kr) continue;
        CK(hipMemsetAsync(dC, 0, cbytes, st));
        if (!launch_dec_ring(a, dW, s.K, M, s.N, s.K, ep, ws, wsb, kr, st, c.rpb, c.cols, c.lds, c.waves)) {
          std::printf("%s ring rows=%d cols=%d lds=%d kr=%d waves=%d unsupported\n", s.name, c.rpb, c.cols, c.lds, kr, c.waves);
          continue;
        }
        CK(hipStreamSynchronize(st));
        const double err = f32 ? 0.0 : maxdiff();
        const double us = timeit([&](int r) {
          GemmA ar = a;
          ar.ptr = dA + maxA * (r % ACOPY);
          launch_dec_ring(ar, dW + maxW * (r % NCOPY), s.K, M, s.N, s.K, ep, ws, wsb, kr, st, c.rpb, c.cols, c.lds, c.waves);
        });
        std::printf("%s N=%5d K=%5d  RING rows=%3d cols=%3d lds=%3d kr=%4d w=%d %7.2f us  %7.1f TF/s  rel diff %.1e\n", s.name,
                    s.N, s.K, c.rpb, c.cols, c.lds, kr, c.waves, us, 2.0 * M * s.N * s.K / us / 1e6, err);
      }
      continue;
    }
    for (int pad : {0, 64}) {
      // pad: activation row stride K + pad (a 64-element pad moves consecutive rows to different L2 channels)
      const GemmA ap{dA, (long long)s.K + pad, 0, 0};
      for (int rpb : {0, 32, 64, 96, 128})
      for (int cols : {32, 64}) {
        if (cols == 64 && (pad || rpb == 0 || rpb == 96)) continue;
        for (int kr : {0, 640, 1280, 2560, 5120}) {
          if (kr > s.K || (kr > 0 && kr != s.K && s.K <= 1280)) continue;
          if (pad && kr != 0) continue;
          CK(hipMemsetAsync(dC, 0, cbytes, st));
          if (!launch_dec_ring(ap, dW, s.K, M, s.N, s.K, ep, ws, wsb, kr, st, rpb, cols)) {
            std::printf("ring kr=%d rows=%d unsupported\n", kr, rpb);
            continue;
          }
          CK(hipStreamSynchronize(st));
          const double err = f32 || pad ? 0.0 : maxdiff();
          const double us = timeit([&](int r) {
            launch_dec_ring(ap, dW + maxW * (r % NCOPY), s.K, M, s.N, s.K, ep, ws, wsb, kr, st, rpb, cols);
          });
          std::printf("%s N=%5d K=%5d  RING kr=%4d rows=%3d cols=%2d pad=%2d %7.2f us  %7.1f GB/s(W)  rel diff %.1e\n", s.name, s.N,
                      s.K, kr, rpb, cols, pad, us, wbytes / us / 1e3, err);
        }
      }
    }
    for (int nc : {2, 4}) {
      CK(hipMemsetAsync(dC, 0, cbytes, st));
      if (!launch_dec_oneshot(a, dW, s.K, M, s.N, s.K, ep, ws, wsb, nc, st)) { std::printf("oneshot nc=%d unsupported\n", nc); continue; }
      CK(hipStreamSynchronize(st));
      const double err = f32 ? 0.0 : maxdiff();
      const double us = timeit([&](int r) {
        launch_dec_oneshot(a, dW + maxW * (r % NCOPY), s.K, M, s.N, s.K, ep, ws, wsb, nc, st);
      });
      std::printf("%s N=%5d K=%5d  ONESHOT nc=%d        %7.2f us  %7.1f GB/s(W)  rel diff %.1e\n", s.name, s.N, s.K, nc, us,
                  wbytes / us / 1e3, err);
    }
    for (int kr : krs) {
      if (kr > s.K) continue;
      CK(hipMemsetAsync(dC, 0, cbytes, st));
      if (!launch_dec_gemm(a, dW, s.K, M, s.N, s.K, ep, ws, wsb, kr, st)) continue;
      CK(hipStreamSynchronize(st));
      const double err = f32 ? 0.0 : maxdiff();     // RESID_F32 accumulates into C: compare bf16 kinds only
      const double us = timeit([&](int r) {
        launch_dec_gemm(a, dW + maxW * (r % NCOPY), s.K, M, s.N, s.K, ep, ws, wsb, kr, st);
      });
      const int sk = (s.K + kr - 1) / kr;
      std::printf("%s N=%5d K=%5d  dec KR=%3d s=%2d    %7.2f us  %7.1f GB/s(W)  rel diff %.1e  blocks %d\n", s.name, s.N,
                  s.K, kr, sk, us, wbytes / us / 1e3, err, s.N / 64 * sk);
      const double us2 = timeit([&](int r) {
        hipLaunchKernelGGL(wstream_kernel, dim3(s.N / 64 * sk), dim3(256), 0, st, dW + maxW * (r % NCOPY), s.N, s.K, kr,
                           sk, sink);
      });
      std::printf("%s                  W stream only      %7.2f us  %7.1f GB/s(W)\n", s.name, us2, wbytes / us2 / 1e3);
      if (s.kind == EPI_BF16 && (kr == 128 || kr == 256 || kr == 448)) {
        for (int abl : {0, 1, 2, 4, 7}) {
          const double u = timeit([&](int r) {
            launch_dec_gemm_body(a, dW + maxW * (r % NCOPY), s.K, M, s.N, s.K, ws, kr, abl, st);
          });
          std::printf("%s                  body abl=%d         %7.2f us  (skip:%s%s%s)\n", s.name, abl, u,
                      (abl & 1) ? " A-dma" : "", (abl & 2) ? " mfma" : "", (abl & 4) ? " store" : "");
        }
        const int sk2 = (s.K + kr - 1) / kr;
        const double u = timeit([&](int) { launch_splitk_combine(ws, sk2, M, s.N, ep, st); });
        std::printf("%s                  combine alone      %7.2f us\n", s.name, u);
      }
    }
  }
  return 0;
}
