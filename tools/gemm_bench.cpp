// GEMM microbenchmark for the library's launch_gemm (tools only; not part of the product).
// Times C = A . W^T on the encoder / cross-KV / decoder shapes with HIP events and spot-checks 256 output
// elements against a host dot product of the same bf16 inputs.
//   usage: gemm_bench [reps]          (VLOG_AMD_GEMM_BIG=0 / VLOG_AMD_GEMM_SKINNY=0 select the other paths)
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>
#include "../vlog_amd/csrc/gemm.h"

void launch_gemm_8p_abl(const GemmA& a, const bf16* w, long long ldw, int M, int N, int K, const GemmEpi& epi, int abl,
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

struct Shape {
  const char* name;
  int M, N, K, kind;
};

int main(int argc, char** argv) {
  const int reps = argc > 1 ? std::atoi(argv[1]) : 5;
  const Shape shapes[] = {
      {"enc.qkv  (16 win)", 24000, 3840, 1280, EPI_BF16},
      {"enc.fc1  (16 win)", 24000, 5120, 1280, EPI_BF16},
      {"enc.fc2  (16 win)", 24000, 1280, 5120, EPI_RESID_F32},
      {"enc.out  (16 win)", 24000, 1280, 1280, EPI_RESID_F32},
      {"cross-kv (16 win)", 24000, 81920, 1280, EPI_BF16},
      {"tiny.qkv (16 win)", 24000, 1152, 384, EPI_BF16},
      {"tiny.fc2 (ragged)", 3001, 384, 1536, EPI_RESID_F32},
      {"dec.qkv  (150 rows)", 150, 3840, 1280, EPI_BF16},
      {"dec.fc1  (150 rows)", 150, 5120, 1280, EPI_BF16},
      {"dec.fc2  (150 rows)", 150, 1280, 5120, EPI_RESID_F32},
      {"dec.out  (150 rows)", 150, 1280, 1280, EPI_RESID_F32},
      {"square 4096", 4096, 4096, 4096, EPI_BF16},             // the guide's 8-phase template reference shape
      {"square 8192", 8192, 8192, 8192, EPI_BF16},
      {"enc.qkv K=4096", 24000, 3840, 4096, EPI_BF16},         // same tiles, 3.2x the K loop
      {"enc.qkv (150 win)", 225000, 3840, 1280, EPI_BF16},     // the bench's encoder pass (150 windows)
      {"enc.fc1 (150 win)", 225000, 5120, 1280, EPI_BF16},
      {"enc.out (150 win)", 225000, 1280, 1280, EPI_RESID_F32},
  };
  size_t maxA = 0, maxW = 0, maxC = 0;
  for (auto& s : shapes) {
    maxA = std::max(maxA, (size_t)s.M * s.K);
    maxW = std::max(maxW, (size_t)s.N * s.K);
    maxC = std::max(maxC, (size_t)s.M * s.N);
  }
  std::mt19937 rng(1);
  std::uniform_real_distribution<float> U(-1.f, 1.f);
  std::vector<uint16_t> hA(maxA), hW(maxW);
  for (auto& v : hA) v = f2b(U(rng));
  for (auto& v : hW) v = f2b(U(rng) * 0.05f);
  bf16 *dA, *dW;
  void* dC;
  float* ws;
  const size_t wsb = 64ull << 20;
  CK(hipMalloc(&dA, maxA * 2));
  CK(hipMalloc(&dW, maxW * 2));
  CK(hipMalloc(&dC, maxC * 4));
  CK(hipMalloc(&ws, wsb));
  CK(hipMemcpy(dA, hA.data(), maxA * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(dW, hW.data(), maxW * 2, hipMemcpyHostToDevice));
  hipStream_t st;
  CK(hipStreamCreate(&st));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const char* only = std::getenv("GEMM_ONLY");   // run only the shapes whose name contains this
  for (auto& s : shapes) {
    if (only && !std::strstr(s.name, only)) continue;
    GemmEpi ep;
    std::memset(&ep, 0, sizeof(ep));
    ep.kind = s.kind;
    ep.out = dC;
    ep.ldc = s.N;
    GemmA a{dA, (long long)s.K, 0, 0};
    CK(hipMemsetAsync(dC, 0, (size_t)s.M * s.N * 4, st));
    launch_gemm(a, dW, s.K, s.M, s.N, s.K, ep, ws, wsb, st);     // reference output (one launch)
    CK(hipStreamSynchronize(st));
    // spot check
    const bool f32 = s.kind == EPI_RESID_F32;
    std::vector<char> out((size_t)s.M * s.N * (f32 ? 4 : 2));
    CK(hipMemcpy(out.data(), dC, out.size(), hipMemcpyDeviceToHost));
    double maxerr = 0;
    std::mt19937 r2(7);
    for (int t = 0; t < 256; ++t) {
      const int m = (int)(r2() % s.M), n = (int)(r2() % s.N);
      double ref = 0;
      for (int k = 0; k < s.K; ++k) ref += (double)b2f(hA[(size_t)m * s.K + k]) * b2f(hW[(size_t)n * s.K + k]);
      const double got = f32 ? ((float*)out.data())[(size_t)m * s.N + n] : b2f(((uint16_t*)out.data())[(size_t)m * s.N + n]);
      maxerr = std::max(maxerr, std::fabs(got - ref) / (1.0 + std::fabs(ref)));
    }
    CK(hipEventRecord(e0, st));
    for (int r = 0; r < reps; ++r) launch_gemm(a, dW, s.K, s.M, s.N, s.K, ep, ws, wsb, st);
    CK(hipEventRecord(e1, st));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double us = 1000.0 * ms / reps;
    const double tf = 2.0 * s.M * s.N * s.K / (us * 1e-6) / 1e12;
    const double gbs = 2.0 * ((double)s.M * s.K + (double)s.N * s.K) / (us * 1e-6) / 1e9;
    std::printf("%-20s M=%6d N=%6d K=%5d  %10.1f us  %7.1f TF/s  %7.1f GB/s(A+W)  max rel err %.2e %s\n", s.name, s.M,
                s.N, s.K, us, tf, gbs, maxerr, maxerr < 2e-2 ? "ok" : "BAD");
  }
  // ablations of the 8-phase encoder GEMM on the qkv / fc1 shapes (bit 0: no epilogue, 1: no MFMA, 2: no DMA)
  if (std::getenv("GEMM_ABL")) {
    for (auto& s : shapes) {
      if (s.M < 1024 || s.kind != EPI_BF16 || s.N > 8192) continue;
      GemmEpi ep;
      std::memset(&ep, 0, sizeof(ep));
      ep.kind = EPI_BF16;
      ep.out = dC;
      ep.ldc = s.N;
      GemmA a{dA, (long long)s.K, 0, 0};
      for (int abl : {0, 1, 2, 3, 4, 5, 7}) {
        launch_gemm_8p_abl(a, dW, s.K, s.M, s.N, s.K, ep, abl, st);
        CK(hipEventRecord(e0, st));
        for (int r = 0; r < reps; ++r) launch_gemm_8p_abl(a, dW, s.K, s.M, s.N, s.K, ep, abl, st);
        CK(hipEventRecord(e1, st));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        const double us = 1000.0 * ms / reps;
        std::printf("%-20s 8p abl=%d (skip%s%s%s)  %9.1f us  %7.1f TF/s\n", s.name, abl, (abl & 1) ? " epi" : "",
                    (abl & 2) ? " mfma" : "", (abl & 4) ? " dma" : "", us, 2.0 * s.M * s.N * s.K / (us * 1e-6) / 1e12);
      }
    }
  }
  return 0;
}
