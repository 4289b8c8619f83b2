// GEMM tile/pipeline tuning harness (measurement tool, not part of the library).
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/gemm_tune.hip build/obj/capi.o -o tools/gemm_tune
// Times each kernel variant of gemm.hpp / gemm2.hpp on a set of bf16 shapes with HIP events
// (median of 20 launches after 3 warm-ups) and checks every variant against the first one.
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>
#include <functional>
#include <string>
#include <cmath>

#include "../retr_amd/csrc/gemm2.hpp"
#include "../retr_amd/csrc/epilogues.hpp"

using namespace retr;

#define CHK(x)                                                                   \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) {                                                      \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                   \
    }                                                                            \
  } while (0)

__global__ void fill_kernel(bf16* p, long n, unsigned seed) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    unsigned x = (unsigned)i * 2654435761u + seed;
    x ^= x >> 13; x *= 0x5bd1e995u; x ^= x >> 15;
    p[i] = (bf16)(((x & 0xffff) / 65536.f) - 0.5f);
  }
}

struct Shape { int M, N, K; bool trans; const char* what; };

int main(int argc, char** argv) {
  const bool deep = argc > 1 && std::string(argv[1]) == "deep";
  std::vector<Shape> shapes = {
      {4096, 4096, 4096, false, "dense 4k"},
      {25600, 256, 2304, false, "conv3x3 40x40 256"},
      {409600, 64, 576, false, "conv3x3 160x160 64"},
      {102400, 128, 1152, false, "conv3x3 80x80 128"},
      {6400, 2048, 512, false, "conv1x1 20x20 512->2048"},
      {25600, 1024, 256, false, "conv1x1 40x40 256->1024"},
      {409600, 256, 64, false, "conv1x1 160x160 64->256"},
      {102400, 512, 128, false, "conv1x1 80x80 128->512"},
      {2048, 30528, 512, false, "head fwd"},
      {256, 2304, 25600, true, "wgrad 3x3 40x40 256"},
      {1024, 256, 25600, true, "wgrad 1x1 40x40 256->1024"},
      {128, 256, 409600, true, "wgrad 1x1 160x160 256->128"},
  };
  size_t maxA = 0, maxB = 0, maxC = 0;
  for (auto& s : shapes) {
    maxA = std::max(maxA, (size_t)s.M * s.K);
    maxB = std::max(maxB, (size_t)s.N * s.K);
    maxC = std::max(maxC, (size_t)s.M * s.N * (s.trans ? 64 : 1));
  }
  bf16 *A, *B;
  float *C, *C0;
  CHK(hipMalloc(&A, maxA * 2));
  CHK(hipMalloc(&B, maxB * 2));
  CHK(hipMalloc(&C, maxC * 4));
  CHK(hipMalloc(&C0, maxC * 4));
  hipLaunchKernelGGL(fill_kernel, dim3(4096), dim3(256), 0, 0, A, (long)maxA, 1u);
  hipLaunchKernelGGL(fill_kernel, dim3(4096), dim3(256), 0, 0, B, (long)maxB, 7u);
  CHK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0));
  CHK(hipEventCreate(&e1));

  for (auto& s : shapes) {
    if (deep && s.trans) continue;
    const int M = s.M, N = s.N, K = s.K;
    const double flop = 2.0 * M * N * K;
    std::vector<std::pair<std::string, std::function<int(float*)>>> vars;
    if (!s.trans) {
      DenseK<bf16> la{A, (long)K, M, K};
      DenseK<bf16> lb{B, (long)K, N, K};
      auto ep = [=](float* out) { EpiFwd<float, float> e{out, (long)N, nullptr, nullptr, 0, 0, DropoutParams{0, 0, 1.f}, 0}; e.set_vec(); return e; };
      vars.push_back({"reg128x128", [=](float* o) { return launch_gemm<0, bf16, 128, 128>(la, lb, ep(o), M, N, K, 1, 0, "v"); }});
      vars.push_back({"g128x128s2", [=](float* o) { return launch_gemm2<0, 128, 128, 2, 2, 2>(la, lb, ep(o), M, N, K, 1, 0, "v"); }});
      vars.push_back({"g128x128s1e2", [=](float* o) { return launch_gemm2<0, 128, 128, 2, 2, 1, 2>(la, lb, ep(o), M, N, K, 1, 0, "v"); }});
      vars.push_back({"g128x128s2e2", [=](float* o) { return launch_gemm2<0, 128, 128, 2, 2, 2, 2>(la, lb, ep(o), M, N, K, 1, 0, "v"); }});
      vars.push_back({"g256x256s2", [=](float* o) { return launch_gemm2<0, 256, 256, 2, 4, 2>(la, lb, ep(o), M, N, K, 1, 0, "v"); }});
      vars.push_back({"g128x64s3", [=](float* o) { return launch_gemm2<0, 128, 64, 2, 2, 3>(la, lb, ep(o), M, N, K, 1, 0, "v"); }});
      if (deep) {
        // pipeline depth vs blocks per CU (tiles in flight per CU = blocks x (S - 1))
        vars.push_back({"g128x128s3", [=](float* o) { return launch_gemm2<0, 128, 128, 2, 2, 3>(la, lb, ep(o), M, N, K, 1, 0, "v"); }});
        vars.push_back({"g128x128s4", [=](float* o) { return launch_gemm2<0, 128, 128, 2, 2, 4>(la, lb, ep(o), M, N, K, 1, 0, "v"); }});
        vars.push_back({"g128x128w8s2", [=](float* o) { return launch_gemm2<0, 128, 128, 4, 2, 2>(la, lb, ep(o), M, N, K, 1, 0, "v"); }});
        vars.push_back({"g128x128w8s3", [=](float* o) { return launch_gemm2<0, 128, 128, 4, 2, 3>(la, lb, ep(o), M, N, K, 1, 0, "v"); }});
        vars.push_back({"g128x128w8s4", [=](float* o) { return launch_gemm2<0, 128, 128, 4, 2, 4>(la, lb, ep(o), M, N, K, 1, 0, "v"); }});
        vars.push_back({"g256x128w8s2", [=](float* o) { return launch_gemm2<0, 256, 128, 4, 2, 2>(la, lb, ep(o), M, N, K, 1, 0, "v"); }});
        vars.push_back({"g256x128w8s3", [=](float* o) { return launch_gemm2<0, 256, 128, 4, 2, 3>(la, lb, ep(o), M, N, K, 1, 0, "v"); }});
        vars.push_back({"g128x256w8s3", [=](float* o) { return launch_gemm2<0, 128, 256, 2, 4, 3>(la, lb, ep(o), M, N, K, 1, 0, "v"); }});
        vars.push_back({"g64x128s4", [=](float* o) { return launch_gemm2<0, 64, 128, 2, 2, 4>(la, lb, ep(o), M, N, K, 1, 0, "v"); }});
      }
    } else {
      // weight-gradient form: both operands row-contiguous ([k][rows]), split-K partial slabs
      DenseT<bf16> la{A, (long)M, M, K};
      DenseT<bf16> lb{B, (long)N, N, K};
      auto mk = [=](float* out, int splits) { EpiAccF32 e{out, (long)N, 0, 0, 1, nullptr}; e.split_stride = splits > 1 ? (long)M * N : 0; e.set_vec(); return e; };
      for (int sp : {8, 16, 32, 64}) {
        char nm[64];
        snprintf(nm, sizeof nm, "g128x128s2 sk%d", sp);
        vars.push_back({nm, [=](float* o) { return launch_gemm2<0, 128, 128, 2, 2, 2>(la, lb, mk(o, sp), M, N, K, sp, 0, "v"); }});
        snprintf(nm, sizeof nm, "reg128x128 sk%d", sp);
        vars.push_back({nm, [=](float* o) { return launch_gemm<0, bf16, 128, 128>(la, lb, mk(o, sp), M, N, K, sp, 0, "v"); }});
      }
    }
    printf("== %s  M=%d N=%d K=%d\n", s.what, M, N, K);
    bool first = true;
    for (auto& v : vars) {
      float* out = first ? C0 : C;
      for (int i = 0; i < 3; ++i)
        if (v.second(out)) { printf("  %-18s launch failed\n", v.first.c_str()); break; }
      CHK(hipDeviceSynchronize());
      std::vector<float> ts;
      for (int i = 0; i < 20; ++i) {
        CHK(hipEventRecord(e0, 0));
        v.second(out);
        CHK(hipEventRecord(e1, 0));
        CHK(hipEventSynchronize(e1));
        float ms;
        CHK(hipEventElapsedTime(&ms, e0, e1));
        ts.push_back(ms);
      }
      std::sort(ts.begin(), ts.end());
      const float ms = ts[ts.size() / 2];
      double err = 0;
      if (!first && !s.trans) {
        std::vector<float> h0((size_t)M * N), h1((size_t)M * N);
        CHK(hipMemcpy(h0.data(), C0, h0.size() * 4, hipMemcpyDeviceToHost));
        CHK(hipMemcpy(h1.data(), C, h1.size() * 4, hipMemcpyDeviceToHost));
        double num = 0, den = 0;
        for (size_t i = 0; i < h0.size(); i += 7) { num += (h0[i] - h1[i]) * (double)(h0[i] - h1[i]); den += (double)h0[i] * h0[i]; }
        err = std::sqrt(num / (den + 1e-30));
      }
      printf("  %-18s %9.1f us %8.1f TF/s  err %.1e\n", v.first.c_str(), ms * 1e3, flop / (ms * 1e-3) / 1e12, err);
      first = false;
    }
    fflush(stdout);
  }
  return 0;
}
