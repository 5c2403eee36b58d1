// Residual-linear tile lab: the 128x128 counted residual epilogue (ROLE 1 / 4 / 5) against
// smaller tiles with more blocks per CU (epilogue HBM traffic of one block overlapping the
// K loops of the others) on the per-stream decoder shapes; bitwise check against 128x128.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I zipvoice_amd/csrc tools/lab/gemm_res_lab.hip -o tools/lab/gemm_res_lab
//   gemm_res_lab [rounds] [mode,...] [MxNxK;...]   modes: 1 residual, 2 + bypass original, 4 + row vector, 5 = 4 copy only, 3 bias + SwooshL -> bf16
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>
#include <array>
#include <algorithm>

#include "zv_gemm256.inc"

ZvProfiler g_zv_prof;

static __global__ void fill_rand(bf16* p, long n, unsigned seed, float scale) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    unsigned x = (unsigned)i * 2654435761u ^ seed * 0x9E3779B9u;
    x ^= x >> 16; x *= 0x7feb352d; x ^= x >> 15; x *= 0x846ca68b; x ^= x >> 16;
    p[i] = (bf16)(((x & 0xFFFFFF) / 16777216.0f * 2.f - 1.f) * scale);
  }
}
static __global__ void fill_rand_f(float* p, long n, unsigned seed, float scale) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    unsigned x = (unsigned)i * 2246822519u ^ seed * 0x85EBCA6Bu;
    x ^= x >> 16; x *= 0x7feb352d; x ^= x >> 15; x *= 0x846ca68b; x ^= x >> 16;
    p[i] = ((x & 0xFFFFFF) / 16777216.0f * 2.f - 1.f) * scale;
  }
}

struct Bufs {
  bf16 *A, *W, *Ch, *Ch2;
  float *C, *C0, *C2, *bias, *byp, *orig, *rowvec;
};


static GemmParams make_params(int mode, int M, int N, int K, long Kp, long Np, const Bufs& b, bool second) {
  GemmParams p{};
  p.M = M; p.N = N; p.K = K; p.nz2 = 1; p.Brows = (int)Np;
  p.Ah = b.A; p.lda = Kp; p.Bh = b.W; p.ldb = Kp;
  p.bias = b.bias; p.rows_per_group = 1; p.rpb = 1;
  bf16* ch = second ? b.Ch2 : b.Ch;
  float* c = second ? b.C2 : b.C;
  p.Ch = ch; p.ldch = N;
  if (mode == 3) { p.act = 1; return p; }
  p.resid = c; p.ldc = N;
  if (mode != 5) p.C = c;
  if (mode == 2) { p.orig = b.orig; p.byp = b.byp; }
  if (mode == 4 || mode == 5) { p.rowvec = b.rowvec; p.rowvec_ld = N; p.rows_per_group = 1219; }
  return p;
}

template <int ROLE>
static void arm(int a, const GemmParams& p, hipStream_t s) {
  switch (a) {
    case 0: launch_gemm<128, 128, 2, 2, 1, EPI_STD, 2, 2, GEMM_BK, 0, 0, 0, ROLE>(p, 1, s, "lab", true, -1); break;
    case 1: launch_gemm<64, 128, 2, 2, 1, EPI_STD, 2, 3, GEMM_BK, 0, 0, 0, ROLE>(p, 1, s, "lab", true, -1); break;
    case 2: launch_gemm<128, 64, 2, 2, 1, EPI_STD, 2, 3, GEMM_BK, 0, 0, 0, ROLE>(p, 1, s, "lab", true, -1); break;
    case 3: launch_gemm<64, 128, 2, 2, 1, EPI_STD, 3, 2, GEMM_BK, 0, 0, 0, ROLE>(p, 1, s, "lab", true, -1); break;
    case 4: launch_gemm<64, 64, 2, 2, 1, EPI_STD, 4, 2, GEMM_BK, 0, 0, 0, ROLE>(p, 1, s, "lab", true, -1); break;
  }
}
static void run(int mode, int a, const GemmParams& p, hipStream_t s) {
  if (mode == 1) arm<1>(a, p, s);
  else if (mode == 2) arm<2>(a, p, s);
  else if (mode == 3) arm<3>(a, p, s);
  else if (mode == 4) arm<4>(a, p, s);
  else arm<5>(a, p, s);
}

static bool same_bits(const void* a, const void* b, size_t n, size_t* first) {
  std::vector<unsigned char> x(n), y(n);
  ZV_CHECK(hipMemcpy(x.data(), a, n, hipMemcpyDeviceToHost));
  ZV_CHECK(hipMemcpy(y.data(), b, n, hipMemcpyDeviceToHost));
  for (size_t i = 0; i < n; ++i)
    if (x[i] != y[i]) { *first = i; return false; }
  return true;
}

int main(int argc, char** argv) {
  int rounds = argc > 1 ? atoi(argv[1]) : 5;
  std::vector<int> modes = {1, 4, 5};
  if (argc > 2) {
    modes.clear();
    for (char* t = strtok(argv[2], ","); t; t = strtok(nullptr, ",")) modes.push_back(atoi(t));
  }
  std::vector<std::array<int, 3>> shapes = {{26005, 512, 512}, {26005, 512, 560}, {13003, 512, 560},
                                            {6502, 512, 560}, {78016, 512, 560}};
  if (argc > 3) {
    shapes.clear();
    for (char* t = strtok(argv[3], ";"); t; t = strtok(nullptr, ";")) {
      int m, n, k;
      if (sscanf(t, "%dx%dx%d", &m, &n, &k) == 3) shapes.push_back({m, n, k});
    }
  }
  hipStream_t s;
  ZV_CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipEvent_t e0, e1;
  ZV_CHECK(hipEventCreate(&e0));
  ZV_CHECK(hipEventCreate(&e1));
  constexpr int arms = 5;
  const char* names[arms] = {"128x128o2", "64x128o3", "128x64o3", "64x128s3", "64x64s4"};
  for (auto& sh : shapes) {
    const int M = sh[0], N = sh[1], K = sh[2];
    const long Kp = round_up(K, 64), Np = round_up(N, 256);
    Bufs b{};
    ZV_CHECK(hipMalloc(&b.A, (size_t)M * Kp * 2));
    ZV_CHECK(hipMalloc(&b.W, (size_t)Np * Kp * 2));
    ZV_CHECK(hipMalloc(&b.Ch, (size_t)M * N * 2));
    ZV_CHECK(hipMalloc(&b.Ch2, (size_t)M * N * 2));
    ZV_CHECK(hipMalloc(&b.C, (size_t)M * N * 4));
    ZV_CHECK(hipMalloc(&b.C0, (size_t)M * N * 4));
    ZV_CHECK(hipMalloc(&b.C2, (size_t)M * N * 4));
    ZV_CHECK(hipMalloc(&b.bias, (size_t)Np * 4));
    ZV_CHECK(hipMalloc(&b.byp, (size_t)Np * 4));
    ZV_CHECK(hipMalloc(&b.orig, (size_t)M * N * 4));
    hipLaunchKernelGGL(fill_rand_f, dim3(64), dim3(256), 0, s, b.byp, Np, 6u, 1.0f);
    hipLaunchKernelGGL(fill_rand_f, dim3(4096), dim3(256), 0, s, b.orig, (long)M * N, 4u, 1.0f);
    ZV_CHECK(hipMalloc(&b.rowvec, (size_t)(M / 1219 + 1) * N * 4));
    const float ws = 1.0f / sqrtf((float)K);
    hipLaunchKernelGGL(fill_rand, dim3(4096), dim3(256), 0, s, b.A, (long)M * Kp, 1u, 1.0f);
    hipLaunchKernelGGL(fill_rand, dim3(4096), dim3(256), 0, s, b.W, Np * Kp, 2u, ws);
    hipLaunchKernelGGL(fill_rand_f, dim3(4096), dim3(256), 0, s, b.C0, (long)M * N, 3u, 1.0f);
    hipLaunchKernelGGL(fill_rand_f, dim3(64), dim3(256), 0, s, b.bias, Np, 5u, 0.5f);
    hipLaunchKernelGGL(fill_rand_f, dim3(64), dim3(256), 0, s, b.rowvec, (long)(M / 1219 + 1) * N, 7u, 0.5f);
    ZV_CHECK(hipStreamSynchronize(s));
    for (int mode : modes) {
      std::string okstr;
      ZV_CHECK(hipMemcpyAsync(b.C, b.C0, (size_t)M * N * 4, hipMemcpyDeviceToDevice, s));
      ZV_CHECK(hipMemsetAsync(b.Ch, 0, (size_t)M * N * 2, s));
      run(mode, 0, make_params(mode, M, N, K, Kp, Np, b, false), s);
      for (int a = 1; a < arms; ++a) {
        ZV_CHECK(hipMemcpyAsync(b.C2, b.C0, (size_t)M * N * 4, hipMemcpyDeviceToDevice, s));
        ZV_CHECK(hipMemsetAsync(b.Ch2, 0, (size_t)M * N * 2, s));
        run(mode, a, make_params(mode, M, N, K, Kp, Np, b, true), s);
        ZV_CHECK(hipStreamSynchronize(s));
        size_t first = 0;
        bool ok = same_bits(b.Ch, b.Ch2, (size_t)M * N * 2, &first);
        if (ok && mode != 5 && mode != 3) ok = same_bits(b.C, b.C2, (size_t)M * N * 4, &first);
        okstr += ok ? "=" : "D";
      }
      std::vector<std::vector<float>> t(arms);
      for (int r = 0; r < rounds; ++r) {
        for (int a = 0; a < arms; ++a) {
          GemmParams p = make_params(mode, M, N, K, Kp, Np, b, a > 0);
          run(mode, a, p, s);
          ZV_CHECK(hipEventRecord(e0, s));
          for (int i = 0; i < 10; ++i) run(mode, a, p, s);
          ZV_CHECK(hipEventRecord(e1, s));
          ZV_CHECK(hipEventSynchronize(e1));
          float ms;
          ZV_CHECK(hipEventElapsedTime(&ms, e0, e1));
          t[a].push_back(ms / 10);
        }
      }
      // algorithmic bytes: A (bf16) + resid read + fp32 write (not mode 5) + bf16 copy
      const double by = (double)M * K * 2 + (double)M * N * (mode == 3 ? 2 : 4 + (mode == 5 ? 0 : 4) + 2 + (mode == 2 ? 4 : 0));
      printf("M=%d N=%d K=%d mode=%d bits[%s]", M, N, K, mode, okstr.c_str());
      for (int a = 0; a < arms; ++a) {
        std::vector<float> v = t[a];
        std::sort(v.begin(), v.end());
        const double us = v[v.size() / 2] * 1e3;
        printf("  %s %.1fus %.2fTB/s", names[a], us, by / (us * 1e-6) / 1e12);
      }
      printf("\n");
      fflush(stdout);
    }
    hipFree(b.A); hipFree(b.W); hipFree(b.Ch); hipFree(b.Ch2); hipFree(b.C); hipFree(b.C0); hipFree(b.C2);
    hipFree(b.bias); hipFree(b.rowvec); hipFree(b.byp); hipFree(b.orig);
  }
  return 0;
}
