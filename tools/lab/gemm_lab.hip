// GEMM lab: the 256x256 phased kernel (zv_gemm256.inc) against the 128x128 kernel
// (zv_gemm.inc) on the model's shapes, random bf16 operands, same process, interleaved
// rounds.  Checks the two kernels' outputs bitwise (same MFMA sequence per accumulator).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I zipvoice_amd/csrc tools/lab/gemm_lab.hip -o tools/lab/gemm_lab
//   gemm_lab [rounds] [mode,...] [MxNxK;...]
// modes: 9 none (mainloop only), 3 bias+SwooshL -> bf16, 1 residual (+bias, fp32 + bf16 copy),
//        2 residual + bypass original, 4 residual + row vector, 6 GLU
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

template <int EPI, int ROLE, int V>
static void run256(const GemmParams& p, hipStream_t s) {
  // V: 0 staged epilogue, 1 direct (swapped operands) + drain, 2 direct without the drain
  // V: 0 staged epilogue, 1 direct persistent, 2 direct one tile per block
  if constexpr (V == 0) launch_gemm256<EPI, ROLE, 0, 0, 0, 0>(p, s, "lab");
  else if constexpr (V == 1) launch_gemm256<EPI, ROLE, 0, 0, 1, 0>(p, s, "lab");
  else launch_gemm256<EPI, ROLE, 0, 0, 1, 0>(p, s, "lab", false);
}

template <int EPI, int ROLE>
static void run128(const GemmParams& p, hipStream_t s) {
  launch_gemm<128, 128, 2, 2, 1, EPI, 2, 2, GEMM_BK, 0, 0, 0, ROLE>(p, 1, s, "lab", true, -1);
}

// mode -> (params, launchers)
static GemmParams make_params(int mode, int M, int N, int K, long Kp, long Np, const Bufs& b, bool second) {
  GemmParams p{};
  p.M = M; p.N = N; p.K = K; p.nz2 = 1; p.Brows = (int)Np;
  p.Ah = b.A; p.lda = Kp; p.Bh = b.W; p.ldb = Kp;
  p.bias = b.bias; p.rows_per_group = 1; p.rpb = 1;
  bf16* ch = second ? b.Ch2 : b.Ch;
  float* c = second ? b.C2 : b.C;
  switch (mode) {
    case 9: break;
    case 3: p.act = 1; p.Ch = ch; p.ldch = N; break;
    case 1: p.C = c; p.resid = c; p.ldc = N; p.Ch = ch; p.ldch = N; break;
    case 2: p.C = c; p.resid = c; p.ldc = N; p.Ch = ch; p.ldch = N; p.orig = b.orig; p.byp = b.byp; break;
    case 4: p.C = c; p.resid = c; p.ldc = N; p.Ch = ch; p.ldch = N; p.rowvec = b.rowvec; p.rowvec_ld = N;
            p.rows_per_group = 1219; break;
    case 6: p.Ch = ch; p.ldch = N / 2; break;   // GLU: N permuted columns -> N/2 channels
  }
  return p;
}

template <int PB>
static void launch_mode(int mode, bool big, const GemmParams& p, hipStream_t s) {   // PB: 256 variant
  if (big) {
    switch (mode) {
      case 9: run256<EPI_STD, 9, PB>(p, s); break;
      case 3: run256<EPI_STD, 3, PB>(p, s); break;
      case 1: run256<EPI_STD, 1, PB>(p, s); break;
      case 2: run256<EPI_STD, 2, PB>(p, s); break;
      case 4: run256<EPI_STD, 4, PB>(p, s); break;
      case 6: run256<EPI_GLU, 3, PB>(p, s); break;
    }
  } else {
    switch (mode) {
      case 9:     // the 128 kernel's general epilogue with no output: nothing stored
        launch_gemm<128, 128, 2, 2, 1, EPI_STD, 2, 2>(p, 1, s, "lab", true, -1);
        break;
      case 3: run128<EPI_STD, 3>(p, s); break;
      case 1: run128<EPI_STD, 1>(p, s); break;
      case 2: run128<EPI_STD, 2>(p, s); break;
      case 4: run128<EPI_STD, 4>(p, s); break;
      case 6: run128<EPI_GLU, 3>(p, s); break;
    }
  }
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
  std::vector<int> modes = {9, 3, 1};
  if (argc > 2) {
    modes.clear();
    for (char* t = strtok(argv[2], ","); t; t = strtok(nullptr, ",")) modes.push_back(atoi(t));
  }
  std::vector<std::array<int, 3>> shapes = {{78016, 512, 1536}, {78016, 1536, 512}, {78016, 1152, 512},
                                            {78016, 1024, 512}, {78016, 512, 512}, {39008, 512, 1536},
                                            {26005, 1536, 512}, {26005, 1024, 512}, {26005, 512, 1536},
                                            {78016, 1920, 512},
                                            {8192, 8192, 8192}};
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
    ZV_CHECK(hipMalloc(&b.orig, (size_t)M * N * 4));
    ZV_CHECK(hipMalloc(&b.bias, (size_t)Np * 4));
    ZV_CHECK(hipMalloc(&b.byp, (size_t)Np * 4));
    ZV_CHECK(hipMalloc(&b.rowvec, (size_t)(M / 1219 + 1) * N * 4));
    const float ws = 1.0f / sqrtf((float)K);
    hipLaunchKernelGGL(fill_rand, dim3(4096), dim3(256), 0, s, b.A, (long)M * Kp, 1u, 1.0f);
    hipLaunchKernelGGL(fill_rand, dim3(4096), dim3(256), 0, s, b.W, Np * Kp, 2u, ws);
    hipLaunchKernelGGL(fill_rand_f, dim3(4096), dim3(256), 0, s, b.C0, (long)M * N, 3u, 1.0f);
    hipLaunchKernelGGL(fill_rand_f, dim3(4096), dim3(256), 0, s, b.orig, (long)M * N, 4u, 1.0f);
    hipLaunchKernelGGL(fill_rand_f, dim3(64), dim3(256), 0, s, b.bias, Np, 5u, 0.5f);
    hipLaunchKernelGGL(fill_rand_f, dim3(64), dim3(256), 0, s, b.byp, Np, 6u, 1.0f);
    hipLaunchKernelGGL(fill_rand_f, dim3(64), dim3(256), 0, s, b.rowvec, (long)(M / 1219 + 1) * N, 7u, 0.5f);
    ZV_CHECK(hipStreamSynchronize(s));
    for (int mode : modes) {
      // correctness: both kernels from the same residual start
      bool ok = true;
      size_t first = 0;
      if (mode != 9) {
        ZV_CHECK(hipMemcpyAsync(b.C, b.C0, (size_t)M * N * 4, hipMemcpyDeviceToDevice, s));
        ZV_CHECK(hipMemcpyAsync(b.C2, b.C0, (size_t)M * N * 4, hipMemcpyDeviceToDevice, s));
        ZV_CHECK(hipMemsetAsync(b.Ch, 0, (size_t)M * N * 2, s));
        ZV_CHECK(hipMemsetAsync(b.Ch2, 0, (size_t)M * N * 2, s));
        launch_mode<0>(mode, false, make_params(mode, M, N, K, Kp, Np, b, false), s);
        for (int v = 0; v < 3 && ok; ++v) {
          ZV_CHECK(hipMemcpyAsync(b.C2, b.C0, (size_t)M * N * 4, hipMemcpyDeviceToDevice, s));
          ZV_CHECK(hipMemsetAsync(b.Ch2, 0, (size_t)M * N * 2, s));
          GemmParams q = make_params(mode, M, N, K, Kp, Np, b, true);
          if (v == 0) launch_mode<0>(mode, true, q, s);
          else if (v == 1) launch_mode<1>(mode, true, q, s);
          else launch_mode<2>(mode, true, q, s);
          ZV_CHECK(hipStreamSynchronize(s));
          const size_t chn = (size_t)M * (mode == 6 ? N / 2 : N) * 2;
          ok = same_bits(b.Ch, b.Ch2, chn, &first);
          if (ok && (mode == 1 || mode == 2 || mode == 4)) ok = same_bits(b.C, b.C2, (size_t)M * N * 4, &first);
          if (!ok) printf("[variant %d] ", v);
        }
      }
      // timing: interleaved rounds, 10 launches per arm per round
      const int arms = 4;
      std::vector<std::vector<float>> t(arms);
      for (int r = 0; r < rounds; ++r) {
        for (int a = 0; a < arms; ++a) {
          GemmParams p = make_params(mode, M, N, K, Kp, Np, b, a > 0);
          auto go = [&]() {
            if (a == 0) launch_mode<0>(mode, false, p, s);
            else if (a == 1) launch_mode<0>(mode, true, p, s);
            else if (a == 2) launch_mode<1>(mode, true, p, s);
            else launch_mode<2>(mode, true, p, s);
          };
          go();
          ZV_CHECK(hipEventRecord(e0, s));
          for (int i = 0; i < 10; ++i) go();
          ZV_CHECK(hipEventRecord(e1, s));
          ZV_CHECK(hipEventSynchronize(e1));
          float ms;
          ZV_CHECK(hipEventElapsedTime(&ms, e0, e1));
          t[a].push_back(ms / 10);
        }
      }
      const double fl = 2.0 * M * N * (double)K;
      printf("M=%d N=%d K=%d mode=%d %s", M, N, K, mode, mode == 9 ? "" : (ok ? "bitwise-equal" : "DIFF"));
      if (!ok) printf("@%zu", first);
      const char* names[arms] = {"k128", "k256stg", "k256dir", "k256dirNP"};
      for (int a = 0; a < arms; ++a) {
        std::vector<float> v = t[a];
        std::sort(v.begin(), v.end());
        printf("  %s %.1fus %.0fTF", names[a], v[v.size() / 2] * 1e3, fl / (v[v.size() / 2] * 1e-3) / 1e12);
      }
      printf("\n");
      fflush(stdout);
    }
    hipFree(b.A); hipFree(b.W); hipFree(b.Ch); hipFree(b.Ch2); hipFree(b.C); hipFree(b.C0); hipFree(b.C2);
    hipFree(b.orig); hipFree(b.bias); hipFree(b.byp); hipFree(b.rowvec);
  }
  return 0;
}
