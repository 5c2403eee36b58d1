// FFN lab: the fused FeedForward kernel (zv_ffn.inc) against the unfused pair the engine runs
// (in_proj on the 256x256 kernel with the SwooshL epilogue -> 16-bit hidden in HBM -> out_proj
// on the 128x128 kernel with the counted residual epilogue), random operands, same process,
// interleaved rounds.  The two differ only in the out-projection's K summation order (and so in
// the hidden tile's rounding where that flips), so the check is relative, not bitwise.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I zipvoice_amd/csrc tools/lab/ffn_lab.hip -o tools/lab/ffn_lab
//   ffn_lab [rounds] [mode,...] [MxH;...]      modes: 1 residual, 2 + bypass original, 4 + row vector
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#include <array>
#include <algorithm>
#include <cmath>

#include "zv_gemm256.inc"
#include "zv_ffn.inc"

ZvProfiler g_zv_prof;

static __global__ void fill_rand(bf16* p, long n, unsigned seed, float scale) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    unsigned x = (unsigned)i * 2654435761u ^ seed * 0x9E3779B9u;
    x ^= x >> 16; x *= 0x7feb352d; x ^= x >> 15; x *= 0x846ca68b; x ^= x >> 16;
    p[i] = (bf16)(((x & 0xFFFFFF) / 16777216.0f * 2.f - 1.f) * scale);
  }
}
static __global__ void fill_rand_f(float* p, long n, unsigned seed, float scale, float off) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    unsigned x = (unsigned)i * 2246822519u ^ seed * 0x85EBCA6Bu;
    x ^= x >> 16; x *= 0x7feb352d; x ^= x >> 15; x *= 0x846ca68b; x ^= x >> 16;
    p[i] = ((x & 0xFFFFFF) / 16777216.0f * 2.f - 1.f) * scale + off;
  }
}
static __global__ void diff_kernel(const float* a, const float* b, long n, float* out) {
  float mx = 0.f, sm = 0.f, ref = 0.f;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const float d = fabsf(a[i] - b[i]);
    mx = fmaxf(mx, d); sm += d; ref += fabsf(b[i]);
  }
  atomicMax((int*)&out[0], __float_as_int(mx));
  atomicAdd(&out[1], sm);
  atomicAdd(&out[2], ref);
}

int main(int argc, char** argv) {
  int rounds = argc > 1 ? atoi(argv[1]) : 5;
  std::vector<int> modes = {1, 2, 4};
  if (argc > 2) {
    modes.clear();
    for (char* t = strtok(argv[2], ","); t; t = strtok(nullptr, ",")) modes.push_back(atoi(t));
  }
  std::vector<std::array<int, 2>> shapes = {{78016, 1152}, {78016, 1536}, {78016, 1920}, {26005, 1536}, {39008, 1536}};
  if (argc > 3) {
    shapes.clear();
    for (char* t = strtok(argv[3], ";"); t; t = strtok(nullptr, ";")) {
      int m, h;
      if (sscanf(t, "%dx%d", &m, &h) == 2) shapes.push_back({m, h});
    }
  }
  hipStream_t s;
  ZV_CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipEvent_t e0, e1;
  ZV_CHECK(hipEventCreate(&e0));
  ZV_CHECK(hipEventCreate(&e1));
  const int D = FFN_D;
  for (auto& sh : shapes) {
    const int M = sh[0], H = sh[1];
    const long Hp = round_up(H, 256);
    bf16 *X, *W1, *W2, *hid, *Ch, *Ch2, *W1f, *W2f;
    float *C0, *C, *C2, *b1, *b2, *orig, *byp, *rowvec, *dd;
    ZV_CHECK(hipMalloc(&X, (size_t)M * D * 2));
    ZV_CHECK(hipMalloc(&W1, (size_t)Hp * D * 2));
    ZV_CHECK(hipMalloc(&W2, (size_t)D * Hp * 2));
    ZV_CHECK(hipMalloc(&W1f, (size_t)H * D * 2));
    ZV_CHECK(hipMalloc(&W2f, (size_t)H * D * 2));
    ZV_CHECK(hipMalloc(&hid, (size_t)M * H * 2));
    ZV_CHECK(hipMalloc(&Ch, (size_t)M * D * 2));
    ZV_CHECK(hipMalloc(&Ch2, (size_t)M * D * 2));
    ZV_CHECK(hipMalloc(&C0, (size_t)M * D * 4));
    ZV_CHECK(hipMalloc(&C, (size_t)M * D * 4));
    ZV_CHECK(hipMalloc(&C2, (size_t)M * D * 4));
    ZV_CHECK(hipMalloc(&orig, (size_t)M * D * 4));
    ZV_CHECK(hipMalloc(&b1, (size_t)Hp * 4));
    ZV_CHECK(hipMalloc(&b2, (size_t)D * 4));
    ZV_CHECK(hipMalloc(&byp, (size_t)D * 4));
    ZV_CHECK(hipMalloc(&rowvec, (size_t)(M / 1219 + 1) * D * 4));
    ZV_CHECK(hipMalloc(&dd, 16));
    hipLaunchKernelGGL(fill_rand, dim3(4096), dim3(256), 0, s, X, (long)M * D, 1u, 1.0f);
    hipLaunchKernelGGL(fill_rand, dim3(4096), dim3(256), 0, s, W1, Hp * D, 2u, 1.0f / sqrtf((float)D));
    hipLaunchKernelGGL(fill_rand, dim3(4096), dim3(256), 0, s, W2, (long)D * Hp, 3u, 1.0f / sqrtf((float)H));
    hipLaunchKernelGGL(fill_rand_f, dim3(4096), dim3(256), 0, s, C0, (long)M * D, 4u, 1.0f, 0.f);
    hipLaunchKernelGGL(fill_rand_f, dim3(4096), dim3(256), 0, s, orig, (long)M * D, 5u, 1.0f, 0.f);
    hipLaunchKernelGGL(fill_rand_f, dim3(64), dim3(256), 0, s, b1, Hp, 6u, 1.0f, 0.f);
    hipLaunchKernelGGL(fill_rand_f, dim3(64), dim3(256), 0, s, b2, (long)D, 7u, 0.5f, 0.f);
    hipLaunchKernelGGL(fill_rand_f, dim3(64), dim3(256), 0, s, byp, (long)D, 8u, 0.4f, 0.5f);
    hipLaunchKernelGGL(fill_rand_f, dim3(64), dim3(256), 0, s, rowvec, (long)(M / 1219 + 1) * D, 9u, 0.5f, 0.f);
    hipLaunchKernelGGL(zv_ffn_pack_w1_kernel, dim3(cdiv((long)H * D, 256)), dim3(256), 0, s, W1, (long)D, H, W1f);
    hipLaunchKernelGGL(zv_ffn_pack_w2_kernel, dim3(cdiv((long)H * D, 256)), dim3(256), 0, s, W2, Hp, H, W2f);
    ZV_CHECK(hipStreamSynchronize(s));
    for (int mode : modes) {
      GemmParams g1{};
      g1.M = M; g1.N = H; g1.K = D; g1.nz2 = 1; g1.Brows = (int)Hp;
      g1.Ah = X; g1.lda = D; g1.Bh = W1; g1.ldb = D; g1.bias = b1; g1.act = 1;
      g1.Ch = hid; g1.ldch = H; g1.rows_per_group = 1; g1.rpb = 1;
      GemmParams g2{};
      g2.M = M; g2.N = D; g2.K = H; g2.nz2 = 1; g2.Brows = D;
      g2.Ah = hid; g2.lda = H; g2.Bh = W2; g2.ldb = Hp; g2.bias = b2;
      g2.C = C; g2.resid = C; g2.ldc = D; g2.Ch = Ch; g2.ldch = D; g2.rows_per_group = 1; g2.rpb = 1;
      FfnParams f{};
      f.M = M; f.H = H; f.X = X; f.ldx = D; f.W1f = W1f; f.b1 = b1; f.W2f = W2f; f.b2 = b2;
      f.resid = C2; f.C = C2; f.ldc = D; f.Ch = Ch2; f.ldch = D; f.rows_per_group = 1;
      if (mode == 2) { g2.orig = orig; g2.byp = byp; f.orig = orig; f.byp = byp; }
      if (mode == 4) { g2.rowvec = rowvec; g2.rowvec_ld = D; g2.rows_per_group = 1219;
                       f.rowvec = rowvec; f.rowvec_ld = D; f.rows_per_group = 1219; }
      auto unfused = [&]() {
        launch_gemm256<EPI_STD, 3>(g1, s, "lab", false);
        if (mode == 1) launch_gemm<128, 128, 2, 2, 1, EPI_STD, 2, 2, GEMM_BK, 0, 0, 0, 1>(g2, 1, s, "lab", true, -1);
        else if (mode == 2) launch_gemm<128, 128, 2, 2, 1, EPI_STD, 2, 2, GEMM_BK, 0, 0, 0, 2>(g2, 1, s, "lab", true, -1);
        else launch_gemm<128, 128, 2, 2, 1, EPI_STD, 2, 2, GEMM_BK, 0, 0, 0, 4>(g2, 1, s, "lab", true, -1);
      };
      auto fused = [&]() { launch_ffn(f, s, "lab"); };
      auto abl = [&](int a) {
        if (a == 1) launch_ffn<1>(f, s, "lab");
        else if (a == 2) launch_ffn<2>(f, s, "lab");
        else launch_ffn<3>(f, s, "lab");
      };
      // correctness from the same residual start
      ZV_CHECK(hipMemcpyAsync(C, C0, (size_t)M * D * 4, hipMemcpyDeviceToDevice, s));
      ZV_CHECK(hipMemcpyAsync(C2, C0, (size_t)M * D * 4, hipMemcpyDeviceToDevice, s));
      unfused();
      fused();
      // the module output alone: (C - C0) for residual modes; compare C and C2 relative to |C - C0|
      ZV_CHECK(hipMemsetAsync(dd, 0, 16, s));
      hipLaunchKernelGGL(diff_kernel, dim3(1024), dim3(256), 0, s, C2, C, (long)M * D, dd);
      float h[4];
      ZV_CHECK(hipMemcpyAsync(h, dd, 16, hipMemcpyDeviceToHost, s));
      ZV_CHECK(hipStreamSynchronize(s));
      // timing: interleaved rounds, 10 launches per arm per round
      const int arms = mode == 1 ? 5 : 2;     // mode 1: + the ablations (no DMA, no MFMA, no epilogue)
      std::vector<float> t[5];
      for (int r = 0; r < rounds; ++r) {
        for (int a = 0; a < arms; ++a) {
          auto go = [&]() { if (a == 0) unfused(); else if (a == 1) fused(); else abl(a - 1); };
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
      const double fl = 4.0 * M * D * (double)H;
      const double bytes_f = (double)M * D * (2 + 8 + 2 + (mode == 2 ? 4 : 0));
      printf("M=%d H=%d mode=%d  |fused-unfused| max %.3e mean %.3e (mean |C| %.3e)", M, H, mode, h[0],
             h[1] / ((double)M * D), h[2] / ((double)M * D));
      const char* names[5] = {"unfused", "fused", "noDMA", "noMFMA", "noEpi"};
      for (int a = 0; a < arms; ++a) {
        std::vector<float> v = t[a];
        std::sort(v.begin(), v.end());
        const double ms = v[v.size() / 2];
        printf("  %s %.1fus %.0fTF", names[a], ms * 1e3, fl / (ms * 1e-3) / 1e12);
        if (a == 1) printf(" (%.2f TB/s stream)", bytes_f / (ms * 1e-3) / 1e12);
      }
      printf("\n");
      fflush(stdout);
    }
    hipFree(X); hipFree(W1); hipFree(W2); hipFree(W1f); hipFree(W2f); hipFree(hid); hipFree(Ch);
    hipFree(Ch2); hipFree(C0); hipFree(C); hipFree(C2); hipFree(orig); hipFree(b1); hipFree(b2);
    hipFree(byp); hipFree(rowvec); hipFree(dd);
  }
  return 0;
}
