// Probe of the block-scaled fp8 MFMA's internal sum (v_mfma_scale_f32_16x16x128_f8f6f4): how
// many bits below the largest product does a product keep?  Row r of A holds 1.0 at K 0 and
// 1.5 * 2^-j at K 32 (the second K block's E8M0 scale is 127 - j), B is 1.0 at K 0 and K 32, so
// C[r][*] = 1 + 1.5 * 2^-j exactly in fp32 for j <= 22.  The first j where C differs from that
// gives the alignment width W of the internal adder; the second table sums n equal small
// products (n = 1..96, each 1.5 * 2^-j) under a large one to see whether the losses add up.
// The GEMM test's bound (tests/test_gpu_fp8.py GEMM_RTOL) is derived from W.
// build: hipcc --offload-arch=gfx950 -O2 tools/probe/mx8_align.hip -o tools/probe/mx8_align
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
typedef int v8i __attribute__((ext_vector_type(8)));
typedef float f4 __attribute__((ext_vector_type(4)));

__global__ void probe(const uint8_t* A, const uint8_t* B, const uint8_t* sa, const uint8_t* sb, float* C) {
  const int l = threadIdx.x, r = l & 15, c = l >> 4;
  v8i a, b;
  for (int w = 0; w < 8; ++w) {
    const int off = (w < 4 ? 16 * c : 64 + 16 * c) + 4 * (w & 3);
    a[w] = *reinterpret_cast<const int*>(A + r * 128 + off);
    b[w] = *reinterpret_cast<const int*>(B + r * 128 + off);
  }
  f4 acc = {0, 0, 0, 0};
  acc = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, acc, 0, 0, 0, (int)sa[r * 4 + c], 0,
                                                          (int)sb[r * 4 + c]);
  for (int i = 0; i < 4; ++i) C[(c * 4 + i) * 16 + r] = acc[i];
}

static float run(const uint8_t* hA, const uint8_t* hB, const uint8_t* hsa, const uint8_t* hsb, float* hC) {
  uint8_t *dA, *dB, *dsa, *dsb; float* dC;
  hipMalloc(&dA, 2048); hipMalloc(&dB, 2048); hipMalloc(&dsa, 64); hipMalloc(&dsb, 64); hipMalloc(&dC, 1024);
  hipMemcpy(dA, hA, 2048, hipMemcpyHostToDevice); hipMemcpy(dB, hB, 2048, hipMemcpyHostToDevice);
  hipMemcpy(dsa, hsa, 64, hipMemcpyHostToDevice); hipMemcpy(dsb, hsb, 64, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, dA, dB, dsa, dsb, dC);
  hipMemcpy(hC, dC, 1024, hipMemcpyDeviceToHost);
  hipFree(dA); hipFree(dB); hipFree(dsa); hipFree(dsb); hipFree(dC);
  return 0;
}

static double e4m3(uint8_t v) {
  const int e = (v >> 3) & 15, m = v & 7;
  const double x = e ? std::ldexp(1.0 + m / 8.0, e - 7) : std::ldexp(m / 8.0, -6);
  return (v >> 7) ? -x : x;
}
static uint8_t enc(double x) {           // the e4m3 code of an exactly representable value
  for (int v = 0; v < 256; ++v)
    if (!(((v >> 3) & 15) == 15 && (v & 7) == 7) && e4m3((uint8_t)v) == x) return (uint8_t)v;
  fprintf(stderr, "not representable: %g\n", x);
  exit(2);
}

// Row r of A against row r of B: C[r][r] is element r * 17 (element index = A row * 16 + B row).
// Every case cancels a large pair (+1 - 1) inside K block 0, so the exact result is the sum of
// the small products alone, representable in fp32 at any magnitude.
int main() {
  uint8_t A[2048], B[2048], sa[64], sb[64];
  float C[256];
  // (1) one small product 1.5 * 2^-j in the same K block as +1 and -1, j = a + b with A = 1.5 * 2^-a,
  // B = 2^-b (e4m3 reaches 1.5 * 2^-8 and 2^-9: j <= 17); (2) the same in K block 1 (scale 127 - j)
  for (int same = 1; same >= 0; --same) {
    printf("%s: j, C, exact, C/exact\n", same ? "small product in the large pair's K block"
                                             : "small product in another K block (block scale 2^-j)");
    for (int L = 0; L < 2; ++L) {
      memset(A, 0, sizeof A); memset(B, 0, sizeof B);
      for (int i = 0; i < 64; ++i) sa[i] = sb[i] = 127;
      for (int r = 0; r < 16; ++r) {
        const int j = 16 * L + r;
        A[r * 128 + 0] = enc(1.0); A[r * 128 + 1] = enc(-1.0);
        B[r * 128 + 0] = enc(1.0); B[r * 128 + 1] = enc(1.0);
        if (same) {
          if (j > 17) continue;
          const int a = j < 8 ? j : 8, b = j - a;
          A[r * 128 + 2] = enc(1.5 * std::ldexp(1.0, -a)); B[r * 128 + 2] = enc(std::ldexp(1.0, -b));
        } else {
          A[r * 128 + 32] = enc(1.5); B[r * 128 + 32] = enc(1.0);
          sa[r * 4 + 1] = (uint8_t)(127 - j);
        }
      }
      run(A, B, sa, sb, C);
      for (int r = 0; r < 16; ++r) {
        const int j = 16 * L + r;
        if (same && j > 17) continue;
        const double got = C[r * 16 + r], exp = 1.5 * std::ldexp(1.0, -j);
        printf("  j=%2d  %.6e  %.6e  %.4f\n", j, got, exp, got / exp);
      }
    }
  }
  // (3) n equal small products 1.5 * 2^-j (n = 1..29) beside the cancelling pair, same K block
  printf("n small products 1.5*2^-j beside +1 -1 in one K block: j, n, C/exact\n");
  for (int j : {8, 10, 12, 14, 16, 17}) {
    printf("  j=%2d:", j);
    for (int n : {1, 2, 3, 4, 8, 16, 29}) {
      memset(A, 0, sizeof A); memset(B, 0, sizeof B);
      for (int i = 0; i < 64; ++i) sa[i] = sb[i] = 127;
      const int a = j < 8 ? j : 8, b = j - a;
      for (int r = 0; r < 16; ++r) {
        A[r * 128 + 0] = enc(1.0); A[r * 128 + 1] = enc(-1.0);
        B[r * 128 + 0] = enc(1.0); B[r * 128 + 1] = enc(1.0);
        for (int k = 0; k < n; ++k) { A[r * 128 + 2 + k] = enc(1.5 * std::ldexp(1.0, -a)); B[r * 128 + 2 + k] = enc(std::ldexp(1.0, -b)); }
      }
      run(A, B, sa, sb, C);
      printf("  n=%2d %.4f", n, C[0] / (n * 1.5 * std::ldexp(1.0, -j)));
    }
    printf("\n");
  }
  // (4) the largest product 448 * 448 and a small one 1.5 * 2^-17 in one K block: kept bits
  memset(A, 0, sizeof A); memset(B, 0, sizeof B);
  for (int i = 0; i < 64; ++i) sa[i] = sb[i] = 127;
  for (int r = 0; r < 16; ++r) {
    A[r * 128 + 0] = enc(448.0); A[r * 128 + 1] = enc(-448.0);
    B[r * 128 + 0] = enc(448.0); B[r * 128 + 1] = enc(448.0);
    A[r * 128 + 2] = enc(1.5 * std::ldexp(1.0, -(r < 8 ? r : 8))); B[r * 128 + 2] = enc(std::ldexp(1.0, -(r < 8 ? 0 : r - 8)));
  }
  run(A, B, sa, sb, C);
  printf("beside +-448^2 (2^17.6): j, C/exact\n");
  for (int r = 0; r < 16; ++r) printf("  j=%2d %.4f\n", r, C[r * 16 + r] / (1.5 * std::ldexp(1.0, -r)));
  // (5) the sign of the truncation: a negative small product -1.5 * 2^-j beside +1 - 1
  memset(A, 0, sizeof A); memset(B, 0, sizeof B);
  for (int i = 0; i < 64; ++i) sa[i] = sb[i] = 127;
  for (int r = 0; r < 14; ++r) {     // j <= 17: e4m3 reaches 1.5 * 2^-8 and 2^-9
    const int j = 4 + r, a = j < 8 ? j : 8, b = j - a;
    A[r * 128 + 0] = enc(1.0); A[r * 128 + 1] = enc(-1.0);
    B[r * 128 + 0] = enc(1.0); B[r * 128 + 1] = enc(1.0);
    A[r * 128 + 2] = enc(-1.5 * std::ldexp(1.0, -a)); B[r * 128 + 2] = enc(std::ldexp(1.0, -b));
  }
  run(A, B, sa, sb, C);
  printf("negative small product -1.5*2^-j beside +1 -1: j, C, C/exact\n");
  for (int r = 0; r < 14; ++r) printf("  j=%2d %.6e %.4f\n", 4 + r, C[r * 16 + r], C[r * 16 + r] / (-1.5 * std::ldexp(1.0, -(4 + r))));
  return 0;
}
