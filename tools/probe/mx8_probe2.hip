// Diagnostic probe of v_mfma_scale_f32_16x16x128_f8f6f4 (fp8 e4m3 A and B): prints the
// result of structured inputs so the lane maps of data and scales can be read off.
// build: hipcc --offload-arch=gfx950 -O2 tools/probe/mx8_probe2.hip -o tools/probe/mx8_probe2
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstring>
typedef int v8i __attribute__((ext_vector_type(8)));
typedef float f4 __attribute__((ext_vector_type(4)));

// A, B: per-lane register images (64 lanes x 32 bytes), scales per lane (64 bytes)
__global__ void probe(const uint8_t* A, const uint8_t* B, const int* sa, const int* sb, float* C) {
  const int l = threadIdx.x;
  v8i a, b;
  for (int w = 0; w < 8; ++w) {
    a[w] = *reinterpret_cast<const int*>(A + l * 32 + 4 * w);
    b[w] = *reinterpret_cast<const int*>(B + l * 32 + 4 * w);
  }
  f4 acc = {0, 0, 0, 0};
  acc = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, acc, 0, 0, 0, sa[l], 0, sb[l]);
  for (int i = 0; i < 4; ++i) C[((l >> 4) * 4 + i) * 16 + (l & 15)] = acc[i];
}

static uint8_t *dA, *dB; static int *dsa, *dsb; static float* dC;
static void run(const uint8_t* A, const uint8_t* B, const int* sa, const int* sb, float* C) {
  hipMemcpy(dA, A, 2048, hipMemcpyHostToDevice); hipMemcpy(dB, B, 2048, hipMemcpyHostToDevice);
  hipMemcpy(dsa, sa, 256, hipMemcpyHostToDevice); hipMemcpy(dsb, sb, 256, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, dA, dB, dsa, dsb, dC);
  hipMemcpy(C, dC, 1024, hipMemcpyDeviceToHost);
}
static void show(const char* t, const float* C) {
  printf("%s\n", t);
  for (int i = 0; i < 16; ++i) {
    for (int j = 0; j < 16; ++j) printf(" %6g", C[i * 16 + j]);
    printf("\n");
  }
}
int main() {
  (void)hipMalloc(&dA, 2048); (void)hipMalloc(&dB, 2048); (void)hipMalloc(&dsa, 256); (void)hipMalloc(&dsb, 256); (void)hipMalloc(&dC, 1024);
  uint8_t A[2048], B[2048]; int sa[64], sb[64]; float C[256];
  const uint8_t ONE = 0x38;   // e4m3 1.0
  // 1: all ones, unit scales -> expect 128 everywhere
  memset(A, ONE, 2048); memset(B, ONE, 2048);
  for (int i = 0; i < 64; ++i) sa[i] = sb[i] = 127;
  run(A, B, sa, sb, C); show("ones, scales 127", C);
  // 2: A lane L byte j = 1 only for one (L, j); B ones -> which C entries get it
  int probes[][2] = {{0, 0}, {0, 31}, {1, 0}, {16, 0}, {17, 5}, {48, 0}};
  for (auto& pr : probes) {
    memset(A, 0, 2048); A[pr[0] * 32 + pr[1]] = ONE;
    run(A, B, sa, sb, C);
    printf("A lane %d byte %d -> nonzero C at:", pr[0], pr[1]);
    for (int i = 0; i < 256; ++i) if (C[i] != 0) printf(" (%d,%d)=%g", i / 16, i % 16, C[i]);
    printf("\n");
  }
  // 3: scale test: ones data, sa[L] = 128 (x2) for one lane L
  memset(A, ONE, 2048);
  int sl[] = {0, 1, 16, 32, 48};
  for (int L : sl) {
    for (int i = 0; i < 64; ++i) sa[i] = 127;
    sa[L] = 128;
    run(A, B, sa, sb, C);
    printf("sa lane %d = 2 -> C row sums deviating:", L);
    for (int i = 0; i < 256; ++i) if (C[i] != 128) printf(" (%d,%d)=%g", i / 16, i % 16, C[i]);
    printf("\n");
  }
  for (int i = 0; i < 64; ++i) sa[i] = 127;
  // 4: A lane 0 byte 0 = 1 only, B lane L byte j = 1 only: product appears?
  memset(A, 0, 2048); A[0] = ONE;
  for (int L = 0; L < 64; L += 16) {
    memset(B, 0, 2048); B[L * 32 + 0] = ONE;
    run(A, B, sa, sb, C);
    printf("A(l0,b0) B(l%d,b0):", L);
    for (int i = 0; i < 256; ++i) if (C[i] != 0) printf(" (%d,%d)=%g", i / 16, i % 16, C[i]);
    printf("\n");
  }
  return 0;
}
