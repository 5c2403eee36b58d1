// Probe of the block-scaled fp8 MFMA (v_mfma_scale_f32_16x16x128_f8f6f4) operand map on
// gfx950.  Data: lane l (row l&15, c = l>>4) holds the 16-B chunks c and c + 4 of its 128-B
// K row (bytes 0-15: K 16c .. 16c+15, bytes 16-31: K 64+16c ..), the same chunks as the
// bf16 16x16x32 map over two K steps.  Scales: lane l supplies the E8M0 scale of K block c
// = K [32c, 32c+32) of row l&15 (not of the bytes it holds).  Compares the MFMA against a
// host fp64 sum over random e4m3 bytes and random scales.  (A first hypothesis, lane l
// holding K [32c, 32c+32) itself, measured max rel. error 1.2e2: tools/probe/mx8_probe2.hip.)
// build: hipcc --offload-arch=gfx950 -O2 tools/probe/mx8_probe.hip -o tools/probe/mx8_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <cstdint>
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
  for (int i = 0; i < 4; ++i) C[(c * 4 + i) * 16 + r] = acc[i];   // row (l>>4)*4+i, col l&15
}

static double e4m3(uint8_t v) {
  const int s = v >> 7, e = (v >> 3) & 15, m = v & 7;
  if (e == 15 && m == 7) return NAN;
  const double x = e ? std::ldexp(1.0 + m / 8.0, e - 7) : std::ldexp(m / 8.0, -6);
  return s ? -x : x;
}

int main() {
  uint8_t hA[16 * 128], hB[16 * 128], hsa[64], hsb[64];
  srand(1);
  for (int i = 0; i < 16 * 128; ++i) {
    uint8_t v;
    do v = rand() & 255; while (((v >> 3) & 15) == 15 && (v & 7) == 7);
    hA[i] = v;
    do v = rand() & 255; while (((v >> 3) & 15) == 15 && (v & 7) == 7);
    hB[i] = v;
  }
  for (int i = 0; i < 64; ++i) { hsa[i] = 120 + rand() % 15; hsb[i] = 120 + rand() % 15; }
  uint8_t *dA, *dB, *dsa, *dsb; float* dC;
  hipMalloc(&dA, sizeof hA); hipMalloc(&dB, sizeof hB); hipMalloc(&dsa, 64); hipMalloc(&dsb, 64);
  hipMalloc(&dC, 256 * 4);
  hipMemcpy(dA, hA, sizeof hA, hipMemcpyHostToDevice); hipMemcpy(dB, hB, sizeof hB, hipMemcpyHostToDevice);
  hipMemcpy(dsa, hsa, 64, hipMemcpyHostToDevice); hipMemcpy(dsb, hsb, 64, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, dA, dB, dsa, dsb, dC);
  float hC[256];
  hipMemcpy(hC, dC, sizeof hC, hipMemcpyDeviceToHost);
  double maxrel = 0;
  for (int i = 0; i < 16; ++i)
    for (int j = 0; j < 16; ++j) {
      double ref = 0, mag = 0;
      for (int k = 0; k < 128; ++k) {
        const double p = e4m3(hA[i * 128 + k]) * std::ldexp(1.0, hsa[i * 4 + k / 32] - 127) *
                         e4m3(hB[j * 128 + k]) * std::ldexp(1.0, hsb[j * 4 + k / 32] - 127);
        ref += p; mag += std::fabs(p);
      }
      maxrel = std::fmax(maxrel, std::fabs(hC[i * 16 + j] - ref) / (mag + 1e-30));
    }
  // the instruction's internal sum of the 128 scaled products is not exact: measured 1.2e-4
  // of sum |a*b| here (scales spread over 2^14); a wrong lane map gives O(1) - O(100)
  printf("mx8 probe: max |mfma - ref| / sum|a*b| = %.3e (%s)\n", maxrel, maxrel < 5e-4 ? "PASS" : "FAIL");
  return maxrel < 5e-4 ? 0 : 1;
}
