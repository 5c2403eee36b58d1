// Probe of the fused FeedForward's chunk-step skeleton (zv_ffn.inc): cycles per 64-MFMA step of
// the slot interleave alone, without the activation, the fragment reads or the epilogue.  One
// block of 4 waves per CU (launch bounds 256, 1; the output tiles in the AGPRs, x in VGPRs as in
// the kernel), 256 blocks, s_memtime around `steps` chunk steps per wave:
//   V0  in-projection chain only (32 dependent MFMAs, VGPR accumulator)
//   V1  out-projection only (16 AGPR tiles, 2 MFMAs each)
//   V2  the step's interleave: in-projection on even slots (VGPR acc), out-projection on odd (AGPR)
//   V3  as V2 with the in-projection accumulator in AGPRs too
//   V4  V2 + the step's 16 weight DMA pieces (1 KiB each, L2-resident source) in 4 bursts of 4
//       (slots 1/17/33/49) + vmcnt(0) + barrier per step, as the kernel
//   V5  V4 with the pieces spread one per 3 slots (slots 0, 3, ..., 45)
//   V6  V2 + vmcnt(0) + barrier per step, no DMA
//   V7  V2 + 2 independent v_fma_f32 per slot (VALU fillers)
//   V8  V2 + 1 ds_read_b128 per slot, read into the consumed fragment's register 4 MFMAs of its
//       kind ahead of use (the kernel's fragment ring)
//   V9  V4 + V8 + the activation's micro-op pattern (per 4 slots: add+fmamk, min+exp, add+log,
//       fmamk+max+fmamk on a dependent chain) + the per-step barrier: the whole chunk step's skeleton
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/probe/ffn_mfma_probe.hip -o tools/probe/ffn_mfma_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <type_traits>
#include <utility>

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

template <int N, typename F, int... I>
__device__ __forceinline__ void sfor_impl(F&& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, typename F>
__device__ __forceinline__ void sfor(F&& f) { sfor_impl<N>(f, std::make_integer_sequence<int, N>{}); }

__device__ __forceinline__ void mma_v(f32x16& acc, const bf16x8& a, const bf16x8& b) {
  asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+v"(acc) : "v"(a), "v"(b));
}
__device__ __forceinline__ void mma_a(f32x16& acc, const bf16x8& a, const bf16x8& b) {
  asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
}
__device__ __forceinline__ void dma1(const void* sbase, unsigned voff, unsigned lds, int off) {
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2 offset:%3"
               :: "s"(lds), "v"(voff), "s"(sbase), "n"(0) : "memory", "m0");
}

template <int V>
__global__ __launch_bounds__(256, 1) void probe(const __bf16* src, const void* w, float* sink, unsigned long long* cyc, int steps) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  bf16x8 xf[32], fa[4], fb[4], hb[2];
#pragma unroll
  for (int s = 0; s < 32; ++s) xf[s] = *reinterpret_cast<const bf16x8*>(src + (s * 64 + lane) * 8);
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    fa[q] = *reinterpret_cast<const bf16x8*>(src + ((32 + q) * 64 + lane) * 8);
    fb[q] = *reinterpret_cast<const bf16x8*>(src + ((36 + q) * 64 + lane) * 8);
  }
  hb[0] = xf[3]; hb[1] = xf[5];
  f32x16 out[16], h{};
#pragma unroll
  for (int j = 0; j < 16; ++j) { out[j] = f32x16{}; asm volatile("" : "+a"(out[j])); }
  if constexpr (V == 3) asm volatile("" : "+a"(h));
  float f0 = lane, f1 = lane + 1, f2 = lane + 2, f3 = lane + 3;
  const unsigned lfr = lane * 16;
  __syncthreads();
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int st = 0; st < steps; ++st) {
    const unsigned ldsb = (unsigned)(uintptr_t)smem + (st & 1) * 65536 + wave * 16384;
    sfor<64>([&](auto K_) {
      constexpr int k = decltype(K_)::value, i = k >> 1;
      float& g0 = f0; float& g1 = f1; float& g2 = f2; float& g3 = f3;   // (captured in every instantiation)
      if constexpr ((k & 1) == 0) {
        if constexpr (V != 1) {
          if constexpr (V == 3) mma_a(h, fa[i & 3], xf[i]);
          else mma_v(h, fa[i & 3], xf[i]);
        }
      } else {
        if constexpr (V != 0) mma_a(out[i >> 1], fb[i & 3], hb[i & 1]);
      }
      if constexpr (V == 8 || V == 9) {
        // after MFMA i of its kind: its fragment register gets the one for MFMA i + 4
        if constexpr ((k & 1) == 0) fa[i & 3] = *reinterpret_cast<const bf16x8*>(smem + 131072 + ((i + 4) & 7) * 1024 + lfr);
        else fb[i & 3] = *reinterpret_cast<const bf16x8*>(smem + 139264 + ((i + 4) & 7) * 1024 + lfr);
      }
      if constexpr (V == 9) {
        constexpr int sub = k & 3;
        if constexpr (sub == 0) asm volatile("v_add_f32 %0, %0, %1\n\tv_fmamk_f32 %1, %0, 0x3fb8aa3b, %2" : "+v"(g0), "+v"(g1) : "v"(g3));
        if constexpr (sub == 1) asm volatile("v_min_f32 %0, 0x42fc0000, %1\n\tv_exp_f32 %0, %0" : "=v"(g2) : "v"(g1));
        if constexpr (sub == 2) asm volatile("v_add_f32 %0, 1.0, %0\n\tv_log_f32 %0, %0" : "+v"(g2));
        if constexpr (sub == 3) asm volatile("v_fmamk_f32 %0, %1, 0xbda3d70a, %2\n\tv_max_f32 %1, %1, %2\n\tv_fmamk_f32 %0, %1, 0x3f317218, %0" : "+v"(g3), "+v"(g2) : "v"(g1));
      }
      if constexpr (V == 4 || V == 9) {
        if constexpr (k == 1 || k == 17 || k == 33 || k == 49) {
          const int b = (k - 1) / 16;
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const char* sb = (const char*)w + ((long)(st & 7) * 65536 + wave * 16384 + (b * 4 + q) * 1024);
            dma1(sb, lfr, ldsb + (b * 4 + q) * 1024, 0);
          }
        }
      }
      if constexpr (V == 5) {
        if constexpr (k % 3 == 0 && k / 3 < 16) {
          constexpr int q = k / 3;
          const char* sb = (const char*)w + ((long)(st & 7) * 65536 + wave * 16384 + q * 1024);
          dma1(sb, lfr, ldsb + q * 1024, 0);
        }
      }
      if constexpr (V == 7) {
        asm volatile("v_fma_f32 %0, %0, %1, %1\n\tv_fma_f32 %2, %2, %3, %3" : "+v"(g0), "+v"(g1), "+v"(g2), "+v"(g3));
      }
    });
    if constexpr (V == 4 || V == 5 || V == 6 || V == 9) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
    }
  }
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_nop 7\n\ts_nop 7\n\ts_nop 3" ::: "memory");
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  float acc = f0 + f1 + f2 + f3;
#pragma unroll
  for (int j = 0; j < 16; ++j) { asm volatile("" : "+a"(out[j])); acc += out[j][lane & 15]; }
  acc += h[lane & 15];
  sink[blockIdx.x * 256 + threadIdx.x] = acc;
  if (lane == 0) cyc[blockIdx.x * 4 + wave] = t1 - t0;
}

template <int V>
static void run(const __bf16* src, const void* w, float* sink, unsigned long long* cyc, int steps, int blocks) {
  hipFuncSetAttribute((const void*)probe<V>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  for (int rep = 0; rep < 3; ++rep) hipLaunchKernelGGL(probe<V>, dim3(blocks), dim3(256), 160 * 1024, 0, src, w, sink, cyc, steps);
  hipDeviceSynchronize();
  unsigned long long* h = (unsigned long long*)malloc(blocks * 4 * 8);
  hipMemcpy(h, cyc, blocks * 4 * 8, hipMemcpyDeviceToHost);
  double s = 0, mx = 0;
  for (int i = 0; i < blocks * 4; ++i) { s += h[i]; mx = h[i] > mx ? h[i] : mx; }
  const int mf = (V == 0 || V == 1) ? 32 : 64;
  printf("V%d  %5.0f clk/step (max %5.0f)  %5.1f clk/MFMA  (%d blocks, %d steps)\n", V, s / (blocks * 4) / steps,
         mx / steps, s / (blocks * 4) / steps / mf, blocks, steps);
  free(h);
}

int main(int argc, char** argv) {
  const int blocks = argc > 1 ? atoi(argv[1]) : 256, steps = argc > 2 ? atoi(argv[2]) : 400;
  __bf16* src; void* w; float* sink; unsigned long long* cyc;
  hipMalloc(&src, 64 * 64 * 16);
  hipMemset(src, 0x3c, 64 * 64 * 16);
  hipMalloc(&w, 8 * 65536);
  hipMemset(w, 0x3c, 8 * 65536);
  hipMalloc(&sink, blocks * 256 * 4);
  hipMalloc(&cyc, blocks * 4 * 8);
  run<0>(src, w, sink, cyc, steps, blocks);
  run<1>(src, w, sink, cyc, steps, blocks);
  run<2>(src, w, sink, cyc, steps, blocks);
  run<3>(src, w, sink, cyc, steps, blocks);
  run<4>(src, w, sink, cyc, steps, blocks);
  run<5>(src, w, sink, cyc, steps, blocks);
  run<6>(src, w, sink, cyc, steps, blocks);
  run<7>(src, w, sink, cyc, steps, blocks);
  run<8>(src, w, sink, cyc, steps, blocks);
  run<9>(src, w, sink, cyc, steps, blocks);
  printf("(constant operands: compare variants; s_memtime counts shader cycles)\n");
  return 0;
}
