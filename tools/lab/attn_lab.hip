// Attention lab: the fused attention consumers of zv_flash.inc on the model's shapes, random
// operands, one launch per (kernel, shape) timed alone with HIP events:
//   stats  zv_attn_stats_kernel<1, 1>      head-0 row max / sum (Toeplitz scoring)
//   na     zv_attn_na_kernel<1, 3, 8, 1>   NonlinAttention (384 value channels)
//   sa     zv_attn_sa_tp_kernel<0>         SelfAttention (4 heads x 12)
// plus the variant arms under test (each compared with its baseline: max / mean |delta|).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I zipvoice_amd/csrc tools/lab/attn_lab.hip -o tools/lab/attn_lab
//   attn_lab [rounds] [BxL;...] [arms]
// Work units: a "pair" is one (query, key) of one head; SA counts 4 heads, NA / stats head 0.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#include <array>
#include <string>
#include <cmath>

#include "zv_flash.inc"
#ifdef ATTN_LAB_V2
#include "zv_flash2.inc"
#endif

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
// copy of the [q | k | p] operand with the k and p columns scaled by log2(e) (the base-2
// score form: what folding log2(e) into the projection weights produces, rounded once)
static __global__ void scale_kp(const bf16* a, bf16* o, long rows, int ld, int c0, int c1) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < rows * ld; i += (long)gridDim.x * blockDim.x) {
    const int c = (int)(i % ld);
    const float v = (float)a[i];
    o[i] = (c >= c0 && c < c1) ? (bf16)(v * 1.4426950408889634f) : a[i];
  }
}
// V^T with 16 rows per head: rows h*16 + d = src rows h*12 + d (d < 12), row 12 ones, 13-15 zero
// (what the engine's padded value projection writes)
static __global__ void pad_heads(const bf16* src, bf16* dst, int B, int H, int Lpad) {
  const long n = (long)B * H * 16 * Lpad;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const int col = (int)(i % Lpad);
    const long r = i / Lpad;
    const int d = (int)(r % 16), h = (int)(r / 16 % H), b = (int)(r / 16 / H);
    dst[i] = d < 12 ? src[((long)b * H * 12 + h * 12 + d) * Lpad + col] : (bf16)(d == 12 ? 1.f : 0.f);
  }
}
// max |a - b|, sum |a - b|, sum |b| over the valid entries of (rows, ld) 16-bit outputs (cols < nc)
static __global__ void diff16(const bf16* a, const bf16* b, long rows, int ld, int nc, float* out) {
  float mx = 0.f, sm = 0.f, ref = 0.f;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < rows * ld; i += (long)gridDim.x * blockDim.x) {
    if ((int)(i % ld) >= nc) continue;
    const float x = (float)a[i], y = (float)b[i];
    const float d = fabsf(x - y);
    mx = (d == d) ? fmaxf(mx, d) : INFINITY; sm += d; ref += fabsf(y);
  }
  atomicMax((int*)&out[0], __float_as_int(mx));
  atomicAdd(&out[1], sm);
  atomicAdd(&out[2], ref);
}

struct Bufs {
  int B, L, Lpad;
  bf16 *qkp, *qkp2, *vt_sa, *vt_sa2, *xt, *y, *o_sa, *o_sa2, *o_na, *o_na2;
  float* P;
  float2 *stats, *stats2;
};

int main(int argc, char** argv) {
  const int rounds = argc > 1 ? atoi(argv[1]) : 5;
  std::vector<std::array<int, 2>> shapes = {{21, 1219}, {21, 610}, {21, 305}, {64, 1219}, {64, 610},
                                            {64, 305}, {16, 3376}};
  if (argc > 2 && argv[2][0]) {
    shapes.clear();
    for (char* t = strtok(argv[2], ";"); t; t = strtok(nullptr, ";")) {
      int b, l;
      if (sscanf(t, "%dx%d", &b, &l) == 2) shapes.push_back({b, l});
    }
  }
  const std::string arms = argc > 3 ? argv[3] : "stats,na,sa";
  auto on = [&](const char* a) {
    const std::string s = "," + arms + ",", k = std::string(",") + a + ",";
    return s.find(k) != std::string::npos;
  };
  hipStream_t s;
  ZV_CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipEvent_t e0, e1;
  ZV_CHECK(hipEventCreate(&e0));
  ZV_CHECK(hipEventCreate(&e1));
  float* dd;
  ZV_CHECK(hipMalloc(&dd, 16));
  constexpr int H = 4, QKN = 2 * H * ATT_QD + H * ATT_PD, VD = 12, HV = H * VD, HID = 384;
  for (auto& sh : shapes) {
    Bufs u{};
    u.B = sh[0]; u.L = sh[1]; u.Lpad = (int)round_up(u.L, 64);
    const long M = (long)u.B * u.L;
    ZV_CHECK(hipMalloc(&u.qkp, M * QKN * 2));
    ZV_CHECK(hipMalloc(&u.qkp2, M * QKN * 2));
    ZV_CHECK(hipMalloc(&u.P, (2L * u.L - 1) * H * ATT_PD * 4));
    ZV_CHECK(hipMalloc(&u.stats, M * 8));
    ZV_CHECK(hipMalloc(&u.stats2, M * 8));
    ZV_CHECK(hipMalloc(&u.vt_sa, (long)u.B * HV * u.Lpad * 2));
    ZV_CHECK(hipMalloc(&u.vt_sa2, (long)u.B * H * 16 * u.Lpad * 2));
    ZV_CHECK(hipMalloc(&u.xt, (long)u.B * HID * u.Lpad * 2));
    ZV_CHECK(hipMalloc(&u.y, M * HID * 2));
    for (bf16** b : {&u.o_sa, &u.o_sa2}) ZV_CHECK(hipMalloc(b, M * 64 * 2));
    for (bf16** b : {&u.o_na, &u.o_na2}) ZV_CHECK(hipMalloc(b, M * HID * 2));
    hipLaunchKernelGGL(fill_rand, dim3(2048), dim3(256), 0, s, u.qkp, M * QKN, 1u, 1.0f);
    hipLaunchKernelGGL(fill_rand_f, dim3(256), dim3(256), 0, s, u.P, (2L * u.L - 1) * H * ATT_PD, 2u, 1.5f);
    hipLaunchKernelGGL(fill_rand, dim3(2048), dim3(256), 0, s, u.vt_sa, (long)u.B * HV * u.Lpad, 3u, 1.0f);
    hipLaunchKernelGGL(fill_rand, dim3(2048), dim3(256), 0, s, u.xt, (long)u.B * HID * u.Lpad, 4u, 1.0f);
    hipLaunchKernelGGL(fill_rand, dim3(2048), dim3(256), 0, s, u.y, M * HID, 5u, 1.0f);
    hipLaunchKernelGGL(scale_kp, dim3(2048), dim3(256), 0, s, u.qkp, u.qkp2, M, QKN, H * ATT_QD, QKN);
    hipLaunchKernelGGL(pad_heads, dim3(2048), dim3(256), 0, s, u.vt_sa, u.vt_sa2, u.B, H, u.Lpad);
    ZV_CHECK(hipStreamSynchronize(s));

    FlashParams fp{};
    fp.qh = u.qkp; fp.ldq = QKN; fp.P = u.P; fp.key_pad = nullptr; fp.stats = u.stats;
    fp.B = u.B; fp.L = u.L; fp.H = H;
    FlashParams fs = fp;   // SelfAttention
    fs.vh = u.vt_sa; fs.ldv = u.Lpad; fs.sv_b = (long)HV * u.Lpad; fs.vrows_per_head = VD; fs.nv = VD;
    fs.oh = u.o_sa; fs.ldo = 64; fs.ocol_per_head = VD;
    FlashParams fn = fp;   // NonlinAttention
    fn.vh = u.xt; fn.ldv = u.Lpad; fn.sv_b = (long)HID * u.Lpad; fn.vrows_per_head = 0; fn.nv = HID;
    fn.mulh = u.y; fn.ldmul = HID; fn.oh = u.o_na; fn.ldo = HID; fn.ocol_per_head = 0;

    const double pairs = (double)u.B * u.L * u.L;
    auto timeit = [&](const char* name, double flop_per_pair, auto&& fn_launch) {
      fn_launch();   // warm
      ZV_CHECK(hipStreamSynchronize(s));
      float best = 1e30f, tot = 0.f;
      for (int r = 0; r < rounds; ++r) {
        ZV_CHECK(hipEventRecord(e0, s));
        fn_launch();
        ZV_CHECK(hipEventRecord(e1, s));
        ZV_CHECK(hipEventSynchronize(e1));
        float ms = 0.f;
        ZV_CHECK(hipEventElapsedTime(&ms, e0, e1));
        best = std::min(best, ms); tot += ms;
      }
      const double us = 1e3 * tot / rounds;
      printf("  %-10s %8.2f us (best %8.2f)  %6.1f TF/s  %.3f ns/kpair\n", name, us, 1e3 * best,
             flop_per_pair * pairs / (us * 1e-6) / 1e12, us * 1e3 / (pairs / 1e3));
    };
    auto cmp = [&](const char* what, const bf16* a, const bf16* b, int ld, int nc) {
      ZV_CHECK(hipMemsetAsync(dd, 0, 16, s));
      hipLaunchKernelGGL(diff16, dim3(1024), dim3(256), 0, s, a, b, M, ld, nc, dd);
      float h[4];
      ZV_CHECK(hipMemcpyAsync(h, dd, 16, hipMemcpyDeviceToHost, s));
      ZV_CHECK(hipStreamSynchronize(s));
      printf("  %-10s vs base: max %.3e mean %.3e (mean |base| %.3e)\n", what, h[0], h[1] / (M * nc), h[2] / (M * nc));
    };
    printf("B=%d L=%d\n", u.B, u.L);
    // the baseline chain: stats -> NA, SA
    launch_attn_stats<1, 1>(fp, s);
    launch_attn_na<1, 3, 8, 1>(fn, s);
    launch_attn_sa_tp<0>(fs, s);
    ZV_CHECK(hipStreamSynchronize(s));
    if (on("stats")) timeit("stats", 72.0, [&] { launch_attn_stats<1, 1>(fp, s); });
    if (on("na")) timeit("na", 72.0 + 2.0 * HID, [&] { launch_attn_na<1, 3, 8, 1>(fn, s); });
    if (on("sa")) timeit("sa", H * (72.0 + 2.0 * VD), [&] { launch_attn_sa_tp<0>(fs, s); });
#ifdef ATTN_LAB_V2
    {
      FlashParams f2 = fs;
      f2.qh = u.qkp2; f2.oh = u.o_sa2; f2.vh = u.vt_sa2; f2.sv_b = (long)H * 16 * u.Lpad; f2.vrows_per_head = 16;
      if (on("sa2")) {
        launch_attn_sa2<2>(f2, s);
        ZV_CHECK(hipStreamSynchronize(s));
        cmp("sa2", u.o_sa2, u.o_sa, 64, HV);
        timeit("sa2", H * (72.0 + 2.0 * VD), [&] { launch_attn_sa2<2>(f2, s); });
      }
      if (on("sa2w3")) {
        launch_attn_sa2<2, 3>(f2, s);
        ZV_CHECK(hipStreamSynchronize(s));
        cmp("sa2w3", u.o_sa2, u.o_sa, 64, HV);
        timeit("sa2w3", H * (72.0 + 2.0 * VD), [&] { launch_attn_sa2<2, 3>(f2, s); });
      }
      if (on("sa3")) {
        launch_attn_sa3<2>(f2, s);
        ZV_CHECK(hipStreamSynchronize(s));
        cmp("sa3", u.o_sa2, u.o_sa, 64, HV);
        timeit("sa3", H * (72.0 + 2.0 * VD), [&] { launch_attn_sa3<2>(f2, s); });
        launch_attn_sa3<2, 3>(f2, s);
        ZV_CHECK(hipStreamSynchronize(s));
        cmp("sa3w3", u.o_sa2, u.o_sa, 64, HV);
        timeit("sa3w3", H * (72.0 + 2.0 * VD), [&] { launch_attn_sa3<2, 3>(f2, s); });
        launch_attn_sa3<1, 4>(f2, s);
        ZV_CHECK(hipStreamSynchronize(s));
        cmp("sa3q1", u.o_sa2, u.o_sa, 64, HV);
        timeit("sa3q1", H * (72.0 + 2.0 * VD), [&] { launch_attn_sa3<1, 4>(f2, s); });
      }
      if (on("sa2s")) {   // short sequences: fewer query tiles per wave (more blocks)
        launch_attn_sa2<1, 4>(f2, s);
        ZV_CHECK(hipStreamSynchronize(s));
        cmp("sa2q1", u.o_sa2, u.o_sa, 64, HV);
        timeit("sa2q1", H * (72.0 + 2.0 * VD), [&] { launch_attn_sa2<1, 4>(f2, s); });
        launch_attn_sa3<1, 4>(f2, s);
        ZV_CHECK(hipStreamSynchronize(s));
        cmp("sa3q1", u.o_sa2, u.o_sa, 64, HV);
        timeit("sa3q1", H * (72.0 + 2.0 * VD), [&] { launch_attn_sa3<1, 4>(f2, s); });
      }
      if (on("sa2q")) {   // the register-fed form with more query tiles per wave (long sequences)
        launch_attn_sa2<3, 1>(f2, s);
        ZV_CHECK(hipStreamSynchronize(s));
        cmp("sa2q3", u.o_sa2, u.o_sa, 64, HV);
        timeit("sa2q3", H * (72.0 + 2.0 * VD), [&] { launch_attn_sa2<3, 1>(f2, s); });
        launch_attn_sa2<4, 1>(f2, s);
        ZV_CHECK(hipStreamSynchronize(s));
        cmp("sa2q4", u.o_sa2, u.o_sa, 64, HV);
        timeit("sa2q4", H * (72.0 + 2.0 * VD), [&] { launch_attn_sa2<4, 1>(f2, s); });
        launch_attn_sa3<4, 1>(f2, s);
        ZV_CHECK(hipStreamSynchronize(s));
        cmp("sa3q4w1", u.o_sa2, u.o_sa, 64, HV);
        timeit("sa3q4w1", H * (72.0 + 2.0 * VD), [&] { launch_attn_sa3<4, 1>(f2, s); });
        launch_attn_sa3<3, 1>(f2, s);
        ZV_CHECK(hipStreamSynchronize(s));
        cmp("sa3q3w1", u.o_sa2, u.o_sa, 64, HV);
        timeit("sa3q3w1", H * (72.0 + 2.0 * VD), [&] { launch_attn_sa3<3, 1>(f2, s); });
      }
      if (on("sa3q")) {   // more query tiles per wave (K / V / Toeplitz reads shared by more tiles)
        launch_attn_sa3<3, 2>(f2, s);
        ZV_CHECK(hipStreamSynchronize(s));
        cmp("sa3q3", u.o_sa2, u.o_sa, 64, HV);
        timeit("sa3q3", H * (72.0 + 2.0 * VD), [&] { launch_attn_sa3<3, 2>(f2, s); });
        launch_attn_sa3<4, 1>(f2, s);
        ZV_CHECK(hipStreamSynchronize(s));
        cmp("sa3q4", u.o_sa2, u.o_sa, 64, HV);
        timeit("sa3q4", H * (72.0 + 2.0 * VD), [&] { launch_attn_sa3<4, 1>(f2, s); });
        launch_attn_sa3<4, 2>(f2, s);
        ZV_CHECK(hipStreamSynchronize(s));
        cmp("sa3q4w2", u.o_sa2, u.o_sa, 64, HV);
        timeit("sa3q4w2", H * (72.0 + 2.0 * VD), [&] { launch_attn_sa3<4, 2>(f2, s); });
      }
      if (on("pipe")) {
        launch_attn_sa2<2, 2, 0, 1>(f2, s);
        ZV_CHECK(hipStreamSynchronize(s));
        cmp("sa2pipe", u.o_sa2, u.o_sa, 64, HV);
        timeit("sa2pipe", H * (72.0 + 2.0 * VD), [&] { launch_attn_sa2<2, 2, 0, 1>(f2, s); });
        launch_attn_sa2<1, 3, 0, 1>(f2, s);
        ZV_CHECK(hipStreamSynchronize(s));
        cmp("sa2pq1", u.o_sa2, u.o_sa, 64, HV);
        timeit("sa2pq1", H * (72.0 + 2.0 * VD), [&] { launch_attn_sa2<1, 3, 0, 1>(f2, s); });
        launch_attn_sa2<1, 4, 0, 1>(f2, s);
        ZV_CHECK(hipStreamSynchronize(s));
        cmp("sa2pq1w4", u.o_sa2, u.o_sa, 64, HV);
        timeit("sa2pq1w4", H * (72.0 + 2.0 * VD), [&] { launch_attn_sa2<1, 4, 0, 1>(f2, s); });
      }
      if (on("abl")) {
        timeit("sa2-noexp", H * (72.0 + 2.0 * VD), [&] { launch_attn_sa2<2, 2, 1>(f2, s); });
        timeit("sa2-nopos", H * (72.0 + 2.0 * VD), [&] { launch_attn_sa2<2, 2, 2>(f2, s); });
        timeit("sa2-nopv", H * (72.0 + 2.0 * VD), [&] { launch_attn_sa2<2, 2, 3>(f2, s); });
        timeit("sa2-noKV", H * (72.0 + 2.0 * VD), [&] { launch_attn_sa2<2, 2, 4>(f2, s); });
        timeit("sa2-noV", H * (72.0 + 2.0 * VD), [&] { launch_attn_sa2<2, 2, 5>(f2, s); });
      }
      if (on("sa2w4")) {
        launch_attn_sa2<2, 4>(f2, s);
        ZV_CHECK(hipStreamSynchronize(s));
        cmp("sa2w4", u.o_sa2, u.o_sa, 64, HV);
        timeit("sa2w4", H * (72.0 + 2.0 * VD), [&] { launch_attn_sa2<2, 4>(f2, s); });
      }
      if (on("sa2q1")) {
        launch_attn_sa2<1>(f2, s);
        ZV_CHECK(hipStreamSynchronize(s));
        cmp("sa2q1", u.o_sa2, u.o_sa, 64, HV);
        timeit("sa2q1", H * (72.0 + 2.0 * VD), [&] { launch_attn_sa2<1>(f2, s); });
      }
      FlashParams n2 = fn;
      n2.qh = u.qkp2; n2.oh = u.o_na2;
      if (on("na2")) {
        launch_attn_na2<3>(n2, s);
        ZV_CHECK(hipStreamSynchronize(s));
        cmp("na2", u.o_na2, u.o_na, HID, HID);
        timeit("na2", 72.0 + 2.0 * HID, [&] { launch_attn_na2<3>(n2, s); });
      }
      if (on("na2q")) {   // 4 query tiles per block (8 waves)
        launch_attn_na2<3, 4>(n2, s);
        ZV_CHECK(hipStreamSynchronize(s));
        cmp("na2q4", u.o_na2, u.o_na, HID, HID);
        timeit("na2q4", 72.0 + 2.0 * HID, [&] { launch_attn_na2<3, 4>(n2, s); });
      }
      // the exact (fallback) paths: scores pushed past the no-maximum range (every q scaled by
      // 2^6 -> |scores| ~ 2^7: the range check must fail and the exact path take over)
      if (on("exact")) {
        bf16* q3;
        ZV_CHECK(hipMalloc(&q3, M * QKN * 2));
        hipLaunchKernelGGL(scale_kp, dim3(2048), dim3(256), 0, s, u.qkp2, q3, M, QKN, 0, H * ATT_QD);
        for (int i = 0; i < 5; ++i)
          hipLaunchKernelGGL(scale_kp, dim3(2048), dim3(256), 0, s, q3, q3, M, QKN, 0, H * ATT_QD);
        FlashParams e1 = fp; e1.qh = q3;   // first generation on unscaled = q3 / log2(e) ... compare
        (void)e1;
        FlashParams f3 = f2; f3.qh = q3;
        FlashParams n3 = n2; n3.qh = q3;
        launch_attn_sa2<2>(f3, s);
        launch_attn_na2<3>(n3, s);
        launch_attn_sa3<2>(f3, s);
        ZV_CHECK(hipStreamSynchronize(s));
        printf("  exact paths ran (large scores)\n");
        timeit("sa2-exact", H * (72.0 + 2.0 * VD), [&] { launch_attn_sa2<2>(f3, s); });
        timeit("na2-exact", 72.0 + 2.0 * HID, [&] { launch_attn_na2<3>(n3, s); });
        // exactness: the v3 exact paths against the v2 exact paths on the same (large) scores
        FlashParams f4 = f3; f4.oh = u.o_sa;
        launch_attn_sa3<2>(f4, s);
        launch_attn_sa2<2>(f3, s);
        ZV_CHECK(hipStreamSynchronize(s));
        cmp("sa3x-sa2x", u.o_sa, u.o_sa2, 64, HV);
        timeit("sa3-exact", H * (72.0 + 2.0 * VD), [&] { launch_attn_sa3<2>(f3, s); });
        ZV_CHECK(hipFree(q3));
      }
    }
#endif
    for (void* b : {(void*)u.qkp, (void*)u.qkp2, (void*)u.P, (void*)u.stats, (void*)u.stats2, (void*)u.vt_sa, (void*)u.vt_sa2,
                    (void*)u.xt, (void*)u.y, (void*)u.o_sa, (void*)u.o_sa2, (void*)u.o_na, (void*)u.o_na2})
      ZV_CHECK(hipFree(b));
  }
  return 0;
}
