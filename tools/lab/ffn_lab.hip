// FFN lab: the fused FeedForward kernel (zv_ffn.inc) on the model's shapes, random operands:
//   unfused  the pair the engine runs below the fused threshold (in_proj on the 256x256 kernel with
//            the SwooshL epilogue -> 16-bit hidden in HBM -> out_proj on the 128x128 kernel with
//            the counted residual epilogue): the relative check (K summation order differs);
//   classic  the fused kernel, one row block per block (w = nc);
//   pers     the fused kernel on the persistent line schedule (must equal classic bit for bit);
//   seg3     pers with the rows cut into three ranges with their own buffers (bit for bit);
//   noEpi    pers without the epilogue (ablation).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I zipvoice_amd/csrc tools/lab/ffn_lab.hip -o tools/lab/ffn_lab
//   ffn_lab [rounds] [mode,...] [MxH;...] [blocks] [arms]   modes: 1 residual, 2 + bypass original,
//           4 + row vector, 8 FF3 + BiasNorm epilogue (no unfused arm)
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
// max |a - b|, sum |a - b|, sum |b|, count of bit differences
static __global__ void diff_kernel(const float* a, const float* b, long n, float* out) {
  float mx = 0.f, sm = 0.f, ref = 0.f;
  unsigned nd = 0;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const float d = fabsf(a[i] - b[i]);
    mx = fmaxf(mx, d); sm += d; ref += fabsf(b[i]);
    nd += __float_as_uint(a[i]) != __float_as_uint(b[i]);
  }
  atomicMax((int*)&out[0], __float_as_int(mx));
  atomicAdd(&out[1], sm);
  atomicAdd(&out[2], ref);
  atomicAdd((unsigned*)&out[3], nd);
}
static __global__ void diff16_kernel(const bf16* a, const bf16* b, long n, unsigned* out) {
  unsigned nd = 0;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    nd += (float)a[i] != (float)b[i];
  atomicAdd(out, nd);
}

int main(int argc, char** argv) {
  int rounds = argc > 1 ? atoi(argv[1]) : 5;
  std::vector<int> modes = {1, 2, 4, 8};
  if (argc > 2) {
    modes.clear();
    for (char* t = strtok(argv[2], ","); t; t = strtok(nullptr, ",")) modes.push_back(atoi(t));
  }
  std::vector<std::array<int, 2>> shapes = {{78016, 1152}, {78016, 1536}, {78016, 1920}, {39008, 1536},
                                            {19504, 1536}, {26005, 1536}};
  if (argc > 3) {
    shapes.clear();
    for (char* t = strtok(argv[3], ";"); t; t = strtok(nullptr, ";")) {
      int m, h;
      if (sscanf(t, "%dx%d", &m, &h) == 2) shapes.push_back({m, h});
    }
  }
  const int blocks_max = argc > 4 ? atoi(argv[4]) : 0;
  // arms to time (counter runs time one): a subset of "unfused,classic,pers,seg3,noEpi"
  const char* arm_sel = argc > 5 ? argv[5] : "unfused,classic,pers,seg3,noEpi,noDMA";
  hipStream_t s;
  ZV_CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipEvent_t e0, e1;
  ZV_CHECK(hipEventCreate(&e0));
  ZV_CHECK(hipEventCreate(&e1));
  const int D = FFN_D;
  float* part; unsigned* flag;
  ZV_CHECK(hipMalloc(&part, 512 * FFN_PART_FLOATS * 4));
  ZV_CHECK(hipMalloc(&flag, 4096));
  ZV_CHECK(hipMemset(flag, 0, 4096));
  unsigned long long* dbg;
  ZV_CHECK(hipMalloc(&dbg, 1024 * 4 * FFN_DBG_WORDS * 8));
  for (auto& sh : shapes) {
    const int M = sh[0], H = sh[1];
    const long Hp = round_up(H, 256);
    bf16 *X, *W1, *W2, *hid, *Ch, *Ch2, *Ch3, *W1f, *W2f, *Cl2, *Cl3, *C2h2, *C2h3;
    float *C0, *C, *C2, *C3, *b1, *b2, *orig, *byp, *rowvec, *nb, *dd;
    const size_t MD = (size_t)M * D;
    ZV_CHECK(hipMalloc(&X, MD * 2));
    ZV_CHECK(hipMalloc(&W1, (size_t)Hp * D * 2));
    ZV_CHECK(hipMalloc(&W2, (size_t)D * Hp * 2));
    ZV_CHECK(hipMalloc(&W1f, (size_t)H * D * 2));
    ZV_CHECK(hipMalloc(&W2f, (size_t)H * D * 2));
    ZV_CHECK(hipMalloc(&hid, (size_t)M * H * 2));
    for (bf16** b : {&Ch, &Ch2, &Ch3, &Cl2, &Cl3, &C2h2, &C2h3}) ZV_CHECK(hipMalloc(b, MD * 2));
    for (float** b : {&C0, &C, &C2, &C3, &orig}) ZV_CHECK(hipMalloc(b, MD * 4));
    ZV_CHECK(hipMalloc(&b1, (size_t)Hp * 4));
    ZV_CHECK(hipMalloc(&b2, (size_t)D * 4));
    ZV_CHECK(hipMalloc(&byp, (size_t)D * 4));
    ZV_CHECK(hipMalloc(&nb, (size_t)D * 4));
    ZV_CHECK(hipMalloc(&rowvec, (size_t)(M / 1219 + 1) * D * 4));
    ZV_CHECK(hipMalloc(&dd, 16));
    hipLaunchKernelGGL(fill_rand, dim3(4096), dim3(256), 0, s, X, (long)MD, 1u, 1.0f);
    hipLaunchKernelGGL(fill_rand, dim3(4096), dim3(256), 0, s, W1, Hp * D, 2u, 1.0f / sqrtf((float)D));
    hipLaunchKernelGGL(fill_rand, dim3(4096), dim3(256), 0, s, W2, (long)D * Hp, 3u, 1.0f / sqrtf((float)H));
    hipLaunchKernelGGL(fill_rand_f, dim3(4096), dim3(256), 0, s, C0, (long)MD, 4u, 1.0f, 0.f);
    hipLaunchKernelGGL(fill_rand_f, dim3(4096), dim3(256), 0, s, orig, (long)MD, 5u, 1.0f, 0.f);
    hipLaunchKernelGGL(fill_rand_f, dim3(64), dim3(256), 0, s, b1, Hp, 6u, 1.0f, 0.f);
    hipLaunchKernelGGL(fill_rand_f, dim3(64), dim3(256), 0, s, b2, (long)D, 7u, 0.5f, 0.f);
    hipLaunchKernelGGL(fill_rand_f, dim3(64), dim3(256), 0, s, byp, (long)D, 8u, 0.4f, 0.5f);
    hipLaunchKernelGGL(fill_rand_f, dim3(64), dim3(256), 0, s, nb, (long)D, 10u, 0.1f, 0.f);
    hipLaunchKernelGGL(fill_rand_f, dim3(64), dim3(256), 0, s, rowvec, (long)(M / 1219 + 1) * D, 9u, 0.5f, 0.f);
    hipLaunchKernelGGL(zv_ffn_pack_w1_kernel, dim3(cdiv((long)H * D, 256)), dim3(256), 0, s, W1, (long)D, H, W1f);
    hipLaunchKernelGGL(zv_ffn_pack_w2_kernel, dim3(cdiv((long)H * D, 256)), dim3(256), 0, s, W2, Hp, H, W2f);
    ZV_CHECK(hipStreamSynchronize(s));
    for (int mode : modes) {
      const bool norm = mode == 8;
      GemmParams g1{};
      g1.M = M; g1.N = H; g1.K = D; g1.nz2 = 1; g1.Brows = (int)Hp;
      g1.Ah = X; g1.lda = D; g1.Bh = W1; g1.ldb = D; g1.bias = b1; g1.act = 1;
      g1.Ch = hid; g1.ldch = H; g1.rows_per_group = 1; g1.rpb = 1;
      GemmParams g2{};
      g2.M = M; g2.N = D; g2.K = H; g2.nz2 = 1; g2.Brows = D;
      g2.Ah = hid; g2.lda = H; g2.Bh = W2; g2.ldb = Hp; g2.bias = b2;
      g2.C = C; g2.resid = C; g2.ldc = D; g2.Ch = Ch; g2.ldch = D; g2.rows_per_group = 1; g2.rpb = 1;
      // fused params on output set k (C2 / C3 with their copies), `nseg` ranges, persistent or not
      auto fparams = [&](float* Co, bf16* Cho, bf16* Clo, bf16* C2ho, int nseg, bool pers) {
        FfnParams f{};
        f.H = H; f.nseg = nseg; f.ldx = D; f.ldc = D; f.ldch = D; f.rows_per_group = 1;
        f.W1f = W1f; f.b1 = b1; f.W2f = W2f; f.b2 = b2;
        if (pers) { f.part = part; f.flag = flag; f.part_slots = 512; }
        f.dbg = dbg;
        const int cut[4] = {0, M / 3 + 77, 2 * M / 3 + 5, M};
        for (int i = 0; i < nseg; ++i) {
          const int r0 = nseg == 1 ? 0 : cut[i], r1 = nseg == 1 ? M : cut[i + 1];
          FfnSeg& g = f.seg[i];
          g.M = r1 - r0; g.X = X + (long)r0 * D;
          g.resid = Co + (long)r0 * D; g.C = Co + (long)r0 * D; g.Ch = Cho + (long)r0 * D;
          if (mode == 2) { g.orig = orig + (long)r0 * D; f.byp = byp; }
          // (one row vector for every row: rowvec_ld 0, so every range points at the same one)
          if (mode == 4) { g.rowvec = rowvec; f.rowvec_ld = 0; f.rows_per_group = 1219; }
          if (norm) {
            // FF3 + BiasNorm: resid = the working stream (C0 copy in Co), orig = C (in place)
            g.resid = orig + (long)r0 * D; g.orig = Co + (long)r0 * D; g.C = Co + (long)r0 * D;
            g.C2h = C2ho + (long)r0 * D;   // the engine's 16-bit set: the next layer's copy (no Cl)
            g.rowvec = rowvec; f.rowvec_ld = 0; f.rows_per_group = 1219;
            f.byp = byp; f.nb = nb; f.log_scale = 0.3f;
          }
        }
        return f;
      };
      if (mode == 2) { g2.orig = orig; g2.byp = byp; }
      if (mode == 4) { g2.rowvec = rowvec; g2.rowvec_ld = 0; g2.rows_per_group = 1219; }
      auto unfused = [&]() {
        launch_gemm256<EPI_STD, 3>(g1, s, "lab", false);
        if (mode == 1) launch_gemm<128, 128, 2, 2, 1, EPI_STD, 2, 2, GEMM_BK, 0, 0, 0, 1>(g2, 1, s, "lab", true, -1);
        else if (mode == 2) launch_gemm<128, 128, 2, 2, 1, EPI_STD, 2, 2, GEMM_BK, 0, 0, 0, 2>(g2, 1, s, "lab", true, -1);
        else launch_gemm<128, 128, 2, 2, 1, EPI_STD, 2, 2, GEMM_BK, 0, 0, 0, 4>(g2, 1, s, "lab", true, -1);
      };
      const FfnParams fc = fparams(C2, Ch2, Cl2, C2h2, 1, false);
      const FfnParams fp = fparams(C3, Ch3, Cl3, C2h3, 1, true);
      const FfnParams f3 = fparams(C3, Ch3, Cl3, C2h3, 3, true);
      auto reset = [&](float* Co) { ZV_CHECK(hipMemcpyAsync(Co, C0, MD * 4, hipMemcpyDeviceToDevice, s)); };
      auto cmp = [&](const float* a, const float* b, float (&h)[4]) {
        ZV_CHECK(hipMemsetAsync(dd, 0, 16, s));
        hipLaunchKernelGGL(diff_kernel, dim3(1024), dim3(256), 0, s, a, b, (long)MD, dd);
        ZV_CHECK(hipMemcpyAsync(h, dd, 16, hipMemcpyDeviceToHost, s));
        ZV_CHECK(hipStreamSynchronize(s));
      };
      auto cmp16 = [&](const bf16* a, const bf16* b) {
        ZV_CHECK(hipMemsetAsync(dd, 0, 16, s));
        hipLaunchKernelGGL(diff16_kernel, dim3(1024), dim3(256), 0, s, a, b, (long)MD, (unsigned*)dd);
        unsigned h = 0;
        ZV_CHECK(hipMemcpyAsync(&h, dd, 4, hipMemcpyDeviceToHost, s));
        ZV_CHECK(hipStreamSynchronize(s));
        return h;
      };
      printf("M=%d H=%d mode=%d", M, H, mode);
      // correctness from the same residual start
      float h[4];
      if (!norm) {
        reset(C); reset(C2);
        unfused();
        launch_ffn(fc, s, "lab", blocks_max);
        cmp(C2, C, h);
        printf("  |classic-unfused| max %.3e mean %.3e", h[0], h[1] / (double)MD);
      }
      reset(C2); launch_ffn(fc, s, "lab", blocks_max);
      reset(C3); launch_ffn(fp, s, "lab", blocks_max);
      cmp(C3, C2, h);
      unsigned n16 = cmp16(Ch3, Ch2) + (norm ? cmp16(Cl3, Cl2) + cmp16(C2h3, C2h2) : 0);
      printf("  pers!=classic %u+%u", ((unsigned*)h)[3], n16);
      reset(C3); launch_ffn(f3, s, "lab", blocks_max);
      cmp(C3, C2, h);
      n16 = cmp16(Ch3, Ch2) + (norm ? cmp16(Cl3, Cl2) + cmp16(C2h3, C2h2) : 0);
      // every hand-off flag must be back at zero between launches (a C item that did not reset
      // its flag would let the next launch's C item skip its wait and read stale tiles)
      std::vector<unsigned> hf(1024);
      ZV_CHECK(hipMemcpy(hf.data(), flag, 4096, hipMemcpyDeviceToHost));
      unsigned nflag = 0;
      for (unsigned v : hf) nflag += v != 0;
      printf("  seg3!=classic %u+%u  flags set %u", ((unsigned*)h)[3], n16, nflag);
      const int nc = H / FFN_HC;
      const FfnSchedule sc = ffn_schedule(cdiv(M, FFN_BM), nc, blocks_max > 0 ? blocks_max : zv_num_cus(), true);
      printf("  (R %d nc %d w %d blocks %d)\n", cdiv(M, FFN_BM), nc, sc.w, sc.blocks);
      // timing: interleaved rounds, 10 launches per arm per round (no resets: residual in place)
      const char* names[6] = {"unfused", "classic", "pers", "seg3", "noEpi", "noDMA"};
      std::vector<float> t[6];
      for (int r = 0; r < rounds; ++r) {
        for (int a = norm ? 1 : 0; a < 6; ++a) {
          if (!strstr(arm_sel, names[a])) continue;
          auto go = [&]() {
            if (a == 0) unfused();
            else if (a == 1) launch_ffn(fc, s, "lab", blocks_max);
            else if (a == 2) launch_ffn(fp, s, "lab", blocks_max);
            else if (a == 3) launch_ffn(f3, s, "lab", blocks_max);
            else if (a == 4) launch_ffn<3>(fp, s, "lab", blocks_max);
            else launch_ffn<1>(fp, s, "lab", blocks_max);
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
      const double fl = 4.0 * M * D * (double)H;
      printf("   ");
      for (int a = norm ? 1 : 0; a < 6; ++a) {
        if (t[a].empty()) continue;
        std::vector<float> v = t[a];
        std::sort(v.begin(), v.end());
        const double ms = v[v.size() / 2];
        printf("  %s %.1fus %.0fTF", names[a], ms * 1e3, fl / (ms * 1e-3) / 1e12);
      }
      printf("\n");
#if FFN_TIMING
      // the last launch's per-wave clock totals (FFN_TIMING build): where a chunk step goes
      {
        const int nb = ffn_schedule(cdiv(M, FFN_BM), H / FFN_HC, blocks_max > 0 ? blocks_max : zv_num_cus(), true).blocks;
        const int W = FFN_DBG_WORDS;
        std::vector<unsigned long long> hd((size_t)nb * 4 * W);
        ZV_CHECK(hipMemcpy(hd.data(), dbg, hd.size() * 8, hipMemcpyDeviceToHost));
        double tot = 0, rt = 0, vm = 0, bar = 0, st = 0, epi = 0, xw = 0, it = 0, lp = 0;
        for (int b = 0; b < nb * 4; ++b) {
          const unsigned long long* d = &hd[(size_t)b * W];
          tot += d[0]; rt += d[1]; vm += d[2]; bar += d[3]; st += d[4]; epi += d[6]; xw += d[7]; it += d[8]; lp += d[9];
        }
        const double nw = nb * 4.0;
        printf("    timing (last launch, per wave): %.0f clk total, %.1f us (%.2f GHz), %.0f steps, per step %.0f clk, "
               "vmcnt wait %.0f, barrier %.0f\n", tot / nw, rt / nw / 100.0, tot / rt * 0.1, st / nw, tot / st, vm / st, bar / st);
        printf("      %.1f items: epilogue %.0f clk/item (%.0f%%), item start (x landed) %.0f clk/item (%.0f%%), steady loop %.0f%%, "
               "rest %.0f%%\n", it / nw, epi / it, 100 * epi / tot, xw / it, 100 * xw / tot, 100 * lp / tot,
               100 * (tot - epi - xw - lp) / tot);
      }
#endif
      fflush(stdout);
    }
    for (void* b : std::initializer_list<void*>{X, W1, W2, W1f, W2f, hid, Ch, Ch2, Ch3, Cl2, Cl3, C2h2, C2h3,
                                                C0, C, C2, C3, orig, b1, b2, byp, nb, rowvec, dd})
      hipFree(b);
  }
  return 0;
}
