// Timing lab of the second-generation attention consumers (zv_flash2.inc) on one decoder stream's
// shape, built twice -- bf16 operands and fp16 operands (-DZV_OPERAND_F16, the parity-grade mode's
// library, with its per-query offsets) -- to see what the operand format costs per launch:
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I zipvoice_amd/csrc tools/lab/attn2_time_lab.hip -o tools/lab/attn2_time_bf16
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -DZV_OPERAND_F16 -I zipvoice_amd/csrc tools/lab/attn2_time_lab.hip -o tools/lab/attn2_time_f16
//   attn2_time_{bf16,f16} [B L [iters [scale]]]
// Random operands (uniform, |q|, |k| <= scale): scores of a few units, every query on the fast path.
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "zv_flash2.inc"

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
// V^T rows of the SelfAttention heads: row 12 of every 16 the ones row
static __global__ void ones_rows(bf16* v, long rows, int Lpad) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < rows * Lpad; i += (long)gridDim.x * blockDim.x) {
    const long r = i / Lpad;
    if (r % 16 == 12) v[i] = (bf16)1.f;
    else if (r % 16 > 12) v[i] = (bf16)0.f;
  }
}

int main(int argc, char** argv) {
  const int B = argc > 2 ? atoi(argv[1]) : 21, L = argc > 2 ? atoi(argv[2]) : 1219;
  const int iters = argc > 3 ? atoi(argv[3]) : 20;
  const float scale = argc > 4 ? (float)atof(argv[4]) : 0.5f;
  const int H = 4, nv_na = 384;
  const long ldq = 2L * H * ATT_QD + H * ATT_PD, Lpad = round_up(L, 64), M = (long)B * L;
  bf16 *q, *vsa, *vna, *y, *osa, *ona;
  float* P;
  unsigned* cnt;
  ZV_CHECK(hipMalloc(&q, M * ldq * 2));
  ZV_CHECK(hipMalloc(&vsa, (long)B * 16 * H * Lpad * 2));
  ZV_CHECK(hipMalloc(&vna, (long)B * nv_na * Lpad * 2));
  ZV_CHECK(hipMalloc(&y, M * nv_na * 2));
  ZV_CHECK(hipMalloc(&osa, M * 48 * 2));
  ZV_CHECK(hipMalloc(&ona, M * nv_na * 2));
  ZV_CHECK(hipMalloc(&P, (long)(2 * L - 1) * H * ATT_PD * 4));
  ZV_CHECK(hipMalloc(&cnt, 16));
  ZV_CHECK(hipMemset(cnt, 0, 16));
  fill_rand<<<1024, 256>>>(q, M * ldq, 1, scale);
  fill_rand<<<1024, 256>>>(vsa, (long)B * 16 * H * Lpad, 2, 1.f);
  ones_rows<<<1024, 256>>>(vsa, (long)B * 16 * H, (int)Lpad);
  fill_rand<<<1024, 256>>>(vna, (long)B * nv_na * Lpad, 3, 1.f);
  fill_rand<<<1024, 256>>>(y, M * nv_na, 4, 1.f);
  fill_rand_f<<<1024, 256>>>(P, (long)(2 * L - 1) * H * ATT_PD, 5, scale);
  ZV_CHECK(hipDeviceSynchronize());
  FlashParams f{};
  f.qh = q; f.ldq = ldq; f.P = P; f.B = B; f.L = L; f.H = H; f.fallback = cnt;
  FlashParams fs = f, fn = f;
  fs.vh = vsa; fs.ldv = Lpad; fs.sv_b = 16L * H * Lpad; fs.vrows_per_head = 16; fs.nv = 12;
  fs.oh = osa; fs.ldo = 48; fs.ocol_per_head = 12;
  fn.vh = vna; fn.ldv = Lpad; fn.sv_b = (long)nv_na * Lpad; fn.nv = nv_na; fn.mulh = y; fn.ldmul = nv_na;
  fn.oh = ona; fn.ldo = nv_na;
  hipEvent_t e0, e1;
  ZV_CHECK(hipEventCreate(&e0));
  ZV_CHECK(hipEventCreate(&e1));
  auto time = [&](const char* name, auto launch) {
    launch();
    ZV_CHECK(hipDeviceSynchronize());
    ZV_CHECK(hipEventRecord(e0, 0));
    for (int i = 0; i < iters; ++i) launch();
    ZV_CHECK(hipEventRecord(e1, 0));
    ZV_CHECK(hipEventSynchronize(e1));
    float ms = 0.f;
    ZV_CHECK(hipEventElapsedTime(&ms, e0, e1));
    unsigned c[4];
    ZV_CHECK(hipMemcpy(c, cnt, 16, hipMemcpyDeviceToHost));
    printf("%-6s %-10s B=%d L=%d: %8.2f us per launch (exact-path runs so far %u)\n", ZV_OPERAND_NAME, name, B, L,
           1e3f * ms / iters, c[2]);
  };
  const int q3 = sa3_qpw(L);
  if (q3 == 4) time("sa3<4>", [&] { launch_attn_sa3<4>(fs, 0); });
  if (q3 == 3) time("sa3<3>", [&] { launch_attn_sa3<3>(fs, 0); });
  if (q3 == 2) time("sa3<2>", [&] { launch_attn_sa3<2>(fs, 0); });
  if (q3 == 0) time("sa2<2>", [&] { launch_attn_sa2<2>(fs, 0); });
  if (na2_qtiles(L) == 4) time("na2<3,4>", [&] { launch_attn_na2<3, 4>(fn, 0); });
  else time("na2<3,8>", [&] { launch_attn_na2<3>(fn, 0); });
  // the exact path alone (every unit forced), for its cost
  fs.force_exact = fn.force_exact = 1;
  if (q3 == 4) time("sa3<4>!x", [&] { launch_attn_sa3<4>(fs, 0); });
  if (na2_qtiles(L) != 4) time("na2<3,8>!x", [&] { launch_attn_na2<3>(fn, 0); });
  return 0;
}
