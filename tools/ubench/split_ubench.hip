// Microbenchmark + accuracy check of the split-bf16 direct conv (csrc/split.h)
// on the conv2 forward problem (B=32, 32x32, 32 -> 64 channels, 5x5, both
// towers) and conv3 fwd / conv2 dgrad shapes.  Build: make -C tools/ubench
#include <cmath>
#include <cstring>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../../distributed-deep-q_amd/csrc/split.h"

using namespace ddq;

#define CK(x)                                                                      \
  do {                                                                             \
    hipError_t e = (x);                                                            \
    if (e != hipSuccess) {                                                         \
      printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); \
      exit(1);                                                                     \
    }                                                                              \
  } while (0)

static uint16_t bf16_bits(float x) {   // RNE
  uint32_t u;
  memcpy(&u, &x, 4);
  u += 0x7fff + ((u >> 16) & 1);
  return (uint16_t)(u >> 16);
}
static float bf16_val(uint16_t b) {
  uint32_t u = (uint32_t)b << 16;
  float f;
  memcpy(&f, &u, 4);
  return f;
}
static void split_host(const std::vector<float>& x, std::vector<uint16_t>& s) {
  const size_t E = x.size();
  s.resize(3 * E);
  for (size_t e = 0; e < E; ++e) {
    const uint16_t h = bf16_bits(x[e]);
    const float r = x[e] - bf16_val(h);
    const uint16_t m = bf16_bits(r);
    const uint16_t l = bf16_bits(r - bf16_val(m));
    s[e] = h; s[E + e] = m; s[2 * E + e] = l;
  }
}

struct Prob {
  int B, H, CP, N, KS, pad, nz;
};

template <int CPT, int CP, int N, int KS, int TY, int TX, int WM, int WN>
static void run(const char* name, const Prob& P, int reps) {
  const int B = P.B, H = P.H, W = H, T = KS * KS;
  srand(1);
  auto rnd = [] { return (float)rand() / RAND_MAX * 2.f - 1.f; };
  std::vector<float> x((size_t)B * H * W * CPT), w((size_t)N * T * CPT), bias(N);
  for (auto& v : x) v = fmaxf(rnd(), 0.f) * 3.f;            // ReLU'd, pooled-like
  for (auto& v : w) v = rnd() * 0.05f;
  for (auto& v : bias) v = rnd() * 0.01f;
  std::vector<uint16_t> xs, ws;
  split_host(x, xs);
  split_host(w, ws);
  const size_t Eo = (size_t)B * (H / 2) * (W / 2) * N;
  __bf16 *dx, *dw;
  float *db, *dout;
  __bf16* dos;
  uint8_t* dm;
  CK(hipMalloc(&dx, xs.size() * 2));
  CK(hipMalloc(&dw, ws.size() * 2));
  CK(hipMalloc(&db, N * 4));
  CK(hipMalloc(&dout, 2 * Eo * 4));
  CK(hipMalloc(&dos, 2 * 3 * Eo * 2));
  CK(hipMalloc(&dm, 2 * Eo));
  CK(hipMemcpy(dx, xs.data(), xs.size() * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(dw, ws.data(), ws.size() * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(db, bias.data(), N * 4, hipMemcpyHostToDevice));
  SplitArgs a{};
  a.B = B; a.H = H; a.W = W; a.pad = P.pad;
  for (int z = 0; z < 2; ++z) {
    a.in[z] = dx; a.wk[z] = dw; a.bias[z] = db;
    a.out[z] = dout + z * Eo; a.out_split[z] = dos + z * 3 * Eo; a.mask[z] = dm + z * Eo;
  }
  a.in_elems = x.size(); a.wk_elems = w.size(); a.out_elems = Eo;
  CK((launch_split_conv<CPT, CP, N, KS, TY, TX, WM, WN, 1, false>(a, P.nz, 0)));
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventRecord(e0, 0));
  for (int i = 0; i < reps; ++i) CK((launch_split_conv<CPT, CP, N, KS, TY, TX, WM, WN, 1, false>(a, P.nz, 0)));
  CK(hipEventRecord(e1, 0));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  const double us = ms * 1e3 / reps;
  const double flops = 2.0 * P.nz * B * H * W * (double)N * CPT * T;
  // accuracy on sampled pooled outputs (fp64 reference), err / sum|terms|
  std::vector<float> out(Eo);
  std::vector<uint16_t> os(3 * Eo);
  CK(hipMemcpy(out.data(), dout, Eo * 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(os.data(), dos, 3 * Eo * 2, hipMemcpyDeviceToHost));
  double worst = 0, worst_rel = 0, split_err = 0;
  int bad_route = 0;
  for (int s = 0; s < 4000; ++s) {
    const size_t e = ((size_t)rand() * 7919u) % Eo;
    const int n = e % N, pxx = (e / N) % (W / 2), pyy = (e / N / (W / 2)) % (H / 2);
    const int b = e / N / (W / 2) / (H / 2);
    double best = -1e300, bmag = 0;
    double vals[4], mags[4];
    for (int q = 0; q < 4; ++q) {
      const int y = 2 * pyy + (q >> 1), xx = 2 * pxx + (q & 1);
      double acc = bias[n], mag = fabs(bias[n]);
      for (int ky = 0; ky < KS; ++ky)
        for (int kx = 0; kx < KS; ++kx) {
          const int gy = y + ky - P.pad, gx = xx + kx - P.pad;
          if (gy < 0 || gy >= H || gx < 0 || gx >= W) continue;
          for (int c = 0; c < CPT; ++c) {
            const double t = (double)x[(((size_t)b * H + gy) * W + gx) * CPT + c] *
                             w[((size_t)n * T + ky * KS + kx) * CPT + c];
            acc += t; mag += fabs(t);
          }
        }
      vals[q] = acc; mags[q] = mag;
    }
    int arg = 0;
    for (int q = 0; q < 4; ++q) if (vals[q] > best) { best = vals[q]; arg = q; bmag = mags[q]; }
    (void)arg;
    const double ref = best > 0 ? best : 0;
    const double err = fabs(out[e] - ref);
    worst = fmax(worst, err / (bmag + 1e-30));
    if (fabs(ref) > 0.1 * bmag) worst_rel = fmax(worst_rel, err / fabs(ref));
    const double rec = (double)bf16_val(os[e]) + bf16_val(os[Eo + e]) + bf16_val(os[2 * Eo + e]);
    split_err = fmax(split_err, fabs(rec - out[e]) / (fabs(out[e]) + 1e-30));
  }
  printf("%-34s %8.2f us  %7.1f TF/s (bf16x6 eq. peak 419)  err/|terms| %.3g  rel %.3g  split %.3g%s\n",
         name, us, flops / us * 1e-6, worst, worst_rel, split_err, bad_route ? " ROUTE" : "");
  CK(hipFree(dx)); CK(hipFree(dw)); CK(hipFree(db)); CK(hipFree(dout)); CK(hipFree(dos)); CK(hipFree(dm));
}

template <int TY, int TX, int WM>
static void run_conv1(const char* name, int reps) {
  const int B = 32, H = 64, W = 64, N = 32;
  srand(2);
  std::vector<float> x((size_t)B * H * W * 4), w(32 * 4 * 49), bias(N);
  const float lv[3] = {0.f, 200.f, 255.f};
  for (auto& v : x) { const int r = rand() % 10; v = r < 8 ? lv[0] : (r < 9 ? lv[1] : lv[2]); }
  for (auto& v : w) v = ((float)rand() / RAND_MAX * 2.f - 1.f) * 0.01f;
  for (auto& v : bias) v = ((float)rand() / RAND_MAX * 2.f - 1.f) * 0.01f;
  // kernel layout [n][ky][kx 0..7][ci] from Caffe (n, ci, ky, kx), kx 7 = 0
  std::vector<float> wk(kConv1WPlane, 0.f);
  for (int n = 0; n < 32; ++n)
    for (int ci = 0; ci < 4; ++ci)
      for (int ky = 0; ky < 7; ++ky)
        for (int kx = 0; kx < 7; ++kx)
          wk[((n * 7 + ky) * 8 + kx) * 4 + ci] = w[((n * 4 + ci) * 7 + ky) * 7 + kx];
  std::vector<uint16_t> ws;
  split_host(wk, ws);
  const size_t Eo = (size_t)B * (H / 2) * (W / 2) * N;
  float *dx, *db, *dout;
  __bf16 *dw, *dos;
  uint8_t* dm;
  CK(hipMalloc(&dx, x.size() * 4));
  CK(hipMalloc(&dw, ws.size() * 2));
  CK(hipMalloc(&db, N * 4));
  CK(hipMalloc(&dout, 2 * Eo * 4));
  CK(hipMalloc(&dos, 2 * 3 * Eo * 2));
  CK(hipMalloc(&dm, 2 * Eo));
  CK(hipMemcpy(dx, x.data(), x.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dw, ws.data(), ws.size() * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(db, bias.data(), N * 4, hipMemcpyHostToDevice));
  Conv1Args a{};
  a.B = B; a.H = H; a.W = W;
  for (int z = 0; z < 2; ++z) {
    a.in[z] = dx; a.wk[z] = dw; a.bias[z] = db; a.out[z] = dout + z * Eo;
    a.out_split[z] = dos + z * 3 * Eo; a.mask[z] = dm + z * Eo;
  }
  a.out_elems = Eo;
  CK((launch_split_conv1<TY, TX, WM>(a, 2, 0, kConv1WPlane)));
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventRecord(e0, 0));
  for (int i = 0; i < reps; ++i) CK((launch_split_conv1<TY, TX, WM>(a, 2, 0, kConv1WPlane)));
  CK(hipEventRecord(e1, 0));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  const double us = ms * 1e3 / reps;
  const double flops = 2.0 * 2 * B * H * W * 32.0 * 196;
  std::vector<float> out(Eo);
  std::vector<uint8_t> mk(Eo);
  CK(hipMemcpy(out.data(), dout, Eo * 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(mk.data(), dm, Eo, hipMemcpyDeviceToHost));
  double worst = 0;
  int route_bad = 0;
  for (int s = 0; s < 4000; ++s) {
    const size_t e = ((size_t)rand() * 7919u) % Eo;
    const int n = e % N, pxx = (e / N) % (W / 2), pyy = (e / N / (W / 2)) % (H / 2);
    const int b = e / N / (W / 2) / (H / 2);
    double best = -1e300, bmag = 0, vals[4];
    int arg = 0;
    for (int q = 0; q < 4; ++q) {
      const int y = 2 * pyy + (q >> 1), xx = 2 * pxx + (q & 1);
      double acc = bias[n], mag = fabs(bias[n]);
      for (int ky = 0; ky < 7; ++ky)
        for (int kx = 0; kx < 7; ++kx) {
          const int gy = y + ky - 3, gx = xx + kx - 3;
          if (gy < 0 || gy >= H || gx < 0 || gx >= W) continue;
          for (int c = 0; c < 4; ++c) {
            const double t = (double)x[(((size_t)b * H + gy) * W + gx) * 4 + c] *
                             w[((n * 4 + c) * 7 + ky) * 7 + kx];
            acc += t; mag += fabs(t);
          }
        }
      vals[q] = acc;
      if (acc > best) { best = acc; arg = q; bmag = mag; }
    }
    (void)vals;
    const double ref = best > 0 ? best : 0;
    worst = fmax(worst, fabs(out[e] - ref) / (bmag + 1e-30));
    if ((best > 0 ? arg : 4) != mk[e]) ++route_bad;
  }
  printf("%-34s %8.2f us  %7.1f TF/s  err/|terms| %.3g  route mismatches %d/4000\n", name, us,
         flops / us * 1e-6, worst, route_bad);
  CK(hipFree(dx)); CK(hipFree(dw)); CK(hipFree(db)); CK(hipFree(dout)); CK(hipFree(dos)); CK(hipFree(dm));
}

int main(int argc, char** argv) {
  const int only = argc > 1 ? atoi(argv[1]) : -1;
  int id = 0;
  auto want = [&]() { return only < 0 || only == id++; };
  Prob c2{32, 32, 32, 64, 5, 2, 2};
  if (want()) run<32, 32, 64, 5, 16, 16, 8, 2>("0 conv2 fwd 16x16 16w (TN1)", c2, 50);
  if (want()) run<32, 32, 64, 5, 16, 16, 8, 1>("1 conv2 fwd 16x16 8w (TN2)", c2, 50);
  if (want()) run<32, 16, 64, 5, 16, 32, 16, 1>("2 conv2 fwd 16x32 16w TN2 ch16", c2, 50);
  Prob d2{32, 32, 64, 32, 5, 2, 1};
  if (want()) run<64, 32, 32, 5, 16, 16, 8, 1>("3 conv2 dgrad-shape 16x16 8w ch32", d2, 50);
  if (want()) run<64, 32, 32, 5, 16, 16, 4, 1>("4 conv2 dgrad-shape 16x16 4w ch32", d2, 50);
  if (want()) run<64, 16, 32, 5, 16, 32, 16, 1>("5 conv2 dgrad-shape 16x32 16w ch16", d2, 50);
  Prob c3{32, 16, 64, 64, 3, 1, 2};
  if (want()) run<64, 64, 64, 3, 8, 8, 2, 2>("6 conv3 fwd 8x8 4w", c3, 50);
  if (want()) run<64, 32, 64, 3, 8, 16, 4, 2>("7 conv3 fwd 8x16 8w ch32", c3, 50);
  if (want()) run<64, 32, 64, 3, 16, 16, 8, 2>("8 conv3 fwd 16x16 16w ch32", c3, 50);
  Prob d3{32, 16, 64, 64, 3, 1, 1};
  if (want()) run<64, 32, 64, 3, 8, 16, 4, 2>("9 conv3 dgrad-shape 8x16 8w ch32", d3, 50);
  if (want()) run<64, 64, 64, 3, 8, 8, 2, 2>("10 conv3 dgrad-shape 8x8 4w", d3, 50);
  if (want()) run_conv1<16, 32, 8>("11 conv1 fwd 16x32 8w", 50);
  if (want()) run_conv1<16, 32, 4>("12 conv1 fwd 16x32 4w (TM4)", 50);
  if (want()) run_conv1<16, 16, 4>("13 conv1 fwd 16x16 4w", 50);
  if (want()) run_conv1<32, 32, 16>("14 conv1 fwd 32x32 16w", 50);
  if (want()) run<64, 32, 32, 5, 16, 8, 4, 1>("15 conv2 dgrad-shape 16x8 4w ch32", d2, 50);
  if (want()) run<64, 32, 32, 5, 8, 16, 4, 1>("16 conv2 dgrad-shape 8x16 4w ch32", d2, 50);
  if (want()) run<64, 32, 32, 5, 8, 8, 2, 1>("17 conv2 dgrad-shape 8x8 2w ch32", d2, 50);
  if (want()) run<64, 64, 32, 5, 8, 16, 4, 1>("18 conv2 dgrad-shape 8x16 4w ch64", d2, 50);
  if (want()) run<64, 64, 32, 5, 8, 8, 2, 1>("19 conv2 dgrad-shape 8x8 2w ch64", d2, 50);
  if (want()) run<64, 32, 32, 5, 16, 16, 2, 1>("20 conv2 dgrad-shape 16x16 2w TM4 ch32", d2, 50);
  if (want()) run<64, 32, 32, 5, 8, 16, 2, 1>("21 conv2 dgrad-shape 8x16 2w TM2 ch32", d2, 50);
  if (want()) run<64, 64, 32, 5, 16, 8, 4, 1>("22 conv2 dgrad-shape 16x8 4w ch64", d2, 50);
  if (want()) run<64, 64, 64, 3, 8, 16, 4, 2>("23 conv3 dgrad-shape 8x16 8w ch64", d3, 50);
  if (want()) run<64, 64, 64, 3, 8, 8, 2, 1>("24 conv3 dgrad-shape 8x8 2w TN2", d3, 50);
  if (want()) run<64, 64, 64, 3, 4, 16, 2, 2>("25 conv3 dgrad-shape 4x16 4w", d3, 50);
  if (want()) run<32, 32, 64, 5, 16, 16, 4, 2>("26 conv2 fwd 16x16 8w TM2", c2, 50);
  if (want()) run<32, 32, 64, 5, 16, 16, 4, 1>("27 conv2 fwd 16x16 4w TM2 TN2", c2, 50);
  if (want()) run<32, 32, 64, 5, 16, 16, 2, 2>("28 conv2 fwd 16x16 4w TM4", c2, 50);
  if (want()) run<64, 64, 64, 3, 16, 8, 4, 1>("29 conv3 fwd 16x8 4w TN2", c3, 50);
  if (want()) run<64, 32, 64, 3, 16, 16, 8, 1>("30 conv3 fwd 16x16 8w TN2 ch32", c3, 50);
  if (want()) run<64, 64, 64, 3, 8, 16, 4, 1>("31 conv3 fwd 8x16 4w TN2", c3, 50);
  if (want()) run<64, 32, 64, 3, 4, 8, 1, 2>("32 conv3 fwd 4x8 2w ch32", c3, 50);
  if (want()) run<64, 64, 64, 3, 4, 8, 1, 2>("33 conv3 fwd 4x8 2w", c3, 50);
  if (want()) run<64, 32, 64, 3, 8, 8, 2, 2>("34 conv3 fwd 8x8 4w ch32", c3, 50);
  if (want()) run<64, 64, 64, 3, 4, 16, 2, 2>("35 conv3 fwd 4x16 4w", c3, 50);
  return 0;
}
