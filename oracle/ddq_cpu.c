/*
 * ORACLE -- test infrastructure only (checker + bench.py cpu_baseline leg).
 * NOT product code; the shipped path never links or loads this library.
 *
 * Plain-C fp32 restatement of the reference's CPU training step, following
 * the algorithm of the (absent) Caffe CPU layers the reference runs in
 * `--mode cpu` (main.py:148-149; train_val.prototxt:38-483):
 *   CONVOLUTION  = per-image im2col + SGEMM (W[Cout x K] * col[K x HW]) + bias
 *   RELU in place, POOLING MAX 2x2/2 with first-max argmax,
 *   INNER_PRODUCT = SGEMM, DROPOUT = identity (TEST phase, main.py:147),
 *   ELTWISE PROD/SUM/MAX, SLICE, EUCLIDEAN_LOSS = sum(d^2)/(2N),
 *   backward: weight diffs zeroed then accumulated over images, bottom diff
 *   via W^T * top_diff + col2im; ReLU mask top > 0; pool routes to argmax.
 * plus the param-server apply rules (param-server/server.py:81-124).
 *
 * Parity status: the Caffe submodule (kjchavez/caffe, commit unknown,
 * .gitmodules:1-3) cannot be built here, so this restatement is not pinned by
 * reference outputs ("parity unpinned"); tests cross-check it against the
 * float64 numpy restatement (oracle/ref_numpy.py).
 *
 * Parallelism: `threads` OpenMP threads -- conv layers over the images of
 * the batch (Caffe's CPU conv loops over images with one BLAS call each),
 * the fc layers as batch GEMMs split over column slices.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define NA 4
#define FC4 512

typedef struct {
  int S;
  long w[5], b[5], wn[5], bn[5], total;
} layout_t;

static layout_t mk_layout(int S) {
  layout_t L;
  const long s4 = S / 8, k4 = 64 * s4 * s4;
  const long wn[5] = {32 * 4 * 49, 64 * 32 * 25, 64 * 64 * 9, 512 * k4, 4 * 512};
  const long bn[5] = {32, 64, 64, 512, 4};
  long o = 0;
  L.S = S;
  for (int i = 0; i < 5; ++i) {
    L.w[i] = o; L.wn[i] = wn[i]; o += wn[i];
    L.b[i] = o; L.bn[i] = bn[i]; o += bn[i];
  }
  L.total = o;
  return L;
}

long ddq_cpu_num_params(int S) { return mk_layout(S).total; }

/*
 * Packed, cache-blocked SGEMM (the GotoBLAS/BLIS scheme Caffe's CPU path gets
 * from its BLAS): C[M x N] (+)= op(A)[M x K] * op(B)[K x N], row-major with
 * leading dimensions; ta / tb read A / B transposed.  B is packed into
 * KC x NR column panels, A into MR x KC row panels, and a register-tiled
 * micro-kernel (AVX-512 12x32 or AVX2 6x16 FMA, chosen at run time) runs
 * over the packed panels.  Sequential: callers parallelise over images or
 * over column slices (pgemm).
 */
#include <immintrin.h>

#define KC 384
#define NC 3072
#define MC 192

typedef void (*ukern_t)(int kc, const float* a, const float* b, float* c, int ldc, int mr, int nr);

__attribute__((target("avx512f,fma"))) static void uk_avx512(int kc, const float* a,
                                                           const float* b, float* c, int ldc,
                                                           int mr, int nr) {
  __m512 acc[12][2];
  for (int i = 0; i < 12; ++i) acc[i][0] = acc[i][1] = _mm512_setzero_ps();
  for (int k = 0; k < kc; ++k) {
    const __m512 b0 = _mm512_loadu_ps(b + 32 * k), b1 = _mm512_loadu_ps(b + 32 * k + 16);
    for (int i = 0; i < 12; ++i) {
      const __m512 ai = _mm512_set1_ps(a[12 * k + i]);
      acc[i][0] = _mm512_fmadd_ps(ai, b0, acc[i][0]);
      acc[i][1] = _mm512_fmadd_ps(ai, b1, acc[i][1]);
    }
  }
  if (mr == 12 && nr == 32) {
    for (int i = 0; i < 12; ++i) {
      float* ci = c + (size_t)i * ldc;
      _mm512_storeu_ps(ci, _mm512_add_ps(_mm512_loadu_ps(ci), acc[i][0]));
      _mm512_storeu_ps(ci + 16, _mm512_add_ps(_mm512_loadu_ps(ci + 16), acc[i][1]));
    }
  } else {
    float t[12][32];
    for (int i = 0; i < 12; ++i) {
      _mm512_storeu_ps(t[i], acc[i][0]);
      _mm512_storeu_ps(t[i] + 16, acc[i][1]);
    }
    for (int i = 0; i < mr; ++i)
      for (int j = 0; j < nr; ++j) c[(size_t)i * ldc + j] += t[i][j];
  }
}

__attribute__((target("avx2,fma"))) static void uk_avx2(int kc, const float* a, const float* b,
                                                      float* c, int ldc, int mr, int nr) {
  __m256 acc[6][2];
  for (int i = 0; i < 6; ++i) acc[i][0] = acc[i][1] = _mm256_setzero_ps();
  for (int k = 0; k < kc; ++k) {
    const __m256 b0 = _mm256_loadu_ps(b + 16 * k), b1 = _mm256_loadu_ps(b + 16 * k + 8);
    for (int i = 0; i < 6; ++i) {
      const __m256 ai = _mm256_broadcast_ss(a + 6 * k + i);
      acc[i][0] = _mm256_fmadd_ps(ai, b0, acc[i][0]);
      acc[i][1] = _mm256_fmadd_ps(ai, b1, acc[i][1]);
    }
  }
  float t[6][16];
  for (int i = 0; i < 6; ++i) {
    _mm256_storeu_ps(t[i], acc[i][0]);
    _mm256_storeu_ps(t[i] + 8, acc[i][1]);
  }
  for (int i = 0; i < mr; ++i)
    for (int j = 0; j < nr; ++j) c[(size_t)i * ldc + j] += t[i][j];
}

static int g_mr, g_nr;
static ukern_t g_uk;

static void gemm_init(void) {
  if (g_uk) return;
  __builtin_cpu_init();
  if (__builtin_cpu_supports("avx512f")) { g_mr = 12; g_nr = 32; g_uk = uk_avx512; }
  else { g_mr = 6; g_nr = 16; g_uk = uk_avx2; }
}

/* force the micro-kernel (tests): 512 = AVX-512, 256 = AVX2; returns the one in use */
int ddq_cpu_set_isa(int isa) {
  gemm_init();
  if (isa == 512 && __builtin_cpu_supports("avx512f")) { g_mr = 12; g_nr = 32; g_uk = uk_avx512; }
  if (isa == 256) { g_mr = 6; g_nr = 16; g_uk = uk_avx2; }
  return g_uk == uk_avx512 ? 512 : 256;
}

/* per-thread packing buffers */
static __thread float* t_ap;
static __thread float* t_bp;

static void sgemm(int ta, int tb, int M, int N, int K, const float* A, int lda, const float* B,
                  int ldb, float* C, int ldc, int accumulate) {
  const int MR = g_mr, NR = g_nr;
  if (!accumulate)
    for (int m = 0; m < M; ++m) memset(C + (size_t)m * ldc, 0, sizeof(float) * N);
  if (!t_ap) {
    t_ap = (float*)aligned_alloc(64, sizeof(float) * (MC + 16) * KC);
    t_bp = (float*)aligned_alloc(64, sizeof(float) * (NC + 32) * KC);
  }
  float *ap = t_ap, *bp = t_bp;
  for (int jc = 0; jc < N; jc += NC) {
    const int nc = N - jc < NC ? N - jc : NC;
    for (int pc = 0; pc < K; pc += KC) {
      const int kc = K - pc < KC ? K - pc : KC;
      /* B block -> NR-wide panels [panel][k][NR], zero padded */
      for (int jp = 0; jp < nc; jp += NR) {
        float* dst = bp + (size_t)(jp / NR) * kc * NR;
        const int nr = nc - jp < NR ? nc - jp : NR;
        for (int k = 0; k < kc; ++k) {
          float* d = dst + (size_t)k * NR;
          if (!tb) {
            const float* src = B + (size_t)(pc + k) * ldb + jc + jp;
            memcpy(d, src, sizeof(float) * nr);
          } else {
            for (int j = 0; j < nr; ++j) d[j] = B[(size_t)(jc + jp + j) * ldb + pc + k];
          }
          for (int j = nr; j < NR; ++j) d[j] = 0.f;
        }
      }
      for (int ic = 0; ic < M; ic += MC) {
        const int mc = M - ic < MC ? M - ic : MC;
        /* A block -> MR-tall panels [panel][k][MR], zero padded */
        for (int ip = 0; ip < mc; ip += MR) {
          float* dst = ap + (size_t)(ip / MR) * kc * MR;
          const int mr = mc - ip < MR ? mc - ip : MR;
          for (int k = 0; k < kc; ++k) {
            float* d = dst + (size_t)k * MR;
            for (int i = 0; i < mr; ++i)
              d[i] = ta ? A[(size_t)(pc + k) * lda + ic + ip + i]
                        : A[(size_t)(ic + ip + i) * lda + pc + k];
            for (int i = mr; i < MR; ++i) d[i] = 0.f;
          }
        }
        for (int jr = 0; jr < nc; jr += NR)
          for (int ir = 0; ir < mc; ir += MR)
            g_uk(kc, ap + (size_t)(ir / MR) * kc * MR, bp + (size_t)(jr / NR) * kc * NR,
                 C + (size_t)(ic + ir) * ldc + jc + jr, ldc, mc - ir < MR ? mc - ir : MR,
                 nc - jr < NR ? nc - jr : NR);
      }
    }
  }
}

/* sgemm split over column slices of C across the OpenMP team */
static void pgemm(int ta, int tb, int M, int N, int K, const float* A, int lda, const float* B,
                  int ldb, float* C, int ldc, int accumulate, int nth) {
  const int NR = g_nr;
  int slice = (N + nth - 1) / nth;
  slice = (slice + NR - 1) / NR * NR;
  const int ns = (N + slice - 1) / slice;
#pragma omp parallel for schedule(static) num_threads(nth)
  for (int s = 0; s < ns; ++s) {
    const int n0 = s * slice, nn = N - n0 < slice ? N - n0 : slice;
    sgemm(ta, tb, M, nn, K, A, lda, tb ? B + (size_t)n0 * ldb : B + n0, ldb, C + n0, ldc,
          accumulate);
  }
}

static void im2col(const float* x, int C, int H, int W, int k, int pad, float* col) {
  for (int c = 0; c < C; ++c)
    for (int ky = 0; ky < k; ++ky)
      for (int kx = 0; kx < k; ++kx) {
        float* dst = col + ((size_t)(c * k + ky) * k + kx) * H * W;
        for (int y = 0; y < H; ++y) {
          const int yy = y + ky - pad;
          for (int xx0 = 0; xx0 < W; ++xx0) {
            const int xx = xx0 + kx - pad;
            dst[y * W + xx0] = (yy >= 0 && yy < H && xx >= 0 && xx < W)
                                   ? x[((size_t)c * H + yy) * W + xx] : 0.f;
          }
        }
      }
}

static void col2im(const float* col, int C, int H, int W, int k, int pad, float* x) {
  memset(x, 0, sizeof(float) * (size_t)C * H * W);
  for (int c = 0; c < C; ++c)
    for (int ky = 0; ky < k; ++ky)
      for (int kx = 0; kx < k; ++kx) {
        const float* src = col + ((size_t)(c * k + ky) * k + kx) * H * W;
        for (int y = 0; y < H; ++y) {
          const int yy = y + ky - pad;
          if (yy < 0 || yy >= H) continue;
          for (int x0 = 0; x0 < W; ++x0) {
            const int xx = x0 + kx - pad;
            if (xx >= 0 && xx < W) x[((size_t)c * H + yy) * W + xx] += src[y * W + x0];
          }
        }
      }
}

static const int COUT[3] = {32, 64, 64}, CIN[3] = {4, 32, 64}, KS[3] = {7, 5, 3}, PAD[3] = {3, 2, 1};

/* One image's conv stack (Caffe's conv layers loop over the images of the
 * batch, im2col + GEMM each).  act[l]: post-ReLU conv output (Cout,H,W),
 * pool[l]: pooled (Cout,H/2,W/2), arg[l]: argmax 0..3 (first max). */
typedef struct {
  float* act[3];
  float* pool[3];
  unsigned char* arg[3];
} conv_ws;

static size_t conv_ws_floats(int S) {
  size_t f = 0;
  for (int l = 0, H = S; l < 3; ++l, H /= 2) f += (size_t)COUT[l] * H * H * 5 / 4;
  return f;
}

static void conv_ws_bind(conv_ws* ws, int S, float* f, unsigned char* u) {
  for (int l = 0, H = S; l < 3; ++l, H /= 2) {
    const size_t n = (size_t)COUT[l] * H * H;
    ws->act[l] = f; f += n;
    ws->pool[l] = f; f += n / 4;
    ws->arg[l] = u; u += n / 4;
  }
}

static size_t col_floats(int S) {
  size_t m = 0;
  for (int l = 0, H = S; l < 3; ++l, H /= 2) {
    const size_t c = (size_t)CIN[l] * KS[l] * KS[l] * H * H;
    if (c > m) m = c;
  }
  return m;
}

static void conv_stack_fwd(const layout_t* L, const float* th, const float* x, conv_ws* ws,
                           float* col) {
  const float* in = x;
  int H = L->S;
  for (int l = 0; l < 3; ++l) {
    const int K = CIN[l] * KS[l] * KS[l], HW = H * H;
    im2col(in, CIN[l], H, H, KS[l], PAD[l], col);
    sgemm(0, 0, COUT[l], HW, K, th + L->w[l], K, col, HW, ws->act[l], HW, 0);
    for (int c = 0; c < COUT[l]; ++c) {
      const float b = th[L->b[l] + c];
      float* a = ws->act[l] + (size_t)c * HW;
      for (int i = 0; i < HW; ++i) { const float v = a[i] + b; a[i] = v > 0.f ? v : 0.f; }
    }
    const int Hp = H / 2;
    for (int c = 0; c < COUT[l]; ++c)
      for (int py = 0; py < Hp; ++py)
        for (int px = 0; px < Hp; ++px) {
          const float* a = ws->act[l] + (size_t)c * HW;
          float mx = -3.402823466e38f;
          int arg = 0;
          for (int d = 0; d < 4; ++d) {
            const float v = a[(2 * py + (d >> 1)) * H + 2 * px + (d & 1)];
            if (v > mx) { mx = v; arg = d; }
          }
          ws->pool[l][((size_t)c * Hp + py) * Hp + px] = mx;
          ws->arg[l][((size_t)c * Hp + py) * Hp + px] = (unsigned char)arg;
        }
    in = ws->pool[l];
    H = Hp;
  }
}

/* fc4 (ReLU) + fc5 over the batch (Caffe's INNER_PRODUCT: one GEMM per layer
 * for the whole batch): pool3 (B, k4) -> h4 (B, 512) -> out (B, 4) */
static void fc_fwd(const layout_t* L, const float* th, int B, const float* pool3, float* h4,
                   float* out, int nth) {
  const int s4 = L->S / 8, k4 = 64 * s4 * s4;
  pgemm(0, 1, B, FC4, k4, pool3, k4, th + L->w[3], k4, h4, FC4, 0, nth);
  for (int n = 0; n < B; ++n)
    for (int o = 0; o < FC4; ++o) {
      const float v = h4[(size_t)n * FC4 + o] + th[L->b[3] + o];
      h4[(size_t)n * FC4 + o] = v > 0.f ? v : 0.f;
    }
  for (int n = 0; n < B; ++n)
    for (int a = 0; a < NA; ++a) {
      const float* w = th + L->w[4] + (size_t)a * FC4;
      float acc = 0.f;
      for (int k = 0; k < FC4; ++k) acc += w[k] * h4[(size_t)n * FC4 + k];
      out[n * NA + a] = acc + th[L->b[4] + a];
    }
}

/*
 * BaristaNet.full_pass (baristanet.py:138-140): forward both towers, target,
 * loss, Q backward -- every layer once (the Q forward activations are kept
 * for the backward).  Inputs in Caffe shapes.  blobs: Q_out[B*4], P_out[B*4],
 * Q_sa[B], P_sa[B], target[B], loss[1] (may be NULL).  grad: P floats.
 */
int ddq_cpu_full_pass(int B, int S, const float* thQ, const float* thP, const float* state,
                      const float* action, const float* reward, const float* next_state,
                      const float* nonterm, float gamma, float* grad, float* blobs, int threads) {
  if (S % 8 || B < 1) return -1;
  gemm_init();
  const layout_t L = mk_layout(S);
  const size_t img = (size_t)4 * S * S;
  const int s4 = S / 8, k4 = 64 * s4 * s4;
  int nth = threads > 0 ? threads : 1;
#ifndef _OPENMP
  nth = 1;
#endif
  const size_t wsf = conv_ws_floats(S), wsu = wsf;   /* arg bytes <= floats */
  const size_t colf = col_floats(S);
  const long conv_total = L.w[3];                    /* conv1..conv3 weights + biases */
  float* qws_f = (float*)malloc(sizeof(float) * wsf * B);
  unsigned char* qws_u = (unsigned char*)malloc(wsu * B);
  float* pws_f = (float*)malloc(sizeof(float) * wsf * nth);
  unsigned char* pws_u = (unsigned char*)malloc(wsu * nth);
  float* cols = (float*)malloc(sizeof(float) * colf * nth);
  float* pool3 = (float*)malloc(sizeof(float) * (size_t)2 * B * k4);   /* Q rows, then P rows */
  float* h4 = (float*)malloc(sizeof(float) * (size_t)2 * B * FC4);
  float* out = (float*)malloc(sizeof(float) * 2 * B * NA);
  float* dq = (float*)malloc(sizeof(float) * B * NA);
  float* dh4 = (float*)malloc(sizeof(float) * (size_t)B * FC4);
  float* dpool3 = (float*)malloc(sizeof(float) * (size_t)B * k4);
  float* gpart = (float*)calloc((size_t)nth * conv_total, sizeof(float));
  const size_t tmpf = (size_t)32 * S * S;            /* largest conv output */
  const size_t dcolf = colf;
  float* bwd = (float*)malloc(sizeof(float) * (2 * tmpf + dcolf) * nth);
  if (!qws_f || !qws_u || !pws_f || !pws_u || !cols || !pool3 || !h4 || !out || !dq || !dh4 ||
      !dpool3 || !gpart || !bwd)
    return -2;
  float* qsa = blobs ? blobs + 2 * B * NA : NULL;

  /* conv stacks: Q on state (kept), P on next_state (pool3 only) */
#pragma omp parallel for schedule(dynamic, 1) num_threads(nth)
  for (int j = 0; j < 2 * B; ++j) {
    int tid = 0;
#ifdef _OPENMP
    tid = omp_get_thread_num();
#endif
    conv_ws ws;
    const int n = j % B, q = j < B;
    if (q) conv_ws_bind(&ws, S, qws_f + wsf * n, qws_u + wsu * n);
    else conv_ws_bind(&ws, S, pws_f + wsf * tid, pws_u + wsu * tid);
    conv_stack_fwd(&L, q ? thQ : thP, (q ? state : next_state) + n * img, &ws,
                   cols + colf * tid);
    memcpy(pool3 + ((size_t)(q ? 0 : B) + n) * k4, ws.pool[2], sizeof(float) * k4);
  }
  fc_fwd(&L, thQ, B, pool3, h4, out, nth);
  fc_fwd(&L, thP, B, pool3 + (size_t)B * k4, h4 + (size_t)B * FC4, out + B * NA, nth);
  const float* qout = out;
  const float* pout = out + B * NA;

  /* head: Q_sa, P_sa (max * nonterm), target, Euclidean loss, dQ */
  float loss = 0.f;
  for (int n = 0; n < B; ++n) {
    const float* q = qout + n * NA;
    const float* a = action + n * NA;
    float s = 0.f;
    for (int k = 0; k < NA; ++k) s += q[k] * a[k];
    const float* p = pout + n * NA;
    float mx = p[0];
    for (int k = 1; k < NA; ++k) mx = p[k] > mx ? p[k] : mx;
    mx = mx * nonterm[n];
    const float t = gamma * mx + 1.0f * reward[n];
    if (qsa) { qsa[n] = s; qsa[B + n] = mx; qsa[2 * B + n] = t; }
    const float d = s - t;
    loss += d * d;
    for (int k = 0; k < NA; ++k) dq[n * NA + k] = a[k] * d / (float)B;
  }
  loss = loss / (float)B / 2.f;

  /* fc5 / fc4 backward over the batch */
  memset(grad, 0, sizeof(float) * L.total);
  for (int n = 0; n < B; ++n)
    for (int a = 0; a < NA; ++a) {
      const float d = dq[n * NA + a];
      for (int k = 0; k < FC4; ++k) grad[L.w[4] + a * FC4 + k] += d * h4[(size_t)n * FC4 + k];
      grad[L.b[4] + a] += d;
    }
  for (int n = 0; n < B; ++n)
    for (int k = 0; k < FC4; ++k) {
      float v = 0.f;
      for (int a = 0; a < NA; ++a) v += dq[n * NA + a] * thQ[L.w[4] + a * FC4 + k];
      dh4[(size_t)n * FC4 + k] = h4[(size_t)n * FC4 + k] > 0.f ? v : 0.f;
    }
  pgemm(1, 0, FC4, k4, B, dh4, FC4, pool3, k4, grad + L.w[3], k4, 0, nth);   /* dW4 */
  for (int n = 0; n < B; ++n)
    for (int o = 0; o < FC4; ++o) grad[L.b[3] + o] += dh4[(size_t)n * FC4 + o];
  pgemm(0, 0, B, k4, FC4, dh4, FC4, thQ + L.w[3], k4, dpool3, k4, 0, nth);   /* dpool3 */

  /* conv backward per image (weight diffs accumulated per thread) */
#pragma omp parallel for schedule(dynamic, 1) num_threads(nth)
  for (int n = 0; n < B; ++n) {
    int tid = 0;
#ifdef _OPENMP
    tid = omp_get_thread_num();
#endif
    float* g = gpart + (size_t)tid * conv_total;
    float* dtop = bwd + (2 * tmpf + dcolf) * tid;
    float* dbot = dtop + tmpf;
    float* dcol = dbot + tmpf;
    float* col = cols + colf * tid;
    conv_ws ws;
    conv_ws_bind(&ws, S, qws_f + wsf * n, qws_u + wsu * n);
    const float* dpool = dpool3 + (size_t)n * k4;
    int H = S / 4;
    for (int l = 2; l >= 0; --l) {
      const int HW = H * H, Hp = H / 2, K = CIN[l] * KS[l] * KS[l];
      /* un-pool to the argmax + ReLU mask -> dtop (Cout,H,H) */
      memset(dtop, 0, sizeof(float) * COUT[l] * HW);
      for (int c = 0; c < COUT[l]; ++c)
        for (int py = 0; py < Hp; ++py)
          for (int px = 0; px < Hp; ++px) {
            const size_t pi = ((size_t)c * Hp + py) * Hp + px;
            const int ar = ws.arg[l][pi];
            const size_t ai = (size_t)c * HW + (2 * py + (ar >> 1)) * H + 2 * px + (ar & 1);
            if (ws.act[l][ai] > 0.f) dtop[ai] = dpool[pi];
          }
      const float* bottom = l == 0 ? state + n * img : ws.pool[l - 1];
      im2col(bottom, CIN[l], H, H, KS[l], PAD[l], col);
      sgemm(0, 1, COUT[l], K, HW, dtop, HW, col, HW, g + L.w[l], K, 1);   /* dW += dtop col^T */
      for (int c = 0; c < COUT[l]; ++c) {
        float s = 0.f;
        for (int i = 0; i < HW; ++i) s += dtop[(size_t)c * HW + i];
        g[L.b[l] + c] += s;
      }
      if (l > 0) {
        sgemm(1, 0, K, HW, COUT[l], thQ + L.w[l], K, dtop, HW, dcol, HW, 0);   /* W^T dtop */
        col2im(dcol, CIN[l], H, H, KS[l], PAD[l], dbot);
        dpool = dbot;   /* consumed by the next un-pool before col2im rewrites it */
      }
      H *= 2;
    }
  }
#pragma omp parallel for schedule(static) num_threads(nth)
  for (long i = 0; i < conv_total; ++i) {
    float v = 0.f;
    for (int t = 0; t < nth; ++t) v += gpart[(size_t)t * conv_total + i];
    grad[i] = v;
  }
  if (blobs) {
    memcpy(blobs, qout, sizeof(float) * B * NA);
    memcpy(blobs + B * NA, pout, sizeof(float) * B * NA);
    blobs[2 * B * NA + 3 * B] = loss;
  }
  free(qws_f); free(qws_u); free(pws_f); free(pws_u); free(cols); free(pool3); free(h4);
  free(out); free(dq); free(dh4); free(dpool3); free(gpart); free(bwd);
  return 0;
}

/* FLOPs (2 x MACs) of one full_pass: both towers' forward + the Q backward
 * (weight and data gradients; conv1 has no data gradient). */
double ddq_cpu_step_flops(int B, int S) {
  const double s2 = S / 2, s3 = S / 4, s4 = S / 8, k4 = 64 * s4 * s4;
  const double c1 = 2.0 * B * S * S * 32 * 196, c2 = 2.0 * B * s2 * s2 * 64 * 800;
  const double c3 = 2.0 * B * s3 * s3 * 64 * 576, fc = 2.0 * B * 512 * k4;
  return 2 * (c1 + c2 + c3 + fc) + (c1 + 2 * c2 + 2 * c3 + 2 * fc);
}

/* server.py rules on flat buffers; first != 0 on the first call after reset. */
int ddq_cpu_apply(int rule, long n, float* theta, const float* g, float* state, int first,
                  float lr, float decay, float eps) {
  const float omd = (float)(1.0 - (double)decay);
  for (long i = 0; i < n; ++i) {
    const float gi = g[i];
    if (rule == 0) {
      theta[i] = theta[i] - lr * gi;
    } else if (rule == 1) {
      const float g2 = gi * gi;
      const float cu = first ? g2 : state[i];
      state[i] = first ? g2 : decay * state[i] + omd * g2;
      theta[i] = theta[i] - (lr * gi) / sqrtf(cu + eps);
    } else if (rule == 2) {
      const float acc = first ? gi * gi : state[i] + gi * gi;
      state[i] = acc;
      theta[i] = theta[i] - (lr * gi) / sqrtf(acc + eps);
    } else {
      return -1;
    }
  }
  return 0;
}

/* sample_direct gather (replay.py:159-183) for a sorted index list. */
int ddq_cpu_gather(int B, int S, long N, const unsigned char* st, const unsigned char* act,
                   const short* rew, const unsigned char* nt, const int* idx, float* state,
                   float* action, float* reward, float* next_state, float* nonterm) {
  const size_t img = (size_t)4 * S * S;
  for (int b = 0; b < B; ++b) {
    const long i = idx[b], nx = (i + 1 == N) ? 0 : i + 1;
    for (size_t p = 0; p < img; ++p) {
      state[b * img + p] = st[i * img + p];
      next_state[b * img + p] = st[nx * img + p];
    }
    for (int a = 0; a < NA; ++a) action[b * NA + a] = (a == act[nx]) ? 1.f : 0.f;
    reward[b] = rew[nx];
    nonterm[b] = nt[nx] ? 1.f : 0.f;
  }
  return 0;
}
