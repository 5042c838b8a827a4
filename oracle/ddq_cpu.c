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
 * Parallelism: OpenMP over images (the batch) -- the Caffe CPU path is
 * single-threaded BLAS per image; `threads` selects the cores used.
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

/* C[M x N] (+)= A[M x K] * B[K x N], row-major, optional transposes. */
static void sgemm(int ta, int tb, int M, int N, int K, const float* A, const float* B, float* C,
                  int accumulate) {
  if (!accumulate) memset(C, 0, sizeof(float) * (size_t)M * N);
  for (int m = 0; m < M; ++m) {
    float* c = C + (size_t)m * N;
    for (int k = 0; k < K; ++k) {
      const float a = ta ? A[(size_t)k * M + m] : A[(size_t)m * K + k];
      if (a == 0.f) continue;
      if (!tb) {
        const float* b = B + (size_t)k * N;
        for (int n = 0; n < N; ++n) c[n] += a * b[n];
      } else {
        for (int n = 0; n < N; ++n) c[n] += a * B[(size_t)n * K + k];
      }
    }
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

/* One tower forward for one image.  act[l]: post-ReLU conv output (Cout,H,W),
 * pool[l]: pooled (Cout,H/2,W/2), arg[l]: argmax 0..3. */
typedef struct {
  float* act[3];
  float* pool[3];
  unsigned char* arg[3];
  float* h4;
  float* out;
  float* col;
} tower_ws;

static void tower_fwd(const layout_t* L, const float* th, const float* x, tower_ws* ws) {
  const float* in = x;
  int H = L->S;
  for (int l = 0; l < 3; ++l) {
    const int K = CIN[l] * KS[l] * KS[l], HW = H * H;
    im2col(in, CIN[l], H, H, KS[l], PAD[l], ws->col);
    sgemm(0, 0, COUT[l], HW, K, th + L->w[l], ws->col, ws->act[l], 0);
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
  const int k4 = 64 * H * H;
  for (int n = 0; n < FC4; ++n) {
    const float* w = th + L->w[3] + (size_t)n * k4;
    float acc = 0.f;
    for (int k = 0; k < k4; ++k) acc += w[k] * in[k];
    acc += th[L->b[3] + n];
    ws->h4[n] = acc > 0.f ? acc : 0.f;
  }
  for (int a = 0; a < NA; ++a) {
    const float* w = th + L->w[4] + (size_t)a * FC4;
    float acc = 0.f;
    for (int k = 0; k < FC4; ++k) acc += w[k] * ws->h4[k];
    ws->out[a] = acc + th[L->b[4] + a];
  }
}

static int ws_alloc(const layout_t* L, tower_ws* ws) {
  int H = L->S;
  size_t colmax = 0;
  for (int l = 0; l < 3; ++l) {
    const size_t HW = (size_t)H * H;
    ws->act[l] = (float*)malloc(sizeof(float) * COUT[l] * HW);
    ws->pool[l] = (float*)malloc(sizeof(float) * COUT[l] * HW / 4);
    ws->arg[l] = (unsigned char*)malloc(COUT[l] * HW / 4);
    const size_t c = (size_t)CIN[l] * KS[l] * KS[l] * HW;
    if (c > colmax) colmax = c;
    H /= 2;
  }
  ws->h4 = (float*)malloc(sizeof(float) * FC4);
  ws->out = (float*)malloc(sizeof(float) * NA);
  ws->col = (float*)malloc(sizeof(float) * colmax);
  return ws->col ? 0 : -2;
}

static void ws_free(tower_ws* ws) {
  for (int l = 0; l < 3; ++l) { free(ws->act[l]); free(ws->pool[l]); free(ws->arg[l]); }
  free(ws->h4); free(ws->out); free(ws->col);
}

/*
 * BaristaNet.full_pass (baristanet.py:138-140): forward both towers, target,
 * loss, Q backward.  Inputs in Caffe shapes.  blobs: Q_out[B*4], P_out[B*4],
 * Q_sa[B], P_sa[B], target[B], loss[1] (may be NULL).  grad: P floats.
 */
int ddq_cpu_full_pass(int B, int S, const float* thQ, const float* thP, const float* state,
                      const float* action, const float* reward, const float* next_state,
                      const float* nonterm, float gamma, float* grad, float* blobs, int threads) {
  if (S % 8 || B < 1) return -1;
  const layout_t L = mk_layout(S);
  const size_t img = (size_t)4 * S * S;
  float* qout = (float*)malloc(sizeof(float) * B * NA);
  float* pout = (float*)malloc(sizeof(float) * B * NA);
  float* qsa = (float*)malloc(sizeof(float) * B);
  float* psa = (float*)malloc(sizeof(float) * B);
  float* tgt = (float*)malloc(sizeof(float) * B);
  float* dq = (float*)malloc(sizeof(float) * B * NA);
  int nth = threads > 0 ? threads : 1;
#ifdef _OPENMP
  omp_set_num_threads(nth);
#else
  nth = 1;
#endif
  float* gpart = (float*)calloc((size_t)nth * L.total, sizeof(float));
  if (!qout || !pout || !gpart) return -2;

  /* forward P tower (all images) */
#pragma omp parallel
  {
    tower_ws ws;
    ws_alloc(&L, &ws);
#pragma omp for schedule(static)
    for (int n = 0; n < B; ++n) {
      tower_fwd(&L, thP, next_state + n * img, &ws);
      memcpy(pout + n * NA, ws.out, sizeof(float) * NA);
    }
    ws_free(&ws);
  }
  /* Q tower forward + per-image backward (needs the loss scale 1/B only) */
  float loss = 0.f;
  /* first pass: Q forward outputs for Q_sa / target (cheap to recompute) */
#pragma omp parallel
  {
    tower_ws ws;
    ws_alloc(&L, &ws);
#pragma omp for schedule(static)
    for (int n = 0; n < B; ++n) {
      tower_fwd(&L, thQ, state + n * img, &ws);
      memcpy(qout + n * NA, ws.out, sizeof(float) * NA);
    }
    ws_free(&ws);
  }
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
    qsa[n] = s; psa[n] = mx; tgt[n] = t;
    const float d = s - t;
    loss += d * d;
    for (int k = 0; k < NA; ++k) dq[n * NA + k] = a[k] * d / (float)B;
  }
  loss = loss / (float)B / 2.f;

#pragma omp parallel
  {
    int tid = 0;
#ifdef _OPENMP
    tid = omp_get_thread_num();
#endif
    float* g = gpart + (size_t)tid * L.total;
    tower_ws ws;
    ws_alloc(&L, &ws);
    int H1 = S;
    size_t maxact = (size_t)32 * S * S;
    float* dtop = (float*)malloc(sizeof(float) * maxact);
    float* dbot = (float*)malloc(sizeof(float) * maxact);
    float* dcol = (float*)malloc(sizeof(float) * (size_t)64 * 25 * (S / 2) * (S / 2));
    float* dh4 = (float*)malloc(sizeof(float) * FC4);
    (void)H1;
#pragma omp for schedule(static)
    for (int n = 0; n < B; ++n) {
      tower_fwd(&L, thQ, state + n * img, &ws);
      const float* d = dq + n * NA;
      /* Q_out: W5 diff += dQ^T h4, b5 diff += dQ, dh4 = dQ W5 * (h4 > 0) */
      for (int a = 0; a < NA; ++a) {
        for (int k = 0; k < FC4; ++k) g[L.w[4] + a * FC4 + k] += d[a] * ws.h4[k];
        g[L.b[4] + a] += d[a];
      }
      for (int k = 0; k < FC4; ++k) {
        float v = 0.f;
        for (int a = 0; a < NA; ++a) v += d[a] * thQ[L.w[4] + a * FC4 + k];
        dh4[k] = ws.h4[k] > 0.f ? v : 0.f;
      }
      const int s4 = S / 8, k4 = 64 * s4 * s4;
      for (int o = 0; o < FC4; ++o) {
        const float v = dh4[o];
        if (v == 0.f) continue;
        float* gw = g + L.w[3] + (size_t)o * k4;
        for (int k = 0; k < k4; ++k) gw[k] += v * ws.pool[2][k];
        g[L.b[3] + o] += v;
      }
      /* dpool3 = dh4 W4 */
      float* dpool = dbot;
      memset(dpool, 0, sizeof(float) * k4);
      for (int o = 0; o < FC4; ++o) {
        const float v = dh4[o];
        if (v == 0.f) continue;
        const float* w = thQ + L.w[3] + (size_t)o * k4;
        for (int k = 0; k < k4; ++k) dpool[k] += v * w[k];
      }
      int H = S / 4;
      for (int l = 2; l >= 0; --l) {
        const int HW = H * H, Hp = H / 2, K = CIN[l] * KS[l] * KS[l];
        /* un-pool + ReLU mask -> dtop (Cout,H,H) */
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
        im2col(bottom, CIN[l], H, H, KS[l], PAD[l], ws.col);
        sgemm(0, 1, COUT[l], K, HW, dtop, ws.col, g + L.w[l], 1);
        for (int c = 0; c < COUT[l]; ++c) {
          float s = 0.f;
          for (int i = 0; i < HW; ++i) s += dtop[(size_t)c * HW + i];
          g[L.b[l] + c] += s;
        }
        if (l > 0) {
          sgemm(1, 0, K, HW, COUT[l], thQ + L.w[l], dtop, dcol, 0);
          col2im(dcol, CIN[l], H, H, KS[l], PAD[l], dbot);
          dpool = dbot;
        }
        H *= 2;
      }
    }
    free(dtop); free(dbot); free(dcol); free(dh4);
    ws_free(&ws);
  }
  memset(grad, 0, sizeof(float) * L.total);
  for (int t = 0; t < nth; ++t)
    for (long i = 0; i < L.total; ++i) grad[i] += gpart[(size_t)t * L.total + i];
  if (blobs) {
    memcpy(blobs, qout, sizeof(float) * B * NA);
    memcpy(blobs + B * NA, pout, sizeof(float) * B * NA);
    memcpy(blobs + 2 * B * NA, qsa, sizeof(float) * B);
    memcpy(blobs + 2 * B * NA + B, psa, sizeof(float) * B);
    memcpy(blobs + 2 * B * NA + 2 * B, tgt, sizeof(float) * B);
    blobs[2 * B * NA + 3 * B] = loss;
  }
  free(qout); free(pout); free(qsa); free(psa); free(tgt); free(dq); free(gpart);
  return 0;
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
