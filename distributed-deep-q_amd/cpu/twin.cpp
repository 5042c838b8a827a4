// libddq_cpu.so -- the CPU-mode twin of libddq_hip.so (include/ddq_hip.h).
//
// The reference runs its Barista worker in Caffe CPU mode when asked
// (`--mode cpu`, main.py:128,149-151; BASELINE.json configs[0]: "Caffe CPU
// mode, single Barista worker driven by barista.dummy_client (plumbing, no
// GPU)").  This library exports every ddq_* symbol of the C-ABI so the same
// host layer (ddq.DeepQNet(mode="cpu"), the Barista worker, the param server)
// runs on a machine without a GPU.  It computes what the HIP library computes
// -- the deepq network of models/deepq/train_val.prototxt:38-483 (both
// towers, Q(s,a), the Bellman target 0.85 max_a P + r, the Euclidean loss, the
// Q backward), the replay ring of replay.py and the param-server update rules
// of server.py:49-124 -- with plain C++ loops over NCHW fp32 tensors,
// accumulating every dot product in double and rounding once per layer
// output (so it is no less exact than the GPU's fp32-exact split products).
// The update rules round exactly as the HIP library's apply_rule (built with
// -ffp-contract=off): the same fp32 operations in the same order.
//
// What needs a GPU stream or a communicator (device index draws, large-batch
// gathers, hipGraph steps, RCCL exchanges, in-process groups, the async param
// server, kernel timing) returns DDQ_ESTATE ("CPU mode") -- the reference's
// CPU mode has none of those either.
#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/ddq_hip.h"

namespace {

thread_local std::string g_err;

constexpr int kA = 4;          // actions (barista/constants.py:8)
constexpr int kC = 4;          // frames per state (expgain.py:9)
constexpr int kH4 = 512;       // fc4 units (train_val.prototxt:165)

struct Layout {
  int S;
  int64_t w[5], b[5], wn[5], bn[5], total;
};

Layout make_layout(int S) {
  Layout L{};
  L.S = S;
  const int64_t s4 = S / 8;
  const int64_t wn[5] = {32ll * 4 * 49, 64ll * 32 * 25, 64ll * 64 * 9, kH4 * 64 * s4 * s4, kA * kH4};
  const int64_t bn[5] = {32, 64, 64, kH4, kA};
  int64_t o = 0;
  for (int i = 0; i < 5; ++i) {
    L.w[i] = o; L.wn[i] = wn[i]; o += wn[i];
    L.b[i] = o; L.bn[i] = bn[i]; o += bn[i];
  }
  L.total = o;
  return L;
}

// conv layer geometry: (cin, cout, k, pad) of train_val.prototxt:39-158
struct Conv { int cin, cout, k, pad; };
constexpr Conv kConv[3] = {{4, 32, 7, 3}, {32, 64, 5, 2}, {64, 64, 3, 1}};

// One tower's activations for a batch (NCHW fp32).
struct Tower {
  std::vector<float> x[3];       // input of conv l (x[0]: the frames)
  std::vector<uint8_t> route[3]; // pool l routing: 0..3 first max in window order, 4: ReLU'd
  std::vector<float> pool3;      // (B, 64, S/8, S/8) = fc4's input, Caffe flatten order
  std::vector<float> h4, out;    // (B, 512), (B, 4)
};

}  // namespace

struct ddq_ctx {
  int B = 0, S = 0;
  float gamma = 0.85f;
  Layout L{};
  std::vector<float> theta[2], grad, opt;
  int first = 1;                 // the next apply is the first since a reset
  int64_t iter = 0;
  // minibatch (Caffe shapes)
  std::vector<float> state, next_state, action, reward, nonterm;
  std::vector<int32_t> idx;
  // blobs of the last forward
  std::vector<float> q_out, p_out, q_sa, p_sa, target;
  float loss = 0.f;
  Tower tw[2];
  // replay ring (replay.py:23-68)
  std::vector<uint8_t> r_state, r_action, r_nonterm;
  std::vector<int16_t> r_reward;
  int64_t head = 0, valid = 0, capacity = 0;
  int64_t steps = 0;
  std::string err;
};

namespace {

int fail(ddq_ctx* c, int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  if (c) c->err = buf;
  g_err = buf;
  return code;
}

int cpu_only(ddq_ctx* c, const char* what) {
  return fail(c, DDQ_ESTATE, "%s: not available in CPU mode (libddq_cpu.so); use libddq_hip.so",
              what);
}

// ---- forward ----
// out[b][co][y][x] = bias[co] + sum_{ci,ky,kx} W[co][ci][ky][kx] in[b][ci][y+ky-p][x+kx-p]
void conv_fwd(const float* in, int B, int H, const Conv& cv, const float* W, const float* bias,
              float* out) {
  const int k = cv.k, p = cv.pad, HW = H * H;
#pragma omp parallel for collapse(2) schedule(static)
  for (int b = 0; b < B; ++b)
    for (int co = 0; co < cv.cout; ++co) {
      std::vector<double> acc(HW, (double)bias[co]);
      for (int ci = 0; ci < cv.cin; ++ci) {
        const float* src = in + ((size_t)b * cv.cin + ci) * HW;
        const float* w = W + ((size_t)co * cv.cin + ci) * k * k;
        for (int ky = 0; ky < k; ++ky)
          for (int kx = 0; kx < k; ++kx) {
            const double wv = w[ky * k + kx];
            const int y0 = std::max(0, p - ky), y1 = std::min(H, H + p - ky);
            const int x0 = std::max(0, p - kx), x1 = std::min(H, H + p - kx);
            for (int y = y0; y < y1; ++y) {
              const float* row = src + (y + ky - p) * H + (kx - p);
              double* a = acc.data() + y * H;
              for (int x = x0; x < x1; ++x) a[x] += wv * row[x];
            }
          }
      }
      float* dst = out + ((size_t)b * cv.cout + co) * HW;
      for (int i = 0; i < HW; ++i) dst[i] = (float)acc[i];
    }
}

// ReLU (in place, train_val.prototxt RELU layers) + 2x2 / 2 max pool with the
// first maximum of the window in (0,0) (0,1) (1,0) (1,1) order; route 4 when
// the window's maximum is not positive (no gradient passes the ReLU there)
void relu_pool(const float* pre, int B, int C, int H, float* out, uint8_t* route) {
  const int Ho = H / 2;
#pragma omp parallel for collapse(2) schedule(static)
  for (int b = 0; b < B; ++b)
    for (int c = 0; c < C; ++c) {
      const float* s = pre + ((size_t)b * C + c) * H * H;
      for (int y = 0; y < Ho; ++y)
        for (int x = 0; x < Ho; ++x) {
          const float v[4] = {s[(2 * y) * H + 2 * x], s[(2 * y) * H + 2 * x + 1],
                              s[(2 * y + 1) * H + 2 * x], s[(2 * y + 1) * H + 2 * x + 1]};
          int arg = 0;
          float mx = v[0];
          for (int q = 1; q < 4; ++q)
            if (v[q] > mx) { mx = v[q]; arg = q; }
          const size_t o = (((size_t)b * C + c) * Ho + y) * Ho + x;
          out[o] = mx > 0.f ? mx : 0.f;
          route[o] = (uint8_t)(mx > 0.f ? arg : 4);
        }
    }
}

// y[b][n] = bias[n] + sum_k W[n][k] x[b][k]
void dense(const float* x, int B, int K, int N, const float* W, const float* bias, float* y,
           bool relu) {
#pragma omp parallel for collapse(2) schedule(static)
  for (int b = 0; b < B; ++b)
    for (int n = 0; n < N; ++n) {
      double a = bias[n];
      const float* w = W + (size_t)n * K;
      const float* xb = x + (size_t)b * K;
      for (int k = 0; k < K; ++k) a += (double)w[k] * xb[k];
      const float v = (float)a;
      y[(size_t)b * N + n] = relu ? (v > 0.f ? v : 0.f) : v;
    }
}

void tower_fwd(ddq_ctx* c, int z, const float* frames, int B) {
  const Layout& L = c->L;
  const float* th = c->theta[z].data();
  Tower& t = c->tw[z];
  int H = c->S;
  t.x[0].assign(frames, frames + (size_t)B * kC * H * H);
  std::vector<float> pre;
  for (int l = 0; l < 3; ++l) {
    const Conv& cv = kConv[l];
    pre.assign((size_t)B * cv.cout * H * H, 0.f);
    conv_fwd(t.x[l].data(), B, H, cv, th + L.w[l], th + L.b[l], pre.data());
    const size_t np = (size_t)B * cv.cout * (H / 2) * (H / 2);
    std::vector<float>& nxt = l < 2 ? t.x[l + 1] : t.pool3;
    nxt.assign(np, 0.f);
    t.route[l].assign(np, 4);
    relu_pool(pre.data(), B, cv.cout, H, nxt.data(), t.route[l].data());
    H /= 2;
  }
  const int K4 = 64 * H * H;
  t.h4.assign((size_t)B * kH4, 0.f);
  dense(t.pool3.data(), B, K4, kH4, th + L.w[3], th + L.b[3], t.h4.data(), true);
  t.out.assign((size_t)B * kA, 0.f);
  dense(t.h4.data(), B, kH4, kA, th + L.w[4], th + L.b[4], t.out.data(), false);
}

// ---- backward (Q tower) ----
// gW[co][ci][ky][kx] = sum_{b,y,x} d[b][co][y][x] in[b][ci][y+ky-p][x+kx-p]; gb[co] = sum d.
// Per (co, ci) the products accumulate elementwise into one double row per
// tap ([tap][x]: independent lanes, so the inner loop vectorises), summed
// over x at the end.
void conv_wgrad(const float* in, const float* d, int B, int H, const Conv& cv, float* gW,
                float* gb) {
  const int k = cv.k, p = cv.pad, HW = H * H;
#pragma omp parallel for collapse(2) schedule(dynamic)
  for (int co = 0; co < cv.cout; ++co)
    for (int ci = 0; ci < cv.cin; ++ci) {
      std::vector<double> acc((size_t)k * k * H, 0.0);
      for (int b = 0; b < B; ++b) {
        const float* src = in + ((size_t)b * cv.cin + ci) * HW;
        const float* dd = d + ((size_t)b * cv.cout + co) * HW;
        for (int ky = 0; ky < k; ++ky)
          for (int kx = 0; kx < k; ++kx) {
            const int y0 = std::max(0, p - ky), y1 = std::min(H, H + p - ky);
            const int x0 = std::max(0, p - kx), x1 = std::min(H, H + p - kx);
            double* a = acc.data() + (size_t)(ky * k + kx) * H;
            for (int y = y0; y < y1; ++y) {
              const float* row = src + (y + ky - p) * H + (kx - p);
              const float* dr = dd + y * H;
              for (int x = x0; x < x1; ++x) a[x] += (double)dr[x] * row[x];
            }
          }
      }
      float* g = gW + ((size_t)co * cv.cin + ci) * k * k;
      for (int t = 0; t < k * k; ++t) {
        double v = 0.0;
        for (int x = 0; x < H; ++x) v += acc[(size_t)t * H + x];
        g[t] = (float)v;
      }
    }
#pragma omp parallel for schedule(static)
  for (int co = 0; co < cv.cout; ++co) {
    double a = 0.0;
    for (int b = 0; b < B; ++b) {
      const float* dd = d + ((size_t)b * cv.cout + co) * HW;
      for (int i = 0; i < HW; ++i) a += dd[i];
    }
    gb[co] = (float)a;
  }
}

// dx[b][ci][iy][ix] = sum_{co,ky,kx} d[b][co][iy-ky+p][ix-kx+p] W[co][ci][ky][kx]
void conv_dgrad(const float* d, int B, int H, const Conv& cv, const float* W, float* dx) {
  const int k = cv.k, p = cv.pad, HW = H * H;
#pragma omp parallel for collapse(2) schedule(static)
  for (int b = 0; b < B; ++b)
    for (int ci = 0; ci < cv.cin; ++ci) {
      std::vector<double> acc(HW, 0.0);
      for (int co = 0; co < cv.cout; ++co) {
        const float* dd = d + ((size_t)b * cv.cout + co) * HW;
        const float* w = W + ((size_t)co * cv.cin + ci) * k * k;
        for (int ky = 0; ky < k; ++ky)
          for (int kx = 0; kx < k; ++kx) {
            const double wv = w[ky * k + kx];
            // input pixel iy receives output pixel y = iy - ky + p
            const int iy0 = std::max(0, ky - p), iy1 = std::min(H, H + ky - p);
            const int ix0 = std::max(0, kx - p), ix1 = std::min(H, H + kx - p);
            for (int iy = iy0; iy < iy1; ++iy) {
              const float* row = dd + (iy - ky + p) * H + (p - kx);
              double* a = acc.data() + iy * H;
              for (int ix = ix0; ix < ix1; ++ix) a[ix] += wv * row[ix];
            }
          }
      }
      float* dst = dx + ((size_t)b * cv.cin + ci) * HW;
      for (int i = 0; i < HW; ++i) dst[i] = (float)acc[i];
    }
}

// the pooled gradient routed to its window's first maximum (0 elsewhere and
// for ReLU'd windows): the pre-activation gradient of the conv below
void unpool(const float* dpool, const uint8_t* route, int B, int C, int Ho, float* dpre) {
  const int H = 2 * Ho;
  std::fill(dpre, dpre + (size_t)B * C * H * H, 0.f);
#pragma omp parallel for collapse(2) schedule(static)
  for (int b = 0; b < B; ++b)
    for (int c = 0; c < C; ++c)
      for (int y = 0; y < Ho; ++y)
        for (int x = 0; x < Ho; ++x) {
          const size_t o = (((size_t)b * C + c) * Ho + y) * Ho + x;
          const int r = route[o];
          if (r < 4)
            dpre[(((size_t)b * C + c) * H + 2 * y + (r >> 1)) * H + 2 * x + (r & 1)] = dpool[o];
        }
}

int forward_backward(ddq_ctx* c) {
  const int B = c->B, S = c->S;
  const Layout& L = c->L;
  tower_fwd(c, 0, c->state.data(), B);
  tower_fwd(c, 1, c->next_state.data(), B);
  const Tower& q = c->tw[0];
  const Tower& p = c->tw[1];
  c->q_out = q.out;
  c->p_out = p.out;
  c->q_sa.assign(B, 0.f); c->p_sa.assign(B, 0.f); c->target.assign(B, 0.f);
  // head: ELTWISE PROD + SLICE + SUM (Q(s,a)), SLICE + MAX * non_terminal (max_a
  // P), SUM with coefficients (gamma, 1), EUCLIDEAN_LOSS (train_val.prototxt:385-483)
  std::vector<double> dq((size_t)B * kA, 0.0);
  double loss = 0.0;
  for (int b = 0; b < B; ++b) {
    double qs = 0.0, pm = p.out[(size_t)b * kA];
    for (int a = 0; a < kA; ++a) {
      qs += (double)q.out[(size_t)b * kA + a] * c->action[(size_t)b * kA + a];
      pm = std::max(pm, (double)p.out[(size_t)b * kA + a]);
    }
    const float qsf = (float)qs;
    const float psf = (float)(pm * c->nonterm[b]);
    const float tg = (float)((double)c->gamma * psf + 1.0 * c->reward[b]);
    c->q_sa[b] = qsf; c->p_sa[b] = psf; c->target[b] = tg;
    const double diff = (double)qsf - tg;
    loss += diff * diff;
    for (int a = 0; a < kA; ++a) dq[(size_t)b * kA + a] = c->action[(size_t)b * kA + a] * diff / B;
  }
  c->loss = (float)(loss / B / 2.0);
  float* g = c->grad.data();
  const float* th = c->theta[0].data();
  const int s4 = S / 8, K4 = 64 * s4 * s4;
  // Q_out (IP 512 -> 4)
  for (int a = 0; a < kA; ++a) {
    double gb = 0.0;
    for (int b = 0; b < B; ++b) gb += dq[(size_t)b * kA + a];
    g[L.b[4] + a] = (float)gb;
    for (int n = 0; n < kH4; ++n) {
      double gw = 0.0;
      for (int b = 0; b < B; ++b) gw += dq[(size_t)b * kA + a] * q.h4[(size_t)b * kH4 + n];
      g[L.w[4] + (size_t)a * kH4 + n] = (float)gw;
    }
  }
  // dh4 = (dQ W5) masked by the ReLU
  std::vector<float> dh4((size_t)B * kH4, 0.f);
  for (int b = 0; b < B; ++b)
    for (int n = 0; n < kH4; ++n) {
      if (!(q.h4[(size_t)b * kH4 + n] > 0.f)) continue;
      double v = 0.0;
      for (int a = 0; a < kA; ++a) v += dq[(size_t)b * kA + a] * th[L.w[4] + (size_t)a * kH4 + n];
      dh4[(size_t)b * kH4 + n] = (float)v;
    }
  // fc4 (IP K4 -> 512)
#pragma omp parallel for schedule(static)
  for (int n = 0; n < kH4; ++n) {
    double gb = 0.0;
    for (int b = 0; b < B; ++b) gb += dh4[(size_t)b * kH4 + n];
    g[L.b[3] + n] = (float)gb;
    for (int k = 0; k < K4; ++k) {
      double gw = 0.0;
      for (int b = 0; b < B; ++b) gw += (double)dh4[(size_t)b * kH4 + n] * q.pool3[(size_t)b * K4 + k];
      g[L.w[3] + (size_t)n * K4 + k] = (float)gw;
    }
  }
  std::vector<float> dpool((size_t)B * K4, 0.f);
#pragma omp parallel for collapse(2) schedule(static)
  for (int b = 0; b < B; ++b)
    for (int k = 0; k < K4; ++k) {
      double v = 0.0;
      for (int n = 0; n < kH4; ++n)
        v += (double)dh4[(size_t)b * kH4 + n] * th[L.w[3] + (size_t)n * K4 + k];
      dpool[(size_t)b * K4 + k] = (float)v;
    }
  // conv3 -> conv1
  std::vector<float> dpre, dx;
  int Ho = s4;
  for (int l = 2; l >= 0; --l) {
    const Conv& cv = kConv[l];
    const int H = 2 * Ho;
    dpre.assign((size_t)B * cv.cout * H * H, 0.f);
    unpool(dpool.data(), q.route[l].data(), B, cv.cout, Ho, dpre.data());
    conv_wgrad(q.x[l].data(), dpre.data(), B, H, cv, g + L.w[l], g + L.b[l]);
    if (l > 0) {
      dx.assign((size_t)B * cv.cin * H * H, 0.f);
      conv_dgrad(dpre.data(), B, H, cv, th + L.w[l], dx.data());
      dpool.swap(dx);
    }
    Ho = H;
  }
  return DDQ_OK;
}

// server.py:81-124 + Caffe SGDSolver momentum, the HIP library's apply_rule
// operation for operation (fp32, no contraction: -ffp-contract=off)
float apply_rule(const ddq_update_cfg& u, bool first, bool is_bias, float th, float g, float& st) {
  switch (u.rule) {
    case DDQ_RULE_SGD:
      return th - u.lr * g;
    case DDQ_RULE_RMSPROP: {
      const float g2 = g * g;
      const float c_use = first ? g2 : st;
      st = first ? g2 : (u.decay * st + (1.0f - u.decay) * g2);
      return th - (u.lr * g) / sqrtf(c_use + u.eps);
    }
    case DDQ_RULE_ADAGRAD: {
      const float acc = first ? g * g : st + g * g;
      st = acc;
      return th - (u.lr * g) / sqrtf(acc + u.eps);
    }
    default: {
      const float lr = u.lr * (is_bias ? 2.f : 1.f);
      const float wd = is_bias ? 0.f : u.weight_decay;
      const float v = u.momentum * (first ? 0.f : st) + lr * (g + wd * th);
      st = v;
      return th - v;
    }
  }
}

void gather(ddq_ctx* c) {
  const int B = c->B, SS = c->S * c->S;
  const size_t slot = (size_t)kC * SS;
  for (int b = 0; b < B; ++b) {
    const int64_t i = c->idx[b];
    const int64_t nxt = i + 1 == c->capacity ? 0 : i + 1;   // replay.py:159-183
    for (size_t e = 0; e < slot; ++e) {
      c->state[(size_t)b * slot + e] = c->r_state[(size_t)i * slot + e];
      c->next_state[(size_t)b * slot + e] = c->r_state[(size_t)nxt * slot + e];
    }
    const int a = c->r_action[nxt];
    for (int k = 0; k < kA; ++k) c->action[(size_t)b * kA + k] = k == a ? 1.f : 0.f;
    c->reward[b] = (float)c->r_reward[nxt];
    c->nonterm[b] = c->r_nonterm[nxt] ? 1.f : 0.f;
  }
}

}  // namespace

extern "C" {

int ddq_abi_version(void) { return DDQ_ABI_VERSION; }

const char* ddq_last_error(const ddq_ctx* c) { return c ? c->err.c_str() : g_err.c_str(); }

int ddq_create(ddq_ctx** out, int device, const ddq_net_desc* d) {
  (void)device;
  if (!out || !d) return fail(nullptr, DDQ_EINVAL, "null argument");
  *out = nullptr;
  if (d->channels != 4 || d->actions != 4)
    return fail(nullptr, DDQ_EINVAL, "channels and actions must be 4 (got %d, %d)", d->channels,
                d->actions);
  if (d->frame < 16 || d->frame % 8 != 0 || d->frame > 1024)
    return fail(nullptr, DDQ_EINVAL, "frame side must be a multiple of 8 in [16,1024] (got %d)",
                d->frame);
  if (d->batch < 1 || d->batch > 1024)
    return fail(nullptr, DDQ_EINVAL, "batch must be in [1,1024] (got %d)", d->batch);
  ddq_ctx* c = new ddq_ctx();
  c->B = d->batch; c->S = d->frame; c->gamma = d->gamma;
  c->L = make_layout(c->S);
  const int64_t P = c->L.total;
  for (auto& t : c->theta) t.assign(P, 0.f);
  c->grad.assign(P, 0.f);
  c->opt.assign(P, 0.f);
  const size_t img = (size_t)c->B * kC * c->S * c->S;
  c->state.assign(img, 0.f); c->next_state.assign(img, 0.f);
  c->action.assign((size_t)c->B * kA, 0.f);
  c->reward.assign(c->B, 0.f); c->nonterm.assign(c->B, 0.f);
  c->idx.assign(c->B, 0);
  c->q_out.assign((size_t)c->B * kA, 0.f); c->p_out.assign((size_t)c->B * kA, 0.f);
  c->q_sa.assign(c->B, 0.f); c->p_sa.assign(c->B, 0.f); c->target.assign(c->B, 0.f);
  *out = c;
  return DDQ_OK;
}

int ddq_destroy(ddq_ctx* c) {
  delete c;
  return DDQ_OK;
}

int ddq_set_stream(ddq_ctx* c, void* s) {
  if (!c) return fail(nullptr, DDQ_EINVAL, "null ctx");
  return s ? cpu_only(c, "ddq_set_stream") : DDQ_OK;
}

int ddq_get_stream(const ddq_ctx* c, void** s) {
  if (!c || !s) return fail(nullptr, DDQ_EINVAL, "null argument");
  *s = nullptr;   // no stream: every call completes before it returns
  return DDQ_OK;
}

int ddq_synchronize(ddq_ctx* c) { return c ? DDQ_OK : fail(nullptr, DDQ_EINVAL, "null ctx"); }

int ddq_inject_fault(ddq_ctx* c, int32_t fault) {
  if (!c) return fail(nullptr, DDQ_EINVAL, "null ctx");
  return fault == DDQ_FAULT_NONE ? DDQ_OK
                                 : fail(c, DDQ_ESTATE, "no small-map step on this ctx (CPU mode)");
}

int ddq_small_path(const ddq_ctx* c, char* why, int32_t cap) {
  if (!c) return fail(nullptr, DDQ_EINVAL, "null ctx");
  if (why && cap > 0) snprintf(why, (size_t)cap, "%s", "CPU mode");
  return 0;
}

int64_t ddq_num_params(const ddq_ctx* c) { return c ? c->L.total : -1; }

int ddq_param_layout(const ddq_ctx* c, ddq_blob_desc* out, int32_t cap, int32_t* n) {
  if (!c || !n) return fail(nullptr, DDQ_EINVAL, "null argument");
  const char* names[5] = {"Qconv1", "Qconv2", "Qconv3", "Qfc4", "Q_out"};
  *n = 10;
  if (!out) return DDQ_OK;
  if (cap < 10) return fail(const_cast<ddq_ctx*>(c), DDQ_EINVAL, "layout needs 10 entries");
  const int s4 = c->S / 8;
  for (int l = 0; l < 5; ++l)
    for (int i = 0; i < 2; ++i) {
      ddq_blob_desc& d = out[2 * l + i];
      memset(&d, 0, sizeof(d));
      snprintf(d.name, sizeof(d.name), "%s", names[l]);
      d.index = i;
      if (i == 0) {
        if (l < 3) {
          d.shape[0] = kConv[l].cout; d.shape[1] = kConv[l].cin;
          d.shape[2] = d.shape[3] = kConv[l].k;
        } else {
          d.shape[0] = d.shape[1] = 1;
          d.shape[2] = l == 3 ? kH4 : kA;
          d.shape[3] = l == 3 ? 64 * s4 * s4 : kH4;
        }
        d.offset = c->L.w[l]; d.count = c->L.wn[l];
      } else {
        d.shape[0] = d.shape[1] = d.shape[2] = 1;
        d.shape[3] = (int)c->L.bn[l];
        d.offset = c->L.b[l]; d.count = c->L.bn[l];
      }
    }
  return DDQ_OK;
}

int ddq_set_params(ddq_ctx* c, int32_t which, const float* src, int64_t n, int32_t on_dev) {
  if (!c || !src) return fail(c, DDQ_EINVAL, "null argument");
  if (on_dev) return cpu_only(c, "device pointers");
  if (which != 0 && which != 1) return fail(c, DDQ_EINVAL, "which must be 0 (Q) or 1 (P)");
  if (n != c->L.total)
    return fail(c, DDQ_EINVAL, "expected %lld params, got %lld", (long long)c->L.total, (long long)n);
  std::copy(src, src + n, c->theta[which].begin());
  return DDQ_OK;
}

int ddq_get_params(ddq_ctx* c, int32_t which, float* dst, int64_t n, int32_t on_dev) {
  if (!c || !dst) return fail(c, DDQ_EINVAL, "null argument");
  if (on_dev) return cpu_only(c, "device pointers");
  if (which != 0 && which != 1) return fail(c, DDQ_EINVAL, "which must be 0 (Q) or 1 (P)");
  if (n != c->L.total) return fail(c, DDQ_EINVAL, "size mismatch");
  std::copy(c->theta[which].begin(), c->theta[which].end(), dst);
  return DDQ_OK;
}

int ddq_get_grads(ddq_ctx* c, float* dst, int64_t n, int32_t on_dev) {
  if (!c || !dst) return fail(c, DDQ_EINVAL, "null argument");
  if (on_dev) return cpu_only(c, "device pointers");
  if (n != c->L.total) return fail(c, DDQ_EINVAL, "size mismatch");
  std::copy(c->grad.begin(), c->grad.end(), dst);
  return DDQ_OK;
}

int ddq_set_grads(ddq_ctx* c, const float* src, int64_t n, int32_t on_dev) {
  if (!c || !src) return fail(c, DDQ_EINVAL, "null argument");
  if (on_dev) return cpu_only(c, "device pointers");
  if (n != c->L.total) return fail(c, DDQ_EINVAL, "size mismatch");
  std::copy(src, src + n, c->grad.begin());
  return DDQ_OK;
}

int ddq_sync_target(ddq_ctx* c) {
  if (!c) return fail(nullptr, DDQ_EINVAL, "null ctx");
  c->theta[1] = c->theta[0];
  return DDQ_OK;
}

// ---- replay (replay.py) ----
int ddq_replay_create(ddq_ctx* c, int64_t capacity) {
  if (!c) return fail(nullptr, DDQ_EINVAL, "null ctx");
  if (capacity < 2 || capacity > (int64_t)INT32_MAX)
    return fail(c, DDQ_EINVAL, "capacity must be in [2, 2^31) (got %lld)", (long long)capacity);
  if (c->capacity) return fail(c, DDQ_ESTATE, "replay already created");
  c->r_state.assign((size_t)capacity * kC * c->S * c->S, 0);
  c->r_action.assign(capacity, 0);
  c->r_reward.assign(capacity, 0);
  c->r_nonterm.assign(capacity, 0);
  c->capacity = capacity;
  c->head = c->valid = 0;
  return DDQ_OK;
}

int ddq_replay_add(ddq_ctx* c, int32_t action, int32_t reward, const uint8_t* state) {
  if (!c) return fail(nullptr, DDQ_EINVAL, "null ctx");
  if (!c->capacity) return fail(c, DDQ_ESTATE, "no replay buffer (call ddq_replay_create)");
  if (action < 0 || action > 255) return fail(c, DDQ_EINVAL, "action must fit uint8");
  if (reward < -32768 || reward > 32767) return fail(c, DDQ_EINVAL, "reward must fit int16");
  const size_t slot = (size_t)kC * c->S * c->S;
  const int64_t h = c->head;
  c->r_action[h] = (uint8_t)action;
  c->r_reward[h] = (int16_t)reward;
  c->r_nonterm[h] = state ? 1 : 0;   // a terminal transition keeps the slot's old frames
  if (state) std::copy(state, state + slot, c->r_state.begin() + h * slot);
  c->head = (c->head + 1) % c->capacity;
  c->valid = std::min(c->capacity, c->valid + 1);
  return DDQ_OK;
}

int ddq_replay_info(const ddq_ctx* c, int64_t* head, int64_t* valid, int64_t* capacity) {
  if (!c) return fail(nullptr, DDQ_EINVAL, "null ctx");
  if (head) *head = c->head;
  if (valid) *valid = c->valid;
  if (capacity) *capacity = c->capacity;
  return DDQ_OK;
}

int ddq_replay_import(ddq_ctx* c, const uint8_t* state, const uint8_t* action,
                      const int16_t* reward, const uint8_t* nonterm, int64_t n, int64_t head,
                      int64_t valid) {
  if (!c || !state || !action || !reward || !nonterm) return fail(c, DDQ_EINVAL, "null argument");
  if (!c->capacity) return fail(c, DDQ_ESTATE, "no replay buffer");
  if (n != c->capacity)
    return fail(c, DDQ_EINVAL, "import size %lld != capacity %lld", (long long)n,
                (long long)c->capacity);
  if (head < 0 || head >= n || valid < 0 || valid > n)
    return fail(c, DDQ_EINVAL, "head/valid out of range");
  const size_t slot = (size_t)kC * c->S * c->S;
  std::copy(state, state + slot * n, c->r_state.begin());
  std::copy(action, action + n, c->r_action.begin());
  std::copy(reward, reward + n, c->r_reward.begin());
  std::copy(nonterm, nonterm + n, c->r_nonterm.begin());
  c->head = head;
  c->valid = valid;
  return DDQ_OK;
}

int ddq_replay_export(ddq_ctx* c, uint8_t* state, uint8_t* action, int16_t* reward,
                      uint8_t* nonterm, int64_t n) {
  if (!c) return fail(nullptr, DDQ_EINVAL, "null ctx");
  if (!c->capacity) return fail(c, DDQ_ESTATE, "no replay buffer");
  if (n != c->capacity) return fail(c, DDQ_EINVAL, "export size mismatch");
  if (state) std::copy(c->r_state.begin(), c->r_state.end(), state);
  if (action) std::copy(c->r_action.begin(), c->r_action.end(), action);
  if (reward) std::copy(c->r_reward.begin(), c->r_reward.end(), reward);
  if (nonterm) std::copy(c->r_nonterm.begin(), c->r_nonterm.end(), nonterm);
  return DDQ_OK;
}

int ddq_replay_sample(ddq_ctx* c, const int32_t* idx, int32_t batch) {
  if (!c || !idx) return fail(c, DDQ_EINVAL, "null argument");
  if (!c->capacity) return fail(c, DDQ_ESTATE, "no replay buffer");
  if (batch >= c->valid)
    return fail(c, DDQ_EINVAL, "Can't draw sample of size %d from replay dataset of size %lld",
                batch, (long long)c->valid);
  if (batch != c->B) return fail(c, DDQ_EINVAL, "sample size %d != net batch %d", batch, c->B);
  for (int i = 0; i < batch; ++i) {
    if (idx[i] < 0 || idx[i] >= c->valid)
      return fail(c, DDQ_EINVAL, "index %d out of [0,valid)", idx[i]);
    if (i && idx[i] <= idx[i - 1]) return fail(c, DDQ_EINVAL, "indices must be sorted and distinct");
  }
  for (int i = 0; i < batch; ++i) {
    const int64_t nxt = idx[i] + 1 == c->capacity ? 0 : idx[i] + 1;
    if (c->r_action[nxt] >= kA)
      return fail(c, DDQ_ERANGE, "stored action index out of range for %d actions", kA);
  }
  std::copy(idx, idx + batch, c->idx.begin());
  gather(c);
  return DDQ_OK;
}

int ddq_replay_sample_device_async(ddq_ctx* c, uint64_t) {
  return cpu_only(c, "ddq_replay_sample_device_async (device index stream)");
}

int ddq_read_minibatch(ddq_ctx* c, float* state, float* action, float* reward, float* next_state,
                       float* nonterm) {
  if (!c) return fail(nullptr, DDQ_EINVAL, "null ctx");
  if (state) std::copy(c->state.begin(), c->state.end(), state);
  if (next_state) std::copy(c->next_state.begin(), c->next_state.end(), next_state);
  if (action) std::copy(c->action.begin(), c->action.end(), action);
  if (reward) std::copy(c->reward.begin(), c->reward.end(), reward);
  if (nonterm) std::copy(c->nonterm.begin(), c->nonterm.end(), nonterm);
  return DDQ_OK;
}

int ddq_write_minibatch(ddq_ctx* c, const float* state, const float* action, const float* reward,
                        const float* next_state, const float* nonterm) {
  if (!c) return fail(nullptr, DDQ_EINVAL, "null ctx");
  if (state) std::copy(state, state + c->state.size(), c->state.begin());
  if (next_state) std::copy(next_state, next_state + c->next_state.size(), c->next_state.begin());
  if (action) std::copy(action, action + c->action.size(), c->action.begin());
  if (reward) std::copy(reward, reward + c->reward.size(), c->reward.begin());
  if (nonterm) std::copy(nonterm, nonterm + c->nonterm.size(), c->nonterm.begin());
  return DDQ_OK;
}

int ddq_replay_fill_tiled(ddq_ctx* c, const uint8_t*, const uint8_t*, const int16_t*,
                          const uint8_t*, int64_t, int64_t, int64_t) {
  return cpu_only(c, "ddq_replay_fill_tiled");
}

int ddq_replay_sample_batch_async(ddq_ctx* c, int32_t, uint64_t, int32_t*, float*, float*, float*,
                                  float*, float*) {
  return cpu_only(c, "ddq_replay_sample_batch_async");
}

int ddq_replay_gather_batch_async(ddq_ctx* c, const int32_t*, int32_t, float*, float*, float*,
                                  float*, float*) {
  return cpu_only(c, "ddq_replay_gather_batch_async");
}

int ddq_replay_status(ddq_ctx* c) {
  if (!c) return fail(nullptr, DDQ_EINVAL, "null ctx");
  return c->capacity ? DDQ_OK : fail(c, DDQ_ESTATE, "no replay buffer");
}

int ddq_read_indices(ddq_ctx* c, int32_t* idx, int32_t batch) {
  if (!c || !idx || batch != c->B) return fail(c, DDQ_EINVAL, "bad argument");
  std::copy(c->idx.begin(), c->idx.end(), idx);
  return DDQ_OK;
}

int ddq_replay_draws(ddq_ctx* c, int64_t*) { return cpu_only(c, "ddq_replay_draws"); }
int ddq_index_log_enable(ddq_ctx* c, int64_t) { return cpu_only(c, "ddq_index_log_enable"); }
int ddq_index_log_read(ddq_ctx* c, int64_t, int64_t, int32_t*) {
  return cpu_only(c, "ddq_index_log_read");
}

// ---- compute ----
int ddq_forward_backward_async(ddq_ctx* c) {
  if (!c) return fail(nullptr, DDQ_EINVAL, "null ctx");
  return forward_backward(c);
}

int ddq_forward_backward(ddq_ctx* c, float* loss) {
  const int rc = ddq_forward_backward_async(c);
  if (rc == DDQ_OK && loss) *loss = c->loss;
  return rc;
}

int ddq_forward_q(ddq_ctx* c) {
  if (!c) return fail(nullptr, DDQ_EINVAL, "null ctx");
  tower_fwd(c, 0, c->state.data(), c->B);
  c->q_out = c->tw[0].out;
  return DDQ_OK;
}

int ddq_read_blob(ddq_ctx* c, const char* name, float* dst, int64_t n) {
  if (!c || !name || !dst) return fail(c, DDQ_EINVAL, "null argument");
  struct { const char* nm; const float* p; int64_t cnt; } t[] = {
      {"Q_out", c->q_out.data(), 4ll * c->B}, {"P_out", c->p_out.data(), 4ll * c->B},
      {"Q_sa", c->q_sa.data(), c->B},         {"P_sa", c->p_sa.data(), c->B},
      {"target_Q_sa", c->target.data(), c->B}, {"loss", &c->loss, 1}};
  for (auto& e : t)
    if (strcmp(e.nm, name) == 0) {
      if (n != e.cnt) return fail(c, DDQ_EINVAL, "blob %s has %lld elements", name, (long long)e.cnt);
      std::copy(e.p, e.p + n, dst);
      return DDQ_OK;
    }
  return fail(c, DDQ_EINVAL, "unknown blob '%s'", name);
}

int ddq_read_pool_mask(ddq_ctx* c, int32_t layer, uint8_t* dst, int64_t n) {
  if (!c || !dst) return fail(c, DDQ_EINVAL, "null argument");
  if (layer < 1 || layer > 3) return fail(c, DDQ_EINVAL, "layer must be 1..3");
  const int C = layer == 1 ? 32 : 64, Hp = c->S >> layer;
  const int64_t cnt = (int64_t)c->B * C * Hp * Hp;
  if (n != cnt) return fail(c, DDQ_EINVAL, "mask %d has %lld elements", layer, (long long)cnt);
  const std::vector<uint8_t>& r = c->tw[0].route[layer - 1];
  if ((int64_t)r.size() != cnt) return fail(c, DDQ_ESTATE, "no forward pass yet");
  std::copy(r.begin(), r.end(), dst);
  return DDQ_OK;
}

int ddq_select_action(ddq_ctx* c, const uint8_t* states, int32_t n, int32_t* actions) {
  if (!c || !states || !actions) return fail(c, DDQ_EINVAL, "null argument");
  if (n < 1 || n > c->B) return fail(c, DDQ_EINVAL, "n must be in [1,B]");
  const size_t e = (size_t)n * kC * c->S * c->S;
  std::vector<float> in(states, states + e);
  Tower keep = c->tw[0];            // acting does not touch the last training pass
  tower_fwd(c, 0, in.data(), n);
  for (int b = 0; b < n; ++b) {     // first maximum (the GPU's argmax)
    const float* q = c->tw[0].out.data() + (size_t)b * kA;
    int best = 0;
    for (int a = 1; a < kA; ++a)
      if (q[a] > q[best]) best = a;
    actions[b] = best;
  }
  c->tw[0] = std::move(keep);
  return DDQ_OK;
}

// ---- apply (server.py:49-124) ----
int ddq_apply_async(ddq_ctx* c, const ddq_update_cfg* u) {
  if (!c) return fail(nullptr, DDQ_EINVAL, "null ctx");
  if (!u) return fail(c, DDQ_EINVAL, "null update cfg");
  if (u->rule < 0 || u->rule > 3) return fail(c, DDQ_EINVAL, "unknown update rule %d", u->rule);
  const Layout& L = c->L;
  const bool first = c->first != 0;
  float* th = c->theta[0].data();
  for (int l = 0; l < 5; ++l)
    for (int bias = 0; bias < 2; ++bias) {
      const int64_t o = bias ? L.b[l] : L.w[l], cnt = bias ? L.bn[l] : L.wn[l];
      for (int64_t i = o; i < o + cnt; ++i) {
        float st = c->opt[i];
        th[i] = apply_rule(*u, first, bias != 0, th[i], c->grad[i], st);
        if (u->rule != DDQ_RULE_SGD) c->opt[i] = st;
      }
    }
  c->first = 0;
  c->iter++;
  return DDQ_OK;
}

int ddq_apply(ddq_ctx* c, const ddq_update_cfg* u) { return ddq_apply_async(c, u); }

int ddq_reset_optimizer(ddq_ctx* c) {
  if (!c) return fail(nullptr, DDQ_EINVAL, "null ctx");
  std::fill(c->opt.begin(), c->opt.end(), 0.f);
  c->first = 1;
  c->iter = 0;
  c->steps = 0;
  return DDQ_OK;
}

int ddq_get_optimizer_state(ddq_ctx* c, float* dst, int64_t n) {
  if (!c || !dst) return fail(c, DDQ_EINVAL, "null argument");
  if (n != c->L.total) return fail(c, DDQ_EINVAL, "size mismatch");
  std::copy(c->opt.begin(), c->opt.end(), dst);
  return DDQ_OK;
}

// ---- what needs a GPU: RCCL, graphs, groups, async exchange, timing ----
int ddq_comm_get_unique_id(uint8_t id[128]) {
  (void)id;
  return cpu_only(nullptr, "ddq_comm_get_unique_id (RCCL)");
}
int ddq_comm_init(ddq_ctx* c, const uint8_t[128], int32_t, int32_t) {
  return cpu_only(c, "ddq_comm_init (RCCL)");
}
int ddq_allreduce_grads(ddq_ctx* c) { return cpu_only(c, "ddq_allreduce_grads (RCCL)"); }
int ddq_allreduce_grads_async(ddq_ctx* c) { return cpu_only(c, "ddq_allreduce_grads_async (RCCL)"); }
int ddq_step_async(ddq_ctx* c, const ddq_step_cfg*) {
  return cpu_only(c, "ddq_step_async (device index stream)");
}
int ddq_step_graph_async(ddq_ctx* c, const ddq_step_cfg*, int32_t) {
  return cpu_only(c, "ddq_step_graph_async (hipGraph)");
}
int ddq_step_pipelined_async(ddq_ctx* c, const ddq_step_cfg*, int32_t) {
  return cpu_only(c, "ddq_step_pipelined_async (hipGraph)");
}
int ddq_step_prepare(ddq_ctx* c, const ddq_step_cfg*, int32_t) {
  return cpu_only(c, "ddq_step_prepare (hipGraph)");
}
int ddq_group_init(ddq_ctx** ctxs, int32_t) {
  return cpu_only(ctxs ? ctxs[0] : nullptr, "ddq_group_init");
}
int ddq_group_step(ddq_ctx** ctxs, int32_t, const ddq_step_cfg*) {
  return cpu_only(ctxs ? ctxs[0] : nullptr, "ddq_group_step");
}
int64_t ddq_step_count(const ddq_ctx* c) { return c ? c->steps : -1; }
int ddq_async_begin(ddq_ctx* c, const ddq_step_cfg*) { return cpu_only(c, "ddq_async_begin"); }
int ddq_async_ready(ddq_ctx* c, int32_t*) { return cpu_only(c, "ddq_async_ready"); }
int ddq_async_tick(ddq_ctx* c, const ddq_step_cfg*, int32_t) { return cpu_only(c, "ddq_async_tick"); }
int ddq_group_async_run(ddq_ctx** ctxs, int32_t, const ddq_step_cfg*, int32_t, int32_t*) {
  return cpu_only(ctxs ? ctxs[0] : nullptr, "ddq_group_async_run");
}
int ddq_group_async_ticks(ddq_ctx** ctxs, int32_t, const ddq_step_cfg*, int32_t, const int32_t*) {
  return cpu_only(ctxs ? ctxs[0] : nullptr, "ddq_group_async_ticks");
}
int ddq_set_straggle(ddq_ctx* c, int64_t) { return cpu_only(c, "ddq_set_straggle"); }
int ddq_profile_step(ddq_ctx* c, const ddq_step_cfg*, char*, float*, int32_t, int32_t*) {
  return cpu_only(c, "ddq_profile_step");
}
int ddq_time_layer(ddq_ctx* c, const char*, int32_t, float*) { return cpu_only(c, "ddq_time_layer"); }

double ddq_step_flops(const ddq_ctx* c) {
  if (!c) return 0.0;
  const double s1 = c->S, s2 = c->S / 2, s3 = c->S / 4, s4 = c->S / 8;
  const double F = (double)c->B * (6272 * s1 * s1 + 51200 * s2 * s2 + 36864 * s3 * s3 +
                                   32768 * s4 * s4 + 2048);
  return 2.0 * (4.0 * F - (double)c->B * 6272 * s1 * s1);
}

}  // extern "C"
