// Train-step kernels around the network: cross-entropy with ignore_index (nn.CrossEntropyLoss
// as wrapped by utils/loss.py:103-124; train.py:183-192), classifier Dropout(0.1)
// (models/fast_scnn.py:229), the fused multi-tensor SGD over the flat parameter arena
// (torch.optim.SGD momentum 0.9 / wd 1e-4, train.py:195-198) and fp32 -> bf16 weight casts.
#include "kernels.hpp"

#include <algorithm>
#include <cstring>

namespace fscnn {

// ---- cross entropy over NCHW logits, ignore_index --------------------------------------------

template <typename T>
__global__ __launch_bounds__(256) void ce_fwd_kernel(CeArgs a) {
  __shared__ float r1[256], r2[256];
  long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  long long total = (long long)a.N * a.HW;
  float loss = 0.f, cnt = 0.f;
  if (i < total) {
    long long n = i / a.HW, p = i - n * a.HW;
    long long t = a.target[i];
    if (t != a.ignore_index && t >= 0 && t < a.C && (!a.prob || a.prob[i] <= *a.thr)) {
      const T* lb = (const T*)a.logits + (size_t)n * a.C * a.HW + p;
      float mx = -INFINITY;
      for (int c = 0; c < a.C; ++c) mx = fmaxf(mx, ld1(lb + (size_t)c * a.HW));
      float se = 0.f;
      for (int c = 0; c < a.C; ++c) se += expf(ld1(lb + (size_t)c * a.HW) - mx);
      const float w = a.weight ? a.weight[t] : 1.f;
      loss = w * (mx + logf(se) - ld1(lb + (size_t)t * a.HW));
      cnt = w;
    }
  }
  r1[threadIdx.x] = loss;
  r2[threadIdx.x] = cnt;
  __syncthreads();
  for (int off = 128; off > 0; off >>= 1) {
    if (threadIdx.x < off) {
      r1[threadIdx.x] += r1[threadIdx.x + off];
      r2[threadIdx.x] += r2[threadIdx.x + off];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    a.part[2 * blockIdx.x] = r1[0];
    a.part[2 * blockIdx.x + 1] = r2[0];
  }
}

// merge partials (fp64, fixed order) -> out[0] = mean loss, out[1] = count
__global__ __launch_bounds__(256) void ce_finalize_kernel(const float* part, int P, float* out) {
  __shared__ double r1[256], r2[256];
  double s1 = 0.0, s2 = 0.0;
  for (int p = threadIdx.x; p < P; p += 256) {
    s1 += part[2 * p];
    s2 += part[2 * p + 1];
  }
  r1[threadIdx.x] = s1;
  r2[threadIdx.x] = s2;
  __syncthreads();
  for (int off = 128; off > 0; off >>= 1) {
    if (threadIdx.x < off) {
      r1[threadIdx.x] += r1[threadIdx.x + off];
      r2[threadIdx.x] += r2[threadIdx.x + off];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    out[0] = r2[0] > 0 ? (float)(r1[0] / r2[0]) : NAN;  // aten: mean over zero valid -> nan
    out[1] = (float)r2[0];
  }
}

int ce_parts(int N, long long HW) { return (int)(((long long)N * HW + 255) / 256); }

int ce_fwd(const CeArgs& a, float* out, int dtype, hipStream_t st) {
  int P = ce_parts(a.N, a.HW);
  if (dtype == DT_F32) prof_launch(ce_fwd_kernel<float>, P, 256, 0, st, a);
  else if (dtype == DT_F16) prof_launch(ce_fwd_kernel<f16>, P, 256, 0, st, a);
  else prof_launch(ce_fwd_kernel<bf16>, P, 256, 0, st, a);
  int rc = check_launch("ce_fwd");
  if (rc) return rc;
  prof_launch(ce_finalize_kernel, 1, 256, 0, st, a.part, P, out);
  return check_launch("ce_finalize");
}

// dlogits = (softmax - onehot) * grad_out / count ; 0 for ignored pixels
template <typename T>
__global__ __launch_bounds__(256) void ce_bwd_kernel(CeArgs a, const float* gout, const float* stats) {
  long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  long long total = (long long)a.N * a.HW;
  if (i >= total) return;
  long long n = i / a.HW, p = i - n * a.HW;
  long long t = a.target[i];
  const T* lb = (const T*)a.logits + (size_t)n * a.C * a.HW + p;
  T* db = (T*)a.dlogits + (size_t)n * a.C * a.HW + p;
  if (t == a.ignore_index || t < 0 || t >= a.C || (a.prob && !(a.prob[i] <= *a.thr))) {
    for (int c = 0; c < a.C; ++c) st1(db + (size_t)c * a.HW, 0.f);
    return;
  }
  float g = gout[0] / stats[1] * (a.weight ? a.weight[t] : 1.f);
  float mx = -INFINITY;
  for (int c = 0; c < a.C; ++c) mx = fmaxf(mx, ld1(lb + (size_t)c * a.HW));
  float se = 0.f;
  for (int c = 0; c < a.C; ++c) se += expf(ld1(lb + (size_t)c * a.HW) - mx);
  float inv = 1.f / se;
  for (int c = 0; c < a.C; ++c) {
    float pr = expf(ld1(lb + (size_t)c * a.HW) - mx) * inv;
    st1(db + (size_t)c * a.HW, (pr - (c == t ? 1.f : 0.f)) * g);
  }
}

int ce_bwd(const CeArgs& a, const float* gout, const float* stats, int dtype, hipStream_t st) {
  int P = ce_parts(a.N, a.HW);
  if (dtype == DT_F32) prof_launch(ce_bwd_kernel<float>, P, 256, 0, st, a, gout, stats);
  else if (dtype == DT_F16) prof_launch(ce_bwd_kernel<f16>, P, 256, 0, st, a, gout, stats);
  else prof_launch(ce_bwd_kernel<bf16>, P, 256, 0, st, a, gout, stats);
  return check_launch("ce_bwd");
}

// ---- OHEM selection (SoftmaxCrossEntropyOHEMLoss.forward, utils/loss.py:143-176) -------------
// prob[i] = softmax probability of the label (exp(x - max) / sum, the reference's numpy order in
// fp32) for labelled pixels, 2.0 (sorts after every probability) for ignored ones; counts[0] +=
// #labelled, counts[1] += #(prob <= thresh).  Integer counters: exact.
template <typename T>
__global__ __launch_bounds__(256) void ohem_prob_kernel(CeArgs a, float thresh, float* prob,
                                                        unsigned long long* counts) {
  __shared__ unsigned s_c[2];
  if (threadIdx.x < 2) s_c[threadIdx.x] = 0u;
  __syncthreads();
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long total = (long long)a.N * a.HW;
  if (i < total) {
    const long long n = i / a.HW, p = i - n * a.HW;
    const long long t = a.target[i];
    float pr = 2.f;
    if (t != a.ignore_index && t >= 0 && t < a.C) {
      const T* lb = (const T*)a.logits + (size_t)n * a.C * a.HW + p;
      float mx = -INFINITY;
      for (int c = 0; c < a.C; ++c) mx = fmaxf(mx, ld1(lb + (size_t)c * a.HW));
      float se = 0.f;
      for (int c = 0; c < a.C; ++c) se += expf(ld1(lb + (size_t)c * a.HW) - mx);
      pr = expf(ld1(lb + (size_t)t * a.HW) - mx) / se;
      atomicAdd(&s_c[0], 1u);
      if (pr <= thresh) atomicAdd(&s_c[1], 1u);
    }
    prob[i] = pr;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    if (s_c[0]) atomicAdd(&counts[0], (unsigned long long)s_c[0]);
    if (s_c[1]) atomicAdd(&counts[1], (unsigned long long)s_c[1]);
  }
}

int ohem_prob(const CeArgs& a, float thresh, float* prob, unsigned long long* counts, int dtype,
              hipStream_t st) {
  const int P = ce_parts(a.N, a.HW);
  if (dtype == DT_F32) prof_launch(ohem_prob_kernel<float>, P, 256, 0, st, a, thresh, prob, counts);
  else if (dtype == DT_F16) prof_launch(ohem_prob_kernel<f16>, P, 256, 0, st, a, thresh, prob, counts);
  else prof_launch(ohem_prob_kernel<bf16>, P, 256, 0, st, a, thresh, prob, counts);
  return check_launch("ohem_prob");
}

// k-th smallest of n non-negative floats (the OHEM threshold pred[argsort(pred)[k-1]]): radix
// select on the IEEE bit patterns (monotone for non-negative floats), 11 + 11 + 10 bits, one
// histogram launch per digit and a host pick of the digit (the reference does this step on the
// host in numpy too).
__global__ __launch_bounds__(256) void radix_hist_kernel(const float* key, long long n, int shift,
                                                         unsigned bins, int pshift,
                                                         unsigned prefix, unsigned* hist) {
  __shared__ unsigned s_h[2048];
  for (unsigned j = threadIdx.x; j < bins; j += blockDim.x) s_h[j] = 0u;
  __syncthreads();
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x) {
    const unsigned u = __float_as_uint(key[i]);
    const bool in = pshift >= 32 || (u >> pshift) == prefix;
    if (in) atomicAdd(&s_h[(u >> shift) & (bins - 1)], 1u);
  }
  __syncthreads();
  for (unsigned j = threadIdx.x; j < bins; j += blockDim.x)
    if (s_h[j]) atomicAdd(&hist[j], s_h[j]);
}

// The OHEM threshold's k-th smallest label probability as a device-side radix selection (no host round trip, so a train step with the OHEM
// criterion never synchronises): state = {active, k, prefix, pshift}, hist 2048 bins, thr_out.
//   init  : thr = inf if min_kept >= #labelled (reference: keep every labelled pixel), else
//           thresh; the radix select runs only when #(prob <= thresh) < k = min(#labelled, min_kept)
//   3 x (hist over the keys matching the prefix, pick: one workgroup scans the bins, extends the
//        prefix and re-zeroes the bins for the next digit)
//   final : thr = the selected bit pattern when the select ran.
struct OhemSel {
  unsigned active, prefix;
  int pshift;
  unsigned pad;
  unsigned long long k;
};

__global__ void ohem_sel_init_kernel(const unsigned long long* counts, long long min_kept,
                                     float thresh, OhemSel* s, unsigned* hist, float* thr) {
  for (int j = threadIdx.x; j < 2048; j += blockDim.x) hist[j] = 0u;
  if (threadIdx.x != 0) return;
  const unsigned long long num_valid = counts[0], n_le = counts[1];
  s->active = 0u; s->prefix = 0u; s->pshift = 32; s->k = 0ull;
  if ((unsigned long long)min_kept >= num_valid) {  // (min_kept >= 0)
    *thr = INFINITY;
    return;
  }
  *thr = thresh;
  if (min_kept > 0) {
    const unsigned long long k = (unsigned long long)min_kept < num_valid ? (unsigned long long)min_kept
                                                                          : num_valid;
    if (n_le < k) { s->active = 1u; s->k = k; }
  }
}

__global__ __launch_bounds__(256) void ohem_sel_hist_kernel(const float* key, long long n, int shift,
                                                            unsigned bins, const OhemSel* s,
                                                            unsigned* hist) {
  if (!s->active) return;
  const int pshift = s->pshift;
  const unsigned prefix = s->prefix;
  __shared__ unsigned s_h[2048];
  for (unsigned j = threadIdx.x; j < bins; j += blockDim.x) s_h[j] = 0u;
  __syncthreads();
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x) {
    const unsigned u = __float_as_uint(key[i]);
    const bool in = pshift >= 32 || (u >> pshift) == prefix;
    if (in) atomicAdd(&s_h[(u >> shift) & (bins - 1)], 1u);
  }
  __syncthreads();
  for (unsigned j = threadIdx.x; j < bins; j += blockDim.x)
    if (s_h[j]) atomicAdd(&hist[j], s_h[j]);
}

// one workgroup: exclusive scan of the bins in 256 chunks, the chunk holding the k-th key picks
__global__ __launch_bounds__(256) void ohem_sel_pick_kernel(OhemSel* s, unsigned* hist, unsigned bins,
                                                            int width, int shift) {
  if (!s->active) return;
  __shared__ unsigned long long s_sum[256];
  const unsigned per = (bins + 255) / 256;
  const unsigned b0 = threadIdx.x * per;
  unsigned long long own = 0;
  for (unsigned j = 0; j < per; ++j)
    if (b0 + j < bins) own += hist[b0 + j];
  s_sum[threadIdx.x] = own;
  __syncthreads();
  if (threadIdx.x == 0) {  // 256 serial adds: tiny
    unsigned long long run = 0;
    for (int t = 0; t < 256; ++t) {
      const unsigned long long v = s_sum[t];
      s_sum[t] = run;
      run += v;
    }
  }
  __syncthreads();
  const unsigned long long k = s->k;
  unsigned long long before = s_sum[threadIdx.x];
  __syncthreads();
  if (before < k && before + own >= k) {  // exactly one thread
    unsigned long long kk = k - before;
    unsigned b = b0;
    for (;; ++b) {
      const unsigned long long h = hist[b];
      if (h >= kk) break;
      kk -= h;
    }
    s->prefix = (s->prefix << width) | b;
    s->pshift = shift;
    s->k = kk;
  }
  __syncthreads();
  for (unsigned j = threadIdx.x; j < bins; j += blockDim.x) hist[j] = 0u;
}

__global__ void ohem_sel_final_kernel(const OhemSel* s, float* thr) {
  if (threadIdx.x == 0 && s->active) *thr = __uint_as_float(s->prefix);
}

int ohem_threshold_dev(const float* key, long long n, const unsigned long long* counts,
                       long long min_kept, float thresh, unsigned* work, float* thr,
                       hipStream_t st) {
  if (n <= 0 || min_kept < 0) {
    set_error("ohem_threshold: n=%lld min_kept=%lld", n, min_kept);
    return E_INVALID;
  }
  OhemSel* s = reinterpret_cast<OhemSel*>(work + 2048);
  prof_launch(ohem_sel_init_kernel, 1, 256, 0, st, counts, min_kept, thresh, s, work, thr);
  static const int shifts[3] = {21, 10, 0}, widths[3] = {11, 11, 10};
  const unsigned grid = (unsigned)std::min<long long>((n + 255) / 256, 2048);
  for (int d = 0; d < 3; ++d) {
    const unsigned bins = 1u << widths[d];
    prof_launch(ohem_sel_hist_kernel, grid, 256, 0, st, key, n, shifts[d], bins, s, work);
    prof_launch(ohem_sel_pick_kernel, 1, 256, 0, st, s, work, bins, widths[d], shifts[d]);
  }
  prof_launch(ohem_sel_final_kernel, 1, 64, 0, st, s, thr);
  return check_launch("ohem_threshold");
}

// ---- Dice / Focal+Dice (utils/loss.py:12-100; train.py:183-188 for binary lane segmentation) ----
// p1 = softmax(logits)[:, 1] (C > 1) or sigmoid(logits[:, 0]) (C == 1), t = float(target):
//   dice = (2 sum(p1 t) + s) / (sum p1 + sum t + s), DiceLoss = 1 - dice;
//   focal = mean_i alpha (1 - pt_i)^gamma ce_i with (FocalDiceLoss.focal_loss, :81-95)
//     C > 1: ce_i = lse_i - x_{t_i}, pt_i = exp(-ce_i);
//     C = 1: p = sigmoid(x), ce_i = F.binary_cross_entropy(p, t) = -(t max(log p, -100) +
//            (1 - t) max(log(1 - p), -100)), pt_i = t == 1 ? p : 1 - p.
// Forward: per-block partials of (sum p1 t, sum p1, sum t, sum focal), merged in fixed order in
// fp64.  Backward: dL/dx_c = wd * dDice/dp1 * dp1/dx_c + wf/n * dfocal/dce * (p_c - [c == t]);
// C = 1: autograd's chain through where / pow / BCE (aten's BCE backward divides by
// max(p (1 - p), 1e-12)) and sigmoid.
struct DiceArgs {
  const void* logits;
  const long long* target;
  long long N, HW;
  int C;
  float alpha, gamma;
  int focal;  // compute the focal term
};

template <typename T>
__device__ __forceinline__ void dice_pixel(const DiceArgs& a, long long i, float& p1, float& tf,
                                           float& ce, float& pt, float* pc, int cmax) {
  const long long n = i / a.HW, p = i - n * a.HW;
  const T* lb = (const T*)a.logits + (size_t)n * a.C * a.HW + p;
  const long long t = a.target[i];
  tf = (float)t;
  if (a.C == 1) {
    p1 = 1.f / (1.f + expf(-ld1(lb)));
    ce = 0.f;
    pt = 0.f;
    if (a.focal) {
      ce = -(tf * fmaxf(logf(p1), -100.f) + (1.f - tf) * fmaxf(logf(1.f - p1), -100.f));
      pt = tf == 1.f ? p1 : 1.f - p1;
    }
    return;
  }
  float mx = -INFINITY;
  for (int c = 0; c < a.C; ++c) mx = fmaxf(mx, ld1(lb + (size_t)c * a.HW));
  float se = 0.f;
  for (int c = 0; c < a.C; ++c) se += expf(ld1(lb + (size_t)c * a.HW) - mx);
  p1 = expf(ld1(lb + a.HW) - mx) / se;
  const long long tc = t < 0 ? 0 : (t >= a.C ? a.C - 1 : t);
  ce = mx + logf(se) - ld1(lb + (size_t)tc * a.HW);
  pt = expf(-ce);
  if (pc)
    for (int c = 0; c < cmax && c < a.C; ++c) pc[c] = expf(ld1(lb + (size_t)c * a.HW) - mx) / se;
}

template <typename T>
__global__ __launch_bounds__(256) void dice_fwd_kernel(DiceArgs a, float* part) {
  __shared__ float r[4][256];
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  float v[4] = {0.f, 0.f, 0.f, 0.f};
  if (i < a.N * a.HW) {
    float p1, tf, ce, pt;
    dice_pixel<T>(a, i, p1, tf, ce, pt, nullptr, 0);
    v[0] = p1 * tf;
    v[1] = p1;
    v[2] = tf;
    v[3] = a.focal ? a.alpha * powf(1.f - pt, a.gamma) * ce : 0.f;
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) r[k][threadIdx.x] = v[k];
  __syncthreads();
  for (int off = 128; off > 0; off >>= 1) {
    if (threadIdx.x < off)
#pragma unroll
      for (int k = 0; k < 4; ++k) r[k][threadIdx.x] += r[k][threadIdx.x + off];
    __syncthreads();
  }
  if (threadIdx.x < 4) part[4 * blockIdx.x + threadIdx.x] = r[threadIdx.x][0];
}

__global__ __launch_bounds__(256) void dice_finalize_kernel(const float* part, int P, double* out) {
  __shared__ double r[4][256];
  double s[4] = {0.0, 0.0, 0.0, 0.0};
  for (int p = threadIdx.x; p < P; p += 256)
#pragma unroll
    for (int k = 0; k < 4; ++k) s[k] += part[4 * p + k];
#pragma unroll
  for (int k = 0; k < 4; ++k) r[k][threadIdx.x] = s[k];
  __syncthreads();
  for (int off = 128; off > 0; off >>= 1) {
    if (threadIdx.x < off)
#pragma unroll
      for (int k = 0; k < 4; ++k) r[k][threadIdx.x] += r[k][threadIdx.x + off];
    __syncthreads();
  }
  if (threadIdx.x < 4) out[threadIdx.x] = r[threadIdx.x][0];
}

// stats: (I, P, T, focal sum) from dice_fwd; grad = wd * dDice + wf * dFocal, scaled by gout
template <typename T>
__global__ __launch_bounds__(256) void dice_bwd_kernel(DiceArgs a, const double* stats,
                                                       const float* gout, float smooth, float wd,
                                                       float wf, void* dlogits) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= a.N * a.HW) return;
  const long long n = i / a.HW, p = i - n * a.HW;
  float p1, tf, ce, pt;
  dice_pixel<T>(a, i, p1, tf, ce, pt, nullptr, 0);
  const double I = stats[0], den = stats[1] + stats[2] + (double)smooth;
  // d(1 - dice)/dp1 = -(2 t den - (2 I + s)) / den^2
  const float gd = (float)(-(2.0 * tf * den - (2.0 * I + smooth)) / (den * den)) * wd * gout[0];
  float gf = 0.f;
  if (a.focal && a.C > 1) {
    const float om = 1.f - pt;
    const float dfdce = a.alpha * (powf(om, a.gamma) + ce * a.gamma * powf(om, a.gamma - 1.f) * pt);
    gf = dfdce * wf * gout[0] / (float)(a.N * a.HW);
  }
  const T* lb = (const T*)a.logits + (size_t)n * a.C * a.HW + p;
  T* db = (T*)dlogits + (size_t)n * a.C * a.HW + p;
  if (a.C == 1) {
    const float s = p1 * (1.f - p1);  // sigmoid backward
    float g = gd * s;
    if (a.focal) {
      const float om = 1.f - pt;
      const float dce = (p1 - tf) / fmaxf(s, 1e-12f) * s;
      const float dpt = (tf == 1.f ? 1.f : -1.f) * s;
      const float df = a.alpha * (powf(om, a.gamma) * dce - a.gamma * powf(om, a.gamma - 1.f) * dpt * ce);
      g += df * wf * gout[0] / (float)(a.N * a.HW);
    }
    st1(db, g);
    return;
  }
  float mx = -INFINITY;
  for (int c = 0; c < a.C; ++c) mx = fmaxf(mx, ld1(lb + (size_t)c * a.HW));
  float se = 0.f;
  for (int c = 0; c < a.C; ++c) se += expf(ld1(lb + (size_t)c * a.HW) - mx);
  const long long t = a.target[i];
  for (int c = 0; c < a.C; ++c) {
    const float pcv = expf(ld1(lb + (size_t)c * a.HW) - mx) / se;
    const float dice_c = gd * p1 * ((c == 1 ? 1.f : 0.f) - pcv);
    const float focal_c = gf * (pcv - (c == t ? 1.f : 0.f));
    st1(db + (size_t)c * a.HW, dice_c + focal_c);
  }
}

int dice_loss_fwd(const void* logits, int dtype, const long long* target, int N, int C, long long HW,
                  float alpha, float gamma, int focal, float* part, double* stats, hipStream_t st) {
  if (C < 1) {
    set_error("dice_loss: C=%d", C);
    return E_INVALID;
  }
  DiceArgs a{logits, target, N, HW, C, alpha, gamma, focal};
  const int P = ce_parts(N, HW);
  if (dtype == DT_F32) prof_launch(dice_fwd_kernel<float>, P, 256, 0, st, a, part);
  else if (dtype == DT_F16) prof_launch(dice_fwd_kernel<f16>, P, 256, 0, st, a, part);
  else prof_launch(dice_fwd_kernel<bf16>, P, 256, 0, st, a, part);
  if (int rc = check_launch("dice_fwd")) return rc;
  prof_launch(dice_finalize_kernel, 1, 256, 0, st, part, P, stats);
  return check_launch("dice_finalize");
}

int dice_loss_bwd(const void* logits, int dtype, const long long* target, int N, int C, long long HW,
                  float alpha, float gamma, int focal, const double* stats, const float* gout,
                  float smooth, float wd, float wf, void* dlogits, hipStream_t st) {
  DiceArgs a{logits, target, N, HW, C, alpha, gamma, focal};
  const int P = ce_parts(N, HW);
  if (dtype == DT_F32) prof_launch(dice_bwd_kernel<float>, P, 256, 0, st, a, stats, gout, smooth, wd, wf, dlogits);
  else if (dtype == DT_F16) prof_launch(dice_bwd_kernel<f16>, P, 256, 0, st, a, stats, gout, smooth, wd, wf, dlogits);
  else prof_launch(dice_bwd_kernel<bf16>, P, 256, 0, st, a, stats, gout, smooth, wd, wf, dlogits);
  return check_launch("dice_bwd");
}

// ---- dropout on an NHWC activation, mask indexed in NCHW order (matches the oracle) ----------

// Channel-owning sweep (common.hpp chan_sweep): a thread keeps one 16-B channel vector's lazy-BN
// tables in registers and visits pixels p0, p0 + P, ..., U pixels' loads issued back to back.
// The per-element arithmetic and the keep decision (a hash of the NCHW index) are unchanged.
template <typename T>
__global__ __launch_bounds__(256) void dropout_kernel(DropArgs a, uint32_t thr, unsigned P) {
  constexpr int V = VecW<T>::V;
  constexpr int U = 4;
  const unsigned CV = (unsigned)(a.C / V), HW = (unsigned)(a.H * a.W);
  const unsigned t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= P * CV) return;
  const unsigned p0 = t / CV, cv = t - p0 * CV;
  const long long npix = (long long)a.N * HW;
  const uint64_t seed = (a.seed_ptr ? *a.seed_ptr : a.seed) + a.seed_add;
  const bool lazy = a.x_scale != nullptr;
  float xs[V], xh[V];
#pragma unroll
  for (int j = 0; j < V; ++j) {
    xs[j] = lazy ? a.x_scale[cv * V + j] : 1.f;
    xh[j] = lazy ? a.x_shift[cv * V + j] : 0.f;
  }
  const float s = 1.f / (1.f - a.p);
  for (long long q0 = p0; q0 < npix; q0 += (long long)U * P) {
    float v[U][V];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long long q = q0 + (long long)u * P;
      const size_t pix = (size_t)(q < npix ? q : q0);
      ldv((const T*)a.x + pix * a.ldx + cv * V, v[u]);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long long q = q0 + (long long)u * P;
      if (q >= npix) break;
      const unsigned pix = (unsigned)q;
      const unsigned n = pix / HW, hw = pix - n * HW;
      if (lazy) {  // lazy BN+ReLU of the producer's z (the activation itself is never stored)
#pragma unroll
        for (int j = 0; j < V; ++j) v[u][j] = round_as<T>(fmaxf(fmaf(v[u][j], xs[j], xh[j]), 0.f));
      }
#pragma unroll
      for (int j = 0; j < V; ++j) {
        const uint64_t nchw = ((uint64_t)n * a.C + cv * V + j) * HW + hw;
        v[u][j] = dropout_keep(seed, nchw, thr) ? v[u][j] * s : 0.f;
      }
      stv((T*)a.y + (size_t)pix * a.ldy + cv * V, v[u]);
    }
  }
}

int dropout(const DropArgs& a, int dtype, hipStream_t st) {
  const int V = dtype == DT_F32 ? 4 : 8;
  const long long total = (long long)a.N * a.H * a.W * (a.C / V);
  if (a.C % V || a.ldx % V || a.ldy % V || total >= (1LL << 31)) {
    set_error("dropout: C=%d ldx=%d ldy=%d", a.C, a.ldx, a.ldy);
    return E_UNSUPPORTED;
  }
  const unsigned P = chan_sweep((long long)a.N * a.H * a.W, a.C / V);
  const unsigned grid = (unsigned)(((long long)P * (a.C / V) + 255) / 256);
  uint32_t thr = dropout_threshold(a.p);
  if (dtype == DT_F32) prof_launch(dropout_kernel<float>, grid, 256, 0, st, a, thr, P);
  else if (dtype == DT_F16) prof_launch(dropout_kernel<f16>, grid, 256, 0, st, a, thr, P);
  else prof_launch(dropout_kernel<bf16>, grid, 256, 0, st, a, thr, P);
  return check_launch("dropout");
}

// ---- SegmentationMetric counters (utils/metric.py:73-105) -------------------------------------
// counts[0] = correct = #(p == t, t >= 0), counts[1] = labeled = #(t >= 0) (batch_pix_accuracy:
// labels >= C, e.g. 255, count as labeled), then per class c < C: inter = #(p == t == c),
// area_pred = #(p == c, t >= 0), area_lab = #(t == c) (batch_intersection_union's histograms over
// [1, C] of the +1-shifted values).  Integer counts: LDS histograms, one global integer add per
// non-zero bin and workgroup, so the result is exact and order independent.  Accumulates.
constexpr int SM_CMAX = 1024;

template <typename TP>
__global__ __launch_bounds__(256) void seg_metric_kernel(const TP* pred, const long long* tgt,
                                                         long long n, int C,
                                                         unsigned long long* counts) {
  __shared__ unsigned s_h[3 * SM_CMAX];
  __shared__ unsigned s_cl[2];
  for (int j = threadIdx.x; j < 3 * C; j += blockDim.x) s_h[j] = 0u;
  if (threadIdx.x < 2) s_cl[threadIdx.x] = 0u;
  __syncthreads();
  unsigned correct = 0, labeled = 0;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x) {
    const long long t = tgt[i];
    const long long p = (long long)pred[i];
    if (t >= 0) {
      ++labeled;
      correct += p == t ? 1u : 0u;
      if (p >= 0 && p < C) atomicAdd(&s_h[C + (int)p], 1u);
    }
    if (t >= 0 && t < C) {
      atomicAdd(&s_h[2 * C + (int)t], 1u);
      if (p == t) atomicAdd(&s_h[(int)t], 1u);
    }
  }
  atomicAdd(&s_cl[0], correct);
  atomicAdd(&s_cl[1], labeled);
  __syncthreads();
  for (int j = threadIdx.x; j < 3 * C; j += blockDim.x)
    if (s_h[j]) atomicAdd(&counts[2 + j], (unsigned long long)s_h[j]);
  if (threadIdx.x == 0) {
    atomicAdd(&counts[0], (unsigned long long)s_cl[0]);
    atomicAdd(&counts[1], (unsigned long long)s_cl[1]);
  }
}

int seg_metric(const void* pred, int pred_u8, const long long* target, long long n, int C,
               long long* counts, hipStream_t st) {
  if (C < 1 || C > SM_CMAX || n < 0) {
    set_error("seg_metric: nclass %d (1..%d), n %lld", C, SM_CMAX, n);
    return E_INVALID;
  }
  if (n == 0) return OK;
  const long long blocks = (n + 255) / 256;
  const unsigned grid = (unsigned)(blocks < 1024 ? blocks : 1024);
  unsigned long long* c = reinterpret_cast<unsigned long long*>(counts);
  if (pred_u8) prof_launch(seg_metric_kernel<uint8_t>, grid, 256, 0, st, (const uint8_t*)pred, target, n, C, c);
  else prof_launch(seg_metric_kernel<long long>, grid, 256, 0, st, (const long long*)pred, target, n, C, c);
  return check_launch("seg_metric");
}

// ---- GPU input path ---------------------------------------------------
// transforms.ToTensor() + transforms.Normalize(mean, std) (train.py:104-107, eval.py:22-25,
// demo.py:37-40) on a batch of uint8 HWC RGB images, written as the NCHW network input:
//     y[n][c][h][w] = (x[n][h][w][c] / 255 - mean[c]) / std[c]
// with torchvision's fp32 operation order (div, sub, div), so the fp32 result is bit-identical.
// Thread = 4 consecutive pixels of one row: 12 input bytes, 4-wide stores per channel plane.
template <typename TO>
__global__ __launch_bounds__(256) void normalize_u8_kernel(const uint8_t* x, long long npix4,
                                                           long long HW, float m0, float m1,
                                                           float m2, float s0, float s1, float s2,
                                                           TO* y) {
  const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= npix4) return;
  const long long p0 = t * 4;            // first pixel (flat over N*H*W; HW % 4 == 0 host-checked)
  const long long n = p0 / HW, hw = p0 - n * HW;
  const uint8_t* src = x + p0 * 3;
  const float mean[3] = {m0, m1, m2}, sd[3] = {s0, s1, s2};
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    float v[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = ((float)src[3 * j + c] / 255.f - mean[c]) / sd[c];
    TO* dst = y + ((size_t)n * 3 + c) * HW + hw;
    if constexpr (sizeof(TO) == 4) {
      *reinterpret_cast<float4*>(dst) = make_float4(v[0], v[1], v[2], v[3]);
    } else {
      uint2 u;
      u.x = (uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16);
      u.y = (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16);
      *reinterpret_cast<uint2*>(dst) = u;
    }
  }
}

int normalize_u8(const uint8_t* x, int N, int H, int W, const float* mean, const float* std,
                 void* y, int out_dtype, hipStream_t st) {
  const long long HW = (long long)H * W;
  if (N < 1 || H < 1 || W < 1 || HW % 4 || (uintptr_t)y % 16) {
    set_error("normalize_u8: N=%d H=%d W=%d (H*W must be a multiple of 4, y 16-B aligned)", N, H, W);
    return E_INVALID;
  }
  const long long npix4 = (long long)N * HW / 4;
  const unsigned grid = (unsigned)((npix4 + 255) / 256);
  if (out_dtype == DT_F32)
    prof_launch(normalize_u8_kernel<float>, grid, 256, 0, st, x, npix4, HW, mean[0], mean[1], mean[2],
                                                     std[0], std[1], std[2], (float*)y);
  else
    prof_launch(normalize_u8_kernel<bf16>, grid, 256, 0, st, x, npix4, HW, mean[0], mean[1], mean[2],
                                                    std[0], std[1], std[2], (bf16*)y);
  return check_launch("normalize_u8");
}

// Dataset label-id -> train-id remap (data_loader/cityscapes.py:56-71 `_class_to_index`:
// key[digitize(v, mapping=range(-1, K-1), right=True)] == key[v + 1] for v in [-1, K-2]) as a
// lookup table on the device: out[i] = lut[in[i] + offset], and `invalid` (the reference
// asserts instead) for ids outside the table.
__global__ __launch_bounds__(256) void remap_labels_kernel(const uint8_t* in, long long n,
                                                           const long long* lut, int lut_size,
                                                           int offset, long long invalid,
                                                           long long* out) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int k = (int)in[i] + offset;
  out[i] = (k >= 0 && k < lut_size) ? lut[k] : invalid;
}

int remap_labels(const uint8_t* in, long long n, const long long* lut, int lut_size, int offset,
                 long long invalid, long long* out, hipStream_t st) {
  if (n < 0 || lut_size < 1) {
    set_error("remap_labels: n=%lld lut_size=%d", n, lut_size);
    return E_INVALID;
  }
  if (n == 0) return OK;
  prof_launch(remap_labels_kernel, (unsigned)((n + 255) / 256), 256, 0, st, in, n, lut, lut_size, offset,
                                                                    invalid, out);
  return check_launch("remap_labels");
}

__global__ void set_u64_kernel(uint64_t* p, uint64_t v) { *p = v; }

int set_u64(uint64_t* p, uint64_t v, hipStream_t st) {
  prof_launch(set_u64_kernel, 1, 1, 0, st, p, v);
  return check_launch("set_u64");
}

// ---- fused SGD over a flat fp32 arena ------------------------------------------------------
// d = g + wd*p; buf = first ? d : momentum*buf + (1-dampening)*d; d = nesterov ? d + m*buf : buf;
// p -= lr*d     (torch.optim.SGD semantics)

__global__ __launch_bounds__(256) void sgd_kernel(SgdArgs a) {
  long long i = ((long long)blockIdx.x * blockDim.x + threadIdx.x) * 4;
  if (i >= a.n) return;
  int cnt = (int)min((long long)4, a.n - i);
  for (int j = 0; j < cnt; ++j) {
    float p = a.p[i + j];
    float d = a.g[i + j] * a.grad_scale + a.weight_decay * p;
    if (a.momentum != 0.f) {
      float b = a.first ? d : a.momentum * a.buf[i + j] + (1.f - a.dampening) * d;
      a.buf[i + j] = b;
      d = a.nesterov ? d + a.momentum * b : b;
    }
    a.p[i + j] = p - a.lr * d;
  }
}

int sgd(const SgdArgs& a, hipStream_t st) {
  unsigned grid = (unsigned)((a.n + 1023) / 1024);
  prof_launch(sgd_kernel, grid, 256, 0, st, a);
  return check_launch("sgd");
}

// ---- per-step weight preparation ---------------------------------------------------------------
// One launch builds the compute-dtype weight operands of a training step from the fp32 master
// arena P: the plain cast of the whole arena (bf16 steps) and, for every dense conv, W^T
// [cin*k*k][ld] zero-padded past cout (the dgrad's non-transposed B operand).  Element i of the
// flattened job table belongs to the job whose [start, start') range holds it.
// One workgroup per 2048-element chunk of one job (t.cstart: the chunks of job k are
// [cstart[k], cstart[k+1])), found by a workgroup-uniform binary search, so the job record is read
// once per workgroup and the thread's 8 elements (256 apart) are independent loads in flight
// together; 32-bit index arithmetic within a job (host-checked).  (r06: a flat element range
// with the job searched and advanced per thread was a chain of dependent table and data loads,
// 17-19 us per step for ~3.4 M elements.)
constexpr int PREP_PER = 8;
constexpr int PREP_CHUNK = 256 * PREP_PER;
template <typename T>
__global__ __launch_bounds__(256) void weights_prep_kernel(PrepTable t, const float* P, T* dst) {
  const int b = blockIdx.x;
  int lo = 0, hi = t.n - 1;
  while (lo < hi) {  // last job whose first chunk <= b (uniform)
    const int mid = (lo + hi + 1) >> 1;
    if (t.cstart[mid] <= b) lo = mid;
    else hi = mid - 1;
  }
  const PrepJob& J = t.j[lo];
  const int len = (int)(t.start[lo + 1] - t.start[lo]);
  const int i0 = (b - t.cstart[lo]) * PREP_CHUNK + threadIdx.x;
  if (J.trans == 3) {  // one term of the bf16 truncation split, planes [3][R][Cc]
    const int plane = J.R * J.Cc;
    float f[PREP_PER];
#pragma unroll
    for (int e = 0; e < PREP_PER; ++e) {
      const int idx = i0 + 256 * e, ic = idx < len ? idx : 0;
      const int p = ic >= plane ? (ic >= 2 * plane ? 2 : 1) : 0;
      f[e] = P[J.src + (ic - p * plane)];
    }
#pragma unroll
    for (int e = 0; e < PREP_PER; ++e) {
      const int idx = i0 + 256 * e;
      if (idx >= len) break;
      const int p = idx >= plane ? (idx >= 2 * plane ? 2 : 1) : 0;
      const uint32_t h0 = __float_as_uint(f[e]) & 0xFFFF0000u;
      const float r1 = f[e] - __uint_as_float(h0);
      const uint32_t h1 = __float_as_uint(r1) & 0xFFFF0000u;
      const float r2 = r1 - __uint_as_float(h1);
      const uint32_t term = p == 0 ? h0 : (p == 1 ? h1 : __float_as_uint(r2) & 0xFFFF0000u);
      reinterpret_cast<uint16_t*>(dst)[J.dst + idx] = (uint16_t)(term >> 16);
    }
    return;
  }
  float v[PREP_PER];
#pragma unroll
  for (int e = 0; e < PREP_PER; ++e) {
    const int idx = i0 + 256 * e, ic = idx < len ? idx : 0;
    if (J.trans == 2) {
      v[e] = 0.f;  // zero fill (counters)
    } else if (J.trans) {
      const int n = ic / J.ld;
      const int k = ic - n * J.ld;
      v[e] = k < J.R ? P[J.src + (long long)(k < J.R ? k : 0) * J.Cc + n] : 0.f;
    } else {
      v[e] = P[J.src + ic];
    }
  }
#pragma unroll
  for (int e = 0; e < PREP_PER; ++e) {
    const int idx = i0 + 256 * e;
    if (idx < len) st1(dst + J.dst + idx, v[e]);
  }
}

int weights_prep(PrepTable& t, const float* P, void* dst, int dtype, hipStream_t st) {
  if (t.n <= 0 || t.n > PREP_MAXJOBS) {
    set_error("weights_prep: %d jobs", t.n);
    return E_INVALID;
  }
  t.total = 0;
  for (int k = 0; k < t.n; ++k) {
    t.start[k] = t.total;
    t.total += t.j[k].trans == 1 ? (long long)t.j[k].Cc * t.j[k].ld
                                 : (t.j[k].trans == 3 ? 3LL : 1LL) * t.j[k].R * t.j[k].Cc;
  }
  t.start[t.n] = t.total;
  for (int k = 0; k < t.n; ++k)
    if (t.start[k + 1] - t.start[k] >= (1LL << 31)) {
      set_error("weights_prep: job %d has %lld elements", k, t.start[k + 1] - t.start[k]);
      return E_INVALID;
    }
  t.cstart[0] = 0;
  for (int k = 0; k < t.n; ++k)
    t.cstart[k + 1] = t.cstart[k] + (int)((t.start[k + 1] - t.start[k] + PREP_CHUNK - 1) / PREP_CHUNK);
  const unsigned grid = (unsigned)t.cstart[t.n];
  if (grid == 0) return OK;
  if (dtype == DT_F32) prof_launch(weights_prep_kernel<float>, grid, 256, 0, st, t, P, (float*)dst);
  else if (dtype == DT_F16) prof_launch(weights_prep_kernel<f16>, grid, 256, 0, st, t, P, (f16*)dst);
  else prof_launch(weights_prep_kernel<bf16>, grid, 256, 0, st, t, P, (bf16*)dst);
  return check_launch("weights_prep");
}

// ---- casts ------------------------------------------------------------------------------------
__global__ void cast_f32_bf16_kernel(const float* x, uint16_t* y, long long n) {
  long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) y[i] = f2bf(x[i]);
}
int cast_f32_bf16(const float* x, void* y, long long n, hipStream_t st) {
  prof_launch(cast_f32_bf16_kernel, (unsigned)((n + 255) / 256), 256, 0, st, x, (uint16_t*)y, n);
  return check_launch("cast_f32_bf16");
}

__global__ void fill_kernel(float* x, long long n, float v) {
  long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) x[i] = v;
}
int fill_f32(float* x, long long n, float v, hipStream_t st) {
  if (n <= 0) return OK;
  prof_launch(fill_kernel, (unsigned)((n + 255) / 256), 256, 0, st, x, n, v);
  return check_launch("fill");
}

}  // namespace fscnn
