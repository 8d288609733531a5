// BatchNorm2d (eps 1e-5, momentum 0.1, affine, tracked stats) for every BN of
// models/fast_scnn.py (:56,:71,:74,:87,:108,:199,:203,:27).
//
// eval : bn_fold   — one launch folds ALL BNs of the net (+ preceding conv bias) into
//                    per-channel scale/shift consumed by the producing kernel's epilogue.
// train: producers emit partial (mean, M2, count) records; bn_finalize merges them (Chan, fp64,
//        fixed order) into mean / invstd / scale / shift, and updates running_mean,
//        running_var (unbiased, n/(n-1)) and num_batches_tracked like aten's batch_norm;
//        bn_apply normalises (+ residual / second branch, + ReLU).
// backward: bn_bwd_reduce (per-block sums of dy_r and dy_r*xhat) -> bn_bwd_finalize
//        (dgamma, dbeta into the gradient arena + coefficients) -> bn_bwd_apply (dz).
#include "kernels.hpp"

namespace fscnn {

constexpr float BN_EPS = 1e-5f;

// ---- eval fold of every BN in one launch ------------------------------------------------------

__global__ void bn_fold_kernel(FoldTable t) {
  const FoldEntry& e = t.e[blockIdx.x];
  for (int c = threadIdx.x; c < e.C; c += blockDim.x) {
    float s = e.gamma[c] / sqrtf(e.rvar[c] + BN_EPS);
    float b = e.bias ? e.bias[c] : 0.f;
    e.scale[c] = s;
    e.shift[c] = e.beta[c] + (b - e.rmean[c]) * s;
  }
}

int bn_fold(const FoldTable& t, hipStream_t st) {
  if (t.n <= 0 || t.n > MAX_FOLD) {
    set_error("bn_fold: bad table size %d", t.n);
    return E_INVALID;
  }
  bn_fold_kernel<<<t.n, 256, 0, st>>>(t);
  return check_launch("bn_fold");
}

// ---- train: merge partial records ------------------------------------------------------------

__global__ __launch_bounds__(256) void bn_finalize_kernel(BnFinalizeArgs a) {
  const int c = blockIdx.x;
  __shared__ double sn[256], sm[256], s2[256];
  Welford w = {0.0, 0.0, 0.0};
  for (int p = threadIdx.x; p < a.P; p += 256) {
    const float* rec = a.part + (size_t)p * 3 * a.C;
    Welford b = {(double)rec[2 * a.C + c], (double)rec[c], (double)rec[a.C + c]};
    if (b.n > 0) w = wf_merge(w, b);
  }
  sn[threadIdx.x] = w.n;
  sm[threadIdx.x] = w.mean;
  s2[threadIdx.x] = w.m2;
  __syncthreads();
  for (int off = 128; off > 0; off >>= 1) {
    if (threadIdx.x < off) {
      Welford x = {sn[threadIdx.x], sm[threadIdx.x], s2[threadIdx.x]};
      Welford y = {sn[threadIdx.x + off], sm[threadIdx.x + off], s2[threadIdx.x + off]};
      Welford z = (y.n > 0) ? wf_merge(x, y) : x;
      sn[threadIdx.x] = z.n;
      sm[threadIdx.x] = z.mean;
      s2[threadIdx.x] = z.m2;
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    double n = sn[0], mean = sm[0] + (a.bias ? (double)a.bias[c] : 0.0);
    double var = n > 0 ? s2[0] / n : 0.0;
    float invstd = (float)(1.0 / sqrt(var + (double)BN_EPS));
    float scale = a.gamma[c] * invstd;
    a.mean[c] = (float)mean;
    a.invstd[c] = invstd;
    a.scale[c] = scale;
    a.shift[c] = a.beta[c] - (float)mean * scale;
    if (a.rmean) {
      float m = a.momentum;
      a.rmean[c] = (1.f - m) * a.rmean[c] + m * (float)mean;
      float unb = n > 1 ? (float)(s2[0] / (n - 1.0)) : (float)var;
      a.rvar[c] = (1.f - m) * a.rvar[c] + m * unb;
    }
    if (a.nbt && c == 0) a.nbt[0] += 1;
  }
}

int bn_finalize(const BnFinalizeArgs& a, hipStream_t st) {
  bn_finalize_kernel<<<a.C, 256, 0, st>>>(a);
  return check_launch("bn_finalize");
}

// ---- train: normalise  y = act(z*scale + shift [+ z2*scale2 + shift2] [+ res]) ---------------

template <typename T>
__global__ __launch_bounds__(256) void bn_apply_kernel(BnApplyArgs a) {
  constexpr int V = VecW<T>::V;
  const int CV = a.C / V;
  // 32-bit index math (M*C/V < 2^31 is enforced by the planner)
  const unsigned i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (unsigned)a.M * (unsigned)CV) return;
  const unsigned mu = i / (unsigned)CV;
  const int c = (int)(i - mu * (unsigned)CV) * V;
  const long long m = mu;
  float z[V], o[V];
  ldv((const T*)a.z + m * a.ldz + c, z);
#pragma unroll
  for (int j = 0; j < V; ++j) o[j] = z[j] * a.scale[c + j] + a.shift[c + j];
  if (a.z2) {
    ldv((const T*)a.z2 + m * a.ldz2 + c, z);
#pragma unroll
    for (int j = 0; j < V; ++j) o[j] += z[j] * a.scale2[c + j] + a.shift2[c + j];
  }
  if (a.res) {
    ldv((const T*)a.res + m * a.ldres + c, z);
#pragma unroll
    for (int j = 0; j < V; ++j) o[j] += z[j];
  }
  if (a.relu) {
#pragma unroll
    for (int j = 0; j < V; ++j) o[j] = fmaxf(o[j], 0.f);
  }
  stv((T*)a.y + m * a.ldy + c, o);
}

int bn_apply(const BnApplyArgs& a, int dtype, hipStream_t st) {
  int V = dtype == DT_F32 ? 4 : 8;
  if (a.C % V) { set_error("bn_apply: C=%d not a multiple of %d", a.C, V); return E_INVALID; }
  long long total = a.M * (a.C / V);
  unsigned grid = (unsigned)((total + 255) / 256);
  if (dtype == DT_F32) bn_apply_kernel<float><<<grid, 256, 0, st>>>(a);
  else bn_apply_kernel<bf16><<<grid, 256, 0, st>>>(a);
  return check_launch("bn_apply");
}

// ---- backward -------------------------------------------------------------------------------
// dy_r = dy * [mask > 0] (mask = the saved post-activation output, if the BN is followed by a
// ReLU or the FFM's ReLU), xhat = (z - mean) * invstd.

template <typename T>
__global__ __launch_bounds__(256) void bn_bwd_reduce_kernel(BnBwdArgs a) {
  constexpr int V = VecW<T>::V;
  const int CV = a.C / V;
  // block = (channel vectors along x, row groups along y)
  const int cv = blockIdx.x * blockDim.x + threadIdx.x;
  const int BX = blockDim.x, BY = blockDim.y;
  extern __shared__ float red[];  // [BY][BX*V*2]
  float s1[V], s2[V];
#pragma unroll
  for (int j = 0; j < V; ++j) { s1[j] = 0.f; s2[j] = 0.f; }
  if (cv < CV) {
    const int c = cv * V;
    float mu[V], is[V];
#pragma unroll
    for (int j = 0; j < V; ++j) { mu[j] = a.mean[c + j]; is[j] = a.invstd[c + j]; }
    long long mb = (long long)blockIdx.y * a.rows_per_block;
    long long me = min(a.M, mb + a.rows_per_block);
    for (long long m = mb + threadIdx.y; m < me; m += BY) {
      float g[V], z[V];
      ldv((const T*)a.dy + m * a.lddy + c, g);
      if (a.mask) {
        float mk[V];
        ldv((const T*)a.mask + m * a.ldmask + c, mk);
#pragma unroll
        for (int j = 0; j < V; ++j) g[j] = mk[j] > 0.f ? g[j] : 0.f;
      }
      ldv((const T*)a.z + m * a.ldz + c, z);
#pragma unroll
      for (int j = 0; j < V; ++j) {
        s1[j] += g[j];
        s2[j] += g[j] * (z[j] - mu[j]) * is[j];
      }
    }
  }
#pragma unroll
  for (int j = 0; j < V; ++j) {
    red[(threadIdx.y * BX + threadIdx.x) * 2 * V + j] = s1[j];
    red[(threadIdx.y * BX + threadIdx.x) * 2 * V + V + j] = s2[j];
  }
  __syncthreads();
  if (threadIdx.y == 0 && cv < CV) {
    float* rec = a.part + (size_t)blockIdx.y * 2 * a.C;
#pragma unroll
    for (int j = 0; j < V; ++j) {
      float t1 = 0.f, t2 = 0.f;
      for (int k = 0; k < BY; ++k) {
        t1 += red[(k * BX + threadIdx.x) * 2 * V + j];
        t2 += red[(k * BX + threadIdx.x) * 2 * V + V + j];
      }
      rec[cv * V + j] = t1;
      rec[a.C + cv * V + j] = t2;
    }
  }
}

static void bn_bwd_shape(int C, int V, int& bx, int& by) {
  int cv = C / V;
  bx = cv < 64 ? cv : 64;
  by = 256 / bx;
}

int bn_bwd_parts(long long M, int C, int dtype, int* rows_per_block) {
  int V = dtype == DT_F32 ? 4 : 8, bx, by;
  bn_bwd_shape(C, V, bx, by);
  int gx = cdiv(C / V, bx);
  long long target = 2048 / gx;
  long long rpb = (M + target - 1) / target;
  if (rpb < by) rpb = by;
  *rows_per_block = (int)rpb;
  return (int)((M + rpb - 1) / rpb);
}

int bn_bwd_reduce(const BnBwdArgs& a, int dtype, hipStream_t st) {
  int V = dtype == DT_F32 ? 4 : 8, bx, by;
  if (a.C % V) { set_error("bn_bwd_reduce: C=%d", a.C); return E_INVALID; }
  bn_bwd_shape(a.C, V, bx, by);
  int rpb;
  int P = bn_bwd_parts(a.M, a.C, dtype, &rpb);
  BnBwdArgs b = a;
  b.rows_per_block = rpb;
  dim3 grid(cdiv(a.C / V, bx), P), block(bx, by);
  size_t shm = (size_t)bx * by * V * 2 * sizeof(float);
  if (dtype == DT_F32) bn_bwd_reduce_kernel<float><<<grid, block, shm, st>>>(b);
  else bn_bwd_reduce_kernel<bf16><<<grid, block, shm, st>>>(b);
  return check_launch("bn_bwd_reduce");
}

// merge [P][2][C] -> dgamma, dbeta (written to the gradient arena) and coef [2][C];
// one workgroup per channel, fixed-order strided partial sums + tree (deterministic)
__global__ __launch_bounds__(256) void bn_bwd_finalize_kernel(const float* part, int P, int C,
                                                              double count, float* dgamma,
                                                              float* dbeta, float* coef) {
  const int c = blockIdx.x;
  __shared__ double r1[256], r2[256];
  double s1 = 0.0, s2 = 0.0;
  for (int p = threadIdx.x; p < P; p += 256) {
    s1 += part[(size_t)p * 2 * C + c];
    s2 += part[(size_t)p * 2 * C + C + c];
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
    if (dbeta) dbeta[c] = (float)r1[0];
    if (dgamma) dgamma[c] = (float)r2[0];
    coef[c] = (float)(r1[0] / count);
    coef[C + c] = (float)(r2[0] / count);
  }
}

int bn_bwd_finalize(const float* part, int P, int C, double count, float* dgamma, float* dbeta,
                    float* coef, hipStream_t st) {
  bn_bwd_finalize_kernel<<<C, 256, 0, st>>>(part, P, C, count, dgamma, dbeta, coef);
  return check_launch("bn_bwd_finalize");
}

// dz = scale * (dy_r - coef0 - xhat * coef1)   (train);  dz = scale * dy_r (eval: coef null)
template <typename T>
__global__ __launch_bounds__(256) void bn_bwd_apply_kernel(BnBwdArgs a) {
  constexpr int V = VecW<T>::V;
  const int CV = a.C / V;
  // 32-bit index math (M*C/V < 2^31 is enforced by the planner)
  const unsigned i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (unsigned)a.M * (unsigned)CV) return;
  const unsigned mu = i / (unsigned)CV;
  const int c = (int)(i - mu * (unsigned)CV) * V;
  const long long m = mu;
  float g[V], z[V], o[V];
  ldv((const T*)a.dy + m * a.lddy + c, g);
  if (a.mask) {
    float mk[V];
    ldv((const T*)a.mask + m * a.ldmask + c, mk);
#pragma unroll
    for (int j = 0; j < V; ++j) g[j] = mk[j] > 0.f ? g[j] : 0.f;
  }
  if (a.coef) {
    ldv((const T*)a.z + m * a.ldz + c, z);
#pragma unroll
    for (int j = 0; j < V; ++j) {
      float xh = (z[j] - a.mean[c + j]) * a.invstd[c + j];
      o[j] = a.scale[c + j] * (g[j] - a.coef[c + j] - xh * a.coef[a.C + c + j]);
    }
  } else {
#pragma unroll
    for (int j = 0; j < V; ++j) o[j] = a.scale[c + j] * g[j];
  }
  stv((T*)a.dz + m * a.lddz + c, o);
}

int bn_bwd_apply(const BnBwdArgs& a, int dtype, hipStream_t st) {
  int V = dtype == DT_F32 ? 4 : 8;
  long long total = a.M * (a.C / V);
  unsigned grid = (unsigned)((total + 255) / 256);
  if (dtype == DT_F32) bn_bwd_apply_kernel<float><<<grid, 256, 0, st>>>(a);
  else bn_bwd_apply_kernel<bf16><<<grid, 256, 0, st>>>(a);
  return check_launch("bn_bwd_apply");
}

}  // namespace fscnn
