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
#include "bn_finish.hpp"

namespace fscnn {

// ---- eval fold of every BN in one launch ------------------------------------------------------

__global__ void bn_fold_kernel(FoldTable t) {
  const FoldEntry& e = t.e[blockIdx.x];
  for (int c = threadIdx.x; c < e.C; c += blockDim.x) {
    float s = e.gamma[c] / sqrtf(e.rvar[c] + BN_EPS);
    float b = e.bias ? e.bias[c] : 0.f;
    e.scale[c] = s;
    e.shift[c] = e.beta[c] + (b - e.rmean[c]) * s;
    if (e.mean) {
      e.mean[c] = e.rmean[c];
      e.invstd[c] = 1.f / sqrtf(e.rvar[c] + BN_EPS);
    }
  }
}

int bn_fold(const FoldTable& t, hipStream_t st) {
  if (t.n <= 0 || t.n > MAX_FOLD) {
    set_error("bn_fold: bad table size %d", t.n);
    return E_INVALID;
  }
  prof_launch(bn_fold_kernel, t.n, 256, 0, st, t);
  return check_launch("bn_fold");
}

// ---- train: merge partial records ------------------------------------------------------------
// Two coalesced levels, in place (the records are consumed), workgroups of 64 channels x BN_TY:
//   fold : workgroup (64-channel chunk, q) — thread (c, ty) merges records p = q + Q*(ty + TY*k),
//          i.e. every record of residue class q mod Q, which no other thread touches; the TY
//          partials are summed in fixed order and the result overwrites record slot q.
//   final: workgroup per 64-channel chunk merges slots 0..Q-1 (fixed order) and finishes.
// Merges run in fp64 on (n, n*mean, M2 + n*mean^2) sums (no division until the end: an fp64
// divide is a ~40-instruction sequence, and a chain of them dominated the finalize); lanes walk
// channels, so every record row is read as contiguous 256-B segments.
constexpr int BN_Q = 64;
constexpr int BN_TY = 16;

__device__ __forceinline__ void bn_stats_fold_body(float* part, int P, int C, int Q) {
  __shared__ double sh[3][BN_TY][64];
  const int cx = threadIdx.x, ty = threadIdx.y;
  const int c = blockIdx.x * 64 + cx, q = blockIdx.y;
  double n = 0.0, s1 = 0.0, s2 = 0.0;
  if (c < C) {
    // batches of 8 records: all loads issued before the fp64 accumulation (no serialized trips)
    for (int p0 = q + Q * ty; p0 < P; p0 += 8 * BN_TY * Q) {
      float rm[8], r2[8], rn[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int p = p0 + BN_TY * Q * u;
        const float* rec = part + (size_t)(p < P ? p : p0) * 3 * C;  // clamped + select
        const float t0 = rec[c], t1 = rec[C + c], t2 = rec[2 * C + c];
        rm[u] = p < P ? t0 : 0.f;
        r2[u] = p < P ? t1 : 0.f;
        rn[u] = p < P ? t2 : 0.f;
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const double cn = rn[u], m = rm[u];
        n += cn;
        s1 += cn * m;
        s2 += (double)r2[u] + cn * m * m;
      }
    }
  }
  sh[0][ty][cx] = n;
  sh[1][ty][cx] = s1;
  sh[2][ty][cx] = s2;
  __syncthreads();
  if (ty == 0 && c < C) {
    n = s1 = s2 = 0.0;
#pragma unroll
    for (int t = 0; t < BN_TY; ++t) {
      n += sh[0][t][cx];
      s1 += sh[1][t][cx];
      s2 += sh[2][t][cx];
    }
    float* rec = part + (size_t)q * 3 * C;
    const double mean = n > 0.0 ? s1 / n : 0.0;
    st_wt(rec + c, (float)mean);
    st_wt(rec + C + c, n > 0.0 ? (float)fmax(s2 - n * mean * mean, 0.0) : 0.f);
    st_wt(rec + 2 * C + c, (float)n);
  }
}

__global__ __launch_bounds__(1024) void bn_stats_fold_kernel(float* part, int P, int C, int Q) {
  bn_stats_fold_body(part, P, C, Q);
}

// merge the Q <= BN_Q folded records of channels [64*chunk, 64*chunk + 64) and finish
__device__ __forceinline__ void bn_finalize_chunk(const BnFinalizeArgs& a, int Q, int chunk) {
  __shared__ double sh[3][BN_TY][64];
  const int cx = threadIdx.x, ty = threadIdx.y;
  const int c = chunk * 64 + cx;
  BnFwdIn in;  // the finish's inputs, in flight with the record loads
  if (ty == 0 && c < a.C) in = bn_fwd_load(a, c);
  double n = 0.0, s1 = 0.0, s2 = 0.0;
  if (c < a.C) {
    constexpr int U = BN_Q / BN_TY;
    float rm[U], r2[U], rn[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int q = ty + BN_TY * u;
      const float* rec = a.part + (size_t)(q < Q ? q : 0) * 3 * a.C;  // clamped + select
      const float t0 = ld_wt(rec + 2 * a.C + c), t1 = ld_wt(rec + c), t2 = ld_wt(rec + a.C + c);
      rn[u] = q < Q ? t0 : 0.f;
      rm[u] = q < Q ? t1 : 0.f;
      r2[u] = q < Q ? t2 : 0.f;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const double cn = rn[u], m = rm[u];
      n += cn;
      s1 += cn * m;
      s2 += (double)r2[u] + cn * m * m;
    }
  }
  sh[0][ty][cx] = n;
  sh[1][ty][cx] = s1;
  sh[2][ty][cx] = s2;
  __syncthreads();
  if (ty != 0 || c >= a.C) return;
  n = s1 = s2 = 0.0;
#pragma unroll
  for (int t = 0; t < BN_TY; ++t) {
    n += sh[0][t][cx];
    s1 += sh[1][t][cx];
    s2 += sh[2][t][cx];
  }
  bn_fwd_finish(a, c, n, s1, s2, in);
}

__global__ __launch_bounds__(1024) void bn_finalize_kernel(BnFinalizeArgs a, int Q) {
  bn_finalize_chunk(a, Q, blockIdx.x);
}

// Fold + finalize in ONE launch: every (chunk, q) workgroup folds its residue class into slot q
// (write-through stores), then arrives on the chunk's counter (common.hpp arrive_last); the last
// workgroup of a chunk reads the slots back with sc1 loads and finishes the chunk.  Counters are
// zero on entry (zeroed by the step's weights_prep launch) and reset by the last arriver.
__global__ __launch_bounds__(1024) void bn_stats_fold_fin_kernel(BnFinalizeArgs a, int Q,
                                                                 unsigned* ctr) {
  bn_stats_fold_body(a.part, a.P, a.C, Q);
  if (!arrive_last(ctr + blockIdx.x, gridDim.y)) return;
  bn_finalize_chunk(a, Q, blockIdx.x);
  reset_counter(ctr + blockIdx.x);
}

int bn_finalize(const BnFinalizeArgs& a, hipStream_t st) {
  if (a.P <= 0 || a.C <= 0) {
    set_error("bn_finalize: P=%d C=%d", a.P, a.C);
    return E_INVALID;
  }
  ProfScope ps(PK_BN_FIN, st, 12.0 * a.P * a.C, 0.0);
  int Q = a.P;
  const dim3 blk(64, BN_TY);
  if (a.P > BN_Q) {
    Q = BN_Q;
    if (a.counters) {
      prof_launch(bn_stats_fold_fin_kernel, dim3(cdiv(a.C, 64), Q), blk, 0, st, a, Q, a.counters);
      return check_launch("bn_finalize");
    }
    prof_launch(bn_stats_fold_kernel, dim3(cdiv(a.C, 64), Q), blk, 0, st, a.part, a.P, a.C, Q);
  }
  prof_launch(bn_finalize_kernel, cdiv(a.C, 64), blk, 0, st, a, Q);
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
  for (int j = 0; j < V; ++j) o[j] = fmaf(z[j], a.scale[c + j], a.shift[c + j]);  // == relu_z mask
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
  ProfScope ps(PK_BN_APPLY, st,
               (dtype == DT_F32 ? 4.0 : 2.0) * a.M * a.C *
                   (2 + (a.z2 ? 1 : 0) + (a.res ? 1 : 0)),
               0.0);
  unsigned grid = (unsigned)((total + 255) / 256);
  if (dtype == DT_F32) prof_launch(bn_apply_kernel<float>, grid, 256, 0, st, a);
  else if (dtype == DT_F16) prof_launch(bn_apply_kernel<f16>, grid, 256, 0, st, a);
  else prof_launch(bn_apply_kernel<bf16>, grid, 256, 0, st, a);
  return check_launch("bn_apply");
}

// ---- backward -------------------------------------------------------------------------------
// dy_r = dy * [mask > 0] (mask = the saved post-activation output, if the BN is followed by a
// ReLU or the FFM's ReLU), xhat = (z - mean) * invstd.

// MODE: 0 = no ReLU, 1 = mask tensor (y > 0), 2 = relu_z (mask recomputed from z).  The mode is
// a template parameter and rows past the end are clamped + zero-weighted, so a batch's loads are
// issued back to back with no branch (a branch between loads and use forces vmcnt(0) waits).
// PAIR (mask mode): a second BN on the same dy and mask (BnBwdArgs::z2): its sum of dy_r*xhat2
// comes from the same pass (dy and the mask read once); its sum of dy_r is the first BN's
template <typename T, int MODE, bool PAIR = false>
__global__ __launch_bounds__(256) void bn_bwd_reduce_kernel(BnBwdArgs a) {
  constexpr int V = VecW<T>::V;
  constexpr int NS = PAIR ? 3 : 2;  // sums per channel: s1, s2 (, s3)
  const int CV = a.C / V;
  // block = (channel vectors along x, row groups along y)
  const int cv = blockIdx.x * blockDim.x + threadIdx.x;
  const int BX = blockDim.x, BY = blockDim.y;
  extern __shared__ float red[];  // [BY][BX*V*NS]
  float s1[V], s2[V], s3[PAIR ? V : 1];
#pragma unroll
  for (int j = 0; j < V; ++j) { s1[j] = 0.f; s2[j] = 0.f; if constexpr (PAIR) s3[j] = 0.f; }
  if (cv < CV) {
    const int c = cv * V;
    float mu[V], is[V], fs[V], fb[V], mu2[PAIR ? V : 1], is2[PAIR ? V : 1];
#pragma unroll
    for (int j = 0; j < V; ++j) {
      mu[j] = a.mean[c + j];
      is[j] = a.invstd[c + j];
      if (MODE == 2) {
        fs[j] = a.scale[c + j];
        fb[j] = a.shift[c + j];
      }
      if constexpr (PAIR) {
        mu2[j] = a.mean2[c + j];
        is2[j] = a.invstd2[c + j];
      }
    }
    const long long mb = (long long)blockIdx.y * a.rows_per_block;
    const long long me = min(a.M, mb + a.rows_per_block);
    constexpr int U = 4;  // rows per batch (8 measured slower: 256 VGPRs, occupancy 2)
    for (long long m0 = mb + threadIdx.y; m0 < me; m0 += U * BY) {
      float g[U][V], z[U][V], mk[U][V], z2[PAIR ? U : 1][V];
      float ok[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const long long mr = m0 + (long long)u * BY;
        ok[u] = mr < me ? 1.f : 0.f;
        const long long m = mr < me ? mr : me - 1;
        ldv((const T*)a.dy + m * a.lddy + c, g[u]);
        ldv((const T*)a.z + m * a.ldz + c, z[u]);
        if (MODE == 1) ldv((const T*)a.mask + m * a.ldmask + c, mk[u]);
        if constexpr (PAIR) ldv((const T*)a.z2 + m * a.ldz + c, z2[u]);
      }
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int j = 0; j < V; ++j) {
          float gv = g[u][j] * ok[u];
          if (MODE == 1) gv = mk[u][j] > 0.f ? gv : 0.f;
          if (MODE == 2) gv = fmaf(z[u][j], fs[j], fb[j]) > 0.f ? gv : 0.f;
          s1[j] += gv;
          s2[j] += gv * (z[u][j] - mu[j]) * is[j];
          if constexpr (PAIR) s3[j] += gv * (z2[u][j] - mu2[j]) * is2[j];
        }
    }
  }
#pragma unroll
  for (int j = 0; j < V; ++j) {
    red[(threadIdx.y * BX + threadIdx.x) * NS * V + j] = s1[j];
    red[(threadIdx.y * BX + threadIdx.x) * NS * V + V + j] = s2[j];
    if constexpr (PAIR) red[(threadIdx.y * BX + threadIdx.x) * NS * V + 2 * V + j] = s3[j];
  }
  __syncthreads();
  if (threadIdx.y == 0 && cv < CV) {
    float* rec = a.part + (size_t)blockIdx.y * 2 * a.C;
    float* rec2 = PAIR ? a.part2 + (size_t)blockIdx.y * 2 * a.C : nullptr;
#pragma unroll
    for (int j = 0; j < V; ++j) {
      float t1 = 0.f, t2 = 0.f, t3 = 0.f;
      for (int k = 0; k < BY; ++k) {
        t1 += red[(k * BX + threadIdx.x) * NS * V + j];
        t2 += red[(k * BX + threadIdx.x) * NS * V + V + j];
        if constexpr (PAIR) t3 += red[(k * BX + threadIdx.x) * NS * V + 2 * V + j];
      }
      rec[cv * V + j] = t1;
      rec[a.C + cv * V + j] = t2;
      if constexpr (PAIR) {
        rec2[cv * V + j] = t1;
        rec2[a.C + cv * V + j] = t3;
      }
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
  ProfScope ps(PK_BN_BWD_RED, st, (dtype == DT_F32 ? 4.0 : 2.0) * a.M * a.C * (a.mask ? 3 : 2),
               0.0);
  BnBwdArgs b = a;
  b.rows_per_block = rpb;
  dim3 grid(cdiv(a.C / V, bx), P), block(bx, by);
  size_t shm = (size_t)bx * by * V * (a.z2 ? 3 : 2) * sizeof(float);
  const int mode = b.relu_z ? 2 : (b.mask ? 1 : 0);
  if (a.z2) {  // paired BNs (mask mode)
    if (mode != 1 || !a.part2 || !a.mean2 || !a.invstd2) {
      set_error("bn_bwd_reduce: a paired BN needs the mask mode and its own records / statistics");
      return E_INVALID;
    }
    if (dtype == DT_F32) prof_launch(bn_bwd_reduce_kernel<float, 1, true>, grid, block, shm, st, b);
    else if (dtype == DT_F16) prof_launch(bn_bwd_reduce_kernel<f16, 1, true>, grid, block, shm, st, b);
    else prof_launch(bn_bwd_reduce_kernel<bf16, 1, true>, grid, block, shm, st, b);
    return check_launch("bn_bwd_reduce");
  }
#define BN_RED(T, M) prof_launch(bn_bwd_reduce_kernel<T, M>, grid, block, shm, st, b)
  if (dtype == DT_F32) {
    if (mode == 0) BN_RED(float, 0); else if (mode == 1) BN_RED(float, 1); else BN_RED(float, 2);
  } else if (dtype == DT_F16) {
    if (mode == 0) BN_RED(f16, 0); else if (mode == 1) BN_RED(f16, 1); else BN_RED(f16, 2);
  } else {
    if (mode == 0) BN_RED(bf16, 0); else if (mode == 1) BN_RED(bf16, 1); else BN_RED(bf16, 2);
  }
#undef BN_RED
  return check_launch("bn_bwd_reduce");
}

// merge [P][2][C] -> dgamma, dbeta (written to the gradient arena) and coef [2][C]; same
// two-level in-place scheme as bn_finalize (fold residue classes mod Q, then fixed-order merge)
__device__ __forceinline__ void bn_bwd_fold_body(float* part, int P, int C, int Q) {
  __shared__ double sh[2][BN_TY][64];
  const int cx = threadIdx.x, ty = threadIdx.y;
  const int c = blockIdx.x * 64 + cx, q = blockIdx.y;
  double s1 = 0.0, s2 = 0.0;
  if (c < C)
    for (int p0 = q + Q * ty; p0 < P; p0 += 8 * BN_TY * Q) {
      float a1[8], a2[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int p = p0 + BN_TY * Q * u;
        const size_t pc = (size_t)(p < P ? p : p0) * 2 * C;  // clamped + select
        const float t1 = part[pc + c], t2 = part[pc + C + c];
        a1[u] = p < P ? t1 : 0.f;
        a2[u] = p < P ? t2 : 0.f;
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        s1 += a1[u];
        s2 += a2[u];
      }
    }
  sh[0][ty][cx] = s1;
  sh[1][ty][cx] = s2;
  __syncthreads();
  if (ty == 0 && c < C) {
    s1 = s2 = 0.0;
#pragma unroll
    for (int t = 0; t < BN_TY; ++t) {
      s1 += sh[0][t][cx];
      s2 += sh[1][t][cx];
    }
    st_wt(part + (size_t)q * 2 * C + c, (float)s1);
    st_wt(part + (size_t)q * 2 * C + C + c, (float)s2);
  }
}

__global__ __launch_bounds__(1024) void bn_bwd_fold_kernel(float* part, int P, int C, int Q) {
  bn_bwd_fold_body(part, P, C, Q);
}

__device__ __forceinline__ void bn_bwd_finalize_chunk(const float* part, int Q, int C, double count,
                                                      float* dgamma, float* dbeta, float* coef,
                                                      int chunk, const BnBwdTab& t) {
  __shared__ double sh[2][BN_TY][64];
  const int cx = threadIdx.x, ty = threadIdx.y;
  const int c = chunk * 64 + cx;
  BnBwdIn in;  // the finish's inputs, in flight with the record loads
  if (ty == 0 && c < C) in = bn_bwd_load(t, c);
  double s1 = 0.0, s2 = 0.0;
  if (c < C) {
    constexpr int U = BN_Q / BN_TY;
    float a1[U], a2[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int q = ty + BN_TY * u;
      const size_t qc = (size_t)(q < Q ? q : 0) * 2 * C;  // clamped + select
      const float t1 = ld_wt(part + qc + c), t2 = ld_wt(part + qc + C + c);
      a1[u] = q < Q ? t1 : 0.f;
      a2[u] = q < Q ? t2 : 0.f;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      s1 += a1[u];
      s2 += a2[u];
    }
  }
  sh[0][ty][cx] = s1;
  sh[1][ty][cx] = s2;
  __syncthreads();
  if (ty != 0 || c >= C) return;
  s1 = s2 = 0.0;
#pragma unroll
  for (int t = 0; t < BN_TY; ++t) {
    s1 += sh[0][t][cx];
    s2 += sh[1][t][cx];
  }
  bn_bwd_finish(c, C, s1, s2, count, dgamma, dbeta, coef, t, in);
}

__global__ __launch_bounds__(1024) void bn_bwd_finalize_kernel(const float* part, int Q, int C,
                                                               double count, float* dgamma,
                                                               float* dbeta, float* coef,
                                                               BnBwdTab t) {
  bn_bwd_finalize_chunk(part, Q, C, count, dgamma, dbeta, coef, blockIdx.x, t);
}

__global__ __launch_bounds__(1024) void bn_bwd_fold_fin_kernel(float* part, int P, int C, int Q,
                                                               double count, float* dgamma,
                                                               float* dbeta, float* coef,
                                                               unsigned* ctr, BnBwdTab t) {
  bn_bwd_fold_body(part, P, C, Q);
  if (!arrive_last(ctr + blockIdx.x, gridDim.y)) return;
  bn_bwd_finalize_chunk(part, Q, C, count, dgamma, dbeta, coef, blockIdx.x, t);
  reset_counter(ctr + blockIdx.x);
}

int bn_bwd_finalize(float* part, int P, int C, double count, float* dgamma, float* dbeta,
                    float* coef, hipStream_t st, unsigned* counters, const BnBwdTab& tab) {
  ProfScope ps(PK_BN_FIN, st, 8.0 * P * C, 0.0);
  int Q = P;
  const dim3 blk(64, BN_TY);
  if (P > BN_Q) {
    Q = BN_Q;
    if (counters) {
      prof_launch(bn_bwd_fold_fin_kernel, dim3(cdiv(C, 64), Q), blk, 0, st, part, P, C, Q, count, dgamma,
                                                                  dbeta, coef, counters, tab);
      return check_launch("bn_bwd_finalize");
    }
    prof_launch(bn_bwd_fold_kernel, dim3(cdiv(C, 64), Q), blk, 0, st, part, P, C, Q);
  }
  prof_launch(bn_bwd_finalize_kernel, cdiv(C, 64), blk, 0, st, part, Q, C, count, dgamma, dbeta, coef, tab);
  return check_launch("bn_bwd_finalize");
}

// dz = scale * (dy_r - coef0 - xhat * coef1)   (train);  dz = scale * dy_r (eval: coef null)
// Each thread owns ONE channel vector c: its per-channel tables (scale, shift, mean, invstd, the
// two coefficients; the second BN's for PAIR) are loaded once into registers, and the thread
// sweeps pixels mu0, mu0 + P, mu0 + 2P, ... (the grid covers P pixels x all CV channel vectors per
// sweep, so every sweep is one contiguous, coalesced span of the tensor).  U pixels' loads are
// issued back to back (clamped rows, stores predicated) before their use.  The per-element
// arithmetic is unchanged, so dz is bit-identical to a one-vector-per-thread pass — that form
// re-read 6 table vectors (12 16-B loads) for every 2 data loads.
// the BN-backward output with streaming (non-temporal) stores: its consumer is the next launch,
// and fewer dirty L2 lines are left for the kernel boundary to write back (r05 A/B: 5.737 / 5.742
// vs 5.754 / 5.746 ms per cfg3 step)
__device__ __forceinline__ void stv_o(float* p, const float (&v)[4]) {
  typedef float f4 __attribute__((ext_vector_type(4)));
  f4 t = {v[0], v[1], v[2], v[3]};
  __builtin_nontemporal_store(t, (f4*)p);
}
template <typename T> __device__ __forceinline__ void stv_o(T* p, const float (&v)[8]) {
  typedef unsigned u4 __attribute__((ext_vector_type(4)));
  u4 w;
#pragma unroll
  for (int i = 0; i < 4; ++i) w[i] = (uint32_t)s16_from<T>(v[2 * i]) | ((uint32_t)s16_from<T>(v[2 * i + 1]) << 16);
  __builtin_nontemporal_store(w, (u4*)p);
}
template <typename T, int MODE, bool TRAIN, bool PAIR, int U>
__global__ __launch_bounds__(256) void bn_bwd_apply_kernel(BnBwdArgs a, unsigned P) {
  constexpr int V = VecW<T>::V;
  const unsigned CV = (unsigned)(a.C / V);
  const unsigned i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= P * CV) return;
  const unsigned mu0 = i / CV;
  const int c = (int)(i - mu0 * CV) * V;
  constexpr bool SH = MODE == 2, ST = TRAIN;
  float t_sc[V], t_sh[SH ? V : 1], t_mn[ST ? V : 1], t_is[ST ? V : 1], t_c0[ST ? V : 1],
      t_c1[ST ? V : 1];
  float p_mn[PAIR ? V : 1], p_is[PAIR ? V : 1], p_sc[PAIR ? V : 1], p_c0[PAIR ? V : 1],
      p_c1[PAIR ? V : 1];
#pragma unroll
  for (int j = 0; j < V; ++j) {
    t_sc[j] = a.scale[c + j];
    if constexpr (SH) t_sh[j] = a.shift[c + j];
    if constexpr (ST) {
      t_mn[j] = a.mean[c + j];
      t_is[j] = a.invstd[c + j];
      t_c0[j] = a.coef[c + j];
      t_c1[j] = a.coef[a.C + c + j];
    }
    if constexpr (PAIR) {
      p_mn[j] = a.mean2[c + j];
      p_is[j] = a.invstd2[c + j];
      p_sc[j] = a.scale2[c + j];
      p_c0[j] = a.coef2[c + j];
      p_c1[j] = a.coef2[a.C + c + j];
    }
  }
  const long long M = a.M;
  for (long long m0 = mu0; m0 < M; m0 += (long long)U * P) {
    float g[U][V], z[U][V], mk[U][V], z2[PAIR ? U : 1][V];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long long mm = m0 + (long long)u * P;
      const long long m = mm < M ? mm : m0;
      ldv((const T*)a.dy + m * a.lddy + c, g[u]);
      if (TRAIN || MODE == 2) ldv((const T*)a.z + m * a.ldz + c, z[u]);
      if (MODE == 1) ldv((const T*)a.mask + m * a.ldmask + c, mk[u]);
      if constexpr (PAIR) ldv((const T*)a.z2 + m * a.ldz + c, z2[u]);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long long m = m0 + (long long)u * P;
      if (m >= M) break;
      if constexpr (PAIR) {  // second BN on the same dy and mask (train, mask mode)
        float o2[V];
#pragma unroll
        for (int j = 0; j < V; ++j) {
          const float gv = mk[u][j] > 0.f ? g[u][j] : 0.f;
          const float xh = (z2[u][j] - p_mn[j]) * p_is[j];
          o2[j] = p_sc[j] * (gv - p_c0[j] - xh * p_c1[j]);
        }
        stv_o((T*)a.dz2 + m * a.lddz + c, o2);
      }
      float o[V];
#pragma unroll
      for (int j = 0; j < V; ++j) {
        float gv = g[u][j];
        if (MODE == 1) gv = mk[u][j] > 0.f ? gv : 0.f;
        if constexpr (SH) gv = fmaf(z[u][j], t_sc[j], t_sh[j]) > 0.f ? gv : 0.f;
        if constexpr (ST) {
          const float xh = (z[u][j] - t_mn[j]) * t_is[j];
          o[j] = t_sc[j] * (gv - t_c0[j] - xh * t_c1[j]);
        } else {
          o[j] = t_sc[j] * gv;
        }
      }
      stv_o((T*)a.dz + m * a.lddz + c, o);
    }
  }
}

template <typename T, int U>
static void bn_bwd_apply_launch_u(const BnBwdArgs& a, unsigned P, hipStream_t st) {
  const int mode = a.relu_z ? 2 : (a.mask ? 1 : 0);
  const unsigned grid = (unsigned)(((long long)P * (a.C / VecW<T>::V) + 255) / 256);
  if (a.z2) prof_launch(bn_bwd_apply_kernel<T, 1, true, true, (U > 2 ? 2 : U)>, grid, 256, 0, st, a, P);
  else if (a.coef) {
    if (mode == 0) prof_launch(bn_bwd_apply_kernel<T, 0, true, false, U>, grid, 256, 0, st, a, P);
    else if (mode == 1) prof_launch(bn_bwd_apply_kernel<T, 1, true, false, U>, grid, 256, 0, st, a, P);
    else prof_launch(bn_bwd_apply_kernel<T, 2, true, false, U>, grid, 256, 0, st, a, P);
  } else {
    if (mode == 0) prof_launch(bn_bwd_apply_kernel<T, 0, false, false, U>, grid, 256, 0, st, a, P);
    else if (mode == 1) prof_launch(bn_bwd_apply_kernel<T, 1, false, false, U>, grid, 256, 0, st, a, P);
    else prof_launch(bn_bwd_apply_kernel<T, 2, false, false, U>, grid, 256, 0, st, a, P);
  }
}

// U = pixels in flight per thread: 4 when a thread sweeps >= 4 pixels, else 1 (a one-pixel
// thread would issue U - 1 clamped duplicate loads)
template <typename T>
static void bn_bwd_apply_launch(const BnBwdArgs& a, hipStream_t st) {
  const unsigned P = chan_sweep(a.M, a.C / VecW<T>::V);
  if ((a.M + P - 1) / P >= 4) bn_bwd_apply_launch_u<T, 4>(a, P, st);
  else bn_bwd_apply_launch_u<T, 1>(a, P, st);
}

int bn_bwd_apply(const BnBwdArgs& a, int dtype, hipStream_t st) {
  if (a.z2) {  // paired BNs: train, mask mode
    if (!a.mask || !a.coef || !a.coef2 || !a.dz2 || !a.mean2 || !a.invstd2 || !a.scale2) {
      set_error("bn_bwd_apply: a paired BN needs the mask mode, both coefficient sets and dz2");
      return E_INVALID;
    }
  }
  ProfScope ps(PK_BN_BWD, st,
               a.z2 ? (dtype == DT_F32 ? 4.0 : 2.0) * a.M * a.C * 6
                    : (dtype == DT_F32 ? 4.0 : 2.0) * a.M * a.C *
                          (2 + (a.coef || a.relu_z ? 1 : 0) + (a.mask ? 1 : 0)),
               0.0);
  if (dtype == DT_F32) bn_bwd_apply_launch<float>(a, st);
  else if (dtype == DT_F16) bn_bwd_apply_launch<f16>(a, st);
  else bn_bwd_apply_launch<bf16>(a, st);
  return check_launch("bn_bwd_apply");
}


}  // namespace fscnn
