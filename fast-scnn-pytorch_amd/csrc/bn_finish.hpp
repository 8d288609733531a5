// Per-channel BatchNorm finish arithmetic shared by the finalize kernels (bn.hip) and the
// in-kernel finish of the streaming GEMM producers (gemm_stream.hip): one definition, so both
// paths give bit-identical mean / invstd / scale / shift / running statistics / coefficients.
#pragma once
#include "kernels.hpp"

namespace fscnn {

constexpr float BN_EPS = 1e-5f;

// forward: fp64 sums over the merged records, n = sum count, s1 = sum n*mean,
// s2 = sum (M2 + n*mean^2) -> mean / invstd / scale / shift and aten's running-stat update
// (unbiased variance n/(n-1), momentum) of channel c.  The per-channel inputs are loaded apart
// (bn_fwd_load) so an in-kernel finisher can issue them before its last fold: a load after a
// store through a pointer that may alias it is its own memory round trip, and this runs at the
// very end of a producer (r06: gamma, beta, rmean, rvar were up to four dependent round trips
// behind the stores).  Returns (scale, shift).
struct BnFwdIn {
  float g = 0.f, be = 0.f, rm = 0.f, rv = 0.f;
  double bias = 0.0;
  long long nb = 0;
};
__device__ __forceinline__ BnFwdIn bn_fwd_load(const BnFinalizeArgs& a, int c) {
  BnFwdIn r;
  r.g = a.gamma[c];
  r.be = a.beta[c];
  r.bias = a.bias ? (double)a.bias[c] : 0.0;
  if (a.rmean) {
    r.rm = a.rmean[c];
    r.rv = a.rvar[c];
  }
  if (a.nbt && c == 0) r.nb = a.nbt[0];
  return r;
}
__device__ __forceinline__ float2 bn_fwd_finish(const BnFinalizeArgs& a, int c, double n,
                                                double s1, double s2, const BnFwdIn& in) {
  const double mu = n > 0.0 ? s1 / n : 0.0;
  const double m2 = n > 0.0 ? fmax(s2 - n * mu * mu, 0.0) : 0.0;
  const double mean = mu + in.bias;
  const double var = n > 0 ? m2 / n : 0.0;
  const float invstd = (float)(1.0 / sqrt(var + (double)BN_EPS));
  const float scale = in.g * invstd;
  const float shift = in.be - (float)mean * scale;
  a.mean[c] = (float)mean;
  a.invstd[c] = invstd;
  a.scale[c] = scale;
  a.shift[c] = shift;
  if (a.rmean) {
    const float m = a.momentum;
    a.rmean[c] = (1.f - m) * in.rm + m * (float)mean;
    const float unb = n > 1 ? (float)(m2 / (n - 1.0)) : (float)var;
    a.rvar[c] = (1.f - m) * in.rv + m * unb;
  }
  if (a.nbt && c == 0) a.nbt[0] = in.nb + 1;
  return make_float2(scale, shift);
}
__device__ __forceinline__ float2 bn_fwd_finish(const BnFinalizeArgs& a, int c, double n,
                                                double s1, double s2) {
  return bn_fwd_finish(a, c, n, s1, s2, bn_fwd_load(a, c));
}

// backward: s1 = sum dy_r, s2 = sum dy_r * xhat of channel c (C channels) -> dbeta, dgamma, the
// apply coefficients and (t.tab) the BN-backward operand table
// dz = scale*(dy_r - c0 - (z - mean)*invstd*c1) = al*dy_r + gz*z + be
// count == BN_FROZEN_COUNT: a BN normalised with its running statistics (eval-mode autograd,
// models/fast_scnn.py in .eval() with grad enabled): mean and invstd are constants, so the batch
// terms vanish (c0 = c1 = 0) and dz = scale * dy_r; dgamma / dbeta keep their sums.  (Inputs
// loaded apart, as in the forward.)
struct BnBwdIn {
  float sc = 0.f, isd = 0.f, mu = 0.f, sh = 1.f;
};
__device__ __forceinline__ BnBwdIn bn_bwd_load(const BnBwdTab& t, int c) {
  BnBwdIn r;
  if (t.tab) {
    r.sc = t.scale[c];
    r.isd = t.invstd[c];
    r.mu = t.mean[c];
    if (t.relu) r.sh = t.shift[c];
  }
  return r;
}
__device__ __forceinline__ void bn_bwd_finish(int c, int C, double s1, double s2, double count,
                                              float* dgamma, float* dbeta, float* coef,
                                              const BnBwdTab& t, const BnBwdIn& in) {
  if (dbeta) dbeta[c] = (float)s1;
  if (dgamma) dgamma[c] = (float)s2;
  const bool frozen = count == BN_FROZEN_COUNT;
  const float c0 = frozen ? 0.f : (float)(s1 / count), c1 = frozen ? 0.f : (float)(s2 / count);
  coef[c] = c0;
  coef[C + c] = c1;
  if (t.tab) {
    const float gz = -in.sc * c1 * in.isd;
    float4 v;
    v.x = in.sc;
    v.y = -in.sc * c0 - gz * in.mu;
    v.z = gz;
    v.w = t.relu ? in.sc : 0.f;
    float* e = t.tab + (size_t)c * BWDX_STRIDE;
    *reinterpret_cast<float4*>(e) = v;
    e[4] = in.sh;
  }
}
__device__ __forceinline__ void bn_bwd_finish(int c, int C, double s1, double s2, double count,
                                              float* dgamma, float* dbeta, float* coef,
                                              const BnBwdTab& t) {
  bn_bwd_finish(c, C, s1, s2, count, dgamma, dbeta, coef, t, bn_bwd_load(t, c));
}

// ---- generic in-kernel finish over per-workgroup records ----------------------------------
// For producers whose workgroup writes ONE record row p < P of records part[P][R][N] (R = 3:
// mean, M2, count; R = 2: s1, s2) for a contiguous channel slice [c0, c0 + nc), stored with
// write-through stores (st_wt).  Same protocol as the streaming GEMM's finish (common.hpp
// arrive_last): workgroups arrive in teams of TS consecutive rows; a team's last arriver folds
// the team's rows into the team's first row; the channel chunk's last team arriver folds the
// team rows and finishes each channel with the finalize kernels' arithmetic.  Every fold is one
// or two batches of loads deep (TS <= 2 * 8 * slices, nteam <= TAIL_TMAX).  fp64 sums in fixed
// order: deterministic run to run.  Counters: ctr[chunk], ctr[TAIL_TEAM0 + chunk*TAIL_TMAX + team].
constexpr int TAIL_TEAM0 = 64;
constexpr int TAIL_TMAX = 32;
__host__ __device__ inline int tail_team_size(int P) {
  const int t = (P + TAIL_TMAX - 1) / TAIL_TMAX;
  return t < 16 ? 16 : t;
}
// whether a producer with P record rows and `chunks` channel chunks fits the counter budget
__host__ __device__ inline bool tail_fits(int P, int chunks) {
  return P > 0 && P <= 64 * TAIL_TMAX && chunks <= (BN_COUNTERS - TAIL_TEAM0) / TAIL_TMAX &&
         chunks <= TAIL_TEAM0;
}
constexpr int TAIL_CMAX = 1024;  // channels of the team-sum scratch (Plan::tsum)

__device__ __forceinline__ void st_wt64(double* p, double v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double ld_wt64(const double* p) {
  return __hip_atomic_load(const_cast<double*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// fold of `count` rows for channels [c0, c0 + nc) (nc <= workgroup size): TEAM = false reads
// the float records part[first + i][R][N] (R = 3 forward (mean, M2, count), 2 backward);
// TEAM = true reads the fp64 team sums tsum[i][3][N] (n, s1, s2).  Returns (n, s1, s2) sums in
// the slice-0 threads (tid < nc).
template <bool FWD, bool TEAM>
__device__ inline void tail_fold(const float* part, const double* tsum, int N, int c0, int nc,
                                 int first, int count, double* s_f, double (&sum)[3]) {
  const int tid = threadIdx.x + blockDim.x * (threadIdx.y + blockDim.y * threadIdx.z);
  const int nthr = blockDim.x * blockDim.y * blockDim.z;  // <= 256, >= nc
  const int S = nthr / nc;
  const int col = tid % nc, sl = tid / nc;
  const int n = c0 + col;
  constexpr int R = TEAM ? 3 : (FWD ? 3 : 2);
  // rows per thread per batch (all loads before the sums): the last arriver's fold is a chain of
  // dependent write-through load batches at the END of its producer, so it wants few, wide ones
  constexpr int U = R == 3 ? 8 : 16;
  double t0 = 0.0, t1 = 0.0, t2 = 0.0;
  if (sl < S && n < N) {
    for (int i0 = sl; i0 < count; i0 += U * S) {
      double v[U][R];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int i = i0 + u * S;
        const int row = first + (i < count ? i : i0);
#pragma unroll
        for (int j = 0; j < R; ++j) {
          if constexpr (TEAM) v[u][j] = ld_wt64(tsum + ((size_t)row * 3 + j) * N + n);
          else v[u][j] = ld_wt(part + ((size_t)row * R + j) * N + n);
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (i0 + u * S >= count) break;
        if constexpr (TEAM) {
          t0 += v[u][0];
          t1 += v[u][1];
          t2 += v[u][2];
        } else if constexpr (FWD) {  // (mean, M2, count) -> (n, n*mean, M2 + n*mean^2)
          const double cn = v[u][2], m = v[u][0];
          t0 += cn;
          t1 += cn * m;
          t2 += v[u][1] + cn * m * m;
        } else {
          t1 += v[u][0];
          t2 += v[u][1];
        }
      }
    }
  }
  __syncthreads();  // s_f free (a previous fold's / the kernel's readers are done)
  s_f[tid] = t0;
  s_f[nthr + tid] = t1;
  s_f[2 * nthr + tid] = t2;
  __syncthreads();
  sum[0] = sum[1] = sum[2] = 0.0;
  if (sl == 0) {
    for (int j = 0; j < S; ++j) {
      sum[0] += s_f[j * nc + col];
      sum[1] += s_f[nthr + j * nc + col];
      sum[2] += s_f[2 * nthr + j * nc + col];
    }
  }
}

// First half, every workgroup after its record stores (st_wt): true in the team's last arriver.
// Producers that store a large output tile call it BEFORE those stores, so the arrival's vmcnt(0)
// drain covers only the records.
__device__ inline bool tail_arrive(int P, int p, int chunk, const BnTail& t) {
  const int TS = tail_team_size(P);
  const int team = p / TS;
  const int tsize = min(TS, P - team * TS);
  return arrive_last(t.counters + TAIL_TEAM0 + chunk * TAIL_TMAX + team, (unsigned)tsize);
}

// Second half, in a team's last arriver (every thread of it): fold the team's rows into its fp64
// team sums, arrive on the chunk, and (chunk's last team) finish every channel.  Channel slices
// wider than the workgroup are folded in passes of nthr channels.  The team sums stay fp64
// (t.tsum): a float team row would round the batch mean to fp32 before the final fold, which is
// visible in x_hat wherever |mean| >> std.
// lds: >= 3 * workgroup-size doubles of LDS the kernel no longer reads (aliased scratch, so
// kernels that never finish in-kernel carry no extra LDS)
template <bool FWD>
__device__ inline void tail_complete(float* part, int P, int N, int p, int c0, int nc, int chunk,
                                     const BnTail& t, double* lds) {
  unsigned* ctr = t.counters;
  const int TS = tail_team_size(P);
  const int team = p / TS, nteam = (P + TS - 1) / TS;
  const int tsize = min(TS, P - team * TS);
  const int tid = threadIdx.x + blockDim.x * (threadIdx.y + blockDim.y * threadIdx.z);
  const int nthr = blockDim.x * blockDim.y * blockDim.z;
  for (int cb = 0; cb < nc; cb += nthr) {
    const int ncb = min(nthr, nc - cb), n = c0 + cb + tid;
    double s[3];
    tail_fold<FWD, false>(part, nullptr, N, c0 + cb, ncb, team * TS, tsize, lds, s);
    if (tid < ncb && n < N) {
#pragma unroll
      for (int j = 0; j < 3; ++j) st_wt64(t.tsum + ((size_t)team * 3 + j) * N + n, s[j]);
    }
  }
  reset_counter(ctr + TAIL_TEAM0 + chunk * TAIL_TMAX + team);
  if (!arrive_last(ctr + chunk, (unsigned)nteam)) return;
  for (int cb = 0; cb < nc; cb += nthr) {
    const int ncb = min(nthr, nc - cb), n = c0 + cb + tid;
    const bool own = tid < ncb && n < N;
    BnFwdIn fin;  // the finish's inputs in flight with the fold's loads
    BnBwdIn bin;
    if (own) {
      if constexpr (FWD) fin = bn_fwd_load(t.fwd, n);
      else bin = bn_bwd_load(t.tab, n);
    }
    double s[3];
    tail_fold<FWD, true>(nullptr, t.tsum, N, c0 + cb, ncb, 0, nteam, lds, s);
    if (own) {
      if constexpr (FWD) bn_fwd_finish(t.fwd, n, s[0], s[1], s[2], fin);
      else bn_bwd_finish(n, N, s[1], s[2], t.count, t.dgamma, t.dbeta, t.coef, t.tab, bin);
    }
  }
  reset_counter(ctr + chunk);
}

// both halves, for producers whose records are their last stores
template <bool FWD>
__device__ inline void tail_finish(float* part, int P, int N, int p, int c0, int nc, int chunk,
                                   const BnTail& t, double* lds) {
  if (tail_arrive(P, p, chunk, t)) tail_complete<FWD>(part, P, N, p, c0, nc, chunk, t, lds);
}

}  // namespace fscnn
