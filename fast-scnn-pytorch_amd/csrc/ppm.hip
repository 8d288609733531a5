// PPM branches of the training step in one launch each way (models/fast_scnn.py:123-145
// PyramidPooling: conv1..conv4 = _ConvBNReLU(128 -> 32, 1x1) on the 1/2/3/6 adaptive-pool bins).
//
// Each branch is a tiny problem (M = k*k*N pooled pixels: 8 / 32 / 72 / 288 rows at N = 8) whose
// GEMM + BN statistics + finish + apply took 3 launches forward and 5 backward through the general
// kernels (~5 us each, almost all launch latency).  Here one workgroup owns a whole branch, so the
// BatchNorm reductions are block-local: forward = conv, batch statistics (fp64, fixed order), the
// finish of bn_finish.hpp (running statistics included), ReLU apply; backward = the BN-backward sums
// + finish, dz, weight gradient (stored into the fp32 gradient arena) and input gradient.
// Arithmetic follows the general path: z rounded to the storage type, statistics of that stored
// value, y = relu(fmaf(z_stored, scale, shift)) (bn_apply), dz = scale*(g - c0 - xhat*c1) rounded
// to the storage type before both GEMMs read it (bn_bwd_apply).
#include "bn_finish.hpp"

#include <algorithm>

namespace fscnn {

constexpr int PPM_T = 512;  // threads: 16 row slices x 32 channels
constexpr int PPM_C = 32;

size_t ppm_branch_lds(int M, int K) {
  const size_t fwd = (size_t)PPM_C * (K + 1) * 4 + (size_t)M * PPM_C * 4;
  const size_t bwd = (size_t)PPM_C * K * 4 + (size_t)M * (PPM_C + 1) * 4;
  return fwd > bwd ? fwd : bwd;
}

template <typename T>
__global__ __launch_bounds__(PPM_T) void ppm_fwd_kernel(PpmFwdArgs a) {
  constexpr int V = VecW<T>::V;
  const PpmBranchFwd& b = a.b[blockIdx.x];
  const int K = a.K, M = b.M, tid = threadIdx.x;
  const int n = tid & 31, sl = tid >> 5;
  extern __shared__ float sm[];
  float* s_w = sm;                       // [C][K + 1]
  float* s_z = s_w + PPM_C * (K + 1);    // [M][C], unrounded conv output
  __shared__ double s_r[2][PPM_T];
  __shared__ float s_ss[2][PPM_C];
  const T* Wt = (const T*)b.w;
  for (int i = tid; i < PPM_C * K; i += PPM_T) {
    const int r = i / K, k = i - r * K;
    s_w[r * (K + 1) + k] = ld1(Wt + i);
  }
  __syncthreads();
  const T* X = (const T*)b.x;
  T* Z = (T*)b.z;
  const float* wr = s_w + n * (K + 1);
  // (a chunk of 8 k-vectors is loaded before its FMAs: the row walk is a chain of load
  //  round trips otherwise — the loop trip counts are runtime values)
  for (int m = sl; m < M; m += 16) {
    const T* xr = X + (size_t)m * K;
    float acc = 0.f;
    int k = 0;
    for (; k + 8 * V <= K; k += 8 * V) {
      float xv[8][V];
#pragma unroll
      for (int u = 0; u < 8; ++u) ldv(xr + k + u * V, xv[u]);
#pragma unroll
      for (int u = 0; u < 8; ++u)
#pragma unroll
        for (int j = 0; j < V; ++j) acc = fmaf(xv[u][j], wr[k + u * V + j], acc);
    }
    for (; k < K; k += V) {
      float xv[V];
      ldv(xr + k, xv);
#pragma unroll
      for (int j = 0; j < V; ++j) acc = fmaf(xv[j], wr[k + j], acc);
    }
    s_z[m * PPM_C + n] = round_as<T>(acc);  // the stored value (statistics and apply)
    st1(Z + (size_t)m * PPM_C + n, acc);
  }
  __syncthreads();
  double t1 = 0.0, t2 = 0.0;
  for (int m = sl; m < M; m += 16) {
    const double v = s_z[m * PPM_C + n];
    t1 += v;
    t2 += v * v;
  }
  s_r[0][tid] = t1;
  s_r[1][tid] = t2;
  __syncthreads();
  if (tid < PPM_C) {
    double s1 = 0.0, s2 = 0.0;
    for (int j = 0; j < 16; ++j) {
      s1 += s_r[0][j * PPM_C + tid];
      s2 += s_r[1][j * PPM_C + tid];
    }
    bn_fwd_finish(b.f, tid, (double)M, s1, s2);  // s2 = sum z^2 = sum (M2 + n mean^2)
    s_ss[0][tid] = b.f.scale[tid];
    s_ss[1][tid] = b.f.shift[tid];
  }
  __syncthreads();
  T* Y = (T*)b.y;
  const float sc = s_ss[0][n], sh = s_ss[1][n];
  for (int m = sl; m < M; m += 16)
    st1(Y + (size_t)m * b.ldy + n, fmaxf(fmaf(round_as<T>(s_z[m * PPM_C + n]), sc, sh), 0.f));
}

// 16-bit plans, K = 128 (the PPM input): the branch's whole pooled input X [M][128] is staged in
// LDS with one batch of 16-B loads per thread and each thread keeps its channel's 128 weights in
// registers, so the row walk reads only LDS (the kernel above walks its rows as a chain of
// dependent L2 round trips: 34 us for the four branches at cfg3).  Same per-row fmaf order (k
// ascending), so the values are identical.
constexpr int PPM_K = 128;
template <typename T>
__global__ __launch_bounds__(PPM_T) void ppm_fwd_lds_kernel(PpmFwdArgs a) {
  constexpr int V = VecW<T>::V;
  const PpmBranchFwd& b = a.b[blockIdx.x];
  const int M = b.M, tid = threadIdx.x;
  const int n = tid & 31, sl = tid >> 5;
  extern __shared__ float sm[];
  float* s_z = sm;                                              // [M][C], unrounded conv output
  T* s_x = reinterpret_cast<T*>(s_z + (size_t)M * PPM_C);       // [M][K]
  __shared__ double s_r[2][PPM_T];
  __shared__ float s_ss[2][PPM_C];
  const T* X = (const T*)b.x;
  {
    const int nv = M * PPM_K / V;
    constexpr int LPT = 288 * PPM_K / 8 / PPM_T;  // 9: the largest branch (M <= 288 checked)
    uint4 raw[LPT];
#pragma unroll
    for (int u = 0; u < LPT; ++u) {
      const int i = tid + u * PPM_T;
      raw[u] = *reinterpret_cast<const uint4*>(X + (size_t)(i < nv ? i : 0) * V);
    }
#pragma unroll
    for (int u = 0; u < LPT; ++u) {
      const int i = tid + u * PPM_T;
      if (i < nv) *reinterpret_cast<uint4*>(s_x + (size_t)i * V) = raw[u];
    }
  }
  float wr[PPM_K];
  const T* Wt = (const T*)b.w + (size_t)n * PPM_K;
#pragma unroll
  for (int k = 0; k < PPM_K; k += V) ldv(Wt + k, *reinterpret_cast<float(*)[V]>(&wr[k]));
  __syncthreads();
  T* Z = (T*)b.z;
  for (int m = sl; m < M; m += 16) {
    const T* xr = s_x + (size_t)m * PPM_K;
    float acc = 0.f;
#pragma unroll
    for (int k = 0; k < PPM_K; k += V) {
      float xv[V];
      ldv(xr + k, xv);
#pragma unroll
      for (int j = 0; j < V; ++j) acc = fmaf(xv[j], wr[k + j], acc);
    }
    s_z[m * PPM_C + n] = round_as<T>(acc);  // the stored value (statistics and apply)
    st1(Z + (size_t)m * PPM_C + n, acc);
  }
  __syncthreads();
  double t1 = 0.0, t2 = 0.0;
  for (int m = sl; m < M; m += 16) {
    const double v = s_z[m * PPM_C + n];
    t1 += v;
    t2 += v * v;
  }
  s_r[0][tid] = t1;
  s_r[1][tid] = t2;
  __syncthreads();
  if (tid < PPM_C) {
    double s1 = 0.0, s2 = 0.0;
    for (int j = 0; j < 16; ++j) {
      s1 += s_r[0][j * PPM_C + tid];
      s2 += s_r[1][j * PPM_C + tid];
    }
    bn_fwd_finish(b.f, tid, (double)M, s1, s2);
    s_ss[0][tid] = b.f.scale[tid];
    s_ss[1][tid] = b.f.shift[tid];
  }
  __syncthreads();
  T* Y = (T*)b.y;
  const float sc = s_ss[0][n], sh = s_ss[1][n];
  for (int m = sl; m < M; m += 16)
    st1(Y + (size_t)m * b.ldy + n, fmaxf(fmaf(round_as<T>(s_z[m * PPM_C + n]), sc, sh), 0.f));
}

// G workgroups per branch (a.wg0): each recomputes the branch's BN-backward sums and dz (tiny,
// block-local, identical arithmetic in every workgroup) and then owns a 1/G slice of the weight
// gradient's k and of the input gradient's rows — one workgroup per branch was LDS-bound on the
// 288-row branch's dx (2 LDS reads per FMA on one CU)
template <typename T>
__global__ __launch_bounds__(PPM_T) void ppm_bwd_kernel(PpmBwdArgs a) {
  int bi = 0;
  while (bi + 1 < a.nb && (int)blockIdx.x >= a.wg0[bi + 1]) ++bi;
  const int gpart = blockIdx.x - a.wg0[bi], NG = a.wg0[bi + 1] - a.wg0[bi];
  const PpmBranchBwd& b = a.b[bi];
  const int K = a.K, M = b.M, tid = threadIdx.x;
  const int n = tid & 31, sl = tid >> 5;
  constexpr int DZ = PPM_C + 1;  // padded dz row
  extern __shared__ float sm[];
  float* s_w = sm;                  // [C][K]
  float* s_dz = s_w + PPM_C * K;    // [M][C + 1], dz as stored (rounded)
  __shared__ double s_r[2][PPM_T];
  const T* Wt = (const T*)b.w;
  for (int i = tid; i < PPM_C * K; i += PPM_T) s_w[i] = ld1(Wt + i);
  const T* G = (const T*)b.dy;
  const T* Y = (const T*)b.y;
  const T* Z = (const T*)b.z;
  // BN backward in fp64 from the stored z: the branch's batch statistics are recomputed here
  // (block-local, M <= 512 values per channel) and x_hat, the sums and dz formed in fp64.  The
  // pool-1 branch normalises N values per channel (2 at batch 2): x_hat = +-a with 1 - a^2 =
  // eps / (d^2 + eps) small, so dz = scale (dy - c0 - x_hat c1) cancels to ~(1 - a^2) |dy| and
  // a float x_hat (relative error 1e-7) made it ~1 % rounding noise, which the pool backward
  // spreads over every upstream gradient.
  // the slice's rows are loaded once, 4 rows per batch of loads, and kept for the dz pass
  constexpr int RMAX = 32;  // rows per slice held in registers (M <= 16 * RMAX)
  float gr[RMAX], zr[RMAX];
  double t0 = 0.0;
  const int nr = M > sl ? (M - sl + 15) / 16 : 0;
#pragma unroll
  for (int i0 = 0; i0 < RMAX; i0 += 4) {
    if (i0 >= nr) continue;
    float g4[4], y4[4], z4[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int m = sl + 16 * (i0 + u < nr ? i0 + u : 0);
      g4[u] = ld1(G + (size_t)m * b.lddy + n);
      y4[u] = ld1(Y + (size_t)m * b.ldy + n);
      z4[u] = ld1(Z + (size_t)m * PPM_C + n);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const bool ok = i0 + u < nr;
      gr[i0 + u] = (ok && y4[u] > 0.f) ? g4[u] : 0.f;
      zr[i0 + u] = ok ? z4[u] : 0.f;
      t0 += ok ? (double)z4[u] : 0.0;
    }
  }
  // (fixed-order block sums of the 16 row slices: deterministic)
  auto colsum = [&](double v, int k) -> double {
    __syncthreads();
    s_r[k][tid] = v;
    __syncthreads();
    double r = 0.0;
    for (int j = 0; j < 16; ++j) r += s_r[k][j * PPM_C + n];
    return r;
  };
  const double mean = colsum(t0, 0) / (double)M;
  double tv = 0.0;
#pragma unroll
  for (int i = 0; i < RMAX; ++i)
    if (i < nr) tv += ((double)zr[i] - mean) * ((double)zr[i] - mean);
  const double istd = 1.0 / sqrt(colsum(tv, 1) / (double)M + (double)BN_EPS);
  double t1 = 0.0, t2 = 0.0;
#pragma unroll
  for (int i = 0; i < RMAX; ++i) {
    if (i >= nr) continue;
    t1 += (double)gr[i];
    t2 += (double)gr[i] * (((double)zr[i] - mean) * istd);
  }
  const double s1 = colsum(t1, 0), s2 = colsum(t2, 1);
  if (tid < PPM_C && gpart == 0) {  // dgamma = sum dy_r x_hat, dbeta = sum dy_r
    b.dgamma[n] = (float)s2;
    b.dbeta[n] = (float)s1;
  }
  const double c0 = s1 / (double)M, c1 = s2 / (double)M;
  const double scale = (double)b.gamma[n] * istd;
#pragma unroll
  for (int i = 0; i < RMAX; ++i) {
    if (i >= nr) continue;
    const double xh = ((double)zr[i] - mean) * istd;
    s_dz[(sl + 16 * i) * DZ + n] = round_as<T>((float)(scale * ((double)gr[i] - c0 - xh * c1)));
  }
  __syncthreads();
  // weight gradient dW[c][k] = sum_m dz[m][c] x[m][k]: thread (k, 8-channel group), m ascending
  const T* X = (const T*)b.x;
  const int kb = K * gpart / NG, ke = K * (gpart + 1) / NG, KS = ke - kb;
  for (int p = tid; p < KS * (PPM_C / 8); p += PPM_T) {
    const int k = kb + p % KS, cg = p / KS;
    float acc[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = 0.f;
    int m = 0;
    for (; m + 16 <= M; m += 16) {  // 16 loads in flight, then the FMAs in ascending m
      float xv[16];
#pragma unroll
      for (int u = 0; u < 16; ++u) xv[u] = ld1(X + (size_t)(m + u) * K + k);
#pragma unroll
      for (int u = 0; u < 16; ++u)
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] = fmaf(s_dz[(m + u) * DZ + cg * 8 + j], xv[u], acc[j]);
    }
    for (; m < M; ++m) {
      const float xv = ld1(X + (size_t)m * K + k);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] = fmaf(s_dz[m * DZ + cg * 8 + j], xv, acc[j]);
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) b.dw[(size_t)(cg * 8 + j) * K + k] = acc[j];
  }
  // input gradient dx[m][k] = sum_c dz[m][c] W[c][k]
  T* DX = (T*)b.dx;
  const int mb = M * gpart / NG, me = M * (gpart + 1) / NG;
  for (int p = mb * K + tid; p < me * K; p += PPM_T) {
    const int m = p / K, k = p - m * K;
    float acc = 0.f;
#pragma unroll 8
    for (int c = 0; c < PPM_C; ++c) acc = fmaf(s_dz[m * DZ + c], s_w[c * K + k], acc);
    st1(DX + (size_t)m * K + k, acc);
  }
}

static bool ppm_check(int nb, int K, int C, int maxM, int dtype) {
  if (nb < 1 || nb > 4 || C != PPM_C || K < 8 || K % 8 || K > 1024 || maxM < 1 || maxM > 512 ||
      ppm_branch_lds(maxM, K) > 150 * 1024 || dtype < DT_F32 || dtype > DT_F16) {
    set_error("ppm_branches: nb=%d K=%d C=%d M=%d dtype=%d not supported", nb, K, C, maxM, dtype);
    return false;
  }
  return true;
}

bool ppm_branches_ok(int maxM, int K, int dtype) {
  // maxM <= 16 slices x 32 rows: the backward keeps a slice's rows in registers
  return maxM <= 512 && ppm_branch_lds(maxM, K) <= 150 * 1024 && K >= 8 && K % 8 == 0 && K <= 1024 &&
         dtype >= DT_F32 && dtype <= DT_F16;
}

int ppm_branches_fwd(const PpmFwdArgs& a, int dtype, hipStream_t st) {
  int maxM = 0;
  for (int i = 0; i < a.nb; ++i) maxM = a.b[i].M > maxM ? a.b[i].M : maxM;
  if (!ppm_check(a.nb, a.K, a.C, maxM, dtype)) return E_INVALID;
  const size_t lds = (size_t)PPM_C * (a.K + 1) * 4 + (size_t)maxM * PPM_C * 4;
  double rows = 0.0;
  for (int i = 0; i < a.nb; ++i) rows += a.b[i].M;
  ProfScope ps(PK_PPM, st, rows * (a.K + 2.0 * PPM_C) * (dtype == DT_F32 ? 4 : 2),
               2.0 * a.K * PPM_C * rows);
  if (dtype != DT_F32 && a.K == PPM_K && maxM <= 288) {
    const size_t l2 = (size_t)maxM * PPM_C * 4 + (size_t)maxM * PPM_K * 2;
    if (dtype == DT_F16) prof_launch(ppm_fwd_lds_kernel<f16>, a.nb, PPM_T, l2, st, a);
    else prof_launch(ppm_fwd_lds_kernel<bf16>, a.nb, PPM_T, l2, st, a);
    return check_launch("ppm_branches_fwd");
  }
  if (dtype == DT_F32) prof_launch(ppm_fwd_kernel<float>, a.nb, PPM_T, lds, st, a);
  else if (dtype == DT_F16) prof_launch(ppm_fwd_kernel<f16>, a.nb, PPM_T, lds, st, a);
  else prof_launch(ppm_fwd_kernel<bf16>, a.nb, PPM_T, lds, st, a);
  return check_launch("ppm_branches_fwd");
}

int ppm_branches_bwd(const PpmBwdArgs& a, int dtype, hipStream_t st) {
  int maxM = 0;
  for (int i = 0; i < a.nb; ++i) maxM = a.b[i].M > maxM ? a.b[i].M : maxM;
  if (!ppm_check(a.nb, a.K, a.C, maxM, dtype)) return E_INVALID;
  const size_t lds = (size_t)PPM_C * a.K * 4 + (size_t)maxM * (PPM_C + 1) * 4;
  double rows = 0.0;
  for (int i = 0; i < a.nb; ++i) rows += a.b[i].M;
  ProfScope ps(PK_PPM, st, rows * (2.0 * a.K + 3.0 * PPM_C) * (dtype == DT_F32 ? 4 : 2),
               4.0 * a.K * PPM_C * rows);
  PpmBwdArgs b = a;
  b.wg0[0] = 0;
  for (int i = 0; i < a.nb; ++i) b.wg0[i + 1] = b.wg0[i] + std::max(1, std::min(16, a.b[i].M / 32));
  const int nwg = b.wg0[a.nb];
  if (dtype == DT_F32) prof_launch(ppm_bwd_kernel<float>, nwg, PPM_T, lds, st, b);
  else if (dtype == DT_F16) prof_launch(ppm_bwd_kernel<f16>, nwg, PPM_T, lds, st, b);
  else prof_launch(ppm_bwd_kernel<bf16>, nwg, PPM_T, lds, st, b);
  return check_launch("ppm_branches_bwd");
}

}  // namespace fscnn
