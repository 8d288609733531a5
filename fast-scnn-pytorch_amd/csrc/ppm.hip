// PPM branches of the training step in one launch each way (models/fast_scnn.py:123-145
// PyramidPooling: conv1..conv4 = _ConvBNReLU(128 -> 32, 1x1) on the 1/2/3/6 adaptive-pool bins).
//
// Each branch is a tiny problem (M = k*k*N pooled pixels: 8 / 32 / 72 / 288 rows at N = 8) whose
// GEMM + BN statistics + finish + apply took 3 launches forward and 5 backward through the general
// kernels (~5 us each, almost all launch latency).  Here one workgroup owns a whole branch, so the
// BatchNorm reductions are block-local: forward = conv, batch statistics (fp64, fixed order), the
// finish of bn_finish.hpp (running statistics included), ReLU apply; backward = the BN-backward sums
// + finish, dz, weight gradient (stored into the fp32 gradient arena) and input gradient.
// Arithmetic follows the general path: z rounded to the storage type, statistics of the unrounded
// value, y = relu(fmaf(z_stored, scale, shift)) (bn_apply), dz = scale*(g - c0 - xhat*c1) rounded
// to the storage type before both GEMMs read it (bn_bwd_apply).
#include "bn_finish.hpp"

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
  for (int m = sl; m < M; m += 16) {
    const T* xr = X + (size_t)m * K;
    float acc = 0.f;
    for (int k = 0; k < K; k += V) {
      float xv[V];
      ldv(xr + k, xv);
#pragma unroll
      for (int j = 0; j < V; ++j) acc = fmaf(xv[j], wr[k + j], acc);
    }
    s_z[m * PPM_C + n] = acc;
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

template <typename T>
__global__ __launch_bounds__(PPM_T) void ppm_bwd_kernel(PpmBwdArgs a) {
  const PpmBranchBwd& b = a.b[blockIdx.x];
  const int K = a.K, M = b.M, tid = threadIdx.x;
  const int n = tid & 31, sl = tid >> 5;
  constexpr int DZ = PPM_C + 1;  // padded dz row
  extern __shared__ float sm[];
  float* s_w = sm;                  // [C][K]
  float* s_dz = s_w + PPM_C * K;    // [M][C + 1], dz as stored (rounded)
  __shared__ double s_r[2][PPM_T];
  __shared__ float s_cf[2 * PPM_C];
  const T* Wt = (const T*)b.w;
  for (int i = tid; i < PPM_C * K; i += PPM_T) s_w[i] = ld1(Wt + i);
  const T* G = (const T*)b.dy;
  const T* Y = (const T*)b.y;
  const T* Z = (const T*)b.z;
  const float mean = b.mean[n], istd = b.invstd[n], scale = b.scale[n];
  // BN backward sums: dy masked by the forward ReLU (y > 0), xhat of the stored z
  double t1 = 0.0, t2 = 0.0;
  for (int m = sl; m < M; m += 16) {
    const float g = ld1(G + (size_t)m * b.lddy + n);
    const float gv = ld1(Y + (size_t)m * b.ldy + n) > 0.f ? g : 0.f;
    const float xh = (ld1(Z + (size_t)m * PPM_C + n) - mean) * istd;
    t1 += gv;
    t2 += (double)gv * xh;
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
    bn_bwd_finish(tid, PPM_C, s1, s2, (double)M, b.dgamma, b.dbeta, s_cf, BnBwdTab());
  }
  __syncthreads();
  const float c0 = s_cf[n], c1 = s_cf[PPM_C + n];
  for (int m = sl; m < M; m += 16) {
    const float g = ld1(G + (size_t)m * b.lddy + n);
    const float gv = ld1(Y + (size_t)m * b.ldy + n) > 0.f ? g : 0.f;
    const float xh = (ld1(Z + (size_t)m * PPM_C + n) - mean) * istd;
    s_dz[m * DZ + n] = round_as<T>(scale * (gv - c0 - xh * c1));
  }
  __syncthreads();
  // weight gradient dW[c][k] = sum_m dz[m][c] x[m][k]: thread (k, 8-channel group), m ascending
  const T* X = (const T*)b.x;
  for (int p = tid; p < K * (PPM_C / 8); p += PPM_T) {
    const int k = p % K, cg = p / K;
    float acc[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = 0.f;
    for (int m = 0; m < M; ++m) {
      const float xv = ld1(X + (size_t)m * K + k);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] = fmaf(s_dz[m * DZ + cg * 8 + j], xv, acc[j]);
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) b.dw[(size_t)(cg * 8 + j) * K + k] = acc[j];
  }
  // input gradient dx[m][k] = sum_c dz[m][c] W[c][k]
  T* DX = (T*)b.dx;
  for (int p = tid; p < M * K; p += PPM_T) {
    const int m = p / K, k = p - m * K;
    float acc = 0.f;
#pragma unroll 8
    for (int c = 0; c < PPM_C; ++c) acc = fmaf(s_dz[m * DZ + c], s_w[c * K + k], acc);
    st1(DX + (size_t)m * K + k, acc);
  }
}

static bool ppm_check(int nb, int K, int C, int maxM, int dtype) {
  if (nb < 1 || nb > 4 || C != PPM_C || K < 8 || K % 8 || K > 1024 || maxM < 1 ||
      ppm_branch_lds(maxM, K) > 150 * 1024 || (dtype != DT_F32 && dtype != DT_BF16)) {
    set_error("ppm_branches: nb=%d K=%d C=%d M=%d dtype=%d not supported", nb, K, C, maxM, dtype);
    return false;
  }
  return true;
}

bool ppm_branches_ok(int maxM, int K, int dtype) {
  return ppm_branch_lds(maxM, K) <= 150 * 1024 && K >= 8 && K % 8 == 0 && K <= 1024 &&
         (dtype == DT_F32 || dtype == DT_BF16);
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
  if (dtype == DT_F32) ppm_fwd_kernel<float><<<a.nb, PPM_T, lds, st>>>(a);
  else ppm_fwd_kernel<bf16><<<a.nb, PPM_T, lds, st>>>(a);
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
  if (dtype == DT_F32) ppm_bwd_kernel<float><<<a.nb, PPM_T, lds, st>>>(a);
  else ppm_bwd_kernel<bf16><<<a.nb, PPM_T, lds, st>>>(a);
  return check_launch("ppm_branches_bwd");
}

}  // namespace fscnn
