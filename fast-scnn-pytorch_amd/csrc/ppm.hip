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
#include <type_traits>

namespace fscnn {

constexpr int PPM_T = 512;  // threads: 16 row slices x 32 channels
constexpr int PPM_C = 32;
constexpr int PPM_K = 128;  // the PPM input channels (the backward MMA form stages [M][128] rows)

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
    const float2 ss = bn_fwd_finish(b.f, tid, (double)M, s1, s2);  // s2 = sum z^2
    s_ss[0][tid] = ss.x;
    s_ss[1][tid] = ss.y;
  }
  __syncthreads();
  T* Y = (T*)b.y;
  const float sc = s_ss[0][n], sh = s_ss[1][n];
  for (int m = sl; m < M; m += 16)
    st1(Y + (size_t)m * b.ldy + n, fmaxf(fmaf(round_as<T>(s_z[m * PPM_C + n]), sc, sh), 0.f));
}

// ---- matrix-core forms (r06) ---------------------------------------------------------------
// One 16-row x 32-col tile of z = X W^T per wave on the matrix cores, in the k order of the tiled
// GEMM (gemm.hip gemm_nt_kernel), so the inference form is bit-identical to the four pointwise
// launches it replaces: chunks of 32 (fp32) / 64 (16-bit) k; fp32 inference runs the three-term
// bf16 split of both operands per chunk (X3: lane group lq supplies vectors lq and lq + 4), fp32
// training exact v_mfma_f32_16x16x4_f32 and 16-bit v_mfma_f32_16x16x32 in halves h = 0, 1 (lane
// group lq supplies vector lq + 4h).  Lanes load their fragments straight from global memory: the
// pooled rows and the 32 x 128 weights are read once per tile and stay in L2.  (The FMA forms
// walked a branch's rows on one CU: ppm_fwd_lds 27.5 us per cfg3 step, four pointwise launches
// 33 us at cfg2; a branch is at most 18 tiles.)
// Every fragment of a tile is loaded before its first MFMA (K is a compile-time 128): these
// launches are a handful of dependent memory round trips, not arithmetic.
template <typename T>
struct PpmFrag {  // one lane's k-vectors of one row: chunk c, half / split vector j
  static constexpr int V = VecW<T>::V, KC = 8 * V, NCH = PPM_K / KC;
  uint4 v[NCH][2];
  __device__ __forceinline__ void load(const T* row, int lq) {
#pragma unroll
    for (int c = 0; c < NCH; ++c)
#pragma unroll
      for (int j = 0; j < 2; ++j) v[c][j] = *reinterpret_cast<const uint4*>(row + c * KC + (lq + 4 * j) * V);
  }
};

template <typename T, bool X3>
__device__ __forceinline__ void ppm_mma(const PpmFrag<T>& a, const PpmFrag<T> (&b)[2],
                                        f32x4 (&acc)[2]) {
  constexpr int NCH = PpmFrag<T>::NCH;
#pragma unroll
  for (int nt = 0; nt < 2; ++nt) acc[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    if constexpr (X3) {
      uint4 a3[3];
      gs_split3(a.v[c][0], a.v[c][1], a3);
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) {
        uint4 b3[3];
        gs_split3(b[nt].v[c][0], b[nt].v[c][1], b3);
        gs_mma_x3(a3, b3, acc[nt]);
      }
    } else {
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int nt = 0; nt < 2; ++nt) {
          const uint4 av = a.v[c][h], bv = b[nt].v[c][h];
          if constexpr (sizeof(T) == 4) {
            acc[nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(av.x), __uint_as_float(bv.x), acc[nt], 0, 0, 0);
            acc[nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(av.y), __uint_as_float(bv.y), acc[nt], 0, 0, 0);
            acc[nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(av.z), __uint_as_float(bv.z), acc[nt], 0, 0, 0);
            acc[nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(av.w), __uint_as_float(bv.w), acc[nt], 0, 0, 0);
          } else if constexpr (std::is_same<T, f16>::value) {
            h16x8 a8, b8;
            __builtin_memcpy(&a8, &av, 16);
            __builtin_memcpy(&b8, &bv, 16);
            acc[nt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a8, b8, acc[nt], 0, 0, 0);
          } else {
            i16x8 a8, b8;
            __builtin_memcpy(&a8, &av, 16);
            __builtin_memcpy(&b8, &bv, 16);
            acc[nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a8, b8, acc[nt], 0, 0, 0);
          }
        }
    }
  }
}

// training: one workgroup per branch (its batch statistics stay block-local); wave w takes row
// tiles w + 8j (j < PPM_TPW: M <= 512); then the statistics / finish / apply of ppm_fwd_kernel
// over the stored z
constexpr int PPM_TPW = 4;
template <typename T>
__global__ __launch_bounds__(PPM_T) void ppm_fwd_mma_kernel(PpmFwdArgs a) {
  const PpmBranchFwd& b = a.b[blockIdx.x];
  const int M = b.M, tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6, li = lane & 15, lq = lane >> 4;
  extern __shared__ float sm[];
  float* s_z = sm;  // [M][C], the stored (rounded) conv output
  __shared__ double s_r[2][PPM_T];
  __shared__ float s_ss[2][PPM_C];
  const T* X = (const T*)b.x;
  const T* Wt = (const T*)b.w;
  T* Z = (T*)b.z;
  stamp(a.stamps, 0);
  PpmFrag<T> bw[2], af[PPM_TPW];
  bw[0].load(Wt + (size_t)li * PPM_K, lq);
  bw[1].load(Wt + (size_t)(16 + li) * PPM_K, lq);
#pragma unroll
  for (int j = 0; j < PPM_TPW; ++j) {
    const int r = (wave + 8 * j) * 16 + li;
    af[j].load(X + (size_t)(r < M ? r : 0) * PPM_K, lq);
  }
  f32x4 acc[PPM_TPW][2];
#pragma unroll
  for (int j = 0; j < PPM_TPW; ++j) ppm_mma<T, false>(af[j], bw, acc[j]);
  stamp(a.stamps, 1);
#pragma unroll
  for (int j = 0; j < PPM_TPW; ++j)
#pragma unroll
    for (int nt = 0; nt < 2; ++nt)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int m = (wave + 8 * j) * 16 + lq * 4 + q, c = nt * 16 + li;
        if (m < M) {
          s_z[m * PPM_C + c] = round_as<T>(acc[j][nt][q]);
          st1(Z + (size_t)m * PPM_C + c, acc[j][nt][q]);
        }
      }
  __syncthreads();
  stamp(a.stamps, 2);
  const int n = tid & 31, sl = tid >> 5;
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
    const float2 ss = bn_fwd_finish(b.f, tid, (double)M, s1, s2);
    s_ss[0][tid] = ss.x;
    s_ss[1][tid] = ss.y;
  }
  __syncthreads();
  stamp(a.stamps, 3);
  T* Y = (T*)b.y;
  const float sc = s_ss[0][n], sh = s_ss[1][n];
  for (int m = sl; m < M; m += 16)
    st1(Y + (size_t)m * b.ldy + n, fmaxf(fmaf(s_z[m * PPM_C + n], sc, sh), 0.f));
  stamp(a.stamps, 4);
}

// inference: two waves per 16-row tile of any branch, wave w the 16 output channels 16w .. 16w+15
// (each wave's MFMA sequence is the pair form's for its column tile: the same values), y =
// relu(z * scale + shift) with the folded eval BN (b.f.scale / b.f.shift as inputs), the tiled
// GEMM's epilogue arithmetic
template <typename T, bool X3>
__device__ __forceinline__ void ppm_mma1(const PpmFrag<T>& a, const PpmFrag<T>& b, f32x4& acc) {
  constexpr int NCH = PpmFrag<T>::NCH;
  acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    if constexpr (X3) {
      uint4 a3[3], b3[3];
      gs_split3(a.v[c][0], a.v[c][1], a3);
      gs_split3(b.v[c][0], b.v[c][1], b3);
      gs_mma_x3(a3, b3, acc);
    } else {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const uint4 av = a.v[c][h], bv = b.v[c][h];
        if constexpr (sizeof(T) == 4) {
          acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(av.x), __uint_as_float(bv.x), acc, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(av.y), __uint_as_float(bv.y), acc, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(av.z), __uint_as_float(bv.z), acc, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(av.w), __uint_as_float(bv.w), acc, 0, 0, 0);
        } else if constexpr (std::is_same<T, f16>::value) {
          h16x8 a8, b8;
          __builtin_memcpy(&a8, &av, 16);
          __builtin_memcpy(&b8, &bv, 16);
          acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(a8, b8, acc, 0, 0, 0);
        } else {
          i16x8 a8, b8;
          __builtin_memcpy(&a8, &av, 16);
          __builtin_memcpy(&b8, &bv, 16);
          acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a8, b8, acc, 0, 0, 0);
        }
      }
    }
  }
}

template <typename T>
__global__ __launch_bounds__(128) void ppm_eval_mma_kernel(PpmFwdArgs a) {
  int t = blockIdx.x, bi = 0;
  while (bi + 1 < a.nb && t >= (a.b[bi].M + 15) / 16) t -= (a.b[bi++].M + 15) / 16;
  const PpmBranchFwd& b = a.b[bi];
  const int M = b.M, lane = threadIdx.x & 63, nt = threadIdx.x >> 6, li = lane & 15, lq = lane >> 4;
  const int r = t * 16 + li;
  const int c = nt * 16 + li;
  PpmFrag<T> bw, af;
  bw.load((const T*)b.w + (size_t)c * PPM_K, lq);
  af.load((const T*)b.x + (size_t)(r < M ? r : 0) * PPM_K, lq);
  const float sc = b.f.scale[c], sh = b.f.shift[c];
  f32x4 acc;
  ppm_mma1<T, sizeof(T) == 4>(af, bw, acc);
  T* Y = (T*)b.y;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int m = t * 16 + lq * 4 + q;
    const float v = acc[q] * sc + sh;
    if (m < M) st1(Y + (size_t)m * b.ldy + c, fmaxf(v, 0.f));
  }
}

// G workgroups per branch (a.wg0): each recomputes the branch's BN-backward sums and dz (tiny,
// block-local, identical arithmetic in every workgroup) and then owns a 1/G slice of the weight
// gradient's k and of the input gradient's rows — one workgroup per branch was LDS-bound on the
// 288-row branch's dx (2 LDS reads per FMA on one CU)
//
// MMA (16-bit plans, K = 128, M <= 288; up to 4 workgroups per branch, r06): the branch's pooled rows are
// staged in LDS beside dz and W, and both products run on the matrix cores -- dW (32 x K, reduced
// over M) as 2 x 8 tiles of v_mfma_f32_16x16x32 over 32-row steps, dX (M x K, reduced over the 32
// channels) as one MFMA per 16 x 16 tile.  (The FMA form's weight gradient walked each k column
// of X with 56 active threads per workgroup: ppm_bwd 35 us per cfg3 step.)
template <typename T, bool MMA>
__global__ __launch_bounds__(PPM_T) void ppm_bwd_kernel(PpmBwdArgs a) {
  int bi = 0;
  while (bi + 1 < a.nb && (int)blockIdx.x >= a.wg0[bi + 1]) ++bi;
  const int gpart = blockIdx.x - a.wg0[bi], NG = a.wg0[bi + 1] - a.wg0[bi];
  const PpmBranchBwd& b = a.b[bi];
  const int K = a.K, M = b.M, tid = threadIdx.x;
  stamp(a.stamps, 0);
  const int n = tid & 31, sl = tid >> 5;
  constexpr int DZ = PPM_C + 1;  // padded dz row
  extern __shared__ float sm[];
  float* s_w = sm;                  // [C][K]
  float* s_dz = s_w + PPM_C * K;    // [M][C + 1], dz as stored (rounded)
  T* s_x = reinterpret_cast<T*>(s_dz + ((size_t)M * DZ + 3) / 4 * 4);  // (MMA) rows [M][K]
  __shared__ double s_r[2][PPM_T];
  const T* Wt = (const T*)b.w;
  // (MMA: every staging load of the workgroup is issued before the first is consumed -- compile-
  //  time counts; a loop with a runtime trip count is one memory round trip per iteration)
  constexpr int XPT = 288 * PPM_K / 8 / PPM_T;  // 9 row vectors per thread (M <= 288)
  uint4 xr[MMA ? XPT : 1], wv;
  if constexpr (MMA) {
    const uint4* xs = reinterpret_cast<const uint4*>(b.x);
    const int nv = M * PPM_K / 8;
#pragma unroll
    for (int u = 0; u < XPT; ++u) {
      const int i = tid + u * PPM_T;
      xr[u] = xs[i < nv ? i : 0];
    }
    wv = reinterpret_cast<const uint4*>(Wt)[tid];  // 32 x 128 = one 8-element vector per thread
  } else {
    for (int i = tid; i < PPM_C * K; i += PPM_T) s_w[i] = ld1(Wt + i);
  }
  const T* G = (const T*)b.dy;
  const T* Y = (const T*)b.y;
  const T* Z = (const T*)b.z;
  // BN backward in fp64 from the stored z: the branch's batch statistics are recomputed here
  // (block-local, M <= 512 values per channel) and x_hat, the sums and dz formed in fp64.  The
  // pool-1 branch normalises N values per channel (2 at batch 2): x_hat = +-a with 1 - a^2 =
  // eps / (d^2 + eps) small, so dz = scale (dy - c0 - x_hat c1) cancels to ~(1 - a^2) |dy| and
  // a float x_hat (relative error 1e-7) made it ~1 % rounding noise, which the pool backward
  // spreads over every upstream gradient.
  // the slice's rows are loaded once, RB rows per batch of loads (MMA: all 18 at once), and kept
  // for the dz pass
  constexpr int RMAX = MMA ? 18 : 32;  // rows per slice held in registers (M <= 16 * RMAX)
  constexpr int RB = MMA ? 18 : 4;
  float gr[RMAX], zr[RMAX];
  double t0 = 0.0;
  const int nr = M > sl ? (M - sl + 15) / 16 : 0;
#pragma unroll
  for (int i0 = 0; i0 < RMAX; i0 += RB) {
    if (i0 >= nr) continue;
    float g4[RB], y4[RB], z4[RB];
#pragma unroll
    for (int u = 0; u < RB; ++u) {
      const int m = sl + 16 * (i0 + u < nr ? i0 + u : 0);
      g4[u] = ld1(G + (size_t)m * b.lddy + n);
      y4[u] = ld1(Y + (size_t)m * b.ldy + n);
      z4[u] = ld1(Z + (size_t)m * PPM_C + n);
    }
#pragma unroll
    for (int u = 0; u < RB; ++u) {
      const bool ok = i0 + u < nr;
      gr[i0 + u] = (ok && y4[u] > 0.f) ? g4[u] : 0.f;
      zr[i0 + u] = ok ? z4[u] : 0.f;
      t0 += ok ? (double)z4[u] : 0.0;
    }
  }
  if constexpr (MMA) {  // the staged rows and weights into LDS (read after the dz barrier)
    const int nv = M * PPM_K / 8;
#pragma unroll
    for (int u = 0; u < XPT; ++u) {
      const int i = tid + u * PPM_T;
      if (i < nv) reinterpret_cast<uint4*>(s_x)[i] = xr[u];
    }
    float w8[8];
    unpack<T>(wv, w8);
#pragma unroll
    for (int e = 0; e < 8; ++e) s_w[tid * 8 + e] = w8[e];
  }
  stamp(a.stamps, 1);
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
  stamp(a.stamps, 2);
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
  stamp(a.stamps, 3);
  if constexpr (MMA) {
    using Op = C0Mma<std::is_same<T, f16>::value ? 2 : 1>;
    const int lane = tid & 63, wave = tid >> 6, li = lane & 15, lq = lane >> 4;
    // dW[c][k] = sum_m dz[m][c] x[m][k]: A = dz^T (row c, 8 consecutive m), B = x (col k, same m)
    // (three 32-row steps per iteration, their LDS reads issued together; steps past M add
    //  zero products)
    // (NG workgroups per branch: workgroup gpart takes tiles wave + 8 gpart + 8 NG i)
    for (int t = wave + 8 * gpart; t < 2 * (K / 16); t += 8 * NG) {
      const int ct = t & 1, kt = t >> 1;
      const int c = ct * 16 + li, k = kt * 16 + li;
      f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
      for (int m0 = 0; m0 < M; m0 += 96) {
        float av[3][8], bv[3][8];
#pragma unroll
        for (int u = 0; u < 3; ++u)
#pragma unroll
          for (int e = 0; e < 8; ++e) {  // (clamped reads + selects: a branch around each LDS
            const int m = m0 + 32 * u + lq * 8 + e;  // read serialises them: 13 us for this loop)
            const bool ok = m < M;
            const int mm = ok ? m : 0;
            const float x = ld1(s_x + (size_t)mm * K + k), d = s_dz[mm * DZ + c];
            av[u][e] = ok ? d : 0.f;
            bv[u][e] = ok ? x : 0.f;
          }
#pragma unroll
        for (int u = 0; u < 3; ++u) Op::mma(Op::pack(av[u]), Op::pack(bv[u]), acc);
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) b.dw[(size_t)(ct * 16 + lq * 4 + q) * K + k] = acc[q];
    }
    stamp(a.stamps, 4);
    // dX[m][k] = sum_c dz[m][c] W[c][k]: A = dz (row m, channels 8lq..), B = W^T (col k, same c);
    // three tiles per iteration (reads together)
    T* DX = (T*)b.dx;
    const int mt_n = (M + 15) / 16, ntile = mt_n * (K / 16);
    for (int t0 = wave + 8 * gpart; t0 < ntile; t0 += 24 * NG) {
      float av[3][8], bv[3][8];
#pragma unroll
      for (int u = 0; u < 3; ++u) {
        const int t = t0 + u * 8 * NG, tt = t < ntile ? t : t0;
        const int mt = tt % mt_n, kt = tt / mt_n;
        const int m = mt * 16 + li, k = kt * 16 + li;
        const int mm = m < M ? m : 0;  // (rows past M: garbage rows of A, never stored)
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          av[u][e] = s_dz[mm * DZ + lq * 8 + e];
          bv[u][e] = s_w[(lq * 8 + e) * K + k];
        }
      }
#pragma unroll
      for (int u = 0; u < 3; ++u) {
        const int t = t0 + u * 8 * NG;
        const int mt = t % mt_n, kt = t / mt_n;
        f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
        Op::mma(Op::pack(av[u]), Op::pack(bv[u]), acc);
        if (t < ntile) {
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int mo = mt * 16 + lq * 4 + q;
            if (mo < M) st1(DX + (size_t)mo * K + kt * 16 + li, acc[q]);
          }
        }
      }
    }
    stamp(a.stamps, 5);
    return;
  }
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
  double rows = 0.0;
  for (int i = 0; i < a.nb; ++i) rows += a.b[i].M;
  if (a.eval) {  // inference: no statistics, any M; the matrix-core form only
    if (a.nb < 1 || a.nb > 4 || a.C != PPM_C || a.K != PPM_K || maxM < 1 ||
        dtype < DT_F32 || dtype > DT_F16) {
      set_error("ppm_branches_fwd (eval): nb=%d K=%d C=%d M=%d dtype=%d not supported", a.nb, a.K,
                a.C, maxM, dtype);
      return E_UNSUPPORTED;
    }
    unsigned tiles = 0;
    for (int i = 0; i < a.nb; ++i) tiles += (unsigned)((a.b[i].M + 15) / 16);
    ProfScope ps(PK_PPM, st, rows * (a.K + PPM_C) * (dtype == DT_F32 ? 4 : 2),
                 2.0 * a.K * PPM_C * rows);
    if (dtype == DT_F32) prof_launch(ppm_eval_mma_kernel<float>, tiles, 128, 0, st, a);
    else if (dtype == DT_F16) prof_launch(ppm_eval_mma_kernel<f16>, tiles, 128, 0, st, a);
    else prof_launch(ppm_eval_mma_kernel<bf16>, tiles, 128, 0, st, a);
    return check_launch("ppm_branches_fwd");
  }
  if (!ppm_check(a.nb, a.K, a.C, maxM, dtype)) return E_INVALID;
  ProfScope ps(PK_PPM, st, rows * (a.K + 2.0 * PPM_C) * (dtype == DT_F32 ? 4 : 2),
               2.0 * a.K * PPM_C * rows);
  if (a.K == PPM_K && maxM <= 16 * 8 * PPM_TPW) {
    const size_t l2 = (size_t)maxM * PPM_C * 4;
    PpmFwdArgs as = a;
    as.stamps = stamp_region();
    if (dtype == DT_F32) prof_launch(ppm_fwd_mma_kernel<float>, a.nb, PPM_T, l2, st, as);
    else if (dtype == DT_F16) prof_launch(ppm_fwd_mma_kernel<f16>, a.nb, PPM_T, l2, st, as);
    else prof_launch(ppm_fwd_mma_kernel<bf16>, a.nb, PPM_T, l2, st, as);
    return check_launch("ppm_branches_fwd");
  }
  const size_t lds = (size_t)PPM_C * (a.K + 1) * 4 + (size_t)maxM * PPM_C * 4;
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
  b.stamps = stamp_region();
  if (dtype != DT_F32 && a.K == PPM_K && maxM <= 288) {  // one workgroup per branch
    // up to 4 workgroups per branch (one per 64 rows): each recomputes the branch's BN-backward
    // sums and dz, and takes every NG-th group of 8 dW / dX tiles (the 288-row branch's 144 dX
    // tiles were 18 per wave on one CU)
    for (int i = 0; i < a.nb; ++i) b.wg0[i + 1] = b.wg0[i] + std::max(1, std::min(4, a.b[i].M / 64));
    const size_t l2 = lds + 16 + (size_t)maxM * a.K * 2;
    if (dtype == DT_F16) prof_launch(ppm_bwd_kernel<f16, true>, b.wg0[a.nb], PPM_T, l2, st, b);
    else prof_launch(ppm_bwd_kernel<bf16, true>, b.wg0[a.nb], PPM_T, l2, st, b);
    return check_launch("ppm_branches_bwd");
  }
  for (int i = 0; i < a.nb; ++i) b.wg0[i + 1] = b.wg0[i] + std::max(1, std::min(16, a.b[i].M / 32));
  const int nwg = b.wg0[a.nb];
  if (dtype == DT_F32) prof_launch(ppm_bwd_kernel<float, false>, nwg, PPM_T, lds, st, b);
  else if (dtype == DT_F16) prof_launch(ppm_bwd_kernel<f16, false>, nwg, PPM_T, lds, st, b);
  else prof_launch(ppm_bwd_kernel<bf16, false>, nwg, PPM_T, lds, st, b);
  return check_launch("ppm_branches_bwd");
}

}  // namespace fscnn
