// LearningToDownsample.conv: dense 3x3, stride 2, PADDING 0, 3 -> 32 channels, no bias
// (models/fast_scnn.py:153 with the _ConvBNReLU default padding=0 at :52).
//
// Reads the caller's NCHW image (fp32 or bf16) directly and writes NHWC [N,Ho,Wo,32].
// One workgroup = one output row segment of 256 pixels: the 3 input rows x (2*256+1) columns x
// 3 channels it needs are staged once in LDS (coalesced), each thread computes one pixel x 32
// channels with the 864 weights broadcast from LDS, and the 256x32 tile is written back through
// LDS as one contiguous, fully coalesced block.  HBM-bound: 12 B (fp32 in) read + 128 B written
// per output pixel against 1,728 flops.
#include "kernels.hpp"

namespace fscnn {

constexpr int C0_OUT = 32;
constexpr int C0_TILE = 256;             // output pixels per workgroup
constexpr int C0_IN_W = 2 * C0_TILE + 1;  // staged input columns
constexpr int C0_OSTR = 36;              // LDS floats per staged output pixel (16B aligned)


template <typename TO>
__global__ __launch_bounds__(256) void conv0_fwd_kernel(Conv0Args a) {
  __shared__ float s_in[3 * 3 * C0_IN_W];          // [ci][r][col]
  __shared__ float s_w[27 * C0_OUT];               // [tap][co]
  __shared__ __attribute__((aligned(16))) float s_out[C0_TILE * C0_OSTR];
  __shared__ float s_red[8 * C0_OUT];

  const int tid = threadIdx.x;
  const int wo0 = blockIdx.x * C0_TILE;
  const int row = blockIdx.y;  // n * Ho + ho
  const int n = row / a.Ho, ho = row - n * a.Ho;
  const int npx = min(C0_TILE, a.Wo - wo0);

  for (int i = tid; i < 27 * C0_OUT; i += 256) {
    int co = i / 27, t = i - co * 27;
    s_w[t * C0_OUT + co] = a.w[i];
  }
  const int col0 = 2 * wo0;
  const int ncol = min(C0_IN_W, a.W - col0);
  for (int i = tid; i < 9 * C0_IN_W; i += 256) {
    int cr = i / C0_IN_W, c = i - cr * C0_IN_W;  // cr = ci*3 + r
    int ci = cr / 3, r = cr - ci * 3;
    const bool ok = c < ncol;  // clamped load + select (branch-free)
    const size_t off = (((size_t)n * 3 + ci) * a.H + (2 * ho + r)) * a.W + col0 + (ok ? c : 0);
    const float v = a.x_bf16 ? bf2f(((const uint16_t*)a.x)[off]) : ((const float*)a.x)[off];
    s_in[i] = ok ? v : 0.f;
  }
  __syncthreads();

  float acc[C0_OUT];
#pragma unroll
  for (int co = 0; co < C0_OUT; ++co) acc[co] = 0.f;
  if (tid < npx) {
#pragma unroll
    for (int ci = 0; ci < 3; ++ci)
#pragma unroll
      for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int c = 0; c < 3; ++c) {
          float v = s_in[(ci * 3 + r) * C0_IN_W + 2 * tid + c];
          const float4* wp = reinterpret_cast<const float4*>(&s_w[((ci * 3 + r) * 3 + c) * C0_OUT]);
#pragma unroll
          for (int q = 0; q < C0_OUT / 4; ++q) {
            float4 w4 = wp[q];
            acc[4 * q + 0] = fmaf(v, w4.x, acc[4 * q + 0]);
            acc[4 * q + 1] = fmaf(v, w4.y, acc[4 * q + 1]);
            acc[4 * q + 2] = fmaf(v, w4.z, acc[4 * q + 2]);
            acc[4 * q + 3] = fmaf(v, w4.w, acc[4 * q + 3]);
          }
        }
  }
  // epilogue: BN fold (+ReLU) in eval, raw in train
#pragma unroll
  for (int co = 0; co < C0_OUT; ++co) {
    float v = acc[co];
    if (a.scale) v = v * a.scale[co] + a.shift[co];
    if (a.relu) v = fmaxf(v, 0.f);
    acc[co] = v;
  }
#pragma unroll
  for (int q = 0; q < C0_OUT / 4; ++q)
    *reinterpret_cast<float4*>(&s_out[tid * C0_OSTR + 4 * q]) =
        make_float4(acc[4 * q], acc[4 * q + 1], acc[4 * q + 2], acc[4 * q + 3]);
  __syncthreads();

  // coalesced store of npx*32 contiguous elements
  constexpr int V = VecW<TO>::V;
  TO* y = (TO*)a.y + ((size_t)row * a.Wo + wo0) * C0_OUT;
  const int nvec = npx * C0_OUT / V;
  for (int i = tid; i < nvec; i += 256) {
    int p = (i * V) / C0_OUT, c = (i * V) - p * C0_OUT;
    float v[V];
#pragma unroll
    for (int j = 0; j < V; ++j) v[j] = s_out[p * C0_OSTR + c + j];
    stv(y + (size_t)i * V, v);
  }

  if (a.part) {
    // per-channel (mean, M2, count) over this block's npx pixels: thread = (channel, group of 8)
    const int c = tid & 31, g = tid >> 5;
    float s = 0.f;
    for (int p = g; p < npx; p += 8) s += s_out[p * C0_OSTR + c];
    s_red[g * C0_OUT + c] = s;
    __syncthreads();
    float mean = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) mean += s_red[k * C0_OUT + c];
    mean /= (float)npx;
    __syncthreads();
    float m2 = 0.f;
    for (int p = g; p < npx; p += 8) {
      float d = s_out[p * C0_OSTR + c] - mean;
      m2 += d * d;
    }
    s_red[g * C0_OUT + c] = m2;
    __syncthreads();
    if (g == 0) {
      float t = 0.f;
#pragma unroll
      for (int k = 0; k < 8; ++k) t += s_red[k * C0_OUT + c];
      size_t pi = (size_t)blockIdx.y * gridDim.x + blockIdx.x;
      float* rec = a.part + pi * 3 * C0_OUT;
      rec[c] = mean;
      rec[C0_OUT + c] = t;
      rec[2 * C0_OUT + c] = (float)npx;
    }
  }
}

int conv0_parts(int N, int Ho, int Wo) { return N * Ho * cdiv(Wo, C0_TILE); }

int conv0_fwd(const Conv0Args& a, int y_dtype, hipStream_t st) {
  if (a.Ho != (a.H - 3) / 2 + 1 || a.Wo != (a.W - 3) / 2 + 1 || a.H < 3 || a.W < 3) {
    set_error("conv0_fwd: bad shape H=%d W=%d Ho=%d Wo=%d", a.H, a.W, a.Ho, a.Wo);
    return E_INVALID;
  }
  dim3 grid(cdiv(a.Wo, C0_TILE), a.N * a.Ho);
  const double px = (double)a.N * a.Ho * a.Wo;
  ProfScope ps(PK_CONV0_FWD, st,
               (a.x_bf16 ? 2.0 : 4.0) * a.N * 3.0 * a.H * a.W + (y_dtype == DT_F32 ? 4.0 : 2.0) * px * 32,
               2.0 * 27 * 32 * px);
  if (y_dtype == DT_F32)
    conv0_fwd_kernel<float><<<grid, 256, 0, st>>>(a);
  else
    conv0_fwd_kernel<bf16><<<grid, 256, 0, st>>>(a);
  return check_launch("conv0_fwd");
}

// ---- weight gradient --------------------------------------------------------------------------
// dW[co][ci][kh][kw] = sum_{n,ho,wo} dZ[n,ho,wo,co] * x[n,ci,2ho+kh,2wo+kw] is a GEMM with
// M = 32 taps (27 used), N = 32 output channels and K = N*Ho*Wo pixels (4.2 M at cfg3):
// dW^T[tap][co] = sum_p X[p][tap] dZ[p][co].  Each workgroup walks pixel tiles (256 pixels of one
// output row) grid-stride; per tile it stages X^T[tap][p] (gathered from the NCHW image) and
// dZ^T[co][p] (transposed from the NHWC gradient) in LDS, so every MFMA operand is one 16-B
// ds_read per lane (8 consecutive pixels).  Wave w owns pixels [64w, 64w+64) of the tile and
// keeps the full 32x32 accumulator (4 tiles of 16x16); the 4 waves are summed through LDS at the
// end and one [864] partial per workgroup is written (reduced in fixed order by reduce_slabs).
// HBM-bound: the x strip and the dZ tile are read once.
constexpr int CW_TP = 256;  // pixels per tile
constexpr int CW_MAXP = 1024;  // max workgroups (partials)

template <typename T>
struct CwOps;

template <>
struct CwOps<float> {
  static constexpr int LD = CW_TP + 4;  // LDS row stride (elements)
  static __device__ __forceinline__ void mma(const float* a, const float* b, f32x4& acc) {
    // 8 consecutive pixels per lane group; 8 k-steps of 16x16x4 (k = 8*lq + m)
    const float4 a0 = *reinterpret_cast<const float4*>(a), a1 = *reinterpret_cast<const float4*>(a + 4);
    const float4 b0 = *reinterpret_cast<const float4*>(b), b1 = *reinterpret_cast<const float4*>(b + 4);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a0.x, b0.x, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a0.y, b0.y, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a0.z, b0.z, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a0.w, b0.w, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a1.x, b1.x, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a1.y, b1.y, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a1.z, b1.z, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a1.w, b1.w, acc, 0, 0, 0);
  }
};

template <>
struct CwOps<bf16> {
  static constexpr int LD = CW_TP + 8;
  static __device__ __forceinline__ void mma(const bf16* a, const bf16* b, f32x4& acc) {
    i16x8 av, bv;
    __builtin_memcpy(&av, a, 16);
    __builtin_memcpy(&bv, b, 16);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, bv, acc, 0, 0, 0);
  }
};

template <typename T>
__device__ __forceinline__ T cw_cvt(float v);
template <>
__device__ __forceinline__ float cw_cvt<float>(float v) { return v; }
template <>
__device__ __forceinline__ bf16 cw_cvt<bf16>(float v) {
  bf16 r;
  r.x = f2bf(v);
  return r;
}

template <typename T>
__global__ __launch_bounds__(256) void conv0_wgrad_kernel(Conv0WgradArgs a) {
  constexpr int LD = CwOps<T>::LD;
  constexpr int V = VecW<T>::V;
  constexpr int SX = 32 * LD * sizeof(T);
  constexpr int BYTES = 2 * SX > 4 * 1024 * 4 ? 2 * SX : 4 * 1024 * 4;
  __shared__ __attribute__((aligned(16))) unsigned char s_raw[BYTES];
  T* sX = reinterpret_cast<T*>(s_raw);        // [32 taps][LD]
  T* sD = reinterpret_cast<T*>(s_raw + SX);   // [32 co][LD]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int li = lane & 15, lq = lane >> 4;
  const int segs = cdiv(a.Wo, CW_TP);
  const long long tiles = (long long)a.N * a.Ho * segs;
  const size_t HW = (size_t)a.H * a.W;

  // taps 27..31 of X^T stay zero
  for (int i = tid; i < 5 * LD; i += 256) sX[27 * LD + i] = cw_cvt<T>(0.f);
  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  for (long long t = blockIdx.x; t < tiles; t += gridDim.x) {
    const int seg = (int)(t % segs);
    const long long row = t / segs;  // n * Ho + ho
    const int n = (int)(row / a.Ho), ho = (int)(row - (long long)n * a.Ho);
    const int wo0 = seg * CW_TP;
    const int npx = min(CW_TP, a.Wo - wo0);
    // ---- global loads first (registers), then one barrier, then LDS writes -----------------
    // X^T: thread = pixel p, 27 taps
    float xv[27];
    {
      const int p = tid;
      const bool ok = p < npx;
#pragma unroll
      for (int cr = 0; cr < 9; ++cr) {
        const int ci = cr / 3, kh = cr - ci * 3;
        const size_t base = ((size_t)n * 3 + ci) * HW + (size_t)(2 * ho + kh) * a.W + 2 * (wo0 + p);
#pragma unroll
        for (int kw = 0; kw < 3; ++kw) {
          const size_t o = ok ? base + kw : 0;  // clamped load + select (branch-free)
          const float v = a.x_bf16 ? bf2f(((const uint16_t*)a.x)[o]) : ((const float*)a.x)[o];
          xv[cr * 3 + kw] = ok ? v : 0.f;
        }
      }
    }
    // dZ tile: npx*32 contiguous elements as 16-B vectors (V elements), transposed into sD
    constexpr int NV = CW_TP * 32 / V / 256;  // vectors per thread (4 bf16 / 8 f32)
    uint4 dv[NV];
    const T* dz = (const T*)a.dz + ((size_t)row * a.Wo + wo0) * 32;
#pragma unroll
    for (int q = 0; q < NV; ++q) {
      const int i = tid + 256 * q;
      const int p = (i * V) >> 5;
      dv[q] = sel4(p < npx, *reinterpret_cast<const uint4*>(dz + (size_t)(p < npx ? i : 0) * V));
    }
    __syncthreads();  // previous tile's MFMA reads are done
#pragma unroll
    for (int k = 0; k < 27; ++k) sX[k * LD + tid] = cw_cvt<T>(xv[k]);
#pragma unroll
    for (int q = 0; q < NV; ++q) {
      const int i = tid + 256 * q;
      const int p = (i * V) >> 5, c0 = (i * V) & 31;
      const T* e = reinterpret_cast<const T*>(&dv[q]);
#pragma unroll
      for (int j = 0; j < V; ++j) sD[(c0 + j) * LD + p] = e[j];
    }
    __syncthreads();
    // ---- MFMA: wave's 64 pixels, 2 steps of 32 ------------------------------------------------
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int kb = wave * 64 + ks * 32 + 8 * lq;
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          CwOps<T>::mma(&sX[(16 * i + li) * LD + kb], &sD[(16 * j + li) * LD + kb], acc[i][j]);
    }
  }
  // ---- sum the 4 waves' 32x32 accumulators; acc[i][j][r] = dW^T[16i + 4lq + r][16j + li] -----
  __syncthreads();
  float* red = reinterpret_cast<float*>(s_raw);  // [4 waves][32 tap][32 co]
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        red[wave * 1024 + (16 * i + 4 * lq + r) * 32 + 16 * j + li] = acc[i][j][r];
  __syncthreads();
  float* out = a.slab + (size_t)blockIdx.x * 864;
  for (int o = tid; o < 864; o += 256) {
    const int co = o / 27, tap = o - co * 27;
    const int k = tap * 32 + co;
    out[o] = (red[k] + red[1024 + k]) + (red[2048 + k] + red[3072 + k]);
  }
}

int conv0_wgrad_parts(int N, int Ho, int Wo, int) {
  const long long tiles = (long long)N * Ho * cdiv(Wo, CW_TP);
  return (int)(tiles < CW_MAXP ? tiles : CW_MAXP);
}

int conv0_wgrad(const Conv0WgradArgs& a, int dz_dtype, hipStream_t st) {
  const int P = conv0_wgrad_parts(a.N, a.Ho, a.Wo, 0);
  if ((uintptr_t)a.dz % 16) {
    set_error("conv0_wgrad: dZ must be 16-B aligned");
    return E_INVALID;
  }
  const double px = (double)a.N * a.Ho * a.Wo;
  ProfScope ps(PK_CONV0_WGRAD, st,
               (a.x_bf16 ? 2.0 : 4.0) * a.N * 3.0 * a.H * a.W + (dz_dtype == DT_F32 ? 4.0 : 2.0) * px * 32,
               2.0 * 27 * 32 * px);
  if (dz_dtype == DT_F32)
    conv0_wgrad_kernel<float><<<P, 256, 0, st>>>(a);
  else
    conv0_wgrad_kernel<bf16><<<P, 256, 0, st>>>(a);
  return check_launch("conv0_wgrad");
}

}  // namespace fscnn
