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
    float v = 0.f;
    if (c < ncol) {
      size_t off = (((size_t)n * 3 + ci) * a.H + (2 * ho + r)) * a.W + col0 + c;
      v = a.x_bf16 ? bf2f(((const uint16_t*)a.x)[off]) : ((const float*)a.x)[off];
    }
    s_in[i] = v;
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
// dW[co][ci][kh][kw] = sum_{n,ho,wo} dZ[n,ho,wo,co] * x[n,ci,2ho+kh,2wo+kw].
// One workgroup per (row of output pixels, 256-wide segment), like the forward; each thread
// owns one pixel, the 27 input taps and the 32 dZ values, and the block reduces the 864
// products over its pixels through LDS.  Output: partial slab [part][864] (deterministic
// reduction by reduce_slabs).

template <typename T>
__global__ __launch_bounds__(256) void conv0_wgrad_kernel(Conv0WgradArgs a) {
  // Each thread accumulates 864/256 ~ 3.4 weights over all pixels of the block's rows: thread
  // t owns outputs o = t, t+256, t+512, t+768 (<864).  Per pixel tile the inputs and dZ are
  // staged in LDS.
  __shared__ float s_in[3 * 3 * C0_IN_W];
  __shared__ float s_dz[C0_TILE * 33];
  const int tid = threadIdx.x;
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
  int oo[4], oco[4], otap[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    oo[j] = tid + 256 * j;
    oco[j] = oo[j] / 27;
    otap[j] = oo[j] - oco[j] * 27;
  }
  const int wo0 = blockIdx.x * C0_TILE;
  const int npx = min(C0_TILE, a.Wo - wo0);
  const int col0 = 2 * wo0;
  const int ncol = min(C0_IN_W, a.W - col0);
  const int nrows = a.N * a.Ho;
  for (int rr = 0; rr < a.rows_per_block; ++rr) {
    int row = blockIdx.y * a.rows_per_block + rr;
    if (row >= nrows) break;
    int n = row / a.Ho, ho = row - n * a.Ho;
    __syncthreads();
    for (int i = tid; i < 9 * C0_IN_W; i += 256) {
      int cr = i / C0_IN_W, c = i - cr * C0_IN_W;
      int ci = cr / 3, r = cr - ci * 3;
      float v = 0.f;
      if (c < ncol) {
        size_t off = (((size_t)n * 3 + ci) * a.H + (2 * ho + r)) * a.W + col0 + c;
        v = a.x_bf16 ? bf2f(((const uint16_t*)a.x)[off]) : ((const float*)a.x)[off];
      }
      s_in[i] = v;
    }
    const T* dz = (const T*)a.dz + ((size_t)row * a.Wo + wo0) * C0_OUT;
    for (int i = tid; i < C0_TILE * C0_OUT; i += 256) {
      int p = i >> 5, c = i & 31;
      s_dz[p * 33 + c] = (p < npx) ? ld1(dz + i) : 0.f;
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (oo[j] < 27 * C0_OUT) {
        int ci = otap[j] / 9, rc = otap[j] - ci * 9;
        int r = rc / 3, c = rc - r * 3;
        const float* xin = &s_in[(ci * 3 + r) * C0_IN_W + c];
        float s = 0.f;
        for (int p = 0; p < npx; ++p) s = fmaf(s_dz[p * 33 + oco[j]], xin[2 * p], s);
        acc[j] += s;
      }
    }
  }
  size_t pi = (size_t)blockIdx.y * gridDim.x + blockIdx.x;
#pragma unroll
  for (int j = 0; j < 4; ++j)
    if (oo[j] < 27 * C0_OUT) a.slab[pi * 864 + oo[j]] = acc[j];
}

int conv0_wgrad_parts(int N, int Ho, int Wo, int rows_per_block) {
  return cdiv(N * Ho, rows_per_block) * cdiv(Wo, C0_TILE);
}

int conv0_wgrad(const Conv0WgradArgs& a, int dz_dtype, hipStream_t st) {
  dim3 grid(cdiv(a.Wo, C0_TILE), cdiv(a.N * a.Ho, a.rows_per_block));
  if (dz_dtype == DT_F32)
    conv0_wgrad_kernel<float><<<grid, 256, 0, st>>>(a);
  else
    conv0_wgrad_kernel<bf16><<<grid, 256, 0, st>>>(a);
  return check_launch("conv0_wgrad");
}

}  // namespace fscnn
