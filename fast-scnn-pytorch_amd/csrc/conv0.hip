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


// MFMA helpers for the im2col GEMM out[px][co] = sum_k patch[px][k] * W[co][k], K = 27 -> 32:
// lane (li, lq) supplies k = 8*lq .. 8*lq+7 for its row (pixel li / channel li).
template <int BF>
struct C0Mma;
template <>
struct C0Mma<2> {  // fp16 operands (inference plans of dtype fp16): v_mfma_f32_16x16x32_f16
  using Frag = h16x8;
  static __device__ __forceinline__ Frag pack(const float (&v)[8]) {
    Frag f;
#pragma unroll
    for (int e = 0; e < 8; ++e) f[e] = (_Float16)v[e];
    return f;
  }
  static __device__ __forceinline__ void mma(const Frag& a, const Frag& b, f32x4& acc) {
    acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, acc, 0, 0, 0);
  }
};
template <>
struct C0Mma<1> {  // bf16 operands, one v_mfma_f32_16x16x32_bf16 per 16 px x 16 co
  using Frag = i16x8;
  static __device__ __forceinline__ Frag pack(const float (&v)[8]) {
    Frag f;
#pragma unroll
    for (int e = 0; e < 8; ++e) f[e] = (short)f2bf(v[e]);
    return f;
  }
  static __device__ __forceinline__ void mma(const Frag& a, const Frag& b, f32x4& acc) {
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc, 0, 0, 0);
  }
};
template <>
struct C0Mma<0> {  // exact fp32: 8 x v_mfma_f32_16x16x4_f32 (k = 8*lq + e)
  struct Frag { float v[8]; };
  static __device__ __forceinline__ Frag pack(const float (&v)[8]) {
    Frag f;
#pragma unroll
    for (int e = 0; e < 8; ++e) f.v[e] = v[e];
    return f;
  }
  static __device__ __forceinline__ void mma(const Frag& a, const Frag& b, f32x4& acc) {
#pragma unroll
    for (int e = 0; e < 8; ++e) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.v[e], b.v[e], acc, 0, 0, 0);
  }
};

// XCD-contiguous block order: linear blocks L = x (mod 8) share an XCD, so residue class x takes
// the contiguous logical range [x*T/8, (x+1)*T/8) of (segment, row) in segment-fastest order.
// Output row ho reads input rows 2ho..2ho+2, so row ho+1 re-reads row 2ho+2: with consecutive
// rows on one XCD back to back that re-read is an L2 hit instead of a second HBM fetch.
__device__ __forceinline__ void c0_tile(int& seg, int& row) {
  const int gx = gridDim.x;
  const long long T = (long long)gx * gridDim.y;
  long long L = blockIdx.x + (long long)gx * blockIdx.y;
  if ((T & 7) == 0) L = (L & 7) * (T >> 3) + (L >> 3);
  seg = (int)(L % gx);
  row = (int)(L / gx);
}

template <typename TO, int XB>
__global__ __launch_bounds__(256) void conv0_fwd_kernel(Conv0Args a) {
  // 16-bit output => MFMA operands in that dtype (the plan's compute dtype)
  constexpr int BF = sizeof(TO) == 4 ? 0 : (std::is_same<TO, f16>::value ? 2 : 1);
  using M = C0Mma<BF>;
  using TI = typename std::conditional<XB != 0, uint16_t, float>::type;
  constexpr int VI = 16 / sizeof(TI);               // input elements per 16-B vector
  constexpr int NVR = (C0_IN_W + VI - 1) / VI;      // vectors per staged input row
  constexpr int LPV = (9 * NVR + 255) / 256;        // vector loads per thread
  constexpr int OST = 32 + 16 / sizeof(TO);         // s_out row stride (elements, 16-B aligned)
  // the input strip and the output tile are live in disjoint phases: one LDS region (occupancy)
  // fp32 output (SW): swapped MFMA operands put 4 consecutive channels of one pixel in each lane,
  // stored straight from registers as 16-B vectors, so no output tile in LDS
  constexpr bool SW = false;  // measured slower than the LDS-staged tile (256 vs 230 us, cfg2)
  constexpr int IN_BYTES = (9 * C0_IN_W + VI) * 4;
  constexpr int OUT_BYTES = SW ? 0 : C0_TILE * OST * (int)sizeof(TO);
  __shared__ __attribute__((aligned(16))) char s_raw[IN_BYTES > OUT_BYTES ? IN_BYTES : OUT_BYTES];
  float* s_in = reinterpret_cast<float*>(s_raw);   // [ci][r][col] (+ slack for the last vector)
  TO* s_out = reinterpret_cast<TO*>(s_raw);        // [px][OST]
  __shared__ float s_red[2][4][C0_OUT];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int li = lane & 15, lq = lane >> 4;
  int seg, row;  // row = n * Ho + ho
  c0_tile(seg, row);
  const int wo0 = seg * C0_TILE;
  const int n = row / a.Ho, ho = row - n * a.Ho;
  const int npx = min(C0_TILE, a.Wo - wo0);

  // ---- stage the 3 x 3 x (2*256+1) input strip with 16-B loads (all issued, then stored) ----
  const int col0 = 2 * wo0;
  const int ncol = min(C0_IN_W, a.W - col0);
  const TI* xin = (const TI*)a.x;
  if (a.W % VI != 0) {  // rows not 16-B aligned: scalar staging (odd widths only)
    constexpr int NIN = 9 * C0_IN_W, LPT = (NIN + 255) / 256;
    float v[LPT];
#pragma unroll
    for (int k = 0; k < LPT; ++k) {
      const int i = tid + 256 * k;
      const int cr = i / C0_IN_W, c = i - cr * C0_IN_W;
      const int ci = cr / 3, r = cr - ci * 3;
      const bool ok = i < NIN && c < ncol;
      const size_t off = ok ? (((size_t)n * 3 + ci) * a.H + (2 * ho + r)) * a.W + col0 + c : 0;
      const float t = XB ? in16<XB>((uint16_t)xin[off]) : (float)xin[off];
      v[k] = ok ? t : 0.f;
    }
#pragma unroll
    for (int k = 0; k < LPT; ++k)
      if (tid + 256 * k < NIN) s_in[tid + 256 * k] = v[k];
  } else {
    uint4 raw[LPV];
#pragma unroll
    for (int k = 0; k < LPV; ++k) {
      const int i = tid + 256 * k;
      const int cr = i / NVR, v = i - cr * NVR;  // cr = ci*3 + r
      const int ci = cr / 3, r = cr - ci * 3;
      const bool ok = i < 9 * NVR && v * VI + VI <= ncol;  // whole vector inside the row
      const size_t off = ok ? (((size_t)n * 3 + ci) * a.H + (2 * ho + r)) * a.W + col0 + v * VI : 0;
      raw[k] = sel4(ok, *reinterpret_cast<const uint4*>(xin + off));
    }
#pragma unroll
    for (int k = 0; k < LPV; ++k) {
      const int i = tid + 256 * k;
      if (i >= 9 * NVR) continue;
      const int cr = i / NVR, v = i - cr * NVR;
      const TI* e = reinterpret_cast<const TI*>(&raw[k]);
#pragma unroll
      for (int j = 0; j < VI; ++j) {
        const int c = v * VI + j;
        float f;
        if (XB) f = in16<XB>((uint16_t)e[j]);
        else f = (float)e[j];
        if (c < C0_IN_W) s_in[cr * C0_IN_W + c] = f;
      }
      if (v * VI < ncol && v * VI + VI > ncol) {  // the image's right edge: partial vector
        for (int j = 0; j < VI; ++j) {
          const int c = v * VI + j;
          const int ci = cr / 3, r = cr - ci * 3;
          float f = 0.f;
          if (c < ncol) {
            const size_t o = (((size_t)n * 3 + ci) * a.H + (2 * ho + r)) * a.W + col0 + c;
            f = XB ? in16<XB>((uint16_t)xin[o]) : (float)xin[o];
          }
          if (c < C0_IN_W) s_in[cr * C0_IN_W + c] = f;
        }
      }
    }
  }
  // B fragments (weights) for the two 16-channel tiles: W[16*jt + li][8*lq + e], k >= 27 -> 0
  typename M::Frag bw[2];
#pragma unroll
  for (int jt = 0; jt < 2; ++jt) {
    float wv[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int k = 8 * lq + e;
      const float t = a.w[(16 * jt + li) * 27 + (k < 27 ? k : 0)];
      wv[e] = k < 27 ? t : 0.f;
    }
    bw[jt] = M::pack(wv);
  }
  // tap k -> offset in s_in relative to the pixel's column 2*px: (ci*3 + kh)*IN_W + kw
  int koff[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const int k = 8 * lq + e;
    const int kk = k < 27 ? k : 0;
    const int ci = kk / 9, kh = (kk % 9) / 3, kw = kk % 3;
    koff[e] = (ci * 3 + kh) * C0_IN_W + kw;
  }
  if constexpr (SW) {
    __syncthreads();
    // acc[gi][jt][r] = out[pixel 64w + 16gi + li][channel 16jt + 4lq + r]
    f32x4 acc[4][2];
#pragma unroll
    for (int gi = 0; gi < 4; ++gi) {
      const int px = wave * 64 + gi * 16 + li;
      float av[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) av[e] = 8 * lq + e < 27 ? s_in[koff[e] + 2 * px] : 0.f;
      const typename M::Frag af = M::pack(av);
#pragma unroll
      for (int jt = 0; jt < 2; ++jt) {
        acc[gi][jt] = f32x4{0.f, 0.f, 0.f, 0.f};
        M::mma(bw[jt], af, acc[gi][jt]);
      }
    }
    float* y = (float*)a.y + ((size_t)row * a.Wo + wo0) * C0_OUT;
#pragma unroll
    for (int jt = 0; jt < 2; ++jt) {
      float sc[4], sh[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int c = 16 * jt + 4 * lq + r;
        sc[r] = a.scale ? a.scale[c] : 1.f;
        sh[r] = a.scale ? a.shift[c] : 0.f;
      }
#pragma unroll
      for (int gi = 0; gi < 4; ++gi) {
        const int px = wave * 64 + gi * 16 + li;
        float v[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          v[r] = acc[gi][jt][r] * sc[r] + sh[r];
          if (a.relu) v[r] = fmaxf(v[r], 0.f);
          acc[gi][jt][r] = v[r];
        }
        if (px < npx)
          *reinterpret_cast<float4*>(y + (size_t)px * C0_OUT + 16 * jt + 4 * lq) =
              make_float4(v[0], v[1], v[2], v[3]);
      }
    }
    if (a.part == nullptr) return;
    // per-channel (mean, M2, count) over the block's npx pixels: lanes li hold pixels
    float sum[2][4];
#pragma unroll
    for (int jt = 0; jt < 2; ++jt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float t = 0.f;
#pragma unroll
        for (int gi = 0; gi < 4; ++gi) t += (wave * 64 + gi * 16 + li < npx) ? acc[gi][jt][r] : 0.f;
        t += __shfl_xor(t, 1);
        t += __shfl_xor(t, 2);
        t += __shfl_xor(t, 4);
        t += __shfl_xor(t, 8);
        sum[jt][r] = t;
      }
    if (li == 0)
#pragma unroll
      for (int jt = 0; jt < 2; ++jt)
#pragma unroll
        for (int r = 0; r < 4; ++r) s_red[0][wave][16 * jt + 4 * lq + r] = sum[jt][r];
    __syncthreads();
    float mean[2][4];
#pragma unroll
    for (int jt = 0; jt < 2; ++jt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int c = 16 * jt + 4 * lq + r;
        mean[jt][r] = ((s_red[0][0][c] + s_red[0][1][c]) + (s_red[0][2][c] + s_red[0][3][c])) / (float)npx;
      }
#pragma unroll
    for (int jt = 0; jt < 2; ++jt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float t = 0.f;
#pragma unroll
        for (int gi = 0; gi < 4; ++gi) {
          const float d = acc[gi][jt][r] - mean[jt][r];
          t += (wave * 64 + gi * 16 + li < npx) ? d * d : 0.f;
        }
        t += __shfl_xor(t, 1);
        t += __shfl_xor(t, 2);
        t += __shfl_xor(t, 4);
        t += __shfl_xor(t, 8);
        sum[jt][r] = t;
      }
    if (li == 0)
#pragma unroll
      for (int jt = 0; jt < 2; ++jt)
#pragma unroll
        for (int r = 0; r < 4; ++r) s_red[1][wave][16 * jt + 4 * lq + r] = sum[jt][r];
    __syncthreads();
    if (tid < C0_OUT) {
      const size_t pi = (size_t)row * gridDim.x + seg;
      float* rec = a.part + pi * 3 * C0_OUT;
      const int c = tid;
      rec[c] = ((s_red[0][0][c] + s_red[0][1][c]) + (s_red[0][2][c] + s_red[0][3][c])) / (float)npx;
      rec[C0_OUT + c] = (s_red[1][0][c] + s_red[1][1][c]) + (s_red[1][2][c] + s_red[1][3][c]);
      rec[2 * C0_OUT + c] = (float)npx;
    }
    return;
  } else {
  float fsc[2], fsh[2];  // eval BN fold of the lane's two channels (li, 16 + li)
#pragma unroll
  for (int jt = 0; jt < 2; ++jt) {
    fsc[jt] = a.scale ? a.scale[16 * jt + li] : 1.f;
    fsh[jt] = a.scale ? a.shift[16 * jt + li] : 0.f;
  }
  __syncthreads();

  // ---- wave w: pixels [64w, 64w+64) = 4 groups of 16, x 32 channels; acc[gi][jt][r] is
  //      out[pixel 64w + 16gi + 4lq + r][channel 16jt + li] -------------------------------------
  f32x4 acc[4][2];
#pragma unroll
  for (int gi = 0; gi < 4; ++gi) {
    const int px = wave * 64 + gi * 16 + li;  // A row = pixel
    float av[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) av[e] = 8 * lq + e < 27 ? s_in[koff[e] + 2 * px] : 0.f;
    const typename M::Frag af = M::pack(av);
#pragma unroll
    for (int jt = 0; jt < 2; ++jt) {
      acc[gi][jt] = f32x4{0.f, 0.f, 0.f, 0.f};
      M::mma(af, bw[jt], acc[gi][jt]);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float v = acc[gi][jt][r] * fsc[jt] + fsh[jt];
        if (a.relu) v = fmaxf(v, 0.f);
        acc[gi][jt][r] = v;
      }
    }
  }
  // ---- stage the tile in the storage type, then coalesced 16-B stores ----------------------
  __syncthreads();  // every wave is done reading s_in (aliased by s_out)
#pragma unroll
  for (int gi = 0; gi < 4; ++gi)
#pragma unroll
    for (int jt = 0; jt < 2; ++jt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        TO t;
        if constexpr (BF) t.x = s16_from<TO>(acc[gi][jt][r]);
        else t = acc[gi][jt][r];
        s_out[(wave * 64 + gi * 16 + 4 * lq + r) * OST + 16 * jt + li] = t;
      }
  __syncthreads();
  {
    constexpr int V = VecW<TO>::V;
    TO* y = (TO*)a.y + ((size_t)row * a.Wo + wo0) * C0_OUT;
    const int nvec = npx * C0_OUT / V;
#pragma unroll
    for (int k = 0; k < C0_TILE * C0_OUT / V / 256; ++k) {
      const int i = tid + 256 * k;
      if (i >= nvec) continue;
      const int p = (i * V) / C0_OUT, c = (i * V) - p * C0_OUT;
      *reinterpret_cast<uint4*>(y + (size_t)i * V) = *reinterpret_cast<const uint4*>(&s_out[p * OST + c]);
    }
  }
  if (a.part == nullptr) return;
  // ---- per-channel (mean, M2, count) over the block's npx pixels, from the fp32 registers ----
  float sum[2] = {0.f, 0.f};
#pragma unroll
  for (int gi = 0; gi < 4; ++gi)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const bool ok = wave * 64 + gi * 16 + 4 * lq + r < npx;
#pragma unroll
      for (int jt = 0; jt < 2; ++jt) sum[jt] += ok ? acc[gi][jt][r] : 0.f;
    }
#pragma unroll
  for (int jt = 0; jt < 2; ++jt) {
    sum[jt] += __shfl_xor(sum[jt], 16);
    sum[jt] += __shfl_xor(sum[jt], 32);
  }
  if (lq == 0) {
    s_red[0][wave][li] = sum[0];
    s_red[0][wave][16 + li] = sum[1];
  }
  __syncthreads();
  float mean[2];
#pragma unroll
  for (int jt = 0; jt < 2; ++jt) {
    const int c = 16 * jt + li;
    mean[jt] = ((s_red[0][0][c] + s_red[0][1][c]) + (s_red[0][2][c] + s_red[0][3][c])) / (float)npx;
  }
  float m2[2] = {0.f, 0.f};
#pragma unroll
  for (int gi = 0; gi < 4; ++gi)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const bool ok = wave * 64 + gi * 16 + 4 * lq + r < npx;
#pragma unroll
      for (int jt = 0; jt < 2; ++jt) {
        const float d = acc[gi][jt][r] - mean[jt];
        m2[jt] += ok ? d * d : 0.f;
      }
    }
#pragma unroll
  for (int jt = 0; jt < 2; ++jt) {
    m2[jt] += __shfl_xor(m2[jt], 16);
    m2[jt] += __shfl_xor(m2[jt], 32);
  }
  if (lq == 0) {
    s_red[1][wave][li] = m2[0];
    s_red[1][wave][16 + li] = m2[1];
  }
  __syncthreads();
  if (wave == 0 && lq == 0) {
    const size_t pi = (size_t)row * gridDim.x + seg;
    float* rec = a.part + pi * 3 * C0_OUT;
#pragma unroll
    for (int jt = 0; jt < 2; ++jt) {
      const int c = 16 * jt + li;
      rec[c] = mean[jt];
      rec[C0_OUT + c] = (s_red[1][0][c] + s_red[1][1][c]) + (s_red[1][2][c] + s_red[1][3][c]);
      rec[2 * C0_OUT + c] = (float)npx;
    }
  }
  }  // SW
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
  if (y_dtype == DT_F32) {
    if (a.x_bf16 == 2) conv0_fwd_kernel<float, 2><<<grid, 256, 0, st>>>(a);
    else if (a.x_bf16) conv0_fwd_kernel<float, 1><<<grid, 256, 0, st>>>(a);
    else conv0_fwd_kernel<float, 0><<<grid, 256, 0, st>>>(a);
  } else if (y_dtype == DT_F16) {
    if (a.x_bf16 == 2) conv0_fwd_kernel<f16, 2><<<grid, 256, 0, st>>>(a);
    else if (a.x_bf16) conv0_fwd_kernel<f16, 1><<<grid, 256, 0, st>>>(a);
    else conv0_fwd_kernel<f16, 0><<<grid, 256, 0, st>>>(a);
  } else {
    if (a.x_bf16 == 2) conv0_fwd_kernel<bf16, 2><<<grid, 256, 0, st>>>(a);
    else if (a.x_bf16) conv0_fwd_kernel<bf16, 1><<<grid, 256, 0, st>>>(a);
    else conv0_fwd_kernel<bf16, 0><<<grid, 256, 0, st>>>(a);
  }
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
// max workgroups (partials): one residency round of the bf16 BN-backward-on-load variant (141
// VGPRs: 3 workgroups per CU x 256 CUs); 1024 left a second round one third full
constexpr int CW_MAXP = 768;

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

template <>
struct CwOps<f16> {
  static constexpr int LD = CW_TP + 8;
  static __device__ __forceinline__ void mma(const f16* a, const f16* b, f32x4& acc) {
    h16x8 av, bv;
    __builtin_memcpy(&av, a, 16);
    __builtin_memcpy(&bv, b, 16);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(av, bv, acc, 0, 0, 0);
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
template <>
__device__ __forceinline__ f16 cw_cvt<f16>(float v) {
  f16 r;
  r.x = f2h(v);
  return r;
}

template <typename T, int XB, bool DX = false>
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
  // DX: a thread's dZ vectors all cover channels (tid * V) & 31 .. +V
  BwdXCoef<T> dxc;
  if constexpr (DX) dxc.load(a.tab, (tid * V) & 31);
  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // a contiguous run of row segments per workgroup: consecutive output rows share an input row
  // (2ho+2), re-read from this CU's cache instead of HBM
  const long long t_end = tiles * (blockIdx.x + 1) / gridDim.x;
  for (long long t = tiles * blockIdx.x / gridDim.x; t < t_end; ++t) {
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
          const float v = XB ? in16<XB>(((const uint16_t*)a.x)[o]) : ((const float*)a.x)[o];
          xv[cr * 3 + kw] = ok ? v : 0.f;
        }
      }
    }
    // dZ tile: npx*32 contiguous elements as 16-B vectors (V elements), transposed into sD
    constexpr int NV = CW_TP * 32 / V / 256;  // vectors per thread (4 bf16 / 8 f32)
    uint4 dv[NV], zv[DX ? NV : 1];
    const T* dz = (const T*)a.dz + ((size_t)row * a.Wo + wo0) * 32;
    const T* zb = (const T*)a.zz + ((size_t)row * a.Wo + wo0) * 32;
#pragma unroll
    for (int q = 0; q < NV; ++q) {
      const int i = tid + 256 * q;
      const int p = (i * V) >> 5;
      const size_t o = (size_t)(p < npx ? i : 0) * V;
      dv[q] = *reinterpret_cast<const uint4*>(dz + o);
      if constexpr (DX) zv[q] = *reinterpret_cast<const uint4*>(zb + o);
    }
#pragma unroll
    for (int q = 0; q < NV; ++q) {
      const int i = tid + 256 * q;
      const int p = (i * V) >> 5;
      uint4 v = dv[q];
      if constexpr (DX) v = bwdx_apply<T>(v, zv[q], dxc.al, dxc.be, dxc.gz, dxc.sc, dxc.sh);
      dv[q] = sel4(p < npx, v);
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
               (a.x_bf16 ? 2.0 : 4.0) * a.N * 3.0 * a.H * a.W +
                   (dz_dtype == DT_F32 ? 4.0 : 2.0) * px * 32 * (a.tab ? 2 : 1),
               2.0 * 27 * 32 * px);
  const bool dx = a.tab != nullptr;
  if (dx && (!a.zz || (uintptr_t)a.zz % 16)) {
    set_error("conv0_wgrad: BN-backward transform needs a 16-B aligned z");
    return E_INVALID;
  }
#define CW_LAUNCH(T)                                                                  \
  do {                                                                                \
    if (dx) {                                                                         \
      if (a.x_bf16 == 2) conv0_wgrad_kernel<T, 2, true><<<P, 256, 0, st>>>(a);        \
      else if (a.x_bf16) conv0_wgrad_kernel<T, 1, true><<<P, 256, 0, st>>>(a);        \
      else conv0_wgrad_kernel<T, 0, true><<<P, 256, 0, st>>>(a);                      \
    } else {                                                                          \
      if (a.x_bf16 == 2) conv0_wgrad_kernel<T, 2><<<P, 256, 0, st>>>(a);              \
      else if (a.x_bf16) conv0_wgrad_kernel<T, 1><<<P, 256, 0, st>>>(a);              \
      else conv0_wgrad_kernel<T, 0><<<P, 256, 0, st>>>(a);                            \
    }                                                                                 \
  } while (0)
  if (dz_dtype == DT_F32) CW_LAUNCH(float);
  else if (dz_dtype == DT_F16) CW_LAUNCH(f16);
  else CW_LAUNCH(bf16);
#undef CW_LAUNCH
  return check_launch("conv0_wgrad");
}

}  // namespace fscnn
