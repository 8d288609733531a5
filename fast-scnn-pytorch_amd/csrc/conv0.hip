// LearningToDownsample.conv: dense 3x3, stride 2, PADDING 0, 3 -> 32 channels, no bias
// (models/fast_scnn.py:153 with the _ConvBNReLU default padding=0 at :52).
//
// Reads the caller's NCHW image (fp32 or bf16) directly and writes NHWC [N,Ho,Wo,32].
// One workgroup = one output row segment of 256 pixels: the 3 input rows x (2*256+1) columns x
// 3 channels it needs are staged once in LDS (coalesced), each thread computes one pixel x 32
// channels with the 864 weights broadcast from LDS, and the 256x32 tile is written back through
// LDS as one contiguous, fully coalesced block.  HBM-bound: 12 B (fp32 in) read + 128 B written
// per output pixel against 1,728 flops.
#include "bn_finish.hpp"

namespace fscnn {

constexpr int C0_OUT = 32;
constexpr int C0_TILE = 256;             // output pixels per workgroup
constexpr int C0_IN_W = 2 * C0_TILE + 1;  // staged input columns
constexpr int C0_OSTR = 36;              // LDS floats per staged output pixel (16B aligned)


// (MFMA helpers of the im2col GEMM: common.hpp C0Mma)

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

// C0_RB output rows per workgroup: the 2*C0_RB + 1 input rows are staged once (adjacent output
// rows share an input row), the rows are computed and stored one after the other, and one
// statistics record covers the workgroup (per-row (mean, M2) merged in fixed order).  Measured r04
// at C0_RB = 2 (5 instead of 6 input rows per 2 output rows, half the workgroups, 51 KB LDS: 3 per
// CU): 5.98-5.99 vs 5.955-5.96 ms per cfg3 step, and the fp32 train gradients' merge of two rows'
// statistics in fp32 sat just outside the oracle gate -- one row stays the default.
#ifndef C0_RB_DEFAULT
#define C0_RB_DEFAULT 1
#endif
constexpr int C0_RB = C0_RB_DEFAULT;

template <typename TO, int XB>
__global__ __launch_bounds__(256) void conv0_fwd_kernel(Conv0Args a) {
  // 16-bit output => MFMA operands in that dtype (the plan's compute dtype)
  constexpr int BF = sizeof(TO) == 4 ? 0 : (std::is_same<TO, f16>::value ? 2 : 1);
  using M = C0Mma<BF>;
  using TI = typename std::conditional<XB != 0, uint16_t, float>::type;
  constexpr int RB = C0_RB;
  constexpr int NRI = 2 * RB + 1;                   // staged input rows
  constexpr int VI = 16 / sizeof(TI);               // input elements per 16-B vector
  constexpr int NVR = (C0_IN_W + VI - 1) / VI;      // vectors per staged input row
  constexpr int LPV = (3 * NRI * NVR + 255) / 256;  // vector loads per thread
  constexpr int OST = 32 + 16 / sizeof(TO);         // s_out row stride (elements, 16-B aligned)
  constexpr int IN_BYTES = ((3 * NRI * C0_IN_W + VI) * 4 + 15) / 16 * 16;
  constexpr int OUT_BYTES = C0_TILE * OST * (int)sizeof(TO);
  // one row: the input strip and the output tile are live in disjoint phases (one region); more
  // rows: the strip stays live while each row's tile is staged
  constexpr int RAW = RB == 1 ? (IN_BYTES > OUT_BYTES ? IN_BYTES : OUT_BYTES) : IN_BYTES + OUT_BYTES;
  __shared__ __attribute__((aligned(16))) char s_raw[RAW];
  float* s_in = reinterpret_cast<float*>(s_raw);   // [ci][r][col] (+ slack for the last vector)
  TO* s_out = reinterpret_cast<TO*>(s_raw + (RB == 1 ? 0 : IN_BYTES));  // [px][OST]
  __shared__ float s_red[2][4][C0_OUT];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int li = lane & 15, lq = lane >> 4;
  int seg, rowb;  // rowb = n * HB + hb
  c0_tile(seg, rowb);
  stamp(a.stamps, 0);
  const int HB = cdiv(a.Ho, RB);
  const int wo0 = seg * C0_TILE;
  const int n = rowb / HB, ho0 = (rowb - n * HB) * RB;
  const int nrows = min(RB, a.Ho - ho0);
  const int npx = min(C0_TILE, a.Wo - wo0);

  // ---- stage the 3 x NRI x (2*256+1) input strip (all loads issued, then stored) ------------
  const int col0 = 2 * wo0;
  const int ncol = min(C0_IN_W, a.W - col0);
  const TI* xin = (const TI*)a.x;
  auto rowok = [&](int r) { return 2 * ho0 + r < a.H; };
  if (a.W % VI != 0) {  // rows not 16-B aligned: scalar staging (odd widths only)
    constexpr int NIN = 3 * NRI * C0_IN_W, LPT = (NIN + 255) / 256;
    float v[LPT];
#pragma unroll
    for (int k = 0; k < LPT; ++k) {
      const int i = tid + 256 * k;
      const int cr = i / C0_IN_W, c = i - cr * C0_IN_W;
      const int ci = cr / NRI, r = cr - ci * NRI;
      const bool ok = i < NIN && c < ncol && rowok(r);
      const size_t off = ok ? (((size_t)n * 3 + ci) * a.H + (2 * ho0 + r)) * a.W + col0 + c : 0;
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
      const int cr = i / NVR, v = i - cr * NVR;  // cr = ci*NRI + r
      const int ci = cr / NRI, r = cr - ci * NRI;
      const bool ok = i < 3 * NRI * NVR && v * VI + VI <= ncol && rowok(r);  // whole vector inside
      const size_t off = ok ? (((size_t)n * 3 + ci) * a.H + (2 * ho0 + r)) * a.W + col0 + v * VI : 0;
      raw[k] = sel4(ok, *reinterpret_cast<const uint4*>(xin + off));
    }
#pragma unroll
    for (int k = 0; k < LPV; ++k) {
      const int i = tid + 256 * k;
      if (i >= 3 * NRI * NVR) continue;
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
      const int ci = cr / NRI, r = cr - ci * NRI;
      if (rowok(r) && v * VI < ncol && v * VI + VI > ncol) {  // the image's right edge
        for (int j = 0; j < VI; ++j) {
          const int c = v * VI + j;
          float f = 0.f;
          if (c < ncol) {
            const size_t o = (((size_t)n * 3 + ci) * a.H + (2 * ho0 + r)) * a.W + col0 + c;
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
  // tap k -> offset in s_in relative to the pixel's column 2*px of output row 0
  int koff[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const int k = 8 * lq + e;
    const int kk = k < 27 ? k : 0;
    const int ci = kk / 9, kh = (kk % 9) / 3, kw = kk % 3;
    koff[e] = (ci * NRI + kh) * C0_IN_W + kw;
  }
  float fsc[2], fsh[2];  // eval BN fold of the lane's two channels (li, 16 + li)
#pragma unroll
  for (int jt = 0; jt < 2; ++jt) {
    fsc[jt] = a.scale ? a.scale[16 * jt + li] : 1.f;
    fsh[jt] = a.scale ? a.shift[16 * jt + li] : 0.f;
  }
  __syncthreads();
  stamp(a.stamps, 1);

  float tn = 0.f, tmean[2] = {0.f, 0.f}, tm2[2] = {0.f, 0.f};  // the record (wave 0, lq 0)
  for (int r = 0; r < nrows; ++r) {  // (workgroup-uniform)
    const int ho = ho0 + r;
    // ---- wave w: pixels [64w, 64w+64) = 4 groups of 16, x 32 channels; acc[gi][jt][q] is
    //      out[pixel 64w + 16gi + 4lq + q][channel 16jt + li] -----------------------------------
    f32x4 acc[4][2];
#pragma unroll
    for (int gi = 0; gi < 4; ++gi) {
      const int px = wave * 64 + gi * 16 + li;  // A row = pixel
      float av[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) av[e] = 8 * lq + e < 27 ? s_in[koff[e] + 2 * r * C0_IN_W + 2 * px] : 0.f;
      const typename M::Frag af = M::pack(av);
#pragma unroll
      for (int jt = 0; jt < 2; ++jt) {
        acc[gi][jt] = f32x4{0.f, 0.f, 0.f, 0.f};
        M::mma(af, bw[jt], acc[gi][jt]);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          float v = acc[gi][jt][q] * fsc[jt] + fsh[jt];
          if (a.relu) v = fmaxf(v, 0.f);
          acc[gi][jt][q] = v;
        }
      }
    }
    // ---- stage the row's tile in the storage type, then coalesced 16-B stores ----------------
    __syncthreads();  // RB == 1: every wave is done reading s_in (aliased); else the previous
                      // row's tile stores are done
#pragma unroll
    for (int gi = 0; gi < 4; ++gi)
#pragma unroll
      for (int jt = 0; jt < 2; ++jt)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          TO t;
          if constexpr (BF) t.x = s16_from<TO>(acc[gi][jt][q]);
          else t = acc[gi][jt][q];
          s_out[(wave * 64 + gi * 16 + 4 * lq + q) * OST + 16 * jt + li] = t;
        }
    __syncthreads();
    stamp(a.stamps, 2);
    {
      constexpr int V = VecW<TO>::V;
      TO* y = (TO*)a.y + (((size_t)n * a.Ho + ho) * a.Wo + wo0) * C0_OUT;
      const int nvec = npx * C0_OUT / V;
#pragma unroll
      for (int k = 0; k < C0_TILE * C0_OUT / V / 256; ++k) {
        const int i = tid + 256 * k;
        if (i >= nvec) continue;
        const int p = (i * V) / C0_OUT, c = (i * V) - p * C0_OUT;
        *reinterpret_cast<uint4*>(y + (size_t)i * V) = *reinterpret_cast<const uint4*>(&s_out[p * OST + c]);
      }
    }
    stamp(a.stamps, 3);
    if (a.part == nullptr) continue;
    // ---- per-channel (mean, M2) of the row's npx pixels: the values as stored (16-bit: read back
    // from the staged output tile, so the fp32 accumulators die at the store) ------------------
    auto stored = [&](int gi, int jt, int q) -> float {
      if constexpr (BF) return s16_to<TO>(s_out[(wave * 64 + gi * 16 + 4 * lq + q) * OST + 16 * jt + li].x);
      else return acc[gi][jt][q];
    };
    float sum[2] = {0.f, 0.f};
#pragma unroll
    for (int gi = 0; gi < 4; ++gi)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const bool ok = wave * 64 + gi * 16 + 4 * lq + q < npx;
#pragma unroll
        for (int jt = 0; jt < 2; ++jt) sum[jt] += ok ? stored(gi, jt, q) : 0.f;
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
      for (int q = 0; q < 4; ++q) {
        const bool ok = wave * 64 + gi * 16 + 4 * lq + q < npx;
#pragma unroll
        for (int jt = 0; jt < 2; ++jt) {
          const float d = stored(gi, jt, q) - mean[jt];
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
    if (wave == 0 && lq == 0) {  // merge the row into the record (Chan, fixed row order)
      const float nr = (float)npx;
#pragma unroll
      for (int jt = 0; jt < 2; ++jt) {
        const int c = 16 * jt + li;
        const float rm2 = (s_red[1][0][c] + s_red[1][1][c]) + (s_red[1][2][c] + s_red[1][3][c]);
        if (r == 0) {
          tmean[jt] = mean[jt];
          tm2[jt] = rm2;
        } else {
          const float nt = tn + nr, d = mean[jt] - tmean[jt];
          tmean[jt] += d * (nr / nt);
          tm2[jt] += rm2 + d * d * (tn * nr / nt);
        }
      }
      tn += nr;
    }
    __syncthreads();  // s_red is reused by the next row
  }
  if (a.part != nullptr && wave == 0 && lq == 0) {
    const size_t pi = (size_t)rowb * gridDim.x + seg;
    float* rec = a.part + pi * 3 * C0_OUT;
#pragma unroll
    for (int jt = 0; jt < 2; ++jt) {
      const int c = 16 * jt + li;
      rec[c] = tmean[jt];
      rec[C0_OUT + c] = tm2[jt];
      rec[2 * C0_OUT + c] = tn;
    }
  }
  stamp(a.stamps, 4);
}

int conv0_parts(int N, int Ho, int Wo) { return N * cdiv(Ho, C0_RB) * cdiv(Wo, C0_TILE); }

int conv0_fwd(const Conv0Args& a, int y_dtype, hipStream_t st) {
  if (a.Ho != (a.H - 3) / 2 + 1 || a.Wo != (a.W - 3) / 2 + 1 || a.H < 3 || a.W < 3) {
    set_error("conv0_fwd: bad shape H=%d W=%d Ho=%d Wo=%d", a.H, a.W, a.Ho, a.Wo);
    return E_INVALID;
  }
  dim3 grid(cdiv(a.Wo, C0_TILE), a.N * cdiv(a.Ho, C0_RB));
  Conv0Args as = a;
  as.stamps = stamp_region();
  const double px = (double)a.N * a.Ho * a.Wo;
  ProfScope ps(PK_CONV0_FWD, st,
               (a.x_bf16 ? 2.0 : 4.0) * a.N * 3.0 * a.H * a.W + (y_dtype == DT_F32 ? 4.0 : 2.0) * px * 32,
               2.0 * 27 * 32 * px);
  if (y_dtype == DT_F32) {
    if (a.x_bf16 == 2) prof_launch(conv0_fwd_kernel<float, 2>, grid, 256, 0, st, as);
    else if (a.x_bf16) prof_launch(conv0_fwd_kernel<float, 1>, grid, 256, 0, st, as);
    else prof_launch(conv0_fwd_kernel<float, 0>, grid, 256, 0, st, as);
  } else if (y_dtype == DT_F16) {
    if (a.x_bf16 == 2) prof_launch(conv0_fwd_kernel<f16, 2>, grid, 256, 0, st, as);
    else if (a.x_bf16) prof_launch(conv0_fwd_kernel<f16, 1>, grid, 256, 0, st, as);
    else prof_launch(conv0_fwd_kernel<f16, 0>, grid, 256, 0, st, as);
  } else {
    if (a.x_bf16 == 2) prof_launch(conv0_fwd_kernel<bf16, 2>, grid, 256, 0, st, as);
    else if (a.x_bf16) prof_launch(conv0_fwd_kernel<bf16, 1>, grid, 256, 0, st, as);
    else prof_launch(conv0_fwd_kernel<bf16, 0>, grid, 256, 0, st, as);
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
      if (a.x_bf16 == 2) prof_launch(conv0_wgrad_kernel<T, 2, true>, P, 256, 0, st, a);        \
      else if (a.x_bf16) prof_launch(conv0_wgrad_kernel<T, 1, true>, P, 256, 0, st, a);        \
      else prof_launch(conv0_wgrad_kernel<T, 0, true>, P, 256, 0, st, a);                      \
    } else {                                                                          \
      if (a.x_bf16 == 2) prof_launch(conv0_wgrad_kernel<T, 2>, P, 256, 0, st, a);              \
      else if (a.x_bf16) prof_launch(conv0_wgrad_kernel<T, 1>, P, 256, 0, st, a);              \
      else prof_launch(conv0_wgrad_kernel<T, 0>, P, 256, 0, st, a);                            \
    }                                                                                 \
  } while (0)
  if (dz_dtype == DT_F32) CW_LAUNCH(float);
  else if (dz_dtype == DT_F16) CW_LAUNCH(f16);
  else CW_LAUNCH(bf16);
#undef CW_LAUNCH
  return check_launch("conv0_wgrad");
}

// ---- conv0 input gradient (x.grad; autograd of the image through models/fast_scnn.py:153) --------
// dx[n][ci][h][w] = sum over the output pixels (oh, ow) whose 3x3 stride-2 window (padding 0)
// covers (h, w) -- at most 2 x 2 of them, kh = h - 2oh in {0, 1, 2} -- and the 32 channels of
// dz[n][oh][ow][co] * w[co][ci][kh][kw].  A gather with one thread per image pixel (no atomics,
// deterministic); neighbouring threads share their dz vectors through the cache.  HBM-bound:
// e * 32 * N*Ho*Wo read + dx_e * 3 * N*H*W written.  Runs only when the caller asks for x.grad.
template <typename T, typename TO>
__global__ __launch_bounds__(256) void conv0_dgrad_kernel(Conv0DgradArgs a) {
  constexpr int V = VecW<T>::V;
  __shared__ float sw[9][3][32];  // [kh * 3 + kw][ci][co]
  for (int i = threadIdx.x; i < 864; i += 256) {
    const int co = i / 27, r = i - co * 27, ci = r / 9, k = r - ci * 9;
    sw[k][ci][co] = a.w[i];
  }
  __syncthreads();
  const long long HW = (long long)a.H * a.W;
  const long long p = (long long)blockIdx.x * 256 + threadIdx.x;
  if (p >= (long long)a.N * HW) return;
  const int n = (int)(p / HW);
  const long long hw = p - (long long)n * HW;
  const int h = (int)(hw / a.W), w = (int)(hw - (long long)h * a.W);
  float acc[3] = {0.f, 0.f, 0.f};
#pragma unroll
  for (int dh = 0; dh < 2; ++dh) {
    const int kh = (h & 1) + 2 * dh;
    const int oh = (h - kh) >> 1;
    if (kh > 2 || oh < 0 || oh >= a.Ho) continue;
#pragma unroll
    for (int dw = 0; dw < 2; ++dw) {
      const int kw = (w & 1) + 2 * dw;
      const int ow = (w - kw) >> 1;
      if (kw > 2 || ow < 0 || ow >= a.Wo) continue;
      const T* d = (const T*)a.dz + (((size_t)n * a.Ho + oh) * a.Wo + ow) * 32;
      const int k = kh * 3 + kw;
#pragma unroll
      for (int q = 0; q < 32 / V; ++q) {
        float v[V];
        unpack<T>(*reinterpret_cast<const uint4*>(d + q * V), v);
#pragma unroll
        for (int j = 0; j < V; ++j) {
          const int co = q * V + j;
          acc[0] = fmaf(v[j], sw[k][0][co], acc[0]);
          acc[1] = fmaf(v[j], sw[k][1][co], acc[1]);
          acc[2] = fmaf(v[j], sw[k][2][co], acc[2]);
        }
      }
    }
  }
  TO* dx = (TO*)a.dx + (size_t)n * 3 * HW + hw;
#pragma unroll
  for (int ci = 0; ci < 3; ++ci) st1(dx + ci * HW, acc[ci]);
}

int conv0_dgrad(const Conv0DgradArgs& a, int dz_dtype, hipStream_t st) {
  if (!a.dz || !a.w || !a.dx || a.N < 1 || a.Ho != (a.H - 3) / 2 + 1 || a.Wo != (a.W - 3) / 2 + 1) {
    set_error("conv0_dgrad: bad arguments (N %d, %dx%d -> %dx%d)", a.N, a.H, a.W, a.Ho, a.Wo);
    return E_INVALID;
  }
  if ((uintptr_t)a.dz % 16) {
    set_error("conv0_dgrad: dz must be 16-B aligned");
    return E_INVALID;
  }
  const int blocks = cdiv((long long)a.N * a.H * a.W, 256);
#define C0D_LAUNCH(T)                                                                          \
  do {                                                                                         \
    if (a.dx_dtype == DT_BF16) prof_launch(conv0_dgrad_kernel<T, bf16>, blocks, 256, 0, st, a);         \
    else if (a.dx_dtype == DT_F16) prof_launch(conv0_dgrad_kernel<T, f16>, blocks, 256, 0, st, a);      \
    else prof_launch(conv0_dgrad_kernel<T, float>, blocks, 256, 0, st, a);                              \
  } while (0)
  if (dz_dtype == DT_F32) C0D_LAUNCH(float);
  else if (dz_dtype == DT_F16) C0D_LAUNCH(f16);
  else C0D_LAUNCH(bf16);
#undef C0D_LAUNCH
  return check_launch("conv0_dgrad");
}

// ---- fused: LearningToDownsample.dsconv1.dw input gradient + conv0 weight gradient --------------
// The stride-2 depthwise dgrad (dwconv.hip dw_dgrad_s2, same thread tile and arithmetic: a thread
// owns dx rows h0, h0+1 x columns w0..w0+3 of 4 channels) produces g, the gradient of conv0's BN
// output, which only conv0's weight gradient consumes.  Rather than storing g (268 MB at cfg3) and
// streaming it back with z in a second launch, the workgroup keeps its tile of masked g and of z
// in LDS as [pixel][channel] images (64-B rows, one 8-B store per thread and pixel), gathers the
// conv0 patches x^T [tap][pixel] beside them, and accumulates A = sum x g^T and Zc = sum x (z-mean)^T with
// v_mfma_f32_32x32x16 (taps x channels, k = 16 pixels): the A operand is one ds_read_b128 of x^T,
// the B operands are read column-wise with ds_read_b64_tr_b16 (gfx950's transposing LDS read).
// BN backward is linear in g, z and 1 per channel (bwdx_apply: dz = al*g + gz*z + be), so the
// conv0 gradient is dW = al*A + gz*Zc + (be + gz*mean)*B with B = sum x, formed after the BN
// finish (conv0_wgrad_combine) — the BN's statistics of g are not needed before the pass over g.
// z is centred before the MFMA (rounded to T as z - mean): summed raw, gz*Zx and be*B would both
// grow with |mean| / std and cancel.
// Persistent: LC_MAXP workgroups walk contiguous tile ranges; one BN record and one LC0_SLAB
// partial row per workgroup (fixed-order reductions: deterministic); the BN finish is the
// separate fold+finalize launch.
constexpr int LC_TW = 128;           // tile: 2 dx rows x 128 columns = 256 pixels
constexpr int LC_LDX = 256 + 8;      // x^T image row stride (elements): conflict-free b128 reads
constexpr int LC_MAXP = 512;         // 2 workgroups per CU (1024: 6.00 vs 5.96 ms per step, r04)
typedef float f32x16 __attribute__((ext_vector_type(16)));

template <typename T>
__device__ __forceinline__ void lc_mma(const i16x8& a, const i16x8& b, f32x16& acc) {
  if constexpr (std::is_same<T, f16>::value) {
    h16x8 ah, bh;
    __builtin_memcpy(&ah, &a, 16);
    __builtin_memcpy(&bh, &b, 16);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bh, acc, 0, 0, 0);
  } else {
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc, 0, 0, 0);
  }
}
// 4 x 16-bit storage elements (8 B) <-> fp32
template <typename T>
__device__ __forceinline__ void lc_unpack4(const uint2& t, float (&v)[4]) {
  v[0] = s16_to<T>((uint16_t)(t.x & 0xFFFFu)); v[1] = s16_to<T>((uint16_t)(t.x >> 16));
  v[2] = s16_to<T>((uint16_t)(t.y & 0xFFFFu)); v[3] = s16_to<T>((uint16_t)(t.y >> 16));
}
template <typename T>
__device__ __forceinline__ uint2 lc_pack4(const float (&v)[4]) {
  uint2 t;
  t.x = (uint32_t)s16_from<T>(v[0]) | ((uint32_t)s16_from<T>(v[1]) << 16);
  t.y = (uint32_t)s16_from<T>(v[2]) | ((uint32_t)s16_from<T>(v[3]) << 16);
  return t;
}
__device__ __forceinline__ i16x4 lc_tr(const uint16_t* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) i16x4*)p);
}

template <typename T, int XB>
__global__ __launch_bounds__(256, 2) void ltd_c0_bwd_kernel(LtdC0BwdArgs a) {
  constexpr int V = 4;
  constexpr int SG = 256 * 32 * 2;  // bytes of one [pixel][channel] image
  __shared__ __attribute__((aligned(16))) unsigned char s_raw[2 * SG + 32 * LC_LDX * 2];
  uint16_t* sG = reinterpret_cast<uint16_t*>(s_raw);           // masked g [pixel][channel]
  uint16_t* sZ = reinterpret_cast<uint16_t*>(s_raw + SG);      // z [pixel][channel]
  uint16_t* sX = reinterpret_cast<uint16_t*>(s_raw + 2 * SG);  // x^T [tap][pixel]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int tx = tid & 7, ty = tid >> 3;  // channel quad, 4-column group
  const int cb = tx * V;
  for (int i = tid; i < 5 * LC_LDX; i += 256) sX[27 * LC_LDX + i] = 0;  // taps 27..31: zero

  // depthwise taps [tap][channel] and conv0's BN (mean, invstd, ReLU-mask affine) per channel,
  // read from LDS where used (in registers they would cost 52 VGPRs of the 2-wave budget)
  __shared__ __attribute__((aligned(16))) float s_wt[9 * 32];
  __shared__ __attribute__((aligned(16))) float s_bn[4 * 32];
  for (int i = tid; i < 9 * 32; i += 256) s_wt[(i % 9) * 32 + i / 9] = a.w[i];
  if (tid < 32) {
    const bool m2 = a.bs.mode == 2;
    s_bn[tid] = a.bs.mean[tid];
    s_bn[32 + tid] = a.bs.invstd[tid];
    s_bn[64 + tid] = m2 ? a.bs.scale[tid] : 0.f;  // mode 0: fmaf(z, 0, 1) > 0 always
    s_bn[96 + tid] = m2 ? a.bs.shift[tid] : 1.f;
  }
  __syncthreads();
  float s1[V], s2[V];
#pragma unroll
  for (int j = 0; j < V; ++j) s1[j] = s2[j] = 0.f;
  float bx[3][3];  // sums of the x^T values this thread stages ((pair, kw) fixed per thread)
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int k = 0; k < 3; ++k) bx[i][k] = 0.f;
  f32x16 accA, accZ;
#pragma unroll
  for (int r = 0; r < 16; ++r) accA[r] = accZ[r] = 0.f;

  // tile t -> (image n, column block cbk, row pair hp), hp fastest: a workgroup walks DOWN one
  // column block, so the dy row and the image rows a tile shares with the tile above it were
  // fetched by this workgroup one tile earlier (L2-hot) instead of by another workgroup 8 tiles
  // apart; < 2^31 tiles (host check)
  const int CB = cdiv(a.W, LC_TW), RP = (a.H + 1) / 2;
  const int tiles = a.N * RP * CB;
  const size_t XHW = (size_t)a.XH * a.XW;
  const int t_end = (int)((long long)tiles * (blockIdx.x + 1) / gridDim.x);
  for (int t = (int)((long long)tiles * blockIdx.x / gridDim.x); t < t_end; ++t) {
    const int nc = t / RP, hp = t - nc * RP;
    const int n = nc / CB, cbk = nc - n * CB;
    const int h0 = 2 * hp, wc0 = cbk * LC_TW, w0 = wc0 + 4 * ty;
    // ---- every global load first: dy 2 x 3, z 2 x 4 (8 B each), the x rows of the patches ---
    uint2 gr[2][3], zr[2][4];
    const T* gb = (const T*)a.dy + (size_t)n * a.Ho * a.Wo * 32 + cb;
#pragma unroll
    for (int dr = 0; dr < 2; ++dr)
#pragma unroll
      for (int dc = 0; dc < 3; ++dc) {
        const int ho = hp + dr, wo = w0 / 2 + dc;
        const bool ok = ho < a.Ho && wo < a.Wo && w0 < a.W;
        const uint2 v = *reinterpret_cast<const uint2*>(gb + (ok ? ho * a.Wo + wo : 0) * 32);
        gr[dr][dc] = ok ? v : make_uint2(0u, 0u);
      }
#pragma unroll
    for (int r = 0; r < 2; ++r)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const bool ok = h0 + r < a.H && w0 + q < a.W;
        const size_t pix = ok ? ((size_t)n * a.H + h0 + r) * a.W + w0 + q : 0;
        const uint2 v = *reinterpret_cast<const uint2*>((const T*)a.bs.z + pix * 32 + cb);
        zr[r][q] = ok ? v : make_uint2(0u, 0u);
      }
    // x^T staging items i = tid + 256 * it -> (pair = (ci, kh) = i >> 6, row r, column group u):
    // 9 consecutive image columns 2w .. 2w + 8 of one row give taps kw = 0..2 of 4 pixels
    uint4 xr[3][XB ? 1 : 2];  // 8 columns (raw), the 9th as fp32
    float x8[3];
#pragma unroll
    for (int it = 0; it < 3; ++it) {
      const int i = tid + 256 * it;
      if (i >= 576) break;  // (wave-uniform: it = 2 is wave 0's alone)
      const int pair = i >> 6, r = (i >> 5) & 1, u = i & 31;
      const int ci = pair / 3, kh = pair - 3 * ci;
      const int h = h0 + r, wq = wc0 + 4 * u;
      const bool okr = h < a.H && wq < a.W;
      const int col = okr ? 2 * wq : 0;
      const size_t o = ((size_t)n * 3 + ci) * XHW + (size_t)(okr ? 2 * h + kh : 0) * a.XW + col;
      const bool ok8 = okr && col + 8 < a.XW;
      if constexpr (XB) {
        xr[it][0] = *reinterpret_cast<const uint4*>((const uint16_t*)a.x + o);
        const uint16_t e8 = ((const uint16_t*)a.x)[ok8 ? o + 8 : o];
        x8[it] = ok8 ? in16<XB>(e8) : 0.f;
      } else {
        xr[it][0] = *reinterpret_cast<const uint4*>((const float*)a.x + o);
        xr[it][1] = *reinterpret_cast<const uint4*>((const float*)a.x + o + 4);
        const float e8 = ((const float*)a.x)[ok8 ? o + 8 : o];
        x8[it] = ok8 ? e8 : 0.f;
      }
    }
    // ---- dgrad (dw_dgrad_s2's arithmetic), the masked g rounded as stored, BN records ----------
    uint2 gw[2][4];
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      float acc[4][V];
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int j = 0; j < V; ++j) acc[q][j] = 0.f;
#pragma unroll
      for (int dr = 0; dr < 2; ++dr) {
        const int kh = r + 1 - 2 * dr;
        if (kh < 0 || kh > 2) continue;
#pragma unroll
        for (int dc = 0; dc < 3; ++dc) {
          float g[V];
          lc_unpack4<T>(gr[dr][dc], g);
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int kw = q + 1 - 2 * dc;
            if (kw < 0 || kw > 2) continue;
            const float4 w4 = *reinterpret_cast<const float4*>(s_wt + (kh * 3 + kw) * 32 + cb);
            const float wv[4] = {w4.x, w4.y, w4.z, w4.w};
#pragma unroll
            for (int j = 0; j < V; ++j) acc[q][j] = fmaf(g[j], wv[j], acc[q][j]);
          }
        }
      }
      const float4 bm = *reinterpret_cast<const float4*>(s_bn + cb);
      const float4 bi = *reinterpret_cast<const float4*>(s_bn + 32 + cb);
      const float4 ms = *reinterpret_cast<const float4*>(s_bn + 64 + cb);
      const float4 mh = *reinterpret_cast<const float4*>(s_bn + 96 + cb);
      const float bmv[4] = {bm.x, bm.y, bm.z, bm.w}, biv[4] = {bi.x, bi.y, bi.z, bi.w};
      const float msv[4] = {ms.x, ms.y, ms.z, ms.w}, mhv[4] = {mh.x, mh.y, mh.z, mh.w};
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const bool ok = h0 + r < a.H && w0 + q < a.W;
        float z[V], gv[V], zc[V];
        lc_unpack4<T>(zr[r][q], z);
#pragma unroll
        for (int j = 0; j < V; ++j) {
          float v = round_as<T>(acc[q][j]);
          v = (ok && fmaf(z[j], msv[j], mhv[j]) > 0.f) ? v : 0.f;
          zc[j] = z[j] - bmv[j];
          s1[j] += v;
          s2[j] += v * zc[j] * biv[j];
          gv[j] = v;
        }
        gw[r][q] = lc_pack4<T>(gv);  // exact: v is a T value
        zr[r][q] = lc_pack4<T>(zc);  // the MFMA's centred z (outside the image: x = 0 there)
      }
    }
    // x^T values as T (pixels outside the output: 0), and their sums
    uint2 xw[3][3];
#pragma unroll
    for (int it = 0; it < 3; ++it) {
      const int i = tid + 256 * it;
      if (i >= 576) break;
      const int r = (i >> 5) & 1, u = i & 31;
      const int h = h0 + r, wq = wc0 + 4 * u;
      float xe[9];
      if constexpr (XB) {
        const uint32_t wv[4] = {xr[it][0].x, xr[it][0].y, xr[it][0].z, xr[it][0].w};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          xe[2 * k] = in16<XB>((uint16_t)(wv[k] & 0xFFFFu));
          xe[2 * k + 1] = in16<XB>((uint16_t)(wv[k] >> 16));
        }
      } else {
#pragma unroll
        for (int k = 0; k < 2; ++k) {
          xe[4 * k] = __uint_as_float(xr[it][k].x); xe[4 * k + 1] = __uint_as_float(xr[it][k].y);
          xe[4 * k + 2] = __uint_as_float(xr[it][k].z); xe[4 * k + 3] = __uint_as_float(xr[it][k].w);
        }
      }
      xe[8] = x8[it];
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) {
        float v[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const bool ok = h < a.H && wq + q < a.W;
          v[q] = ok ? round_as<T>(xe[2 * q + kw]) : 0.f;
        }
        bx[it][kw] += (v[0] + v[1]) + (v[2] + v[3]);
        xw[it][kw] = lc_pack4<T>(v);
      }
    }
    __syncthreads();  // the previous tile's MFMA operand reads are done
#pragma unroll
    for (int r = 0; r < 2; ++r)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int p = r * 128 + 4 * ty + q;
        *reinterpret_cast<uint2*>(sG + p * 32 + cb) = gw[r][q];
        *reinterpret_cast<uint2*>(sZ + p * 32 + cb) = zr[r][q];
      }
#pragma unroll
    for (int it = 0; it < 3; ++it) {
      const int i = tid + 256 * it;
      if (i >= 576) break;
      const int pair = i >> 6, r = (i >> 5) & 1, u = i & 31;
#pragma unroll
      for (int kw = 0; kw < 3; ++kw)
        *reinterpret_cast<uint2*>(sX + (pair * 3 + kw) * LC_LDX + r * 128 + 4 * u) = xw[it][kw];
    }
    __syncthreads();
    // ---- MFMA: the wave's 64 pixels in 4 k-steps of 16; D[tap][channel] ---------------------
    {
      const int g4 = lane >> 4, li = lane & 15;
      const int rq = 8 * (g4 >> 1) + (li >> 2), cc = 16 * (g4 & 1) + 4 * (li & 3);
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        const int k0 = wave * 64 + ks * 16;
        i16x8 ax;
        __builtin_memcpy(&ax, sX + (lane & 31) * LC_LDX + k0 + 8 * (lane >> 5), 16);
        const uint16_t* pg = sG + (k0 + rq) * 32 + cc;
        const uint16_t* pz = sZ + (k0 + rq) * 32 + cc;
        const i16x4 g0 = lc_tr(pg), g1 = lc_tr(pg + 4 * 32);
        const i16x4 z0 = lc_tr(pz), z1 = lc_tr(pz + 4 * 32);
        const i16x8 bg = {g0[0], g0[1], g0[2], g0[3], g1[0], g1[1], g1[2], g1[3]};
        const i16x8 bz = {z0[0], z0[1], z0[2], z0[3], z1[0], z1[1], z1[2], z1[3]};
        lc_mma<T>(ax, bg, accA);
        lc_mma<T>(ax, bz, accZ);
      }
    }
  }

  // ---- conv0 partials: the 4 waves' accumulators summed in fixed order -----------------------
  __syncthreads();
  float* red = reinterpret_cast<float*>(s_raw);  // [wave][A|Zx][32 tap][32 channel] (32 KB)
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int m = (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
    red[((wave * 2 + 0) * 32 + m) * 32 + (lane & 31)] = accA[r];
    red[((wave * 2 + 1) * 32 + m) * 32 + (lane & 31)] = accZ[r];
  }
  __syncthreads();
  float* out = a.slab + (size_t)blockIdx.x * LC0_SLAB;
  for (int o = tid; o < 1728; o += 256) {
    const int k = o >= 864 ? 1 : 0, oo = o - 864 * k;
    const int co = oo / 27, tap = oo - 27 * co;
    const int e = (k * 32 + tap) * 32 + co;
    out[o] = (red[e] + red[2048 + e]) + (red[4096 + e] + red[6144 + e]);
  }
#pragma unroll
  for (int it = 0; it < 3; ++it) {
    if (wave + 4 * it >= 9) break;  // (pair = wave + 4 * it, wave-uniform)
#pragma unroll
    for (int kw = 0; kw < 3; ++kw) {
      float v = bx[it][kw];
#pragma unroll
      for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off);
      if (lane == 0) out[1728 + (wave + 4 * it) * 3 + kw] = v;
    }
  }
  // ---- conv0 BN-backward record of the workgroup (the 32 column groups in fixed order) -------
  float* s_br = reinterpret_cast<float*>(s_raw + 2 * SG);  // [256][2 V] (in x^T's space)
#pragma unroll
  for (int j = 0; j < V; ++j) {
    s_br[tid * 2 * V + j] = s1[j];
    s_br[tid * 2 * V + V + j] = s2[j];
  }
  __syncthreads();
  if (tid < 64) {
    const int kind = tid >> 5, c = tid & 31;
    const int qx = c >> 2, j = c & 3;
    float sum = 0.f;
    for (int y = 0; y < 32; ++y) sum += s_br[(y * 8 + qx) * 2 * V + kind * V + j];
    a.bs.part[(size_t)blockIdx.x * 64 + kind * 32 + c] = sum;
  }
}

int ltd_c0_bwd_parts(int N, int H, int W) {
  const long long tiles = (long long)N * ((H + 1) / 2) * cdiv(W, LC_TW);
  return (int)(tiles < LC_MAXP ? tiles : LC_MAXP);
}

bool ltd_c0_bwd_ok(int dtype, int x_dtype, int XW, const void* x) {
  return (dtype == DT_BF16 || dtype == DT_F16) && x_dtype >= 0 && x_dtype <= 2 && XW % 8 == 0 &&
         (uintptr_t)x % 16 == 0;
}

int ltd_c0_bwd(const LtdC0BwdArgs& a, int dtype, hipStream_t st) {
  if (!ltd_c0_bwd_ok(dtype, a.x_dtype, a.XW, a.x) || a.H != (a.XH - 3) / 2 + 1 ||
      a.W != (a.XW - 3) / 2 + 1 || a.Ho != (a.H - 1) / 2 + 1 || a.Wo != (a.W - 1) / 2 + 1) {
    set_error("ltd_c0_bwd: unsupported shape / dtype / alignment");
    return E_INVALID;
  }
  if (!a.bs.part || !a.bs.z || !a.bs.mean || !a.bs.invstd ||
      (a.bs.mode == 2 && (!a.bs.scale || !a.bs.shift)) || !a.slab || (uintptr_t)a.w % 16 ||
      (uintptr_t)a.dy % 8 || (uintptr_t)a.bs.z % 8) {
    set_error("ltd_c0_bwd: inconsistent arguments");
    return E_INVALID;
  }
  if ((long long)a.N * ((a.H + 1) / 2) * cdiv(a.W, LC_TW) > 0x7fffffffLL ||
      (long long)a.Ho * a.Wo > 0x7fffffffLL / 32) {
    set_error("ltd_c0_bwd: tensor too large");
    return E_INVALID;
  }
  const int P = ltd_c0_bwd_parts(a.N, a.H, a.W);
  // the BN finish as its own fold+finalize launch: measured ~15 us per step faster than in the
  // kernel's last workgroups (whose fold would sit on the backward's critical tail)
  const bool fin = a.tail.counters != nullptr;
  {
    const double px = (double)a.N * a.H * a.W;
    ProfScope ps(PK_CONV0_WGRAD, st,
                 2.0 * ((double)a.N * a.Ho * a.Wo * 32 + px * 32) +
                     (a.x_dtype ? 2.0 : 4.0) * a.N * 3.0 * a.XH * a.XW + 36.0 * 32,
                 18.0 * (double)a.N * a.Ho * a.Wo * 32 + 4.0 * 27 * 32 * px);
#define LC_LAUNCH(T, XB) prof_launch(ltd_c0_bwd_kernel<T, XB>, P, 256, 0, st, a)
#define LC_LAUNCH_X(T)                            \
  do {                                            \
    if (a.x_dtype == 2) LC_LAUNCH(T, 2);          \
    else if (a.x_dtype == 1) LC_LAUNCH(T, 1);     \
    else LC_LAUNCH(T, 0);                         \
  } while (0)
    if (dtype == DT_F16) LC_LAUNCH_X(f16);
    else LC_LAUNCH_X(bf16);
#undef LC_LAUNCH_X
#undef LC_LAUNCH
    const int rc = check_launch("ltd_c0_bwd");
    if (rc || !fin) return rc;
  }
  return bn_bwd_finalize(a.bs.part, P, 32, a.tail.count, a.tail.dgamma, a.tail.dbeta, a.tail.coef,
                         st, a.tail.counters, a.tail.tab);
}

__global__ void conv0_wgrad_combine_kernel(const float* s, const float* tab, const float* mean,
                                           float* dw) {
  const int o = blockIdx.x * 256 + threadIdx.x;
  if (o >= 864) return;
  const int co = o / 27, tap = o - 27 * co;
  const float* e = tab + (size_t)co * BWDX_STRIDE;  // al, be, gz (bn_finish.hpp bn_bwd_finish)
  const float be_c = fmaf(e[2], mean[co], e[1]);     // the constant term about the mean
  dw[o] = fmaf(e[0], s[o], fmaf(e[2], s[864 + o], be_c * s[1728 + tap]));
}

int conv0_wgrad_combine(const float* sums, const float* tab, const float* mean, float* dw,
                        hipStream_t st) {
  prof_launch(conv0_wgrad_combine_kernel, cdiv(864, 256), 256, 0, st, sums, tab, mean, dw);
  return check_launch("conv0_wgrad_combine");
}

}  // namespace fscnn
