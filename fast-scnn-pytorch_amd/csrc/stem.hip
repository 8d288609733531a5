// Inference LearningToDownsample stem in one launch: conv (3x3 s2 p0, 3 -> 32) + BN + ReLU
// (models/fast_scnn.py:153 / :52), dsconv1.dw (3x3 s2 p1 depthwise) + BN + ReLU and dsconv1.pw
// (1x1, 32 -> 48) + BN + ReLU (:154, _DSConv :64-78), every BatchNorm folded (eval).
//
// The unfused eval path writes conv0's 32-channel map (H/2) and the depthwise output (H/4) to
// HBM and reads both back: at cfg2 (8 x 3 x 1024 x 2048 fp32) 537 + 134 MB written and read again
// around three launches.  Here a workgroup owns a TH2 x TW2 tile of dsconv1 outputs and computes,
// in LDS only, the (2TH2+1) x (2TW2+1) conv0 pixels its depthwise window reads, then the
// depthwise outputs, then their 48 pointwise channels: HBM sees the image once and the stem
// output once.
//
// (r05 alternatives measured at cfg2 fp32, forward ms per batch: 512-thread workgroups 2.174 vs
// 2.163; a persistent tile loop with the next tile's image in flight 2.381 -- its 80-register
// budget at 3 workgroups per CU spills)
//
// Bit-identical to the three unfused launches (conv0_fwd_kernel, dw_fwd_kernel,
// gemm_stream(_x3)_kernel) by construction: the same MFMA fragments and instruction sequence per
// output (conv0: common.hpp C0Mma over k = 8 lq + e; pointwise: weights as the A operand,
// k = 8 lq .. 8 lq + 7 of one 32-k step, gs_split3 / gs_mma_x3 for fp32), the same depthwise fma
// chain (taps in row-major order from 0), the same folded-BN fma + ReLU, and every intermediate
// rounded to the storage type where the unfused path stores it.  Conv0 pixels outside the map are
// the depthwise's zero padding; halo conv0 pixels are recomputed by both neighbouring tiles.
#include "kernels.hpp"

namespace fscnn {

constexpr int ST_TH = 4, ST_TW = 16;                      // dsconv1 outputs per workgroup
constexpr int ST_CR = 2 * ST_TH + 1, ST_CC = 2 * ST_TW + 1;  // conv0 tile (9 x 33)
constexpr int ST_NPX = ST_CR * ST_CC;                     // 297 conv0 pixels
constexpr int ST_NG = (ST_NPX + 15) / 16;                 // 19 MFMA pixel groups
constexpr int ST_GPW = (ST_NG + 3) / 4;                   // groups per wave (5)
constexpr int ST_IR = 2 * ST_CR + 1, ST_IC = 2 * ST_CC + 1;  // image tile (19 x 67) per channel
constexpr int ST_PS = 36;                                 // LDS floats per staged pixel (32 + pad)
constexpr int ST_NO = ST_TH * ST_TW;                      // 64 dsconv1 outputs
constexpr int ST_C1 = 32, ST_C2 = 48;                     // LTD channels (fast_scnn.py:20)

template <typename T>
struct StPw;
template <>
struct StPw<bf16> {
  static __device__ __forceinline__ void run(const uint4& w, const uint4& x, f32x4& acc) {
    i16x8 wv, xv;
    __builtin_memcpy(&wv, &w, 16);
    __builtin_memcpy(&xv, &x, 16);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wv, xv, acc, 0, 0, 0);
  }
};
template <>
struct StPw<f16> {
  static __device__ __forceinline__ void run(const uint4& w, const uint4& x, f32x4& acc) {
    h16x8 wv, xv;
    __builtin_memcpy(&wv, &w, 16);
    __builtin_memcpy(&xv, &x, 16);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(wv, xv, acc, 0, 0, 0);
  }
};

// 8 T-rounded floats -> one 16-B vector of T bits (exact)
template <typename T>
__device__ __forceinline__ uint4 st_pack8(const float (&v)[8]) {
  uint32_t w[4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
    w[i] = (uint32_t)s16_from<T>(v[2 * i]) | ((uint32_t)s16_from<T>(v[2 * i + 1]) << 16);
  return make_uint4(w[0], w[1], w[2], w[3]);
}

// XB: image dtype code (0 fp32, 1 bf16, 2 fp16); T: the plan's storage type
template <typename T, int XB>
__global__ __launch_bounds__(256, 3) void stem_fwd_kernel(StemArgs a) {
  constexpr int BF = sizeof(T) == 4 ? 0 : (std::is_same<T, f16>::value ? 2 : 1);
  using M = C0Mma<BF>;
  using TI = typename std::conditional<XB != 0, uint16_t, float>::type;
  constexpr int VI = 16 / sizeof(TI);                 // image elements per 16-B vector
  constexpr int NVC = (ST_IC + 2 * VI - 2) / VI;      // vectors per staged image row
  constexpr int SW = NVC * VI;                        // staged row width (floats)
  constexpr int NIV = 3 * ST_IR * NVC;                // image vectors per tile
  constexpr int LPV = (NIV + 255) / 256;
  constexpr int IN_F = 3 * ST_IR * SW;                // staged image floats
  constexpr int C0_F = ST_NPX * ST_PS;                // conv0 tile floats (aliases the image)
  constexpr int R0_F = IN_F > C0_F ? IN_F : C0_F;
  __shared__ __attribute__((aligned(16))) float s_raw[R0_F + ST_NO * ST_PS];
  float* s_in = s_raw;                 // [ci][ir][SW]
  float* s_c0 = s_raw;                 // [px][ST_PS] (after the image is consumed)
  float* s_dw = s_raw + R0_F;          // [o][ST_PS]

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int li = lane & 15, lq = lane >> 4;
  // tile -> (tw, th, n), XCD-contiguous (speed only: neighbouring tiles share halo rows in L2)
  int tw, th, n;
  {
    const int gx = gridDim.x, gy = gridDim.y;
    const long long T_ = (long long)gx * gy * gridDim.z;
    long long L = blockIdx.x + (long long)gx * (blockIdx.y + (long long)gy * blockIdx.z);
    if ((T_ & 7) == 0) L = (L & 7) * (T_ >> 3) + (L >> 3);
    tw = (int)(L % gx);
    const long long r = L / gx;
    th = (int)(r % gy);
    n = (int)(r / gy);
  }
  stamp(a.stamps, 0);
  const int th0 = th * ST_TH, tw0 = tw * ST_TW;       // first dsconv1 output
  const int r1o = 2 * th0 - 1, c1o = 2 * tw0 - 1;     // conv0 tile origin (may be -1: padding)
  const int iro = 2 * r1o, ico = 2 * c1o;             // image tile origin
  const int cbase = (ico >= 0 ? ico / VI : -((-ico + VI - 1) / VI)) * VI;  // floor to a vector
  const int coff = ico - cbase;                        // in [0, VI)

  // ---- stage the 3 x 19 x 67 image tile (aligned vector superset; outside = 0) --------------
  {
    const TI* xin = (const TI*)a.x;
    uint4 raw[LPV];
#pragma unroll
    for (int k = 0; k < LPV; ++k) {
      const int i = tid + 256 * k;
      const int cr = i / NVC, v = i - cr * NVC;  // cr = ci * IR + r
      const int ci = cr / ST_IR, r = cr - ci * ST_IR;
      const int ir = iro + r, ic = cbase + v * VI;
      const bool ok = i < NIV && ir >= 0 && ir < a.H && ic >= 0 && ic + VI <= a.W;
      const size_t off = ok ? (((size_t)n * 3 + ci) * a.H + ir) * a.W + ic : 0;
      raw[k] = sel4(ok, *reinterpret_cast<const uint4*>(xin + off));
    }
#pragma unroll
    for (int k = 0; k < LPV; ++k) {
      const int i = tid + 256 * k;
      if (i >= NIV) continue;
      const int cr = i / NVC, v = i - cr * NVC;
      const TI* e = reinterpret_cast<const TI*>(&raw[k]);
#pragma unroll
      for (int j = 0; j < VI; ++j) {
        float f;
        if (XB) f = in16<XB>((uint16_t)e[j]);
        else f = (float)e[j];
        s_in[cr * SW + v * VI + j] = f;
      }
    }
  }
  // conv0 B fragments W[16 jt + li][8 lq + e] (k >= 27 -> 0), folded BN of the lane's channels
  typename M::Frag bw[2];
  float fsc[2], fsh[2];
#pragma unroll
  for (int jt = 0; jt < 2; ++jt) {
    float wv[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int k = 8 * lq + e;
      const float t = a.w0[(16 * jt + li) * 27 + (k < 27 ? k : 0)];
      wv[e] = k < 27 ? t : 0.f;
    }
    bw[jt] = M::pack(wv);
    fsc[jt] = a.sc0[16 * jt + li];
    fsh[jt] = a.sh0[16 * jt + li];
  }
  int koff[8];  // tap k -> offset in s_in from the pixel's image origin
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const int k = 8 * lq + e;
    const int kk = k < 27 ? k : 0;
    const int ci = kk / 9, kh = (kk % 9) / 3, kw = kk % 3;
    koff[e] = (ci * ST_IR + kh) * SW + kw + coff;
  }
  __syncthreads();
  stamp(a.stamps, 1);

  // ---- conv0 on the 9 x 33 tile: wave w takes pixel groups w, w + 4, ... -------------------
  f32x4 c0v[ST_GPW][2];
#pragma unroll
  for (int gi = 0; gi < ST_GPW; ++gi) {
    const int g = wave + 4 * gi;
    const int px = 16 * g + li;                         // A row = conv0 pixel
    const int p = px < ST_NPX ? px : 0;
    const int cr = p / ST_CC, cc = p - cr * ST_CC;
    float av[8];
#pragma unroll
    for (int e = 0; e < 8; ++e)
      av[e] = 8 * lq + e < 27 ? s_in[koff[e] + 2 * cr * SW + 2 * cc] : 0.f;
    const typename M::Frag af = M::pack(av);
#pragma unroll
    for (int jt = 0; jt < 2; ++jt) {
      f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
      if (g < ST_NG) M::mma(af, bw[jt], acc);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float v = acc[q] * fsc[jt] + fsh[jt];
        acc[q] = round_as<T>(fmaxf(v, 0.f));
      }
      c0v[gi][jt] = acc;
    }
  }
  stamp(a.stamps, 2);
  __syncthreads();  // every wave is done reading the image tile (s_c0 aliases it)
#pragma unroll
  for (int gi = 0; gi < ST_GPW; ++gi) {
    const int g = wave + 4 * gi;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int p = 16 * g + 4 * lq + q;  // output row of the MFMA tile = conv0 pixel
      if (g >= ST_NG || p >= ST_NPX) continue;
      const int cr = p / ST_CC, cc = p - cr * ST_CC;
      const int r1 = r1o + cr, c1 = c1o + cc;
      const bool in = r1 >= 0 && r1 < a.H1 && c1 >= 0 && c1 < a.W1;  // else dw zero padding
#pragma unroll
      for (int jt = 0; jt < 2; ++jt) s_c0[p * ST_PS + 16 * jt + li] = in ? c0v[gi][jt][q] : 0.f;
    }
  }
  __syncthreads();
  stamp(a.stamps, 3);

  // ---- dsconv1.dw: thread (quad qd, outputs os, os + 32); taps in row-major order ----------
  {
    const int qd = tid & 7, os = tid >> 3;
    float wt[9][4], sc[4], sh[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
#pragma unroll
      for (int t = 0; t < 9; ++t) wt[t][j] = a.wd[(4 * qd + j) * 9 + t];
      sc[j] = a.scd[4 * qd + j];
      sh[j] = a.shd[4 * qd + j];
    }
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int o = os + 32 * h;
      const int orow = o / ST_TW, ocol = o - orow * ST_TW;
      float acc[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kh = 0; kh < 3; ++kh)
#pragma unroll
        for (int kw = 0; kw < 3; ++kw) {
          const float4 v = *reinterpret_cast<const float4*>(
              &s_c0[((2 * orow + kh) * ST_CC + 2 * ocol + kw) * ST_PS + 4 * qd]);
          const float vv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[j] = fmaf(vv[j], wt[kh * 3 + kw][j], acc[j]);
        }
      float o4[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float t = acc[j] * sc[j] + sh[j];
        o4[j] = round_as<T>(fmaxf(t, 0.f));
      }
      *reinterpret_cast<float4*>(&s_dw[o * ST_PS + 4 * qd]) = make_float4(o4[0], o4[1], o4[2], o4[3]);
    }
  }
  __syncthreads();
  stamp(a.stamps, 4);

  // ---- dsconv1.pw: wave w = outputs 16w .. 16w + 15 x 48 channels (3 column tiles) --------
  {
    const int o = 16 * wave + li;                        // B column = dsconv1 output (pixel)
    const float4 x0 = *reinterpret_cast<const float4*>(&s_dw[o * ST_PS + 8 * lq]);
    const float4 x1 = *reinterpret_cast<const float4*>(&s_dw[o * ST_PS + 8 * lq + 4]);
    f32x4 acc[3];
    if constexpr (sizeof(T) == 4) {
      uint4 xs[3];
      gs_split3(make_uint4(__float_as_uint(x0.x), __float_as_uint(x0.y), __float_as_uint(x0.z),
                           __float_as_uint(x0.w)),
                make_uint4(__float_as_uint(x1.x), __float_as_uint(x1.y), __float_as_uint(x1.z),
                           __float_as_uint(x1.w)), xs);
#pragma unroll
      for (int nt = 0; nt < 3; ++nt) {
        const float* wr = (const float*)a.wp + (size_t)(16 * nt + li) * ST_C1 + 8 * lq;
        uint4 w3[3];
        gs_split3(*reinterpret_cast<const uint4*>(wr), *reinterpret_cast<const uint4*>(wr + 4), w3);
        acc[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
        gs_mma_x3(w3, xs, acc[nt]);
      }
    } else {
      const float xv[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
      const uint4 xb = st_pack8<T>(xv);
#pragma unroll
      for (int nt = 0; nt < 3; ++nt) {
        const uint4 w = *reinterpret_cast<const uint4*>((const T*)a.wp + (size_t)(16 * nt + li) * ST_C1 + 8 * lq);
        acc[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
        StPw<T>::run(w, xb, acc[nt]);
      }
    }
    const int oh = th0 + o / ST_TW, ow = tw0 + o % ST_TW;
    if (oh < a.H2 && ow < a.W2) {
      T* yp = (T*)a.y + (((size_t)n * a.H2 + oh) * a.W2 + ow) * a.ldy;
#pragma unroll
      for (int nt = 0; nt < 3; ++nt) {
        const int c = 16 * nt + 4 * lq;
        float o4[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float v = acc[nt][r] * a.scp[c + r] + a.shp[c + r];
          o4[r] = fmaxf(v, 0.f);
        }
        st4v(yp + c, o4);
      }
    }
  }
  stamp(a.stamps, 5);
}

// ---- row-walking form ---------------------------------------------------------------------
// A workgroup owns a strip of SW_TW dsconv1 output columns and walks SW_RS output rows down it.
// Each step needs two new conv0 rows (the third, 2 oh - 1, is the previous step's) and four new
// image rows (the fifth is the previous step's): conv0 rows are computed once per strip (no
// vertical halo), the next step's image rows are in flight during the current step, and the
// rings are small (41 KB fp32: 3 workgroups per CU).  Per step: image rows -> ring, conv0 (MFMA)
// -> ring, depthwise -> s_dw, pointwise -> HBM; the arithmetic per output is the one-tile
// kernel's (bit-identical).
constexpr int SW_TW = 32;                      // dsconv1 output columns per workgroup
constexpr int SW_RS = 16;                      // dsconv1 output rows walked per workgroup
constexpr int SW_CC = 2 * SW_TW + 1;           // conv0 columns (65)
constexpr int SW_IC = 2 * SW_CC + 1;           // image columns (131)
constexpr int SW_NIR = 5;                      // image ring rows
constexpr int SW_NCR = 3;                      // conv0 ring rows

template <typename T, int XB>
__global__ __launch_bounds__(256, 3) void stem_walk_kernel(StemArgs a) {
  constexpr int BF = sizeof(T) == 4 ? 0 : (std::is_same<T, f16>::value ? 2 : 1);
  using M = C0Mma<BF>;
  using TI = typename std::conditional<XB != 0, uint16_t, float>::type;
  constexpr int VI = 16 / sizeof(TI);               // image elements per 16-B vector
  constexpr int COFF = VI - 2;                      // image column 4 ow0 - 2 in the staged row
  constexpr int NVC = (SW_IC + COFF + VI - 1) / VI; // vectors per staged image row
  constexpr int SWD = NVC * VI;                     // staged row width (floats)
  constexpr int LP4 = (4 * 3 * NVC + 255) / 256;    // loads per thread: 4 image rows
  constexpr int LP7 = (7 * 3 * NVC + 255) / 256;    // ... 7 image rows (the first step)
  // image row r lives at slots r % 5 and r % 5 + 5, so the 3 rows 2 r1 .. 2 r1 + 2 of a conv0
  // row r1 are 3 consecutive slots from (2 r1) % 5: the tap offsets stay per-lane constants
  __shared__ __attribute__((aligned(16))) float s_img[2 * SW_NIR * 3 * SWD];  // [slot][ci][col]
  __shared__ __attribute__((aligned(16))) float s_wd[9 * ST_C1];             // [tap][ch]
  __shared__ __attribute__((aligned(16))) float s_c0[SW_NCR * SW_CC * ST_PS];  // [row % 3][col][ch]
  __shared__ __attribute__((aligned(16))) float s_dw[SW_TW * ST_PS];        // [o][ch]

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int li = lane & 15, lq = lane >> 4;
  int tw, sg, n;  // strip, row segment, image: XCD-contiguous (speed only)
  {
    const int gx = gridDim.x, gy = gridDim.y;
    const long long T_ = (long long)gx * gy * gridDim.z;
    long long L = blockIdx.x + (long long)gx * (blockIdx.y + (long long)gy * blockIdx.z);
    if ((T_ & 7) == 0) L = (L & 7) * (T_ >> 3) + (L >> 3);
    tw = (int)(L % gx);
    const long long r = L / gx;
    sg = (int)(r % gy);
    n = (int)(r / gy);
  }
  stamp(a.stamps, 0);
  const int ow0 = tw * SW_TW, oh0 = sg * SW_RS;
  const int c1o = 2 * ow0 - 1;                // conv0 column origin (-1: the depthwise padding)
  const int cbase = 4 * ow0 - 2 - COFF;       // first staged image column (a vector boundary)
  const TI* xin = (const TI*)a.x;

  // image rows [r0, r0 + R) of all 3 channels: 16-B vector loads into registers / into the ring
  auto load_rows = [&](int r0, int R, uint4* raw, int LP) {
#pragma unroll
    for (int k = 0; k < LP; ++k) {
      const int i = tid + 256 * k;
      const int row = i / (3 * NVC), rem = i - row * 3 * NVC;
      const int ci = rem / NVC, v = rem - ci * NVC;
      const int ir = r0 + row, ic = cbase + v * VI;
      const bool ok = row < R && ir >= 0 && ir < a.H && ic >= 0 && ic + VI <= a.W;
      const size_t off = ok ? (((size_t)n * 3 + ci) * a.H + ir) * a.W + ic : 0;
      raw[k] = sel4(ok, *reinterpret_cast<const uint4*>(xin + off));
    }
  };
  auto store_rows = [&](int r0, int R, const uint4* raw, int LP) {
#pragma unroll
    for (int k = 0; k < LP; ++k) {
      const int i = tid + 256 * k;
      const int row = i / (3 * NVC), rem = i - row * 3 * NVC;
      if (row >= R) continue;
      const int ci = rem / NVC, v = rem - ci * NVC;
      const int slot = (r0 + row + 4 * SW_NIR) % SW_NIR;  // (r0 >= -2)
      const TI* e = reinterpret_cast<const TI*>(&raw[k]);
      float f[VI];
#pragma unroll
      for (int j = 0; j < VI; ++j) {
        if (XB) f[j] = in16<XB>((uint16_t)e[j]);
        else f[j] = (float)e[j];
      }
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        float* d = s_img + ((slot + h * SW_NIR) * 3 + ci) * SWD + v * VI;
#pragma unroll
        for (int j = 0; j < VI; j += 4)
          *reinterpret_cast<float4*>(d + j) = make_float4(f[j], f[j + 1], f[j + 2], f[j + 3]);
      }
    }
  };
  // conv0 B fragments and folded BN (the one-tile kernel's)
  typename M::Frag bw[2];
  float fsc[2], fsh[2];
#pragma unroll
  for (int jt = 0; jt < 2; ++jt) {
    float wv[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int k = 8 * lq + e;
      const float t = a.w0[(16 * jt + li) * 27 + (k < 27 ? k : 0)];
      wv[e] = k < 27 ? t : 0.f;
    }
    bw[jt] = M::pack(wv);
    fsc[jt] = a.sc0[16 * jt + li];
    fsh[jt] = a.sh0[16 * jt + li];
  }
  int koff[8];  // tap k = 8 lq + e -> (kh * 3 + ci) * SWD + kw + COFF from the row's first slot
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const int k = 8 * lq + e;
    const int kk = k < 27 ? k : 0;
    koff[e] = ((kk % 9) / 3 * 3 + kk / 9) * SWD + kk % 3 + COFF;
  }
  for (int i = tid; i < 9 * ST_C1; i += 256) s_wd[i] = a.wd[(i % ST_C1) * 9 + i / ST_C1];
  // conv0 rows [r0, r0 + NR) x the strip's 65 columns -> conv0 ring (zero outside the map)
  auto conv0_rows = [&](int r0, auto NRc) {
    constexpr int NR = decltype(NRc)::value;
    constexpr int NG = (NR * SW_CC + 15) / 16;
    constexpr int GPW = (NG + 3) / 4;
    f32x4 c0v[GPW][2];
#pragma unroll
    for (int gi = 0; gi < GPW; ++gi) {
      const int g = wave + 4 * gi;
      const int px = 16 * g + li;
      const int p = px < NR * SW_CC ? px : 0;
      const int rr = p / SW_CC, cc = p - rr * SW_CC;
      const float* base = s_img + ((2 * (r0 + rr) + 4 * SW_NIR) % SW_NIR) * 3 * SWD + 2 * cc;
      float av[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) av[e] = 8 * lq + e < 27 ? base[koff[e]] : 0.f;
      const typename M::Frag af = M::pack(av);
#pragma unroll
      for (int jt = 0; jt < 2; ++jt) {
        f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
        if (g < NG) M::mma(af, bw[jt], acc);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float v = acc[q] * fsc[jt] + fsh[jt];
          acc[q] = round_as<T>(fmaxf(v, 0.f));
        }
        c0v[gi][jt] = acc;
      }
    }
#pragma unroll
    for (int gi = 0; gi < GPW; ++gi) {
      const int g = wave + 4 * gi;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int p = 16 * g + 4 * lq + q;
        if (g >= NG || p >= NR * SW_CC) continue;
        const int rr = p / SW_CC, cc = p - rr * SW_CC;
        const int r1 = r0 + rr, c1 = c1o + cc;
        const bool in = r1 >= 0 && r1 < a.H1 && c1 >= 0 && c1 < a.W1;
        float* d = s_c0 + (((r1 + 3 * SW_NCR) % SW_NCR) * SW_CC + cc) * ST_PS;
#pragma unroll
        for (int jt = 0; jt < 2; ++jt) d[16 * jt + li] = in ? c0v[gi][jt][q] : 0.f;
      }
    }
  };

  // ---- first step's rows: image rows 4 oh0 - 2 .. 4 oh0 + 4, conv0 rows 2 oh0 - 1 .. + 1 ------
  {
    uint4 raw[LP7];
    load_rows(4 * oh0 - 2, 7, raw, LP7);
    store_rows(4 * oh0 - 2, 7, raw, LP7);
  }
  __syncthreads();
  conv0_rows(2 * oh0 - 1, std::integral_constant<int, 3>());
  uint4 nxt[LP4];  // the next step's 4 image rows
  load_rows(4 * oh0 + 5, 4, nxt, LP4);
  __syncthreads();
  stamp(a.stamps, 1);

  // per-thread depthwise / pointwise constants
  const int qd = tid & 7, o = tid >> 3;         // depthwise: channel quad, output column
  const int pg = wave & 1;                      // pointwise: pixel group (outputs 16 pg ..)
  const int nt0 = wave < 2 ? 0 : 2, ntn = wave < 2 ? 2 : 1;
  for (int s = 0; s < SW_RS; ++s) {
    const int oh = oh0 + s;
    if (oh >= a.H2) break;  // (workgroup-uniform)
    if (s > 0) {
      store_rows(4 * oh + 1, 4, nxt, LP4);
      if (s + 1 < SW_RS) load_rows(4 * oh + 5, 4, nxt, LP4);
      __syncthreads();
      conv0_rows(2 * oh, std::integral_constant<int, 2>());
      __syncthreads();
    }
    // ---- dsconv1.dw of output row oh: conv0 rows 2 oh - 1 .. 2 oh + 1 (taps in row-major order)
    {
      float acc[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kh = 0; kh < 3; ++kh) {
        const float* rowp = s_c0 + ((2 * oh - 1 + kh + 3 * SW_NCR) % SW_NCR) * SW_CC * ST_PS;
#pragma unroll
        for (int kw = 0; kw < 3; ++kw) {
          const float4 v = *reinterpret_cast<const float4*>(&rowp[(2 * o + kw) * ST_PS + 4 * qd]);
          const float vv[4] = {v.x, v.y, v.z, v.w};
          const float4 w = *reinterpret_cast<const float4*>(&s_wd[(kh * 3 + kw) * ST_C1 + 4 * qd]);
          const float ww[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[j] = fmaf(vv[j], ww[j], acc[j]);
        }
      }
      float o4[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float t = acc[j] * a.scd[4 * qd + j] + a.shd[4 * qd + j];
        o4[j] = round_as<T>(fmaxf(t, 0.f));
      }
      *reinterpret_cast<float4*>(&s_dw[o * ST_PS + 4 * qd]) = make_float4(o4[0], o4[1], o4[2], o4[3]);
    }
    __syncthreads();
    // ---- dsconv1.pw: pixel group pg x column tiles {0, 1} (waves 0, 1) or {2} (waves 2, 3) ---
    {
      const int op = 16 * pg + li;
      const float4 x0 = *reinterpret_cast<const float4*>(&s_dw[op * ST_PS + 8 * lq]);
      const float4 x1 = *reinterpret_cast<const float4*>(&s_dw[op * ST_PS + 8 * lq + 4]);
      f32x4 acc[2];
      if constexpr (sizeof(T) == 4) {
        uint4 xs[3];
        gs_split3(make_uint4(__float_as_uint(x0.x), __float_as_uint(x0.y), __float_as_uint(x0.z),
                             __float_as_uint(x0.w)),
                  make_uint4(__float_as_uint(x1.x), __float_as_uint(x1.y), __float_as_uint(x1.z),
                             __float_as_uint(x1.w)), xs);
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          acc[u] = f32x4{0.f, 0.f, 0.f, 0.f};
          if (u < ntn) {
            const float* wr = (const float*)a.wp + (size_t)(16 * (nt0 + u) + li) * ST_C1 + 8 * lq;
            uint4 w3[3];
            gs_split3(*reinterpret_cast<const uint4*>(wr), *reinterpret_cast<const uint4*>(wr + 4), w3);
            gs_mma_x3(w3, xs, acc[u]);
          }
        }
      } else {
        const float xv[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
        const uint4 xb = st_pack8<T>(xv);
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          acc[u] = f32x4{0.f, 0.f, 0.f, 0.f};
          if (u < ntn) {
            const uint4 w = *reinterpret_cast<const uint4*>(
                (const T*)a.wp + (size_t)(16 * (nt0 + u) + li) * ST_C1 + 8 * lq);
            StPw<T>::run(w, xb, acc[u]);
          }
        }
      }
      const int ow = ow0 + op;
      if (ow < a.W2) {
        T* yp = (T*)a.y + (((size_t)n * a.H2 + oh) * a.W2 + ow) * a.ldy;
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          if (u >= ntn) continue;
          const int c = 16 * (nt0 + u) + 4 * lq;
          float o4[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float v = acc[u][r] * a.scp[c + r] + a.shp[c + r];
            o4[r] = fmaxf(v, 0.f);
          }
          st4v(yp + c, o4);
        }
      }
    }
  }
  stamp(a.stamps, 2);
}

bool stem_ok(const StemArgs& a) {
  const int VI = a.x_dtype ? 8 : 4;
  const int ve = VI == 8 ? 4 : (a.ldy % 4 == 0 ? 4 : 0);  // 4-channel output vectors aligned
  return a.N > 0 && a.H >= 3 && a.W >= 3 && a.W % VI == 0 && ((uintptr_t)a.x & 15) == 0 &&
         ve == 4 && a.ldy >= ST_C2 && a.ldy % 4 == 0 &&
         a.H1 == (a.H - 3) / 2 + 1 && a.W1 == (a.W - 3) / 2 + 1 && a.H2 == (a.H1 - 1) / 2 + 1 &&
         a.W2 == (a.W1 - 1) / 2 + 1 && (long long)a.N * cdiv(a.H2, ST_TH) < 65536;
}

int stem_fwd(const StemArgs& a, int dtype, hipStream_t st) {
  if (!stem_ok(a)) {
    set_error("stem_fwd: unsupported shape N=%d H=%d W=%d (W %% %d, 16-B aligned image)", a.N,
              a.H, a.W, a.x_dtype ? 8 : 4);
    return E_UNSUPPORTED;
  }
  StemArgs as = a;
  as.stamps = stamp_region();
  static const bool walk = [] {
    const char* e = getenv("FSCNN_STEM_WALK");
    return e && e[0] == '1';
  }();
  if (walk) {
    const dim3 gw(cdiv(a.W2, SW_TW), cdiv(a.H2, SW_RS), a.N);
    ProfScope pw_(PK_STEM, st, (a.x_dtype ? 2.0 : 4.0) * a.N * 3.0 * a.H * a.W +
                                   (dtype == DT_F32 ? 4.0 : 2.0) * (double)a.N * a.H2 * a.W2 * ST_C2,
                  0.0);
#define STEMW(T)                                                                  \
  do {                                                                            \
    if (a.x_dtype == 2) stem_walk_kernel<T, 2><<<gw, 256, 0, st>>>(as);           \
    else if (a.x_dtype == 1) stem_walk_kernel<T, 1><<<gw, 256, 0, st>>>(as);      \
    else stem_walk_kernel<T, 0><<<gw, 256, 0, st>>>(as);                          \
  } while (0)
    if (dtype == DT_F32) STEMW(float);
    else if (dtype == DT_F16) STEMW(f16);
    else STEMW(bf16);
#undef STEMW
    return check_launch("stem_fwd");
  }
  const dim3 grid(cdiv(a.W2, ST_TW), cdiv(a.H2, ST_TH), a.N);
  const double px0 = (double)a.N * a.H1 * a.W1, px2 = (double)a.N * a.H2 * a.W2;
  const int E = dtype == DT_F32 ? 4 : 2;
  ProfScope ps(PK_STEM, st, (a.x_dtype ? 2.0 : 4.0) * a.N * 3.0 * a.H * a.W + (double)E * px2 * ST_C2,
               2.0 * 27 * ST_C1 * px0 + 2.0 * 9 * ST_C1 * px2 + 2.0 * ST_C1 * ST_C2 * px2);
#define STEM_L(T)                                                                  \
  do {                                                                             \
    if (a.x_dtype == 2) stem_fwd_kernel<T, 2><<<grid, 256, 0, st>>>(as);            \
    else if (a.x_dtype == 1) stem_fwd_kernel<T, 1><<<grid, 256, 0, st>>>(as);       \
    else stem_fwd_kernel<T, 0><<<grid, 256, 0, st>>>(as);                           \
  } while (0)
  if (dtype == DT_F32) STEM_L(float);
  else if (dtype == DT_F16) STEM_L(f16);
  else STEM_L(bf16);
#undef STEM_L
  return check_launch("stem_fwd");
}

}  // namespace fscnn
