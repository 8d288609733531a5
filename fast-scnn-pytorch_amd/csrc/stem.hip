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
  const dim3 grid(cdiv(a.W2, ST_TW), cdiv(a.H2, ST_TH), a.N);
  StemArgs as = a;
  as.stamps = stamp_region();
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
