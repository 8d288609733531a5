// Inference DSConv in one launch: depthwise 3x3 s1 p1 + BN + ReLU, then 1x1 (128 -> 128) + BN
// (+ a residual) + ReLU, every BatchNorm folded (eval) -- the Classifer's two _DSConv
// (models/fast_scnn.py:228-231, _DSConv :64-79) and the FeatureFusionModule's dwconv +
// conv_lower_res with the high-res branch as the residual (:207-218).
//
// The unfused eval path writes the depthwise output (128 channels at H/8: 134 MB fp32 at cfg2)
// and reads it back in the pointwise GEMM, twice per classifier.  Here a workgroup walks a strip
// of DS_TW output columns down `rs` rows: the three input rows the depthwise window needs sit in
// an LDS ring (each input row is loaded once per strip, the next one in flight during the current
// step), the depthwise output of a row goes to LDS already converted to the pointwise B operand
// (the three bf16 split terms for fp32 plans), and the pointwise weights live in registers
// (already split): HBM sees the input once and the output once.  The loads and stores are buffer
// operations (common.hpp BUF_OOB), so every step issues the same memory operations and the wait
// for the next row leaves the previous stores in flight.
//
// FFM mode (HI): the high-resolution branch (conv_higher_res + BN, :214-215: 64 -> 128 channels at
// the same H x W) is a second GEMM on the same strip -- a row's 16 high-res pixels are loaded with
// the step's other loads, stored to LDS as a B operand, multiplied by that branch's weights
// (registers, pre-split) and used as the residual, so its 128-channel output (134 MB fp32 at cfg2,
// written and read back) never reaches memory either.
//
// Bit-identical to dw_fwd_kernel + gemm_stream(_x3)_kernel by construction: the same depthwise
// fma chain per output (taps in row-major order from 0, fp32), the same folded-BN fma + ReLU and
// rounding to the storage type, and the same pointwise MFMA sequence (weights as the A operand,
// lane (li, lq) holding k = 32 s + 8 lq .. +7, 32-k steps in ascending order, gs_mma_x3 for fp32).
#include "kernels.hpp"

namespace fscnn {

constexpr int DS_C = 128;              // channels in = depthwise channels = pointwise K
constexpr int DS_CO = 128;             // pointwise output channels
constexpr int DS_TW = 16;              // output columns per workgroup (one MFMA pixel group)
constexpr int DS_RP = DS_TW + 2;       // ring pixels per row (the window's halo)
constexpr int DS_PP = DS_C + 4;        // ring floats per pixel (padded)
constexpr int DS_DP = DS_C + 8;        // pointwise operand halves per pixel (padded)
constexpr int DS_UC = 8;               // upsample mode: staged low-resolution columns per strip
constexpr int DS_CH = 64;              // FFM mode: high-resolution branch input channels (K)
constexpr int DS_HP = DS_CH + 8;       // its operand halves per pixel (padded)

template <typename T>
struct DsMma;  // one 16-bit MFMA per operand pair (the 16-bit streaming GEMM's GsMma)
template <>
struct DsMma<bf16> {
  static __device__ __forceinline__ void run(const uint4& w, const uint4& x, f32x4& acc) {
    i16x8 wv, xv;
    __builtin_memcpy(&wv, &w, 16);
    __builtin_memcpy(&xv, &x, 16);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wv, xv, acc, 0, 0, 0);
  }
};
template <>
struct DsMma<f16> {
  static __device__ __forceinline__ void run(const uint4& w, const uint4& x, f32x4& acc) {
    h16x8 wv, xv;
    __builtin_memcpy(&wv, &w, 16);
    __builtin_memcpy(&xv, &x, 16);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(wv, xv, acc, 0, 0, 0);
  }
};
template <>
struct DsMma<float> {
  static __device__ __forceinline__ void run(const uint4&, const uint4&, f32x4&) {}
};

// one logit element (T) through the buffer (range-checked) path
__device__ __forceinline__ void cls_st1(__amdgpu_buffer_rsrc_t r, uint32_t off, float v, float*) {
  __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), r, off, 0, 0);
}
__device__ __forceinline__ void cls_st1(__amdgpu_buffer_rsrc_t r, uint32_t off, float v, bf16*) {
  __builtin_amdgcn_raw_buffer_store_b16(f2bf(v), r, off, 0, 0);
}
__device__ __forceinline__ void cls_st1(__amdgpu_buffer_rsrc_t r, uint32_t off, float v, f16*) {
  __builtin_amdgcn_raw_buffer_store_b16(f2h(v), r, off, 0, 0);
}

template <typename T, bool RES, bool UP, bool CLS = false, bool HI = false>
__global__ __launch_bounds__(256, 2) void dsconv_fwd_kernel(DsArgs a) {
  constexpr bool F32 = sizeof(T) == 4;
  constexpr int NP = F32 ? 3 : 1;                  // pointwise operand planes
  constexpr int VI = 16 / sizeof(T);               // elements per 16-B vector
  constexpr int VPP = DS_C / VI;                   // vectors per input pixel
  constexpr int LP = (DS_RP * VPP + 255) / 256;    // row loads per thread
  __shared__ __attribute__((aligned(16))) float s_ring[3 * DS_RP * DS_PP];   // [row % 3][px][c]
  __shared__ __attribute__((aligned(16))) uint16_t s_d[NP * DS_TW * DS_DP];  // [plane][px][c]
  __shared__ __attribute__((aligned(16))) float s_bn[(HI ? 4 : 2) * DS_CO];  // pointwise (+ high-res) scale, shift
  // FFM mode: the row's high-res pixels as the second GEMM's B operand ([plane][px][k])
  __shared__ __attribute__((aligned(16))) uint16_t s_h[HI ? NP * DS_TW * DS_HP : 8];
  __shared__ __attribute__((aligned(16))) float s_wt[HI && sizeof(T) == 4 ? 9 * DS_C : 4];  // (WT_LDS)
  // upsample mode: the two low-resolution rows x DS_UC columns a ring row interpolates from,
  // double-buffered ([buf][row][col][c], fp32)
  __shared__ __attribute__((aligned(16))) float s_stg[UP ? 2 * 2 * DS_UC * DS_C : 4];
  // classifier mode: its weights as A operand planes ([plane][32 rows][k], rows >= ncls zero)
  // and bias
  __shared__ __attribute__((aligned(16))) uint16_t s_cw[CLS ? NP * 32 * DS_DP : 8];
  __shared__ __attribute__((aligned(16))) float s_cb[CLS ? 32 : 4];

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
  const int ow0 = tw * DS_TW, oh0 = sg * a.rs;
  const size_t img = UP ? (size_t)a.Hi * a.Wi * DS_C : (size_t)a.H * a.W * DS_C;
  const __amdgpu_buffer_rsrc_t xr = buf_rsrc((const T*)a.x + (size_t)n * img, (uint32_t)(img * sizeof(T)));
  const int ldo = CLS ? a.ldl : a.ldy;  // the launch's output: logits (classifier mode) or y
  const size_t ysz = (size_t)a.H * a.W * ldo;
  const __amdgpu_buffer_rsrc_t yr =
      buf_rsrc((T*)(CLS ? a.logits : a.y) + (size_t)n * ysz, (uint32_t)(ysz * sizeof(T)));

  // one input row (the strip's 18 pixels incl. the halo, all channels): per-thread tables
  uint32_t lvo[LP];  // byte offset of the vector in row 0, or BUF_OOB
  int lds[LP];       // ring float offset within a slot, or -1
#pragma unroll
  for (int k = 0; k < LP; ++k) {
    const int i = tid + 256 * k;
    const int px = i / VPP, cv = i - px * VPP;
    const int col = ow0 - 1 + px;
    const bool ok = px < DS_RP && col >= 0 && col < a.W;
    lvo[k] = ok ? (uint32_t)(((size_t)col * DS_C + cv * VI) * sizeof(T)) : BUF_OOB;
    lds[k] = px < DS_RP ? px * DS_PP + cv * VI : -1;
  }
  const uint32_t rowbytes = (uint32_t)((size_t)a.W * DS_C * sizeof(T));
  auto load_row = [&](int r, uint4* raw) {
    const bool rok = r >= 0 && r < a.H;
#pragma unroll
    for (int k = 0; k < LP; ++k) {
      const uint32_t off = rok && lvo[k] != BUF_OOB ? lvo[k] + (uint32_t)r * rowbytes : BUF_OOB;
      const buf_v4u t = __builtin_amdgcn_raw_buffer_load_b128(xr, off, 0, 0);
      raw[k] = make_uint4(t[0], t[1], t[2], t[3]);
    }
  };
  auto store_row = [&](int r, const uint4* raw) {
    float* base = s_ring + ((r + 3) % 3) * DS_RP * DS_PP;  // (r >= -1)
#pragma unroll
    for (int k = 0; k < LP; ++k) {
      if (lds[k] < 0) continue;
      float f[VI];
      if constexpr (F32) {
        f[0] = __uint_as_float(raw[k].x); f[1] = __uint_as_float(raw[k].y);
        f[2] = __uint_as_float(raw[k].z); f[3] = __uint_as_float(raw[k].w);
      } else {
        const uint16_t* e = reinterpret_cast<const uint16_t*>(&raw[k]);
#pragma unroll
        for (int j = 0; j < VI; ++j) f[j] = s16_to<T>(e[j]);
      }
#pragma unroll
      for (int j = 0; j < VI; j += 4)
        *reinterpret_cast<float4*>(base + lds[k] + j) = make_float4(f[j], f[j + 1], f[j + 2], f[j + 3]);
    }
  };

  // ---- upsample mode: a ring row = bilinear (align_corners) of two staged low-res rows --------
  constexpr int LPU = (2 * DS_UC * VPP + 255) / 256;  // staging loads per thread
  const float shs = ac_scale(a.Hi, a.H), sws = ac_scale(a.Wi, a.W);
  const int jlo = UP ? ac_lerp(max(ow0 - 1, 0), a.Wi, a.W, sws).i0 : 0;  // first staged column
  uint32_t uvo[UP ? LPU : 1];  // byte offset of the vector in low-res row 0, or BUF_OOB
  int uls[UP ? LPU : 1];       // staging float offset within a buffer | row << 24, or -1
  if constexpr (UP) {
#pragma unroll
    for (int k = 0; k < LPU; ++k) {
      const int i = tid + 256 * k;
      const int rr = i / (DS_UC * VPP), rem = i - rr * DS_UC * VPP;
      const int j = rem / VPP, cv = rem - j * VPP;
      const bool ok = rr < 2 && jlo + j < a.Wi;
      uvo[k] = ok ? (uint32_t)(((size_t)(jlo + j) * DS_C + cv * VI) * sizeof(T)) : BUF_OOB;
      uls[k] = rr < 2 ? ((rr * DS_UC + j) * DS_C + cv * VI) | (rr << 24) : -1;
    }
  }
  const uint32_t lrowbytes = (uint32_t)((size_t)a.Wi * DS_C * sizeof(T));
  // the two low-res rows of ring row r -> registers
  auto load_up = [&](int r, uint4* raw) {
    const bool rok = r >= 0 && r < a.H;
    const Lerp lh = ac_lerp(rok ? r : 0, a.Hi, a.H, shs);
#pragma unroll
    for (int k = 0; k < LPU; ++k) {
      const int rsel = (uls[k] >> 24) & 1 ? lh.i1 : lh.i0;
      const uint32_t off = rok && uls[k] >= 0 && uvo[k] != BUF_OOB ? uvo[k] + (uint32_t)rsel * lrowbytes : BUF_OOB;
      const buf_v4u t = __builtin_amdgcn_raw_buffer_load_b128(xr, off, 0, 0);
      raw[k] = make_uint4(t[0], t[1], t[2], t[3]);
    }
  };
  auto stage_up = [&](int b, const uint4* raw) {
    float* base = s_stg + b * 2 * DS_UC * DS_C;
#pragma unroll
    for (int k = 0; k < LPU; ++k) {
      if (uls[k] < 0) continue;
      float f[VI];
      if constexpr (F32) {
        f[0] = __uint_as_float(raw[k].x); f[1] = __uint_as_float(raw[k].y);
        f[2] = __uint_as_float(raw[k].z); f[3] = __uint_as_float(raw[k].w);
      } else {
        const uint16_t* e = reinterpret_cast<const uint16_t*>(&raw[k]);
#pragma unroll
        for (int j = 0; j < VI; ++j) f[j] = s16_to<T>(e[j]);
      }
      const int o = uls[k] & 0xFFFFFF;
#pragma unroll
      for (int j = 0; j < VI; j += 4)
        *reinterpret_cast<float4*>(base + o + j) = make_float4(f[j], f[j + 1], f[j + 2], f[j + 3]);
    }
  };
  // ring row r from staging buffer b: up_nhwc's W-then-H lerp2, rounded to the storage type.
  // A thread's items (ring pixel, channel quad) are the same every step: their column taps are
  // computed once (staged columns j0 | j1 << 8 | in-map << 16, and the two weights).
  constexpr int NUI = (DS_RP * (DS_C / 4) + 255) / 256;  // interpolation items per thread
  int ucj[UP ? NUI : 1];
  float ucl0[UP ? NUI : 1], ucl1[UP ? NUI : 1];
  if constexpr (UP) {
#pragma unroll
    for (int k = 0; k < NUI; ++k) {
      const int i = tid + 256 * k;
      const int px = i / (DS_C / 4);
      const int col = ow0 - 1 + px;
      const bool ok = col >= 0 && col < a.W;
      const Lerp lw = ac_lerp(ok ? col : jlo, a.Wi, a.W, sws);
      ucj[k] = (lw.i0 - jlo) | ((lw.i1 - jlo) << 8) | (ok ? 1 << 16 : 0);
      ucl0[k] = lw.l0;
      ucl1[k] = lw.l1;
    }
  }
  auto interp_up = [&](int r, int b) {
    const bool rok = r >= 0 && r < a.H;
    const Lerp lh = ac_lerp(rok ? r : 0, a.Hi, a.H, shs);
    const float* st = s_stg + b * 2 * DS_UC * DS_C;
    float* ring = s_ring + ((r + 3) % 3) * DS_RP * DS_PP;
#pragma unroll
    for (int k = 0; k < NUI; ++k) {
      const int i = tid + 256 * k;
      if (i >= DS_RP * (DS_C / 4)) continue;
      const int px = i / (DS_C / 4), q = i - px * (DS_C / 4);
      const bool ok = rok && (ucj[k] >> 16);
      const int j0 = ucj[k] & 0xFF, j1 = (ucj[k] >> 8) & 0xFF;
      const float l0 = ucl0[k], l1 = ucl1[k];
      const float4 p00 = *reinterpret_cast<const float4*>(st + j0 * DS_C + 4 * q);
      const float4 p01 = *reinterpret_cast<const float4*>(st + j1 * DS_C + 4 * q);
      const float4 p10 = *reinterpret_cast<const float4*>(st + (DS_UC + j0) * DS_C + 4 * q);
      const float4 p11 = *reinterpret_cast<const float4*>(st + (DS_UC + j1) * DS_C + 4 * q);
      const float a00[4] = {p00.x, p00.y, p00.z, p00.w}, a01[4] = {p01.x, p01.y, p01.z, p01.w};
      const float a10[4] = {p10.x, p10.y, p10.z, p10.w}, a11[4] = {p11.x, p11.y, p11.z, p11.w};
      float o[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float v = lerp2(lh.l0, lerp2(l0, a00[j], l1, a01[j]), lh.l1,
                              lerp2(l0, a10[j], l1, a11[j]));
        o[j] = ok ? round_as<T>(v) : 0.f;
      }
      *reinterpret_cast<float4*>(ring + px * DS_PP + 4 * q) = make_float4(o[0], o[1], o[2], o[3]);
    }
  };

  // depthwise: thread = channel quad qd x output pixels 2 pp, 2 pp + 1; taps and BN in registers
  const int qd = tid & 31, pp = tid >> 5;
  // (fp32 FFM mode: the taps in LDS, [9][C], read per kernel row -- the high-res branch's split
  // weights need their 48 registers)
  constexpr bool WT_LDS = HI && F32;
  float wt[WT_LDS ? 1 : 9][4], dsc[4], dsh[4];
  if constexpr (WT_LDS) {
    for (int i = tid; i < 9 * DS_C; i += 256) {
      const int t = i / DS_C, c = i - t * DS_C;
      s_wt[i] = a.wd[c * 9 + t];
    }
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    if constexpr (!WT_LDS) {
#pragma unroll
      for (int t = 0; t < 9; ++t) wt[t][j] = a.wd[(4 * qd + j) * 9 + t];
    }
    dsc[j] = a.scd[4 * qd + j];
    dsh[j] = a.shd[4 * qd + j];
  }
  // pointwise: wave w = output channel tiles 2w, 2w + 1 (weights as the A operand, in registers)
  uint4 wpr[2][4][NP];
#pragma unroll
  for (int u = 0; u < 2; ++u)
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int co = 16 * (2 * wave + u) + li, k = 32 * s + 8 * lq;
      if constexpr (F32) {
        const float* wr = (const float*)a.wp + (size_t)co * DS_C + k;
        gs_split3(*reinterpret_cast<const uint4*>(wr), *reinterpret_cast<const uint4*>(wr + 4), wpr[u][s]);
      } else {
        wpr[u][s][0] = *reinterpret_cast<const uint4*>((const T*)a.wp + (size_t)co * DS_C + k);
      }
    }
  for (int i = tid; i < DS_CO; i += 256) {
    s_bn[i] = a.scp[i];
    s_bn[DS_CO + i] = a.shp[i];
    if constexpr (HI) {
      s_bn[2 * DS_CO + i] = a.sch[i];
      s_bn[3 * DS_CO + i] = a.shh[i];
    }
  }
  // FFM mode: this thread's 16-B vector of a row's DS_TW high-res pixels (16-bit plans: threads
  // >= 128 load nothing), and the high-res weights of the wave's output tiles (pre-split)
  constexpr int VH = DS_CH / VI;  // vectors per high-res pixel
  const size_t himg = HI ? (size_t)a.H * a.W * a.ldxh : 0;
  const __amdgpu_buffer_rsrc_t hr =
      buf_rsrc(HI ? (const T*)a.xh + (size_t)n * himg : (const T*)a.x, (uint32_t)(himg * sizeof(T)));
  const uint32_t hrowbytes = (uint32_t)((size_t)a.W * a.ldxh * sizeof(T));
  uint32_t hvo = BUF_OOB;
  int hls = -1;
  uint4 wph[2][2][HI ? NP : 1];
  if constexpr (HI) {
    const int px = tid / VH, cv = tid - px * VH;
    if (px < DS_TW) {
      hls = px * DS_HP + cv * VI;
      if (ow0 + px < a.W) hvo = (uint32_t)(((size_t)(ow0 + px) * a.ldxh + cv * VI) * sizeof(T));
    }
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int co = 16 * (2 * wave + u) + li, k = 32 * s + 8 * lq;
        if constexpr (F32) {
          const float* wr = (const float*)a.wh + (size_t)co * DS_CH + k;
          gs_split3(*reinterpret_cast<const uint4*>(wr), *reinterpret_cast<const uint4*>(wr + 4), wph[u][s]);
        } else {
          wph[u][s][0] = *reinterpret_cast<const uint4*>((const T*)a.wh + (size_t)co * DS_CH + k);
        }
      }
  }
  if constexpr (CLS) {  // the classifier weights, split once (fp32) into the A operand planes
    for (int i = tid; i < 32 * (DS_CO / 8); i += 256) {
      const int row = i / (DS_CO / 8), k = (i - row * (DS_CO / 8)) * 8;
      const bool ok = row < a.ncls;
      uint4 pl[NP];
      if constexpr (F32) {
        const float* wr = (const float*)a.wc + (size_t)(ok ? row : 0) * DS_CO + k;
        const uint4 lo = ok ? *reinterpret_cast<const uint4*>(wr) : make_uint4(0u, 0u, 0u, 0u);
        const uint4 hi = ok ? *reinterpret_cast<const uint4*>(wr + 4) : make_uint4(0u, 0u, 0u, 0u);
        gs_split3(lo, hi, pl);
      } else {
        pl[0] = ok ? *reinterpret_cast<const uint4*>((const T*)a.wc + (size_t)row * DS_CO + k)
                   : make_uint4(0u, 0u, 0u, 0u);
      }
#pragma unroll
      for (int j = 0; j < NP; ++j)
        *reinterpret_cast<uint4*>(s_cw + (j * 32 + row) * DS_DP + k) = pl[j];
    }
    if (tid < 32) s_cb[tid] = tid < a.ncls ? a.bc[tid] : 0.f;
  }

  // ---- prologue: rows oh0 - 1, oh0 in the ring, row oh0 + 1 in flight ------------------------
  // (upsample mode: rows oh0 - 1, oh0 interpolated into the ring, row oh0 + 1's low-res rows in
  // staging buffer (oh0 - 1) & 1, row oh0 + 2's in flight)
  uint4 nxt[UP ? LPU : LP];
  if constexpr (UP) {
    uint4 raw[LPU];
    load_up(oh0 - 1, raw);
    stage_up(0, raw);
    __syncthreads();
    interp_up(oh0 - 1, 0);
    load_up(oh0, raw);
    stage_up(1, raw);
    __syncthreads();
    interp_up(oh0, 1);
    __syncthreads();
    load_up(oh0 + 1, raw);
    stage_up((oh0 - 1) & 1, raw);
    load_up(oh0 + 2, nxt);
  } else {
    uint4 raw[LP];
    load_row(oh0 - 1, raw);
    store_row(oh0 - 1, raw);
    load_row(oh0, raw);
    store_row(oh0, raw);
    load_row(oh0 + 1, nxt);
  }
  {  // dropped stores: the loop is entered, as it loops, with its stores after the row loads
    // (2 output vectors per step, or 4 logit elements in classifier mode)
    const float z[4] = {0.f, 0.f, 0.f, 0.f};
    if constexpr (CLS) {
#pragma unroll
      for (int j = 0; j < 4; ++j) cls_st1(yr, BUF_OOB + 64 * j, 0.f, (T*)nullptr);
    } else {
      buf_st4(yr, BUF_OOB, z, (T*)nullptr);
      buf_st4(yr, BUF_OOB + 64, z, (T*)nullptr);
    }
  }
  if constexpr (UP) __syncthreads();  // (staging of row oh0 + 1 before step oh0 interpolates it)
  stamp(a.stamps, 1);

  const int oh_end = min(oh0 + a.rs, a.H);
  constexpr bool res = RES;
  const __amdgpu_buffer_rsrc_t rr =
      buf_rsrc(RES ? (const T*)a.r + (size_t)n * a.H * a.W * a.ldr : (const T*)a.x,
               RES ? (uint32_t)((size_t)a.H * a.W * a.ldr * sizeof(T)) : 0u);
  for (int oh = oh0; oh < oh_end; ++oh) {
    // this step's residual, before the row prefetch (so waiting for it does not wait for that)
    float rv[2][4];
    uint4 hraw = make_uint4(0u, 0u, 0u, 0u);  // (FFM mode) this thread's high-res vector of row oh
    if constexpr (HI) {
      const uint32_t off = hvo != BUF_OOB ? hvo + (uint32_t)oh * hrowbytes : BUF_OOB;
      const buf_v4u t = __builtin_amdgcn_raw_buffer_load_b128(hr, off, 0, 0);
      hraw = make_uint4(t[0], t[1], t[2], t[3]);
    }
    if constexpr (RES) {
      const int ow = ow0 + li;
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int c = 16 * (2 * wave + u) + 4 * lq;
        const uint32_t off = ow < a.W ? (uint32_t)((((size_t)oh * a.W + ow) * a.ldr + c) * sizeof(T)) : BUF_OOB;
        if constexpr (F32) {
          const buf_v4u t = __builtin_amdgcn_raw_buffer_load_b128(rr, off, 0, 0);
#pragma unroll
          for (int j = 0; j < 4; ++j) rv[u][j] = __uint_as_float(t[j]);
        } else {
          const buf_v2u t = __builtin_amdgcn_raw_buffer_load_b64(rr, off, 0, 0);
          rv[u][0] = s16_to<T>((uint16_t)(t[0] & 0xFFFF)); rv[u][1] = s16_to<T>((uint16_t)(t[0] >> 16));
          rv[u][2] = s16_to<T>((uint16_t)(t[1] & 0xFFFF)); rv[u][3] = s16_to<T>((uint16_t)(t[1] >> 16));
        }
      }
    }
    if constexpr (UP) {
      stage_up(oh & 1, nxt);      // row oh + 2's low-res rows (its interpolation: next step)
      interp_up(oh + 1, (oh - 1) & 1);  // (the slot of row oh - 2: dw(oh - 1) is done)
      load_up(oh + 3, nxt);       // (also past the end: a fixed count per step)
    } else {
      store_row(oh + 1, nxt);  // (the slot of row oh - 2: its last reader, dw(oh - 1), is done)
      load_row(oh + 2, nxt);   // (also past the end: a fixed count per step)
    }
    __syncthreads();
    if (oh == oh0 + a.rs / 2) stamp(a.stamps, 2);
    // ---- depthwise of row oh, two pixels per thread -> s_d as the pointwise B operand --------
    {
      float acc[2][4];
#pragma unroll
      for (int p = 0; p < 2; ++p)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[p][j] = 0.f;
#pragma unroll
      for (int kh = 0; kh < 3; ++kh) {
        float wk[3][4];
#pragma unroll
        for (int kw = 0; kw < 3; ++kw) {
          if constexpr (WT_LDS) {
            const float4 t = *reinterpret_cast<const float4*>(s_wt + (kh * 3 + kw) * DS_C + 4 * qd);
            wk[kw][0] = t.x; wk[kw][1] = t.y; wk[kw][2] = t.z; wk[kw][3] = t.w;
          } else {
#pragma unroll
            for (int j = 0; j < 4; ++j) wk[kw][j] = wt[kh * 3 + kw][j];
          }
        }
        const float* rowp = s_ring + ((oh - 1 + kh + 3) % 3) * DS_RP * DS_PP + 4 * qd;
#pragma unroll
        for (int ci = 0; ci < 4; ++ci) {  // ring pixels 2 pp + ci
          const float4 v = *reinterpret_cast<const float4*>(rowp + (2 * pp + ci) * DS_PP);
          const float vv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
          for (int p = 0; p < 2; ++p) {
            const int kw = ci - p;
            if (kw < 0 || kw > 2) continue;
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[p][j] = fmaf(vv[j], wk[kw][j], acc[p][j]);
          }
        }
      }
#pragma unroll
      for (int p = 0; p < 2; ++p) {
        float o4[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) o4[j] = round_as<T>(fmaxf(acc[p][j] * dsc[j] + dsh[j], 0.f));
        uint16_t* d = s_d + (2 * pp + p) * DS_DP + 4 * qd;
        if constexpr (F32) {  // gs_split3's terms, one plane each
          uint32_t p0[4], p1[4], p2[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const uint32_t u = __float_as_uint(o4[j]), b0 = u & 0xFFFF0000u;
            const float r1 = o4[j] - __uint_as_float(b0);
            const uint32_t b1 = __float_as_uint(r1) & 0xFFFF0000u;
            const float r2 = r1 - __uint_as_float(b1);
            p0[j] = b0;
            p1[j] = b1;
            p2[j] = __float_as_uint(r2) & 0xFFFF0000u;
          }
          *reinterpret_cast<uint2*>(d) = make_uint2((p0[0] >> 16) | p0[1], (p0[2] >> 16) | p0[3]);
          *reinterpret_cast<uint2*>(d + DS_TW * DS_DP) = make_uint2((p1[0] >> 16) | p1[1], (p1[2] >> 16) | p1[3]);
          *reinterpret_cast<uint2*>(d + 2 * DS_TW * DS_DP) = make_uint2((p2[0] >> 16) | p2[1], (p2[2] >> 16) | p2[3]);
        } else {
          *reinterpret_cast<uint2*>(d) =
              make_uint2((uint32_t)s16_from<T>(o4[0]) | ((uint32_t)s16_from<T>(o4[1]) << 16),
                         (uint32_t)s16_from<T>(o4[2]) | ((uint32_t)s16_from<T>(o4[3]) << 16));
        }
      }
    }
    if constexpr (HI) {  // the high-res vector -> s_h (the split terms, one plane each, for fp32)
      if (hls >= 0) {
        uint16_t* d = s_h + hls;
        if constexpr (F32) {
          const uint32_t v4[4] = {hraw.x, hraw.y, hraw.z, hraw.w};
          uint32_t p0[4], p1[4], p2[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const float f = __uint_as_float(v4[j]);
            const uint32_t b0 = v4[j] & 0xFFFF0000u;
            const float r1 = f - __uint_as_float(b0);
            const uint32_t b1 = __float_as_uint(r1) & 0xFFFF0000u;
            const float r2 = r1 - __uint_as_float(b1);
            p0[j] = b0;
            p1[j] = b1;
            p2[j] = __float_as_uint(r2) & 0xFFFF0000u;
          }
          *reinterpret_cast<uint2*>(d) = make_uint2((p0[0] >> 16) | p0[1], (p0[2] >> 16) | p0[3]);
          *reinterpret_cast<uint2*>(d + DS_TW * DS_HP) = make_uint2((p1[0] >> 16) | p1[1], (p1[2] >> 16) | p1[3]);
          *reinterpret_cast<uint2*>(d + 2 * DS_TW * DS_HP) = make_uint2((p2[0] >> 16) | p2[1], (p2[2] >> 16) | p2[3]);
        } else {
          *reinterpret_cast<uint4*>(d) = hraw;
        }
      }
    }
    __syncthreads();
    if (oh == oh0 + a.rs / 2) stamp(a.stamps, 3);
    // ---- pointwise: 16 pixels x this wave's 32 output channels, K = 128 in four 32-k steps ----
    float ocls[2][4];  // (classifier mode) the pointwise output of this lane
    {
      f32x4 acc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        uint4 xs[NP];
#pragma unroll
        for (int j = 0; j < NP; ++j)
          xs[j] = *reinterpret_cast<const uint4*>(s_d + j * DS_TW * DS_DP + li * DS_DP + 32 * s + 8 * lq);
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          if constexpr (F32) gs_mma_x3(wpr[u][s], xs, acc[u]);
          else DsMma<T>::run(wpr[u][s][0], xs[0], acc[u]);
        }
      }
      if constexpr (HI) {  // the high-res branch: BN_h(W_h * xh), rounded as the unfused path stores it
        f32x4 ah[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          uint4 xs[NP];
#pragma unroll
          for (int j = 0; j < NP; ++j)
            xs[j] = *reinterpret_cast<const uint4*>(s_h + j * DS_TW * DS_HP + li * DS_HP + 32 * s + 8 * lq);
#pragma unroll
          for (int u = 0; u < 2; ++u) {
            if constexpr (F32) gs_mma_x3(wph[u][s], xs, ah[u]);
            else DsMma<T>::run(wph[u][s][0], xs[0], ah[u]);
          }
        }
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const int c = 16 * (2 * wave + u) + 4 * lq;
          const float4 sc = *reinterpret_cast<const float4*>(&s_bn[2 * DS_CO + c]);
          const float4 sh = *reinterpret_cast<const float4*>(&s_bn[3 * DS_CO + c]);
          const float scv[4] = {sc.x, sc.y, sc.z, sc.w}, shv[4] = {sh.x, sh.y, sh.z, sh.w};
          float hv[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) hv[r] = ah[u][r] * scv[r] + shv[r];
          if constexpr (F32) {
#pragma unroll
            for (int r = 0; r < 4; ++r) rv[u][r] = hv[r];
          } else {
            // the fp32 value first, then its 16-bit rounding, as the unfused GEMM stores it (left
            // alone, the compiler fuses the two into v_fma_mix: one rounding instead of two)
#pragma unroll
            for (int r = 0; r < 4; ++r) asm volatile("" : "+v"(hv[r]));
#pragma unroll
            for (int r = 0; r < 4; r += 2) {
              const uint32_t pk = (uint32_t)s16_from<T>(hv[r]) | ((uint32_t)s16_from<T>(hv[r + 1]) << 16);
              rv[u][r] = s16_to<T>((uint16_t)(pk & 0xFFFFu));
              rv[u][r + 1] = s16_to<T>((uint16_t)(pk >> 16));
            }
          }
        }
      }
      const int ow = ow0 + li;
      const uint32_t yoff = ow < a.W ? (uint32_t)((((size_t)oh * a.W + ow) * a.ldy) * sizeof(T)) : BUF_OOB;
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int c = 16 * (2 * wave + u) + 4 * lq;
        const float4 sc = *reinterpret_cast<const float4*>(&s_bn[c]);
        const float4 sh = *reinterpret_cast<const float4*>(&s_bn[DS_CO + c]);
        const float scv[4] = {sc.x, sc.y, sc.z, sc.w}, shv[4] = {sh.x, sh.y, sh.z, sh.w};
        float o4[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float v = acc[u][r] * scv[r] + shv[r];
          if constexpr (RES || HI) v += rv[u][r];
          o4[r] = fmaxf(v, 0.f);
        }
        if constexpr (CLS) {
          ocls[u][0] = o4[0]; ocls[u][1] = o4[1]; ocls[u][2] = o4[2]; ocls[u][3] = o4[3];
        } else {
          buf_st4(yr, yoff == BUF_OOB ? BUF_OOB : yoff + c * (uint32_t)sizeof(T), o4, (T*)nullptr);
        }
      }
    }
    if constexpr (CLS) {
      // ---- classifier 1x1 on the pointwise output: its values (rounded as the unfused path
      // stores them) -> s_d as the classifier's B operand -> 2 waves x 16 classes x 16 pixels
      __syncthreads();  // every wave's pointwise reads of s_d are done
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int c = 16 * (2 * wave + u) + 4 * lq;
        uint16_t* d = s_d + li * DS_DP + c;
        if constexpr (F32) {
          uint32_t p0[4], p1[4], p2[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const uint32_t uu = __float_as_uint(ocls[u][j]), b0 = uu & 0xFFFF0000u;
            const float r1 = ocls[u][j] - __uint_as_float(b0);
            const uint32_t b1 = __float_as_uint(r1) & 0xFFFF0000u;
            const float r2 = r1 - __uint_as_float(b1);
            p0[j] = b0;
            p1[j] = b1;
            p2[j] = __float_as_uint(r2) & 0xFFFF0000u;
          }
          *reinterpret_cast<uint2*>(d) = make_uint2((p0[0] >> 16) | p0[1], (p0[2] >> 16) | p0[3]);
          *reinterpret_cast<uint2*>(d + DS_TW * DS_DP) = make_uint2((p1[0] >> 16) | p1[1], (p1[2] >> 16) | p1[3]);
          *reinterpret_cast<uint2*>(d + 2 * DS_TW * DS_DP) = make_uint2((p2[0] >> 16) | p2[1], (p2[2] >> 16) | p2[3]);
        } else {
          *reinterpret_cast<uint2*>(d) =
              make_uint2((uint32_t)s16_from<T>(ocls[u][0]) | ((uint32_t)s16_from<T>(ocls[u][1]) << 16),
                         (uint32_t)s16_from<T>(ocls[u][2]) | ((uint32_t)s16_from<T>(ocls[u][3]) << 16));
        }
      }
      __syncthreads();
      const int ot = wave & 1;  // class tile (waves 2, 3 compute tile 0, 1 again: dropped stores)
      f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        uint4 xs[NP], ws[NP];
#pragma unroll
        for (int j = 0; j < NP; ++j) {
          xs[j] = *reinterpret_cast<const uint4*>(s_d + j * DS_TW * DS_DP + li * DS_DP + 32 * s + 8 * lq);
          ws[j] = *reinterpret_cast<const uint4*>(s_cw + (j * 32 + 16 * ot + li) * DS_DP + 32 * s + 8 * lq);
        }
        if constexpr (F32) gs_mma_x3(ws, xs, acc);
        else DsMma<T>::run(ws[0], xs[0], acc);
      }
      const int ow = ow0 + li;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int co = 16 * ot + 4 * lq + r;
        const float v = acc[r] * 1.f + s_cb[co];
        const bool ok = wave < 2 && ow < a.W && co < a.ncls;
        cls_st1(yr, ok ? (uint32_t)((((size_t)oh * a.W + ow) * a.ldl + co) * sizeof(T)) : BUF_OOB, v,
                (T*)nullptr);
      }
    }
    if (oh == oh0 + a.rs / 2) stamp(a.stamps, 4);
  }
  stamp(a.stamps, 5);
}

// upsample mode: the low-res columns any strip's 18 ring pixels interpolate from fit DS_UC
static bool ds_up_fits(const DsArgs& a) {
  if (a.Hi <= 0) return true;
  if (a.Wi <= 0 || a.Hi > a.H || a.Wi > a.W) return false;
  const float sw = ac_scale(a.Wi, a.W);
  for (int ow0 = 0; ow0 < a.W; ow0 += DS_TW) {
    const int lo = ac_lerp(std::max(ow0 - 1, 0), a.Wi, a.W, sw).i0;
    const int hi = ac_lerp(std::min(ow0 + DS_TW, a.W - 1), a.Wi, a.W, sw).i1;
    if (hi - lo + 1 > DS_UC) return false;
  }
  return 4LL * a.Hi * a.Wi * DS_C < (long long)BUF_OOB;
}

bool ds_ok(const DsArgs& a) {
  // upsample mode (Hi > 0) is the FFM form only: its low-res input is read through the upsample
  // ring, which the plain strip kernel (no r / xh) does not have
  if (a.Hi > 0 && !a.r && !a.xh) return false;
  // the kernels read / write these with 16-B vector accesses
  if (((uintptr_t)a.wp & 15) || ((uintptr_t)a.wc & 15) || ((uintptr_t)a.logits & 15)) return false;
  if (a.xh && (a.r || a.wc || a.Hi <= 0 || !a.wh || !a.sch || !a.shh || a.ldxh < DS_CH || a.ldxh % 8 ||
               ((uintptr_t)a.xh & 15) || ((uintptr_t)a.wh & 15) || 4LL * a.H * a.W * a.ldxh >= (long long)BUF_OOB))
    return false;
  if (a.wc && (a.r || a.Hi > 0 || !a.bc || !a.logits || a.ncls < 1 || a.ncls > 32 ||
               a.ldl < a.ncls || 4LL * a.H * a.W * a.ldl >= (long long)BUF_OOB))
    return false;
  return ds_up_fits(a) && a.N > 0 && a.N < 65536 && a.H > 0 && a.W > 0 && a.C == DS_C && a.Co == DS_CO &&
         (a.r == nullptr || (a.ldr >= DS_CO && a.ldr % 4 == 0 && ((uintptr_t)a.r & 15) == 0 &&
                             4LL * a.H * a.W * a.ldr < (long long)BUF_OOB)) &&
         a.rs >= 1 && cdiv(a.H, a.rs) < 65536 && a.ldy >= DS_CO && a.ldy % 4 == 0 &&
         ((uintptr_t)a.x & 15) == 0 && ((uintptr_t)a.y & 15) == 0 &&
         // per-image buffer ranges below BUF_OOB (32-bit buffer offsets)
         4LL * a.H * a.W * DS_C < (long long)BUF_OOB && 4LL * a.H * a.W * a.ldy < (long long)BUF_OOB;
}

// rows walked per workgroup: whole rounds of the 2-per-CU grid where the map allows
int ds_rows(int N, int H, int W) {
  const long long slots = 2LL * 256;
  int best = 8;
  double best_eff = -1.0;
  for (int rs = 4; rs <= 16; ++rs) {
    const long long wg = (long long)N * cdiv(W, DS_TW) * cdiv(H, rs);
    const long long rounds = (wg + slots - 1) / slots;
    const double eff = (double)wg / (double)(rounds * slots) * rs / (rs + 2.0);  // (+2: prologue rows)
    if (eff > best_eff + 1e-9) { best_eff = eff; best = rs; }
  }
  return best;
}

int ds_fwd(const DsArgs& a, int dtype, hipStream_t st) {
  if (!ds_ok(a)) {
    set_error("ds_fwd: unsupported shape N=%d H=%d W=%d C=%d Co=%d ldy=%d rs=%d", a.N, a.H, a.W,
              a.C, a.Co, a.ldy, a.rs);
    return E_UNSUPPORTED;
  }
  DsArgs as = a;
  as.stamps = stamp_region();
  const dim3 g(cdiv(a.W, DS_TW), cdiv(a.H, a.rs), a.N);
  const double E = dtype == DT_F32 ? 4.0 : 2.0;
  ProfScope ps(PK_DSCONV, st,
               E * a.N * ((a.Hi > 0 ? (double)a.Hi * a.Wi : (double)a.H * a.W) * DS_C +
                          (double)a.H * a.W * (DS_CO + (a.r ? DS_CO : 0) + (a.xh ? DS_CH : 0))),
               2.0 * a.N * a.H * a.W * (9.0 * DS_C + (double)DS_C * DS_CO + (a.xh ? (double)DS_CH * DS_CO : 0.0) +
                                        (a.wc ? (double)DS_CO * a.ncls : 0.0)));
#define DSK(T)                                                                \
  do {                                                                        \
    if (a.wc) prof_launch(dsconv_fwd_kernel<T, false, false, true>, g, 256, 0, st, as);    \
    else if (a.xh) prof_launch(dsconv_fwd_kernel<T, false, true, false, true>, g, 256, 0, st, as); \
    else if (a.r && a.Hi > 0) prof_launch(dsconv_fwd_kernel<T, true, true>, g, 256, 0, st, as); \
    else if (a.r) prof_launch(dsconv_fwd_kernel<T, true, false>, g, 256, 0, st, as);   \
    else prof_launch(dsconv_fwd_kernel<T, false, false>, g, 256, 0, st, as);           \
  } while (0)
  if (dtype == DT_F32) DSK(float);
  else if (dtype == DT_F16) DSK(f16);
  else DSK(bf16);
#undef DSK
  return check_launch("ds_fwd");
}

// ---- LearningToDownsample.dsconv2 (inference): depthwise 3x3 s2 (48 ch) + BN + ReLU and
// pointwise 48 -> 64 + BN + ReLU in one launch (models/fast_scnn.py:155, _DSConv :64-79) ------
// The unfused eval path writes the depthwise output (48 channels at H/8: 50 MB fp32 at cfg2) and
// reads it back in the pointwise GEMM.  Here a workgroup owns 4 output rows x 16 columns: the
// depthwise outputs (every tap loaded from L2/L1: a stride-2 window shares a third of its input
// with its neighbour) go to LDS as the pointwise B operand, K zero-padded 48 -> 64, and each wave
// multiplies one 16-pixel group by the 64 x 64 weights (LDS, split into three bf16 terms for
// fp32 plans).  Bit-identical to dw_fwd_kernel<T, 2> + the streaming pointwise GEMM
// (gemm_stream_x3_kernel fp32 / gemm_stream_kernel 16-bit, M >= 4096): the same depthwise fma
// chain per output (taps row-major, zero-padded taps included), the same folded-BN fma + ReLU and
// rounding to the storage type, the same MFMA sequence (weights as the A operand, lane (li, lq)
// holding k = 32 s + 8 lq .. +7, s ascending) and epilogue.
constexpr int D2_C = 48, D2_CO = 64, D2_TW = 16, D2_R = 4, D2_PX = D2_TW * D2_R;
constexpr int D2_KV = 8;            // 16-B operand vectors per weight row (K padded to 64)
constexpr int D2_WST = D2_KV + 1;   // padded LDS row stride (vectors)
constexpr int D2_DP = 64 + 8;       // depthwise output row (elements, padded) in LDS

template <typename T>
__global__ __launch_bounds__(256) void ds2_fwd_kernel(Ds2Args a) {
  constexpr bool F32 = sizeof(T) == 4;
  constexpr int NP = F32 ? 3 : 1;
  __shared__ __attribute__((aligned(16))) uint4 s_w[NP * D2_CO * D2_WST];  // [plane][co][k vec]
  __shared__ __attribute__((aligned(16))) T s_d[D2_PX * D2_DP];            // [px][k], k >= 48: 0
  __shared__ __attribute__((aligned(16))) float s_wd[9 * D2_C];            // [tap][c]
  __shared__ float s_bn[2 * D2_C + 2 * D2_CO];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int li = lane & 15, lq = lane >> 4;
  const int ow0 = blockIdx.x * D2_TW, oh0 = blockIdx.y * D2_R, n = blockIdx.z;
  stamp(a.stamps, 0);
  // pointwise weights: [co][48] storage dtype -> operand vectors (fp32: three truncation planes)
  for (int i = tid; i < D2_CO * D2_KV; i += 256) {
    const int r = i / D2_KV, v = i - r * D2_KV, k = v * 8;
    const bool ok = k < D2_C;
    const T* src = (const T*)a.wp + (size_t)r * D2_C + (ok ? k : 0);
    if constexpr (F32) {
      uint4 lo4 = *reinterpret_cast<const uint4*>(src), hi4 = *reinterpret_cast<const uint4*>(src + 4);
      if (!ok) lo4 = hi4 = make_uint4(0u, 0u, 0u, 0u);
      uint4 t[3];
      gs_split3(lo4, hi4, t);
#pragma unroll
      for (int j = 0; j < 3; ++j) s_w[(j * D2_CO + r) * D2_WST + v] = t[j];
    } else {
      const uint4 t = *reinterpret_cast<const uint4*>(src);
      s_w[r * D2_WST + v] = ok ? t : make_uint4(0u, 0u, 0u, 0u);
    }
  }
  for (int i = tid; i < 9 * D2_C; i += 256) s_wd[(i % 9) * D2_C + i / 9] = a.wd[i];
  if (tid < D2_C) {
    s_bn[tid] = a.scd[tid];
    s_bn[D2_C + tid] = a.shd[tid];
  }
  if (tid < D2_CO) {
    s_bn[2 * D2_C + tid] = a.scp[tid];
    s_bn[2 * D2_C + D2_CO + tid] = a.shp[tid];
  }
  // the K padding of the depthwise operand (k = 48 .. 63) is zero
  for (int i = tid; i < D2_PX * 16; i += 256) st1(s_d + (i >> 4) * D2_DP + D2_C + (i & 15), 0.f);
  __syncthreads();
  // ---- depthwise: 64 pixels x 12 channel quads, 3 per thread; all 27 loads in flight ----------
  const T* X = (const T*)a.x + (size_t)n * a.H * a.W * D2_C;
  float xv[3][9][4];
#pragma unroll
  for (int u = 0; u < 3; ++u) {
    const int id = tid + 256 * u, px = id / 12, cq = id - px * 12;
    const int oh = oh0 + px / D2_TW, ow = ow0 + (px & (D2_TW - 1));
#pragma unroll
    for (int kh = 0; kh < 3; ++kh)
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) {
        const int ih = 2 * oh - 1 + kh, iw = 2 * ow - 1 + kw;
        const bool ok = oh < a.Ho && ow < a.Wo && ih >= 0 && ih < a.H && iw >= 0 && iw < a.W;
        const size_t off = ok ? ((size_t)ih * a.W + iw) * D2_C + 4 * cq : 0;
        float v[4];
        ld4v(X + off, v);
#pragma unroll
        for (int j = 0; j < 4; ++j) xv[u][kh * 3 + kw][j] = ok ? v[j] : 0.f;
      }
  }
#pragma unroll
  for (int u = 0; u < 3; ++u) {
    const int id = tid + 256 * u, px = id / 12, cq = id - px * 12;
    const int c0 = 4 * cq;
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const float4 w4 = *reinterpret_cast<const float4*>(s_wd + t * D2_C + c0);
      const float wv[4] = {w4.x, w4.y, w4.z, w4.w};
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[j] = fmaf(xv[u][t][j], wv[j], acc[j]);
    }
    float o[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float t = acc[j] * s_bn[c0 + j] + s_bn[D2_C + c0 + j];
      o[j] = fmaxf(t, 0.f);
    }
    st4v(s_d + px * D2_DP + c0, o);
  }
  __syncthreads();
  stamp(a.stamps, 1);
  // ---- pointwise: wave w = output row oh0 + w, lane li = column ow0 + li ------------------------
  const int px = wave * D2_TW + li;
  f32x4 acc[4];
#pragma unroll
  for (int nt = 0; nt < 4; ++nt) acc[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    const int k = 32 * s + 8 * lq;
    if constexpr (F32) {
      const float* d = reinterpret_cast<const float*>(s_d) + px * D2_DP + k;
      uint4 xs[3];
      gs_split3(*reinterpret_cast<const uint4*>(d), *reinterpret_cast<const uint4*>(d + 4), xs);
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
        uint4 w[3];
#pragma unroll
        for (int j = 0; j < 3; ++j) w[j] = s_w[(j * D2_CO + nt * 16 + li) * D2_WST + 4 * s + lq];
        gs_mma_x3(w, xs, acc[nt]);
      }
    } else {
      const uint4 xs = *reinterpret_cast<const uint4*>(s_d + px * D2_DP + k);
#pragma unroll
      for (int nt = 0; nt < 4; ++nt)
        DsMma<T>::run(s_w[(nt * 16 + li) * D2_WST + 4 * s + lq], xs, acc[nt]);
    }
  }
  const int oh = oh0 + wave, ow = ow0 + li;
  if (oh < a.Ho && ow < a.Wo) {
    T* y = (T*)a.y + (((size_t)n * a.Ho + oh) * a.Wo + ow) * a.ldy;
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      const int nl = nt * 16 + 4 * lq;
      float o[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float v = acc[nt][r] * s_bn[2 * D2_C + nl + r] + s_bn[2 * D2_C + D2_CO + nl + r];
        o[r] = fmaxf(v, 0.f);
      }
      st4v(y + nl, o);
    }
  }
  stamp(a.stamps, 2);
}

bool ds2_ok(const Ds2Args& a) {
  return a.N > 0 && a.N < 65536 && a.H > 0 && a.W > 0 && a.Ho == (a.H - 1) / 2 + 1 &&
         a.Wo == (a.W - 1) / 2 + 1 && cdiv(a.Ho, D2_R) < 65536 && a.ldy >= D2_CO && a.ldy % 4 == 0 &&
         ((uintptr_t)a.x & 15) == 0 && ((uintptr_t)a.y & 15) == 0 && ((uintptr_t)a.wp & 15) == 0 &&
         a.wd && a.scd && a.shd && a.scp && a.shp;
}

int ds2_fwd(const Ds2Args& a, int dtype, hipStream_t st) {
  if (!ds2_ok(a)) {
    set_error("ds2_fwd: unsupported shape N=%d H=%d W=%d -> %dx%d ldy=%d", a.N, a.H, a.W, a.Ho,
              a.Wo, a.ldy);
    return E_UNSUPPORTED;
  }
  Ds2Args as = a;
  as.stamps = stamp_region();
  const dim3 g(cdiv(a.Wo, D2_TW), cdiv(a.Ho, D2_R), a.N);
  const double E = dtype == DT_F32 ? 4.0 : 2.0;
  ProfScope ps(PK_DSCONV, st, E * a.N * ((double)a.H * a.W * D2_C + (double)a.Ho * a.Wo * D2_CO),
               2.0 * a.N * a.Ho * a.Wo * (9.0 * D2_C + (double)D2_C * D2_CO));
  if (dtype == DT_F32) prof_launch(ds2_fwd_kernel<float>, g, 256, 0, st, as);
  else if (dtype == DT_F16) prof_launch(ds2_fwd_kernel<f16>, g, 256, 0, st, as);
  else prof_launch(ds2_fwd_kernel<bf16>, g, 256, 0, st, as);
  return check_launch("ds2_fwd");
}

}  // namespace fscnn
