// Inference LearningToDownsample stem in one launch: conv (3x3 s2 p0, 3 -> 32) + BN + ReLU
// (models/fast_scnn.py:153 / :52), dsconv1.dw (3x3 s2 p1 depthwise) + BN + ReLU and dsconv1.pw
// (1x1, 32 -> 48) + BN + ReLU (:154, _DSConv :64-78), every BatchNorm folded (eval).
//
// The unfused eval path writes conv0's 32-channel map (H/2) and the depthwise output (H/4) to
// HBM and reads both back: at cfg2 (8 x 3 x 1024 x 2048 fp32) 537 + 134 MB written and read again
// around three launches.  Here a workgroup walks a strip of dsconv1 outputs row by row with the
// conv0 rows and image rows its depthwise window needs in LDS rings: HBM sees the image once and
// the stem output once, and each conv0 pixel is computed once per strip.
//
// The kernel is instruction-issue bound (cfg2 fp32: ~7.4 K VALU instructions per wave, three
// waves per SIMD; SQ counters in DESIGN.md), so operands are converted once per element, not
// once per use: the image ring holds conv0's A operand (the bf16 split terms for fp32), the
// depthwise output is stored as the pointwise B operand, the pointwise weights sit in registers
// already split.  r05 history at cfg2 fp32 (stem kernel us): a one-tile kernel (4 x 16 outputs,
// its haloed 9 x 33 conv0 tile recomputed per tile) 265; this walk 245 (first form) -> 206
// (counted vmcnt waits, 31-column strips = 8 whole pixel groups per conv0 row pair) -> 196
// (pre-converted operands).  Rejected: 512-thread one-tile workgroups, a persistent one-tile
// loop (spills).
//
// Bit-identical to the three unfused launches (conv0_fwd_kernel, dw_fwd_kernel,
// gemm_stream(_x3)_kernel) by construction: the same MFMA fragments and instruction sequence per
// output (conv0: common.hpp C0Mma over k = 8 lq + e; pointwise: weights as the A operand,
// k = 8 lq .. 8 lq + 7 of one 32-k step, gs_split3 / gs_mma_x3 for fp32), the same depthwise fma
// chain (taps in row-major order from 0), the same folded-BN fma + ReLU, and every intermediate
// rounded to the storage type where the unfused path stores it.  Conv0 pixels outside the map are
// the depthwise's zero padding.
#include "kernels.hpp"

namespace fscnn {

constexpr int ST_PS = 36;                                 // LDS floats per conv0 pixel (32 + pad)
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

// ---- the walk --------------------------------------------------------------------------------
// A workgroup owns a strip of SW_TW dsconv1 output columns and walks SW_RS output rows down it.
// Each step needs two new conv0 rows (the third, 2 oh - 1, is the previous step's) and four new
// image rows (the fifth is the previous step's; a prologue computes conv0 row 2 oh0 - 1): conv0
// rows are computed once per strip, and the next step's image rows are in flight during the
// current step.  That overlap needs counted waits: the image loads and the output stores are
// buffer operations whose range check replaces the edge branches (an out-of-range lane loads 0 /
// stores nothing), so every step issues the same number of memory operations, and every
// constant lives in LDS (a global load of one inside the loop would wait for the prefetch too).
// Per step: image rows -> ring, conv0 (MFMA) -> ring, depthwise -> s_dw, pointwise -> HBM; the
// arithmetic per output is the one-tile kernel's (bit-identical).
constexpr int SW_TW = 31;                      // dsconv1 output columns per workgroup
constexpr int SW_RS = 16;                      // dsconv1 output rows walked per workgroup
constexpr int SW_CC = 2 * SW_TW + 1;           // conv0 columns (63: two rows = 8 pixel groups)
constexpr int SW_CP = SW_CC + 1;               // conv0 ring row pitch (pixel 63: a dump slot)
constexpr int SW_IC = 2 * SW_CC + 1;           // image columns (127)
constexpr int SW_NIR = 5;                      // image ring rows
constexpr int SW_NCR = 3;                      // conv0 ring rows
template <typename T, int XB>
__global__ __launch_bounds__(256, 3) void stem_walk_kernel(StemArgs a) {
  constexpr int BF = sizeof(T) == 4 ? 0 : (std::is_same<T, f16>::value ? 2 : 1);
  using M = C0Mma<BF>;
  using TI = typename std::conditional<XB != 0, uint16_t, float>::type;
  constexpr int VI = 16 / sizeof(TI);               // image elements per 16-B vector
  constexpr int NVC = (SW_IC + VI - 2 + VI - 1) / VI;  // vectors per staged image row
  constexpr int SWD = NVC * VI;                     // staged row width (floats)
  constexpr int LP4 = (4 * 3 * NVC + 255) / 256;    // loads per thread: 4 image rows
  constexpr int LP5 = (5 * 3 * NVC + 255) / 256;    // ... 5 image rows (the prologue)
  // image row r lives at slot r % 5 (slots 0, 1 also at 5, 6): the 3 rows 2 r1 .. 2 r1 + 2 of
  // conv0 row r1 are 3 consecutive slots from (2 r1) % 5, so the tap offsets are per-lane constants.
  // The ring holds conv0's A operand already converted, once per image element instead of once
  // per tap: fp32 plans the three-term bf16 split (s_ra = term 0 | term 1 << 16, s_rl = term 2),
  // 16-bit plans the rounded value (s_rl).
  constexpr int RING = (SW_NIR + 2) * 3 * SWD;
  __shared__ __attribute__((aligned(16))) uint32_t s_ra[BF == 0 ? RING : 4];  // [slot][ci][col]
  __shared__ __attribute__((aligned(16))) uint16_t s_rl[RING];
  __shared__ __attribute__((aligned(16))) float s_c0[SW_NCR * SW_CP * ST_PS];    // [row % 3][col][ch]
  // depthwise output = the pointwise B operand, already converted: fp32 plans the three bf16
  // split terms, 16-bit plans the stored value ([term][o][ch], rows padded to SW_DP halves)
  constexpr int SW_DP = ST_C1 + 8;
  __shared__ __attribute__((aligned(16))) uint16_t s_dwp[(BF == 0 ? 3 : 1) * 32 * SW_DP];
  __shared__ __attribute__((aligned(16))) float s_wd[9 * ST_C1];                // [tap][ch]
  __shared__ __attribute__((aligned(16))) float s_bn[2 * ST_C1 + 2 * ST_C2];    // scd shd scp shp

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
  const int c1o = 2 * ow0 - 1;                        // conv0 column origin (-1: dw padding)
  const int cbase = ((4 * ow0 - 2 + VI) / VI - 1) * VI;  // first staged image column (aligned)
  const int coff = 4 * ow0 - 2 - cbase;               // image column 2 c1o in the staged row
  const size_t plane = (size_t)a.H * a.W;
  const __amdgpu_buffer_rsrc_t xr =
      buf_rsrc((const TI*)a.x + (size_t)n * 3 * plane, (uint32_t)(3 * plane * sizeof(TI)));
  const size_t ysz = (size_t)a.H2 * a.W2 * a.ldy;
  const __amdgpu_buffer_rsrc_t yr = buf_rsrc((T*)a.y + (size_t)n * ysz, (uint32_t)(ysz * sizeof(T)));

  // image rows [r0, r0 + R) of all 3 channels: 16-B buffer loads into registers / into the ring
  auto load_rows = [&](int r0, int R, uint4* raw, int LP) {
#pragma unroll
    for (int k = 0; k < LP; ++k) {
      const int i = tid + 256 * k;
      const int row = i / (3 * NVC), rem = i - row * 3 * NVC;
      const int ci = rem / NVC, v = rem - ci * NVC;
      const int ir = r0 + row, ic = cbase + v * VI;
      const bool ok = row < R && ir >= 0 && ir < a.H && ic >= 0 && ic + VI <= a.W;
      const uint32_t off = ok ? (uint32_t)(((size_t)ci * a.H + ir) * a.W + ic) * sizeof(TI) : BUF_OOB;
      const buf_v4u t = __builtin_amdgcn_raw_buffer_load_b128(xr, off, 0, 0);
      raw[k] = make_uint4(t[0], t[1], t[2], t[3]);
    }
  };
  // one 16-B image vector -> conv0 A-operand ring words (see s_ra / s_rl)
  auto ring_pack = [&](const TI* e, uint32_t* wa, uint16_t* wl) {
#pragma unroll
    for (int j = 0; j < VI; ++j) {
      const float f = XB ? in16<XB>((uint16_t)e[j]) : (float)e[j];
      if constexpr (BF == 0) {  // gs_split3's terms of f
        const uint32_t u = __float_as_uint(f), b0 = u & 0xFFFF0000u;
        const float r1 = f - __uint_as_float(b0);
        const uint32_t b1 = __float_as_uint(r1) & 0xFFFF0000u;
        const float r2 = r1 - __uint_as_float(b1);
        wa[j] = (u >> 16) | b1;
        wl[j] = (uint16_t)(__float_as_uint(r2) >> 16);
      } else if constexpr (BF == 1) {
        wl[j] = f2bf(f);
      } else {
        const _Float16 hv = (_Float16)f;
        __builtin_memcpy(&wl[j], &hv, 2);
      }
    }
  };
  auto store_rows = [&](int r0, int R, const uint4* raw, int LP) {
#pragma unroll
    for (int k = 0; k < LP; ++k) {
      const int i = tid + 256 * k;
      const int row = i / (3 * NVC), rem = i - row * 3 * NVC;
      if (row >= R) continue;
      const int ci = rem / NVC, v = rem - ci * NVC;
      const int slot = (r0 + row + 4 * SW_NIR) % SW_NIR;  // (r0 >= -4)
      const TI* e = reinterpret_cast<const TI*>(&raw[k]);
      uint32_t wa[VI];
      uint16_t wl[VI];
      ring_pack(e, wa, wl);
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        if (h == 1 && slot >= 2) break;
        const int d = ((slot + h * SW_NIR) * 3 + ci) * SWD + v * VI;
        if constexpr (BF == 0) {
#pragma unroll
          for (int j = 0; j < VI; j += 4)
            *reinterpret_cast<uint4*>(&s_ra[d + j]) = make_uint4(wa[j], wa[j + 1], wa[j + 2], wa[j + 3]);
        }
#pragma unroll
        for (int j = 0; j < VI; j += 4)
          *reinterpret_cast<uint2*>(&s_rl[d + j]) =
              make_uint2(wl[j] | ((uint32_t)wl[j + 1] << 16), wl[j + 2] | ((uint32_t)wl[j + 3] << 16));
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
  // conv0 pixel groups of this wave: g = wave, wave + 4 of a row pair's 8 x 16 pixels
  // (pixel p = 63 rr + cc; p = 126, 127 are padding: they read pixel 0, store to the dump slot)
  int aoff[2], sinfo[2][4];
#pragma unroll
  for (int gi = 0; gi < 2; ++gi) {
    const int pa = 16 * (wave + 4 * gi) + li;
    const int ra = pa >= SW_CC, ca = pa < 2 * SW_CC ? pa - SW_CC * ra : 0;
    aoff[gi] = 2 * ca + coff + (ra << 24);  // bit 24: the second row of the pair
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int ps = 16 * (wave + 4 * gi) + 4 * lq + q;
      const int rs = ps >= SW_CC;
      const int cs = ps < 2 * SW_CC ? ps - SW_CC * rs : SW_CC;  // (padding: the dump slot)
      const int c1 = c1o + cs;
      const bool colok = cs < SW_CC && c1 >= 0 && c1 < a.W1;
      sinfo[gi][q] = cs * ST_PS + li + (rs << 24) + ((int)colok << 25);
    }
  }
  int koff[8];  // tap k = 8 lq + e -> (kh * 3 + ci) * SWD + kw from the row's first slot
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const int k = 8 * lq + e;
    const int kk = k < 27 ? k : 0;
    koff[e] = ((kk % 9) / 3 * 3 + kk / 9) * SWD + kk % 3;
  }
  for (int i = tid; i < 9 * ST_C1; i += 256) s_wd[i] = a.wd[(i % ST_C1) * 9 + i / ST_C1];
  if (tid < ST_C1) {
    s_bn[tid] = a.scd[tid];
    s_bn[ST_C1 + tid] = a.shd[tid];
  }
  if (tid < ST_C2) {
    s_bn[2 * ST_C1 + tid] = a.scp[tid];
    s_bn[2 * ST_C1 + ST_C2 + tid] = a.shp[tid];
  }
  // pointwise weights of this wave's column tiles, in registers (fp32: already split)
  const int nt0 = wave < 2 ? 0 : 2, ntn = wave < 2 ? 2 : 1;
  uint4 wpr[2][BF == 0 ? 3 : 1];
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int nt = u < ntn ? nt0 + u : nt0;
    if constexpr (BF == 0) {
      const float* wr = (const float*)a.wp + (16 * nt + li) * ST_C1 + 8 * lq;
      gs_split3(*reinterpret_cast<const uint4*>(wr), *reinterpret_cast<const uint4*>(wr + 4), wpr[u]);
    } else {
      wpr[u][0] = *reinterpret_cast<const uint4*>((const T*)a.wp + (16 * nt + li) * ST_C1 + 8 * lq);
    }
  }
  // the loop's 4-row loads and ring stores: per-thread tables (the row is the only variable)
  uint32_t lvo[LP4];  // byte offset in the image of the vector's row-0 position
  int lds[LP4];       // ring offset within a slot | row << 24 | (row < 4 && columns in) << 28
#pragma unroll
  for (int k = 0; k < LP4; ++k) {
    const int i = tid + 256 * k;
    const int row = i / (3 * NVC), rem = i - row * 3 * NVC;
    const int ci = rem / NVC, v = rem - ci * NVC;
    const int ic = cbase + v * VI;
    const bool ok = row < 4 && ic >= 0 && ic + VI <= a.W;
    lvo[k] = ok ? (uint32_t)((ci * a.H + row) * a.W + ic) * (uint32_t)sizeof(TI) : 0u;
    lds[k] = (ci * SWD + v * VI) | ((row < 4 ? row : 7) << 24) | ((int)ok << 28);
  }
  const int rowbytes = a.W * (int)sizeof(TI);
  auto load4 = [&](int r0, uint4* raw) {
#pragma unroll
    for (int k = 0; k < LP4; ++k) {
      const int ir = r0 + ((lds[k] >> 24) & 7);
      const bool ok = ((lds[k] >> 28) & 1) && ir >= 0 && ir < a.H;
      const uint32_t off = ok ? lvo[k] + (uint32_t)(r0 * rowbytes) : BUF_OOB;
      const buf_v4u t = __builtin_amdgcn_raw_buffer_load_b128(xr, off, 0, 0);
      raw[k] = make_uint4(t[0], t[1], t[2], t[3]);
    }
  };
  auto store4 = [&](int r0, const uint4* raw) {
    const int r0m = (r0 + 4 * SW_NIR) % SW_NIR;  // (r0 >= -4)
#pragma unroll
    for (int k = 0; k < LP4; ++k) {
      const int row = (lds[k] >> 24) & 7;
      if (row >= 4) continue;
      int slot = r0m + row;
      slot -= slot >= SW_NIR ? SW_NIR : 0;
      const TI* e = reinterpret_cast<const TI*>(&raw[k]);
      uint32_t wa[VI];
      uint16_t wl[VI];
      ring_pack(e, wa, wl);
      const int d0 = slot * 3 * SWD + (lds[k] & 0xFFFFFF);
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        if (h == 1 && slot >= 2) break;
        const int d = d0 + h * SW_NIR * 3 * SWD;
        if constexpr (BF == 0) {
#pragma unroll
          for (int j = 0; j < VI; j += 4)
            *reinterpret_cast<uint4*>(&s_ra[d + j]) = make_uint4(wa[j], wa[j + 1], wa[j + 2], wa[j + 3]);
        }
#pragma unroll
        for (int j = 0; j < VI; j += 4)
          *reinterpret_cast<uint2*>(&s_rl[d + j]) =
              make_uint2(wl[j] | ((uint32_t)wl[j + 1] << 16), wl[j + 2] | ((uint32_t)wl[j + 3] << 16));
      }
    }
  };
  // every conv0 column of the strip inside the map: no zero padding to select
  const bool cols_in = c1o >= 0 && c1o + SW_CC - 1 < a.W1;
  // conv0 rows r0, r0 + 1 (image rows 2 r0 .. 2 r0 + 4 in the ring) -> conv0 ring
  auto conv0_pair = [&](int r0) {
    const int ib0 = ((2 * r0 + 8 * SW_NIR) % SW_NIR) * 3 * SWD;   // (r0 >= -2)
    const int ib1 = ((2 * r0 + 2 + 8 * SW_NIR) % SW_NIR) * 3 * SWD;
    const int cb0 = ((r0 + 3 * SW_NCR) % SW_NCR) * SW_CP * ST_PS;
    const int cb1 = ((r0 + 1 + 3 * SW_NCR) % SW_NCR) * SW_CP * ST_PS;
    const bool rok0 = r0 >= 0 && r0 < a.H1, rok1 = r0 + 1 >= 0 && r0 + 1 < a.H1;
    f32x4 c0v[2][2];
#pragma unroll
    for (int gi = 0; gi < 2; ++gi) {
      const int base = (aoff[gi] & 0xFFFFFF) + ((aoff[gi] >> 24) ? ib1 : ib0);
      typename M::Frag af;
      {
        uint32_t l2[4];
#pragma unroll
        for (int e = 0; e < 8; e += 2) {
          const uint32_t l0 = 8 * lq + e < 27 ? s_rl[base + koff[e]] : 0u;
          const uint32_t l1 = 8 * lq + e + 1 < 27 ? s_rl[base + koff[e + 1]] : 0u;
          l2[e / 2] = l0 | (l1 << 16);
        }
        if constexpr (BF == 0) {
          uint32_t a2[8];
#pragma unroll
          for (int e = 0; e < 8; ++e) a2[e] = 8 * lq + e < 27 ? s_ra[base + koff[e]] : 0u;
          af.t[0] = make_uint4(__builtin_amdgcn_perm(a2[1], a2[0], 0x05040100u),
                               __builtin_amdgcn_perm(a2[3], a2[2], 0x05040100u),
                               __builtin_amdgcn_perm(a2[5], a2[4], 0x05040100u),
                               __builtin_amdgcn_perm(a2[7], a2[6], 0x05040100u));
          af.t[1] = make_uint4(__builtin_amdgcn_perm(a2[1], a2[0], 0x07060302u),
                               __builtin_amdgcn_perm(a2[3], a2[2], 0x07060302u),
                               __builtin_amdgcn_perm(a2[5], a2[4], 0x07060302u),
                               __builtin_amdgcn_perm(a2[7], a2[6], 0x07060302u));
          af.t[2] = make_uint4(l2[0], l2[1], l2[2], l2[3]);
        } else {
          __builtin_memcpy(&af, l2, 16);
        }
      }
#pragma unroll
      for (int jt = 0; jt < 2; ++jt) {
        f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
        M::mma(af, bw[jt], acc);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float v = acc[q] * fsc[jt] + fsh[jt];
          acc[q] = round_as<T>(fmaxf(v, 0.f));
        }
        c0v[gi][jt] = acc;
      }
    }
    if (cols_in && rok0 && rok1) {  // (workgroup-uniform: no padding in these two rows)
#pragma unroll
      for (int gi = 0; gi < 2; ++gi) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int si = sinfo[gi][q];
          float* d = s_c0 + (si & 0xFFFFFF) + (((si >> 24) & 1) ? cb1 : cb0);
          d[0] = c0v[gi][0][q];
          d[16] = c0v[gi][1][q];
        }
      }
    } else {
#pragma unroll
      for (int gi = 0; gi < 2; ++gi) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int si = sinfo[gi][q];
          const bool r1 = (si >> 24) & 1;
          const bool in = ((si >> 25) & 1) && (r1 ? rok1 : rok0);
          float* d = s_c0 + (si & 0xFFFFFF) + (r1 ? cb1 : cb0);
          d[0] = in ? c0v[gi][0][q] : 0.f;
          d[16] = in ? c0v[gi][1][q] : 0.f;
        }
      }
    }
  };

  // ---- prologue: conv0 rows 2 oh0 - 2 (a don't-care: its ring row is rewritten before it is
  // read) and 2 oh0 - 1 from image rows 4 oh0 - 4 .. 4 oh0, then image rows 4 oh0 + 1 .. 4 oh0 + 4.
  // Step s stores the next step's 4 image rows once its own conv0 is done and loads the rows of
  // the step after: two barriers per step, a whole step for the loads to land ----------------
  uint4 nxt[LP4];  // image rows of a coming step, in flight
  {
    uint4 raw[LP5];
    load_rows(4 * oh0 - 4, 5, raw, LP5);
    load_rows(4 * oh0 + 1, 4, nxt, LP4);
    store_rows(4 * oh0 - 4, 5, raw, LP5);
  }
  __syncthreads();
  conv0_pair(2 * oh0 - 2);
  __syncthreads();
  store4(4 * oh0 + 1, nxt);
  load4(4 * oh0 + 5, nxt);
  {  // two dropped stores: the loop is entered, as it loops, with 2 stores after the row loads,
     // so the wait for the rows can leave the stores in flight (vmcnt counts in issue order)
    const float z[4] = {0.f, 0.f, 0.f, 0.f};
    buf_st4(yr, BUF_OOB, z, (T*)nullptr);
    buf_st4(yr, BUF_OOB + 64, z, (T*)nullptr);  // (another address: not merged with the first)
  }
  __syncthreads();
  stamp(a.stamps, 1);

  // per-thread depthwise / pointwise constants
  const int qd = tid & 7, o = tid >> 3;         // depthwise: channel quad, output column
  const int pg = wave & 1;                      // pointwise: pixel group (outputs 16 pg ..)
  for (int s = 0; s < SW_RS; ++s) {
    const int oh = oh0 + s;
    if (oh >= a.H2) break;  // (workgroup-uniform)
    conv0_pair(2 * oh);
    __syncthreads();
    if (s == SW_RS / 2) stamp(a.stamps, 2);  // (stamps 2-4: the middle step's phases)
    store4(4 * oh + 5, nxt);  // (slots of rows 4 oh .. 4 oh + 3: conv0 is done)
    load4(4 * oh + 9, nxt);   // (also near the end: a fixed count per step)
    // ---- dsconv1.dw of output row oh: conv0 rows 2 oh - 1 .. 2 oh + 1 (taps in row-major order)
    // (o = 31 is padding: its reads stay inside LDS, its pointwise output is not stored)
    {
      float acc[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kh = 0; kh < 3; ++kh) {
        const float* rowp = s_c0 + ((2 * oh - 1 + kh + 3 * SW_NCR) % SW_NCR) * SW_CP * ST_PS;
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
      const float4 sc = *reinterpret_cast<const float4*>(&s_bn[4 * qd]);
      const float4 sh = *reinterpret_cast<const float4*>(&s_bn[ST_C1 + 4 * qd]);
      const float scv[4] = {sc.x, sc.y, sc.z, sc.w}, shv[4] = {sh.x, sh.y, sh.z, sh.w};
      float o4[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float t = acc[j] * scv[j] + shv[j];
        o4[j] = round_as<T>(fmaxf(t, 0.f));
      }
      uint16_t* d = s_dwp + o * SW_DP + 4 * qd;
      if constexpr (BF == 0) {  // gs_split3's terms, one plane each
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
        *reinterpret_cast<uint2*>(d + 32 * SW_DP) = make_uint2((p1[0] >> 16) | p1[1], (p1[2] >> 16) | p1[3]);
        *reinterpret_cast<uint2*>(d + 64 * SW_DP) = make_uint2((p2[0] >> 16) | p2[1], (p2[2] >> 16) | p2[3]);
      } else {
        *reinterpret_cast<uint2*>(d) =
            make_uint2((uint32_t)s16_from<T>(o4[0]) | ((uint32_t)s16_from<T>(o4[1]) << 16),
                       (uint32_t)s16_from<T>(o4[2]) | ((uint32_t)s16_from<T>(o4[3]) << 16));
      }
    }
    __syncthreads();
    if (s == SW_RS / 2) stamp(a.stamps, 3);
    // ---- dsconv1.pw: pixel group pg x column tiles {0, 1} (waves 0, 1) or {2} (waves 2, 3) ---
    {
      const int op = 16 * pg + li;
      const uint16_t* xp = s_dwp + op * SW_DP + 8 * lq;
      f32x4 acc[2];
      if constexpr (sizeof(T) == 4) {
        uint4 xs[3];
#pragma unroll
        for (int j = 0; j < 3; ++j) xs[j] = *reinterpret_cast<const uint4*>(xp + 32 * SW_DP * j);
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          acc[u] = f32x4{0.f, 0.f, 0.f, 0.f};
          if (u < ntn) gs_mma_x3(wpr[u], xs, acc[u]);
        }
      } else {
        const uint4 xb = *reinterpret_cast<const uint4*>(xp);
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          acc[u] = f32x4{0.f, 0.f, 0.f, 0.f};
          if (u < ntn) StPw<T>::run(wpr[u][0], xb, acc[u]);
        }
      }
      const int ow = ow0 + op;
      const uint32_t yoff = op < SW_TW && ow < a.W2
                                ? (uint32_t)(((size_t)oh * a.W2 + ow) * a.ldy) * sizeof(T)
                                : BUF_OOB;
#pragma unroll
      for (int u = 0; u < 2; ++u) {  // (u >= ntn: a dropped store, so every step issues two)
        const int c = u < ntn ? 16 * (nt0 + u) + 4 * lq : 0;
        const float4 sc = *reinterpret_cast<const float4*>(&s_bn[2 * ST_C1 + c]);
        const float4 sh = *reinterpret_cast<const float4*>(&s_bn[2 * ST_C1 + ST_C2 + c]);
        const float scv[4] = {sc.x, sc.y, sc.z, sc.w}, shv[4] = {sh.x, sh.y, sh.z, sh.w};
        float o4[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float v = acc[u][r] * scv[r] + shv[r];
          o4[r] = fmaxf(v, 0.f);
        }
        buf_st4(yr, yoff == BUF_OOB || u >= ntn ? BUF_OOB : yoff + c * (uint32_t)sizeof(T), o4,
               (T*)nullptr);
      }
    }
    if (s == SW_RS / 2) stamp(a.stamps, 4);
  }
  stamp(a.stamps, 5);
}

bool stem_ok(const StemArgs& a) {
  const int VI = a.x_dtype ? 8 : 4;
  const int ve = VI == 8 ? 4 : (a.ldy % 4 == 0 ? 4 : 0);  // 4-channel output vectors aligned
  return a.N > 0 && a.H >= 3 && a.W >= 3 && a.W % VI == 0 && ((uintptr_t)a.x & 15) == 0 &&
         ((uintptr_t)a.y & 15) == 0 && ((uintptr_t)a.wp & 15) == 0 &&
         ve == 4 && a.ldy >= ST_C2 && a.ldy % 4 == 0 &&
         a.H1 == (a.H - 3) / 2 + 1 && a.W1 == (a.W - 3) / 2 + 1 && a.H2 == (a.H1 - 1) / 2 + 1 &&
         a.W2 == (a.W1 - 1) / 2 + 1 && a.N < 65536 && cdiv(a.H2, SW_RS) < 65536 &&
         // per-image buffer ranges below BUF_OOB (32-bit buffer offsets)
         3LL * a.H * a.W * (a.x_dtype ? 2 : 4) < (long long)BUF_OOB &&
         4LL * a.H2 * a.W2 * a.ldy < (long long)BUF_OOB;
}

int stem_fwd(const StemArgs& a, int dtype, hipStream_t st) {
  if (!stem_ok(a)) {
    set_error("stem_fwd: unsupported shape N=%d H=%d W=%d (W %% %d, 16-B aligned image)", a.N,
              a.H, a.W, a.x_dtype ? 8 : 4);
    return E_UNSUPPORTED;
  }
  StemArgs as = a;
  as.stamps = stamp_region();
  const dim3 gw(cdiv(a.W2, SW_TW), cdiv(a.H2, SW_RS), a.N);
  ProfScope pw_(PK_STEM, st, (a.x_dtype ? 2.0 : 4.0) * a.N * 3.0 * a.H * a.W +
                                 (dtype == DT_F32 ? 4.0 : 2.0) * (double)a.N * a.H2 * a.W2 * ST_C2,
                // conv0 (27 -> 32), the depthwise 3 x 3 (32) and the pointwise 32 -> 48
                2.0 * a.N * (27.0 * 32 * a.H1 * a.W1 + (9.0 * 32 + 32.0 * ST_C2) * a.H2 * a.W2));
#define STEMW(T)                                                            \
  do {                                                                      \
    if (a.x_dtype == 2) prof_launch(stem_walk_kernel<T, 2>, gw, 256, 0, st, as);      \
    else if (a.x_dtype == 1) prof_launch(stem_walk_kernel<T, 1>, gw, 256, 0, st, as); \
    else prof_launch(stem_walk_kernel<T, 0>, gw, 256, 0, st, as);                     \
  } while (0)
  if (dtype == DT_F32) STEMW(float);
  else if (dtype == DT_F16) STEMW(f16);
  else STEMW(bf16);
#undef STEMW
  return check_launch("stem_fwd");
}

}  // namespace fscnn
