// Fused inverted-residual block, inference (models/fast_scnn.py:95-115 LinearBottleneck with
// stride 1):  y = BN_p(W_p * relu(BN_d(dw3x3(relu(BN_e(W_e * x)))))) (+ x when Cin == Cout)
// with every BatchNorm folded into a per-channel (scale, shift) (eval).
//
// The unfused path writes the 6x-expanded tensor twice and reads it twice (expand output, dw
// input, dw output, project input: 4 x 50 MB fp32 per bottleneck3 block at cfg2) and pays three
// launches of a latency-bound 16 K-row problem.  Here one workgroup owns an 8 x 8 output tile:
//   * the haloed 10 x 10 input tile (100 pixels, padded to 7 MFMA row tiles of 16) is staged in
//     LDS once;
//   * the expanded channels are produced 64 at a time: expand GEMM (MFMA, weights as the A
//     operand so each lane holds 4 consecutive channels of one pixel) + BN + ReLU into an LDS
//     chunk (halo pixels outside the image are zero: the depthwise's padding applies to ITS
//     input), the depthwise 3x3 + BN + ReLU from that chunk into a second LDS chunk, and the
//     project GEMM accumulates the chunk's contribution in registers;
//   * the project epilogue applies its BN and the residual and stores NHWC vectors.
// Only the block input (read once, + halo from L2) and output touch HBM.
//
// Arithmetic: 16-bit plans (bf16 / fp16) use one v_mfma_f32_16x16x32_{bf16,f16} per operand pair;
// fp32 plans keep every MFMA operand as three bf16 planes (the exact truncation split of
// common.hpp gs_split3, applied per element) and run six bf16 MFMAs per product (gs_mma_x3), the
// dropped terms being below fp32's own product rounding.  Intermediate values are rounded to the
// plan's storage type exactly where the unfused path stores them (expand output, dw output).
#include "kernels.hpp"

namespace fscnn {

// Tiles per stride: stride 1 = an 8 x 8 output tile over a 10 x 10 haloed input tile; stride 2
// (bottleneck1.0 / 2.0) = a 4 x 8 output tile over a 9 x 17 input tile, whose fp32 split planes
// and expand chunk still fit LDS (an 8 x 8 stride-2 tile would need 17 x 17 input pixels).
template <int S>
struct IrTile {
  static constexpr int TH = S == 1 ? 8 : 4, TW = 8;          // output tile
  static constexpr int HH = S * (TH - 1) + 3, HW = S * (TW - 1) + 3;  // haloed input tile
  static constexpr int HALO = HH * HW;                         // 100 / 153 pixels
  static constexpr int RT = (HALO + 15) / 16;                  // 7 / 10 MFMA row tiles
  static constexpr int ROWS = RT * 16;                         // 112 / 160
  static constexpr int PX = TH * TW;                           // 64 / 32 output pixels
  static constexpr int XROWS = HALO + 1;  // staged input rows: the halo + a zero row that the
                                          // MFMA rows past it read
  static constexpr int RPW = (RT + 1) / 2;                     // expand row tiles per wave
  static constexpr int NPT = S == 1 ? 2 : 1;                   // depthwise pixels per thread
  static constexpr int PT = PX / 16;                           // project pixel tiles
};
constexpr int IR_EC = 64;                          // expanded channels per chunk
constexpr int IR_ELD = IR_EC + 4;                  // fp32 row stride of the expand chunk
// Operand rows are padded by 16 uint16 (8 dwords): with row strides of 40, 56 or 72 dwords
// (Cin 64 / 96 / 128, and the 64-channel depthwise chunk) the 16 lanes of every ds_read_b128
// lane group ({li 0-3, 12-15 of one k-half, li 4-11 of the next}) hit 16 distinct 4-bank slots.

// per-element truncation split of an fp32 value into three bf16 terms (see gs_split3)
__device__ __forceinline__ void ir_split(float f, uint16_t& b0, uint16_t& b1, uint16_t& b2) {
  const uint32_t u = __float_as_uint(f);
  const uint32_t h0 = u & 0xFFFF0000u;
  const float r1 = f - __uint_as_float(h0);
  const uint32_t h1 = __float_as_uint(r1) & 0xFFFF0000u;
  const float r2 = r1 - __uint_as_float(h1);
  b0 = (uint16_t)(h0 >> 16);
  b1 = (uint16_t)(h1 >> 16);
  b2 = (uint16_t)(__float_as_uint(r2) >> 16);
}

// operand planes: 1 (16-bit storage) or 3 (fp32 as three bf16 terms)
template <typename T>
struct IrP {
  static constexpr int P = sizeof(T) == 4 ? 3 : 1;
};

// 8 consecutive k of a weight row -> P operand planes (16 B each)
template <typename T>
__device__ __forceinline__ void ir_ldw(const T* p, bool ok, uint4 (&w)[IrP<T>::P]) {
  if constexpr (sizeof(T) == 4) {
    const float* f = reinterpret_cast<const float*>(p);
    const uint4 lo = ok ? *reinterpret_cast<const uint4*>(f) : make_uint4(0u, 0u, 0u, 0u);
    const uint4 hi = ok ? *reinterpret_cast<const uint4*>(f + 4) : make_uint4(0u, 0u, 0u, 0u);
    gs_split3(lo, hi, w);
  } else {
    w[0] = ok ? *reinterpret_cast<const uint4*>(p) : make_uint4(0u, 0u, 0u, 0u);
  }
}

template <typename T>
__device__ __forceinline__ void ir_mma(const uint4 (&a)[IrP<T>::P], const uint4 (&b)[IrP<T>::P],
                                       f32x4& acc) {
  if constexpr (sizeof(T) == 4) {
    gs_mma_x3(a, b, acc);
  } else if constexpr (std::is_same<T, f16>::value) {
    h16x8 av, bv;
    __builtin_memcpy(&av, &a[0], 16);
    __builtin_memcpy(&bv, &b[0], 16);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(av, bv, acc, 0, 0, 0);
  } else {
    i16x8 av, bv;
    __builtin_memcpy(&av, &a[0], 16);
    __builtin_memcpy(&bv, &b[0], 16);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, bv, acc, 0, 0, 0);
  }
}

constexpr int IR_PRM = IR_EC * 9 + 4 * IR_EC;  // per-chunk depthwise weights + BN_e / BN_d tables

// LDS bytes of one launch (KS = Cin / 32)
template <typename T, int S>
__host__ __device__ constexpr size_t ir_lds(int KS) {
  using G = IrTile<S>;
  return (size_t)IrP<T>::P * G::XROWS * (32 * KS + 16) * 2  // input tile planes
         + (size_t)G::ROWS * IR_ELD * 4                       // expand chunk (fp32)
         + (size_t)IrP<T>::P * G::PX * (IR_EC + 16) * 2       // depthwise chunk planes
         + G::ROWS * 4                                        // halo validity
         + (size_t)2 * IR_PRM * 4;                            // chunk parameters, double-buffered
}

// 512 threads = 8 waves (2 per SIMD: one workgroup fills a CU when the fp32 tiles need ~150 KB).
//   expand: wave w owns expanded-channel tile (w & 3) of the chunk and halo row tiles
//           4 (w >> 2) .. +3, all accumulators live (independent MFMA chains);
//   depthwise: thread = 4 channels x 2 output pixels, weights / BN tables from LDS;
//   project: wave w owns one 16-channel output tile and PPW pixel tiles.
// Software pipeline over chunks: the NEXT chunk's weights (expand / project rows of this wave in
// registers, the depthwise weights and BN tables via the other LDS parameter buffer) are loaded
// while the current chunk computes, so the L2 / HBM latency of the weight reads is paid once.
constexpr int IR_THREADS = 512;
constexpr int IR_WAVES = IR_THREADS / 64;

// KS: Cin / 32 (2, 3, 4); PPW: project pixel tiles per wave (4 when Cout > 64, else 2);
// PRE (fp32): the weights come pre-split (a.we3 / a.wp3), no per-chunk split arithmetic
template <typename T, int KS, int PPW, bool PRE = false, int S = 1>
__global__ __launch_bounds__(IR_THREADS) void ir_block_kernel(IrArgs a) {
  using G = IrTile<S>;
  constexpr int IR_TH = G::TH, IR_TW = G::TW, IR_HW = G::HW, IR_HALO = G::HALO, IR_RT = G::RT;
  constexpr int IR_ROWS = G::ROWS, IR_PX = G::PX, IR_XROWS = G::XROWS, NPT = G::NPT;
  constexpr int P = IrP<T>::P;
  constexpr int R = sizeof(T) == 4 ? (PRE ? 3 : 2) : 1;  // raw 16-B vectors per 8 weights
  constexpr int CIN = 32 * KS;
  constexpr int XLD = CIN + 16;      // uint16 per input-tile row (conflict-free operand reads)
  constexpr int DLD = IR_EC + 16;    // uint16 per depthwise-chunk row
  constexpr int RPW = G::RPW;        // expand row tiles per wave (stride 1: the last half holds 3)
  extern __shared__ __attribute__((aligned(16))) unsigned char s_dyn[];
  uint16_t* sX = reinterpret_cast<uint16_t*>(s_dyn);                   // [P][101][XLD]
  float* sE = reinterpret_cast<float*>(sX + (size_t)P * IR_XROWS * XLD);  // [112][IR_ELD]
  uint16_t* sD = reinterpret_cast<uint16_t*>(sE + IR_ROWS * IR_ELD);     // [P][64][DLD]
  float* sV = reinterpret_cast<float*>(sD + (size_t)P * IR_PX * DLD);    // [112] 1 = in image
  float* sPrm = sV + IR_ROWS;  // [2][IR_PRM]: wd [64][9], sc_e, sh_e, sc_d, sh_d [64]

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform (scalar branches)
  const int li = lane & 15, lq = lane >> 4;
  const int tiles_x = cdiv(a.W, IR_TW), tiles_y = cdiv(a.H, IR_TH);
  int t = blockIdx.x;
  const int n = t / (tiles_x * tiles_y);
  t -= n * tiles_x * tiles_y;
  const int y0 = (t / tiles_x) * IR_TH, x0 = (t % tiles_x) * IR_TW;
  const T* X = (const T*)a.x;
  const T* We = (const T*)a.we;
  const T* Wp = (const T*)a.wp;
  const int otiles = a.Cout / 16;
  const int ect = wave & 3, erh = (wave >> 2) * RPW;  // expand: channel tile, first row tile
  const int dq = tid & 15, dg = tid >> 4;              // depthwise: channel quad, pixel pair
  const int doy = dg / (IR_TW / NPT), dox = (dg % (IR_TW / NPT)) * NPT;
  // project: output tile, first pixel tile (all G::PT pixel tiles per wave, or half of them)
  const int pot = PPW == G::PT ? wave : (wave & 3);
  const int ppt = PPW == G::PT ? 0 : PPW * (wave >> 2);
  const bool pon = pot < otiles;

  // ---- per-chunk loads (issued one chunk ahead) ----------------------------------------------
  uint4 rwe[KS][R], rwp[2][R];  // raw expand / project weight vectors of this lane
  float rprm[2];                // this thread's share of the chunk parameter table
  auto fetch_we = [&](int e0) {
    const int erow = e0 + ect * 16 + li;
#pragma unroll
    for (int s = 0; s < KS; ++s)
#pragma unroll
      for (int h = 0; h < R; ++h) {
        if constexpr (PRE)
          rwe[s][h] = *reinterpret_cast<const uint4*>(
              a.we3 + ((size_t)h * a.E + erow) * CIN + 32 * s + 8 * lq);
        else
          rwe[s][h] = *reinterpret_cast<const uint4*>(We + (size_t)erow * CIN + 32 * s + 8 * lq +
                                                      h * 4);
      }
  };
  auto fetch_wp = [&](int e0) {
    const int orow = (pon ? pot : 0) * 16 + li;
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int h = 0; h < R; ++h) {
        if constexpr (PRE)
          rwp[s][h] = *reinterpret_cast<const uint4*>(
              a.wp3 + ((size_t)h * a.Cout + orow) * a.E + e0 + 32 * s + 8 * lq);
        else
          rwp[s][h] = *reinterpret_cast<const uint4*>(Wp + (size_t)orow * a.E + e0 + 32 * s +
                                                      8 * lq + h * 4);
      }
  };
  // parameter entries tid and tid + 512 of the chunk table: entry i < 576 is wd[e0 * 9 + i], the
  // rest BN_e / BN_d (scale, shift) of channel e0 + (i - 576) % 64 -> per-thread base pointers
  const float* psrc[2];
  int pmul[2];
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int i = tid + u * IR_THREADS;
    if (i < IR_EC * 9) {
      psrc[u] = a.wd + i;
      pmul[u] = 9;
    } else {
      const int j = min(i, IR_PRM - 1) - IR_EC * 9, tab = j / IR_EC, c = j - tab * IR_EC;
      const float* src = tab == 0 ? a.sc_e : (tab == 1 ? a.sh_e : (tab == 2 ? a.sc_d : a.sh_d));
      psrc[u] = src + c;
      pmul[u] = 1;
    }
  }
  auto fetch_prm = [&](int e0) {
#pragma unroll
    for (int u = 0; u < 2; ++u) rprm[u] = psrc[u][(size_t)e0 * pmul[u]];
  };
  auto put_prm = [&](int buf) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int i = tid + u * IR_THREADS;
      if (i < IR_PRM) sPrm[buf * IR_PRM + i] = rprm[u];
    }
  };
  auto operand = [&](const uint4 (&raw)[R], uint4 (&op)[P]) {
    if constexpr (P == 3 && !PRE) {
      gs_split3(raw[0], raw[1], op);
    } else {
#pragma unroll
      for (int p = 0; p < P; ++p) op[p] = raw[p];
    }
  };

  fetch_we(0);
  fetch_prm(0);
  put_prm(0);
  // ---- stage the haloed input tile (zero outside the image / past the 100 halo pixels) -------
  {
    constexpr int VPR = CIN / 8;  // 8-element groups per row
    for (int i = tid; i < IR_XROWS * VPR; i += IR_THREADS) {
      const int r = i / VPR, v = i - r * VPR;
      const int hy = r / IR_HW, hx = r - hy * IR_HW;
      const int gy = S * y0 - 1 + hy, gx = S * x0 - 1 + hx;
      const bool ok = r < IR_HALO && gy >= 0 && gy < a.Hi && gx >= 0 && gx < a.Wi;
      const size_t off = ok ? (((size_t)n * a.Hi + gy) * a.Wi + gx) * a.ldx + v * 8 : 0;
      if constexpr (P == 3) {
        uint4 lo = *reinterpret_cast<const uint4*>((const float*)X + off);
        uint4 hi = *reinterpret_cast<const uint4*>((const float*)X + off + 4);
        lo = sel4(ok, lo);
        hi = sel4(ok, hi);
        uint4 sp[3];
        gs_split3(lo, hi, sp);
#pragma unroll
        for (int p = 0; p < 3; ++p)
          *reinterpret_cast<uint4*>(sX + ((size_t)p * IR_XROWS + r) * XLD + v * 8) = sp[p];
      } else {
        const uint4 q = sel4(ok, *reinterpret_cast<const uint4*>(X + off));
        *reinterpret_cast<uint4*>(sX + (size_t)r * XLD + v * 8) = q;
      }
      if (v == 0) sV[r] = ok ? 1.f : 0.f;
    }
    for (int r = IR_XROWS + tid; r < IR_ROWS; r += IR_THREADS) sV[r] = 0.f;
  }

  f32x4 accp[PPW];
#pragma unroll
  for (int j = 0; j < PPW; ++j) accp[j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nchunks = a.E / IR_EC;
  for (int ch = 0; ch < nchunks; ++ch) {
    const int e0 = ch * IR_EC;
    const float* prm = sPrm + (ch & 1) * IR_PRM;
    uint4 we[KS][P];
#pragma unroll
    for (int s = 0; s < KS; ++s) operand(rwe[s], we[s]);
    fetch_wp(e0);  // in flight during the expand and the depthwise
    if (ch + 1 < nchunks) fetch_prm(e0 + IR_EC);
    __syncthreads();  // input tile + this chunk's parameters staged; sE free
    // ---- expand: E[px][16 ect + ..] for this wave's halo row tiles --------------------------
    {
      f32x4 acc[RPW];
#pragma unroll
      for (int j = 0; j < RPW; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < KS; ++s)
#pragma unroll
        for (int j = 0; j < RPW; ++j) {
          const int rt = min(erh + j, IR_RT - 1);  // (stride 1: waves 4-7 compute tile 6 twice)
          const int row = min(rt * 16 + li, IR_HALO);  // rows past the halo: the zero row
          uint4 b[P];
#pragma unroll
          for (int p = 0; p < P; ++p)
            b[p] = *reinterpret_cast<const uint4*>(sX + ((size_t)p * IR_XROWS + row) * XLD +
                                                   32 * s + 8 * lq);
          ir_mma<T>(we[s], b, acc[j]);
        }
      const int c = ect * 16 + 4 * lq;
      const float4 sc = *reinterpret_cast<const float4*>(prm + IR_EC * 9 + c);
      const float4 sh = *reinterpret_cast<const float4*>(prm + IR_EC * 9 + IR_EC + c);
#pragma unroll
      for (int j = 0; j < RPW; ++j) {
        const int rt = min(erh + j, IR_RT - 1);  // rows >= 100: never read by the depthwise
        const int px = rt * 16 + li;
        const float valid = sV[px];
        float4 o;
        o.x = valid * round_as<T>(fmaxf(fmaf(acc[j][0], sc.x, sh.x), 0.f));
        o.y = valid * round_as<T>(fmaxf(fmaf(acc[j][1], sc.y, sh.y), 0.f));
        o.z = valid * round_as<T>(fmaxf(fmaf(acc[j][2], sc.z, sh.z), 0.f));
        o.w = valid * round_as<T>(fmaxf(fmaf(acc[j][3], sc.w, sh.w), 0.f));
        *reinterpret_cast<float4*>(sE + (size_t)px * IR_ELD + c) = o;
      }
    }
    __syncthreads();
    // ---- depthwise 3x3 + BN + ReLU of the chunk -> sD (operand planes) ----------------------
    {
      float w[4][9];
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int k = 0; k < 9; ++k) w[j][k] = prm[(4 * dq + j) * 9 + k];
      constexpr int NC = S * (NPT - 1) + 3;  // input columns of the thread's window
      float4 v[3][NC];
#pragma unroll
      for (int kh = 0; kh < 3; ++kh)
#pragma unroll
        for (int c = 0; c < NC; ++c)
          v[kh][c] = *reinterpret_cast<const float4*>(
              sE + (size_t)((S * doy + kh) * IR_HW + S * dox + c) * IR_ELD + 4 * dq);
      float acc[NPT][4];
#pragma unroll
      for (int i = 0; i < NPT; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = 0.f;
#pragma unroll
      for (int kh = 0; kh < 3; ++kh)
#pragma unroll
        for (int kw = 0; kw < 3; ++kw)
#pragma unroll
          for (int i = 0; i < NPT; ++i) {
            const float4 q = v[kh][S * i + kw];
            const float qq[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[i][j] = fmaf(qq[j], w[j][kh * 3 + kw], acc[i][j]);
          }
      const float4 sc4 = *reinterpret_cast<const float4*>(prm + IR_EC * 11 + 4 * dq);
      const float4 sh4 = *reinterpret_cast<const float4*>(prm + IR_EC * 12 + 4 * dq);
      const float sc[4] = {sc4.x, sc4.y, sc4.z, sc4.w}, sh[4] = {sh4.x, sh4.y, sh4.z, sh4.w};
#pragma unroll
      for (int i = 0; i < NPT; ++i) {
        const int p = doy * IR_TW + dox + i;
        uint16_t h[3][4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float o = fmaxf(fmaf(acc[i][j], sc[j], sh[j]), 0.f);
          if constexpr (P == 3) ir_split(o, h[0][j], h[1][j], h[2][j]);
          else h[0][j] = s16_from<T>(o);
        }
#pragma unroll
        for (int pl = 0; pl < P; ++pl) {
          const uint2 u = make_uint2((uint32_t)h[pl][0] | ((uint32_t)h[pl][1] << 16),
                                     (uint32_t)h[pl][2] | ((uint32_t)h[pl][3] << 16));
          *reinterpret_cast<uint2*>(sD + ((size_t)pl * IR_PX + p) * DLD + 4 * dq) = u;
        }
      }
    }
    // the next chunk's parameters into the other buffer (last read during the previous chunk,
    // whose readers have all passed this chunk's barriers)
    if (ch + 1 < nchunks) put_prm((ch + 1) & 1);
    __syncthreads();
    // ---- project: accumulate W_p[16 pot .., e0 .. e0 + 64) * D ---------------------------------
    uint4 wp[2][P];
#pragma unroll
    for (int s = 0; s < 2; ++s) operand(rwp[s], wp[s]);
    if (ch + 1 < nchunks) fetch_we(e0 + IR_EC);  // in flight during the project
    if (pon) {
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int j = 0; j < PPW; ++j) {
          const int pt = ppt + j;
          uint4 b[P];
#pragma unroll
          for (int p = 0; p < P; ++p)
            b[p] = *reinterpret_cast<const uint4*>(sD + ((size_t)p * IR_PX + pt * 16 + li) * DLD +
                                                   32 * s + 8 * lq);
          ir_mma<T>(wp[s], b, accp[j]);
        }
    }
  }
  // ---- epilogue: BN_p (+ residual) -> NHWC ------------------------------------------------
  if (!pon) return;
  T* Y = (T*)a.y;
  const int c = pot * 16 + 4 * lq;
  const float4 sc = *reinterpret_cast<const float4*>(a.sc_p + c);
  const float4 sh = *reinterpret_cast<const float4*>(a.sh_p + c);
#pragma unroll
  for (int j = 0; j < PPW; ++j) {
    const int px = (ppt + j) * 16 + li;
    const int gy = y0 + px / IR_TW, gx = x0 + px % IR_TW;
    if (gy >= a.H || gx >= a.W) continue;
    const size_t pix = ((size_t)n * a.H + gy) * a.W + gx;
    float rv[4] = {0.f, 0.f, 0.f, 0.f};
    if (a.residual) ld4v(X + pix * a.ldx + c, rv);
    float v[4];
    v[0] = fmaf(accp[j][0], sc.x, sh.x) + rv[0];
    v[1] = fmaf(accp[j][1], sc.y, sh.y) + rv[1];
    v[2] = fmaf(accp[j][2], sc.z, sh.z) + rv[2];
    v[3] = fmaf(accp[j][3], sc.w, sh.w) + rv[3];
    st4v(Y + pix * a.ldy + c, v);
  }
}

bool ir_block_ok(const IrArgs& a0, int dtype) {
  IrArgs a = a0;
  if (a.Hi <= 0) { a.Hi = a.H; a.Wi = a.W; }
  const int V = dtype == DT_F32 ? 4 : 8;
  const int KS = a.Cin / 32;
  if (a.Cin % 32 || KS < 2 || KS > 4 || a.E % IR_EC || a.E <= 0 || a.Cout % 16 ||
      a.Cout > 128 || a.Cout <= 0 || a.H < 1 || a.W < 1 || a.N < 1)
    return false;
  if (a.stride != 1 && a.stride != 2) return false;
  if (a.stride == 1 ? (a.Hi != a.H || a.Wi != a.W)
                    : (a.H != (a.Hi - 1) / 2 + 1 || a.W != (a.Wi - 1) / 2 + 1 || a.residual))
    return false;
  if (a.ldx % V || a.ldy % V || a.ldx < a.Cin || a.ldy < a.Cout) return false;
  if (a.residual && a.Cin != a.Cout) return false;
  const size_t lds = a.stride == 1
      ? (dtype == DT_F32 ? ir_lds<float, 1>(KS) : ir_lds<bf16, 1>(KS))
      : (dtype == DT_F32 ? ir_lds<float, 2>(KS) : ir_lds<bf16, 2>(KS));
  return lds <= 160 * 1024 - 1024;
}

template <typename T, int KS, int S>
static void ir_launch_ks(const IrArgs& a, dim3 grid, hipStream_t st) {
  const size_t lds = ir_lds<T, S>(KS);
  constexpr int PT = IrTile<S>::PT;  // project pixel tiles: all per wave above 64 outputs
  if constexpr (sizeof(T) == 4) {
    if (a.we3 && a.wp3) {
      if (a.Cout > 64) prof_launch(ir_block_kernel<T, KS, PT, true, S>, grid, IR_THREADS, lds, st, a);
      else prof_launch(ir_block_kernel<T, KS, PT / 2, true, S>, grid, IR_THREADS, lds, st, a);
      return;
    }
  }
  if (a.Cout > 64) prof_launch(ir_block_kernel<T, KS, PT, false, S>, grid, IR_THREADS, lds, st, a);
  else prof_launch(ir_block_kernel<T, KS, PT / 2, false, S>, grid, IR_THREADS, lds, st, a);
}

template <typename T, int S>
static void ir_launch_s(const IrArgs& a, dim3 grid, hipStream_t st) {
  switch (a.Cin / 32) {
    case 2: ir_launch_ks<T, 2, S>(a, grid, st); break;
    case 3: ir_launch_ks<T, 3, S>(a, grid, st); break;
    default: ir_launch_ks<T, 4, S>(a, grid, st); break;
  }
}

template <typename T>
static void ir_launch(const IrArgs& a, dim3 grid, hipStream_t st) {
  if (a.stride == 2) ir_launch_s<T, 2>(a, grid, st);
  else ir_launch_s<T, 1>(a, grid, st);
}

int ir_block_fwd(const IrArgs& a0, int dtype, hipStream_t st) {
  IrArgs a = a0;
  if (a.Hi <= 0) { a.Hi = a.H; a.Wi = a.W; }
  if (!ir_block_ok(a, dtype)) {
    set_error("ir_block_fwd: unsupported block (Cin %d E %d Cout %d ldx %d ldy %d residual %d "
              "stride %d)", a.Cin, a.E, a.Cout, a.ldx, a.ldy, a.residual, a.stride);
    return E_UNSUPPORTED;
  }
  const int TH = a.stride == 2 ? IrTile<2>::TH : IrTile<1>::TH;
  const int TW = a.stride == 2 ? IrTile<2>::TW : IrTile<1>::TW;
  const long long tiles = (long long)a.N * cdiv(a.H, TH) * cdiv(a.W, TW);
  if (tiles > 0x7fffffffLL) {
    set_error("ir_block_fwd: grid too large");
    return E_UNSUPPORTED;
  }
  const dim3 grid((unsigned)tiles);
  const double E = dtype == DT_F32 ? 4.0 : 2.0;
  const double M = (double)a.N * a.H * a.W, Mi = (double)a.N * a.Hi * a.Wi;
  ProfScope ps(PK_IR, st,
               E * (Mi * a.Cin + M * a.Cout * (a.residual ? 2 : 1)) +
                   E * ((double)a.E * (a.Cin + a.Cout)) + 4.0 * 9 * a.E,
               2.0 * (Mi * a.E * a.Cin + M * a.E * a.Cout) + 18.0 * M * a.E);
  if (dtype == DT_F32) ir_launch<float>(a, grid, st);
  else if (dtype == DT_F16) ir_launch<f16>(a, grid, st);
  else ir_launch<bf16>(a, grid, st);
  return check_launch("ir_block_fwd");
}

// ================================================================================================
// Training form of the bottleneck's first two layers (models/fast_scnn.py:102-107: expand
// _ConvBNReLU + depthwise _DWConv's conv), recomputing the 6x-expanded tensor instead of storing
// it.  Train-mode BatchNorm needs the expand output's batch statistics before anything can be
// normalised, so the expand runs twice: a statistics-only pass (the streaming GEMM with no output
// stores, gemm_stream.hip) finishes BN_e, then this launch recomputes the expand per tile, applies
// BN_e + ReLU in LDS and runs the depthwise 3x3 on it, storing only the depthwise's pre-BN output
// (the unfused path's dw z, bit-identical: same MFMA k order as the streaming GEMM, same rounding
// of the expand output to the storage type, bn_apply's relu(fmaf(z, scale, shift)) rounded to the
// storage type, the depthwise's tap order) and one (mean, M2, count) record per workgroup and
// channel for BN_d (statistics of the stored values).  The 201 MB (bottleneck1.0, cfg3) expand
// output is neither written nor read back; the backward recomputes it (net.cpp).
// 16-bit plans only (bf16 / fp16: one MFMA per operand pair).
// ================================================================================================
constexpr int IRT_PRM = IR_EC * 9 + 2 * IR_EC;  // per-chunk depthwise weights + BN_e (scale, shift)

template <typename T, int S>
__host__ __device__ constexpr size_t ir_train_lds(int KS) {
  using G = IrTile<S>;
  return (size_t)G::XROWS * (32 * KS + 16) * 2  // input tile
         + (size_t)G::ROWS * IR_ELD * 4           // expand chunk (fp32)
         + G::ROWS * 4                            // halo validity
         + (size_t)2 * IRT_PRM * 4                // chunk parameters, double-buffered
         + (size_t)IR_WAVES * IR_EC * 4 + IR_EC * 4;  // statistics rows + channel means
}

template <typename T, int KS, int S>
__global__ __launch_bounds__(IR_THREADS) void ir_train_fwd_kernel(IrArgs a) {
  using G = IrTile<S>;
  constexpr int IR_TH = G::TH, IR_TW = G::TW, IR_HW = G::HW, IR_HALO = G::HALO, IR_RT = G::RT;
  constexpr int IR_ROWS = G::ROWS, IR_XROWS = G::XROWS, NPT = G::NPT;
  constexpr int CIN = 32 * KS;
  constexpr int XLD = CIN + 16;
  constexpr int RPW = G::RPW;
  extern __shared__ __attribute__((aligned(16))) unsigned char s_dyn[];
  uint16_t* sX = reinterpret_cast<uint16_t*>(s_dyn);                      // [101][XLD]
  float* sE = reinterpret_cast<float*>(sX + (size_t)IR_XROWS * XLD);      // [ROWS][IR_ELD]
  float* sV = sE + IR_ROWS * IR_ELD;                                      // [ROWS] 1 = in image
  float* sPrm = sV + IR_ROWS;                                             // [2][IRT_PRM]
  float* sRed = sPrm + 2 * IRT_PRM;                                       // [8 waves][64]
  float* sMean = sRed + IR_WAVES * IR_EC;                                 // [64]

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int li = lane & 15, lq = lane >> 4;
  const int tiles_x = cdiv(a.W, IR_TW), tiles_y = cdiv(a.H, IR_TH);
  int t = blockIdx.x;
  const int n = t / (tiles_x * tiles_y);
  t -= n * tiles_x * tiles_y;
  const int y0 = (t / tiles_x) * IR_TH, x0 = (t % tiles_x) * IR_TW;
  const T* X = (const T*)a.x;
  const T* We = (const T*)a.we;
  const int ect = wave & 3, erh = (wave >> 2) * RPW;
  const int dq = tid & 15, dg = tid >> 4;
  const int doy = dg / (IR_TW / NPT), dox = (dg % (IR_TW / NPT)) * NPT;
  // valid output pixels of the tile (the BN_d record's count) and of this thread
  const int vh = min(IR_TH, a.H - y0), vw = min(IR_TW, a.W - x0);
  const float cnt = (float)(vh * vw);
  bool pv[NPT];
#pragma unroll
  for (int i = 0; i < NPT; ++i) pv[i] = doy < vh && dox + i < vw;

  uint4 rwe[KS];
  float rprm[2];
  auto fetch_we = [&](int e0) {
    const int erow = e0 + ect * 16 + li;
#pragma unroll
    for (int s = 0; s < KS; ++s)
      rwe[s] = *reinterpret_cast<const uint4*>(We + (size_t)erow * CIN + 32 * s + 8 * lq);
  };
  // parameter entries tid and tid + 512: entry i < 576 is wd[e0 * 9 + i], then BN_e scale, shift
  const float* psrc[2];
  int pmul[2];
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int i = tid + u * IR_THREADS;
    if (i < IR_EC * 9) {
      psrc[u] = a.wd + i;
      pmul[u] = 9;
    } else {
      const int j = min(i, IRT_PRM - 1) - IR_EC * 9, tab = j / IR_EC, c = j - tab * IR_EC;
      psrc[u] = (tab == 0 ? a.sc_e : a.sh_e) + c;
      pmul[u] = 1;
    }
  }
  auto fetch_prm = [&](int e0) {
#pragma unroll
    for (int u = 0; u < 2; ++u) rprm[u] = psrc[u][(size_t)e0 * pmul[u]];
  };
  auto put_prm = [&](int buf) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int i = tid + u * IR_THREADS;
      if (i < IRT_PRM) sPrm[buf * IRT_PRM + i] = rprm[u];
    }
  };

  fetch_we(0);
  fetch_prm(0);
  put_prm(0);
  // ---- stage the haloed input tile (the producer's lazily applied BN + ReLU when given) -------
  {
    constexpr int VPR = CIN / 8;
    for (int i = tid; i < IR_XROWS * VPR; i += IR_THREADS) {
      const int r = i / VPR, v = i - r * VPR;
      const int hy = r / IR_HW, hx = r - hy * IR_HW;
      const int gy = S * y0 - 1 + hy, gx = S * x0 - 1 + hx;
      const bool ok = r < IR_HALO && gy >= 0 && gy < a.Hi && gx >= 0 && gx < a.Wi;
      const size_t off = ok ? (((size_t)n * a.Hi + gy) * a.Wi + gx) * a.ldx + v * 8 : 0;
      uint4 q = *reinterpret_cast<const uint4*>(X + off);
      if (a.x_scale) q = bnrelu_vec<T>(q, a.x_scale + v * 8, a.x_shift + v * 8);
      *reinterpret_cast<uint4*>(sX + (size_t)r * XLD + v * 8) = sel4(ok, q);
      if (v == 0) sV[r] = ok ? 1.f : 0.f;
    }
    for (int r = IR_XROWS + tid; r < IR_ROWS; r += IR_THREADS) sV[r] = 0.f;
  }

  T* Y = (T*)a.y;
  const int nchunks = a.E / IR_EC;
  for (int ch = 0; ch < nchunks; ++ch) {
    const int e0 = ch * IR_EC;
    const float* prm = sPrm + (ch & 1) * IRT_PRM;
    uint4 we[KS];
#pragma unroll
    for (int s = 0; s < KS; ++s) we[s] = rwe[s];
    if (ch + 1 < nchunks) {
      fetch_we(e0 + IR_EC);  // in flight during this chunk
      fetch_prm(e0 + IR_EC);
    }
    __syncthreads();  // input tile + this chunk's parameters staged; sE free
    // ---- expand, rounded to the storage type (the unfused z), BN_e + ReLU, halo zeroed ----------
    {
      f32x4 acc[RPW];
#pragma unroll
      for (int j = 0; j < RPW; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < KS; ++s)
#pragma unroll
        for (int j = 0; j < RPW; ++j) {
          const int rt = min(erh + j, IR_RT - 1);
          const int row = min(rt * 16 + li, IR_HALO);
          uint4 b[1];
          b[0] = *reinterpret_cast<const uint4*>(sX + (size_t)row * XLD + 32 * s + 8 * lq);
          uint4 w1[1] = {we[s]};
          ir_mma<T>(w1, b, acc[j]);
        }
      const int c = ect * 16 + 4 * lq;
      const float4 sc = *reinterpret_cast<const float4*>(prm + IR_EC * 9 + c);
      const float4 sh = *reinterpret_cast<const float4*>(prm + IR_EC * 10 + c);
#pragma unroll
      for (int j = 0; j < RPW; ++j) {
        const int rt = min(erh + j, IR_RT - 1);
        const int px = rt * 16 + li;
        const float valid = sV[px];
        float4 o;
        o.x = valid * round_as<T>(fmaxf(fmaf(round_as<T>(acc[j][0]), sc.x, sh.x), 0.f));
        o.y = valid * round_as<T>(fmaxf(fmaf(round_as<T>(acc[j][1]), sc.y, sh.y), 0.f));
        o.z = valid * round_as<T>(fmaxf(fmaf(round_as<T>(acc[j][2]), sc.z, sh.z), 0.f));
        o.w = valid * round_as<T>(fmaxf(fmaf(round_as<T>(acc[j][3]), sc.w, sh.w), 0.f));
        *reinterpret_cast<float4*>(sE + (size_t)px * IR_ELD + c) = o;
      }
    }
    __syncthreads();
    // ---- depthwise 3x3 of the chunk: pre-BN output stored, its statistics per channel ---------
    float v[NPT][4];
    {
      float w[4][9];
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int k = 0; k < 9; ++k) w[j][k] = prm[(4 * dq + j) * 9 + k];
      constexpr int NC = S * (NPT - 1) + 3;
      float4 xv[3][NC];
#pragma unroll
      for (int kh = 0; kh < 3; ++kh)
#pragma unroll
        for (int c = 0; c < NC; ++c)
          xv[kh][c] = *reinterpret_cast<const float4*>(
              sE + (size_t)((S * doy + kh) * IR_HW + S * dox + c) * IR_ELD + 4 * dq);
      float acc[NPT][4];
#pragma unroll
      for (int i = 0; i < NPT; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = 0.f;
#pragma unroll
      for (int kh = 0; kh < 3; ++kh)
#pragma unroll
        for (int kw = 0; kw < 3; ++kw)
#pragma unroll
          for (int i = 0; i < NPT; ++i) {
            const float4 q = xv[kh][S * i + kw];
            const float qq[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[i][j] = fmaf(qq[j], w[j][kh * 3 + kw], acc[i][j]);
          }
#pragma unroll
      for (int i = 0; i < NPT; ++i) {
#pragma unroll
        for (int j = 0; j < 4; ++j) v[i][j] = round_as<T>(acc[i][j]);
        if (pv[i]) {
          const size_t pix = ((size_t)n * a.H + y0 + doy) * a.W + x0 + dox + i;
          st4v(Y + pix * a.ldy + e0 + 4 * dq, v[i]);
        }
      }
    }
    if (ch + 1 < nchunks) put_prm((ch + 1) & 1);  // (its last readers finished chunk ch - 1)
    // ---- BN_d record of the chunk: mean over the tile's valid pixels, then M2 ------------------
    float s4[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float s = 0.f;
#pragma unroll
      for (int i = 0; i < NPT; ++i) s += pv[i] ? v[i][j] : 0.f;
      s += __shfl_xor(s, 16);
      s += __shfl_xor(s, 32);
      s4[j] = s;
    }
    if (lq == 0) *reinterpret_cast<float4*>(sRed + wave * IR_EC + 4 * dq) = make_float4(s4[0], s4[1], s4[2], s4[3]);
    __syncthreads();
    if (tid < IR_EC) {
      float s = 0.f;
#pragma unroll
      for (int w8 = 0; w8 < IR_WAVES; ++w8) s += sRed[w8 * IR_EC + tid];
      sMean[tid] = s / cnt;
    }
    __syncthreads();
    {
      const float4 mu = *reinterpret_cast<const float4*>(sMean + 4 * dq);
      const float m4[4] = {mu.x, mu.y, mu.z, mu.w};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float s = 0.f;
#pragma unroll
        for (int i = 0; i < NPT; ++i) {
          const float d = v[i][j] - m4[j];
          s += pv[i] ? d * d : 0.f;
        }
        s += __shfl_xor(s, 16);
        s += __shfl_xor(s, 32);
        s4[j] = s;
      }
    }
    __syncthreads();  // every thread read sMean / the sums rows
    if (lq == 0) *reinterpret_cast<float4*>(sRed + wave * IR_EC + 4 * dq) = make_float4(s4[0], s4[1], s4[2], s4[3]);
    __syncthreads();
    if (tid < IR_EC) {
      float m2 = 0.f;
#pragma unroll
      for (int w8 = 0; w8 < IR_WAVES; ++w8) m2 += sRed[w8 * IR_EC + tid];
      float* rec = a.part + (size_t)blockIdx.x * 3 * a.E + e0 + tid;
      rec[0] = sMean[tid];
      rec[a.E] = m2;
      rec[2 * a.E] = cnt;
    }
  }
}

bool ir_train_ok(const IrArgs& a0, int dtype) {
  IrArgs a = a0;
  if (a.Hi <= 0) { a.Hi = a.H; a.Wi = a.W; }
  if (dtype != DT_BF16 && dtype != DT_F16) return false;
  const int KS = a.Cin / 32;
  if (a.Cin % 32 || KS < 2 || KS > 4 || a.E % IR_EC || a.E <= 0 || a.H < 1 || a.W < 1 ||
      a.N < 1 || !a.part || !a.sc_e || !a.sh_e || !a.wd || !a.we || !a.x || !a.y)
    return false;
  if (a.stride != 1 && a.stride != 2) return false;
  if (a.stride == 1 ? (a.Hi != a.H || a.Wi != a.W)
                    : (a.H != (a.Hi - 1) / 2 + 1 || a.W != (a.Wi - 1) / 2 + 1))
    return false;
  if (a.ldx % 8 || a.ldx < a.Cin || a.ldy < a.E || a.ldy % 4) return false;
  if (((uintptr_t)a.x & 15) || ((uintptr_t)a.we & 15) || ((uintptr_t)a.y & 7)) return false;
  if ((a.x_scale == nullptr) != (a.x_shift == nullptr)) return false;
  const size_t lds = a.stride == 1 ? ir_train_lds<bf16, 1>(KS) : ir_train_lds<bf16, 2>(KS);
  return lds <= 160 * 1024 - 1024;
}

long long ir_train_parts(int N, int H, int W, int stride) {
  const int TH = stride == 2 ? IrTile<2>::TH : IrTile<1>::TH, TW = stride == 2 ? IrTile<2>::TW : IrTile<1>::TW;
  return (long long)N * cdiv(H, TH) * cdiv(W, TW);
}

template <typename T, int S>
static void ir_train_launch_s(const IrArgs& a, dim3 grid, hipStream_t st) {
  switch (a.Cin / 32) {
    case 2: prof_launch(ir_train_fwd_kernel<T, 2, S>, grid, IR_THREADS, ir_train_lds<T, S>(2), st, a); break;
    case 3: prof_launch(ir_train_fwd_kernel<T, 3, S>, grid, IR_THREADS, ir_train_lds<T, S>(3), st, a); break;
    default: prof_launch(ir_train_fwd_kernel<T, 4, S>, grid, IR_THREADS, ir_train_lds<T, S>(4), st, a); break;
  }
}

int ir_train_fwd(const IrArgs& a0, int dtype, hipStream_t st) {
  IrArgs a = a0;
  if (a.Hi <= 0) { a.Hi = a.H; a.Wi = a.W; }
  if (!ir_train_ok(a, dtype)) {
    set_error("ir_train_fwd: unsupported block (dtype %d Cin %d E %d ldx %d ldy %d stride %d)",
              dtype, a.Cin, a.E, a.ldx, a.ldy, a.stride);
    return E_UNSUPPORTED;
  }
  const long long tiles = ir_train_parts(a.N, a.H, a.W, a.stride);
  if (tiles > 0x7fffffffLL) {
    set_error("ir_train_fwd: grid too large");
    return E_UNSUPPORTED;
  }
  const dim3 grid((unsigned)tiles);
  const double M = (double)a.N * a.H * a.W, Mi = (double)a.N * a.Hi * a.Wi;
  ProfScope ps(PK_IR, st, 2.0 * (Mi * a.Cin + M * a.E) + 2.0 * a.E * a.Cin + 4.0 * 9 * a.E,
               2.0 * Mi * a.E * a.Cin + 18.0 * M * a.E);
  if (dtype == DT_F16) {
    if (a.stride == 2) ir_train_launch_s<f16, 2>(a, grid, st);
    else ir_train_launch_s<f16, 1>(a, grid, st);
  } else {
    if (a.stride == 2) ir_train_launch_s<bf16, 2>(a, grid, st);
    else ir_train_launch_s<bf16, 1>(a, grid, st);
  }
  return check_launch("ir_train_fwd");
}

}  // namespace fscnn
