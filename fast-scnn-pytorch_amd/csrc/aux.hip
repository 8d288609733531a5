// Auxiliary head of FastSCNN(num_classes, aux=True) (models/fast_scnn.py:24-31, 42-45):
//     Conv2d(64, 32, 3, padding=1, bias=False) -> BatchNorm2d(32) -> ReLU -> Dropout(0.1)
//     -> Conv2d(32, num_classes, 1) -> bilinear(align_corners=True) to the input size
// on the LearningToDownsample output (NHWC [N][H3][W3][64]).
//
// The dense 3x3 conv (K = 64 * 9 = 576) is an explicit im2col followed by the MFMA pointwise GEMM
// of gemm.hip.  The column order k = c*9 + kh*3 + kw is PyTorch's weight order, so the weight
// operand is the [32][64][3][3] parameter read as [32][576] as it lies in the arena, and the
// weight-gradient GEMM over the same columns writes dW in PyTorch layout.  The input gradient is
// dcol = dZ * W (the dgrad GEMM) folded back by col2im, a fixed-order gather
//     dx[n][h][w][c] (+)= sum_{kh,kw} dcol[n][h+1-kh][w+1-kw][c*9 + kh*3 + kw]
// (no scatter, no atomics).  Both are HBM-bound copies: im2col reads e*P*64 and writes e*P*576
// bytes for P pixels; col2im reads e*P*576 and writes (or reads and writes) e*P*64.
#include "kernels.hpp"

namespace fscnn {

// thread = one (pixel, channel); a wave covers whole pixels, so its 9-element runs form
// contiguous 64*9-element segments of the column row
template <typename R>  // raw storage word (bits copied): uint32_t for fp32, uint16_t for bf16
__global__ __launch_bounds__(256) void im2col3_kernel(Im2ColArgs a) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long total = (long long)a.N * a.H * a.W * a.C;
  if (i >= total) return;
  const int c = (int)(i % a.C);
  const long long pix = i / a.C;
  const int w = (int)(pix % a.W);
  const long long r = pix / a.W;
  const int h = (int)(r % a.H), n = (int)(r / a.H);
  const R* x = (const R*)a.x;
  R* col = (R*)a.col + pix * a.ldcol + c * 9;
#pragma unroll
  for (int kh = 0; kh < 3; ++kh) {
    const int hh = h + kh - 1;
#pragma unroll
    for (int kw = 0; kw < 3; ++kw) {
      const int ww = w + kw - 1;
      const bool ok = hh >= 0 && hh < a.H && ww >= 0 && ww < a.W;
      const R v = x[ok ? (((size_t)n * a.H + hh) * a.W + ww) * a.ldx + c : 0];
      col[kh * 3 + kw] = ok ? v : (R)0;
    }
  }
}

template <typename T>
__global__ __launch_bounds__(256) void col2im3_kernel(Col2ImArgs a) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long total = (long long)a.N * a.H * a.W * a.C;
  if (i >= total) return;
  const int c = (int)(i % a.C);
  const long long pix = i / a.C;
  const int w = (int)(pix % a.W);
  const long long r = pix / a.W;
  const int h = (int)(r % a.H), n = (int)(r / a.H);
  const T* dcol = (const T*)a.dcol;
  float s = 0.f;
#pragma unroll
  for (int kh = 0; kh < 3; ++kh) {
    const int ho = h + 1 - kh;
#pragma unroll
    for (int kw = 0; kw < 3; ++kw) {
      const int wo = w + 1 - kw;
      const bool ok = ho >= 0 && ho < a.H && wo >= 0 && wo < a.W;
      const size_t off =
          ok ? (((size_t)n * a.H + ho) * a.W + wo) * a.ldcol + c * 9 + kh * 3 + kw : 0;
      const float v = ld1(dcol + off);
      s += ok ? v : 0.f;
    }
  }
  T* dx = (T*)a.dx + pix * a.lddx + c;
  st1(dx, a.accumulate ? ld1(dx) + s : s);
}

int im2col3(const Im2ColArgs& a, int dtype, hipStream_t st) {
  const long long total = (long long)a.N * a.H * a.W * a.C;
  if (total <= 0 || total >= (1LL << 40) || a.ldx < a.C || a.ldcol < 9 * a.C) {
    set_error("im2col3: bad geometry (C=%d ldx=%d ldcol=%d)", a.C, a.ldx, a.ldcol);
    return E_INVALID;
  }
  const unsigned grid = (unsigned)((total + 255) / 256);
  if (dtype == DT_F32) prof_launch(im2col3_kernel<uint32_t>, grid, 256, 0, st, a);
  else prof_launch(im2col3_kernel<uint16_t>, grid, 256, 0, st, a);
  return check_launch("im2col3");
}

int col2im3(const Col2ImArgs& a, int dtype, hipStream_t st) {
  const long long total = (long long)a.N * a.H * a.W * a.C;
  if (total <= 0 || total >= (1LL << 40) || a.lddx < a.C || a.ldcol < 9 * a.C) {
    set_error("col2im3: bad geometry (C=%d lddx=%d ldcol=%d)", a.C, a.lddx, a.ldcol);
    return E_INVALID;
  }
  const unsigned grid = (unsigned)((total + 255) / 256);
  if (dtype == DT_F32) prof_launch(col2im3_kernel<float>, grid, 256, 0, st, a);
  else if (dtype == DT_F16) prof_launch(col2im3_kernel<f16>, grid, 256, 0, st, a);
  else prof_launch(col2im3_kernel<bf16>, grid, 256, 0, st, a);
  return check_launch("col2im3");
}

}  // namespace fscnn
