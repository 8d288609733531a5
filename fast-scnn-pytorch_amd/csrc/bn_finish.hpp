// Per-channel BatchNorm finish arithmetic shared by the finalize kernels (bn.hip) and the
// in-kernel finish of the streaming GEMM producers (gemm_stream.hip): one definition, so both
// paths give bit-identical mean / invstd / scale / shift / running statistics / coefficients.
#pragma once
#include "kernels.hpp"

namespace fscnn {

constexpr float BN_EPS = 1e-5f;

// forward: fp64 sums over the merged records, n = sum count, s1 = sum n*mean,
// s2 = sum (M2 + n*mean^2) -> mean / invstd / scale / shift and aten's running-stat update
// (unbiased variance n/(n-1), momentum) of channel c
__device__ __forceinline__ void bn_fwd_finish(const BnFinalizeArgs& a, int c, double n, double s1,
                                              double s2) {
  const double mu = n > 0.0 ? s1 / n : 0.0;
  const double m2 = n > 0.0 ? fmax(s2 - n * mu * mu, 0.0) : 0.0;
  const double mean = mu + (a.bias ? (double)a.bias[c] : 0.0);
  const double var = n > 0 ? m2 / n : 0.0;
  const float invstd = (float)(1.0 / sqrt(var + (double)BN_EPS));
  const float scale = a.gamma[c] * invstd;
  a.mean[c] = (float)mean;
  a.invstd[c] = invstd;
  a.scale[c] = scale;
  a.shift[c] = a.beta[c] - (float)mean * scale;
  if (a.rmean) {
    const float m = a.momentum;
    a.rmean[c] = (1.f - m) * a.rmean[c] + m * (float)mean;
    const float unb = n > 1 ? (float)(m2 / (n - 1.0)) : (float)var;
    a.rvar[c] = (1.f - m) * a.rvar[c] + m * unb;
  }
  if (a.nbt && c == 0) a.nbt[0] += 1;
}

// backward: s1 = sum dy_r, s2 = sum dy_r * xhat of channel c (C channels) -> dbeta, dgamma, the
// apply coefficients and (t.tab) the BN-backward operand table
// dz = scale*(dy_r - c0 - (z - mean)*invstd*c1) = al*dy_r + gz*z + be
__device__ __forceinline__ void bn_bwd_finish(int c, int C, double s1, double s2, double count,
                                              float* dgamma, float* dbeta, float* coef,
                                              const BnBwdTab& t) {
  if (dbeta) dbeta[c] = (float)s1;
  if (dgamma) dgamma[c] = (float)s2;
  const float c0 = (float)(s1 / count), c1 = (float)(s2 / count);
  coef[c] = c0;
  coef[C + c] = c1;
  if (t.tab) {
    const float sc = t.scale[c];
    const float gz = -sc * c1 * t.invstd[c];
    float4 v;
    v.x = sc;
    v.y = -sc * c0 - gz * t.mean[c];
    v.z = gz;
    v.w = t.relu ? sc : 0.f;
    float* e = t.tab + (size_t)c * BWDX_STRIDE;
    *reinterpret_cast<float4*>(e) = v;
    e[4] = t.relu ? t.shift[c] : 1.f;
  }
}

}  // namespace fscnn
