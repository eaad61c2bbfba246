// refmath.h -- the reference's elementary functions, bit for bit.
//
// The reference's numbers come from four libraries: numpy 2.2.6's np.log /
// np.exp on contiguous float64 arrays run Intel SVML's AVX-512 high-accuracy
// kernels (__svml_log8_ha, __svml_exp8_ha, bundled in numpy's
// _multiarray_umath); scipy.special.expit is 1 / (1 + exp(-x)) with glibc
// 2.35's exp (the FMA variant its ifunc picks on an FMA CPU); np.logaddexp is
// x + log1p(exp(y - x)) with glibc's exp and log1p; the L-BFGS-B control calls
// OpenBLAS 0.3.28 (lbfgsb1.h restates those small kernels).  Each function
// below restates one of them operation for operation -- the same constants
// (refmath_tables.h, read from the installed libraries by
// tools/gen_refmath_tables.py), the same fused multiply-adds and roundings
// -- so a device evaluation gives the reference's bits.  tests/host/
// refmath_check.cpp compares every function with the library itself over 2 x
// 10^7 inputs per range on the CPU, and tests/test_gpu_exact.py the device builds
// with numpy / scipy on the GPU box.
//
// Domain: finite inputs in the ranges the path produces (documented per
// function); outside them the functions still return the mathematically
// right value but are not held to the libraries' bits.
//
// Header-only, host and device (hipcc) or host only (g++ with
// -ffp-contract=off: every fused operation below is an explicit fma()).
//
// Attribution: the algorithms restated here are glibc 2.35's exp (Szabolcs
// Nagy, Arm; LGPL-2.1-or-later) and log1p (fdlibm, Sun Microsystems: "Developed
// at SunPro, a Sun Microsystems, Inc. business. Permission to use, copy,
// modify, and distribute this software is freely granted, provided that this
// notice is preserved."), and Intel SVML's log / exp kernels as bundled in
// numpy (BSD-3-Clause, Intel Corporation).  No library source is copied; see
// THIRD_PARTY_NOTICES.md.
#pragma once

#include <stdint.h>

#include "refmath_tables.h"

#if defined(__HIPCC__)
#define NEMO_RM __host__ __device__ __forceinline__
#define NEMO_RMM __host__ __device__ __forceinline__
#else
#define NEMO_RM static inline
#define NEMO_RMM inline
#endif

#if defined(__clang__)
#define NEMO_RM_NOCONTRACT _Pragma("clang fp contract(off)")
#else
#define NEMO_RM_NOCONTRACT
#endif

namespace nemo {
namespace refmath {

NEMO_RM double as_double(uint64_t u) { return __builtin_bit_cast(double, u); }

NEMO_RM uint64_t as_u64(double d) { return __builtin_bit_cast(uint64_t, d); }
NEMO_RM double fma_(double a, double b, double c) { return __builtin_fma(a, b, c); }

// n / d rounded to nearest, for d in [1, 4) and n = 0 or |n| in [2^-60, 4):
// on the device the core of the compiler's division sequence (reciprocal,
// two Newton steps, the residual correction) without v_div_scale /
// v_div_fmas's scaling and v_div_fixup's special cases, which leave such
// operands unchanged -- the same bits as `n / d` in three fewer instructions
// (tests/test_gpu_exact.py).  A smaller |n| (the residual would lose bits)
// still gives a finite value near n / d.  On the host n / d
NEMO_RM double div_rn(double n, double d) {
#if defined(__HIP_DEVICE_COMPILE__)
  const double y0 = __builtin_amdgcn_rcp(d);
  const double y1 = __builtin_fma(y0, __builtin_fma(-d, y0, 1.0), y0);
  const double y = __builtin_fma(y1, __builtin_fma(-d, y1, 1.0), y1);
  const double q = n * y;
  return __builtin_fma(__builtin_fma(-d, q, n), y, q);
#else
  return n / d;
#endif
}

// svml_log's reduction row for n = the number of vrcp14 switch points at or
// below the mantissa (kRcp14Switch): r = RNE_1/32(vrcp14pd(m)) = (32 - n) / 32,
// the exponent adjustment (1 when r < 0.75) minus the exponent bias 1023, and
// T(r) = log_hi + log_lo
NEMO_RM void svml_log_row(int n, double* row) {
  const double r = (double)(32 - n) * 0.03125;
  const int j = (int)(as_u64(r) >> 48) & 15;
  row[0] = r;
  row[1] = (r < 0.75 ? 1.0 : 0.0) - 1023.0;   // the exponent's adjustment and its bias, exact
  row[2] = as_double(kSvmlLogHi[j]);
  row[3] = as_double(kSvmlLogLo[j]);
}

// Where the functions read their tables: by default the constant arrays of
// refmath_tables.h; a device kernel passes copies in LDS (per-lane indices)
struct ConstTabs {
  // svml_log: the row of the 22-bit mantissa prefix p22
  NEMO_RMM void log_row(uint32_t p22, double& r, double& kadj, double& hi, double& lo) const {
    int n = 0;
    for (int t = 0; t < 16; ++t) n += p22 >= kRcp14Switch[t] ? 1 : 0;
    double row[4];
    svml_log_row(n, row);
    r = row[0], kadj = row[1], hi = row[2], lo = row[3];
  }
  NEMO_RMM void exp_row(int j, double& hi, double& lo) const {
    hi = as_double(kSvmlExpHi[j]);
    lo = as_double(kSvmlExpLo[j]);
  }
  NEMO_RMM uint64_t gexp(int i) const { return kGlibcExpTab[i]; }
};
// The LDS form: the step function bucketed by the top 6 bits of p22 (one
// switch point at most per bucket, kRcp14InBucket) and svml_log's rows per
// (bucket, above its switch point): two dependent reads per log.  Equal to
// ConstTabs for every prefix (tests/test_exact_spec.py).
struct LdsTabs {
  const uint32_t* rthr_p;   // [64] kRcp14InBucket
  const double* lrow_p;     // [64][2][4] svml_log_row(kRcp14Base[b] + above)
  const double* erow_p;     // [16][2] SVML exp's 2^(j/16) hi, lo
  const uint64_t* gexp_p;   // [256] glibc exp's table
  NEMO_RMM void log_row(uint32_t p22, double& r, double& kadj, double& hi, double& lo) const {
    const uint32_t b = p22 >> 16;
    const double* row = lrow_p + 4 * (2 * b + (p22 >= rthr_p[b] ? 1 : 0));
    r = row[0], kadj = row[1], hi = row[2], lo = row[3];
  }
  NEMO_RMM void exp_row(int j, double& hi, double& lo) const {
    hi = erow_p[2 * j];
    lo = erow_p[2 * j + 1];
  }
  NEMO_RMM uint64_t gexp(int i) const { return gexp_p[i]; }
};

// ---------------------------------------------------------------------------
// glibc 2.35 exp (sysdeps/ieee754/dbl-64/e_exp.c, Szabolcs Nagy's table
// method, N = 128, degree-5 polynomial), compiled with -mfma as __exp_fma:
// kd = fma(InvLn2N, x, Shift); r = fma(kd, NegLn2loN, fma(kd, NegLn2hiN, x));
// tmp = fma(r2 * r2, fma(r, C5, C4), fma(r2, fma(r, C3, C2), tail + r));
// result fma(scale, tmp, scale).  All inputs (specialcase for |x| > 512
// included).
// ---------------------------------------------------------------------------
NEMO_RM double glibc_exp_special(double tmp, uint64_t sbits, uint64_t ki) {
  NEMO_RM_NOCONTRACT
  if ((ki & 0x80000000u) == 0) {
    // k > 0: the exponent of scale may have overflowed by <= 460
    sbits -= 1009ull << 52;
    const double scale = as_double(sbits);
    return 0x1p1009 * fma_(scale, tmp, scale);
  }
  // k < 0: the subnormal range, rounded once
  sbits += 1022ull << 52;
  const double scale = as_double(sbits);
  double y = scale + scale * tmp;  // __exp_fma's specialcase is not fused (measured)
  if (y < 1.0) {
    double lo = (scale - y) + scale * tmp;
    const double hi = 1.0 + y;
    lo = ((1.0 - hi) + y) + lo;
    y = (hi + lo) - 1.0;
    if (y == 0.0) y = 0.0;
  }
  return 0x1p-1022 * y;
}

template <class TB = ConstTabs>
NEMO_RM double glibc_exp(double x, const TB& tb = TB{}) {
  NEMO_RM_NOCONTRACT
  constexpr double kInvLn2N = 0x1.71547652b82fep0 * 128;
  constexpr double kShift = 0x1.8p52;
  constexpr double kNegLn2hiN = -0x1.62e42fefa0000p-8;
  constexpr double kNegLn2loN = -0x1.cf79abc9e3b3ap-47;
  constexpr double C2 = 0x1.ffffffffffdbdp-2, C3 = 0x1.555555555543cp-3;
  constexpr double C4 = 0x1.55555cf172b91p-5, C5 = 0x1.1111167a4d017p-7;
  uint32_t abstop = (uint32_t)(as_u64(x) >> 52) & 0x7ff;
  // top12(0x1p-54) = 0x3c9, top12(512) = 0x408, top12(1024) = 0x409
  if (abstop - 0x3c9u >= 0x408u - 0x3c9u) {
    if (abstop - 0x3c9u >= 0x80000000u) return 1.0 + x;  // tiny x
    if (abstop >= 0x409u) {
      if (as_u64(x) == 0xfff0000000000000ull) return 0.0;
      if (abstop >= 0x7ffu) return 1.0 + x;
      return (as_u64(x) >> 63) ? 0.0 : __builtin_inf();
    }
    abstop = 0;  // large |x|: specialcase below
  }
  double kd = fma_(kInvLn2N, x, kShift);
  const uint64_t ki = as_u64(kd);
  kd -= kShift;
  const double r = fma_(kd, kNegLn2loN, fma_(kd, kNegLn2hiN, x));
  const uint64_t idx = 2 * (ki % 128);
  const uint64_t top = ki << 45;
  const double tail = as_double(tb.gexp((int)idx));
  const uint64_t sbits = tb.gexp((int)idx + 1) + top;
  const double r2 = r * r;
  const double tmp = fma_(r2 * r2, fma_(r, C5, C4), fma_(r2, fma_(r, C3, C2), tail + r));
  if (abstop == 0) return glibc_exp_special(tmp, sbits, ki);
  const double scale = as_double(sbits);
  return fma_(scale, tmp, scale);
}

// scipy.special.expit for float64: 1 / (1 + exp(-x)) (scipy 1.15 special,
// std::exp = glibc exp)
template <class TB = ConstTabs>
NEMO_RM double expit(double x, const TB& tb = TB{}) {
  NEMO_RM_NOCONTRACT
  return 1.0 / (1.0 + glibc_exp(-x, tb));
}

// ---------------------------------------------------------------------------
// glibc 2.35 log1p (sysdeps/ieee754/dbl-64/s_log1p.c, the fdlibm algorithm;
// no FMA variant on x86_64), for x > -1 finite.
// ---------------------------------------------------------------------------
NEMO_RM double glibc_log1p(double x) {
  NEMO_RM_NOCONTRACT
  constexpr double ln2_hi = 6.93147180369123816490e-01, ln2_lo = 1.90821492927058770002e-10;
  constexpr double Lp1 = 6.666666666666735130e-01, Lp2 = 3.999999999940941908e-01,
                   Lp3 = 2.857142874366239149e-01, Lp4 = 2.222219843214978396e-01,
                   Lp5 = 1.818357216161805012e-01, Lp6 = 1.531383769920937332e-01,
                   Lp7 = 1.479819860511658591e-01;
  const int32_t hx = (int32_t)(as_u64(x) >> 32);
  const int32_t ax = hx & 0x7fffffff;
  int32_t k = 1, hu = 0;
  double f = 0.0, c = 0.0;
  if (hx < 0x3FDA827A) {  // x < 0.41422
    if (ax >= 0x3ff00000) return x == -1.0 ? -__builtin_inf() : __builtin_nan("");
    if (ax < 0x3e200000) {  // |x| < 2^-29
      if (ax < 0x3c900000) return x;
      return x - x * x * 0.5;
    }
    if (hx > 0 || hx <= (int32_t)0xbfd2bec4) {  // -0.2929 < x < 0.41422
      k = 0;
      f = x;
      hu = 1;
    }
  } else if (hx >= 0x7ff00000) {
    return x + x;
  }
  if (k != 0) {
    double u;
    if (hx < 0x43400000) {
      u = 1.0 + x;
      hu = (int32_t)(as_u64(u) >> 32);
      k = (hu >> 20) - 1023;
      c = (k > 0) ? 1.0 - (u - x) : x - (u - 1.0);
      c /= u;
    } else {
      u = x;
      hu = (int32_t)(as_u64(u) >> 32);
      k = (hu >> 20) - 1023;
      c = 0;
    }
    hu &= 0x000fffff;
    const uint64_t lo = as_u64(u) & 0xffffffffull;
    if (hu < 0x6a09e) {
      u = as_double(((uint64_t)(uint32_t)(hu | 0x3ff00000) << 32) | lo);  // normalize u
    } else {
      k += 1;
      u = as_double(((uint64_t)(uint32_t)(hu | 0x3fe00000) << 32) | lo);  // normalize u/2
      hu = (0x00100000 - hu) >> 2;
    }
    f = u - 1.0;
  }
  const double hfsq = 0.5 * f * f;
  if (hu == 0) {  // |f| < 2^-20
    if (f == 0.0) {
      if (k == 0) return 0.0;
      c += k * ln2_lo;
      return k * ln2_hi + c;
    }
    const double R = hfsq * (1.0 - 0.66666666666666666 * f);
    if (k == 0) return f - R;
    return k * ln2_hi - ((R - (k * ln2_lo + c)) - f);
  }
  const double s = f / (2.0 + f);
  const double z = s * s;
  const double R1 = z * Lp1, z2 = z * z;
  const double R2 = Lp2 + z * Lp3, z4 = z2 * z2;
  const double R3 = Lp4 + z * Lp5, z6 = z4 * z2;
  const double R4 = Lp6 + z * Lp7;
  const double R = R1 + z2 * R2 + z4 * R3 + z6 * R4;
  if (k == 0) return f - (hfsq - s * (hfsq + R));
  return k * ln2_hi - ((hfsq - (s * (hfsq + R) + (k * ln2_lo + c))) - f);
}

// glibc_log1p for x in [0, 1] (logaddexp's argument exp(-|x - y|)) with one
// path for most lanes: x < 0.41422 (k = 0, f = x) is the default, the
// normalising branch (x >= 0.41422: 1 + x split into 2^k u and its rounding
// error c, one more division) and the k != 0 form run only in waves with a
// lane that needs them, and both divisions are div_rn.  The tiny and |f| <
// 2^-20 cases stay branches (rare).  Same bits as glibc_log1p on [0, 1]
// (tests/host/refmath_check.cpp, tests/test_gpu_exact.py).
NEMO_RM double log1p_unit(double x) {
  NEMO_RM_NOCONTRACT
  constexpr double ln2_hi = 6.93147180369123816490e-01, ln2_lo = 1.90821492927058770002e-10;
  constexpr double Lp1 = 6.666666666666735130e-01, Lp2 = 3.999999999940941908e-01,
                   Lp3 = 2.857142874366239149e-01, Lp4 = 2.222219843214978396e-01,
                   Lp5 = 1.818357216161805012e-01, Lp6 = 1.531383769920937332e-01,
                   Lp7 = 1.479819860511658591e-01;
  const int32_t hx = (int32_t)(as_u64(x) >> 32);
  double f = x, c = 0.0;
  int32_t k = 0, hu = 1;
  if (hx >= 0x3FDA827A) {
    // u = 1 + x normalised to [sqrt(2)/2, sqrt(2)), k its exponent
    const double u = 1.0 + x;
    const int32_t hu0 = (int32_t)(as_u64(u) >> 32);
    k = (hu0 >> 20) - 1023;
    c = div_rn(k > 0 ? 1.0 - (u - x) : x - (u - 1.0), u);
    hu = hu0 & 0x000fffff;
    const bool up = hu >= 0x6a09e;
    const uint64_t lo = as_u64(u) & 0xffffffffull;
    f = as_double(((uint64_t)(uint32_t)(hu | (up ? 0x3fe00000 : 0x3ff00000)) << 32) | lo) - 1.0;
    k = up ? k + 1 : k;
    hu = up ? (0x00100000 - hu) >> 2 : hu;
  }
  const double hfsq = 0.5 * f * f;
  const double s = div_rn(f, 2.0 + f);
  const double z = s * s;
  const double R1 = z * Lp1, z2 = z * z;
  const double R2 = Lp2 + z * Lp3, z4 = z2 * z2;
  const double R3 = Lp4 + z * Lp5, z6 = z4 * z2;
  const double R4 = Lp6 + z * Lp7;
  const double R = R1 + z2 * R2 + z4 * R3 + z6 * R4;
  double r;
  if (k == 0) r = f - (hfsq - s * (hfsq + R));
  else r = k * ln2_hi - ((hfsq - (s * (hfsq + R) + (k * ln2_lo + c))) - f);
  if (hu == 0) {  // |f| < 2^-20 (x = 1 here)
    if (f == 0.0) {
      r = k == 0 ? 0.0 : k * ln2_hi + (c + k * ln2_lo);
    } else {
      const double Rs = hfsq * (1.0 - 0.66666666666666666 * f);
      r = k == 0 ? f - Rs : k * ln2_hi - ((Rs - (k * ln2_lo + c)) - f);
    }
  }
  if (hx < 0x3e200000) r = hx < 0x3c900000 ? x : x - x * x * 0.5;  // |x| < 2^-29
  return r;
}

// numpy's npy_logaddexp (npymath, float64): glibc exp and log1p; the two
// branches on the sign of x - y select their operands instead (one exp and
// one log1p per lane, not one of each per branch taken in the wave)
template <class TB = ConstTabs>
NEMO_RM double logaddexp(double x, double y, const TB& tb = TB{}) {
  NEMO_RM_NOCONTRACT
  constexpr double kLogE2 = 0.693147180559945309417232121458176568;
  const double tmp = x - y;
  const bool pos = tmp > 0;
  const double m = pos ? x : y;
  const double a = pos ? -tmp : tmp;   // -|x - y|
  double r = m + log1p_unit(glibc_exp(a, tb));
  if (tmp != tmp) r = tmp;
  if (x == y) r = x + kLogE2;
  return r;
}

// ---------------------------------------------------------------------------
// numpy np.log (float64, contiguous) = __svml_log8_ha: x = 2^k m, m in [1, 2)
// (vgetmantpd / vgetexppd); r = RNE_{1/32}(vrcp14pd(m)) (kRcp14Switch); R =
// fma(r, m, -1); log x = k ln2 + T(r) + p(R) with k + 1 and T = -log(2 r) for
// r < 0.75, evaluated as below.  For positive normal x (the path's logs:
// arguments 1 + c e and 1 - w + w e^T).
// ---------------------------------------------------------------------------
constexpr double kSvmlLn2Hi = 0x1.62e42fefa0000p-1, kSvmlLn2Lo = 0x1.cf79abc9e0000p-40;

// svml_log after its reduction row: m the mantissa in [1, 2), r the row's
// reduction point, H = fma(k, ln2_hi, T_hi) and L = fma(ln2_lo, k, T_lo) with
// k the adjusted exponent -- each operation as the kernel does it (a caller
// whose two arguments share a row and exponent computes H and L once)
NEMO_RM double svml_log_core(double m, double r, double H, double L) {
  NEMO_RM_NOCONTRACT
  constexpr double C180 = 0x1.c81cd309d7c70p-4, C1c0 = -0x1.007357e93af62p-3;
  constexpr double C200 = 0x1.249229cee81efp-3, C240 = -0x1.55553fb28db06p-3;
  constexpr double C280 = 0x1.9999999cc9f5cp-3, C2c0 = -0x1.00000000c05bdp-2;
  constexpr double C300 = 0x1.5555555555466p-2, C340 = -0x1.fffffffffffc6p-2;
  const double R = fma_(r, m, -1.0);
  double p7 = fma_(R, C200, C240);
  double p1 = fma_(R, C180, C1c0);
  const double R2 = R * R;
  double p9 = fma_(R, C280, C2c0);
  const double p8 = fma_(R, C300, C340);
  p1 = fma_(R2, p1, p7);
  const double R4 = R2 * R2;
  p9 = fma_(R2, p9, p8);
  const double P = fma_(R4, p1, p9);
  const double S = H + R;
  const double D = S - H;
  const double E = R - D;
  const double Q = fma_(R2, P, E);
  return S + (Q + L);
}

NEMO_RM double svml_mant(uint64_t b) { return as_double((b & 0x000fffffffffffffull) | 0x3ff0000000000000ull); }

template <class TB = ConstTabs>
NEMO_RM double svml_log(double x, const TB& tb = TB{}) {
  NEMO_RM_NOCONTRACT
  const uint64_t b = as_u64(x);
  const double m = svml_mant(b);
  const uint32_t p22 = (uint32_t)(b >> 30) & 0x3fffff;
  double r, kadj, thi, tlo;
  tb.log_row(p22, r, kadj, thi, tlo);
  const double k = (double)(int)((b >> 52) & 0x7ff) + kadj;   // e - 1023, + 1 when r < 0.75
  return svml_log_core(m, r, fma_(k, kSvmlLn2Hi, thi), fma_(kSvmlLn2Lo, k, tlo));
}

// ---------------------------------------------------------------------------
// numpy np.exp (float64, contiguous) = __svml_exp8_ha: t = RZ(x log2e + S)
// (the one fused multiply-add rounded toward zero, restated from a
// round-to-nearest fma and the sign of its residual), kf = t - S on a 1/16
// grid, j its fraction, r = x - kf ln2 (two fused steps), degree-6
// polynomial, 2^(j/16) (1 + p) scaled by 2^floor(kf).  |x| < 707.70 (the
// library's fast path); below -707.70 the library's rare path gives a tiny
// or zero result, here 0 (the path's only np.exp of such arguments are
// order weights exp(cell - cs) of negligible rows, whose c = a / b then
// enters log(c e + 1) as 1 + tiny = 1 either way).
// ---------------------------------------------------------------------------
template <class TB = ConstTabs>
NEMO_RM double svml_exp(double x, const TB& tb = TB{}) {
  NEMO_RM_NOCONTRACT
  constexpr double kLog2e = 0x1.71547652b82fep+0;
  constexpr double kS = 0x1.8000000003ff0p+48;
  constexpr double kLn2Hi = 0x1.62e42fefa39efp-1, kLn2Lo = 0x1.abc9e3b39803fp-56;
  constexpr double C240 = 0x1.7411836940c04p-10, C280 = 0x1.1101cbbc265c0p-7;
  constexpr double C2c0 = 0x1.55557242d68fep-5, C300 = 0x1.5555553939732p-3;
  constexpr double C340 = 0x1.000000000d008p-1, C380 = 0x1.fffffffffff70p-1;
  if (!(__builtin_fabs(x) < 0x1.61da04cbafe44p+9)) {
    if (x != x) return x;
    return x > 0 ? __builtin_inf() : 0.0;
  }
  // RZ(x log2e + S): the exact sum is positive, so RZ = round down
  double t = fma_(x, kLog2e, kS);
  {
    const double ph = x * kLog2e;
    const double pl = fma_(x, kLog2e, -ph);  // exact low part of the product
    const double s = (kS - t) + ph;          // exact: |kS - t| and |ph| agree within 1/32
    const bool below = s != 0.0 ? s < 0.0 : pl < 0.0;  // exact sum < t: t was rounded up
    if (below) t = as_double(as_u64(t) - 1);
  }
  const double kf = t - kS;
  const int j = (int)(as_u64(t) & 15);
  const double r = fma_(-kf, kLn2Lo, fma_(-kf, kLn2Hi, x));
  const double r2 = r * r;
  double p12 = fma_(r, C240, C280);
  const double p9 = fma_(r, C2c0, C300);
  const double p11 = fma_(r, C340, C380);
  p12 = fma_(r2, p12, p9);
  p12 = fma_(r2, p12, p11);
  double thi, tlo;
  tb.exp_row(j, thi, tlo);
  const double q = fma_(p12, r, tlo);
  const double y = fma_(thi, q, thi);
  const double kfl = __builtin_floor(kf);
  return __builtin_ldexp(y, (int)kfl);
}

}  // namespace refmath
}  // namespace nemo
