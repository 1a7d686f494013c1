/*
 * ptmi_math.h — the arithmetic contract shared by the HIP kernels and the CPU
 * oracle (plain C).
 *
 * The reference evaluates transcendental functions with whatever Taichi's
 * backend lowers ti.sin/ti.cos/ti.log/ti.acos/ti.atan2/ti.pow to
 * (src/render_server/taichi_renderer/kernels.py:51-55, 96-97, 441, 786, 1013),
 * which is backend dependent and not reproducible here. This
 * header *defines* them once, using only IEEE-754 operations that are
 * correctly rounded on both gfx950 and x86-64 (+ - * /, sqrtf, fmaf, floorf,
 * rintf), so the CPU oracle and the GPU produce bit-identical results:
 *   - compile both sides with -ffp-contract=off (no implicit FMA),
 *   - HIP with correctly rounded f32 division / sqrt (the hipcc default,
 *     passed explicitly: -fhip-fp32-correctly-rounded-divide-sqrt),
 *   - explicit fmaf() only where written here.
 * Polynomials are the classic Cephes single-precision minimax sets
 * (sinf/cosf, logf, atanf, asinf), accurate to ~1-2 ulp on their ranges.
 *
 * Valid in C99 (gcc, oracle) and HIP C++ (hipcc, device + host).
 */
#ifndef PTMI_MATH_H
#define PTMI_MATH_H

#include <stdint.h>
#include <math.h>

#if defined(__HIPCC__) || defined(__HIP__)
#define PT_HD __host__ __device__ __forceinline__
#else
#define PT_HD static inline
#endif

#define PT_PI_F 3.14159265358979323846f
#define PT_PIO2_F 1.57079632679489661923f
#define PT_PIO4_F 0.78539816339744830962f
#define PT_2PI_F 6.28318530717958647692f

typedef struct pt_v3 { float x, y, z; } pt_v3;

PT_HD pt_v3 pt_v3f(float x, float y, float z) { pt_v3 r; r.x = x; r.y = y; r.z = z; return r; }
PT_HD pt_v3 pt_add(pt_v3 a, pt_v3 b) { return pt_v3f(a.x + b.x, a.y + b.y, a.z + b.z); }
PT_HD pt_v3 pt_sub(pt_v3 a, pt_v3 b) { return pt_v3f(a.x - b.x, a.y - b.y, a.z - b.z); }
PT_HD pt_v3 pt_mul(pt_v3 a, pt_v3 b) { return pt_v3f(a.x * b.x, a.y * b.y, a.z * b.z); }
PT_HD pt_v3 pt_scale(pt_v3 a, float s) { return pt_v3f(a.x * s, a.y * s, a.z * s); }
PT_HD pt_v3 pt_divs(pt_v3 a, float s) { return pt_v3f(a.x / s, a.y / s, a.z / s); }
PT_HD pt_v3 pt_neg(pt_v3 a) { return pt_v3f(-a.x, -a.y, -a.z); }
/* dot = (x + y) + z, left to right (Taichi's Matrix.dot is a sum over a*b). */
PT_HD float pt_dot(pt_v3 a, pt_v3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
PT_HD pt_v3 pt_cross(pt_v3 a, pt_v3 b) {
    return pt_v3f(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
/* Taichi Matrix.normalized(): v * (1 / sqrt(v.dot(v)))  (SURVEY.md Q31). */
PT_HD pt_v3 pt_normalize(pt_v3 a) { float inv = 1.0f / sqrtf(pt_dot(a, a)); return pt_scale(a, inv); }

/* ti.min / ti.max. Default: IEEE-754 minNum/maxNum (fminf/fmaxf: a NaN
 * operand yields the other operand), which gfx950 executes as one
 * v_min/v_max(3)_f32 and glibc implements identically; PTMI_SELECT_MINMAX
 * selects the compare-and-select form instead. The integrator never feeds
 * these a signed-zero pair whose sign reaches arithmetic. */
#ifdef PTMI_SELECT_MINMAX
PT_HD float pt_minf(float a, float b) { return (a < b) ? a : b; }
PT_HD float pt_maxf(float a, float b) { return (a > b) ? a : b; }
#else
PT_HD float pt_minf(float a, float b) { return fminf(a, b); }
PT_HD float pt_maxf(float a, float b) { return fmaxf(a, b); }
#endif

PT_HD uint32_t pt_f2u_bits(float x) { union { float f; uint32_t u; } c; c.f = x; return c.u; }
PT_HD float pt_u2f_bits(uint32_t u) { union { float f; uint32_t u; } c; c.u = u; return c.f; }

/* ti.cast(x, ti.i32): truncation; saturating, NaN -> 0 (the gfx950
 * v_cvt_i32_f32 behaviour, made explicit so x86 agrees). */
PT_HD int32_t pt_f2i(float x) {
    if (!(x == x)) return 0;
    if (x >= 2147483648.0f) return 2147483647;
    if (x <= -2147483648.0f) return (int32_t)(-2147483647 - 1);
    return (int32_t)x;
}

/* sin and cos of x (|x| up to ~1e5 at ~1 ulp): 3-part Cody-Waite reduction by
 * pi/2 with fmaf, then Cephes sinf/cosf kernels on [-pi/4, pi/4]. */
PT_HD void pt_sincosf(float x, float *s_out, float *c_out) {
    float k = rintf(x * 0.636619772367581343f);
    float r = fmaf(-k, 1.57079637050628662109375f, x);
    r = fmaf(-k, -4.37113882867379289e-8f, r);
    r = fmaf(-k, -1.71512451000593173e-15f, r);
    float z = r * r;
    float ps = fmaf(fmaf(-1.9515295891e-4f, z, 8.3321608736e-3f), z, -1.6666654611e-1f);
    float s = fmaf(ps * z, r, r);
    float pc = fmaf(fmaf(2.443315711809948e-5f, z, -1.388731625493765e-3f), z, 4.166664568298827e-2f);
    float c = fmaf(pc * z, z, fmaf(-0.5f, z, 1.0f));
    int32_t q = pt_f2i(k) & 3;
    float so, co;
    if (q == 0) { so = s; co = c; }
    else if (q == 1) { so = c; co = -s; }
    else if (q == 2) { so = -s; co = -c; }
    else { so = -c; co = s; }
    *s_out = so;
    *c_out = co;
}
PT_HD float pt_sinf(float x) { float s, c; pt_sincosf(x, &s, &c); return s; }
PT_HD float pt_cosf(float x) { float s, c; pt_sincosf(x, &s, &c); return c; }

/* Natural log for positive normal x (Cephes logf). x <= 0 -> NaN/-inf paths
 * are never taken by the integrator (kernels.py:441 clamps to >= 1e-10). */
PT_HD float pt_logf(float x) {
    if (!(x > 0.0f)) return (x == 0.0f) ? -INFINITY : NAN;
    uint32_t b = pt_f2u_bits(x);
    int32_t e = (int32_t)((b >> 23) & 0xffu);
    if (e == 0) { /* subnormal: scale up by 2^25 */
        x = x * 33554432.0f;
        b = pt_f2u_bits(x);
        e = (int32_t)((b >> 23) & 0xffu) - 25;
    }
    e -= 126;
    float m = pt_u2f_bits((b & 0x007fffffu) | 0x3f000000u); /* [0.5, 1) */
    if (m < 0.707106781186547524f) { e -= 1; m = m + m - 1.0f; }
    else { m = m - 1.0f; }
    float z = m * m;
    float y = 7.0376836292e-2f;
    y = fmaf(y, m, -1.1514610310e-1f);
    y = fmaf(y, m, 1.1676998740e-1f);
    y = fmaf(y, m, -1.2420140846e-1f);
    y = fmaf(y, m, 1.4249322787e-1f);
    y = fmaf(y, m, -1.6668057665e-1f);
    y = fmaf(y, m, 2.0000714765e-1f);
    y = fmaf(y, m, -2.4999993993e-1f);
    y = fmaf(y, m, 3.3333331174e-1f);
    y = y * m * z;
    float fe = (float)e;
    y = fmaf(fe, -2.12194440e-4f, y);
    y = fmaf(-0.5f, z, y);
    float r = m + y;
    r = fmaf(fe, 0.693359375f, r);
    return r;
}

/* atan on |x| (Cephes atanf), sign restored by caller. */
PT_HD float pt_atan_pos(float x) {
    float y0, t;
    if (x > 2.414213562373095f) { y0 = PT_PIO2_F; t = -1.0f / x; }
    else if (x > 0.4142135623730950f) { y0 = PT_PIO4_F; t = (x - 1.0f) / (x + 1.0f); }
    else { y0 = 0.0f; t = x; }
    float z = t * t;
    float p = fmaf(fmaf(fmaf(8.05374449538e-2f, z, -1.38776856032e-1f), z, 1.99777106478e-1f), z,
                   -3.33329491539e-1f);
    return y0 + fmaf(p * z, t, t);
}
PT_HD float pt_atanf(float x) {
    uint32_t sb = pt_f2u_bits(x) & 0x80000000u;
    float a = pt_atan_pos(pt_u2f_bits(pt_f2u_bits(x) & 0x7fffffffu));
    return pt_u2f_bits(pt_f2u_bits(a) ^ sb);  /* odd, incl. signed zero */
}
/* atan2 with IEEE signed-zero conventions for the y = +-0 cases. */
PT_HD float pt_atan2f(float y, float x) {
    uint32_t ysign = pt_f2u_bits(y) >> 31;
    uint32_t xsign = pt_f2u_bits(x) >> 31;
    if (x == 0.0f) {
        if (y == 0.0f) {
            float r = xsign ? PT_PI_F : 0.0f;
            return ysign ? -r : r;
        }
        return ysign ? -PT_PIO2_F : PT_PIO2_F;
    }
    float a = pt_atanf(y / x);
    if (!xsign) return a;
    return ysign ? a - PT_PI_F : a + PT_PI_F;
}

/* asin core for |x| <= 0.5 (Cephes asinf polynomial). */
PT_HD float pt_asin_core(float x) {
    float z = x * x;
    float p = fmaf(fmaf(fmaf(fmaf(4.2163199048e-2f, z, 2.4181311049e-2f), z, 4.5470025998e-2f), z,
                        7.4953002686e-2f), z, 1.6666752422e-1f);
    return fmaf(p * z, x, x);
}
PT_HD float pt_acosf(float x) {
    if (x < -0.5f) return PT_PI_F - 2.0f * pt_asin_core(sqrtf(0.5f * (1.0f + x)));
    if (x > 0.5f) return 2.0f * pt_asin_core(sqrtf(0.5f * (1.0f - x)));
    return PT_PIO2_F - pt_asin_core(x);
}

/* ti.pow(x, 5.0) in Schlick's reflectance (kernels.py:786), defined as
 * ((x*x)*(x*x))*x. */
PT_HD float pt_pow5f(float x) { float x2 = x * x; return (x2 * x2) * x; }

/* Correctly rounded x / a through a reciprocal of a shared by many quotients
 * (the HIP sphere test divides both roots by the per-ray a = dot(d, d)); the
 * oracle itself always writes x / a. pt_recip_for_div(a) is RN(1/a), or NaN
 * when a is outside [2^-50, 2^50]. In pt_div_by, q = RN(x * ra) is within one
 * ulp of x/a, the remainder x - a*q is exact in one fma, and RN(q + rem * ra)
 * is RN(x/a) (Markstein's theorem) unless something under- or overflows.
 * With a and q in [2^-50, 2^50] nothing does: the remainder is a multiple of
 * 2^(e_a + e_q - 46) >= 2^-146 of at most 24 significant bits, so it is
 * exactly representable. Any other quotient (and NaN) takes the plain
 * division. tests/test_contract.py checks pt_div_by == x / a bit for bit. */
PT_HD float pt_recip_for_div(float a) {
    return (a >= 0x1p-50f && a <= 0x1p50f) ? 1.0f / a : __builtin_nanf("");
}
PT_HD float pt_div_by(float x, float a, float ra) {
    const float q = x * ra;
    float r = fmaf(fmaf(-a, q, x), ra, q);
    const float aq = fabsf(q);
    if (__builtin_expect(!(aq >= 0x1p-50f && aq <= 0x1p50f), 0)) r = x / a;
    return r;
}

#endif /* PTMI_MATH_H */
