/*
 * combine_ops.h - element semantics of the UCG combine on CDNA4.
 *
 * One functor per (element type, op) giving dst' = src (op) dst exactly as
 * the reduce_cb_f contract computes it (api/ucg.h:149-150 as called from
 * builtin/ops/builtin_comp_step.inl:96-102; arithmetic pinned against MPICH
 * 3.3.2 by tests/golden). Everything is done on raw bits where the hardware's
 * own NaN choice could differ from the host MPI library's:
 *   NaN result -> dst NaN ? quiet(dst) : src NaN ? quiet(src) : default NaN.
 * Non-NaN results are single IEEE ops (v_add/v_mul, RNE, denormals kept:
 * the kernels are built without fast-math or denormal flushing).
 */
#ifndef UCG_COMBINE_OPS_H_
#define UCG_COMBINE_OPS_H_

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "ucg_builtin_dev.h"

namespace ucgdev {

typedef uint16_t f16_bits;   /* IEEE binary16 storage */
typedef uint16_t bf16_bits;  /* bfloat16 storage      */

/* Distinct storage tags so fp16 and bf16 get different functors. */
struct f16_t  { uint16_t b; };
struct bf16_t { uint16_t b; };

__device__ __forceinline__ bool isnan32(float x) { return x != x; }
__device__ __forceinline__ bool isnan64(double x) { return x != x; }

/* ---- fp32 / fp64 arithmetic with the host NaN identity ------------------ */
__device__ __forceinline__ float fix32(float s, float d, float r)
{
    if (__builtin_expect(isnan32(r), 0)) {
        uint32_t rb = 0xffc00000u;
        rb = isnan32(s) ? (__float_as_uint(s) | 0x00400000u) : rb;
        rb = isnan32(d) ? (__float_as_uint(d) | 0x00400000u) : rb;
        return __uint_as_float(rb);
    }
    return r;
}

__device__ __forceinline__ double fix64(double s, double d, double r)
{
    if (__builtin_expect(isnan64(r), 0)) {
        uint64_t rb = 0xfff8000000000000ull;
        rb = isnan64(s) ? ((uint64_t)__double_as_longlong(s) | 0x0008000000000000ull) : rb;
        rb = isnan64(d) ? ((uint64_t)__double_as_longlong(d) | 0x0008000000000000ull) : rb;
        return __longlong_as_double((long long)rb);
    }
    return r;
}

/* ---- fp16 / bf16 <-> fp32 ---------------------------------------------- */
__device__ __forceinline__ float h2f(uint16_t h)
{
    return (float)__builtin_bit_cast(_Float16, h);   /* exact */
}
__device__ __forceinline__ uint16_t f2h_rne(float f)
{
    return __builtin_bit_cast(uint16_t, (_Float16)f); /* v_cvt_f16_f32, RNE */
}
__device__ __forceinline__ float b2f(uint16_t h)
{
    return __uint_as_float((uint32_t)h << 16);
}
__device__ __forceinline__ uint16_t f2b_rne(float f)   /* f is not NaN */
{
    uint32_t x = __float_as_uint(f);
    return (uint16_t)((x + 0x7fffu + ((x >> 16) & 1u)) >> 16);
}

/* NaN identity for 16-bit floats, decided on the original bits */
__device__ __forceinline__ uint16_t nan16(uint16_t s, uint16_t d, bool s_nan,
                                          bool d_nan, uint16_t quiet,
                                          uint16_t dflt)
{
    uint16_t r = dflt;
    r = s_nan ? (uint16_t)(s | quiet) : r;
    r = d_nan ? (uint16_t)(d | quiet) : r;
    return r;
}

/* ------------------------------------------------------------------------ */
/* functors                                                                 */
/* ------------------------------------------------------------------------ */
template <typename T, int OP> struct Comb;

/* integers: wrap through the unsigned type of the same width */
template <typename T> struct UnsignedOf;
template <> struct UnsignedOf<int8_t>   { typedef uint8_t  U; typedef uint32_t W; };
template <> struct UnsignedOf<uint8_t>  { typedef uint8_t  U; typedef uint32_t W; };
template <> struct UnsignedOf<int16_t>  { typedef uint16_t U; typedef uint32_t W; };
template <> struct UnsignedOf<uint16_t> { typedef uint16_t U; typedef uint32_t W; };
template <> struct UnsignedOf<int32_t>  { typedef uint32_t U; typedef uint32_t W; };
template <> struct UnsignedOf<uint32_t> { typedef uint32_t U; typedef uint32_t W; };
template <> struct UnsignedOf<int64_t>  { typedef uint64_t U; typedef uint64_t W; };
template <> struct UnsignedOf<uint64_t> { typedef uint64_t U; typedef uint64_t W; };

template <typename T, int OP> struct CombInt {
    typedef typename UnsignedOf<T>::U U;
    typedef typename UnsignedOf<T>::W W;
    __device__ __forceinline__ static T apply(T s, T d)
    {
        switch (OP) {
        case UCG_DEV_OP_SUM:  return (T)(U)((W)(U)s + (W)(U)d);
        case UCG_DEV_OP_PROD: return (T)(U)((W)(U)s * (W)(U)d);
        case UCG_DEV_OP_MAX:  return (d > s) ? d : s;
        case UCG_DEV_OP_MIN:  return (d < s) ? d : s;
        case UCG_DEV_OP_LAND: return (T)(s && d);
        case UCG_DEV_OP_LOR:  return (T)(s || d);
        case UCG_DEV_OP_LXOR: return (T)((!s) != (!d));
        case UCG_DEV_OP_BAND: return (T)(s & d);
        case UCG_DEV_OP_BOR:  return (T)(s | d);
        default:              return (T)(s ^ d);
        }
    }
};

#define UCGDEV_INT_COMB(_T) \
    template <int OP> struct Comb<_T, OP> : CombInt<_T, OP> {};
UCGDEV_INT_COMB(int8_t)
UCGDEV_INT_COMB(uint8_t)
UCGDEV_INT_COMB(int16_t)
UCGDEV_INT_COMB(uint16_t)
UCGDEV_INT_COMB(int32_t)
UCGDEV_INT_COMB(uint32_t)
UCGDEV_INT_COMB(int64_t)
UCGDEV_INT_COMB(uint64_t)

template <int OP> struct Comb<float, OP> {
    __device__ __forceinline__ static float apply(float s, float d)
    {
        switch (OP) {
        case UCG_DEV_OP_SUM:  return fix32(s, d, s + d);
        case UCG_DEV_OP_PROD: return fix32(s, d, s * d);
        case UCG_DEV_OP_MAX:  return (d > s) ? d : s;
        default:              return (d < s) ? d : s;
        }
    }
};

template <int OP> struct Comb<double, OP> {
    __device__ __forceinline__ static double apply(double s, double d)
    {
        switch (OP) {
        case UCG_DEV_OP_SUM:  return fix64(s, d, s + d);
        case UCG_DEV_OP_PROD: return fix64(s, d, s * d);
        case UCG_DEV_OP_MAX:  return (d > s) ? d : s;
        default:              return (d < s) ? d : s;
        }
    }
};

template <int OP> struct Comb<f16_t, OP> {
    __device__ __forceinline__ static f16_t apply(f16_t s, f16_t d)
    {
        const float a = h2f(s.b), b = h2f(d.b);
        f16_t o;
        if (OP == UCG_DEV_OP_MAX) {
            o.b = (b > a) ? d.b : s.b;
            return o;
        }
        if (OP == UCG_DEV_OP_MIN) {
            o.b = (b < a) ? d.b : s.b;
            return o;
        }
        float r = (OP == UCG_DEV_OP_SUM) ? (a + b) : (a * b);
        /* keep the fp32 result in a register: without this barrier hipcc
         * (ROCm 7.2) folds fptrunc(fmul(fpext a, fpext b)) into
         * v_fma_mixlo_f16 a, b, +0, i.e. fma(a, b, +0), which turns an exact
         * -0 product into +0 (caught by tests/golden: (+0) x (-0)) */
        __asm__ volatile("" : "+v"(r));
        if (__builtin_expect(isnan32(r), 0)) {
            o.b = nan16(s.b, d.b, isnan32(a), isnan32(b), 0x0200u, 0xfe00u);
        } else {
            o.b = f2h_rne(r);
        }
        return o;
    }
};

template <int OP> struct Comb<bf16_t, OP> {
    __device__ __forceinline__ static bf16_t apply(bf16_t s, bf16_t d)
    {
        const float a = b2f(s.b), b = b2f(d.b);
        bf16_t o;
        if (OP == UCG_DEV_OP_MAX) {
            o.b = (b > a) ? d.b : s.b;
            return o;
        }
        if (OP == UCG_DEV_OP_MIN) {
            o.b = (b < a) ? d.b : s.b;
            return o;
        }
        const float r = (OP == UCG_DEV_OP_SUM) ? (a + b) : (a * b);
        if (__builtin_expect(isnan32(r), 0)) {
            o.b = nan16(s.b, d.b, isnan32(a), isnan32(b), 0x0040u, 0xffc0u);
        } else {
            o.b = f2b_rne(r);
        }
        return o;
    }
};

/* storage type of a ucg_dev_dtype_t */
template <int DT> struct DtType;
template <> struct DtType<UCG_DEV_DT_INT8>     { typedef int8_t   T; };
template <> struct DtType<UCG_DEV_DT_UINT8>    { typedef uint8_t  T; };
template <> struct DtType<UCG_DEV_DT_INT16>    { typedef int16_t  T; };
template <> struct DtType<UCG_DEV_DT_UINT16>   { typedef uint16_t T; };
template <> struct DtType<UCG_DEV_DT_INT32>    { typedef int32_t  T; };
template <> struct DtType<UCG_DEV_DT_UINT32>   { typedef uint32_t T; };
template <> struct DtType<UCG_DEV_DT_INT64>    { typedef int64_t  T; };
template <> struct DtType<UCG_DEV_DT_UINT64>   { typedef uint64_t T; };
template <> struct DtType<UCG_DEV_DT_FLOAT16>  { typedef f16_t    T; };
template <> struct DtType<UCG_DEV_DT_BFLOAT16> { typedef bf16_t   T; };
template <> struct DtType<UCG_DEV_DT_FLOAT32>  { typedef float    T; };
template <> struct DtType<UCG_DEV_DT_FLOAT64>  { typedef double   T; };

constexpr bool dt_is_float(int dt)
{
    return dt == UCG_DEV_DT_FLOAT16 || dt == UCG_DEV_DT_BFLOAT16 ||
           dt == UCG_DEV_DT_FLOAT32 || dt == UCG_DEV_DT_FLOAT64;
}

constexpr bool pair_supported(int dt, int op)
{
    return !(dt_is_float(dt) && op > UCG_DEV_OP_MIN);
}

} /* namespace ucgdev */

#endif
