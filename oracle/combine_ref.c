/*
 * combine_ref.c - CPU ORACLE (test infrastructure only; see combine_ref.h).
 *
 * Plain C restatement of the reduce_cb_f contract as UCG's builtin planner
 * uses it (builtin/ops/builtin_comp_step.inl:96-120) with the arithmetic of
 * the host MPI library's local reduce (MPI_Reduce_local semantics, pinned by
 * MPICH 3.3.2 golden vectors in tests/golden). The floating-point NaN rule is
 * written out explicitly so that the result does not depend on which operand
 * order gcc picks for `s + d`:
 *   dst NaN -> quiet(dst); else src NaN -> quiet(src); else invalid -> the
 *   default NaN (sign and quiet bit set)    [x86 SSE with dst as operand 1,
 *   observed from MPICH: see tests/golden/README.md].
 */
#include "combine_ref.h"

#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

/* ------------------------------------------------------------------------ */
/* bit helpers                                                              */
/* ------------------------------------------------------------------------ */
static inline uint32_t f2u(float f)    { uint32_t u; memcpy(&u, &f, 4); return u; }
static inline float    u2f(uint32_t u) { float f;    memcpy(&f, &u, 4); return f; }
static inline uint64_t d2u(double f)   { uint64_t u; memcpy(&u, &f, 8); return u; }
static inline double   u2d(uint64_t u) { double f;   memcpy(&f, &u, 8); return f; }

static const size_t ora_sizes[ORA_DT_LAST] = {1, 1, 2, 2, 4, 4, 8, 8, 2, 2, 4, 8};

size_t ucg_oracle_dtype_size(int dt)
{
    return (dt >= 0 && dt < ORA_DT_LAST) ? ora_sizes[dt] : 0;
}

static int is_float_dt(int dt)
{
    return dt == ORA_F16 || dt == ORA_BF16 || dt == ORA_F32 || dt == ORA_F64;
}

int ucg_oracle_is_supported(int dt, int op)
{
    if (dt < 0 || dt >= ORA_DT_LAST || op < 0 || op >= ORA_OP_LAST) {
        return 0;
    }
    /* MPI: logical and bitwise ops are defined for integer types only */
    return !(is_float_dt(dt) && op > ORA_MIN);
}

/* ------------------------------------------------------------------------ */
/* fp16 / bf16 conversions                                                  */
/* ------------------------------------------------------------------------ */
float ucg_oracle_half_to_float(uint16_t h)
{
    uint32_t sign = (uint32_t)(h & 0x8000u) << 16;
    uint32_t exp  = (h >> 10) & 0x1f;
    uint32_t mant = h & 0x3ffu;
    if (exp == 0x1f) {                       /* inf / NaN: keep payload bits */
        return u2f(sign | 0x7f800000u | (mant << 13));
    }
    if (exp == 0) {
        if (mant == 0) {
            return u2f(sign);
        }
        /* subnormal: normalise */
        int e = -1;
        do {
            e++;
            mant <<= 1;
        } while ((mant & 0x400u) == 0);
        mant &= 0x3ffu;
        return u2f(sign | ((uint32_t)(127 - 15 - e) << 23) | (mant << 13));
    }
    return u2f(sign | ((exp + 127 - 15) << 23) | (mant << 13));
}

/* IEEE round-to-nearest-even; NaN keeps the top payload bits (numpy's rule:
 * a payload that truncates to zero becomes 1 so that a NaN stays a NaN). */
uint16_t ucg_oracle_float_to_half(float f)
{
    uint32_t x    = f2u(f);
    uint16_t sign = (uint16_t)((x >> 16) & 0x8000u);
    uint32_t ax   = x & 0x7fffffffu;

    if (ax > 0x7f800000u) {
        uint16_t r = (uint16_t)(0x7c00u | ((ax & 0x7fffffu) >> 13));
        if (r == 0x7c00u) {
            r++;
        }
        return sign | r;
    }
    if (ax >= 0x477ff000u) {                 /* >= 65520 rounds to inf */
        return sign | 0x7c00u;
    }
    if (ax >= 0x38800000u) {                 /* normal half */
        uint32_t h   = (((ax >> 23) - 112u) << 10) | ((ax & 0x7fffffu) >> 13);
        uint32_t rem = ax & 0x1fffu;
        if (rem > 0x1000u || (rem == 0x1000u && (h & 1u))) {
            h++;
        }
        return sign | (uint16_t)h;
    }
    uint32_t e = ax >> 23;
    if (e < 102) {                           /* < 2^-25 (or tie) -> 0 */
        return sign;
    }
    uint32_t mant  = (ax & 0x7fffffu) | 0x800000u;
    uint32_t shift = 126u - e;               /* 14 .. 24 */
    uint32_t h     = mant >> shift;
    uint32_t rem   = mant & ((1u << shift) - 1u);
    uint32_t half  = 1u << (shift - 1u);
    if (rem > half || (rem == half && (h & 1u))) {
        h++;
    }
    return sign | (uint16_t)h;
}

float ucg_oracle_bf16_to_float(uint16_t h)
{
    return u2f((uint32_t)h << 16);
}

uint16_t ucg_oracle_float_to_bf16(float f)
{
    uint32_t x = f2u(f);
    if ((x & 0x7fffffffu) > 0x7f800000u) {   /* NaN: truncate (quiet input) */
        uint16_t r = (uint16_t)(x >> 16);
        if ((r & 0x7fu) == 0) {
            r |= 0x40u;
        }
        return r;
    }
    return (uint16_t)((x + 0x7fffu + ((x >> 16) & 1u)) >> 16);
}

/* ------------------------------------------------------------------------ */
/* floating-point elementwise rules                                         */
/* ------------------------------------------------------------------------ */
static inline float f32_arith(float s, float d, float r)
{
    /* r = s (op) d as computed by IEEE hardware; fix up NaN identity */
    uint32_t rb = f2u(r);
    rb = (r != r) ? 0xffc00000u : rb;
    rb = (s != s) ? (f2u(s) | 0x00400000u) : rb;
    rb = (d != d) ? (f2u(d) | 0x00400000u) : rb;
    return u2f(rb);
}

static inline double f64_arith(double s, double d, double r)
{
    uint64_t rb = d2u(r);
    rb = (r != r) ? 0xfff8000000000000ull : rb;
    rb = (s != s) ? (d2u(s) | 0x0008000000000000ull) : rb;
    rb = (d != d) ? (d2u(d) | 0x0008000000000000ull) : rb;
    return u2d(rb);
}

#define ORA_FLOAT_LOOP(_T, _ARITH, _expr_sum, _expr_prod)                     \
    do {                                                                      \
        const _T *s = (const _T*)src;                                         \
        _T *d       = (_T*)dst;                                               \
        size_t i;                                                             \
        switch (op) {                                                         \
        case ORA_SUM:                                                         \
            for (i = 0; i < count; i++) {                                     \
                d[i] = _ARITH(s[i], d[i], _expr_sum);                         \
            }                                                                 \
            return 0;                                                         \
        case ORA_PROD:                                                        \
            for (i = 0; i < count; i++) {                                     \
                d[i] = _ARITH(s[i], d[i], _expr_prod);                        \
            }                                                                 \
            return 0;                                                         \
        case ORA_MAX:                                                         \
            for (i = 0; i < count; i++) {                                     \
                d[i] = (d[i] > s[i]) ? d[i] : s[i];                           \
            }                                                                 \
            return 0;                                                         \
        case ORA_MIN:                                                         \
            for (i = 0; i < count; i++) {                                     \
                d[i] = (d[i] < s[i]) ? d[i] : s[i];                           \
            }                                                                 \
            return 0;                                                         \
        default:                                                              \
            return -1;                                                        \
        }                                                                     \
    } while (0)

/* fp16 / bf16: widen exactly, apply the fp32 rule, round once */
static int reduce_f16like(int op, int is_bf16, const uint16_t *s, uint16_t *d,
                          size_t count)
{
    size_t i;
    for (i = 0; i < count; i++) {
        float a = is_bf16 ? ucg_oracle_bf16_to_float(s[i]) :
                            ucg_oracle_half_to_float(s[i]);
        float b = is_bf16 ? ucg_oracle_bf16_to_float(d[i]) :
                            ucg_oracle_half_to_float(d[i]);
        float r;
        switch (op) {
        case ORA_SUM:
            r = f32_arith(a, b, a + b);
            break;
        case ORA_PROD:
            r = f32_arith(a, b, a * b);
            break;
        case ORA_MAX:
            d[i] = (b > a) ? d[i] : s[i];
            continue;
        case ORA_MIN:
            d[i] = (b < a) ? d[i] : s[i];
            continue;
        default:
            return -1;
        }
        d[i] = is_bf16 ? ucg_oracle_float_to_bf16(r) :
                         ucg_oracle_float_to_half(r);
    }
    return 0;
}

/* integer rules: wrap-around via the unsigned type */
#define ORA_INT_LOOP(_T, _U, _W)                                              \
    do {                                                                      \
        const _T *s = (const _T*)src;                                         \
        _T *d       = (_T*)dst;                                               \
        size_t i;                                                             \
        switch (op) {                                                         \
        case ORA_SUM:                                                         \
            for (i = 0; i < count; i++)                                       \
                d[i] = (_T)(_U)((_W)(_U)s[i] + (_W)(_U)d[i]);                 \
            return 0;                                                         \
        case ORA_PROD:                                                        \
            for (i = 0; i < count; i++)                                       \
                d[i] = (_T)(_U)((_W)(_U)s[i] * (_W)(_U)d[i]);                 \
            return 0;                                                         \
        case ORA_MAX:                                                         \
            for (i = 0; i < count; i++) d[i] = (d[i] > s[i]) ? d[i] : s[i];   \
            return 0;                                                         \
        case ORA_MIN:                                                         \
            for (i = 0; i < count; i++) d[i] = (d[i] < s[i]) ? d[i] : s[i];   \
            return 0;                                                         \
        case ORA_LAND:                                                        \
            for (i = 0; i < count; i++) d[i] = (_T)(s[i] && d[i]);            \
            return 0;                                                         \
        case ORA_LOR:                                                         \
            for (i = 0; i < count; i++) d[i] = (_T)(s[i] || d[i]);            \
            return 0;                                                         \
        case ORA_LXOR:                                                        \
            for (i = 0; i < count; i++) d[i] = (_T)((!s[i]) != (!d[i]));      \
            return 0;                                                         \
        case ORA_BAND:                                                        \
            for (i = 0; i < count; i++) d[i] = (_T)(s[i] & d[i]);             \
            return 0;                                                         \
        case ORA_BOR:                                                         \
            for (i = 0; i < count; i++) d[i] = (_T)(s[i] | d[i]);             \
            return 0;                                                         \
        case ORA_BXOR:                                                        \
            for (i = 0; i < count; i++) d[i] = (_T)(s[i] ^ d[i]);             \
            return 0;                                                         \
        default:                                                              \
            return -1;                                                        \
        }                                                                     \
    } while (0)

int ucg_oracle_reduce(int op, int dt, const void *src, void *dst, size_t count)
{
    if (!ucg_oracle_is_supported(dt, op)) {
        return -1;
    }
    switch (dt) {
    case ORA_I8:  ORA_INT_LOOP(int8_t,   uint8_t,  uint32_t);
    case ORA_U8:  ORA_INT_LOOP(uint8_t,  uint8_t,  uint32_t);
    case ORA_I16: ORA_INT_LOOP(int16_t,  uint16_t, uint32_t);
    case ORA_U16: ORA_INT_LOOP(uint16_t, uint16_t, uint32_t);
    case ORA_I32: ORA_INT_LOOP(int32_t,  uint32_t, uint32_t);
    case ORA_U32: ORA_INT_LOOP(uint32_t, uint32_t, uint32_t);
    case ORA_I64: ORA_INT_LOOP(int64_t,  uint64_t, uint64_t);
    case ORA_U64: ORA_INT_LOOP(uint64_t, uint64_t, uint64_t);
    case ORA_F16:
        return reduce_f16like(op, 0, (const uint16_t*)src, (uint16_t*)dst, count);
    case ORA_BF16:
        return reduce_f16like(op, 1, (const uint16_t*)src, (uint16_t*)dst, count);
    case ORA_F32:
        ORA_FLOAT_LOOP(float, f32_arith, s[i] + d[i], s[i] * d[i]);
    case ORA_F64:
        ORA_FLOAT_LOOP(double, f64_arith, s[i] + d[i], s[i] * d[i]);
    default:
        return -1;
    }
}

int ucg_oracle_reduce_fragmented(int op, int dt, const void *src, void *dst,
                                 size_t count, size_t frag_bytes)
{
    size_t sz = ucg_oracle_dtype_size(dt);
    if (sz == 0) {
        return -1;
    }
    size_t per = frag_bytes / sz;
    if (per == 0) {
        return ucg_oracle_reduce(op, dt, src, dst, count);
    }
    size_t done = 0;
    while (done < count) {
        size_t n = (count - done < per) ? (count - done) : per;
        if (ucg_oracle_reduce(op, dt, (const char*)src + done * sz,
                              (char*)dst + done * sz, n)) {
            return -1;
        }
        done += n;
    }
    return 0;
}

/* builtin/plan/builtin_recursive.c:158-169 with factor 2:
 *   step_base = my - (my % (2*step_size)); peer = step_base +
 *   ((my - step_base + step_size) % (2*step_size)), step_size = 2^(step-1) */
uint64_t ucg_oracle_recursive_peer(uint64_t my, unsigned step)
{
    uint64_t step_size = 1ull << (step - 1);
    uint64_t base      = my - (my % (step_size * 2));
    return base + ((my - base + step_size) % (step_size * 2));
}

int ucg_oracle_tree_reduce(int op, int dt, void *dst, const void *const *srcs,
                           unsigned nsrc, unsigned root, const unsigned *order,
                           size_t count)
{
    size_t sz = ucg_oracle_dtype_size(dt);
    unsigned i, k = 0;
    if (sz == 0 || nsrc == 0 || root >= nsrc || !ucg_oracle_is_supported(dt, op)) {
        return -1;
    }
    memcpy(dst, srcs[root], count * sz);           /* init_reduce */
    for (i = 0; i + 1 < nsrc; i++) {
        unsigned child;
        if (order) {
            child = order[i];
        } else {
            child = (k == root) ? ++k : k;   /* ascending, skipping the root */
            k++;
        }
        if (child >= nsrc || child == root) {
            return -1;
        }
        ucg_oracle_reduce(op, dt, srcs[child], dst, count);
    }
    return 0;
}

int ucg_oracle_tree_intra(unsigned my, unsigned size, unsigned root,
                          unsigned *up, unsigned *up_cnt,
                          unsigned *down, unsigned *down_cnt)
{
    unsigned m;
    *up_cnt = *down_cnt = 0;
    if (my >= size || root >= size) {
        return -1;
    }
    /* every other member is one "HOST" distance away: the first member
     * before me at that distance is my parent, and only a member with no
     * parent (master_phase NET) takes children - all members at the first
     * distance it sees. Relabelled so the root plays member 0. */
    if (my != root) {
        up[(*up_cnt)++] = root;
        return 0;
    }
    for (m = 0; m < size; m++) {
        if (m != root) {
            down[(*down_cnt)++] = m;
        }
    }
    return 0;
}

int ucg_oracle_reduce_multi(int op, int dt, void *dst, const void *const *srcs,
                            unsigned nsrc, unsigned self, size_t count)
{
    size_t sz = ucg_oracle_dtype_size(dt);
    unsigned r, step, nsteps = 0;
    if (sz == 0 || nsrc == 0 || (nsrc & (nsrc - 1)) || self >= nsrc ||
        !ucg_oracle_is_supported(dt, op)) {
        return -1;
    }
    while ((1u << nsteps) < nsrc) {
        nsteps++;
    }
    size_t bytes = count * sz;
    char *acc  = malloc(bytes * nsrc + 1);
    char *prev = malloc(bytes * nsrc + 1);
    if (!acc || !prev) {
        free(acc);
        free(prev);
        return -1;
    }
    /* ucg_builtin_init_reduce (builtin_control.c:43-47): recv <- send */
    for (r = 0; r < nsrc; r++) {
        memcpy(acc + r * bytes, srcs[r], bytes);
    }
    for (step = 1; step <= nsteps; step++) {
        /* every member sends its accumulator (the step's send_buffer is the
         * recv_buffer from step 2 on, builtin_control.c:850-857), then
         * combines the incoming one into its own: dst = incoming (op) dst */
        memcpy(prev, acc, bytes * nsrc);
        for (r = 0; r < nsrc; r++) {
            unsigned peer = (unsigned)ucg_oracle_recursive_peer(r, step);
            ucg_oracle_reduce(op, dt, prev + peer * bytes, acc + r * bytes,
                              count);
        }
    }
    memcpy(dst, acc + self * bytes, bytes);
    free(acc);
    free(prev);
    return 0;
}

/* builtin/ops/builtin_control.c:434 and :462 */
size_t ucg_oracle_frag_length(size_t max_short, size_t dt_len)
{
    size_t m = max_short - 8; /* sizeof(ucg_builtin_header_t) */
    return m - (m % dt_len);
}

/* builtin/ops/builtin_control.c:463-465 */
uint64_t ucg_oracle_fragments_total(size_t length, size_t frag_len,
                                    unsigned ep_cnt)
{
    return (uint64_t)ep_cnt * (length / frag_len + ((length % frag_len) > 0));
}

/* ------------------------------------------------------------------------ */
/* synthetic generator                                       */
/* ------------------------------------------------------------------------ */
uint64_t ucg_oracle_splitmix64(uint64_t x)
{
    uint64_t z = x + 0x9e3779b97f4a7c15ull;
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}

static const uint32_t spec_f32[] = {
    0x00000000, 0x80000000, 0x3f800000, 0xbf800000, 0x3fc00000, 0x00000001,
    0x007fffff, 0x00800000, 0x7f7fffff, 0xff7fffff, 0x7f800000, 0xff800000,
    0x7fc00000, 0x7fc12345, 0xffc54321, 0x7f800001, 0xff812345, 0x4b800000,
    0x33800000, 0x3dcccccd, 0x80000001, 0x40400000};
static const uint64_t spec_f64[] = {
    0x0000000000000000ull, 0x8000000000000000ull, 0x3ff0000000000000ull,
    0xbff0000000000000ull, 0x3ff8000000000000ull, 0x0000000000000001ull,
    0x000fffffffffffffull, 0x0010000000000000ull, 0x7fefffffffffffffull,
    0xffefffffffffffffull, 0x7ff0000000000000ull, 0xfff0000000000000ull,
    0x7ff8000000000000ull, 0x7ff8000000012345ull, 0xfff8000000054321ull,
    0x7ff0000000000001ull, 0xfff0000000012345ull, 0x4340000000000000ull,
    0x3ca0000000000000ull, 0x3fb999999999999aull, 0x8000000000000001ull,
    0x4008000000000000ull};
static const uint16_t spec_f16[] = {
    0x0000, 0x8000, 0x3c00, 0xbc00, 0x3e00, 0x0001, 0x03ff, 0x0400, 0x7bff,
    0xfbff, 0x7c00, 0xfc00, 0x7e00, 0x7e45, 0xfe21, 0x7c01, 0xfc23, 0x6800,
    0x1000, 0x2e66, 0x8001, 0x4200};
static const uint16_t spec_bf16[] = {
    0x0000, 0x8000, 0x3f80, 0xbf80, 0x3fc0, 0x0001, 0x007f, 0x0080, 0x7f7f,
    0xff7f, 0x7f80, 0xff80, 0x7fc0, 0x7fc5, 0xffc3, 0x7f81, 0xff85, 0x4380,
    0x3b80, 0x3dcd, 0x8001, 0x4040};
#define SPEC_FLOAT_N (sizeof(spec_f32) / sizeof(spec_f32[0]))
#define SPEC_INT_N   16

static uint64_t spec_int(unsigned bits, unsigned idx)
{
    uint64_t m  = (bits == 64) ? ~0ull : ((1ull << bits) - 1);
    uint64_t mx = m >> 1;
    switch (idx) {
    case 0:  return 0;
    case 1:  return 1;
    case 2:  return m;                          /* -1 */
    case 3:  return 2;
    case 4:  return mx;                         /* signed max */
    case 5:  return mx + 1;                     /* signed min */
    case 6:  return mx - 1;
    case 7:  return mx + 2;                     /* min + 1 */
    case 8:  return 0x5555555555555555ull & m;
    case 9:  return 0xaaaaaaaaaaaaaaaaull & m;
    case 10: return 3;
    case 11: return m - 6;                      /* -7 */
    case 12: return 0x0f0f0f0f0f0f0f0full & m;
    case 13: return 0xf0f0f0f0f0f0f0f0ull & m;
    case 14: return 0x100 & m;
    default: return m - 0xff;
    }
}

size_t ucg_oracle_special_table(int dt, uint64_t *out, size_t max)
{
    size_t i, n;
    switch (dt) {
    case ORA_F32:
    case ORA_F64:
    case ORA_F16:
    case ORA_BF16:
        n = SPEC_FLOAT_N;
        for (i = 0; i < n && i < max; i++) {
            out[i] = (dt == ORA_F32) ? spec_f32[i] :
                     (dt == ORA_F64) ? spec_f64[i] :
                     (dt == ORA_F16) ? spec_f16[i] : spec_bf16[i];
        }
        return n;
    default:
        n = SPEC_INT_N;
        for (i = 0; i < n && i < max; i++) {
            out[i] = spec_int((unsigned)ucg_oracle_dtype_size(dt) * 8, (unsigned)i);
        }
        return n;
    }
}

static uint64_t gen_bits(int dt, int dist, uint64_t h)
{
    uint64_t sign = h >> 63;
    if (dist == ORA_DIST_SPECIAL) {
        uint64_t tab[32];
        size_t n = ucg_oracle_special_table(dt, tab, 32);
        return tab[h % n];
    }
    if (dist == ORA_DIST_EXACT) {
        int64_t v = (int64_t)(h % 2049u) - 1024;
        switch (dt) {
        case ORA_F16:  return ucg_oracle_float_to_half((float)v);
        case ORA_BF16: return ucg_oracle_float_to_bf16((float)v);
        case ORA_F32:  return f2u((float)v);
        case ORA_F64:  return d2u((double)v);
        default:       return (uint64_t)v; /* truncated to the width below */
        }
    }
    /* ORA_DIST_ROUND */
    switch (dt) {
    case ORA_F16: {
        uint64_t e = ((h >> 10) & 0xff) % 17;       /* biased 7..23 */
        return (sign << 15) | ((e + 7) << 10) | (h & 0x3ff);
    }
    case ORA_BF16: {
        uint64_t e = ((h >> 7) & 0xff) % 17;        /* biased 119..135 */
        return (sign << 15) | ((e + 119) << 7) | (h & 0x7f);
    }
    case ORA_F32: {
        uint64_t e = ((h >> 23) & 0xff) % 17;       /* biased 119..135 */
        return (sign << 31) | ((e + 119) << 23) | (h & 0x7fffff);
    }
    case ORA_F64: {
        uint64_t e = ((h >> 52) & 0x7ff) % 17;      /* biased 1015..1031 */
        return (sign << 63) | ((e + 1015) << 52) | (h & 0xfffffffffffffull);
    }
    default:
        return h;                                   /* full-range integers */
    }
}

void ucg_oracle_fill(int dt, int dist, uint64_t seed, void *dst, size_t count)
{
    ucg_oracle_fill_range(dt, dist, seed, 0, dst, count);
}

void ucg_oracle_fill_range(int dt, int dist, uint64_t seed, size_t start, void *dst,
                           size_t count)
{
    uint64_t key = ucg_oracle_splitmix64(seed);
    size_t sz = ucg_oracle_dtype_size(dt), i;
    for (i = 0; i < count; i++) {
        uint64_t b = gen_bits(dt, dist, ucg_oracle_splitmix64(key ^ (uint64_t)(start + i)));
        switch (sz) {
        case 1: ((uint8_t*)dst)[i]  = (uint8_t)b;  break;
        case 2: ((uint16_t*)dst)[i] = (uint16_t)b; break;
        case 4: ((uint32_t*)dst)[i] = (uint32_t)b; break;
        case 8: ((uint64_t*)dst)[i] = b;           break;
        default: return;
        }
    }
}

/* ------------------------------------------------------------------------ */
/* CPU baseline timing                                                      */
/* ------------------------------------------------------------------------ */
typedef struct {
    int op, dt;
    const char *src;
    char *dst;
    size_t count, frag_bytes;
} ora_job_t;

static void *ora_worker(void *arg)
{
    ora_job_t *j = (ora_job_t*)arg;
    ucg_oracle_reduce_fragmented(j->op, j->dt, j->src, j->dst, j->count,
                                 j->frag_bytes);
    return NULL;
}

static double now_s(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + ts.tv_nsec * 1e-9;
}

static int cmp_dbl(const void *a, const void *b)
{
    double x = *(const double*)a, y = *(const double*)b;
    return (x > y) - (x < y);
}

int ucg_oracle_time_reduce(int op, int dt, const void *src, void *dst,
                           size_t count, size_t frag_bytes, int threads,
                           int reps, double *best, double *median)
{
    size_t sz = ucg_oracle_dtype_size(dt);
    int t, r;
    if (sz == 0 || reps <= 0 || !ucg_oracle_is_supported(dt, op)) {
        return -1;
    }
    if (threads < 1) {
        threads = 1;
    }
    if (threads > 256) {
        threads = 256;
    }
    double *times = malloc(sizeof(double) * reps);
    ora_job_t jobs[256];
    pthread_t tids[256];
    size_t per = count / threads;
    if (!times) {
        return -1;
    }
    for (t = 0; t < threads; t++) {
        size_t lo = per * t, hi = (t == threads - 1) ? count : per * (t + 1);
        jobs[t].op = op;
        jobs[t].dt = dt;
        jobs[t].src = (const char*)src + lo * sz;
        jobs[t].dst = (char*)dst + lo * sz;
        jobs[t].count = hi - lo;
        jobs[t].frag_bytes = frag_bytes;
    }
    for (r = 0; r < reps; r++) {
        double t0 = now_s();
        if (threads == 1) {
            ora_worker(&jobs[0]);
        } else {
            for (t = 0; t < threads; t++) {
                pthread_create(&tids[t], NULL, ora_worker, &jobs[t]);
            }
            for (t = 0; t < threads; t++) {
                pthread_join(tids[t], NULL);
            }
        }
        times[r] = now_s() - t0;
    }
    qsort(times, reps, sizeof(double), cmp_dbl);
    *best   = times[0];
    *median = times[reps / 2];
    free(times);
    return 0;
}
