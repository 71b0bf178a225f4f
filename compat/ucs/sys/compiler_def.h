/* compat: compiler helpers of <ucs/sys/compiler_def.h> used by the UCG API */
#ifndef XUCG_COMPAT_UCS_COMPILER_DEF_H
#define XUCG_COMPAT_UCS_COMPILER_DEF_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
#define BEGIN_C_DECLS extern "C" {
#define END_C_DECLS   }
#else
#define BEGIN_C_DECLS
#define END_C_DECLS
#endif

#define UCS_S_PACKED             __attribute__((packed))
#define UCS_V_ALIGNED(_align)    __attribute__((aligned(_align)))
#define UCS_F_ALWAYS_INLINE      inline __attribute__((always_inline))
#define UCS_F_MAYBE_UNUSED       __attribute__((unused))
#define UCS_SYS_CACHE_LINE_SIZE  64

#define UCS_BIT(_i)              (1ul << (_i))
#define UCS_MASK(_i)             (UCS_BIT(_i) - 1)
#define ucs_offsetof(_t, _m)     offsetof(_t, _m)
#define ucs_container_of(_p, _t, _m) ((_t*)((char*)(_p) - offsetof(_t, _m)))
#define UCS_PTR_BYTE_OFFSET(_p, _off) ((void*)((char*)(_p) + (_off)))

#ifdef __cplusplus
#define UCS_STATIC_ASSERT(_c)    static_assert(_c, #_c)
#else
#define UCS_STATIC_ASSERT(_c)    _Static_assert(_c, #_c)
#endif

/* run a block at load / unload time, once per use (unique by __COUNTER__) */
#define UCS_PP_CAT2(_a, _b)      _a##_b
#define UCS_PP_CAT(_a, _b)       UCS_PP_CAT2(_a, _b)
#define UCS_STATIC_INIT \
    static void __attribute__((constructor)) UCS_PP_CAT(ucs_static_init_, __COUNTER__)(void)
#define UCS_STATIC_CLEANUP \
    static void __attribute__((destructor)) UCS_PP_CAT(ucs_static_cleanup_, __COUNTER__)(void)

#endif
