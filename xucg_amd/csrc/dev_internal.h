/*
 * dev_internal.h - what the device shim's translation units share: error
 * reporting (ucg_builtin_dev_last_error) and the context's device. Not part
 * of the C ABI.
 */
#ifndef UCG_DEV_INTERNAL_H_
#define UCG_DEV_INTERNAL_H_

#include <hip/hip_runtime.h>

#include "ucg_builtin_dev.h"

#define UCG_DEV_HIDDEN __attribute__((visibility("hidden")))

/* records "what: why" for ucg_builtin_dev_last_error() and returns st */
UCG_DEV_HIDDEN ucs_status_t set_error(ucs_status_t st, const char *what, const char *why);
/* UCS_OK, or the status a HIP error maps to (recorded like set_error) */
UCG_DEV_HIDDEN ucs_status_t hip_status(hipError_t e, const char *what);
/* the HIP device of a context (hipSetDevice'd by the entry points) */
UCG_DEV_HIDDEN int dev_ctx_device(const ucg_builtin_dev_ctx_t *ctx);

#define HIP_TRY(_call)                                                        \
    do {                                                                      \
        hipError_t _e = (_call);                                              \
        if (_e != hipSuccess) {                                               \
            return hip_status(_e, #_call);                                    \
        }                                                                     \
    } while (0)

#endif
