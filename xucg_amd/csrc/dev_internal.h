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
/* Wait for the work queued so far on the streams of every live context of
 * `device` (an event recorded on each, then waited for): what the shim itself
 * may still run on a buffer before it is freed, cached or unmapped - without
 * a device-wide synchronisation, which would also wait for RCCL's and the
 * application's unrelated streams. Sets `device` current. */
UCG_DEV_HIDDEN hipError_t dev_streams_drain(int device);

#define HIP_TRY(_call)                                                        \
    do {                                                                      \
        hipError_t _e = (_call);                                              \
        if (_e != hipSuccess) {                                               \
            return hip_status(_e, #_call);                                    \
        }                                                                     \
    } while (0)

#endif
