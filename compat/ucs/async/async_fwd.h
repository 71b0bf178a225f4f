/* compat: the async-context handle and timer callback type */
#ifndef XUCG_COMPAT_UCS_ASYNC_FWD_H
#define XUCG_COMPAT_UCS_ASYNC_FWD_H

#include <ucs/sys/compiler_def.h>
#include <ucs/time/time_def.h>

typedef struct ucs_async_context ucs_async_context_t;

typedef enum {
    UCS_EVENT_SET_EVREAD  = UCS_BIT(0),
    UCS_EVENT_SET_EVWRITE = UCS_BIT(1),
    UCS_EVENT_SET_EVERR   = UCS_BIT(2)
} ucs_event_set_types_t;

typedef void (*ucs_async_event_cb_t)(int id, ucs_event_set_types_t events, void *arg);

#endif
