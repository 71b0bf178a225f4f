/* compat: the UCT handles and types the UCG plan-component API names */
#ifndef XUCG_COMPAT_UCT_H
#define XUCG_COMPAT_UCT_H

#include <stddef.h>
#include <stdint.h>

#include <ucs/async/async_fwd.h>
#include <ucs/sys/compiler_def.h>
#include <ucs/type/status.h>

typedef struct uct_ep    *uct_ep_h;
typedef struct uct_iface *uct_iface_h;
typedef struct uct_md    *uct_md_h;

#define UCT_IFACE_FLAG_AM_SHORT UCS_BIT(0)
#define UCT_IFACE_FLAG_AM_BCOPY UCS_BIT(1)
#define UCT_IFACE_FLAG_AM_ZCOPY UCS_BIT(2)

typedef struct uct_iface_attr {
    struct {
        struct {
            size_t max_short;
            size_t max_bcopy;
            size_t min_zcopy;
            size_t max_zcopy;
            size_t opt_zcopy_align;
            size_t align_mtu;
            size_t max_hdr;
            size_t max_iov;
        } am;
        uint64_t flags;
    } cap;
} uct_iface_attr_t;

typedef struct uct_md_attr {
    struct {
        size_t   max_alloc;
        size_t   max_reg;
        uint64_t flags;
        uint64_t reg_mem_types;
    } cap;
    size_t rkey_packed_size;
} uct_md_attr_t;

typedef enum uct_am_trace_type {
    UCT_AM_TRACE_TYPE_SEND,
    UCT_AM_TRACE_TYPE_RECV,
    UCT_AM_TRACE_TYPE_SEND_DROP,
    UCT_AM_TRACE_TYPE_RECV_DROP,
    UCT_AM_TRACE_TYPE_LAST
} uct_am_trace_type_t;

typedef ucs_status_t (*uct_am_callback_t)(void *arg, void *data, size_t length,
                                          unsigned flags);
typedef void (*uct_am_tracer_t)(void *arg, uct_am_trace_type_t type, uint8_t id,
                                const void *data, size_t length, char *buffer,
                                size_t max);

#endif
