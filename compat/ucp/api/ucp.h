/* compat: the UCP handles the UCG API names (all opaque here) */
#ifndef XUCG_COMPAT_UCP_H
#define XUCG_COMPAT_UCP_H

#include <stdint.h>
#include <stdio.h>

#include <ucs/config/types.h>
#include <ucs/sys/compiler_def.h>
#include <ucs/type/status.h>
#include <uct/api/uct.h>

typedef struct ucp_params   ucp_params_t;
typedef struct ucp_address  ucp_address_t;
typedef struct ucp_context *ucp_context_h;
typedef struct ucp_worker  *ucp_worker_h;
typedef uint64_t            ucp_datatype_t;

#endif
