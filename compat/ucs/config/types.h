/* compat: configuration enums of <ucs/config/types.h> used by the UCG API */
#ifndef XUCG_COMPAT_UCS_CONFIG_TYPES_H
#define XUCG_COMPAT_UCS_CONFIG_TYPES_H

#include <ucs/sys/compiler_def.h>

typedef enum {
    UCS_CONFIG_PRINT_CONFIG = UCS_BIT(0),
    UCS_CONFIG_PRINT_HEADER = UCS_BIT(1),
    UCS_CONFIG_PRINT_DOC    = UCS_BIT(2),
    UCS_CONFIG_PRINT_HIDDEN = UCS_BIT(3)
} ucs_config_print_flags_t;

#define UCS_MEMUNITS_INF ((size_t)-1)
#define UCS_CONFIG_MEMUNITS_INF UCS_MEMUNITS_INF

#endif
